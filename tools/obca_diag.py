"""CPU-oracle convergence census of an OBCA bench workload (development check, no GPU).

    python tools/obca_diag.py c4|c4all|cobs|c4replan LO HI [max_iter] [out.npz]
$TTO_OPTS: oracle TTO_OPT_* bits (switch IPOPT features off for A/B runs).
Solves instances LO..HI-1 of the bench's seed-0 batch with the C oracle (8 threads) and prints status /
iteration counts, so solver changes can be judged on the instances the bench actually runs."""
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402

from oracle import c_oracle as co  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402

G = REPO / "tests" / "golden"


def workload(cfg, B=256):
    obs_all = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))
    g = np.load(G / "reference_numpy.npz")
    if cfg in ("c4", "c4all", "c4replan"):
        N, M = 200, 6
        obs = obs_all[:M]
        if cfg in ("c4", "c4all"):
            cases = json.loads((G / "test_cases.json").read_text())["cases"]
            x0, xg, zg = sc.obca_case_batch(cases, B, N, M, seed=0, obstacles=obs if cfg == "c4" else None,
                                            params=sc.OBCA_PARAMS)
        else:
            x0, xg, zg = sc.obca_replan_batch(g["state_traj"], B, N, M, seed=0)
        P = dict(N=N, params=sc.OBCA_PARAMS, bnd=(sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB), obs=obs,
                 mode=co.OBCA_PLAN)
        return P, dict(x0=x0, x_goal=xg, z_guess=zg)
    N = 50
    obs = g["obstacles"]
    x0, xr, ur = sc.mpc_obs_batch(g["state_traj"], g["input_traj"], B, N, seed=0, obstacles=obs)
    P = dict(N=N, params=dict(sc.OBCA_PARAMS, dt=0.05), bnd=(sc.XLB, sc.XUB, sc.ULB, sc.UUB), obs=obs,
             mode=co.OBCA_TRACK)
    return P, dict(x0=x0, xref=xr, uref=ur)


def main():
    cfg, lo, hi = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    max_iter = int(sys.argv[4]) if len(sys.argv) > 4 else 5000
    P, data = workload(cfg)
    prob = co.make_obca_problem(P["N"], P["params"], sc.OBCA_Q, sc.OBCA_R, *P["bnd"], P["obs"], mode=P["mode"],
                                max_iter=max_iter, opts=int(os.environ.get("TTO_OPTS", "0")))
    sl = {k: v[lo:hi] for k, v in data.items()}
    t = time.time()
    z, st, it, kk = co.obca_solve_batch(prob, **sl, nthreads=8)
    dt = time.time() - t
    print(f"{cfg} [{lo},{hi}) {dt:.1f}s  converged {int((st <= 1).sum())}/{len(st)}")
    print("status", st.tolist())
    print("iters ", it.tolist())
    if len(sys.argv) > 5:
        np.savez(sys.argv[5], status=st, iters=it, kkt=kk, lo=lo, hi=hi)


if __name__ == "__main__":
    main()
