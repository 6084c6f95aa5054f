"""GPU vs CPU-oracle comparison of the OBCA solvers (development check; one summary per workload).

    python tools/obca_check.py [toy|cobs|c4|replan|all] [B]
Both sides start from the reference's duals (mu = 100, lam pattern) and run IPOPT's restoration phase."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402

import ttmpc  # noqa: E402
from oracle import c_oracle as co  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402

G = REPO / "tests" / "golden"
obs_all = sc.obstacles_array(sc.load_obstacles(G / "obstacles.json"))
REF = np.load(G / "reference_numpy.npz")


def report(name, t_gpu, t_cpu, st, stc, it, itc, X, Xc):
    both = (st <= 1) & (stc <= 1)
    dx = np.abs(X - Xc).max(axis=(1, 2))
    print(f"[{name}] B={len(st)}  gpu {t_gpu:.3f}s  cpu {t_cpu:.3f}s")
    print(f"   gpu status {st.tolist()}")
    print(f"   cpu status {stc.tolist()}")
    print(f"   gpu iters {it.tolist()}")
    print(f"   cpu iters {itc.tolist()}")
    print(f"   status agree {int((st == stc).sum())}/{len(st)}; converged gpu {int((st <= 1).sum())} cpu {int((stc <= 1).sum())}")
    print(f"   max|X_gpu - X_cpu| (both converged) {np.array2string(dx[both], precision=1)}")
    sys.stdout.flush()


def run_plan(name, N, M, x0, xg, zg, max_iter=5000, nthreads=8):
    obs = obs_all[:M]
    s = ttmpc.ObcaSolver(N, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB,
                         obs, max_iter=max_iter)
    s.solve(x0[:1], xg[:1], z_guess=zg[:1])  # warm-up (module load)
    t = time.time()
    X, U, Z, st, it, kk = s.solve(x0, xg, z_guess=zg)
    tg = time.time() - t
    P = co.make_obca_problem(N, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB,
                             sc.OBCA_UUB, obs, max_iter=max_iter)
    t = time.time()
    zc, stc, itc, kkc = co.obca_solve_batch(P, x0, xg, z_guess=zg, nthreads=nthreads)
    tc = time.time() - t
    Xc, Uc, _, _ = co.obca_split(zc, N, M)
    report(name, tg, tc, st, stc, it, itc, X, Xc)


def run_track(name, N, M, x0, xr, ur, max_iter=5000, nthreads=8):
    obs = obs_all[:M]
    p = dict(sc.OBCA_PARAMS, dt=0.05)
    s = ttmpc.ObcaSolver(N, p, sc.OBCA_Q, sc.OBCA_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB, obs,
                         variant=ttmpc.TT_VARIANT_TRACK_OBCA, max_iter=max_iter)
    s.solve(x0[:1], xref=xr[:1], uref=ur[:1])
    t = time.time()
    X, U, Z, st, it, kk = s.solve(x0, xref=xr, uref=ur)
    tg = time.time() - t
    P = co.make_obca_problem(N, p, sc.OBCA_Q, sc.OBCA_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB, obs, mode=co.OBCA_TRACK,
                             max_iter=max_iter)
    t = time.time()
    zc, stc, itc, kkc = co.obca_solve_batch(P, x0, xref=xr, uref=ur, nthreads=nthreads)
    tc = time.time() - t
    Xc, Uc, _, _ = co.obca_split(zc, N, M)
    report(name, tg, tc, st, stc, it, itc, X, Xc)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    if which in ("toy", "all"):
        N, M = 60, 1
        obs = np.array([[10.5, 2.6, 3.0, 2.0]])
        x0 = np.array([[0.0, 0.0, 0.02, 0.0, 0.0, 0.0], [0.0, -0.2, 0.0, 0.0, 0.0, 0.0]])
        xg = np.array([[26.0, -0.2, 0.0, 0.0, 0.0, 0.0], [26.0, 0.0, 0.0, 0.0, 0.0, 0.0]])
        zg = np.stack([sc.obca_guess(np.array([a[:2], b[:2]]), np.array([a[2], b[2]]), np.zeros(2), N, M, complete=True)
                       for a, b in zip(x0, xg)])
        obs_all_save = obs_all
        obs_all = obs
        run_plan("toy plan M=1", N, M, x0, xg, zg)
        obs_all = obs_all_save
    if which in ("cobs", "all"):
        x0, xr, ur = sc.mpc_obs_batch(REF["state_traj"], REF["input_traj"], B, 50, seed=0)
        run_track("mpc+obca N=50 M=11", 50, 11, x0, xr, ur)
    if which in ("c4", "all"):
        cases = json.loads((G / "test_cases.json").read_text())["cases"]
        x0, xg, zg = sc.obca_case_batch(cases, B, 200, 6, seed=0)
        run_plan("c4 test_cases N=200 M=6", 200, 6, x0, xg, zg)
    if which in ("replan", "all"):
        x0, xg, zg = sc.obca_replan_batch(REF["state_traj"], B, 200, 6, seed=0)
        run_plan("replan N=200 M=6", 200, 6, x0, xg, zg)
