"""Oracle census of the full-size C4 batches: the CPU restatement of IPOPT
(oracle/c/tt_obca.c) on the exact B = 256 batches that the GPU test
(tests/test_gpu_obca.py::test_c4_full_batch_properties_and_determinism, ``_c4_cases(256, seed=1)``) and the bench
(``bench.py --config c4``, seed 7, collision-free cases; tests/test_gpu_obca.py::test_c4_bench_batch_against_census)
solve.

Writes tests/golden/c4_census.json (per batch and per instance: status / iterations / scaled KKT error / plan
objective, for the unperturbed run and every perturbed run) and tests/golden/c4_census_{test,bench}_x.npz (the
oracle's final states X (256, 201, 6) float64 and objectives, the end points the GPU is compared with).

Each batch is solved once as given and then once per factor f in PERTURB with the guess z * f (f = 1 +- one or two
units in the last place).  An instance whose status changes, or whose converged end point moves (max |dX| > 1e-6),
under any of those perturbations is *rounding-sensitive*: its outcome is decided by last-bit differences, which is
what separates the GPU's arithmetic (device libm, FMA contraction, tree reductions) from the oracle's.  The GPU tests
accept a status mismatch or a different converged end point only on such instances, and compare the GPU's objective
on them with the spread of the oracle's own objectives over the perturbed runs.

Test infrastructure only (never imported by the product).  Runtime: ~25 min per run on 8 host cores, 4 runs per batch.

    python tests/golden/make_c4_census.py [--threads 8] [--only test|bench]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]

from oracle import c_oracle as co  # noqa: E402
from ttmpc import scenarios as sc  # noqa: E402

N, M = 200, 6
# one ulp up, half an ulp down (the next double below 1 is 1 - 2^-53), two ulps up
PERTURB = (1.0 + 2.0 ** -52, 1.0 - 2.0 ** -53, 1.0 + 2.0 ** -51)
SEEDS = {"test": 1, "bench": 7}


def batches():
    cases = json.loads((HERE / "test_cases.json").read_text())["cases"]
    obs = sc.obstacles_array(sc.load_obstacles(HERE / "obstacles.json"))[:M]
    # the GPU test's batch (test_gpu_obca.py _c4_cases: all 7 cases, blocked starts / goals included)
    test = sc.obca_case_batch(cases, 256, N, M, seed=SEEDS["test"])
    # the bench's batch (bench.py main_obca, --config c4, rank 0: rank_seed(0) = 7, collision-free cases)
    bench = sc.obca_case_batch(cases, 256, N, M, seed=SEEDS["bench"], obstacles=obs, params=sc.OBCA_PARAMS)
    return obs, {"test": test, "bench": bench}


def plan_objective(X, U, xg):
    """The plan-mode objective of trajectory_optimization.py:170-190 with the bench's weights Q = I, R = 10 I and the
    100 Q terminal weight (oracle/obca_nlp.py ObcaNLP.cost), per instance: X (B,N+1,6), U (B,N,2), xg (B,6)."""
    Q, R = np.asarray(sc.OBCA_Q, float), np.asarray(sc.OBCA_R, float)
    E = X - xg[:, None, :]
    return (np.einsum("bki,ij,bkj->b", U, R, U) + np.einsum("bki,ij,bkj->b", E[:, :-1], Q, E[:, :-1])
            + 100.0 * np.einsum("bi,ij,bj->b", E[:, -1], Q, E[:, -1]))


def solve(obs, x0, xg, zg, threads):
    P = co.make_obca_problem(N, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB,
                             sc.OBCA_UUB, obs)
    t = time.time()
    z, st, it, kk = co.obca_solve_batch(P, x0, xg, z_guess=zg, nthreads=threads)
    X, U, _, _ = co.obca_split(z, N, M)
    return X, st, it, kk, plan_objective(X, U, xg), time.time() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--only", choices=["test", "bench"], default=None)
    args = ap.parse_args()
    obs, bs = batches()
    out_path = HERE / "c4_census.json"
    out = json.loads(out_path.read_text()) if out_path.exists() else {}
    out["provenance"] = ("tests/golden/make_c4_census.py: oracle/c/tt_obca.c (restated IPOPT incl. the full convergence "
                         "test of round 5) on the C4 batches of the GPU test (seed 1) and the bench (seed 7); each "
                         "batch re-solved with the guess scaled by every factor of 'perturbed'")
    for name in ("bench", "test"):
        if args.only and name != args.only:
            continue
        x0, xg, zg = bs[name]
        blocked = sc.blocked_poses(x0, obs, sc.OBCA_PARAMS) | sc.blocked_poses(xg, obs, sc.OBCA_PARAMS)
        X, st, it, kk, obj, el = solve(obs, x0, xg, zg, args.threads)
        rec = {"seed": SEEDS[name], "B": int(len(x0)), "status": st.tolist(), "iters": it.tolist(),
               "kkt": [float(v) for v in kk], "objective": [float(v) for v in obj],
               "blocked": blocked.astype(int).tolist(), "seconds": round(el, 1)}
        print(name, "unperturbed", np.bincount(st, minlength=6).tolist(), f"{el:.0f}s", flush=True)
        np.savez_compressed(HERE / f"c4_census_{name}_x.npz", X=X, status=st, objective=obj)
        pert = []
        sens = np.zeros(len(x0), dtype=bool)
        for f in PERTURB:
            Xp, stp, itp, _, objp, elp = solve(obs, x0, xg, zg * f, args.threads)
            dx = np.abs(Xp - X).max(axis=(1, 2))
            pert.append({"factor": f, "status": stp.tolist(), "iters": itp.tolist(),
                         "dx_max": [float(v) for v in dx], "objective": [float(v) for v in objp],
                         "seconds": round(elp, 1)})
            # sensitive: the status changes, or a converged instance ends at another point (an unconverged run's
            # last iterate -- max_iter, restoration failure -- is not compared)
            sens |= (stp != st) | ((st <= 1) & (dx > 1e-6))
            print(name, "perturbed", f, np.bincount(stp, minlength=6).tolist(), f"{elp:.0f}s",
                  "sensitive so far:", int(sens.sum()), flush=True)
        rec["perturbed"] = pert
        rec["rounding_sensitive"] = sens.astype(int).tolist()
        print(name, "rounding-sensitive instances:", int(sens.sum()), flush=True)
        out[name] = rec
        out_path.write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
