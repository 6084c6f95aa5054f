"""Oracle census of the full-size C4 batches: the CPU restatement of IPOPT (oracle/c/tt_obca.c) on
the exact B = 256 batches that the GPU test (tests/test_gpu_obca.py::test_c4_full_batch_properties_and_determinism,
``_c4_cases(256, seed=1)``) and the bench (``bench.py --config c4``, seed 7, collision-free cases) solve.

Writes tests/golden/c4_census.json (per-instance status / iterations / scaled KKT error) and, for the test batch,
tests/golden/c4_census_test_x.npz (the oracle's final states X (256, 201, 6) float64, the end points the GPU is compared
with).  The test batch is also solved twice more with the guess perturbed by one unit in the last place (z * (1 + 2^-52)
and z * (1 - 2^-53)): an instance whose status changes, or whose converged end point moves (max |dX| > 1e-6), under
that perturbation is *rounding-sensitive* --
its outcome is decided by last-bit differences, which is what separates the GPU's arithmetic (device libm, FMA
contraction, tree reductions) from the oracle's.  The GPU test accepts a status mismatch only on such instances.

Test infrastructure only (never imported by the product).  Runtime: ~1-2 h on 8 host cores.

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


def batches():
    cases = json.loads((HERE / "test_cases.json").read_text())["cases"]
    obs = sc.obstacles_array(sc.load_obstacles(HERE / "obstacles.json"))[:M]
    # the GPU test's batch (test_gpu_obca.py _c4_cases: all 7 cases, blocked starts / goals included)
    test = sc.obca_case_batch(cases, 256, N, M, seed=1)
    # the bench's batch (bench.py main_obca, --config c4, rank 0: rank_seed(0) = 7, collision-free cases)
    bench = sc.obca_case_batch(cases, 256, N, M, seed=7, obstacles=obs, params=sc.OBCA_PARAMS)
    return obs, {"test": test, "bench": bench}


def solve(obs, x0, xg, zg, threads):
    P = co.make_obca_problem(N, sc.OBCA_PARAMS, sc.OBCA_Q, sc.OBCA_R, sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB,
                             sc.OBCA_UUB, obs)
    t = time.time()
    z, st, it, kk = co.obca_solve_batch(P, x0, xg, z_guess=zg, nthreads=threads)
    return co.obca_split(z, N, M)[0], st, it, kk, time.time() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--only", choices=["test", "bench"], default=None)
    args = ap.parse_args()
    obs, bs = batches()
    out_path = HERE / "c4_census.json"
    out = json.loads(out_path.read_text()) if out_path.exists() else {}
    out["provenance"] = ("tests/golden/make_c4_census.py: oracle/c/tt_obca.c (restated IPOPT incl. the full convergence "
                         "test of round 5) on the C4 batches of the GPU test (seed 1) and the bench (seed 7)")
    for name, (x0, xg, zg) in bs.items():
        if args.only and name != args.only:
            continue
        blocked = sc.blocked_poses(x0, obs, sc.OBCA_PARAMS) | sc.blocked_poses(xg, obs, sc.OBCA_PARAMS)
        X, st, it, kk, el = solve(obs, x0, xg, zg, args.threads)
        rec = {"seed": 1 if name == "test" else 7, "B": int(len(x0)), "status": st.tolist(), "iters": it.tolist(),
               "kkt": [float(v) for v in kk], "blocked": blocked.astype(int).tolist(), "seconds": round(el, 1)}
        print(name, "unperturbed", np.bincount(st, minlength=6).tolist(), f"{el:.0f}s", flush=True)
        if name == "test":
            np.savez_compressed(HERE / "c4_census_test_x.npz", X=X, status=st)
            pert = []
            for f in (1.0 + 2.0 ** -52, 1.0 - 2.0 ** -53):
                Xp, stp, itp, _, elp = solve(obs, x0, xg, zg * f, args.threads)
                dx = np.abs(Xp - X).max(axis=(1, 2))
                pert.append({"factor": f, "status": stp.tolist(), "iters": itp.tolist(),
                             "dx_max": [float(v) for v in dx], "seconds": round(elp, 1)})
                print(name, "perturbed", f, np.bincount(stp, minlength=6).tolist(), f"{elp:.0f}s", flush=True)
            rec["perturbed"] = pert
            # sensitive: the status changes, or a converged instance ends at another point (an unconverged run's last
            # iterate -- max_iter, restoration failure -- is not compared)
            sens = np.zeros(len(x0), dtype=bool)
            for p in pert:
                sens |= (np.asarray(p["status"]) != st) | ((st <= 1) & (np.asarray(p["dx_max"]) > 1e-6))
            rec["rounding_sensitive"] = sens.astype(int).tolist()
            print(name, "rounding-sensitive instances:", int(sens.sum()), flush=True)
        out[name] = rec
        out_path.write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
