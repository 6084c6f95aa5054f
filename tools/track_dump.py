"""Bitwise A/B of tracking-kernel builds: solve fixed batches and dump the results, or compare two dumps.

    TTMPC_LIB=<build> python tools/track_dump.py OUT.npz
    python tools/track_dump.py --compare A.npz B.npz
Batches: C2 (B=1024, N=20, the bench's rank-0 seed), the N = 20 two-wave build (B=4096), C3-shaped (B=512, N=40, psi
stress), the dense-weight path (B=64, N=20), z-guess warm starts (B=256, N=20) and C5 test_cases scenarios (B=2048)."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402

KEYS = ("X", "U", "st", "it", "kk")


def run(out):
    import bench
    import ttmpc
    from ttmpc import scenarios as sc
    res = {}

    def solver(N, Q=sc.MPC_Q, R=sc.MPC_R):
        return ttmpc.BatchSolver(N, sc.PARAMS, Q, R, sc.XLB, sc.XUB, sc.ULB, sc.UUB)

    def put(tag, r):
        for k, v in zip(KEYS, r[:5]):
            res[f"{tag}_{k}"] = v
        print(tag, "status", np.bincount(r[2], minlength=6).tolist(), "iters mean", float(r[3].mean()), flush=True)

    x0, xr, ur = bench.workload("c2", 1024, 20, seed=bench.rank_seed(0))
    put("c2", solver(20).solve(x0, xr, ur))
    x0, xr, ur = bench.workload("c2", 4096, 20, seed=3)
    put("c2occ", solver(20).solve(x0, xr, ur))
    x0, xr, ur = bench.workload("c3", 512, 40, seed=5)
    put("c3", solver(40).solve(x0, xr, ur))
    x0, xr, ur = bench.workload("c2", 64, 20, seed=9)
    Qd = np.eye(6) + 0.1 * (np.ones((6, 6)) - np.eye(6))
    put("dense", solver(20, Q=Qd).solve(x0, xr, ur))
    x0, xr, ur = bench.workload("c5", 2048, 20, seed=4)
    s20 = solver(20)
    X, U, st, it, kk = s20.solve(x0, xr, ur)
    put("c5", (X, U, st, it, kk))
    zg = np.concatenate([np.concatenate([X[:, :-1], U], axis=2).reshape(2048, -1), X[:, -1]], axis=1)[:256]
    put("warm", s20.solve(x0[:256], xr[:256], ur[:256], z_guess=zg))
    np.savez(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in A.files:
        same = np.array_equal(A[k], B[k], equal_nan=True)
        d = np.max(np.abs(A[k].astype(np.float64) - B[k].astype(np.float64))) if A[k].size else 0.0
        print(f"{k:10s} bitwise {same}  max|diff| {d:.3e}")
        ok &= same
    print("ALL_BITWISE" if ok else "DIFFERENT")


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
