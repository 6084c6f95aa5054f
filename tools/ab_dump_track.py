"""Tracking outputs and small-batch latency of one build, for bitwise A/B between builds (diagnostic, GPU box).

    [TTMPC_LIB=variant.so] python tools/ab_dump_track.py OUT.npz N [B] [seed]
    python tools/ab_dump_track.py compare A.npz B.npz

Solves bench.py's synthetic workload (psi range 0.5) at horizon N for B instances (default 1024) through the host call,
saves X, U, status, iterations and KKT error, and prints the p50 wall clock of 200 host calls at B = 1.
"""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402


def main():
    import ttmpc
    from ttmpc import scenarios as sc
    out, N = sys.argv[1], int(sys.argv[2])
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else 11
    s = ttmpc.BatchSolver(N, sc.PARAMS, sc.MPC_Q, sc.MPC_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB)
    x0, xr, ur = sc.synthetic_batch(B, N, seed=seed, psi_range=0.5)
    X, U, st, it, kk = s.solve(x0, xr, ur)
    ts = []
    for r in range(210):
        t0 = time.perf_counter()
        s.solve(x0[r % B: r % B + 1], xr[r % B: r % B + 1], ur[r % B: r % B + 1])
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts[10:]) * 1e3
    np.savez(out, X=X, U=U, st=st, it=it, kk=kk)
    print(json.dumps({"N": N, "B": B, "status_counts": np.bincount(st, minlength=6).tolist(),
                      "iters_mean": float(it.mean()), "b1_p50_ms": round(float(np.percentile(ts, 50)), 4)}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        print({k: bool(np.array_equal(a[k], b[k])) for k in a.files})
    else:
        main()
