"""Host-call latency of small tracking solves (diagnostic, GPU box).

    TT_ZERO_COPY_MAX=0 python tools/latency_host.py OUT.npz     # staged: H2D, launch, D2H
    python tools/latency_host.py OUT.npz                        # default: zero-copy up to B = 64

p50 / p99 wall clock of `BatchSolver.solve` (host arrays in and out, as bench.py's p50_latency and the reference's
simulation.py:519-522 call) at B = 1, 4, 16, 64 on the C1/C2 problem (N = 20), and the outputs of one solve per B
(npz), so two runs can be compared bit for bit.
"""
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]
import numpy as np  # noqa: E402


def main():
    import ttmpc
    from ttmpc import scenarios as sc
    out = sys.argv[1]
    # bench.py's C2 solver and synthetic workload (rank 0's seed)
    solver = ttmpc.BatchSolver(20, sc.PARAMS, sc.MPC_Q, sc.MPC_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB)
    x0, xr, ur = sc.synthetic_batch(1024, 20, seed=0)
    res = {}
    for B in (1, 4, 16, 64):
        ts = []
        for r in range(210):
            o = (r * B) % (1024 - B)
            t0 = time.perf_counter()
            solver.solve(x0[o:o + B], xr[o:o + B], ur[o:o + B])
            ts.append(time.perf_counter() - t0)
        ts = np.array(ts[10:]) * 1e3
        X, U, st, it, kk = solver.solve(x0[:B], xr[:B], ur[:B])
        res.update({f"X{B}": X, f"U{B}": U, f"st{B}": st, f"it{B}": it, f"kk{B}": kk})
        print(json.dumps({"B": B, "zero_copy_max": os.environ.get("TT_ZERO_COPY_MAX", "default"),
                          "p50_ms": round(float(np.percentile(ts, 50)), 4), "p99_ms": round(float(np.percentile(ts, 99)), 4),
                          "min_ms": round(float(ts.min()), 4)}), flush=True)
    # the same B = 1 solve from device buffers (no host staging): launch to completion on the stream, HIP events
    import torch
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(v[:1])).to(dev) for k, v in (("x0", x0), ("xr", xr), ("ur", ur))}
    X = torch.empty((1, 21, 6), dtype=torch.float64, device=dev)
    U = torch.empty((1, 20, 2), dtype=torch.float64, device=dev)
    st = torch.empty(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ev = []
    for r in range(210):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        solver.solve_device(1, t["x0"].data_ptr(), t["xr"].data_ptr(), t["ur"].data_ptr(), X.data_ptr(), U.data_ptr(),
                            st.data_ptr(), stream=s)
        e1.record()
        torch.cuda.synchronize()
        ev.append(e0.elapsed_time(e1))
    ev = np.array(ev[10:])
    print(json.dumps({"B": 1, "device_buffers_event_p50_ms": round(float(np.percentile(ev, 50)), 4),
                      "min_ms": round(float(ev.min()), 4)}), flush=True)
    np.savez(out, **res)


if __name__ == "__main__":
    if sys.argv[1] == "compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        print({k: bool(np.array_equal(a[k], b[k])) for k in a.files})
    else:
        main()
