"""Two ranks through ttmpc.sharded with the real HIP solver (SURVEY §8(e), config C5's data path).

The 8-GPU RCCL run is the driver's; this box has one GPU and RCCL refuses two ranks on one device, so the two ranks
share cuda:0 over a gloo group.  That exercises everything of ShardedBatch.step except the RCCL transport: the
per-rank chunk layout, the asynchronous scatters, the per-chunk device solves, the gathers in instance order, the
padding of a ragged batch and the SUM / MAX statistics reduction.  Results must equal a plain single-process solve
of the same batch bit for bit (instances are independent and the kernel is deterministic)."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]


@pytest.mark.gpu
@pytest.mark.parametrize("B,chunks", [(1000, 1), (1237, 3)])
def test_two_ranks_share_one_gpu_bitwise(tmp_path, B, chunks):
    import torch

    import bench
    import ttmpc
    from ttmpc import scenarios as sc
    N = 20
    x0, xr, ur = bench.workload("c5", B, N, seed=11)
    src, out = tmp_path / "in.npz", tmp_path / "out.npz"
    np.savez(src, x0=x0, xr=xr, ur=ur)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   LOCAL_RANK="0")
        procs.append(subprocess.Popen([sys.executable, str(REPO / "tests" / "helpers" / "sharded_rank.py"), str(src),
                                       str(out), str(B), str(N), str(chunks)], env=env, cwd=str(REPO),
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o)
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)[-4000:]
    g = np.load(out)
    r1 = np.load(str(out).replace(".npz", "_r1.npz"))
    per = int(g["per"])
    assert int(g["instances"]) == B and int(r1["lo"]) == per and int(r1["valid"]) == B - per
    # the same batch solved in one process, one launch
    dev = torch.device("cuda", 0)
    solver = ttmpc.BatchSolver(N, sc.PARAMS, sc.MPC_Q, sc.MPC_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB)
    X, U, st, it, kk = _plain_solve(solver, x0, xr, ur, dev)
    assert np.array_equal(g["X"], X) and np.array_equal(g["U"], U)
    assert np.array_equal(g["st"], st) and np.array_equal(g["it"], it) and np.array_equal(g["kk"], kk)
    assert int(g["converged"]) == int((st <= 1).sum()) and int(g["iters_max"]) == int(it.max())
    assert np.array_equal(r1["st"][: int(r1["valid"])], st[per:])


def _plain_solve(solver, x0, xr, ur, dev):
    import torch
    B, N = x0.shape[0], xr.shape[1] - 1
    f64 = dict(dtype=torch.float64, device=dev)
    tx0, txr, tur = (torch.as_tensor(np.ascontiguousarray(a), **f64) for a in (x0, xr, ur))
    X = torch.empty((B, N + 1, 6), **f64)
    U = torch.empty((B, N, 2), **f64)
    kk = torch.empty(B, **f64)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    solver.solve_device(B, tx0.data_ptr(), txr.data_ptr(), tur.data_ptr(), X.data_ptr(), U.data_ptr(), st.data_ptr(),
                        it.data_ptr(), kk.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize(dev)
    return X.cpu().numpy(), U.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy(), kk.cpu().numpy()
