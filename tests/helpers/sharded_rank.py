"""One rank of the two-rank device test of ttmpc.sharded (tests/test_gpu_multirank.py).

Both ranks run on cuda:0 of the one-GPU box over a gloo process group (RCCL refuses two ranks on one device), so
the scatter -> HIP solve -> gather -> stats all-reduce of ShardedBatch.step runs with device-resident chunks and the
real solver; rank 0 writes the gathered results.   env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT
usage: python tests/helpers/sharded_rank.py IN.npz OUT.npz B_TOTAL N CHUNKS
"""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    src, out, B, N, chunks = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    import ttmpc
    from ttmpc import scenarios as sc
    from ttmpc.sharded import ShardedBatch, gpu_shard_solver
    dist.init_process_group(backend="gloo")
    rank = dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    solver = ttmpc.BatchSolver(N, sc.PARAMS, sc.MPC_Q, sc.MPC_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB)
    sb = ShardedBatch(B, N, gpu_shard_solver(solver), device=dev, chunks=chunks)
    if rank == 0:
        d = np.load(src)
        sb.pack_inputs(d["x0"], d["xr"], d["ur"])
    ssum, smax = sb.step()
    torch.cuda.synchronize(dev)
    stats = ShardedBatch.stats(ssum, smax)
    if rank == 0:
        X, U, st, it, kk = sb.results()
        np.savez(out, X=X, U=U, st=st, it=it, kk=kk, converged=stats["converged"], instances=stats["instances"],
                 iters_max=stats["iters_max"], per=sb.per, valid1=-1)
    else:
        # rank 1's own shard, for the test's check that each rank solved exactly its contiguous range
        np.savez(out.replace(".npz", "_r1.npz"), valid=sb.valid, lo=sb.lo, st=sb.status().cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
