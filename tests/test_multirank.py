"""world_size-2 gloo test of bench.py's multi-rank logic (CPU only).

bench.py shards instances across ranks by seed (rank_seed), runs each shard independently (no
data-path collective) and reduces only the timing/counters on the host (reduce_over_ranks: MAX
wall, SUM solved/instances).  Here each rank solves its shard with the CPU oracle standing in for
the device, so the sharding + reduction path is exercised exactly as on an N-GPU node.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO  # noqa: F401  (puts the repo and package on sys.path)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, N, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from oracle import c_oracle as co
        from oracle import ttmpc_oracle as to
        x0, xr, ur = bench.workload("c2", B, N, seed=bench.rank_seed(rank))
        nlp = to.TrackingNLP(N)
        P = co.make_problem(N, to.DEFAULT_PARAMS, nlp.Q, nlp.R, nlp.xlb, nlp.xub, nlp.ulb, nlp.uub)
        _, st, _, _ = co.solve_batch(P, x0, xr, ur, nthreads=1)
        ok = int(np.sum(st <= 1))
        wall = 0.5 + rank  # distinct per-rank clocks: the reduction must take the max
        res = bench.reduce_over_ranks(dist, wall, ok, B)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), x0=x0, ok=ok, res=np.array(res, dtype=np.float64))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_and_reduction(tmp_path):
    world, B, N = 2, 16, 20
    mp.spawn(_worker, args=(world, _free_port(), B, N, str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{i}.npz") for i in range(world)]
    # disjoint shards: different seeded instances per rank
    assert not np.allclose(r[0]["x0"], r[1]["x0"])
    # every rank sees the same reduced triple: max wall, summed solved, summed instances
    for ri in r:
        wall_max, ok_total, B_total = ri["res"]
        assert wall_max == pytest.approx(0.5 + (world - 1))
        assert int(ok_total) == sum(int(x["ok"]) for x in r)
        assert int(B_total) == world * B
    assert all(int(x["ok"]) == B for x in r)  # the synthetic C2 instances all converge


def test_single_process_reduction_is_identity():
    import bench
    assert bench.reduce_over_ranks(None, 1.25, 7, 9) == (1.25, 7, 9)
    assert len({bench.rank_seed(k) for k in range(8)}) == 8
