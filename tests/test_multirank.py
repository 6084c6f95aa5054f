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


# ---------------------------------------------------------------- C5 scatter / solve / gather (ttmpc.sharded)
def _oracle_shard_solver(N):
    """CPU stand-in for the device solve of one shard (the test's checker, never the product path)."""
    from oracle import c_oracle as co
    from oracle import ttmpc_oracle as to
    nlp = to.TrackingNLP(N)
    P = co.make_problem(N, to.DEFAULT_PARAMS, nlp.Q, nlp.R, nlp.xlb, nlp.xub, nlp.ulb, nlp.uub)

    def run(x0, xr, ur, X, U, st, it, kk):
        z, s, i, k = co.solve_batch(P, x0.numpy(), xr.numpy(), ur.numpy(), nthreads=1)
        from ttmpc import layout
        Xs, Us = layout.unpack(z, N)
        X.copy_(torch.from_numpy(Xs))
        U.copy_(torch.from_numpy(Us))
        st.copy_(torch.from_numpy(s.astype(np.int32)))
        it.copy_(torch.from_numpy(i.astype(np.int32)))
        kk.copy_(torch.from_numpy(k))
    return run


def _sharded_worker(rank, world, port, B, N, outdir, chunks=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from ttmpc.sharded import ShardedBatch
        sb = ShardedBatch(B, N, _oracle_shard_solver(N), chunks=chunks)
        if rank == 0:
            x0, xr, ur = bench.workload("c5", B, N, seed=3)
            sb.pack_inputs(x0, xr, ur)
        ssum, smax = sb.step()
        stats = ShardedBatch.stats(ssum, smax)
        np.savez(os.path.join(outdir, f"s{rank}.npz"), stats=np.array(
            [stats["converged"], stats["instances"], stats["iters_max"], stats["kkt_max"]]), valid=sb.valid)
        if rank == 0:
            X, U, st, it, kk = sb.results()
            np.savez(os.path.join(outdir, "res.npz"), X=X, U=U, st=st, it=it, kk=kk)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("chunks, valid", [(1, [19, 18]), (3, [21, 16])])
def test_two_rank_scatter_solve_gather(tmp_path, chunks, valid):
    """Ragged global batch (B=37 over 2 ranks) scattered from rank 0 in `chunks` pipelined pieces per
    shard (1: 19 + 18 with one padded slot; 3: chunks of 7, 21 + 16 with five padded slots), solved per
    chunk, gathered back in order; equals one unsharded solve of the whole batch."""
    import bench
    from ttmpc import layout
    world, B, N = 2, 37, 20
    mp.spawn(_sharded_worker, args=(world, _free_port(), B, N, str(tmp_path), chunks), nprocs=world, join=True)
    res = np.load(tmp_path / "res.npz")
    x0, xr, ur = bench.workload("c5", B, N, seed=3)
    X = torch.empty((B, N + 1, 6), dtype=torch.float64)
    U = torch.empty((B, N, 2), dtype=torch.float64)
    st = torch.empty(B, dtype=torch.int32)
    it = torch.empty(B, dtype=torch.int32)
    kk = torch.empty(B, dtype=torch.float64)
    _oracle_shard_solver(N)(torch.from_numpy(x0), torch.from_numpy(xr), torch.from_numpy(ur), X, U, st, it, kk)
    assert np.array_equal(res["X"], X.numpy()) and np.array_equal(res["U"], U.numpy())
    assert np.array_equal(res["st"], st.numpy()) and np.array_equal(res["it"], it.numpy())
    assert np.allclose(layout.pack(res["X"], res["U"])[:, :6], x0)      # x_0 = x_init survived the round trip
    s = [np.load(tmp_path / f"s{r}.npz") for r in range(world)]
    assert [int(x["valid"]) for x in s] == valid
    for x in s:
        conv, inst, imax, kmax = x["stats"]
        assert int(inst) == B and int(conv) == int(np.sum(st.numpy() <= 1))
        assert int(imax) == int(it.max()) and kmax == pytest.approx(float(kk.max()))


def test_single_rank_sharded_is_plain_solve():
    import bench
    from ttmpc.sharded import ShardedBatch
    B, N = 5, 20
    sb = ShardedBatch(B, N, _oracle_shard_solver(N))
    x0, xr, ur = bench.workload("c5", B, N, seed=4)
    sb.pack_inputs(x0, xr, ur)
    stats = ShardedBatch.stats(*sb.step())
    X, U, st, it, kk = sb.results()
    assert stats["instances"] == B and stats["converged"] == int(np.sum(st <= 1)) == B
    assert np.allclose(X[:, 0], x0)


def test_bench_self_launches_ranks():
    """`bench.py --gpus 2` with no launcher starts its own two ranks (RANK / LOCAL_RANK / WORLD_SIZE,
    127.0.0.1 rendezvous) and only rank 0 prints; the selftest config runs the gloo reduction path of the
    real configs without touching a GPU."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--config", "selftest"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["wall_max"] == 1.5 and rec["ok_total"] == 3 and rec["instances"] == 2
