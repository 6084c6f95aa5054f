"""Multi-GPU sharding of one global batch of tracking NLPs.

One process per GPU (``torch.distributed``; backend "nccl" = RCCL over xGMI on the GPU box, "gloo" on
CPU tests).  Rank 0 holds the global batch (B_total instances, e.g. 65536 mixed test_cases.json
scenarios).  A step is

    scatter   rank 0 -> every rank: one contiguous input chunk per rank      (one collective)
    solve     each rank solves its B_total / world instances, no coupling   (tt_solve_batch_device)
    gather    every rank -> rank 0: one f64 chunk (X, U, kkt) + one i32 chunk (status, iters)
    reduce    one SUM (converged, instances) and one MAX (iterations, KKT error) all-reduce

Instances are independent in every iteration of the interior-point method, so these four collectives
are the only inter-GPU traffic (the reference has no counterpart: simulation.py solves one NLP at a
time on one core).  Shards are contiguous: rank r owns global instances [r*per, (r+1)*per).  When
B_total is not a multiple of the world size, the tail is padded with copies of instance 0, which are
solved but excluded from the outputs and the statistics.

Chunk layouts (f64, instance-major inside each block, so the solver reads the blocks in place):
    input  chunk  [x0 (per,6) | xref (per,N+1,6) | uref (per,N,2)]
    output chunk  [X (per,N+1,6) | U (per,N,2) | kkt (per,)]       + i32 [status (per,) | iters (per,)]
"""
from __future__ import annotations

import math

import numpy as np
import torch


class ShardedBatch:
    """Scatter / solve / gather of one global batch across the ranks of a process group.

    ``solve_shard(x0, xref, uref, X, U, status, iters, kkt)`` receives tensor views of this rank's
    chunk (on ``device``) and must fill X, U, status, iters, kkt; on a GPU it enqueues
    ``BatchSolver.solve_device`` on the current stream (see ``gpu_shard_solver``)."""

    def __init__(self, B_total: int, N: int, solve_shard, device=None, group=None):
        import torch.distributed as dist
        self.dist = dist if dist.is_available() and dist.is_initialized() else None
        self.group = group
        self.world = self.dist.get_world_size(group) if self.dist else 1
        self.rank = self.dist.get_rank(group) if self.dist else 0
        self.B_total, self.N = int(B_total), int(N)
        self.per = max(1, math.ceil(self.B_total / self.world))
        self.lo = self.rank * self.per
        self.valid = max(0, min(self.per, self.B_total - self.lo))   # real instances on this rank
        self.device = torch.device("cpu") if device is None else torch.device(device)
        self.solve_shard = solve_shard
        per, N = self.per, self.N
        self.in_sizes = (per * 6, per * (N + 1) * 6, per * N * 2)
        self.out_sizes = (per * (N + 1) * 6, per * N * 2, per)
        f64 = dict(dtype=torch.float64, device=self.device)
        self.recv_in = torch.empty(sum(self.in_sizes), **f64)
        self.out_f = torch.empty(sum(self.out_sizes), **f64)
        self.out_i = torch.empty(2 * per, dtype=torch.int32, device=self.device)
        a, b, _ = self.in_sizes
        self.x0 = self.recv_in[:a].view(per, 6)
        self.xr = self.recv_in[a:a + b].view(per, N + 1, 6)
        self.ur = self.recv_in[a + b:].view(per, N, 2)
        a, b, _ = self.out_sizes
        self.X = self.out_f[:a].view(per, N + 1, 6)
        self.U = self.out_f[a:a + b].view(per, N, 2)
        self.kkt = self.out_f[a + b:]
        self.st = self.out_i[:per]
        self.it = self.out_i[per:]
        self.valid_mask = torch.zeros(per, dtype=torch.bool, device=self.device)
        self.valid_mask[: self.valid] = True
        if self.rank == 0:
            self.gather_f = torch.empty((self.world, self.out_f.numel()), **f64)
            self.gather_i = torch.empty((self.world, self.out_i.numel()), dtype=torch.int32, device=self.device)
        self.send_in = None

    # ---- rank 0: lay the global batch out as one input chunk per rank (done once, outside the step) ----
    def pack_inputs(self, x0, xref, uref):
        """Global arrays (B_total,6), (B_total,N+1,6), (B_total,N,2) on rank 0 -> the (world, chunk)
        scatter source, resident on this rank's device."""
        if self.rank != 0:
            return None
        B, N, per, W = self.B_total, self.N, self.per, self.world
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64) if not torch.is_tensor(a) else a,  # noqa: E731
                                      dtype=torch.float64)
        x0, xref, uref = t(x0).reshape(B, 6), t(xref).reshape(B, N + 1, 6), t(uref).reshape(B, N, 2)
        pad = per * W - B
        if pad:
            x0 = torch.cat([x0, x0[:1].expand(pad, 6)])
            xref = torch.cat([xref, xref[:1].expand(pad, N + 1, 6)])
            uref = torch.cat([uref, uref[:1].expand(pad, N, 2)])
        send = torch.cat([x0.reshape(W, -1), xref.reshape(W, -1), uref.reshape(W, -1)], dim=1)
        self.send_in = send.to(self.device).contiguous()
        return self.send_in

    def step(self):
        """One scatter -> solve -> gather -> reduce.  Returns the global statistics (every rank):
        dict(converged, instances, iters_max, kkt_max)."""
        d = self.dist
        if d is None or self.world == 1:
            self.recv_in.copy_(self.send_in[0])
        else:
            src = list(self.send_in.unbind(0)) if self.rank == 0 else None
            d.scatter(self.recv_in, src, src=0, group=self.group)
        self.solve_shard(self.x0, self.xr, self.ur, self.X, self.U, self.st, self.it, self.kkt)
        if d is None or self.world == 1:
            self.gather_f[0].copy_(self.out_f)
            self.gather_i[0].copy_(self.out_i)
        else:
            d.gather(self.out_f, list(self.gather_f.unbind(0)) if self.rank == 0 else None, dst=0, group=self.group)
            d.gather(self.out_i, list(self.gather_i.unbind(0)) if self.rank == 0 else None, dst=0, group=self.group)
        m = self.valid_mask
        ssum = torch.stack([((self.st <= 1) & m).sum(), m.sum()]).to(torch.float64)
        smax = torch.stack([torch.where(m, self.it, 0).max().to(torch.float64),
                            torch.where(m, self.kkt, float("-inf")).max()])
        if d is not None and self.world > 1:
            d.all_reduce(ssum, op=d.ReduceOp.SUM, group=self.group)
            d.all_reduce(smax, op=d.ReduceOp.MAX, group=self.group)
        return ssum, smax

    @staticmethod
    def stats(ssum, smax):
        s, m = ssum.cpu().tolist(), smax.cpu().tolist()
        return {"converged": int(s[0]), "instances": int(s[1]), "iters_max": int(m[0]), "kkt_max": float(m[1])}

    def results(self):
        """Rank 0: the global (X, U, status, iters, kkt) in the original instance order (numpy)."""
        if self.rank != 0:
            return None
        B, N, per, W = self.B_total, self.N, self.per, self.world
        a, b, _ = self.out_sizes
        gf, gi = self.gather_f.cpu(), self.gather_i.cpu()
        X = gf[:, :a].reshape(W * per, N + 1, 6)[:B].numpy()
        U = gf[:, a:a + b].reshape(W * per, N, 2)[:B].numpy()
        kk = gf[:, a + b:].reshape(W * per)[:B].numpy()
        st = gi[:, :per].reshape(W * per)[:B].numpy()
        it = gi[:, per:].reshape(W * per)[:B].numpy()
        return X, U, st, it, kk


def gpu_shard_solver(solver, stream=None):
    """solve_shard callback that enqueues the HIP solver on ``stream`` (default: torch's current
    stream) with the chunk views as device buffers -- no host copies."""
    def run(x0, xr, ur, X, U, st, it, kk):
        s = stream if stream is not None else torch.cuda.current_stream(x0.device)
        solver.solve_device(x0.shape[0], x0.data_ptr(), xr.data_ptr(), ur.data_ptr(), X.data_ptr(), U.data_ptr(),
                            st.data_ptr(), it.data_ptr(), kk.data_ptr(), stream=s.cuda_stream)
    return run
