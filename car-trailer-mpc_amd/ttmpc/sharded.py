"""Multi-GPU sharding of one global batch of tracking NLPs.

One process per GPU (``torch.distributed``; backend "nccl" = RCCL over xGMI on the GPU box, "gloo" on
CPU tests).  Rank 0 holds the global batch (B_total instances, e.g. 65536 mixed test_cases.json
scenarios).  A step moves every rank's shard in ``chunks`` pieces so that the transfers run under the
solves:

    scatter   rank 0 -> every rank, chunk by chunk: all C scatters are issued up front (async)
    solve     chunk c starts on the compute stream once its scatter has landed (stream wait, no host
              sync), while the scatters of chunks c+1.. are still moving
    gather    every rank -> rank 0, chunk c issued right behind solve c (the collective stream waits for
              that solve), so it moves while chunk c+1 solves
    reduce    one SUM (converged, instances) and one MAX (iterations, KKT error) all-reduce

Only the first scatter and the last gather sit on the critical path; with C chunks the exposed transfer
time drops to about 2/C of the serial scatter + gather.  Instances are independent in every iteration of
the interior-point method, so these collectives are the only inter-GPU traffic (the reference has no
counterpart: simulation.py solves one NLP at a time on one core).  Shards are contiguous: rank r owns
global instances [r*per, (r+1)*per), chunk c of it [c*pc, (c+1)*pc).  Padding slots (B_total not a
multiple of world * chunks) hold copies of instance 0: solved, excluded from outputs and statistics.

Chunk layouts (f64, chunk-major, instance-major inside each block, so the solver reads them in place):
    input  chunk  [x0 (pc,6) | xref (pc,N+1,6) | uref (pc,N,2)]
    output chunk  [X (pc,N+1,6) | U (pc,N,2) | kkt (pc,)]       + i32 [status (pc,) | iters (pc,)]
"""
from __future__ import annotations

import math

import numpy as np
import torch


class _Chunk:
    """Views of one chunk of this rank's shard."""

    def __init__(self, recv_in, out_f, out_i, pc, N):
        a, b = pc * 6, pc * (N + 1) * 6
        self.x0 = recv_in[:a].view(pc, 6)
        self.xr = recv_in[a:a + b].view(pc, N + 1, 6)
        self.ur = recv_in[a + b:].view(pc, N, 2)
        a, b = pc * (N + 1) * 6, pc * N * 2
        self.X = out_f[:a].view(pc, N + 1, 6)
        self.U = out_f[a:a + b].view(pc, N, 2)
        self.kkt = out_f[a + b:]
        self.st = out_i[:pc]
        self.it = out_i[pc:]


class ShardedBatch:
    """Scatter / solve / gather of one global batch across the ranks of a process group.

    ``solve_shard(x0, xref, uref, X, U, status, iters, kkt)`` receives tensor views of one chunk (on
    ``device``) and must fill X, U, status, iters, kkt; on a GPU it enqueues ``BatchSolver.solve_device``
    on the current stream (see ``gpu_shard_solver``).  ``chunks`` pieces per shard (>= 1) overlap the
    transfers with the solves."""

    def __init__(self, B_total: int, N: int, solve_shard, device=None, group=None, chunks: int = 1):
        import torch.distributed as dist
        self.dist = dist if dist.is_available() and dist.is_initialized() else None
        self.group = group
        self.world = self.dist.get_world_size(group) if self.dist else 1
        self.rank = self.dist.get_rank(group) if self.dist else 0
        self.B_total, self.N = int(B_total), int(N)
        per0 = max(1, math.ceil(self.B_total / self.world))
        self.chunks = max(1, min(int(chunks), per0))
        self.pc = math.ceil(per0 / self.chunks)             # instances per chunk
        self.per = self.pc * self.chunks                    # shard size (padded)
        self.lo = self.rank * self.per
        self.valid = max(0, min(self.per, self.B_total - self.lo))   # real instances on this rank
        self.device = torch.device("cpu") if device is None else torch.device(device)
        self.solve_shard = solve_shard
        pc, N, C = self.pc, self.N, self.chunks
        self.in_chunk = pc * (6 + (N + 1) * 6 + N * 2)
        self.out_chunk = pc * ((N + 1) * 6 + N * 2 + 1)
        f64 = dict(dtype=torch.float64, device=self.device)
        if self.rank == 0:
            self.gather_f = torch.empty((self.world, C, self.out_chunk), **f64)
            self.gather_i = torch.empty((self.world, C, 2 * pc), dtype=torch.int32, device=self.device)
        self.recv_in = torch.empty((C, self.in_chunk), **f64)
        if self.world == 1:
            # one rank: scatter and gather are the identity, so the shard solves straight out of the packed source
            # (pack_inputs) into the gather block -- no device copies in step()
            self.out_f, self.out_i = self.gather_f[0], self.gather_i[0]
        else:
            self.out_f = torch.empty((C, self.out_chunk), **f64)
            self.out_i = torch.empty((C, 2 * pc), dtype=torch.int32, device=self.device)
        self._bind_parts()
        self.valid_mask = torch.zeros(self.per, dtype=torch.bool, device=self.device)
        self.valid_mask[: self.valid] = True
        self.send_in = None

    def _bind_parts(self):
        self.parts = [_Chunk(self.recv_in[c], self.out_f[c], self.out_i[c], self.pc, self.N) for c in range(self.chunks)]

    # ---- rank 0: lay the global batch out as chunk records per rank (done once, outside the step) ----
    def pack_inputs(self, x0, xref, uref):
        """Global arrays (B_total,6), (B_total,N+1,6), (B_total,N,2) on rank 0 -> the (world, chunks,
        record) scatter source, resident on this rank's device."""
        if self.rank != 0:
            return None
        B, N, pc, W, C = self.B_total, self.N, self.pc, self.world, self.chunks
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64) if not torch.is_tensor(a) else a,  # noqa: E731
                                      dtype=torch.float64)
        x0, xref, uref = t(x0).reshape(B, 6), t(xref).reshape(B, N + 1, 6), t(uref).reshape(B, N, 2)
        pad = pc * C * W - B
        if pad:
            x0 = torch.cat([x0, x0[:1].expand(pad, 6)])
            xref = torch.cat([xref, xref[:1].expand(pad, N + 1, 6)])
            uref = torch.cat([uref, uref[:1].expand(pad, N, 2)])
        WC = W * C
        send = torch.cat([x0.reshape(WC, -1), xref.reshape(WC, -1), uref.reshape(WC, -1)], dim=1)
        self.send_in = send.reshape(W, C, self.in_chunk).to(self.device).contiguous()
        if W == 1:
            self.recv_in = self.send_in[0]
            self._bind_parts()
        return self.send_in

    def solve_local(self):
        """Solve every chunk of this rank's shard from recv_in (no communication)."""
        for p in self.parts:
            self.solve_shard(p.x0, p.xr, p.ur, p.X, p.U, p.st, p.it, p.kkt)

    def step(self):
        """One pipelined scatter -> solve -> gather, then the stats reduction.  Returns the global
        statistics tensors (every rank): see ``stats``."""
        d = self.dist
        C = self.chunks
        if d is None or self.world == 1:
            if self.send_in is None:
                raise RuntimeError("ShardedBatch.step: pack_inputs() first (rank 0 holds the global batch)")
            for p in self.parts:  # views of the packed source and of the gather block (see __init__)
                self.solve_shard(p.x0, p.xr, p.ur, p.X, p.U, p.st, p.it, p.kkt)
        else:
            g = self.group
            root = self.rank == 0
            sc = [d.scatter(self.recv_in[c], list(self.send_in[:, c].unbind(0)) if root else None, src=0, group=g,
                            async_op=True) for c in range(C)]
            gathers = []
            for c, p in enumerate(self.parts):
                sc[c].wait()   # NCCL: the compute stream waits for the scatter; gloo: the host does
                self.solve_shard(p.x0, p.xr, p.ur, p.X, p.U, p.st, p.it, p.kkt)
                gathers.append(d.gather(self.out_f[c], list(self.gather_f[:, c].unbind(0)) if root else None, dst=0,
                                        group=g, async_op=True))
                gathers.append(d.gather(self.out_i[c], list(self.gather_i[:, c].unbind(0)) if root else None, dst=0,
                                        group=g, async_op=True))
            for w in gathers:
                w.wait()
        m = self.valid_mask
        st, it, kk = self.status(), self.iters(), self.out_f[:, -self.pc:].reshape(-1)
        ssum = torch.stack([((st <= 1) & m).sum(), m.sum()]).to(torch.float64)
        smax = torch.stack([torch.where(m, it, 0).max().to(torch.float64), torch.where(m, kk, float("-inf")).max()])
        if d is not None and self.world > 1:
            d.all_reduce(ssum, op=d.ReduceOp.SUM, group=self.group)
            d.all_reduce(smax, op=d.ReduceOp.MAX, group=self.group)
        return ssum, smax

    def status(self):
        """This rank's shard statuses (per,), chunk order = instance order."""
        return self.out_i[:, :self.pc].reshape(-1)

    def iters(self):
        return self.out_i[:, self.pc:].reshape(-1)

    @staticmethod
    def stats(ssum, smax):
        s, m = ssum.cpu().tolist(), smax.cpu().tolist()
        return {"converged": int(s[0]), "instances": int(s[1]), "iters_max": int(m[0]), "kkt_max": float(m[1])}

    def results(self):
        """Rank 0: the global (X, U, status, iters, kkt) in the original instance order (numpy)."""
        if self.rank != 0:
            return None
        B, N, pc = self.B_total, self.N, self.pc
        T = self.world * self.chunks * pc
        a, b = pc * (N + 1) * 6, pc * N * 2
        gf, gi = self.gather_f.cpu(), self.gather_i.cpu()
        X = gf[:, :, :a].reshape(T, N + 1, 6)[:B].numpy()
        U = gf[:, :, a:a + b].reshape(T, N, 2)[:B].numpy()
        kk = gf[:, :, a + b:].reshape(T)[:B].numpy()
        st = gi[:, :, :pc].reshape(T)[:B].numpy()
        it = gi[:, :, pc:].reshape(T)[:B].numpy()
        return X, U, st, it, kk


def gpu_shard_solver(solver, stream=None):
    """solve_shard callback that enqueues the HIP solver on ``stream`` (default: torch's current
    stream) with the chunk views as device buffers -- no host copies."""
    def run(x0, xr, ur, X, U, st, it, kk):
        s = stream if stream is not None else torch.cuda.current_stream(x0.device)
        solver.solve_device(x0.shape[0], x0.data_ptr(), xr.data_ptr(), ur.data_ptr(), X.data_ptr(), U.data_ptr(),
                            st.data_ptr(), it.data_ptr(), kk.data_ptr(), stream=s.cuda_stream)
    return run
