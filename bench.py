"""Benchmark: batched truck-trailer NMPC solves on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W [--config c2|c3|c5|c4|c4all|c4replan|cobs|sim] [--batch B] [--horizon H]

c5 is the sharded path: one global batch on rank 0, RCCL scatter -> solve -> gather (ttmpc/sharded.py).
With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py launches the N ranks itself (one process
per GPU, 127.0.0.1 rendezvous) before touching the GPU, and rank 0 prints the line.

A "step" = one launch of the HIP solver over one batch of B independent NLP instances (B solves),
inputs already resident in HBM.  Default workload = BASELINE configs[1] (C2): B = 1024 instances
per GPU, horizon N = 20, synthetic reference tracking problems (SURVEY.md §8(d) generator, seeded
per rank -> each rank owns its shard, no data-path collective: weak scaling).

Prints ONE JSON line on rank 0.  `value` = solves/s of the whole job (sum over ranks / max time).
`roofline` uses the algorithmic FP64 flop formula of SURVEY.md §8(d) over the per-instance Newton
iteration counts the kernel returns, divided by the kernel time measured with HIP events on the
stream the kernel is launched on.  `cpu_baseline` times the CPU oracle (oracle/, the same NLP and
interior-point constants, banded-LU KKT, OpenMP over instances) on a bounded sample on rank 0, with
as many threads as the host grants this process (OMP_NUM_THREADS, which the GPU pool sets to the
per-GPU CPU share, else every core in os.sched_getaffinity) and on one core.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path[:0] = [str(REPO), str(REPO / "car-trailer-mpc_amd")]

import torch  # noqa: E402

FP64_PEAK_TFLOPS = 78.6    # MI355X dense FP64 (vector = matrix on CDNA4), MI355X_MICROARCH / spec
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec


def flops_per_solve(N, iters):
    """F = lin_evals*F_lin + kkt_solves*(F_ric + F_fwd + F_ipm), nx=6, nu=2,
    lin_evals = iters + 1 (one linearisation per Newton step + the final convergence test),
    kkt_solves = iters (one Riccati factorisation + solve per step; inertia retries not counted)."""
    F_lin = N * (60 + 5 * 20)
    F_ric = N * 1539
    F_fwd = N * 152
    F_ipm = N * 12 * 10
    return (iters + 1) * F_lin + iters * (F_ric + F_fwd + F_ipm)


def io_bytes_per_solve(N):
    """Algorithmic HBM bytes per solve: x0 + xref + uref in, x_out + u_out + status/iters/kkt out."""
    return 8 * (6 + 6 * (N + 1) + 2 * N) + 8 * (6 * (N + 1) + 2 * N) + 4 + 4 + 8


def workload(cfg, B, N, seed):
    from ttmpc import scenarios
    if cfg == "c3":
        return scenarios.synthetic_batch(B, N, seed=seed, psi_range=0.9)
    if cfg == "c5":
        cases = json.loads((REPO / "tests" / "golden" / "test_cases.json").read_text())["cases"]
        return scenarios.test_case_batch(cases, B, N, seed=seed)
    return scenarios.synthetic_batch(B, N, seed=seed)


def cpu_threads():
    """Host threads for the CPU baseline: OMP_NUM_THREADS when the host sets it (the GPU pool sets it to
    the CPU share of one GPU), else every core this process may run on."""
    ncores = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS", "")
    return (max(1, min(ncores, int(env))) if env.isdigit() and int(env) > 0 else ncores), ncores


def spawn_ranks(args):
    """--gpus N without a launcher: start N copies of this script as ranks 0..N-1 (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT), before this process touches the GPU; rank 0
    prints the JSON line.  Returns the first nonzero exit code (0 when every rank succeeded)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    # poll every rank: the first failure terminates the others (a rank left waiting in a collective or the
    # rendezvous for a dead peer would otherwise hang until the process-group timeout)
    while True:
        codes = [p.poll() for p in procs]
        bad = next((c for c in codes if c not in (None, 0)), None)
        if bad is not None:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad
        if all(c == 0 for c in codes):
            return 0
        time.sleep(0.2)


def cpu_baseline(cfg, B, N, seed, budget_s):
    """CPU oracle on a bounded sample of the same workload (rank 0, N=1 only)."""
    import numpy as np

    from oracle import c_oracle as co
    from oracle import ttmpc_oracle as to
    threads, ncores = cpu_threads()
    x0, xr, ur = workload(cfg, B, N, seed)
    nlp = to.TrackingNLP(N)
    P = co.make_problem(N, to.DEFAULT_PARAMS, nlp.Q, nlp.R, nlp.xlb, nlp.xub, nlp.ulb, nlp.uub)
    co.solve_batch(P, x0[: min(B, 64)], xr[: min(B, 64)], ur[: min(B, 64)], nthreads=threads)  # warm

    def rate(nth, budget):
        done, t0 = 0, time.perf_counter()
        chunk = min(B, 256 * nth)
        while True:
            lo = done % B
            hi = min(B, lo + chunk)
            co.solve_batch(P, x0[lo:hi], xr[lo:hi], ur[lo:hi], nthreads=nth)
            done += hi - lo
            el = time.perf_counter() - t0
            if el >= budget:
                return done, el
    done, el = rate(threads, budget_s)
    d1, e1 = rate(1, max(1.0, budget_s / 4))   # also one core, for the per-core comparison
    return {"value": done / el, "unit": "solves/s", "cores": threads, "kind": "port",
            "value_1core": d1 / e1,
            "host_cores_visible": ncores,
            "sample": f"{done} solves of the same {cfg} workload (N={N}) in {el:.1f}s, OpenMP {threads} threads "
                      f"(OMP_NUM_THREADS / affinity) on {ncores} visible host cores (1 core: {d1} solves in {e1:.1f}s); "
                      "oracle/c/tt_oracle.c (IPOPT-restated IPM, banded LU)"}


def local_device():
    """GPU of this rank: LOCAL_RANK (one process per GPU).  TTMPC_BENCH_DEVICE pins every rank to one GPU,
    which only serves to rehearse the multi-rank flow on a one-GPU box (not a measurement setup)."""
    if os.environ.get("TTMPC_BENCH_DEVICE"):
        return int(os.environ["TTMPC_BENCH_DEVICE"])
    return int(os.environ.get("LOCAL_RANK", "0"))


def rank_seed(rank):
    """Each rank owns a disjoint seeded shard of instances (weak scaling, no data-path collective)."""
    return 1000 * rank + 7


def reduce_over_ranks(dist, wall, ok, B):
    """Host-side (gloo) reduction of the per-rank timing: MAX wall clock, SUM of solved/instances.
    Returns (wall_max, ok_total, B_total); identity when dist is None (single process)."""
    if dist is None:
        return wall, ok, B
    t_local = torch.tensor([wall, float(ok), float(B)], dtype=torch.float64)
    tmax = t_local.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tsum = t_local.clone()
    dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    return float(tmax[0]), int(tsum[1]), int(tsum[2])


def p50_latency(solver, x0, xr, ur, reps=200):
    """Host wall clock around one B=1 solve incl. H2D/D2H (mirrors simulation.py:519-522)."""
    import numpy as np
    ts = []
    for r in range(reps + 10):
        t0 = time.perf_counter()
        solver.solve(x0[r % 8: r % 8 + 1], xr[r % 8: r % 8 + 1], ur[r % 8: r % 8 + 1])
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts[10:]) * 1e3
    return float(np.percentile(ts, 50)), float(np.percentile(ts, 99))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c5", "c4", "c4all", "c4replan", "cobs", "sim", "selftest"],
                    help="c2/c3/c5: tracking NMPC; c4: OBCA plans of the collision-free test_cases.json cases "
                         "(trajectory_optimization.py); c4all: all 7 cases (3 are infeasible NLPs); "
                         "c4replan: OBCA re-plans around the committed plan; cobs: MPC+OBCA (mpc_control_obs.py)")
    ap.add_argument("--batch", type=int, default=0, help="instances per GPU (default by config)")
    ap.add_argument("--horizon", type=int, default=0)
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-baseline work (0 = skip)")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--traffic-csv", default="",
                    help="comma-separated rocprofv3 --pmc CSVs (FETCH_SIZE, WRITE_SIZE) of this config; "
                         "default: the committed profiles/ pair when the config is the default C2")
    ap.add_argument("--max-iter", type=int, default=5000, help="OBCA configs: IPOPT max_iter (reference: 5000)")
    ap.add_argument("--chunks", type=int, default=0,
                    help="c5: pipelined scatter/solve/gather chunks per rank shard (one rank: chunk copies); "
                         "0 = auto: 1 (one launch per rank shard, the measured fastest shape)")
    ap.add_argument("--graph", action="store_true", help="sim: replay one captured closed-loop step (hipGraph)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    if args.config == "selftest":
        return main_selftest(args)
    if args.config in ("c4", "c4all", "c4replan", "cobs"):
        return main_obca(args)
    if args.config == "c5":
        return main_c5(args)
    if args.config == "sim":
        return main_sim(args)

    defaults = {"c2": (1024, 20), "c3": (8192, 40)}
    B = args.batch or defaults[args.config][0]
    N = args.horizon or defaults[args.config][1]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = local_device()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")  # host-side barrier/max only: no data-path collective

    import numpy as np

    import ttmpc
    from ttmpc import scenarios as sc  # params / weights / bounds of simulation.py:391-414

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    solver = ttmpc.BatchSolver(N, sc.PARAMS, sc.MPC_Q, sc.MPC_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB, device=local)
    x0, xr, ur = workload(args.config, B, N, seed=rank_seed(rank))
    t = {k: torch.from_numpy(v).to(dev) for k, v in (("x0", x0), ("xr", xr), ("ur", ur))}
    X = torch.empty((B, N + 1, 6), dtype=torch.float64, device=dev)
    U = torch.empty((B, N, 2), dtype=torch.float64, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    kk = torch.empty(B, dtype=torch.float64, device=dev)
    stream = torch.cuda.Stream(dev)  # explicit non-null stream: the kernel and the timing events share it

    def step():
        solver.solve_device(B, t["x0"].data_ptr(), t["xr"].data_ptr(), t["ur"].data_ptr(), X.data_ptr(),
                            U.data_ptr(), st.data_ptr(), it.data_ptr(), kk.data_ptr(), stream=stream.cuda_stream)

    torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    kernel_ms = e0.elapsed_time(e1) / args.steps
    status = st.cpu().numpy()
    iters = it.cpu().numpy()
    kkt = kk.cpu().numpy()
    ok = int(np.sum(status <= 1))
    wall_max, ok_total, B_total = reduce_over_ranks(dist, wall, ok, B)
    if rank != 0:
        dist.destroy_process_group()
        return
    ms_per_step = wall_max / args.steps * 1e3
    value = B_total * args.steps / wall_max
    F = float(np.sum(flops_per_solve(N, iters.astype(np.float64))))
    achieved = F / (kernel_ms * 1e-3) / 1e12
    io = io_bytes_per_solve(N) * B
    traffic = None
    traffic_src = None
    csvs = [p for p in args.traffic_csv.split(",") if p]
    src_note = ""
    if not csvs and (args.config, B, N) in (("c2", 1024, 20), ("c3", 8192, 40)):
        d = REPO / TRACK_PMC[args.config]
        csvs = [str(d / pas / f"{pas}_counter_collection.csv") for pas in ("fetch", "write")]
        src_note = f" (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes of this bench config; HBM bytes per " \
                   f"launch; {TRACK_PMC_SOURCE})"
    if csvs and all(Path(p).exists() for p in csvs):
        traffic = read_traffic(csvs)
        traffic_src = ", ".join(str(Path(p).relative_to(REPO)) if str(p).startswith(str(REPO)) else p for p in csvs) + \
            src_note
    out = {
        "metric": "MPC solves/sec (N=20, nx=6, nu=2; BASELINE label says nx=5, the reference model has 6 states)"
        if N == 20 else f"MPC solves/sec (N={N}, nx=6, nu=2)",
        "value": round(value, 1),
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY §8(d) seeded reference-tracking instances, per-rank shard)",
        "config": {"workload": f"{args.config}: B={B} instances/GPU, N={N}, tracking NMPC (mpc_control.py NLP), "
                               "IPOPT tol 1e-8", "batch_per_gpu": B, "horizon": N,
                   "parallelism": f"dp{world} (independent instance shards)"},
        "solver": {"converged_or_acceptable": ok_total, "instances": B_total,
                   "iters_mean": float(iters.mean()), "iters_max": int(iters.max()),
                   "kkt_max": float(np.max(kkt)), "kernel_ms_per_launch": round(kernel_ms, 4)},
        "roofline": {"bound": "valu_fp64", "achieved": round(achieved, 4), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / FP64_PEAK_TFLOPS, 6), "traffic": traffic,
                     "note": "FP64 VALU/latency-bound kernel (no MFMA): roof = MI355X dense FP64 vector peak 78.6 TF. "
                             "Algorithmic flops: SURVEY §8(d) "
                             f"formula x per-instance iterations ({F / B:.0f} flop/solve avg); HBM algorithmic "
                             f"{io / (kernel_ms * 1e-3) / 1e9:.2f} GB/s = "
                             f"{io / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS:.2e} of 8 TB/s",
                     "traffic_source": traffic_src},
    }
    if not args.no_latency:
        p50, p99 = p50_latency(solver, x0, xr, ur)
        out["p50_latency_ms"] = round(p50, 4)
        out["p99_latency_ms"] = round(p99, 4)
    if args.cpu_budget > 0 and world == 1:
        out["cpu_baseline"] = cpu_baseline(args.config, B, N, rank_seed(rank), args.cpu_budget)
        if "p50_latency_ms" in out:
            # B = 1 latency against one CPU core solving the same NLP (the reference solves one instance per call on
            # one core): the oracle's mean per-solve time on one core of the same sample
            c1 = 1e3 / out["cpu_baseline"]["value_1core"]
            out["latency_vs_cpu_1core"] = {"p50_latency_ms": out["p50_latency_ms"], "cpu_1core_ms_per_solve": round(c1, 4),
                                           "ratio": round(c1 / out["p50_latency_ms"], 3)}
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


def main_selftest(args):
    """Rehearsal of the multi-rank plumbing without a GPU (tests/test_multirank.py): gloo rendezvous on
    127.0.0.1, barrier, and the MAX-wall / SUM-count reduction of the real configs; rank 0 prints one line."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")
        dist.barrier()
    wall_max, ok_total, B_total = reduce_over_ranks(dist, 0.5 + rank, rank + 1, 1)
    if rank == 0:
        print(json.dumps({"metric": "selftest", "n_gpus": world, "wall_max": wall_max, "ok_total": ok_total,
                          "instances": B_total, "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}))
    if dist:
        dist.destroy_process_group()


def main_c5(args):
    """BASELINE configs[4] (C5): ONE global batch of B_total = 65536 mixed test_cases.json scenarios
    (N = 20) resident on rank 0's GPU, sharded over the ranks with RCCL (torch.distributed "nccl"):
    a step = scatter -> per-rank solve -> gather to rank 0 -> stats all-reduce (ttmpc.sharded).
    Total work is fixed as N grows: strong scaling."""
    import numpy as np

    import ttmpc
    from ttmpc import scenarios as sc
    from ttmpc.sharded import ShardedBatch, gpu_shard_solver
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = local_device()
    B_total, N = args.batch or 65536, args.horizon or 20
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="nccl", device_id=dev)
    solver = ttmpc.BatchSolver(N, sc.PARAMS, sc.MPC_Q, sc.MPC_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB, device=local)
    stream = torch.cuda.Stream(dev)
    # chunks apply on one rank too (chunk copies instead of collectives), so e.g. --batch 8192 --chunks 2 times on one
    # GPU exactly the per-rank launch shape of a chunked 8-rank run.  Auto = ONE chunk per rank shard: measured through
    # the sharded path on one GPU at the 8-rank shard size of 8,192 instances, 1 chunk 11.54 M solves/s, 2 chunks
    # 10.20 M, 4 chunks 8.31 M (profiles/r04/session_b/bench_c5_8192x{1,2,4}.json): a smaller launch loses more
    # occupancy (the two-wave N = 20 build needs >= 4096 instances to pay, profiles/r04/occ_by_batch/) than the
    # overlap of an ~11 MB scatter (~0.07 ms over xGMI) can win back.  --chunks > 1 stays available for an RCCL run
    # that shows overlap paying.
    chunks = args.chunks if args.chunks > 0 else 1
    sb = ShardedBatch(B_total, N, gpu_shard_solver(solver, stream), device=dev, chunks=chunks)
    if rank == 0:
        x0, xr, ur = workload("c5", B_total, N, seed=rank_seed(0))
        sb.pack_inputs(x0, xr, ur)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            sb.step()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.steps):
            ssum, smax = sb.step()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
    step_ms_local = e0.elapsed_time(e1) / args.steps
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())
    stats = ShardedBatch.stats(ssum, smax)
    if rank != 0:
        dist.destroy_process_group()
        return
    # kernel-only time of this rank's shard: one more solve on the same stream, HIP events around it
    k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        k0.record(stream)
        sb.solve_local()
        k1.record(stream)
    torch.cuda.synchronize(dev)
    kernel_ms = k0.elapsed_time(k1)
    X, U, st, it, kk = sb.results()
    F_shard = float(np.sum(flops_per_solve(N, sb.iters()[: sb.valid].cpu().numpy().astype(np.float64))))
    achieved = F_shard / (kernel_ms * 1e-3) / 1e12
    out = {
        "metric": "MPC solves/sec (N=20, nx=6, nu=2; BASELINE label says nx=5, the reference model has 6 states)"
        if N == 20 else f"MPC solves/sec (N={N}, nx=6, nu=2)",
        "value": round(B_total * args.steps / wall_max, 1),
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (test_cases.json start/goal poses x Monte-Carlo start perturbations, straight-line "
                "references; the global batch is generated on rank 0 and scattered)",
        "config": {"workload": f"c5: ONE global batch B={B_total}, N={N}, tracking NMPC (mpc_control.py NLP), IPOPT "
                               f"tol 1e-8; scatter/solve/gather over RCCL ({world} ranks x {sb.per} instances, "
                               f"{sb.chunks} pipelined chunks per rank)",
                   "global_batch": B_total, "horizon": N,
                   "parallelism": f"dp{world} (contiguous shards; chunked RCCL scatter + gather overlapped with the "
                                  "solves, stats all-reduce per step)"},
        "solver": {"converged_or_acceptable": stats["converged"], "instances": stats["instances"],
                   "iters_mean": float(it.mean()), "iters_max": stats["iters_max"], "kkt_max": stats["kkt_max"],
                   "step_ms_rank0_hip_events": round(step_ms_local, 4),
                   "kernel_ms_per_launch": round(kernel_ms, 4)},
        "roofline": {"bound": "valu_fp64", "achieved": round(achieved, 4), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / FP64_PEAK_TFLOPS, 6), "traffic": None,
                     "note": "rank-0 shard kernel (track_kernel) only; SURVEY §8(d) flop formula x per-instance "
                             "iterations"},
    }
    if args.cpu_budget > 0 and world == 1:
        out["cpu_baseline"] = cpu_baseline("c5", min(B_total, 8192), N, rank_seed(0), args.cpu_budget)
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


def main_sim(args):
    """Closed-loop Monte-Carlo: simulation.py's loop (N=50, dt=0.05, disturbances on,
    noisy measurements, collision check vs obstacles.json) for B instances started around the plan's start,
    tracking the reference's committed OBCA plan interpolated to 0.05 s.  A step = one closed-loop step of
    every instance: window -> collision check -> solve -> plant update, all on the device."""
    import numpy as np

    import ttmpc
    from ttmpc import scenarios as sc
    from ttmpc import simulation as sim
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = local_device()
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")
    B, N = args.batch or 1024, args.horizon or 50
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    g = np.load(REPO / "tests" / "golden" / "reference_numpy.npz")
    S, U = g["interp_states"], g["interp_inputs"]
    params = dict(sc.PARAMS, horizon=N)
    rng = np.random.default_rng(rank_seed(rank))
    x0 = S[:, 0][None] + rng.normal(scale=[0.3, 0.3, 0.02, 0.02, 0.0, 0.0], size=(B, 6))
    solver = ttmpc.BatchSolver(N, params, sc.MPC_Q, sc.MPC_R, sc.XLB, sc.XUB, sc.ULB, sc.UUB, device=local)
    cl = sim.ClosedLoop(solver, S, U, params, sim.DISTURBANCE_PARAMS, obstacles=g["obstacles"], seed=rank_seed(rank))
    cl.reset(x0)
    dt = 0.05   # the reference's clock: t accumulated with +=, k = floor(t / dt) (simulation.py:484-531)
    t_sim, k_list = 0.0, []
    while len(k_list) < args.warmup + args.steps:
        k_list.append(int(np.floor(t_sim / dt)))
        t_sim += dt
    if args.graph:
        # the step index, the k sequence and the noise of every step on the device; one captured step
        K = args.warmup + args.steps
        d_ks = torch.tensor(k_list, dtype=torch.int32, device=dev)
        d_step = torch.zeros(1, dtype=torch.int32, device=dev)
        noise_all = torch.randn((K, B, 6), generator=cl.gen, dtype=torch.float64, device=dev)
        noise_all.mul_(sim.DISTURBANCE_PARAMS["process_noise_std"])
        logs = (torch.empty((K + 1, B, 6), dtype=torch.float64, device=dev),
                torch.empty((K, B, 2), dtype=torch.float64, device=dev),
                torch.zeros((K, B), dtype=torch.int32, device=dev), torch.zeros((K, B), dtype=torch.int32, device=dev),
                torch.zeros((K, B), dtype=torch.int32, device=dev))
        torch.cuda.synchronize(dev)
        with torch.cuda.stream(cl.stream):
            cl._graph_step(True, d_ks, d_step, noise_all, logs)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=cl.stream):
            cl._graph_step(False, d_ks, d_step, noise_all, logs)
        run_step = lambda k: graph.replay()  # noqa: E731
        warm_steps = k_list[1: args.warmup]
    else:
        run_step = cl.step
        warm_steps = k_list[: args.warmup]
    with torch.cuda.stream(cl.stream):
        for k in warm_steps:
            run_step(k)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(cl.stream)
    with torch.cuda.stream(cl.stream):  # graph replay() launches on the current stream
        for k in k_list[args.warmup:]:
            run_step(k)
    e1.record(cl.stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    st = cl.st.cpu().numpy()
    ok = int(np.sum(st <= 1))
    wall_max, ok_total, B_total = reduce_over_ranks(dist, wall, ok, B)
    if rank != 0:
        dist.destroy_process_group()
        return
    # one more solve alone: the track_kernel share of a closed-loop step
    k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k0.record(cl.stream)
    solver.solve_device(B, cl.x_meas.data_ptr(), cl.xref.data_ptr(), cl.uref.data_ptr(), cl.X.data_ptr(),
                        cl.U.data_ptr(), cl.st.data_ptr(), cl.it.data_ptr(), cl.kkt.data_ptr(),
                        stream=cl.stream.cuda_stream)
    k1.record(cl.stream)
    torch.cuda.synchronize(dev)
    kernel_ms = k0.elapsed_time(k1)
    iters = cl.it.cpu().numpy()
    F = float(np.sum(flops_per_solve(N, iters.astype(np.float64))))
    out = {
        "metric": f"closed-loop MPC steps/sec (simulation.py loop, N={N}, disturbed plant)",
        "value": round(B_total * args.steps / wall_max, 1),
        "unit": "instance-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "the reference's committed OBCA plan (data/state_traj.txt, do_interpolation 0.1 -> 0.05) with "
                "B perturbed starts, DISTURBANCE_PARAMS of simulation.py, device-drawn measurement noise",
        "config": {"workload": f"sim: B={B} closed loops/GPU, N={N}, steps {args.warmup}+{args.steps} of the "
                               "simulation.py loop (window, SAT collision check, solve, disturbed plant update)"
                               + (", one captured step replayed as a hipGraph" if args.graph else ""),
                   "batch_per_gpu": B, "horizon": N, "parallelism": f"dp{world} (independent instances)"},
        "solver": {"converged_or_acceptable_last_step": ok_total, "instances": B_total,
                   "status_counts_last_step": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                   "iters_mean_last_step": float(iters.mean()), "step_ms_hip_events": round(
                       e0.elapsed_time(e1) / args.steps, 4), "kernel_ms_per_solve": round(kernel_ms, 4)},
        "roofline": {"bound": "valu_fp64", "achieved": round(F / (kernel_ms * 1e-3) / 1e12, 4), "peak": FP64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(F / (kernel_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 6),
                     "traffic": None, "note": "track_kernel of one closed-loop step; SURVEY §8(d) flop formula"},
    }
    if args.cpu_budget > 0 and world == 1:
        out["cpu_baseline"] = sim_cpu_baseline(S, U, g["obstacles"], x0, N, params, args.cpu_budget)
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


def sim_cpu_baseline(S, U, obstacles, x0, N, params, budget_s):
    """The oracle's restatement of the simulation.py loop (C IPM per step, numpy plant), OpenMP over
    instances, on a bounded sample."""
    import numpy as np

    from oracle import c_oracle as co
    from oracle import ttmpc_oracle as to
    from ttmpc import layout
    threads, ncores = cpu_threads()
    nlp = to.TrackingNLP(N)
    P = co.make_problem(N, params, nlp.Q, nlp.R, nlp.xlb, nlp.xub, nlp.ulb, nlp.uub)

    def solve(x, Xr, Ur):
        z, st, _, _ = co.solve_batch(P, x, Xr, Ur, nthreads=threads)
        X, Uo = layout.unpack(z, N)
        return X, Uo, st
    Bs = min(len(x0), 16 * threads)
    rng = np.random.default_rng(0)
    done, t0, T = 0, time.perf_counter(), 0.5
    while True:
        K = len(to.step_indices(T, 0.05))
        noise = rng.normal(scale=0.02, size=(K, Bs, 6))
        to.closed_loop(solve, x0[:Bs], S, U, N, T, params, to.DISTURBANCE_PARAMS, noise)
        done += K * Bs
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": done / el, "unit": "instance-steps/s", "cores": threads, "kind": "port",
            "host_cores_visible": ncores,
            "sample": f"{done} instance-steps ({Bs} instances x {T}s loops) in {el:.1f}s; oracle closed loop "
                      f"(oracle/ttmpc_oracle.closed_loop + oracle/c/tt_oracle.c), OpenMP {threads} threads"}


def obca_flops(N, M, iters):
    """SURVEY §8(d) C4 formula per KKT solve: F_ric,obca = (N+1) [M (16^3/3 + 2*16^2*6 + 16*6^2) + F_ric],
    plus the linearisation and forward sweep of the tracking formula; one KKT solve per iteration."""
    F_ric_stage = 1539
    per_kkt = (N + 1) * (M * (16 ** 3 / 3 + 2 * 16 ** 2 * 6 + 16 * 6 ** 2) + F_ric_stage) + N * (152 + 120)
    F_lin = (N + 1) * (160 + 2 * M * 60)
    return (iters + 1) * F_lin + iters * per_kkt


def main_obca(args):
    """OBCA configs: one step = one launch solving B independent OBCA NLPs with the restated IPOPT
    (reference duals mu = 100 / lam pattern, tol 1e-8, max_iter 5000, restoration phase).
    c4      : BASELINE configs[3] as SURVEY §8(d) defines it -- TrajectoryOptimization, 6 obstacle rectangles
              (obstacles.json[0:6]), N=200, dt=0.1, B=256 = test_cases.json cases x Monte-Carlo start
              perturbations, each with the reference's 2-waypoint initialize.json guess (apply_case.py:16-34,
              trajectory_optimization.py:227-274).  Three of the 7 cases (baseline_hybrid_path,
              diagonal_reverse_cross_aisle, angle_test) put the start or the goal pose inside an obstacle of
              that set: their NLPs are infeasible, so c4 draws from the 4 others (perturbed starts that land in
              an obstacle are redrawn) and c4all keeps all 7 (infeasible ones reported separately).
    c4replan: the same planner on re-plans around the reference's committed IPOPT plan (data/state_traj.txt
              subsampled to 8 Hybrid-A*-style waypoints, start perturbed).
    cobs    : MPCTrackingControlObs as simulation.py drives it (N=50, dt=0.05, all 11 obstacles), windows of
              the interpolated plan with perturbed initial states (redrawn while closer than d_min to an
              obstacle: a start inside an obstacle is an infeasible NLP)."""
    import numpy as np

    import ttmpc
    from ttmpc import scenarios as sc
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = local_device()
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    g = np.load(REPO / "tests" / "golden" / "reference_numpy.npz")
    obs_all = sc.obstacles_array(sc.load_obstacles(REPO / "tests" / "golden" / "obstacles.json"))
    blocked = None
    if args.config in ("c4", "c4all", "c4replan"):
        B, N, M = args.batch or 256, args.horizon or 200, 6
        obs = obs_all[:M]
        if args.config in ("c4", "c4all"):
            cases = json.loads((REPO / "tests" / "golden" / "test_cases.json").read_text())["cases"]
            x0, xg, zg = sc.obca_case_batch(cases, B, N, M, seed=rank_seed(rank),
                                            obstacles=obs if args.config == "c4" else None, params=sc.OBCA_PARAMS)
            blocked = sc.blocked_poses(x0, obs, sc.OBCA_PARAMS) | sc.blocked_poses(xg, obs, sc.OBCA_PARAMS)
        else:
            x0, xg, zg = sc.obca_replan_batch(g["state_traj"], B, N, M, seed=rank_seed(rank))
        params, bnd = sc.OBCA_PARAMS, (sc.OBCA_XLB, sc.OBCA_XUB, sc.OBCA_ULB, sc.OBCA_UUB)
        variant, xr, ur = ttmpc.TT_VARIANT_OBCA_PLAN, None, None
    else:
        B, N = args.batch or 256, args.horizon or 50
        obs = g["obstacles"]
        M = obs.shape[0]
        x0, xr, ur = sc.mpc_obs_batch(g["state_traj"], g["input_traj"], B, N, seed=rank_seed(rank), obstacles=obs)
        params, bnd = dict(sc.OBCA_PARAMS, dt=0.05), (sc.XLB, sc.XUB, sc.ULB, sc.UUB)
        variant, xg, zg = ttmpc.TT_VARIANT_TRACK_OBCA, None, None
    solver = ttmpc.ObcaSolver(N, params, sc.OBCA_Q, sc.OBCA_R, *bnd, obs, variant=variant, max_iter=args.max_iter,
                              device=local)
    n = ttmpc.obca_n(N, M)
    T = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_x0, d_xg, d_zg, d_xr, d_ur = T(x0), T(xg), T(zg), T(xr), T(ur)
    X = torch.empty((B, N + 1, 6), dtype=torch.float64, device=dev)
    U = torch.empty((B, N, 2), dtype=torch.float64, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    it = torch.empty(B, dtype=torch.int32, device=dev)
    kk = torch.empty(B, dtype=torch.float64, device=dev)
    stream = torch.cuda.Stream(dev)
    ptr = lambda a: 0 if a is None else a.data_ptr()  # noqa: E731

    def step():
        solver.solve_device(B, ptr(d_x0), ptr(d_xg), ptr(d_xr), ptr(d_ur), ptr(d_zg), X.data_ptr(), U.data_ptr(), 0,
                            st.data_ptr(), it.data_ptr(), kk.data_ptr(), stream=stream.cuda_stream)

    torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    kernel_ms = e0.elapsed_time(e1) / args.steps
    status, iters = st.cpu().numpy(), it.cpu().numpy()
    ok = int(np.sum(status <= 1))
    wall_max, ok_total, B_total = reduce_over_ranks(dist, wall, ok, B)
    if rank != 0:
        dist.destroy_process_group()
        return
    F = float(np.sum(obca_flops(N, M, iters.astype(np.float64))))
    achieved = F / (kernel_ms * 1e-3) / 1e12
    name = {"c4": "c4: TrajectoryOptimization OBCA plans of the 4 collision-free test_cases.json cases x start "
                  "perturbations (2-waypoint initialize.json guess)",
            "c4all": "c4all: TrajectoryOptimization OBCA plans of all 7 test_cases.json cases x start perturbations "
                     "(2-waypoint initialize.json guess; 3 cases infeasible)",
            "c4replan": "c4replan: TrajectoryOptimization re-plans around the committed plan (8-waypoint guess)",
            "cobs": "cobs: MPC+OBCA (MPCTrackingControlObs) windows"}[args.config]
    solver_rec = {"converged_or_acceptable": ok_total, "instances": B_total,
                  "status_counts": {str(k): int(v) for k, v in zip(*np.unique(status, return_counts=True))},
                  "iters_mean": float(iters.mean()), "iters_p50": float(np.median(iters)),
                  "iters_max": int(iters.max()), "kernel_ms_per_launch": round(kernel_ms, 3)}
    if blocked is not None:
        solver_rec["infeasible_by_construction"] = int(blocked.sum())
        solver_rec["converged_of_feasible"] = f"{int(np.sum((status <= 1) & ~blocked))}/{int(np.sum(~blocked))}"
    census = REPO / "tests" / "golden" / "c4_census.json"
    if args.config == "c4" and (B, N, M, rank_seed(rank)) == (256, 200, 6, 7) and census.exists():
        # instance-by-instance agreement with the oracle census of this exact batch (tests/golden/make_c4_census.py): which
        # failures the restated IPOPT shares (its behaviour) and which are the kernel's alone (drift)
        cen = json.loads(census.read_text()).get("bench")
        if cen and cen.get("B") == B:
            stc = np.asarray(cen["status"])
            solver_rec["oracle_census"] = {
                "oracle_status_counts": {str(k): int(v) for k, v in zip(*np.unique(stc, return_counts=True))},
                "equal_status": int((status == stc).sum()),
                "shared_failures": np.flatnonzero((status > 1) & (stc > 1)).tolist(),
                "kernel_only_failures": np.flatnonzero((status > 1) & (stc <= 1)).tolist(),
                "oracle_only_failures": np.flatnonzero((status <= 1) & (stc > 1)).tolist(),
                "source": "tests/golden/c4_census.json (oracle/c/tt_obca.c on the same seeded batch)"}
            if "rounding_sensitive" in cen:
                # round 6: the census re-solves the batch under three one-ulp-class perturbations of the guess; a status
                # disagreement on an instance whose oracle outcome does not move under them was checked against the
                # kernel's own perturbed runs (tests/test_gpu_obca.py::test_c4_bench_batch_against_census)
                sens = np.asarray(cen["rounding_sensitive"], dtype=bool)
                solver_rec["oracle_census"]["oracle_rounding_sensitive"] = int(sens.sum())
                solver_rec["oracle_census"]["status_mismatch_not_oracle_sensitive"] = \
                    np.flatnonzero((status != stc) & ~sens).tolist()
    traffic, traffic_src, traffic_est = obca_traffic(args.config, float(iters.sum()))
    out = {
        "metric": f"OBCA {'plan' if args.config != 'cobs' else 'MPC+OBCA'} solves/sec (N={N}, M={M} obstacles, "
                  f"n={n} variables; converged or acceptable solves only)",
        "value": round(ok_total * args.steps / wall_max, 3),
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "the reference's scenario files (test_cases.json / obstacles.json / data/state_traj.txt) with seeded "
                "Monte-Carlo perturbations",
        "config": {"workload": f"{name}, B={B}/GPU, N={N}, M={M}, IPOPT tol 1e-8, max_iter {args.max_iter}, "
                               "reference dual start, restoration phase",
                   "batch_per_gpu": B, "horizon": N, "obstacles": M,
                   "parallelism": f"dp{world} (independent instance shards)"},
        "solver": solver_rec,
        "roofline": {"bound": "valu_fp64", "achieved": round(achieved, 5), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / FP64_PEAK_TFLOPS, 7), "traffic": traffic, "traffic_source": traffic_src,
                     "traffic_estimated": traffic_est,
                     "note": "latency-bound (serial Riccati over N stages per instance, one workgroup per instance); "
                             "flops: SURVEY §8(d) C4 block-arrow formula x per-instance iterations"},
    }
    if args.cpu_budget > 0 and world == 1:
        out["cpu_baseline"] = obca_cpu_baseline(args.config, N, M, params, bnd, obs, x0, xg, xr, ur, zg, args.max_iter,
                                                args.cpu_budget)
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


def obca_cpu_baseline(cfg, N, M, params, bnd, obs, x0, xg, xr, ur, zg, max_iter, budget_s):
    """The oracle on rounds of `threads` consecutive instances (every case of the batch is represented in the
    first round) until the budget is spent; a round always finishes, so a round of long solves can exceed it."""
    import numpy as np

    from oracle import c_oracle as co
    from ttmpc import scenarios as sc
    threads, ncores = cpu_threads()
    P = co.make_obca_problem(N, params, sc.OBCA_Q, sc.OBCA_R, *bnd, obs, mode=1 if cfg == "cobs" else 0,
                             max_iter=max_iter)
    done, solved, t0 = 0, 0, time.perf_counter()
    B = x0.shape[0]
    while True:
        lo = done % B
        hi = min(B, lo + threads)
        sl = slice(lo, hi)
        _, st, _, _ = co.obca_solve_batch(P, x0[sl], None if xg is None else xg[sl], None if xr is None else xr[sl],
                                          None if ur is None else ur[sl], None if zg is None else zg[sl],
                                          nthreads=threads)
        done += hi - lo
        solved += int(np.sum(st <= 1))
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": solved / el, "unit": "solves/s", "cores": threads, "kind": "port", "host_cores_visible": ncores,
            "sample": f"{done} instances ({solved} solved) of the same {cfg} workload in {el:.1f}s, OpenMP {threads} "
                      f"threads on {ncores} visible host cores; oracle/c/tt_obca.c (same restated IPOPT)"}


# rocprofv3 PMC passes (tools/hbm_passes.sh) that the default C2 / C3 lines quote as roofline.traffic: the kernel
# the bench runs; re-profile after a tracking-kernel change
TRACK_PMC = {"c2": "profiles/r06/final_head/pmc_track_c2", "c3": "profiles/r06/final_head/pmc_track_c3"}
TRACK_PMC_SOURCE = "profiles/r06/final_head/SOURCE.txt"


# committed PMC passes of obca_kernel (FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs, tools/gpu_session.sh hbm:CFG).
# Round 6: passes over ONE FULL launch of each config's own bench batch -- when a launch runs the same IPM iterations
# (deterministic: it does), roofline.traffic is that launch's measured bytes (traffic_estimated false); otherwise the
# pass's bytes per instance-iteration are scaled by the launch's summed iterations (traffic_estimated true)
OBCA_PMC = {"c4": "profiles/r06/final/pmc_obca_c4", "c4all": "profiles/r06/final/pmc_obca_c4all",
            "cobs": "profiles/r06/final/pmc_obca_cobs"}


def obca_traffic(cfg, iters_sum):
    """-> (HBM bytes per launch, source text, estimated?)"""
    d = OBCA_PMC.get(cfg)
    if d is None or not (REPO / d / "fetch" / "fetch_counter_collection.csv").exists():
        return None, None, None
    per_launch = read_traffic([REPO / d / "fetch" / "fetch_counter_collection.csv",
                               REPO / d / "write" / "write_counter_collection.csv"], kernel="obca_kernel")
    rec = json.loads((REPO / d / "fetch.bench.json").read_text())["solver"]
    if per_launch is None:
        return None, None, None
    pass_iters = rec["iters_mean"] * rec["instances"]
    per_iter = per_launch / pass_iters
    if abs(pass_iters - iters_sum) < 0.5:
        src = (f"{d}: 2 x FETCH_SIZE + WRITE_SIZE of one full obca_kernel launch of this batch (the same "
               f"{int(iters_sum)} instance-iterations) = {per_launch / 1e9:.1f} GB, {per_iter / 1e6:.2f} MB per "
               "instance-iteration")
        return round(per_launch, 1), src, False
    src = (f"{d}: 2 x FETCH_SIZE + WRITE_SIZE of obca_kernel = {per_launch / 1e9:.1f} GB over "
           f"{rec['instances']} x {rec['iters_mean']:.2f} instance-iterations = {per_iter / 1e6:.2f} MB per "
           f"instance-iteration, x this launch's {int(iters_sum)} instance-iterations")
    return round(per_iter * iters_sum, 1), src, True


def read_traffic(paths, kernel="track_kernel"):
    """HBM bytes per dispatch of `kernel` = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes), averaged over
    the dispatches in rocprofv3 --pmc counter_collection CSVs (FETCH_SIZE and WRITE_SIZE need separate
    passes on gfx950).  The x2 on FETCH_SIZE is the gfx950 correction of MI355X_MICROARCH.md; it was
    re-calibrated for this kernel's 8-B/lane loads with tools/calib_fetch.hip (1 GiB read -> 524,299 KB
    FETCH_SIZE; 1 GiB written -> 1,048,576 KB WRITE_SIZE; profiles/r01/calib/)."""
    import csv
    acc = {"FETCH_SIZE": [], "WRITE_SIZE": []}
    for path in paths:
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") in acc:
                    acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not acc["FETCH_SIZE"] or not acc["WRITE_SIZE"]:
        return None
    return round(1024 * (2.0 * sum(acc["FETCH_SIZE"]) / len(acc["FETCH_SIZE"]) +
                         sum(acc["WRITE_SIZE"]) / len(acc["WRITE_SIZE"])), 1)


if __name__ == "__main__":
    main()
