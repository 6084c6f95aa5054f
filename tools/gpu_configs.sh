#!/bin/bash
# Tracking configs C3 (B=8192, N=40, psi stress) and C5 shard (B=8192/GPU, test_cases.json) on one GPU:
# bench line + rocprofv3 kernel stats of each.   usage (GPU box): bash tools/gpu_configs.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/configs}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --cpu-budget 10 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { echo BENCH_FAILED $c; tail -20 "$OUT/bench_$c.err"; exit 1; }
  cat "$OUT/bench_$c.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv \
    -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-budget 0 --no-latency > "$OUT/prof_$c.log" 2>&1 || { echo PROF_FAILED $c; tail -20 "$OUT/prof_$c.log"; exit 1; }
  find "$OUT/prof_$c" -name '*kernel_stats.csv' -exec cat {} \;
done
echo CONFIGS_DONE
