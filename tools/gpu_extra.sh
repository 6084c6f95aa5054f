#!/bin/bash
# C5 sharded path (one rank) and the closed-loop Monte-Carlo bench, each with rocprofv3 kernel stats.
# usage (GPU box): bash tools/gpu_extra.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/extra}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --cpu-budget 8 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { echo BENCH_FAILED c5; tail -20 "$OUT/bench_c5.err"; exit 1; }
cat "$OUT/bench_c5.json"
timeout -k 10 300 python bench.py --config sim --steps 40 --warmup 5 --cpu-budget 8 > "$OUT/bench_sim.json" 2> "$OUT/bench_sim.err" || { echo BENCH_FAILED sim; tail -20 "$OUT/bench_sim.err"; exit 1; }
cat "$OUT/bench_sim.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_sim" -o run --output-format csv \
  -- python3 bench.py --config sim --steps 40 --warmup 5 --cpu-budget 0 > "$OUT/prof_sim.log" 2>&1 || { echo PROF_FAILED sim; tail -20 "$OUT/prof_sim.log"; exit 1; }
find "$OUT/prof_sim" -name '*kernel_stats.csv' -exec cat {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv \
  -- python3 bench.py --config c5 --steps 5 --warmup 1 --cpu-budget 0 > "$OUT/prof_c5.log" 2>&1 || { echo PROF_FAILED c5; tail -20 "$OUT/prof_c5.log"; exit 1; }
find "$OUT/prof_c5" -name '*kernel_stats.csv' -exec cat {} \;
echo EXTRA_DONE
