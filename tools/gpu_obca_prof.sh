#!/bin/bash
# OBCA measurement pass on the GPU box: c4 / cobs bench lines + rocprofv3 kernel stats of each.
# usage (GPU box): bash tools/gpu_obca_prof.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/obca}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in c4 cobs; do
  timeout -k 10 400 python bench.py --config $c --steps 3 --warmup 1 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { echo BENCH_FAILED $c; tail -20 "$OUT/bench_$c.err"; exit 1; }
  cat "$OUT/bench_$c.json"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv \
    -- python3 bench.py --config $c --steps 2 --warmup 1 --cpu-budget 0 > "$OUT/prof_$c.log" 2>&1 || { echo PROF_FAILED $c; tail -20 "$OUT/prof_$c.log"; exit 1; }
  find "$OUT/prof_$c" -name '*kernel_stats.csv' -exec cat {} \;
done
echo OBCA_DONE
