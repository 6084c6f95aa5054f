#!/bin/bash
# One GPU verification pass: gpu tests, default bench, rocprof kernel stats of the bench.
# usage (GPU box): bash tools/gpu_check.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAILED; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 3 --cpu-budget 0 --no-latency > "$OUT/prof.log" 2>&1 || { echo PROF_FAILED; tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \;
echo CHECK_DONE
