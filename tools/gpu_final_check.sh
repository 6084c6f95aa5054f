#!/bin/bash
# Final check of HEAD on one GPU: every -m gpu test, smoke(), the default bench line and its rocprof stats.
# usage (GPU box): bash tools/gpu_final_check.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/final_check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo SMOKE_FAILED; tail -20 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAILED; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 3 --cpu-budget 0 --no-latency > "$OUT/prof.log" 2>&1 || { echo PROF_FAILED; tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \;
echo FINAL_CHECK_DONE
