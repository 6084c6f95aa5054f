#!/bin/bash
# End-of-round measurement pass on one GPU: GPU tests, every bench config with its rocprof kernel stats,
# HBM / SQ counter passes of the default bench.   usage (GPU box): bash tools/gpu_final.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/final}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
bench() {
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { echo "BENCH_FAILED $name"; tail -20 "$OUT/bench_$name.err"; exit 1; }
  head -c 300 "$OUT/bench_$name.json"; echo
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$name" -o run --output-format csv \
    -- python3 bench.py "$@" --cpu-budget 0 --no-latency > "$OUT/prof_$name.log" 2>&1 || { echo "PROF_FAILED $name"; tail -20 "$OUT/prof_$name.log"; exit 1; }
}
bench c2
bench c3 --config c3 --steps 10 --warmup 2 --cpu-budget 10
bench c5 --config c5 --steps 5 --warmup 1 --cpu-budget 8
bench sim --config sim --steps 40 --warmup 5 --cpu-budget 8
bench c4 --config c4 --steps 3 --warmup 1
bench cobs --config cobs --steps 3 --warmup 1
bash tools/hbm_passes.sh "$OUT/hbm" || exit 1
echo FINAL_DONE
