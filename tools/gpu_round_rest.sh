#!/bin/bash
# Second half of the round measurement pass (GPU box): every -m gpu test, then the bench lines of the
# non-headline configs (C5, closed loop, OBCA c4 / cobs / c4replan / c4all) and rocprof kernel stats of c4.
# usage: bash tools/gpu_round_rest.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/rest}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
for cfg in c5 sim; do
  timeout -k 10 300 python -u bench.py --config $cfg > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; exit 1; }
  echo done $cfg
done
for cfg in c4 cobs c4replan c4all; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 1 --warmup 1 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; exit 1; }
  echo done $cfg
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/ks_c4" -o ks --output-format csv -- python3 bench.py --config c4 --steps 1 --warmup 1 --cpu-budget 0 > "$OUT/ks_c4.log" 2>&1 || { echo KSTATS_FAILED; exit 1; }
echo ALL_DONE
