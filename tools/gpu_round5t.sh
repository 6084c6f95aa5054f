#!/bin/bash
# Round-5 GPU session T: the full GPU test suite on the current kernels, the default bench (C2) with the rocprof
# summary, the OBCA bench configs, B = 1 OBCA plan latency with / without helpers.   usage: bash tools/gpu_round5t.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5t}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -10
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/obca_plan_latency.py 3 > "$OUT/plan_latency.txt" 2>&1 || { echo LAT_FAILED; tail -5 "$OUT/plan_latency.txt"; exit 1; }
cat "$OUT/plan_latency.txt"
for cfg in c4 cobs c4replan c4all; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 1 --warmup 1 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; tail -10 "$OUT/bench_$cfg.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$cfg.json')); s=d.get('solver', {}); print('$cfg', d['value'], d['ms_per_step'], s.get('status_counts'), s.get('oracle_census', {}).get('equal_status'))"
done
echo R5T_DONE
