#!/bin/bash
# Round-5 GPU session N: the full GPU test suite on the helper-workgroup OBCA kernel, then the OBCA bench configs and
# the C4 tail profile (iterations 4,000-5,000, tools/obca_tail.py).   usage: bash tools/gpu_round5n.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5n}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -10
grep -A3 "C4 census comparison" "$OUT/gpu_tests.log" | head -5
[ $rc -le 1 ] || exit 1
for cfg in c4 cobs c4replan c4all; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 1 --warmup 1 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; tail -10 "$OUT/bench_$cfg.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$cfg.json')); s=d.get('solver', {}); print('$cfg', d['value'], d['ms_per_step'], s.get('status_counts'), s.get('oracle_census', {}).get('equal_status'))"
done
echo R5N_DONE
