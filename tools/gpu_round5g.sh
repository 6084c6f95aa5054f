#!/bin/bash
# Round-5 GPU session: the full GPU test suite, then the tracking configs (C2 + rocprof stats, C3, C5, the 8,192-instance
# shard) and the tracking phase stamps.   usage: bash tools/gpu_round5g.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5g}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -10
grep -A3 "C4 census comparison" "$OUT/gpu_tests.log" | head -5
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { echo BENCH_FAILED; tail -20 "$OUT/bench_c2.err"; exit 1; }
cat "$OUT/bench_c2.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 3 --cpu-budget 0 --no-latency > "$OUT/prof_c2.log" 2>&1 || { echo PROF_FAILED; tail -20 "$OUT/prof_c2.log"; exit 1; }
find "$OUT/prof_c2" -name '*kernel_stats.csv' -exec head -3 {} \;
for spec in "c3:" "c5:" "c5_8192x1:--batch 8192 --chunks 1"; do
  name=${spec%%:*}; a=${spec#*:}
  cfg=${name%%_*}
  timeout -k 10 300 python -u bench.py --config $cfg $a --cpu-budget 0 --no-latency > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { echo "BENCH_FAILED $name"; tail -10 "$OUT/bench_$name.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', d['value'], d['ms_per_step'], d['solver'].get('kernel_ms_per_launch'))"
done
timeout -k 10 120 python -u tools/phase_stamps.py 1024 20 > "$OUT/track_stamps.txt" 2>&1 || { echo TSTAMPS_FAILED; tail -5 "$OUT/track_stamps.txt"; exit 1; }
cat "$OUT/track_stamps.txt"
echo R5G_DONE
