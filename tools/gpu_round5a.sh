#!/bin/bash
# Round-5 GPU session A (GPU box): the GPU test suite with the restated convergence test, the headline bench + rocprof
# stats, tracking phase stamps, the C5 one-chunk shapes, the OBCA bench configs and the C4 tail accounting.
#   usage: bash tools/gpu_round5a.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5a}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1; rc=$?
  echo "gpu tests rc=$rc"; tail -4 "$OUT/gpu_tests.log"; grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -10
  [ $rc -le 1 ] || exit 1
fi
timeout -k 10 300 python bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { echo BENCH_FAILED; tail -20 "$OUT/bench_c2.err"; exit 1; }
cat "$OUT/bench_c2.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 3 --cpu-budget 0 --no-latency > "$OUT/prof_c2.log" 2>&1 || { echo PROF_FAILED; tail -20 "$OUT/prof_c2.log"; exit 1; }
find "$OUT/prof_c2" -name '*kernel_stats.csv' -exec head -3 {} \;
timeout -k 10 120 python -u tools/phase_stamps.py 1024 20 > "$OUT/track_stamps.txt" 2>&1 || { echo TSTAMPS_FAILED; tail -5 "$OUT/track_stamps.txt"; exit 1; }
cat "$OUT/track_stamps.txt"
for spec in "c5:" "c5_8192x1:--batch 8192 --chunks 1" "c3:"; do
  name=${spec%%:*}; a=${spec#*:}
  cfg=${name%%_*}
  timeout -k 10 300 python -u bench.py --config $cfg $a --cpu-budget 0 --no-latency > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { echo "BENCH_FAILED $name"; tail -10 "$OUT/bench_$name.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', d['value'], d['ms_per_step'], d['config']['workload'][-60:])"
done
for cfg in c4 cobs c4replan c4all; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 1 --warmup 1 --cpu-budget 0 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; tail -10 "$OUT/bench_$cfg.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d.get('solver', {}))"
done
timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 "$OUT/tail.npz" > "$OUT/tail.txt" 2>&1 || { echo TAIL_FAILED; tail -5 "$OUT/tail.txt"; exit 1; }
cat "$OUT/tail.txt"
echo R5A_DONE
