#!/bin/bash
# Round-4 GPU session B (GPU box): the full GPU test suite, the headline bench + rocprof stats, the C5 launch shapes,
# the OBCA bench configs and the C4 tail accounting.   usage: bash tools/gpu_round4b.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r4b}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
  echo "gpu tests rc=$rc"; tail -4 "$OUT/gpu_tests.log"; grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -10
  [ $rc -le 1 ] || exit 1
fi
bash tools/ab_obca.sh "$OUT/ab_prep" noprep=$PWD/car-trailer-mpc_amd/ttmpc/variants/libttmpc_noprep.so fuse= > "$OUT/ab_prep.log" 2>&1 || { echo AB_FAILED; tail -5 "$OUT/ab_prep.log"; exit 1; }
grep -A8 "compare_fuse" "$OUT/ab_prep.log"; grep -E "TOTAL|corrections" "$OUT/ab_prep.log"
timeout -k 10 300 python bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { echo BENCH_FAILED; tail -20 "$OUT/bench_c2.err"; exit 1; }
cat "$OUT/bench_c2.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 3 --cpu-budget 0 --no-latency > "$OUT/prof_c2.log" 2>&1 || { echo PROF_FAILED; tail -20 "$OUT/prof_c2.log"; exit 1; }
find "$OUT/prof_c2" -name '*kernel_stats.csv' -exec head -3 {} \;
timeout -k 10 120 python -u tools/phase_stamps.py 1024 20 > "$OUT/track_stamps.txt" 2>&1 || { echo TSTAMPS_FAILED; tail -5 "$OUT/track_stamps.txt"; exit 1; }
cat "$OUT/track_stamps.txt"
for spec in "c5:" "c5_8192x1:--batch 8192 --chunks 1" "c5_8192x2:--batch 8192 --chunks 2" "c5_8192x4:--batch 8192 --chunks 4" "c5_65536x1:--chunks 1"; do
  name=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python -u bench.py --config c5 $a --cpu-budget 0 --no-latency > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { echo "BENCH_FAILED $name"; tail -10 "$OUT/bench_$name.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', d['value'], d['ms_per_step'], d['config']['workload'][-60:])"
done
for cfg in c4 cobs c4replan c4all; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 1 --warmup 1 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; tail -10 "$OUT/bench_$cfg.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d.get('solver', {}))"
done
timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 "$OUT/tail.npz" > "$OUT/tail.txt" 2>&1 || { echo TAIL_FAILED; tail -5 "$OUT/tail.txt"; exit 1; }
cat "$OUT/tail.txt"
echo R4B_DONE
