#!/bin/bash
# Round-4 final measurement, part A (GPU box): every GPU test, the tracking bench lines (C2 headline, C3, C5 and
# its 8-rank shard shape, closed loop) with rocprofv3 kernel stats, and the C2 / C3 PMC passes.
# usage: bash tools/gpu_final4a.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/final4a}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
tail -2 "$OUT/gpu_tests.log"; grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head
[ $rc -le 1 ] || exit 1
bench() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { echo "BENCH_FAILED $name"; tail -20 "$OUT/bench_$name.err"; exit 1; }
  head -c 400 "$OUT/bench_$name.json"; echo
}
kstats() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$name" -o run --output-format csv \
    -- python3 bench.py "$@" --cpu-budget 0 --no-latency > "$OUT/prof_$name.log" 2>&1 || { echo "PROF_FAILED $name"; tail -20 "$OUT/prof_$name.log"; exit 1; }
}
bench c2
kstats c2 --steps 20 --warmup 3
bench c3 --config c3 --steps 10 --warmup 2 --cpu-budget 10
kstats c3 --config c3 --steps 10 --warmup 2
bench c5 --config c5 --steps 5 --warmup 1 --cpu-budget 8
bench c5_8192x2 --config c5 --batch 8192 --chunks 2 --steps 10 --warmup 2 --cpu-budget 0 --no-latency
bench sim --config sim --steps 40 --warmup 5 --cpu-budget 8
bash tools/hbm_passes.sh "$OUT/pmc_c2" c2 > "$OUT/pmc_c2.log" 2>&1 || { echo PMC_C2_FAILED; tail -5 "$OUT/pmc_c2.log"; exit 1; }
bash tools/hbm_passes.sh "$OUT/pmc_c3" c3 > "$OUT/pmc_c3.log" 2>&1 || { echo PMC_C3_FAILED; tail -5 "$OUT/pmc_c3.log"; exit 1; }
echo FINAL4A_DONE
