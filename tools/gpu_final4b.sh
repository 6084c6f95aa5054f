#!/bin/bash
# Round-4 final measurement, part B (GPU box): the OBCA bench lines (C4, C4 re-plan, all cases, MPC+OBCA windows)
# with rocprofv3 kernel stats of C4, the OBCA PMC HBM passes (300-iteration probes), and the C4 tail accounting.
# usage: bash tools/gpu_final4b.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/final4b}
mkdir -p "$OUT"
export TMPDIR=/tmp
bench() {
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { echo "BENCH_FAILED $name"; tail -20 "$OUT/bench_$name.err"; exit 1; }
  head -c 400 "$OUT/bench_$name.json"; echo
}
bench c4 --config c4 --steps 3 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o run --output-format csv \
  -- python3 bench.py --config c4 --steps 2 --warmup 0 --cpu-budget 0 --no-latency > "$OUT/prof_c4.log" 2>&1 || { echo PROF_FAILED; tail -20 "$OUT/prof_c4.log"; exit 1; }
bench c4replan --config c4replan --steps 3 --warmup 1
bench cobs --config cobs --steps 3 --warmup 1
bench c4all --config c4all --steps 2 --warmup 1
for cfg in c4 c4all cobs; do
  bash tools/obca_pmc.sh "$OUT/pmc_$cfg" $cfg 300 hbm > "$OUT/pmc_$cfg.log" 2>&1 || { echo "PMC_FAILED $cfg"; tail -5 "$OUT/pmc_$cfg.log"; exit 1; }
done
timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 "$OUT/tail.npz" > "$OUT/tail.txt" 2>&1 || { echo TAIL_FAILED; tail -5 "$OUT/tail.txt"; exit 1; }
head -30 "$OUT/tail.txt"
echo FINAL4B_DONE
