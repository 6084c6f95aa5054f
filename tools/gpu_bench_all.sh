#!/bin/bash
# Every bench config once on one MI355X (GPU box): bench lines + rocprofv3 kernel stats of the OBCA C4 run.
# usage: bash tools/gpu_bench_all.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/bench_all}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in c2 c3 c5 sim; do
  timeout -k 10 300 python -u bench.py --config $cfg > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; exit 1; }
  echo done $cfg
done
for cfg in c4 cobs c4replan c4all; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 1 --warmup 1 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; exit 1; }
  echo done $cfg
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/ks_c4" -o ks --output-format csv -- python3 bench.py --config c4 --steps 1 --warmup 1 --cpu-budget 0 > "$OUT/ks_c4.log" 2>&1 || { echo KSTATS_FAILED; exit 1; }
echo ALL_DONE
