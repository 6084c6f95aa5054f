#!/bin/bash
# OBCA measurement pass of one commit on one GPU box: PMC HBM passes (c4 and cobs, 300 IPM iterations, separate
# FETCH_SIZE / WRITE_SIZE runs), then the c4 / cobs / c4all bench lines.  Each step prints when it finishes.
# usage (GPU box): bash tools/gpu_obca_final.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/obca_final}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/obca_pmc.sh "$OUT/pmc_c4" c4 300 hbm || exit 1
bash tools/obca_pmc.sh "$OUT/pmc_cobs" cobs 300 hbm || exit 1
for cfg in c4 cobs c4all; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 1 --warmup 1 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; tail -5 "$OUT/bench_$cfg.err"; exit 1; }
  echo "done $cfg"; cat "$OUT/bench_$cfg.json"
done
echo OBCA_FINAL_DONE
