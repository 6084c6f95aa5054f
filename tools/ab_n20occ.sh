#!/bin/bash
# A/B of the N = 20 large-batch build (C5 config, one GPU): shipped stage-unrolled occupancy build vs round 2's generic
# occupancy build (TT_N20_OCC=1) vs no occupancy build (TT_N20_OCC=2).   usage (GPU box): bash tools/ab_n20occ.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/n20occ}
mkdir -p "$OUT"
V=$PWD/car-trailer-mpc_amd/ttmpc/variants
for r in 1 2; do
  for v in new occ1 occ2; do
    if [ $v = new ]; then L=""; else L="TTMPC_LIB=$V/libttmpc_$v.so"; fi
    env $L timeout -k 10 120 python bench.py --config c5 --steps 10 --warmup 2 --cpu-budget 0 --no-latency > "$OUT/${v}_c5_$r.json" || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/${v}_c5_$r.json')); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
