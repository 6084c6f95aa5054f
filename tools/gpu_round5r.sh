#!/bin/bash
# Round-5 GPU session R: A/B of the batched-trial width (OBCA_TRIAL_BATCH 2 / 3 / 4 (in-tree) / 6) on the C4 bench.
# usage: bash tools/gpu_round5r.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5r}
mkdir -p "$OUT"
V=car-trailer-mpc_amd/ttmpc/variants
export TMPDIR=/tmp
for spec in nb4= nb2=$V/libttmpc_nb2.so nb3=$V/libttmpc_nb3.so nb6=$V/libttmpc_nb6.so nb4b=; do
  name=${spec%%=*}; so=${spec#*=}
  TTMPC_LIB=$so timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --cpu-budget 0 > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { echo BENCH_FAILED $name; tail -5 "$OUT/bench_$name.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$name.json')); s=d.get('solver', {}); print('$name', d['value'], d['ms_per_step'], s.get('status_counts'))"
done
echo R5R_DONE
