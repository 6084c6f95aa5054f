#!/bin/bash
# Round-5 GPU session AA: the two-wave N = 20 build with zL / zU in registers and a 102-row stage record (8 instances per
# CU instead of 7).  Tracking A/B against head (bitwise dumps, C2 / C3 / C5, the tracking GPU tests) and the 8,192 shard.
# usage: bash tools/gpu_round5aa.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5aa}
mkdir -p "$OUT"
V=car-trailer-mpc_amd/ttmpc/variants
export TMPDIR=/tmp
bash tools/gpu_track_ab2.sh "$OUT" head new | grep -v "^$" | grep -vE "^(sub|load|linearize|mu\+|riccati|forward|step|merit|soc|update|#)" | tail -30 || exit 1
for r in 1 2; do
  for spec in head=$V/libttmpc_head.so new=; do
    name=${spec%%=*}; so=${spec#*=}
    TTMPC_LIB=$so timeout -k 10 300 python -u bench.py --config c5 --batch 8192 --chunks 1 --cpu-budget 0 --no-latency > "$OUT/c5s_${name}_$r.json" 2> "$OUT/c5s_${name}_$r.err" || { echo BENCH_FAILED $name; tail -5 "$OUT/c5s_${name}_$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/c5s_${name}_$r.json')); print('c5 8192x1 $name $r', d['value'], d['ms_per_step'])"
  done
done
echo R5AA_DONE
