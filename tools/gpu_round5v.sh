#!/bin/bash
# Round-5 GPU session V: the round-4 final kernels (variant r4, commit e4c819e) against the current tree on the tracking
# configs and the closed loop, 2 alternating rounds (what round 5 changed in the tracking kernel, on one box).
# usage: bash tools/gpu_round5v.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5v}
mkdir -p "$OUT"
V=car-trailer-mpc_amd/ttmpc/variants
export TMPDIR=/tmp
for r in 1 2; do
  for spec in cur= r4=$V/libttmpc_r4.so; do
    name=${spec%%=*}; so=${spec#*=}
    for cfg in c2 c3 sim; do
      extra="--cpu-budget 0"; [ $cfg = sim ] && extra="--steps 40 --warmup 5 --cpu-budget 0"; [ $cfg != sim ] && extra="$extra --no-latency"
      TTMPC_LIB=$so timeout -k 10 300 python -u bench.py --config $cfg $extra > "$OUT/${cfg}_${name}_$r.json" 2> "$OUT/${cfg}_${name}_$r.err" || { echo BENCH_FAILED $name $cfg; tail -5 "$OUT/${cfg}_${name}_$r.err"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/${cfg}_${name}_$r.json')); s=d.get('solver',{}); print('$cfg $name $r', d['value'], d['ms_per_step'], s.get('iters_mean', s.get('iters_mean_last_step')), s.get('kernel_ms_per_solve', s.get('kernel_ms_per_launch')))"
    done
  done
done
echo R5V_DONE
