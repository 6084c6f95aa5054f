#!/bin/bash
# Round-5 GPU session X: the switching-condition pows issued first when theta0 <= theta_min.  Tracking A/B (bitwise
# dumps, C2 / C3 / C5, stamps, tracking tests; tools/gpu_track_ab2.sh) and the closed loop, head vs new.
# usage: bash tools/gpu_round5x.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5x}
mkdir -p "$OUT"
V=car-trailer-mpc_amd/ttmpc/variants
export TMPDIR=/tmp
bash tools/gpu_track_ab2.sh "$OUT" head new | grep -v "^$" | tail -40 || exit 1
for r in 1 2; do
  for spec in head=$V/libttmpc_head.so new=; do
    name=${spec%%=*}; so=${spec#*=}
    TTMPC_LIB=$so timeout -k 10 300 python -u bench.py --config sim --steps 40 --warmup 5 --cpu-budget 0 > "$OUT/sim_${name}_$r.json" 2> "$OUT/sim_${name}_$r.err" || { echo BENCH_FAILED $name; tail -5 "$OUT/sim_${name}_$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/sim_${name}_$r.json')); s=d['solver']; print('sim $name $r', d['value'], d['ms_per_step'], s['iters_mean_last_step'], s['kernel_ms_per_solve'])"
  done
done
echo R5X_DONE
