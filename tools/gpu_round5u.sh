#!/bin/bash
# Round-5 GPU session U: the closed loop (N = 50, the generic one-stage-per-lane build) with and without the tracking
# kernel's loads-first order (variant nolf: -DTT_NO_LF), 2 alternating rounds.   usage: bash tools/gpu_round5u.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5u}
mkdir -p "$OUT"
V=car-trailer-mpc_amd/ttmpc/variants
export TMPDIR=/tmp
for r in 1 2; do
  for spec in cur= nolf=$V/libttmpc_nolf.so; do
    name=${spec%%=*}; so=${spec#*=}
    TTMPC_LIB=$so timeout -k 10 300 python -u bench.py --config sim --steps 40 --warmup 5 --cpu-budget 0 > "$OUT/sim_${name}_$r.json" 2> "$OUT/sim_${name}_$r.err" || { echo BENCH_FAILED $name; tail -5 "$OUT/sim_${name}_$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/sim_${name}_$r.json')); print('$name', $r, d['value'], d['ms_per_step'], d['solver'])"
  done
done
echo R5U_DONE
