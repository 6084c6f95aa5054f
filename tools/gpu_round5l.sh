#!/bin/bash
# Round-5 GPU session L: OBCA block passes over the flat block index (phase_nres, phase_factor) -- bitwise A/B against
# the step-0 build (per-block partial of grad phi' d), phase stamps against the round-5 base; the closed-loop bench at
# round 4's step count.   usage: bash tools/gpu_round5l.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5l}
mkdir -p "$OUT"
V=car-trailer-mpc_amd/ttmpc/variants
bash tools/ab_obca.sh "$OUT" dmb=$V/libttmpc_dmb.so new= base=$V/libttmpc_r5base.so || exit 1
timeout -k 10 300 python -u bench.py --config sim --steps 40 --warmup 5 > "$OUT/bench_sim_40.json" 2> "$OUT/bench_sim_40.err" || { echo BENCH_FAILED sim; tail -10 "$OUT/bench_sim_40.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_sim_40.json')); print('sim 5+40', d['value'], d['ms_per_step'], d['solver'])"
echo R5L_DONE
