#!/bin/bash
# Round-5 GPU session W: bisect of the closed-loop (N = 50) kernel time over the round-5 tracking commits: r4 (e4c819e),
# f1e900f (IPOPT's full convergence test and barrier floor), 815f978 (loads first, lazy pows), the current tree.
# usage: bash tools/gpu_round5w.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5w}
mkdir -p "$OUT"
V=car-trailer-mpc_amd/ttmpc/variants
export TMPDIR=/tmp
for r in 1 2; do
  for spec in r4=$V/libttmpc_r4.so f1e900f=$V/libttmpc_f1e900f.so 815f978=$V/libttmpc_815f978.so cur=; do
    name=${spec%%=*}; so=${spec#*=}
    TTMPC_LIB=$so timeout -k 10 300 python -u bench.py --config sim --steps 40 --warmup 5 --cpu-budget 0 > "$OUT/sim_${name}_$r.json" 2> "$OUT/sim_${name}_$r.err" || { echo BENCH_FAILED $name; tail -5 "$OUT/sim_${name}_$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/sim_${name}_$r.json')); s=d['solver']; print('sim $name $r', d['value'], d['ms_per_step'], s['iters_mean_last_step'], s['kernel_ms_per_solve'])"
  done
done
echo R5W_DONE
