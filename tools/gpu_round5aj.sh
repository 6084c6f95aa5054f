#!/bin/bash
# Round-5 GPU session AJ: the B = 1 OBCA plan latency (with / without helpers) and the closed-loop bench (steps 5 + 40)
# on the shipped kernels.   usage: bash tools/gpu_round5aj.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5aj}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/obca_plan_latency.py 3 > "$OUT/plan_latency.txt" 2>&1 || { echo LAT_FAILED; tail -5 "$OUT/plan_latency.txt"; exit 1; }
cat "$OUT/plan_latency.txt"
timeout -k 10 300 python -u bench.py --config sim --steps 40 --warmup 5 > "$OUT/bench_sim_40.json" 2> "$OUT/bench_sim_40.err" || { echo BENCH_FAILED sim; tail -10 "$OUT/bench_sim_40.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_sim_40.json')); print('sim 5+40', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --config sim > "$OUT/bench_sim.json" 2> "$OUT/bench_sim.err" || { echo BENCH_FAILED sim; tail -10 "$OUT/bench_sim.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_sim.json')); print('sim default', d['value'], d['ms_per_step'])"
echo R5AJ_DONE
