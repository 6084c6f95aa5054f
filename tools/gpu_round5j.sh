#!/bin/bash
# Round-5 GPU session J: the C4 census comparison, the OBCA bench configs (C4 with the per-instance oracle census of its
# batch), the closed loop, and the C2 PMC passes of the shipped tracking kernel.   usage: bash tools/gpu_round5j.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5j}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/obca_census_compare.py > "$OUT/c4_census_compare.txt" 2>&1 || { echo CENSUS_FAILED; tail -20 "$OUT/c4_census_compare.txt"; exit 1; }
cat "$OUT/c4_census_compare.txt"
for cfg in c4 cobs c4replan c4all; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 1 --warmup 1 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; tail -10 "$OUT/bench_$cfg.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d.get('solver', {}))"
done
timeout -k 10 300 python -u bench.py --config sim > "$OUT/bench_sim.json" 2> "$OUT/bench_sim.err" || { echo BENCH_FAILED sim; tail -10 "$OUT/bench_sim.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_sim.json')); print('sim', d['value'], d['ms_per_step'])"
bash tools/hbm_passes.sh "$OUT/pmc_c2" c2 || exit 1
python - "$OUT" <<'PY'
import sys, glob
sys.path.insert(0, ".")
from bench import read_traffic
out = sys.argv[1]
f = sorted(glob.glob(f"{out}/pmc_c2/fetch/*counter_collection.csv"))
w = sorted(glob.glob(f"{out}/pmc_c2/write/*counter_collection.csv"))
print("c2 2xFETCH+WRITE bytes per launch:", read_traffic(f[:1] + w[:1]))
PY
echo R5J_DONE
