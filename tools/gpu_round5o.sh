#!/bin/bash
# Round-5 GPU session O: the C4 tail profile of the helper-workgroup kernel (iterations 4,000-5,000) and the OBCA HBM
# passes (FETCH_SIZE / WRITE_SIZE) of the c4, c4all and cobs probes for bench.py's OBCA_PMC.
# usage: bash tools/gpu_round5o.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5o}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 > "$OUT/tail.txt" 2>&1 || { echo TAIL_FAILED; tail -5 "$OUT/tail.txt"; exit 1; }
cat "$OUT/tail.txt"
for cfg in c4 c4all cobs; do
  bash tools/obca_pmc.sh "$OUT/pmc_$cfg" $cfg 300 hbm || exit 1
done
python - "$OUT" <<'PY'
import sys, json
sys.path.insert(0, ".")
from bench import read_traffic
out = sys.argv[1]
for cfg in ("c4", "c4all", "cobs"):
    d = f"{out}/pmc_{cfg}"
    t = read_traffic([f"{d}/fetch/fetch_counter_collection.csv", f"{d}/write/write_counter_collection.csv"], kernel="obca_kernel")
    rec = json.loads(open(f"{d}/fetch.bench.json").read())["solver"]
    print(cfg, "bytes per launch", t, "per instance-iteration MB", t / (rec["iters_mean"] * rec["instances"]) / 1e6)
PY
V=car-trailer-mpc_amd/ttmpc/variants
# A/B: the trial pass's block part as chunks too (variant "trial": a block's barrier product merged as one factor)
TTMPC_LIB=$V/libttmpc_trial.so timeout -k 10 300 python -u tools/obca_stamps.py 256 c4 300 > "$OUT/stamps_trial.txt" 2>&1 || { echo STAMPS_FAILED; tail -5 "$OUT/stamps_trial.txt"; exit 1; }
timeout -k 10 300 python -u tools/obca_stamps.py 256 c4 300 > "$OUT/stamps_cur.txt" 2>&1 || { echo STAMPS_FAILED; tail -5 "$OUT/stamps_cur.txt"; exit 1; }
cat "$OUT/stamps_cur.txt" "$OUT/stamps_trial.txt"
TTMPC_LIB=$V/libttmpc_trial.so timeout -k 10 400 python -u bench.py --config c4 --steps 1 --warmup 1 > "$OUT/bench_c4_trial.json" 2> "$OUT/bench_c4_trial.err" || { echo BENCH_FAILED; tail -10 "$OUT/bench_c4_trial.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c4_trial.json')); s=d.get('solver', {}); print('c4 trial', d['value'], d['ms_per_step'], s.get('status_counts'), s.get('oracle_census', {}).get('equal_status'))"
echo R5O_DONE
