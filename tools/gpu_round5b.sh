#!/bin/bash
# Round-5 GPU session B: the 14 C4 test cases GPU vs oracle with the oracle's IPOPT error at both end points, and the
# C2 / C3 PMC passes of the shipped tracking kernel.   usage: bash tools/gpu_round5b.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/obca_c4cases.py 0 14 > "$OUT/c4cases.txt" 2>&1 || { echo C4CASES_FAILED; tail -20 "$OUT/c4cases.txt"; exit 1; }
cat "$OUT/c4cases.txt"
bash tools/hbm_passes.sh "$OUT/pmc_c2" c2 || exit 1
bash tools/hbm_passes.sh "$OUT/pmc_c3" c3 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o run --output-format csv \
  -- python3 bench.py --config c3 --steps 10 --warmup 2 --cpu-budget 0 --no-latency > "$OUT/prof_c3.log" 2>&1 || { echo PROF_FAILED; tail -20 "$OUT/prof_c3.log"; exit 1; }
find "$OUT/prof_c3" -name '*kernel_stats.csv' -exec head -3 {} \;
python - "$OUT" <<'PY'
import sys
sys.path.insert(0, ".")
from bench import read_traffic
out = sys.argv[1]
for cfg in ("c2", "c3"):
    d = f"{out}/pmc_{cfg}/pmc_{cfg}" if False else f"{out}/pmc_{cfg}"
    import glob
    f = glob.glob(f"{d}/fetch/**/*counter_collection.csv", recursive=True) + glob.glob(f"{d}/fetch/*counter_collection.csv")
    w = glob.glob(f"{d}/write/**/*counter_collection.csv", recursive=True) + glob.glob(f"{d}/write/*counter_collection.csv")
    print(cfg, "2xFETCH+WRITE bytes per launch:", read_traffic(sorted(set(f))[:1] + sorted(set(w))[:1]))
PY
echo R5B_DONE
