#!/bin/bash
# Round-5 GPU session Z: the update pass's block part over the flat block index (update_block), with helpers.
# Bitwise A/B against HEAD (tools/obca_dump.py), c4-300 stamps of both, the C4 tail profile
# and the C4 bench of the new build.   usage: bash tools/gpu_round5p.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5z}
mkdir -p "$OUT"
V=car-trailer-mpc_amd/ttmpc/variants
export TMPDIR=/tmp
bash tools/ab_obca.sh "$OUT" head=$V/libttmpc_head.so new= || exit 1
timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 > "$OUT/tail.txt" 2>&1 || { echo TAIL_FAILED; tail -5 "$OUT/tail.txt"; exit 1; }
head -25 "$OUT/tail.txt"
timeout -k 10 400 python -u bench.py --config c4 --steps 1 --warmup 1 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || { echo BENCH_FAILED; tail -10 "$OUT/bench_c4.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c4.json')); s=d.get('solver', {}); print('c4', d['value'], d['ms_per_step'], s.get('status_counts'), s.get('oracle_census', {}).get('equal_status'))"
echo R5Z_DONE
