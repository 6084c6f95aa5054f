#!/bin/bash
# Round-5 GPU session AD: straight-line sincos (tt_trig.hpp).  The bitwise check of the restated sincos against the
# library, then tracking A/B (dumps, C2 / C3 / C5, stamps, tracking tests) and OBCA A/B (dumps, stamps, C4, the tail)
# against head.   usage: bash tools/gpu_round5ad.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5ad}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=car-trailer-mpc_amd/ttmpc/variants
timeout -k 10 120 ./tools/trig_check 268435456 > "$OUT/trig_check.txt" 2>&1; rc=$?
cat "$OUT/trig_check.txt"; [ $rc -eq 0 ] || exit 1
bash tools/gpu_track_ab2.sh "$OUT/track" head new | grep -v "^$" | tail -40 || exit 1
bash tools/ab_obca.sh "$OUT/obca" head=$V/libttmpc_head.so new= > "$OUT/obca_ab.txt" 2>&1 || { echo OBCA_AB_FAILED; tail -5 "$OUT/obca_ab.txt"; exit 1; }
grep -E "bitwise|TOTAL|==" "$OUT/obca_ab.txt" | head -30
for r in 1 2; do
  for spec in head=$V/libttmpc_head.so new=; do
    name=${spec%%=*}; so=${spec#*=}
    TTMPC_LIB=$so timeout -k 10 400 python -u bench.py --config c4 --steps 1 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/c4_${name}_$r.json" 2> "$OUT/c4_${name}_$r.err" || { echo BENCH_FAILED $name; tail -5 "$OUT/c4_${name}_$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/c4_${name}_$r.json')); print('c4 $name $r', d['value'], d['ms_per_step'])"
  done
done
echo R5AD_DONE
