#!/bin/bash
# Round-5 GPU session AE: the OBCA model's tan / cos through tt_trig.hpp too.  The bitwise check of the restated
# sincos, tan and cos against the library, tracking dumps (bitwise), OBCA A/B (dumps, stamps, C4) against head, and the
# OBCA GPU tests.   usage: bash tools/gpu_round5ae.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5ae}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=car-trailer-mpc_amd/ttmpc/variants
timeout -k 10 120 ./tools/trig_check 268435456 > "$OUT/trig_check.txt" 2>&1; rc=$?
cat "$OUT/trig_check.txt"; [ $rc -eq 0 ] || exit 1
for n in head new; do
  so=""; [ $n = head ] && so=$V/libttmpc_head.so
  TTMPC_LIB=$so timeout -k 10 300 python -u tools/track_dump.py "$OUT/tdump_$n.npz" > "$OUT/tdump_$n.txt" 2>&1 || { echo "TDUMP_FAILED $n"; tail -5 "$OUT/tdump_$n.txt"; exit 1; }
done
python tools/track_dump.py --compare "$OUT/tdump_head.npz" "$OUT/tdump_new.npz" > "$OUT/track_compare_new.txt" 2>&1; tail -1 "$OUT/track_compare_new.txt"
bash tools/ab_obca.sh "$OUT/obca" head=$V/libttmpc_head.so new= > "$OUT/obca_ab.txt" 2>&1 || { echo OBCA_AB_FAILED; tail -5 "$OUT/obca_ab.txt"; exit 1; }
grep -E "bitwise|TOTAL|==|  lin|  trial" "$OUT/obca_ab.txt" | head -30
for r in 1 2; do
  for spec in head=$V/libttmpc_head.so new=; do
    name=${spec%%=*}; so=${spec#*=}
    TTMPC_LIB=$so timeout -k 10 400 python -u bench.py --config c4 --steps 1 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/c4_${name}_$r.json" 2> "$OUT/c4_${name}_$r.err" || { echo BENCH_FAILED $name; tail -5 "$OUT/c4_${name}_$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/c4_${name}_$r.json')); print('c4 $name $r', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_obca.py -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$OUT/t_obca.log" 2>&1; rc=$?
echo "obca tests rc=$rc"; tail -2 "$OUT/t_obca.log"; grep -E "FAILED|ERROR" "$OUT/t_obca.log" | head
echo R5AE_DONE
