#!/bin/bash
# Round-5 GPU session AO: idle helpers pause 4 x 64 cycles between board scans instead of 32 x 64 (variant "sl4")
# against the shipped build: OBCA dumps, stamps, C4 in alternating rounds, the C4 tail.   usage: bash tools/gpu_round5ao.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5ao}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=car-trailer-mpc_amd/ttmpc/variants
bash tools/ab_obca.sh "$OUT/obca" head=$V/libttmpc_head.so sl4=$V/libttmpc_sl4.so > "$OUT/obca_ab.txt" 2>&1 || { echo OBCA_AB_FAILED; tail -5 "$OUT/obca_ab.txt"; exit 1; }
grep -E "bitwise|TOTAL|==" "$OUT/obca_ab.txt" | head -30
for r in 1 2; do
  for spec in head=$V/libttmpc_head.so sl4=$V/libttmpc_sl4.so; do
    name=${spec%%=*}; so=${spec#*=}
    TTMPC_LIB=$so timeout -k 10 400 python -u bench.py --config c4 --steps 1 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/c4_${name}_$r.json" 2> "$OUT/c4_${name}_$r.err" || { echo BENCH_FAILED $name; tail -5 "$OUT/c4_${name}_$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/c4_${name}_$r.json')); print('c4 $name $r', d['value'], d['ms_per_step'])"
  done
done
TTMPC_LIB=$V/libttmpc_sl4.so timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 > "$OUT/tail_sl4.txt" 2>&1 || { echo TAIL_FAILED; tail -5 "$OUT/tail_sl4.txt"; exit 1; }
sed -n 2,20p "$OUT/tail_sl4.txt"
echo R5AO_DONE
