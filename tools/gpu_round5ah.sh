#!/bin/bash
# Round-5 GPU session AH: the helpers' chunk code inlined into the kernel's helper path (no call frame per chunk).
# OBCA A/B against head: bitwise dumps, stamps, C4 in alternating rounds, the C4 tail, and the OBCA GPU tests.
# usage: bash tools/gpu_round5ah.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5ah}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=car-trailer-mpc_amd/ttmpc/variants
bash tools/ab_obca.sh "$OUT/obca" head=$V/libttmpc_head.so new= > "$OUT/obca_ab.txt" 2>&1 || { echo OBCA_AB_FAILED; tail -5 "$OUT/obca_ab.txt"; exit 1; }
grep -E "bitwise|TOTAL|==" "$OUT/obca_ab.txt" | head -30
for r in 1 2; do
  for spec in head=$V/libttmpc_head.so new=; do
    name=${spec%%=*}; so=${spec#*=}
    TTMPC_LIB=$so timeout -k 10 400 python -u bench.py --config c4 --steps 1 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/c4_${name}_$r.json" 2> "$OUT/c4_${name}_$r.err" || { echo BENCH_FAILED $name; tail -5 "$OUT/c4_${name}_$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/c4_${name}_$r.json')); print('c4 $name $r', d['value'], d['ms_per_step'])"
  done
done
for spec in head=$V/libttmpc_head.so new=; do
  name=${spec%%=*}; so=${spec#*=}
  TTMPC_LIB=$so timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 > "$OUT/tail_$name.txt" 2>&1 || { echo TAIL_FAILED $name; tail -5 "$OUT/tail_$name.txt"; exit 1; }
  echo "tail $name"; sed -n 2,20p "$OUT/tail_$name.txt"
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_obca.py -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$OUT/t_obca.log" 2>&1; rc=$?
echo "obca tests rc=$rc"; tail -2 "$OUT/t_obca.log"; grep -E "FAILED|ERROR" "$OUT/t_obca.log" | head
echo R5AH_DONE
