#!/bin/bash
# A/B of library variants at C5 (B = 65536 per launch): bash tools/ab_c5.sh OUT lib1 lib2 ...
OUT=$1; shift
mkdir -p "$OUT"
for round in 1 2; do
  for L in "$@"; do
    n=$(basename "$L" .so)
    TTMPC_LIB="$L" timeout -k 10 120 python bench.py --config c5 --steps 10 --warmup 2 --cpu-budget 0 --no-latency > "$OUT/${n}_c5_r${round}.json" 2>>"$OUT/err.log" || exit 1
    python3 -c "import json,sys; d=json.load(open('$OUT/${n}_c5_r${round}.json')); print('$n c5', $round, d['value'], d['solver'].get('kernel_ms_per_launch'))"
  done
done
