#!/bin/bash
# A/B timing of library variants in one GPU session: bash tools/ab.sh OUT lib1 lib2 ... (bench C2, 3 alternating rounds)
OUT=$1; shift
mkdir -p "$OUT"
for round in 1 2 3; do
  for L in "$@"; do
    n=$(basename "$L" .so)
    TTMPC_LIB="$L" timeout -k 10 120 python bench.py --cpu-budget 0 --no-latency ${AB_ARGS} > "$OUT/${n}_r${round}.json" 2>>"$OUT/err.log" || exit 1
    python3 -c "import json,sys; d=json.load(open('$OUT/${n}_r${round}.json')); print('$n', $round, d['value'], d['solver']['kernel_ms_per_launch'], d['solver']['iters_mean'])"
  done
done
