#!/bin/bash
# Round-4 GPU session D (GPU box): OBCA sweep operand prefetch (hard/soft forward, vector Riccati) -- bitwise A/B and
# phase stamps against the previous build, C4 bench for both, tail accounting, OBCA GPU tests.
# usage: bash tools/gpu_round4d.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r4d}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=$PWD/car-trailer-mpc_amd/ttmpc/variants
bash tools/ab_obca.sh "$OUT/ab_pf" base=$V/libttmpc_base.so pf= > "$OUT/ab_pf.log" 2>&1 || { echo AB_FAILED; tail -5 "$OUT/ab_pf.log"; exit 1; }
cat "$OUT/ab_pf/compare_pf.txt"; grep -E "TOTAL|ref_sweeps|riccati|forward" "$OUT"/ab_pf/stamps_*.txt
for r in 1; do
  for v in base pf; do
    if [ $v = pf ]; then L=""; else L="$V/libttmpc_$v.so"; fi
    TTMPC_LIB=$L timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/${v}_c4_$r.json" 2> "$OUT/${v}_c4_$r.err" || { echo "BENCH_FAILED $v"; tail -5 "$OUT/${v}_c4_$r.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${v}_c4_$r.json')); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 "$OUT/tail.npz" > "$OUT/tail.txt" 2>&1 || { echo TAIL_FAILED; tail -5 "$OUT/tail.txt"; exit 1; }
cat "$OUT/tail.txt"
timeout -k 10 600 python -u -m pytest tests/test_gpu_obca.py -m gpu -v --timeout 300 --timeout-method thread > "$OUT/t_obca.log" 2>&1; rc=$?
echo "obca tests rc=$rc"; tail -3 "$OUT/t_obca.log"; grep -E "FAILED|ERROR" "$OUT/t_obca.log" | head
echo R4D_DONE
