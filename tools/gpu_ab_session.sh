#!/bin/bash
# OBCA A/B session (GPU box): bitwise output comparison + phase stamps (tools/ab_obca.sh) of library variants against
# the first, a C4 bench line for each, then the OBCA GPU tests on the in-tree library.
# usage: bash tools/gpu_ab_session.sh OUTDIR NAME ...   (NAME = a variant under ttmpc/variants/libttmpc_NAME.so, or "new"
# for the in-tree library)   env: TAIL=1 also runs tools/obca_tail.py on the in-tree library
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
V=$PWD/car-trailer-mpc_amd/ttmpc/variants
specs=()
for n in "$@"; do if [ "$n" = new ]; then specs+=("new="); else specs+=("$n=$V/libttmpc_$n.so"); fi; done
bash tools/ab_obca.sh "$OUT/ab" "${specs[@]}" > "$OUT/ab.log" 2>&1 || { echo AB_FAILED; tail -5 "$OUT/ab.log"; exit 1; }
cat "$OUT"/ab/compare_*.txt; cat "$OUT"/ab/stamps_*.txt
for n in "$@"; do
  if [ "$n" = new ]; then L=""; else L="$V/libttmpc_$n.so"; fi
  TTMPC_LIB=$L timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/${n}_c4.json" 2> "$OUT/${n}_c4.err" || { echo "BENCH_FAILED $n"; tail -5 "$OUT/${n}_c4.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/${n}_c4.json')); print('$n', d['value'], d['ms_per_step'])"
done
if [ "${TAIL:-0}" = 1 ]; then
  timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 "$OUT/tail.npz" > "$OUT/tail.txt" 2>&1 || { echo TAIL_FAILED; tail -5 "$OUT/tail.txt"; exit 1; }
  cat "$OUT/tail.txt"
fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_obca.py -m gpu -v --timeout 300 --timeout-method thread > "$OUT/t_obca.log" 2>&1; rc=$?
echo "obca tests rc=$rc"; tail -3 "$OUT/t_obca.log"; grep -E "FAILED|ERROR" "$OUT/t_obca.log" | head
echo AB_SESSION_DONE
