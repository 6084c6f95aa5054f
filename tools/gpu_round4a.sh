#!/bin/bash
# Round-4 GPU session A (GPU box): OBCA lockstep / parity census + OBCA tests, N = 20 occupancy threshold A/B by batch,
# the C4 tail accounting, and the OBCA_RCP cycle cost.   usage: bash tools/gpu_round4a.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r4a}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=$PWD/car-trailer-mpc_amd/ttmpc/variants
bash tools/gpu_lock.sh "$OUT/lock" || exit 1
for B in 1024 2048 3072 4096 8192 16384; do
  for v in new occ0 occ1024 occ2048; do
    if [ $v = new ]; then L=""; else L="$V/libttmpc_$v.so"; fi
    TTMPC_LIB=$L timeout -k 10 120 python bench.py --config c2 --batch $B --steps 20 --warmup 3 --cpu-budget 0 --no-latency > "$OUT/occ_${v}_$B.json" 2> "$OUT/occ_${v}_$B.err" || { echo "OCC_FAILED $v $B"; tail -5 "$OUT/occ_${v}_$B.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/occ_${v}_$B.json')); print('occ', '$v', $B, d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 > "$OUT/tail.txt" 2>&1 || { echo TAIL_FAILED; tail -5 "$OUT/tail.txt"; exit 1; }
cat "$OUT/tail.txt"
for v in new rcp1; do
  if [ $v = new ]; then L=""; else L="$V/libttmpc_$v.so"; fi
  TTMPC_LIB=$L timeout -k 10 300 python -u tools/obca_stamps.py 256 c4 300 > "$OUT/stamps_$v.txt" 2>&1 || { echo "STAMPS_FAILED $v"; tail -5 "$OUT/stamps_$v.txt"; exit 1; }
  echo "== stamps $v"; cat "$OUT/stamps_$v.txt"
done
echo R4A_DONE
