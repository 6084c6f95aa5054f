#!/bin/bash
# Round-5 GPU session S: the correction solve's backward sweep as a dense affine recurrence (riccati_vec_affine).  Not
# bitwise: the OBCA GPU tests (oracle parity, census, lockstep), the dump against HEAD, c4-300 stamps, the C4 tail and
# the C4 bench.   usage: bash tools/gpu_round5s.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5s}
mkdir -p "$OUT"
V=car-trailer-mpc_amd/ttmpc/variants
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_obca.py -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$OUT/gpu_obca_tests.log" 2>&1; rc=$?
echo "obca gpu tests rc=$rc"; tail -3 "$OUT/gpu_obca_tests.log"; grep -E "FAILED|ERROR|Error" "$OUT/gpu_obca_tests.log" | head -10
grep -A3 "C4 census comparison" "$OUT/gpu_obca_tests.log" | head -3
[ $rc -le 1 ] || exit 1
bash tools/ab_obca.sh "$OUT" head=$V/libttmpc_head.so new= || exit 1
timeout -k 10 300 python -u tools/obca_tail.py 256 4000 5000 > "$OUT/tail.txt" 2>&1 || { echo TAIL_FAILED; tail -5 "$OUT/tail.txt"; exit 1; }
head -25 "$OUT/tail.txt"
timeout -k 10 400 python -u bench.py --config c4 --steps 1 --warmup 1 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || { echo BENCH_FAILED; tail -10 "$OUT/bench_c4.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c4.json')); s=d.get('solver', {}); print('c4', d['value'], d['ms_per_step'], s.get('status_counts'), s.get('oracle_census', {}))"
echo R5S_DONE
