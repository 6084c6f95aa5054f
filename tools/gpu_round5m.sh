#!/bin/bash
# Round-5 GPU session M: OBCA block passes over the flat block index + helper workgroups.  Bitwise A/B against the step-0
# build (per-block partial of grad phi' d) with and without helpers, phase stamps, the C4 bench line, the closed loop
# at round 4's step count.   usage: bash tools/gpu_round5m.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5m}
mkdir -p "$OUT"
V=car-trailer-mpc_amd/ttmpc/variants
export TMPDIR=/tmp
TTMPC_LIB=$V/libttmpc_dmb.so timeout -k 10 300 python -u tools/obca_dump.py "$OUT/dmb.npz" 64 1000 > "$OUT/dump_dmb.txt" 2>&1 || { echo DUMP_FAILED dmb; tail -5 "$OUT/dump_dmb.txt"; exit 1; }
OBCA_HELPERS=0 timeout -k 10 300 python -u tools/obca_dump.py "$OUT/new_noh.npz" 64 1000 > "$OUT/dump_new_noh.txt" 2>&1 || { echo DUMP_FAILED noh; tail -5 "$OUT/dump_new_noh.txt"; exit 1; }
python tools/obca_dump.py --compare "$OUT/dmb.npz" "$OUT/new_noh.npz" > "$OUT/compare_noh.txt" 2>&1
timeout -k 10 300 python -u tools/obca_dump.py "$OUT/new_h.npz" 64 1000 > "$OUT/dump_new_h.txt" 2>&1 || { echo DUMP_FAILED h; tail -5 "$OUT/dump_new_h.txt"; exit 1; }
python tools/obca_dump.py --compare "$OUT/dmb.npz" "$OUT/new_h.npz" > "$OUT/compare_h.txt" 2>&1
cat "$OUT"/dump_*.txt "$OUT"/compare_*.txt
for spec in base=$V/libttmpc_r5base.so: noh=:0 h=: ; do
  name=${spec%%=*}; rest=${spec#*=}; so=${rest%%:*}; hl=${rest#*:}
  TTMPC_LIB=$so OBCA_HELPERS=$hl timeout -k 10 300 python -u tools/obca_stamps.py 256 c4 300 > "$OUT/stamps_$name.txt" 2>&1 || { echo STAMPS_FAILED $name; tail -5 "$OUT/stamps_$name.txt"; exit 1; }
  echo "== stamps $name"; cat "$OUT/stamps_$name.txt"
done
timeout -k 10 400 python -u bench.py --config c4 --steps 1 --warmup 1 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || { echo BENCH_FAILED c4; tail -10 "$OUT/bench_c4.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c4.json')); print('c4', d['value'], d['ms_per_step'], d.get('solver', {}))"
timeout -k 10 300 python -u bench.py --config sim --steps 40 --warmup 5 > "$OUT/bench_sim_40.json" 2> "$OUT/bench_sim_40.err" || { echo BENCH_FAILED sim; tail -10 "$OUT/bench_sim_40.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_sim_40.json')); print('sim 5+40', d['value'], d['ms_per_step'], d['solver'])"
echo R5M_DONE
