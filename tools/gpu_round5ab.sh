#!/bin/bash
# Round-5 GPU session AB: validation of the shipped kernels -- the full GPU test suite, smoke(), the default bench (C2)
# with its rocprof summary, every bench config, and the SQ wave-state passes of C3 and C5 (issue vs wait share of the
# tracking waves, for the occupancy analysis).   usage: bash tools/gpu_round5ab.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -10
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > "$OUT/smoke.log" 2>&1 || { echo SMOKE_FAILED; tail -10 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo BENCH_FAILED default; tail -10 "$OUT/bench_default.err"; exit 1; }
head -c 1500 "$OUT/bench_default.json"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv \
  -- python3 bench.py --steps 20 --warmup 3 --cpu-budget 0 --no-latency > "$OUT/prof_c2.log" 2>&1 || { echo PROF_FAILED; tail -10 "$OUT/prof_c2.log"; exit 1; }
for cfg in c3 c5 c4 cobs c4replan c4all; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; tail -10 "$OUT/bench_$cfg.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$cfg.json')); print('$cfg', d['value'], d['unit'], d['ms_per_step'])"
done
for cfg in c3 c5; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --kernel-trace -d "$OUT/pmc_$cfg/waves" -o waves --output-format csv \
    -- python3 bench.py --config $cfg --steps 6 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/pmc_${cfg}_waves.log" 2>&1 || { echo "PMC_FAILED $cfg"; tail -5 "$OUT/pmc_${cfg}_waves.log"; exit 1; }
  timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    --kernel-trace -d "$OUT/pmc_$cfg/insts" -o insts --output-format csv \
    -- python3 bench.py --config $cfg --steps 6 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/pmc_${cfg}_insts.log" 2>&1 || { echo "PMC_FAILED $cfg insts"; tail -5 "$OUT/pmc_${cfg}_insts.log"; exit 1; }
done
echo R5AB_DONE
