#!/bin/bash
# Round profile of the tracking kernel (GPU box): tests, C2/C3 bench lines, rocprofv3 kernel stats and the
# PMC HBM passes of both configs.  usage: bash tools/gpu_track_prof.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > "$OUT/t_parity.log" 2>&1 || { echo TESTS_FAILED; tail -20 "$OUT/t_parity.log"; exit 1; }
for cfg in c2 c3; do
  timeout -k 10 300 python -u bench.py --config $cfg > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { echo BENCH_FAILED $cfg; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ks_$cfg" -o ks --output-format csv -- python3 bench.py --config $cfg --steps 20 --warmup 3 --cpu-budget 0 --no-latency > "$OUT/ks_$cfg.log" 2>&1 || { echo KSTATS_FAILED $cfg; exit 1; }
  bash tools/hbm_passes.sh "$OUT/pmc_$cfg" $cfg || exit 1
done
echo PROF_DONE
