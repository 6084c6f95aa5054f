#!/bin/bash
# Round-5 GPU session AC: the OBCA HBM passes (FETCH_SIZE / WRITE_SIZE, separate rocprofv3 --pmc runs) of the shipped
# kernel on the 300-iteration probes of c4, c4all and cobs, and the rocprofv3 kernel stats of one C4 bench launch.
# usage: bash tools/gpu_round5ac.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5ac}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in c4 c4all cobs; do
  bash tools/obca_pmc.sh "$OUT/pmc_$cfg" $cfg 300 hbm > "$OUT/pmc_$cfg.log" 2>&1 || { echo "PMC_FAILED $cfg"; tail -5 "$OUT/pmc_$cfg.log"; exit 1; }
  echo "pmc $cfg done"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o run --output-format csv \
  -- python3 bench.py --config c4 --steps 1 --warmup 0 --cpu-budget 0 --no-latency > "$OUT/prof_c4.log" 2>&1 || { echo PROF_FAILED; tail -10 "$OUT/prof_c4.log"; exit 1; }
head -3 "$OUT/prof_c4/run_kernel_stats.csv"
echo R5AC_DONE
