#!/bin/bash
# LDS counters of the default (C2) bench launch: bank / address conflicts against LDS active cycles.
# usage: bash tools/lds_pmc.sh [OUTDIR] [CONFIG=c2]
set -o pipefail
OUT=${1:-gpurun_out/ldspmc}
CFG=${2:-c2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAVES --kernel-trace -d $OUT/c2 -o c2 --output-format csv -- python3 bench.py --config $CFG --steps 6 --warmup 1 --cpu-budget 0 --no-latency > $OUT/c2.log 2>&1 || { echo PASS_FAILED; tail -5 $OUT/c2.log; exit 1; }
python3 tools/pmc_summary.py $OUT/c2/c2_counter_collection.csv track_kernel > $OUT/summary.txt && cat $OUT/summary.txt
echo LDS_PMC_DONE
