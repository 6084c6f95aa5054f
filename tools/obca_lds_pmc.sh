#!/bin/bash
# LDS counters of the OBCA kernel on the short C4 probe (B = 256, MAX_ITER IPM iterations): bank / address conflicts
# against LDS active cycles and the LDS instruction count.  usage (GPU box): bash tools/obca_lds_pmc.sh OUTDIR [CFG] [MAX_ITER]
set -o pipefail
OUT=${1:-gpurun_out/obca_ldspmc}
CFG=${2:-c4}
MI=${3:-300}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAVES --kernel-trace -d "$OUT/lds" -o lds --output-format csv \
  -- python3 bench.py --config $CFG --max-iter $MI --steps 1 --warmup 0 --cpu-budget 0 > "$OUT/lds.log" 2>&1 || { echo PASS_FAILED; tail -5 "$OUT/lds.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT/lds/lds_counter_collection.csv" obca_kernel > "$OUT/summary.txt" && cat "$OUT/summary.txt"
echo OBCA_LDS_PMC_DONE
