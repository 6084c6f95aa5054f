#!/bin/bash
# PMC counters of the OBCA kernel on a short C4 run (B=256, 300 IPM iterations): HBM bytes (separate
# FETCH_SIZE / WRITE_SIZE passes), wave / wait counters and the instruction mix.
# usage (GPU box): bash tools/obca_pmc.sh OUTDIR [CONFIG=c4] [MAX_ITER=300] [hbm]   (hbm: FETCH/WRITE passes only)
set -o pipefail
OUT=${1:-gpurun_out/obca_pmc}
CFG=${2:-c4}
MI=${3:-300}
ONLY=${4:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o "$name" --output-format csv \
    -- python3 bench.py --config $CFG --max-iter $MI --steps 1 --warmup 0 --cpu-budget 0 > "$OUT/$name.log" 2>&1 && grep '^{' "$OUT/$name.log" > "$OUT/$name.bench.json" || { echo "PASS_FAILED $name"; tail -5 "$OUT/$name.log"; exit 1; }
}
run fetch FETCH_SIZE
run write WRITE_SIZE
[ "$ONLY" = hbm ] && { echo OBCA_PMC_DONE; exit 0; }
run waves SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM
run vmem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS
echo OBCA_PMC_DONE
