#!/bin/bash
# PMC counters of the OBCA kernel on a short C4 run (B=256, 300 IPM iterations): HBM bytes (separate
# FETCH_SIZE / WRITE_SIZE passes), wave / wait counters and the instruction mix.
# usage (GPU box): bash tools/obca_pmc.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/obca_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o "$name" --output-format csv \
    -- python3 bench.py --config c4 --max-iter 300 --steps 1 --warmup 0 --cpu-budget 0 > "$OUT/$name.log" 2>&1 || { echo "PASS_FAILED $name"; tail -5 "$OUT/$name.log"; exit 1; }
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run waves SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM
run vmem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS
echo OBCA_PMC_DONE
