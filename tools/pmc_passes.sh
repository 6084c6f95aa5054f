#!/bin/bash
# SQ counter passes for the C2 bench (one counter group per rocprofv3 run; no --pmc with tracing domains).
# usage (GPU box): bash tools/pmc_passes.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1; shift
  timeout -k 10 180 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o "$name" --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/$name.log" 2>&1
}
run waves SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU
echo PMC_DONE
