#!/bin/bash
# HBM traffic of one bench config's kernel: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes
# (no tracing domains besides --kernel-trace), then SQ instruction / wave counters.
# usage (GPU box): bash tools/hbm_passes.sh OUTDIR [CONFIG]
set -o pipefail
OUT=${1:-gpurun_out/hbm}
CFG=${2:-c2}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o "$name" --output-format csv \
    -- python3 bench.py --config "$CFG" --steps 6 --warmup 1 --cpu-budget 0 --no-latency > "$OUT/$name.log" 2>&1 || { echo "PASS_FAILED $name"; tail -5 "$OUT/$name.log"; exit 1; }
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run waves SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM
find "$OUT" -name '*counter_collection.csv' | sort
echo HBM_DONE
