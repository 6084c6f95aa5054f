#!/bin/bash
# GPU side of the OBCA parity / lockstep census (tools/obca_parity.py) + the OBCA GPU tests (GPU box).
# usage: bash tools/gpu_lock.sh OUTDIR [SO]
set -o pipefail
OUT=$1; SO=${2:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/obca_parity.py lock-gpu "$OUT/lock_gpu.npz" "$SO" > "$OUT/lock_gpu.txt" 2>&1 || { echo LOCK_FAILED; tail -5 "$OUT/lock_gpu.txt"; exit 1; }
OBCA_PARITY_FULL=1 timeout -k 10 300 python -u tools/obca_parity.py gpu "$OUT/gpu.npz" "$SO" > "$OUT/gpu.txt" 2>&1 || { echo GPU_FAILED; tail -5 "$OUT/gpu.txt"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_obca.py -m gpu -v --timeout 300 --timeout-method thread > "$OUT/t_obca.log" 2>&1; echo "obca tests rc=$?"
tail -15 "$OUT/t_obca.log"
echo LOCK_DONE
