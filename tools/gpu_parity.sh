#!/bin/bash
# GPU side of tools/obca_parity.py for several builds (GPU box).
# usage: bash tools/gpu_parity.sh OUTDIR NAME=SO [NAME=SO ...]   (SO "" = the in-tree library)
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%=*}; so=${spec#*=}
  timeout -k 10 400 python -u tools/obca_parity.py gpu "$OUT/gpu_$name.npz" "$so" > "$OUT/gpu_$name.txt" 2>&1 || { echo "GPU_FAILED $name"; tail -5 "$OUT/gpu_$name.txt"; exit 1; }
  cat "$OUT/gpu_$name.txt"
done
echo PARITY_DONE
