#!/bin/bash
# Round-5 GPU session AG: the forward sweep with alternating lane maps (no ds_bpermute between stages).  Tracking A/B
# against head (bitwise dumps, C2 / C3 / C5 in alternating rounds, stamps, tracking tests) for the in-tree build (all
# unrolled builds) and the fw1 variant (one-wave builds only).   usage: bash tools/gpu_round5ag.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r5ag}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_track_ab2.sh "$OUT" head new fw1 | grep -v "^$" | tail -60 || exit 1
echo R5AG_DONE
