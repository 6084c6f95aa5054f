#!/bin/bash
# Build the library of another git revision as an A/B variant (CPU side): the kernels and ABI of REV, compiled like the
# in-tree build, into car-trailer-mpc_amd/ttmpc/variants/libttmpc_NAME.so (TTMPC_LIB=... selects it in the tools).
# usage: bash tools/build_rev.sh REV NAME [extra hipcc flags]
set -eo pipefail
REV=$1; NAME=$2; shift 2
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
mkdir -p "$T/include" "$T/csrc"
git show "$REV:include/ttmpc.h" > "$T/include/ttmpc.h"
for f in $(git ls-tree --name-only "$REV" car-trailer-mpc_amd/csrc/); do git show "$REV:$f" > "$T/csrc/$(basename "$f")"; done
mkdir -p car-trailer-mpc_amd/ttmpc/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I"$T/include" -I"$T/csrc" "$@" \
  -shared -o "car-trailer-mpc_amd/ttmpc/variants/libttmpc_$NAME.so" "$T"/csrc/tt_track.hip "$T"/csrc/tt_obca.hip \
  "$T"/csrc/tt_sim.hip "$T"/csrc/tt_lqr.hip "$T"/csrc/tt_api.hip
echo "built variants/libttmpc_$NAME.so from $REV"
