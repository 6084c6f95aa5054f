#!/bin/bash
# Registers / scratch / LDS of every kernel in one HIP source (device-only compile, gfx950).
# usage: bash tools/kernel_resources.sh car-trailer-mpc_amd/csrc/tt_track.hip
set -e
SRC=${1:-car-trailer-mpc_amd/csrc/tt_track.hip}
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Icar-trailer-mpc_amd/csrc --cuda-device-only -c "$SRC" -o "$T/b.o"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/b.o" --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/k.elf"
/opt/rocm/lib/llvm/bin/llvm-readobj --notes "$T/k.elf" | grep -E '^ +\.name:|private_segment_fixed_size|\.vgpr_count|vgpr_spill_count' \
  | paste - - - - | awk '{printf "%-90s scratch %5s vgpr %4s spill %s\n", $2, $4, $6, $8}'
rm -rf "$T"
