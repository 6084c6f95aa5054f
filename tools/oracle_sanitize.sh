#!/bin/bash
# The CPU test suite against the ASan + UBSan build of the C oracle (CPU only).
# usage: bash tools/oracle_sanitize.sh [pytest args]   -> log in gpurun_out/sanitize/
set -o pipefail
cd "$(dirname "$0")/.."
make -s -C oracle sanitize || exit 1
mkdir -p gpurun_out/sanitize
TTO_ORACLE_LIB=oracle/build/libttoracle_san.so LD_PRELOAD=$(gcc -print-file-name=libasan.so) \
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
  python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider "$@" 2>&1 | tee gpurun_out/sanitize/pytest_san.log
