#!/bin/bash
# Run a command on the GPU box with a heartbeat file under gpurun_out/ (long solves print nothing for minutes).
# usage: bash tools/gpu_hb.sh OUTDIR -- cmd args...
OUT=$1; shift; shift
mkdir -p "$OUT"
( while true; do date +%T >> "$OUT/heartbeat.txt"; sleep 20; done ) &
HB=$!
"$@"
rc=$?
kill $HB 2>/dev/null
exit $rc
