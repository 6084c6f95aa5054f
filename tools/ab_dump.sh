#!/bin/bash
# Bitwise comparison only (no phase stamps): tools/obca_dump.py of every build, each compared with the first.
# usage (GPU box): bash tools/ab_dump.sh OUTDIR NAME=SO [NAME=SO ...]   (SO "" = the in-tree library)
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
first=""
for spec in "$@"; do
  name=${spec%%=*}; so=${spec#*=}
  TTMPC_LIB=$so timeout -k 10 300 python -u tools/obca_dump.py "$OUT/$name.npz" 64 1000 > "$OUT/dump_$name.txt" 2>&1 || { echo "DUMP_FAILED $name"; tail -5 "$OUT/dump_$name.txt"; exit 1; }
  if [ -z "$first" ]; then first=$name; else python tools/obca_dump.py --compare "$OUT/$first.npz" "$OUT/$name.npz" > "$OUT/compare_$name.txt" 2>&1; fi
  echo "done $name"; [ -n "$first" ] && [ "$first" != "$name" ] && head -1 "$OUT/compare_$name.txt"
done
