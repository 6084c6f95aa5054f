#!/bin/bash
# A/B of OBCA builds on the GPU box: bitwise output comparison against the first (tools/obca_dump.py) and phase
# stamps at B = 256 (tools/obca_stamps.py 256 c4 300).
# usage: bash tools/ab_obca.sh OUTDIR NAME=SO [NAME=SO ...]   (SO "" = the in-tree library)
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
first=""
for spec in "$@"; do
  name=${spec%%=*}; so=${spec#*=}
  TTMPC_LIB=$so timeout -k 10 300 python -u tools/obca_dump.py "$OUT/$name.npz" 64 1000 > "$OUT/dump_$name.txt" 2>&1 || { echo "DUMP_FAILED $name"; tail -5 "$OUT/dump_$name.txt"; exit 1; }
  if [ -z "$first" ]; then first=$name; else python tools/obca_dump.py --compare "$OUT/$first.npz" "$OUT/$name.npz" > "$OUT/compare_$name.txt" 2>&1; fi
  TTMPC_LIB=$so timeout -k 10 300 python -u tools/obca_stamps.py 256 c4 300 > "$OUT/stamps_$name.txt" 2>&1 || { echo "STAMPS_FAILED $name"; tail -5 "$OUT/stamps_$name.txt"; exit 1; }
done
for f in "$OUT"/dump_*.txt "$OUT"/compare_*.txt "$OUT"/stamps_*.txt; do echo "== $f"; cat "$f"; done
