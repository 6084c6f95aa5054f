#!/bin/bash
# Tracking-kernel A/B incl. C5 (GPU box): bitwise dumps (tools/track_dump.py) of each build against the first, C2 / C3 bench
# lines in alternating rounds, phase stamps of the in-tree build, then the tracking GPU tests.
# usage: bash tools/gpu_track_ab2.sh OUTDIR NAME ...   (NAME = ttmpc/variants/libttmpc_NAME.so or "new" = in-tree)
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
V=$PWD/car-trailer-mpc_amd/ttmpc/variants
lib() { if [ "$1" = new ]; then echo ""; else echo "$V/libttmpc_$1.so"; fi; }
first=""
for n in "$@"; do
  TTMPC_LIB=$(lib $n) timeout -k 10 300 python -u tools/track_dump.py "$OUT/dump_$n.npz" > "$OUT/dump_$n.txt" 2>&1 || { echo "DUMP_FAILED $n"; tail -5 "$OUT/dump_$n.txt"; exit 1; }
  if [ -z "$first" ]; then first=$n; else python tools/track_dump.py --compare "$OUT/dump_$first.npz" "$OUT/dump_$n.npz" > "$OUT/compare_$n.txt" 2>&1; tail -1 "$OUT/compare_$n.txt"; fi
done
for r in 1 2 3; do
  for n in "$@"; do
    for cfg in c2 c3 c5; do
      TTMPC_LIB=$(lib $n) timeout -k 10 120 python bench.py --config $cfg --steps 20 --warmup 3 --cpu-budget 0 --no-latency > "$OUT/${n}_${cfg}_$r.json" 2> "$OUT/${n}_${cfg}_$r.err" || { echo "BENCH_FAILED $n $cfg"; tail -5 "$OUT/${n}_${cfg}_$r.err"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/${n}_${cfg}_$r.json')); print('$n', '$cfg', $r, d['value'], d['solver']['kernel_ms_per_launch'])"
    done
  done
done
timeout -k 10 120 python -u tools/phase_stamps.py 1024 20 > "$OUT/track_stamps.txt" 2>&1 || { echo TSTAMPS_FAILED; tail -5 "$OUT/track_stamps.txt"; exit 1; }
cat "$OUT/track_stamps.txt"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sim.py tests/test_gpu_multirank.py -m gpu -v --timeout 300 --timeout-method thread > "$OUT/t_track.log" 2>&1; rc=$?
echo "track tests rc=$rc"; tail -2 "$OUT/t_track.log"; grep -E "FAILED|ERROR" "$OUT/t_track.log" | head
echo TRACK_AB_DONE
