#!/bin/bash
# One GPU session on the box, as a list of steps run in order (replaces round 5's one-off tools/gpu_round5*.sh scripts;
# git history keeps them at d92cdc6, and each profiles/r05/*/SOURCE.txt still names the one that produced it).
# Every step that touches the GPU has its own time limit; the first failing step ends the session (no retries).
#
# usage (GPU box):  bash tools/gpu_session.sh OUTDIR STEP [STEP ...]
# steps:
#   tests[:K]                pytest -m gpu (optionally -k K), log OUT/tests.log
#   smoke                    __graft_entry__.smoke()
#   bench:CFG[:ARGS]         python bench.py --config CFG ARGS (ARGS: comma-separated, e.g. --steps,5) -> OUT/bench_CFG.json
#   ab:CFG:ROUNDS:N1=SO1,..[:ARGS]  alternating rounds of bench CFG over builds (TTMPC_LIB=SO; empty SO = in-tree)
#   prof:CFG[:ARGS]          rocprofv3 --kernel-trace --stats of bench CFG -> OUT/prof_CFG/
#   pmc:CFG:NAME:CTR[,CTR]   one rocprofv3 --pmc pass of bench CFG (one counter group per pass) -> OUT/pmc_CFG/NAME/
#   hbm:CFG[:ARGS]           FETCH_SIZE and WRITE_SIZE passes of bench CFG (separate runs) -> OUT/pmc_CFG/{fetch,write}
#   ubench:NAME              tools/bin/ubench_NAME (built on the CPU side) -> OUT/ubench_NAME.txt
#   py:SCRIPT[:ARGS]         python -u SCRIPT ARGS (diagnostic tools, e.g. tools/obca_tail.py) -> OUT/py_<script>.txt
#   pmcpy:NAME:CTR[,CTR]:SCRIPT[:ARGS]  one rocprofv3 --pmc pass over python3 SCRIPT ARGS -> OUT/pmcpy/NAME/ (+ run.json:
#                            the script's JSON stdout line)
#   listpmc                  rocprofv3 -L (the counters this box offers) -> OUT/counters.txt
#   abobca:N1=SO1,N2=SO2..   tools/ab_obca.sh: bitwise OBCA dumps against the first build + c4 phase stamps -> OUT/obca/
set -o pipefail
OUT=${1:?usage: gpu_session.sh OUTDIR STEP...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
fail() { echo "STEP_FAILED $1"; [ -f "$2" ] && tail -25 "$2"; exit 1; }
args() { echo "${1//,/ }"; }

for step in "$@"; do
  IFS=: read -r kind a1 a2 a3 a4 <<< "$step"
  echo "== $step ($(date +%H:%M:%S))"
  case "$kind" in
    tests)
      log="$OUT/tests.log"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${a1:+-k "$a1"} \
        > "$log" 2>&1 || fail "$step" "$log"
      tail -2 "$log" ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || fail "$step" "$OUT/smoke.log"
      cat "$OUT/smoke.log" ;;
    bench)
      j="$OUT/bench_$a1.json"
      n=2; while [ -e "$j" ]; do j="$OUT/bench_${a1}_$n.json"; n=$((n + 1)); done
      timeout -k 10 600 python -u bench.py --config "$a1" $(args "$a2") > "$j" 2> "${j%.json}.err" || fail "$step" "${j%.json}.err"
      cat "$j" ;;
    ab)
      for r in $(seq 1 "$a2"); do
        for spec in ${a3//,/ }; do
          name=${spec%%=*}; so=${spec#*=}
          j="$OUT/ab_${a1}_${name}_$r.json"
          TTMPC_LIB=$so timeout -k 10 600 python -u bench.py --config "$a1" --cpu-budget 0 --no-latency $(args "$a4") \
            > "$j" 2> "${j%.json}.err" \
            || fail "$step $name" "${j%.json}.err"
          python -c "import json; d=json.load(open('$j')); print('$a1 $name $r', d['value'], d['ms_per_step'])"
        done
      done ;;
    prof)
      d="$OUT/prof_$a1"
      n=2; while [ -e "$d" ]; do d="$OUT/prof_${a1}_$n"; n=$((n + 1)); done
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv \
        -- python3 bench.py --config "$a1" --cpu-budget 0 --no-latency $(args "$a2") > "$d.log" 2>&1 || fail "$step" "$d.log"
      find "$d" -name '*kernel_stats.csv' -exec head -4 {} \; ;;
    pmc)
      d="$OUT/pmc_$a1/$a2"
      mkdir -p "$d"
      timeout -s KILL 300 rocprofv3 --pmc $(args "$a3") --kernel-trace -d "$d" -o "$a2" --output-format csv \
        -- python3 bench.py --config "$a1" --steps 3 --warmup 1 --cpu-budget 0 --no-latency > "$d.log" 2>&1 || fail "$step" "$d.log"
      echo "$d" ;;
    hbm)
      for c in FETCH_SIZE WRITE_SIZE; do
        n=$(echo "$c" | cut -d_ -f1 | tr A-Z a-z)
        d="$OUT/pmc_$a1/$n"
        mkdir -p "$d"
        timeout -s KILL 300 rocprofv3 --pmc "$c" --kernel-trace -d "$d" -o "$n" --output-format csv \
          -- python3 bench.py --config "$a1" --cpu-budget 0 --no-latency $(args "$a2") > "$d.log" 2>&1 || fail "$step $c" "$d.log"
        grep "^{\"metric\"" "$d.log" > "$d.bench.json"
      done ;;
    ubench)
      timeout -k 10 300 "tools/bin/ubench_$a1" > "$OUT/ubench_$a1.txt" 2>&1 || fail "$step" "$OUT/ubench_$a1.txt"
      cat "$OUT/ubench_$a1.txt" ;;
    py)
      f="$OUT/py_$(basename "$a1" .py).txt"
      timeout -k 10 600 python -u "$a1" $(args "$a2") > "$f" 2>&1 || fail "$step" "$f"
      tail -30 "$f" ;;
    pmcpy)
      d="$OUT/pmcpy/$a1"
      mkdir -p "$d"
      timeout -s KILL 400 rocprofv3 --pmc $(args "$a2") --kernel-trace -d "$d" -o "$a1" --output-format csv \
        -- python3 "$a3" $(args "$a4") > "$d.log" 2>&1 || fail "$step" "$d.log"
      grep "^{" "$d.log" > "$d/run.json"
      cat "$d/run.json" ;;
    abobca)
      timeout -k 10 900 bash tools/ab_obca.sh "$OUT/obca" ${a1//,/ } > "$OUT/obca_ab.txt" 2>&1 || fail "$step" "$OUT/obca_ab.txt"
      grep -E "bitwise|identical|differ|TOTAL|total|iters" "$OUT/obca_ab.txt" | head -40 ;;
    listpmc)
      timeout -s KILL 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || fail "$step" "$OUT/counters.txt"
      wc -l "$OUT/counters.txt" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo SESSION_DONE
