#!/bin/bash
# One parameterised GPU session (replaces the per-experiment one-off scripts).
# Each argument is a step, run in order; the session stops at the first
# failing step (a GPU fault, abort or time limit ends it: nothing else runs).
#   tests:<pytest selection>   GPU tests (one process, per-test timeout)
#   bench[:<bench.py args>]    bench.py (driver command shape), JSON line kept
#   prof[:<bench.py args>]     rocprofv3 kernel trace + stats of a short bench
#                              run and the one-call timeline (trace_engine.py)
#   pmc:<name>:<counters>      one rocprofv3 --pmc pass over a short bench run
#   py:<script and args>       any python script (benchmarks/*.py), its log kept
# Logs land under gpurun_out/ (merged back by gpurun).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
i=0
for step in "$@"; do
  i=$((i + 1)); kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  log=$OUT/s${i}_${kind}.log
  echo "[step $i] $step"
  case $kind in
    tests)
      timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $arg -m gpu --maxfail=5 -q -p no:cacheprovider \
        --timeout 120 --timeout-method thread > "$log" 2>&1; rc=$?
      grep -E "^(FAILED|ERROR)" "$log"; tail -2 "$log" ;;
    bench)
      timeout -k 10 300 python bench.py ${arg:---steps 20 --warmup 5} > "$log" 2>&1; rc=$?; tail -1 "$log" ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof$i" -o run \
        --output-format csv -- python3 "$ROOT/bench.py" ${arg:---steps 5 --warmup 2} > "$log" 2>&1); rc=$?
      echo "rocprof rc=$rc"
      if [ $rc -eq 0 ]; then
        python scripts/trace_engine.py $(ls "$OUT"/prof$i/*/run_kernel_trace.csv "$OUT"/prof$i/run_kernel_trace.csv 2>/dev/null | head -1) \
          > "$OUT/step$i.txt" 2>&1; head -30 "$OUT/step$i.txt"
      fi ;;
    pmc)
      name=${arg%%:*}; ctr=${arg#*:}
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$OUT/pmc_$name" -o run \
        --output-format csv -- python3 "$ROOT/${PMC_SCRIPT:-bench.py}" ${PMC_ARGS:---steps 2 --warmup 1} > "$log" 2>&1); rc=$?
      echo "pmc $name rc=$rc" ;;
    py)
      PYTHONPATH=$ROOT${PYTHONPATH:+:$PYTHONPATH} timeout -k 10 ${PY_LIMIT:-600} python -u $arg > "$log" 2>&1; rc=$?
      grep '^{' "$log" | tail -20; [ $rc -ne 0 ] && tail -20 "$log" ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  [ $rc -eq 0 ] || { echo "[step $i] failed rc=$rc"; exit $rc; }
done
