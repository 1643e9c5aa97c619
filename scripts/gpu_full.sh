#!/bin/bash
# Full GPU suite, smoke, 1-GPU bench (+ optional rocprof stats of the bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_full.log 2>&1
rc=$?; tail -4 $OUT/pt_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/bench_full.log 2>&1; rc=$?; tail -1 $OUT/bench_full.log; [ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-0}" = "1" ]; then
  ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_full -o run --output-format csv -- python3 $ROOT/bench.py --steps 5 --warmup 2 > $ROOT/$OUT/prof_full.log 2>&1
  echo "rocprof rc=$?"
fi
