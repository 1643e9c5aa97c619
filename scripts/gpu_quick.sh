#!/bin/bash
# Quick GPU session: selected GPU tests (PYTEST_SEL), bench, optional rocprof.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 ${PYTEST_TIMEOUT:-400} python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_q.log 2>&1
rc=$?; tail -4 $OUT/pytest_q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} > $OUT/bench_q.log 2>&1
rc=$?; tail -1 $OUT/bench_q.log; [ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_q -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 1 ${BENCH_ARGS:-} > $ROOT/$OUT/prof_q.log 2>&1
  echo "rocprof rc=$?"
fi
