#!/bin/bash
# Selected GPU tests, then bench A/B over an env knob: AB_VAR=name AB_VALS="0 1".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
if [ -n "${PYTEST_SEL:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-400} python -u -m pytest $PYTEST_SEL -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_ab.log 2>&1
  rc=$?; tail -4 $OUT/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
fi
for v in ${AB_VALS:-0 1}; do
  env ${AB_VAR:-SL_NONE}=$v timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 ${BENCH_ARGS:-} > $OUT/bench_ab_$v.log 2>&1
  rc=$?; echo "${AB_VAR:-SL_NONE}=$v: $(tail -1 $OUT/bench_ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["check"])')"; [ $rc -eq 0 ] || exit $rc
done
