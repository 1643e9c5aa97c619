#!/bin/bash
# One GPU-box session: build, GPU tests, short bench, rocprof kernel stats.
# Every GPU step has its own time limit; a crash/timeout/abort stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
python -m libskylark_amd._native.build > $OUT/build.log 2>&1 || { echo "build failed"; exit 3; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; ok $rc || { echo "pytest rc=$rc, stopping"; exit $rc; }
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; tail -3 $OUT/bench.log; [ $rc -eq 0 ] || { echo "bench rc=$rc, stopping"; exit $rc; }
if [ "${PROFILE:-1}" = "1" ]; then
  ROOT=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 1 ${BENCH_ARGS:-} > $ROOT/$OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
fi
exit 0
