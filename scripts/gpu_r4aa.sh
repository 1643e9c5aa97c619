#!/bin/bash
# FJLT stage 2 with two columns per lane: tests, bench, kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fjlt.py tests/test_gpu_fjlt_fourstep.py > $OUT/r4aa_tests.log 2>&1
rc=$?; tail -2 $OUT/r4aa_tests.log; [ $rc -ne 0 ] && { grep -m5 -A30 "FAIL\|Error" $OUT/r4aa_tests.log | head -60; exit $rc; }
VARIANTS=fourstep_sampled timeout -k 10 200 python benchmarks/bench_fjlt.py > $OUT/fjlt_r4aa.log 2>&1
rc=$?; grep '^{' $OUT/fjlt_r4aa.log; [ $rc -ne 0 ] && exit $rc
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
VARIANTS=fourstep_sampled timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/fjlt_prof4 -o run --output-format csv -- python3 $ROOT/benchmarks/bench_fjlt.py > $ROOT/$OUT/fjlt_prof4.log 2>&1
