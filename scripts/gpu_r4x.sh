#!/bin/bash
# round-4 closing check: full GPU suite, smoke, FJLT / ADMM benches, bench.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests_v5.txt 2>&1
rc=$?; tail -3 $OUT/gpu_tests_v5.txt; [ $rc -ne 0 ] && { grep -m5 -B5 -A40 "FAILED\|Error" $OUT/gpu_tests_v5.txt | head -80; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_v5.log 2>&1
rc=$?; tail -1 $OUT/smoke_v5.log; [ $rc -ne 0 ] && { tail -20 $OUT/smoke_v5.log; exit $rc; }
VARIANTS=fourstep_sampled timeout -k 10 200 python benchmarks/bench_fjlt.py > $OUT/fjlt_r4x2.log 2>&1
rc=$?; grep '^{' $OUT/fjlt_r4x2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_r4x2.log 2>&1
rc=$?; grep '^{' $OUT/bench_r4x2.log; exit $rc
