#!/bin/bash
# FJLT stage 1: composite radix-20/25 passes -- tests, then radix-plan timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fjlt.py tests/test_gpu_fjlt_fourstep.py > $OUT/r4w_tests.log 2>&1
rc=$?; tail -2 $OUT/r4w_tests.log; [ $rc -ne 0 ] && { grep -m5 -A30 "FAIL\|Error" $OUT/r4w_tests.log | head -60; exit $rc; }
FS_PLANS=4-5-5-5,25-20,20-5-5,25-4-5,4-5-5-5 FS_AB_LIBS=main:$(pwd)/libskylark_amd/_native/libskylark_hip.so \
  timeout -k 10 300 python benchmarks/fjlt_stage1_ab.py > $OUT/fs1_plans.log 2>&1
rc=$?; grep '^{' $OUT/fs1_plans.log; [ $rc -ne 0 ] && { tail -20 $OUT/fs1_plans.log; exit $rc; }
VARIANTS=fourstep_sampled timeout -k 10 200 python benchmarks/bench_fjlt.py > $OUT/fjlt_r4w.log 2>&1
rc=$?; grep '^{' $OUT/fjlt_r4w.log; exit $rc
