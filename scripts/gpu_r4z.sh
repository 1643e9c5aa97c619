#!/bin/bash
# FJLT stage 1 with the first radix pass fused into the loads: tests, A/B, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fjlt.py tests/test_gpu_fjlt_fourstep.py > $OUT/r4z_tests.log 2>&1
rc=$?; tail -2 $OUT/r4z_tests.log; [ $rc -ne 0 ] && { grep -m5 -A30 "FAIL\|Error" $OUT/r4z_tests.log | head -60; exit $rc; }
N=$(pwd)/benchmarks/native
FS_AB_LIBS=prev:$N/libfs_base.so,first:$N/libfs_first.so,firstlast:$(pwd)/libskylark_amd/_native/libskylark_hip.so,prev2:$N/libfs_base.so,first2:$N/libfs_first.so,firstlast2:$(pwd)/libskylark_amd/_native/libskylark_hip.so \
  timeout -k 10 300 python benchmarks/fjlt_stage1_ab.py > $OUT/fs1_fused.log 2>&1
rc=$?; grep '^{' $OUT/fs1_fused.log; [ $rc -ne 0 ] && { tail -20 $OUT/fs1_fused.log; exit $rc; }
VARIANTS=fourstep_sampled timeout -k 10 200 python benchmarks/bench_fjlt.py > $OUT/fjlt_r4z.log 2>&1
rc=$?; grep '^{' $OUT/fjlt_r4z.log; exit $rc
