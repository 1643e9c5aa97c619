#!/bin/bash
# fixed tests, feature-map breakdown on gemm_nt, general engine bench, stamps, cold bench + trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_capi.py tests/test_gpu_kernels.py tests/test_gpu_fused.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_fix.log 2>&1
prc=$?; grep -E "^(FAILED|ERROR)" $OUT/pt_fix.log; tail -2 $OUT/pt_fix.log
case $prc in 124|134|137|139) exit $prc ;; esac
timeout -k 10 180 python benchmarks/feature_breakdown.py > $OUT/feature_breakdown.log 2>&1; rc=$?; grep '^{' $OUT/feature_breakdown.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/rsvd_general_bench.py > $OUT/gen_bench.log 2>&1; rc=$?; grep '^{' $OUT/gen_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/core_stamps.py > $OUT/core_stamps.log 2>&1; rc=$?; grep '^{' $OUT/core_stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/eig_stamps.py > $OUT/eig_stamps.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_prof.sh || exit 1
exit $prc
