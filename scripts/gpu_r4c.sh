#!/bin/bash
# tests (failures do not stop the measurements; faults / timeouts do), phase
# stamps, small-LA microbench, then cold bench + trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash scripts/gpu_tests_from.sh tests/test_gpu_rsvd_general.py tests/test_small_la.py tests/test_gpu_rsvd_faults.py tests/test_gpu_rsvd_boundary.py tests/test_gpu_rsvd_core.py tests/test_nla.py tests/test_capi.py
trc=$?
case $trc in 124|134|137|139) exit $trc ;; esac
timeout -k 10 120 python benchmarks/eig_stamps.py > $OUT/eig_stamps.log 2>&1; rc=$?; grep '^{' $OUT/eig_stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/eig_tridiag_bench.py > $OUT/eig_bench.log 2>&1; rc=$?; grep '^{' $OUT/eig_bench.log | grep -v jacobi; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_prof.sh || exit 1
exit $trc
