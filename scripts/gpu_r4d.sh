#!/bin/bash
# round-4 validation + measurements in one call: GPU tests (failures do not
# stop the measurements; faults / timeouts do), cold bench + trace, general
# engine at the reference's sizes, small-LA microbench, v4-pass PMC counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash scripts/gpu_tests_from.sh tests/test_gpu_rsvd_general.py tests/test_small_la.py tests/test_gpu_rsvd_faults.py tests/test_gpu_rsvd_boundary.py tests/test_gpu_rsvd_core.py tests/test_nla.py tests/test_capi.py tests/test_gpu_kernels.py tests/test_gpu_fused.py tests/test_gpu_gemm_nt.py
trc=$?
case $trc in 124|134|137|139) exit $trc ;; esac
bash scripts/gpu_bench_prof.sh || exit 1
timeout -k 10 180 python benchmarks/bench_gemm_nt.py > $OUT/gemm_bench.log 2>&1; rc=$?; grep '^{' $OUT/gemm_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python benchmarks/rsvd_general_bench.py > $OUT/gen_bench.log 2>&1; rc=$?; grep '^{' $OUT/gen_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/eig_tridiag_bench.py > $OUT/eig_bench.log 2>&1; rc=$?; grep '^{' $OUT/eig_bench.log | grep -v jacobi; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_pass4.sh || exit 1
python scripts/pmc_summary4.py $OUT/pmc4 $OUT/pmc4_csv > $OUT/pmc4.md 2>&1
exit $trc
