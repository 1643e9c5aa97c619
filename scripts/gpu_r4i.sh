#!/bin/bash
# eigensolver diagnostics + boundary stamps, engine tests, cold bench + trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 120 python benchmarks/eig_debug.py > $OUT/eig_debug.log 2>&1; rc=$?; grep '^{' $OUT/eig_debug.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/core_stamps.py > $OUT/core_stamps.log 2>&1; rc=$?; grep '^{' $OUT/core_stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/eig_stamps.py > $OUT/eig_stamps.log 2>&1; rc=$?; grep '^{' $OUT/eig_stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_rsvd_pass.py tests/test_small_la.py tests/test_gpu_rsvd_core.py tests/test_gpu_rsvd_boundary.py tests/test_gpu_oneshot.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_eng.log 2>&1
prc=$?; grep -E "^(FAILED|ERROR)" $OUT/pt_eng.log; tail -2 $OUT/pt_eng.log
case $prc in 124|134|137|139) exit $prc ;; esac
bash scripts/gpu_bench_prof.sh || exit 1
exit $prc
