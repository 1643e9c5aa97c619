#!/bin/bash
# eigensolver accuracy diagnostics, boundary phase stamps, general engine tests + bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 120 python benchmarks/eig_debug.py > $OUT/eig_debug.log 2>&1; rc=$?; cat $OUT/eig_debug.log | grep '^{'; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/core_stamps.py > $OUT/core_stamps.log 2>&1; rc=$?; grep '^{' $OUT/core_stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_rsvd_general.py tests/test_gpu_multirank.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_gen.log 2>&1
prc=$?; grep -E "^(FAILED|ERROR)" $OUT/pt_gen.log; tail -2 $OUT/pt_gen.log
case $prc in 124|134|137|139) exit $prc ;; esac
timeout -k 10 240 python benchmarks/rsvd_general_bench.py > $OUT/gen_bench.log 2>&1; rc=$?; grep '^{' $OUT/gen_bench.log; [ $rc -eq 0 ] || exit $rc
exit $prc
