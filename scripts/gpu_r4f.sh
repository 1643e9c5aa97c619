#!/bin/bash
# in-pass Gram checks (pass-level + engine tests), then the general engine
# bench, the eig phase stamps and the cold bench + trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_rsvd_pass.py tests/test_gpu_oneshot.py tests/test_gpu_rsvd_general.py tests/test_small_la.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_pass.log 2>&1
prc=$?; grep -E "^(FAILED|ERROR)" $OUT/pt_pass.log; tail -2 $OUT/pt_pass.log
case $prc in 124|134|137|139) exit $prc ;; esac
timeout -k 10 240 python benchmarks/rsvd_general_bench.py > $OUT/gen_bench.log 2>&1; rc=$?; grep '^{' $OUT/gen_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/eig_stamps.py > $OUT/eig_stamps.log 2>&1; rc=$?; grep '^{' $OUT/eig_stamps.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_prof.sh || exit 1
exit $prc
