#!/bin/bash
# contiguous Y stores in the final pass: pass / engine tests, pass timing, cold bench + trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_rsvd_pass.py tests/test_gpu_rsvd_core.py tests/test_gpu_rsvd_boundary.py tests/test_gpu_oneshot.py tests/test_gpu_multirank.py tests/test_gpu_rsvd_faults.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_eng.log 2>&1
prc=$?; grep -E "^(FAILED|ERROR)" $OUT/pt_eng.log; tail -2 $OUT/pt_eng.log
case $prc in 124|134|137|139) exit $prc ;; esac
timeout -k 10 300 python benchmarks/pass_nt_ab.py > $OUT/pass_nt_ab.log 2>&1; rc=$?; grep '^{' $OUT/pass_nt_ab.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_prof.sh || exit 1
exit $prc
