#!/bin/bash
# full GPU suite (failures listed, faults / timeouts stop), then the general
# engine bench, small-LA microbench, cold bench + trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=30 -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_all.log 2>&1
trc=$?; grep -E "^(FAILED|ERROR)" $OUT/pt_all.log; tail -2 $OUT/pt_all.log
case $trc in 124|134|137|139) exit $trc ;; esac
timeout -k 10 240 python benchmarks/rsvd_general_bench.py > $OUT/gen_bench.log 2>&1; rc=$?; grep '^{' $OUT/gen_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/eig_stamps.py > $OUT/eig_stamps.log 2>&1; rc=$?; grep '^{' $OUT/eig_stamps.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_prof.sh || exit 1
exit $trc
