#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_small_la.py tests/test_nla.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_eig.log 2>&1
rc=$?; tail -15 $OUT/pt_eig.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/eig_tridiag_bench.py > $OUT/eig_bench.jsonl 2>&1; rc=$?; cat $OUT/eig_bench.jsonl; [ $rc -eq 0 ] || exit $rc
[ "${TAIL:-1}" = "1" ] && bash scripts/gpu_tail.sh
