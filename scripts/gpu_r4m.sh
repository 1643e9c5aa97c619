#!/bin/bash
# config 4: FasterKernelRidge to convergence, BlockADMM iteration time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 500 python benchmarks/krr_cg.py > $OUT/krr_cg.log 2>&1; rc=$?; grep '^{' $OUT/krr_cg.log; tail -3 $OUT/krr_cg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_admm.py > $OUT/admm.log 2>&1; rc=$?; grep '^{' $OUT/admm.log; tail -3 $OUT/admm.log; exit $rc
