#!/bin/bash
# NT GEMM: current (deferred + priority) vs plain loop vs plain loop + priority
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
N=$(pwd)/benchmarks/native
GEMM_AB_LIBS=old:$N/libgemm_old.so,oldprio:$N/libgemm_oldprio.so timeout -k 10 400 python benchmarks/bench_gemm_nt.py > $OUT/gemm_ab_r4y.log 2>&1
rc=$?; grep '^{' $OUT/gemm_ab_r4y.log; [ $rc -ne 0 ] && tail -20 $OUT/gemm_ab_r4y.log; exit $rc
