#!/bin/bash
# FJLT stage-2 rewrite + ADMM pipelined logging + CWT CSR fetch amplification (FETCH_SIZE)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm_nt.py tests/test_gpu_fjlt.py tests/test_gpu_fjlt_fourstep.py tests/test_gpu_ml.py tests/test_gpu_fused.py tests/test_gpu_kernels.py > $OUT/r4s_tests.log 2>&1
rc=$?; tail -2 $OUT/r4s_tests.log; [ $rc -ne 0 ] && { grep -m5 -A30 "FAIL\|Error" $OUT/r4s_tests.log | head -60; exit $rc; }
GEMM_AB_LIBS=old:$(pwd)/benchmarks/native/libgemm_old.so,prio:$(pwd)/benchmarks/native/libgemm_prio.so timeout -k 10 300 python benchmarks/bench_gemm_nt.py > $OUT/gemm_ab_r4s.log 2>&1
rc=$?; grep '^{' $OUT/gemm_ab_r4s.log; [ $rc -ne 0 ] && { tail -20 $OUT/gemm_ab_r4s.log; exit $rc; }
VARIANTS=fourstep_sampled timeout -k 10 200 python benchmarks/bench_fjlt.py > $OUT/fjlt_r4s.log 2>&1
rc=$?; grep '^{' $OUT/fjlt_r4s.log; [ $rc -ne 0 ] && { tail -20 $OUT/fjlt_r4s.log; exit $rc; }
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
VARIANTS=fourstep_sampled timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/fjlt_prof -o run --output-format csv -- python3 $ROOT/benchmarks/bench_fjlt.py > $ROOT/$OUT/fjlt_prof.log 2>&1 || exit 1
cd $ROOT
timeout -k 10 300 python benchmarks/bench_admm.py --iters 10 > $OUT/admm_r4s.log 2>&1
rc=$?; grep '^{' $OUT/admm_r4s.log; [ $rc -ne 0 ] && { tail -20 $OUT/admm_r4s.log; exit $rc; }
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d $ROOT/$OUT/cwt_pmc -o run --output-format csv -- python3 $ROOT/benchmarks/bench_cwt.py > $ROOT/$OUT/cwt_pmc.log 2>&1
rc=$?; grep '^{' $ROOT/$OUT/cwt_pmc.log; exit $rc
