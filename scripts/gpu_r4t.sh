#!/bin/bash
# FJLT stage 1 at 8 columns per workgroup (4 per CU) + gemm_nt priority build tests + CWT fetch bytes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm_nt.py tests/test_gpu_fjlt.py tests/test_gpu_fjlt_fourstep.py tests/test_gpu_fused.py > $OUT/r4t_tests.log 2>&1
rc=$?; tail -2 $OUT/r4t_tests.log; [ $rc -ne 0 ] && { grep -m5 -A30 "FAIL\|Error" $OUT/r4t_tests.log | head -60; exit $rc; }
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
VARIANTS=fourstep_sampled timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/fjlt_prof2 -o run --output-format csv -- python3 $ROOT/benchmarks/bench_fjlt.py > $ROOT/$OUT/fjlt_prof2.log 2>&1 || exit 1
grep '^{' $ROOT/$OUT/fjlt_prof2.log
cd $ROOT
VARIANTS=fourstep_sampled timeout -k 10 200 python benchmarks/bench_fjlt.py > $OUT/fjlt_r4t.log 2>&1
rc=$?; grep '^{' $OUT/fjlt_r4t.log; [ $rc -ne 0 ] && { tail -20 $OUT/fjlt_r4t.log; exit $rc; }
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $ROOT/$OUT/cwt_pmc -o run --output-format csv -- python3 $ROOT/benchmarks/bench_cwt.py > $ROOT/$OUT/cwt_pmc.log 2>&1
rc=$?; grep '^{' $ROOT/$OUT/cwt_pmc.log; exit $rc
