#!/bin/bash
# FJLT four-step stage 2 on scalar twiddles: test + bench + kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fjlt_fourstep.py tests/test_gpu_fjlt.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_fjlt.log 2>&1
prc=$?; grep -E "^(FAILED|ERROR)" $OUT/pt_fjlt.log; tail -2 $OUT/pt_fjlt.log
case $prc in 124|134|137|139) exit $prc ;; esac
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
VARIANTS=fourstep_sampled timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/fjlt_prof -o run --output-format csv -- python3 $ROOT/benchmarks/bench_fjlt.py > $ROOT/$OUT/fjlt_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
cd $ROOT; f=$(ls $OUT/fjlt_prof/*/run_kernel_stats.csv $OUT/fjlt_prof/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && grep "k_fs" "$f" | cut -c1-200
VARIANTS=fourstep_sampled timeout -k 10 120 python benchmarks/bench_fjlt.py > $OUT/fjlt_bench.log 2>&1; grep '^{' $OUT/fjlt_bench.log
exit $prc
