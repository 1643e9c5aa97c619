#!/bin/bash
# C-ABI device test; FJLT four-step kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_capi.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pt_capi.log 2>&1
prc=$?; grep -E "^(FAILED|ERROR)" $OUT/pt_capi.log; tail -2 $OUT/pt_capi.log
case $prc in 124|134|137|139) exit $prc ;; esac
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
VARIANTS=fourstep_sampled timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/fjlt_prof -o run --output-format csv -- python3 $ROOT/benchmarks/bench_fjlt.py > $ROOT/$OUT/fjlt_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep '^{' $ROOT/$OUT/fjlt_prof.log
cd $ROOT; f=$(ls $OUT/fjlt_prof/*/run_kernel_stats.csv $OUT/fjlt_prof/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -12 "$f" | cut -c1-220
exit $prc
