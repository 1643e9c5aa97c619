#!/bin/bash
# 1-GPU bench.py (driver command shape) + rocprofv3 kernel trace of a short run + one-call timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 5 --warmup 2 > $ROOT/$OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $ROOT && python scripts/trace_engine.py $(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step.txt 2>&1; head -40 $OUT/step.txt
