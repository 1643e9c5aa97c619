#!/bin/bash
# bench.py (engine path) + a rocprofv3 kernel trace of a few steps + one-step timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/eb.log 2>&1
rc=$?; tail -1 $OUT/eb.log; [ $rc -eq 0 ] || exit $rc
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_eng -o run --output-format csv -- python3 $ROOT/bench.py --steps 4 --warmup 2 > $ROOT/$OUT/prof_eng.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $ROOT && python scripts/trace_engine.py $(ls $OUT/prof_eng/*/run_kernel_trace.csv $OUT/prof_eng/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/eng_step.txt 2>&1; cat $OUT/eng_step.txt
