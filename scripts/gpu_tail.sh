#!/bin/bash
# randSVD per-call tail: host phase stamps, host eigensolve probe, kernel trace of one step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
SKH_TRACE_SVD=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/tail_bench.log 2> $OUT/tail_trace.log
rc=$?; tail -1 $OUT/tail_bench.log; tail -3 $OUT/tail_trace.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/probe/host_eig_probe2.py > $OUT/tail_eig.log 2>&1; cat $OUT/tail_eig.log
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/$OUT/prof_tail -o run --output-format csv -- python3 $ROOT/bench.py --steps 4 --warmup 2 > $ROOT/$OUT/prof_tail.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $ROOT && python scripts/trace_step.py $(ls $OUT/prof_tail/*/run_kernel_trace.csv $OUT/prof_tail/run_kernel_trace.csv 2>/dev/null | head -1) -v > $OUT/tail_step.txt 2>&1; head -60 $OUT/tail_step.txt
