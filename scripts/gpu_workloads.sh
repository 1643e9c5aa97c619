#!/bin/bash
# Reference workloads + ADMM (config 4) benchmarks on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python benchmarks/bench_reference_workloads.py --out $OUT/reference_workloads.jsonl > $OUT/refw.log 2>&1
rc=$?; cat $OUT/refw.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/bench_admm.py > $OUT/admm_cached.log 2>&1 && tail -1 $OUT/admm_cached.log
timeout -k 10 600 python benchmarks/bench_admm.py --cache 0 > $OUT/admm_nocache.log 2>&1; tail -2 $OUT/admm_nocache.log
