#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_oneshot.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pt_mr.log 2>&1
rc=$?; tail -12 $OUT/pt_mr.log; exit $rc
