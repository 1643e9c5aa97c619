#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 240 python -u -m pytest tests/test_gpu_oneshot.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pt_oneshot.log 2>&1
rc=$?; tail -30 $OUT/pt_oneshot.log; exit $rc
