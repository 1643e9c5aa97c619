#!/bin/bash
# ata pass prefetch: tests + BlockADMM profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_normal_eq.py tests/test_gpu_krylov.py tests/test_gpu_ml.py > $OUT/r4r_tests.log 2>&1
rc=$?; tail -3 $OUT/r4r_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_r4q.sh
