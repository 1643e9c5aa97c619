#!/bin/bash
# round-4 first GPU pass: engine fault / boundary / core tests, cold bench + one-call trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash scripts/gpu_tests_from.sh tests/test_gpu_rsvd_faults.py tests/test_gpu_rsvd_boundary.py tests/test_gpu_rsvd_core.py tests/test_nla.py || exit 1
bash scripts/gpu_bench_prof.sh || exit 1
