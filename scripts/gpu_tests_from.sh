#!/bin/bash
# GPU tests of the given files / node ids (one process), log under gpurun_out/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest "$@" -m gpu --maxfail=5 -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_sel.log 2>&1
rc=$?; grep -E "^(FAILED|ERROR)" $OUT/pt_sel.log; tail -2 $OUT/pt_sel.log; exit $rc
