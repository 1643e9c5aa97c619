#!/bin/bash
# the full GPU suite (failures listed; faults / timeouts stop the script)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=40 -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_all.log 2>&1
trc=$?; grep -E "^(FAILED|ERROR)" $OUT/pt_all.log; tail -2 $OUT/pt_all.log
exit $trc
