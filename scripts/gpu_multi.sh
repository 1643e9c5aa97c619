#!/bin/bash
# Run a list of GPU steps (each "name|timeout|command"), stop at the first
# failure; logs under gpurun_out/<name>.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "== $name"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "step $name rc=$rc"; exit $rc; fi
done
