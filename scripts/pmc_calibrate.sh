#!/bin/bash
# FETCH_SIZE calibration (benchmarks/pmc_calibrate.py): one rocprofv3 --pmc run
# per workload, kernel trace alongside (counters only with kernel trace),
# CSVs and the workloads' JSON lines under gpurun_out/pmc_cal/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_cal
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for OP in ${OPS:-stream ldsdma gather128 gather64 rgather128 rgather64 cwt}; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/$OP -o run -- \
    python3 $R/benchmarks/pmc_calibrate.py --op $OP > $OUT/$OP.log 2>&1 || { echo "pmc $OP failed"; tail -5 $OUT/$OP.log; exit 1; }
  grep '^{' $OUT/$OP.log
done
echo pmc calibration done
