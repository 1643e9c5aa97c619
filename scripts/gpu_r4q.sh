#!/bin/bash
# BlockADMM kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/admm_prof -o run --output-format csv -- python3 $ROOT/benchmarks/bench_admm.py --iters 10 > $ROOT/$OUT/admm_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep '^{' $ROOT/$OUT/admm_prof.log
cd $ROOT; f=$(ls $OUT/admm_prof/*/run_kernel_stats.csv $OUT/admm_prof/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:16]: print(r['Calls'], round(float(r['TotalDurationNs'])/1e6,2), 'ms', round(float(r['AverageNs'])/1e3,1),'us', r['Name'][:90])
"
exit $rc
