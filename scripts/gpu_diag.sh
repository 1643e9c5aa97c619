#!/bin/bash
# small-LA phase stamps, FJLT four-step kernel stats, feature-map GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 120 python benchmarks/core_stamps.py > $OUT/core_stamps.log 2>&1; rc=$?; cat $OUT/core_stamps.log | grep '^{'; [ $rc -eq 0 ] || exit $rc
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_fjlt -o run --output-format csv -- python3 $ROOT/benchmarks/bench_fjlt.py > $ROOT/$OUT/prof_fjlt.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $ROOT
python - <<'PY'
import csv, glob
f = (glob.glob("gpurun_out/prof_fjlt/*/run_kernel_stats.csv") + glob.glob("gpurun_out/prof_fjlt/run_kernel_stats.csv"))[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {r['Name'][:110]}")
PY
bash scripts/gpu_tests_from.sh tests/test_gpu_fused.py tests/test_gpu_fjlt.py
