#!/bin/bash
# rocprofv3 kernel stats of the FJLT sketch bench (four-step stages vs the rocFFT pipeline)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_fjlt -o run --output-format csv -- python3 $ROOT/benchmarks/bench_fjlt.py > $ROOT/$OUT/prof_fjlt.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $ROOT && python - <<'PY'
import csv, glob
f = (glob.glob("gpurun_out/prof_fjlt/*/run_kernel_stats.csv") + glob.glob("gpurun_out/prof_fjlt/run_kernel_stats.csv"))[0]
for r in csv.DictReader(open(f)):
    if "k_fs_" in r["Name"]:
        print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {r['Name'][:100]}")
PY
