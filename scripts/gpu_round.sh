#!/bin/bash
# engine-focused GPU step: core / engine tests, phase stamps, bench + trace, FJLT four-step tests + bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash scripts/gpu_tests_from.sh tests/test_gpu_rsvd_core.py tests/test_nla.py tests/test_capi.py || exit 1
timeout -k 10 120 python benchmarks/core_stamps.py > $OUT/core_stamps.log 2>&1; rc=$?; grep '^{' $OUT/core_stamps.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_prof.sh || exit 1
bash scripts/gpu_tests_from.sh tests/test_gpu_fjlt_fourstep.py || exit 1
timeout -k 10 200 python benchmarks/bench_fjlt.py > $OUT/fjlt.log 2>&1; rc=$?; cat $OUT/fjlt.log | grep '^{'; [ $rc -eq 0 ] || exit $rc
if [ "${FJLT_PROF:-0}" = "1" ]; then
  ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_fjlt -o run --output-format csv -- python3 $ROOT/benchmarks/bench_fjlt.py > $ROOT/$OUT/prof_fjlt.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd $ROOT && python - <<'PY'
import csv, glob
f = (glob.glob("gpurun_out/prof_fjlt/*/run_kernel_stats.csv") + glob.glob("gpurun_out/prof_fjlt/run_kernel_stats.csv"))[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {r['Name'][:100]}")
PY
fi
