#!/bin/bash
# rocprofv3 kernel traces of bench.py for ab_old.so and ab_new.so (same box);
# per-position medians by scripts/call_positions.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
LIB=libskylark_amd/_native/libskylark_hip.so
for v in old new; do
  cp ab_$v.so $LIB
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/abprof_$v -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 3 > $OUT/abprof_$v.log 2>&1) || { echo "prof $v failed"; tail -5 $OUT/abprof_$v.log; exit 1; }
  echo "== $v"; python scripts/call_positions.py $(ls $OUT/abprof_$v/*/run_kernel_trace.csv $OUT/abprof_$v/run_kernel_trace.csv 2>/dev/null | head -1) 3
done
cp ab_new.so $LIB
