#!/bin/bash
# Same-box A/B of two builds of the native library (ab_old.so / ab_new.so at
# the repo root) on an arbitrary command: "$@" runs with each build in place,
# alternating, ROUNDS rounds (default 2); output to gpurun_out/ablib_<v>_<r>.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
LIB=libskylark_amd/_native/libskylark_hip.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in old new; do
    cp ab_$v.so $LIB
    timeout -k 10 ${STEP_TIMEOUT:-200} "$@" > $OUT/ablib_${v}_$r.log 2>&1 || { echo "$v $r failed"; tail -5 $OUT/ablib_${v}_$r.log; cp ab_new.so $LIB; exit 1; }
    grep '^{' $OUT/ablib_${v}_$r.log | sed "s/^/$v $r /"
  done
done
cp ab_new.so $LIB
