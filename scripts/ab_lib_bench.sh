#!/bin/bash
# Same-box A/B of two builds of the native library on bench.py: alternates
# ab_old.so / ab_new.so (repo root) as the in-tree library, 3 rounds each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
LIB=libskylark_amd/_native/libskylark_hip.so
for r in 1 2 3; do
  for v in old new; do
    cp ab_$v.so $LIB
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/ab_${v}_$r.log 2>&1 || { echo "bench $v $r failed"; tail -5 $OUT/ab_${v}_$r.log; exit 1; }
    echo "$v $r $(tail -1 $OUT/ab_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms"]["median"])')"
  done
done
cp ab_new.so $LIB
