#!/bin/bash
# Same-box A/B of two builds of the native library (ab_old.so / ab_new.so at
# the repo root): the pass kernel alone (bench_pass.py) and the headline call
# (bench.py), alternating, 2 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
LIB=libskylark_amd/_native/libskylark_hip.so
for r in 1 2; do
  for v in old new; do
    cp ab_$v.so $LIB
    timeout -k 10 200 python benchmarks/bench_pass.py --variants ${PASS_VARIANTS:-0,256} --finals 0,1 --reps 10 > $OUT/abp_${v}_$r.jsonl 2>&1 || { echo "pass $v $r failed"; tail -5 $OUT/abp_${v}_$r.jsonl; exit 1; }
    grep variant $OUT/abp_${v}_$r.jsonl | sed "s/^/$v $r /"
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/ab_${v}_$r.log 2>&1 || { echo "bench $v $r failed"; tail -5 $OUT/ab_${v}_$r.log; exit 1; }
    echo "$v $r bench $(tail -1 $OUT/ab_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms"]["median"], d["check"]["ok"])')"
  done
done
cp ab_new.so $LIB
