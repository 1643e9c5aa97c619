#!/bin/bash
# GPU session for the fused feature GEMM: tests, throughput, rocprof stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
rm -f $OUT/bench_features.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_fused.log 2>&1
rc=$?; tail -3 $OUT/pytest_fused.log; [ $rc -eq 0 ] || exit $rc
for args in ${FEAT_ARGS:-"--modes fused" "--modes fused --columnwise" "--modes fused --dtype bf16"}; do
  timeout -k 10 300 python benchmarks/bench_features.py $args >> $OUT/bench_features.jsonl 2>> $OUT/bench_features.err || exit $?
done
cat $OUT/bench_features.jsonl
if [ "${PROFILE:-0}" = "1" ]; then
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_feat -o run --output-format csv -- python3 $ROOT/benchmarks/bench_features.py --steps 3 > $ROOT/$OUT/prof_feat.log 2>&1
echo "rocprof rc=$?"
fi
