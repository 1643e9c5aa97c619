#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_nla.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pt_heig.log 2>&1
rc=$?; tail -3 $OUT/pt_heig.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/host_eig_probe3.py; [ $? -eq 0 ] || exit 1
for be in torch scipy numpy; do
  SL_HOST_EIG=$be SKH_TRACE_SVD=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $OUT/heig_$be.log 2> $OUT/heig_$be.trace || exit 1
  echo "$be $(python -c "import json,sys; d=json.loads(open('$OUT/heig_$be.log').read().strip().splitlines()[-1]); print(d['ms_per_step'])") $(tail -1 $OUT/heig_$be.trace)"
done
