#!/bin/bash
# multi-rank rehearsal on the one GPU of the box: multirank / one-shot tests,
# then bench.py under torchrun with 2 and 4 ranks sharing the GPU (gloo: RCCL
# refuses two ranks on one device; answer
# checks; timings are not scaling numbers)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
bash scripts/gpu_mr.sh || exit 1
for n in 2 4; do
  SKH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 2 > $OUT/mr_bench_$n.log 2>&1
  rc=$?; grep '^{' $OUT/mr_bench_$n.log | cut -c1-400; [ $rc -eq 0 ] || { tail -20 $OUT/mr_bench_$n.log; exit $rc; }
done
