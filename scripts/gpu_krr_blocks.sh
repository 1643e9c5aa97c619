set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ml.py -k "split_gram or ridge_split" > gpurun_out/t_krr.log 2>&1 || exit 1
: > gpurun_out/krr_blocks_ab.log
for r in 1 2; do for b in 1 2 4 8; do
  SKH_KRR_GRAM_BLOCKS=$b timeout -k 10 200 python -u benchmarks/bench_krr.py > gpurun_out/krr_b.log 2>&1 || exit 1
  echo "{\"blocks\": $b, \"round\": $r, \"line\": $(grep '^{' gpurun_out/krr_b.log | tail -1)}" >> gpurun_out/krr_blocks_ab.log
done; done
