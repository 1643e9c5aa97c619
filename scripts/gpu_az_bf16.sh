set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ts_products.py > gpurun_out/t_azb.log 2>&1 || exit 1
: > gpurun_out/azb_ab.log
for v in 0 1 0 1; do
  timeout -k 10 300 python benchmarks/rsvd_general_bench.py --cases f32 --reps 7 --az-bf16 $v >> gpurun_out/azb_ab.log 2>&1 || exit 1
done
