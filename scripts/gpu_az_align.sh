set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ts_products.py > gpurun_out/t_aza.log 2>&1 || exit 1
: > gpurun_out/aza_ab.log
for a in 0 1; do
  SL_AZ_ALIGN=$a timeout -k 10 200 python benchmarks/probe/az_time.py shapes >> gpurun_out/aza_ab.log 2>&1 || exit 1
done
for a in 0 1 0 1; do
  timeout -k 10 300 python benchmarks/rsvd_general_bench.py --cases f32,f64 --reps 7 --az-align $a >> gpurun_out/aza_ab.log 2>&1 || exit 1
done
