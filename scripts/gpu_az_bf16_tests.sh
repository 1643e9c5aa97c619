set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ts_products.py tests/test_gpu_rsvd_general.py tests/test_gpu_capi_dist.py > gpurun_out/t_azb2.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/rsvd_general_bench.py --cases f32,f64,f32k128 --reps 7 > gpurun_out/azb_gen.log 2>&1
