set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ts_products.py tests/test_gpu_rsvd_general.py > gpurun_out/t_atq128.log 2>&1 || exit 1
bash scripts/ab_lib_cmd.sh python benchmarks/probe/atq_time.py k128 > gpurun_out/atq128_ab.log 2>&1 || exit 1
bash scripts/ab_lib_cmd.sh python benchmarks/rsvd_general_bench.py --cases f32k128 --reps 5 --no-ref >> gpurun_out/atq128_ab.log 2>&1
