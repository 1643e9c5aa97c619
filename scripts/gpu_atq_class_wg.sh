set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ts_products.py tests/test_gpu_rsvd_general.py > gpurun_out/t_atqc.log 2>&1 || exit 1
bash scripts/ab_lib_cmd.sh python benchmarks/probe/atq_time.py > gpurun_out/atqc_ab.log 2>&1 || exit 1
bash scripts/ab_lib_cmd.sh python benchmarks/rsvd_general_bench.py --cases f32 --reps 7 --no-ref >> gpurun_out/atqc_ab.log 2>&1
