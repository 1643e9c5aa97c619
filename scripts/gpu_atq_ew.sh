set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ts_products.py > gpurun_out/t_atqew.log 2>&1 || exit 1
bash scripts/ab_lib_cmd.sh python benchmarks/probe/atq_time.py k64 > gpurun_out/atqew_ab.log 2>&1
