set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ts_products.py -k "gram" > gpurun_out/t_gram.log 2>&1 || exit 1
bash scripts/ab_lib_cmd.sh python benchmarks/probe/gram_w_time.py > gpurun_out/gram_w_ab.log 2>&1
