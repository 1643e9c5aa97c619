set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_capi_dist.py tests/test_capi.py tests/test_gpu_native_comm.py > gpurun_out/t_capi_dist.log 2>&1
