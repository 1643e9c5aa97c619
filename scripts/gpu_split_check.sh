set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_ml.py tests/test_gpu_gemm_nt.py -k "bf16x2 or split or krr or gemm" > gpurun_out/t_split.log 2>&1 || exit 1
ROOT=$(pwd)
timeout -k 10 200 python -u benchmarks/bench_krr.py > gpurun_out/krr_split.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/lsrn_prof3 -o run --output-format csv -- python3 $ROOT/benchmarks/bench_lsrn.py > $ROOT/gpurun_out/lsrn_split.log 2>&1
