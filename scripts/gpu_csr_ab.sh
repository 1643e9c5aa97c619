set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu -k "csr" > gpurun_out/t_csr.log 2>&1 || exit 1
bash scripts/ab_lib_cmd.sh python benchmarks/csr_sketch_bench.py > gpurun_out/csr_ab.log 2>&1
