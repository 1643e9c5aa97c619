set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "rng or random or sketch or jlt or fjlt or rft" > gpurun_out/t_rng.log 2>&1 || exit 1
timeout -k 10 200 python -u benchmarks/bench_lsrn.py > gpurun_out/lsrn_rng.log 2>&1
