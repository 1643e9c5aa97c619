set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "rng or random or sketch or jlt or fjlt or rft or uniform or normal" > gpurun_out/t_rng.log 2>&1 || exit 1
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/lsrn_prof2 -o run --output-format csv -- python3 $ROOT/benchmarks/bench_lsrn.py > $ROOT/gpurun_out/lsrn_rng.log 2>&1
