set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "kernel or gram or laplac or semigroup or pairwise" > gpurun_out/t_pw.log 2>&1 || exit 1
bash scripts/ab_lib_cmd.sh python benchmarks/probe/pairwise_time.py > gpurun_out/pw_ab.log 2>&1
