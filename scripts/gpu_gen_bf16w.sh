set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rsvd_general.py > gpurun_out/t_gen3.log 2>&1 && \
for r in 1 2; do for v in 1 0; do timeout -k 10 200 python -u benchmarks/rsvd_general_bench.py --cases bf16w --reps 7 --bf16-split $v || exit 1; done; done > gpurun_out/gen_bf16_split_ab.log 2>&1
