set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ts_products.py tests/test_gpu_rsvd_general.py > gpurun_out/t_atqb.log 2>&1 || exit 1
: > gpurun_out/atqb_ab.log
for b in 0 1; do
  SL_ATQ_BF16=$b timeout -k 10 200 python benchmarks/probe/atq_time.py >> gpurun_out/atqb_ab.log 2>&1 || exit 1
done
timeout -k 10 300 python benchmarks/rsvd_general_bench.py --cases f32 --reps 7 >> gpurun_out/atqb_ab.log 2>&1
