set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/ > gpurun_out/t_all_aza.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/rsvd_general_bench.py --cases f32,f64,f32k128,f64k128,bf16w --reps 7 > gpurun_out/aza_gen.log 2>&1 || exit 1
timeout -k 10 200 python bench.py > gpurun_out/aza_bench.log 2>&1
