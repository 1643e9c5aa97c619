set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ts_products.py tests/test_gpu_rsvd_general.py > gpurun_out/t_gen.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/rsvd_general_bench.py --cases f64k128,f32k128 --reps 5 > gpurun_out/gen_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gen128e -- python3 $GRAFT_REPO_ROOT/benchmarks/rsvd_general_bench.py --cases f64k128,f32k128 --reps 3 --no-ref > $GRAFT_REPO_ROOT/gpurun_out/gen_prof.log 2>&1
