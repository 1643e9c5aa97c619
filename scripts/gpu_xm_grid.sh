set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/xm_grid.log
for g in 2048 1280 2560 1024 3840 7813 2048; do
  SL_XM_PIPE_GRID=$g timeout -k 10 120 python benchmarks/probe/xm_pipe_time.py >> gpurun_out/xm_grid.log 2>&1 || exit 1
done
for g in 2048 1280 2048 1280; do
  SL_XM_PIPE_GRID=$g timeout -k 10 200 python bench.py > gpurun_out/xm_bench_$g.log 2>&1 || exit 1
  echo "grid $g $(grep '^{' gpurun_out/xm_bench_$g.log)" >> gpurun_out/xm_grid.log
done
