set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bf16x2" > gpurun_out/t_lsrn.log 2>&1 || exit 1
: > gpurun_out/lsrn_overlap_ab.log
for r in 1 2; do for v in 0 1; do
  SL_LSRN_OVERLAP=$v timeout -k 10 200 python -u benchmarks/bench_lsrn.py > gpurun_out/lsrn_o.log 2>&1 || exit 1
  echo "{\"overlap\": $v, \"round\": $r, \"line\": $(grep '^{' gpurun_out/lsrn_o.log | tail -1)}" >> gpurun_out/lsrn_overlap_ab.log
done; done
