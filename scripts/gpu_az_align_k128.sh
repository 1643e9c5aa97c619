set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/aza_k128.log
for a in 0 1 0 1; do
  timeout -k 10 300 python benchmarks/rsvd_general_bench.py --cases f32k128,f64k128,f64 --reps 5 --no-ref --az-align $a >> gpurun_out/aza_k128.log 2>&1 || exit 1
done
