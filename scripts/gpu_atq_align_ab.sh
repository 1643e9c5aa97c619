set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/atqa_ab.log
for a in 0 1 0 1; do
  SL_AZ_ALIGN=$a timeout -k 10 200 python benchmarks/probe/atq_time.py >> gpurun_out/atqa_ab.log 2>&1 || exit 1
done
