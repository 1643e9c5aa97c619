set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/azb_prof_$v -o run --output-format csv -- python3 $R/benchmarks/rsvd_general_bench.py --cases f32 --reps 3 --no-ref --az-bf16 $v > $R/gpurun_out/azb_prof_$v.log 2>&1 || exit 1
done
