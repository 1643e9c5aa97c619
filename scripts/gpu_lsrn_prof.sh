set -o pipefail
ROOT=$(pwd); mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/lsrn_prof -o run --output-format csv -- python3 $ROOT/benchmarks/bench_lsrn.py > $ROOT/gpurun_out/lsrn_prof.log 2>&1
