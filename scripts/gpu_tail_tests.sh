set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "svd or tsk or fused or fjlt or small or rfut or bench or smoke" > gpurun_out/pt_tail.log 2>&1; rc=$?; tail -5 gpurun_out/pt_tail.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_tail.sh
