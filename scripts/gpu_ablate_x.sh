set -u
mkdir -p gpurun_out
for x in 3 5 7; do SL_TSK_X=$x timeout -k 10 200 python benchmarks/tsk_ablate.py > gpurun_out/ablate_x$x.jsonl 2>&1 || exit 1; done
