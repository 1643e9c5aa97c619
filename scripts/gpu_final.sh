#!/bin/bash
# Round-closing GPU run: full suite, smoke, bench (+ kernel trace), config
# benches, general-engine cases; every step time-limited, stops on failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
PROFILE=1 bash scripts/gpu_full.sh || exit 1
bash scripts/gpu_configs.sh > $OUT/final_configs.log 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/rsvd_general_bench.py --cases f32,f64,f32k128,f64k128,bf16w --reps 5 > $OUT/final_general.log 2>&1 || exit 1
echo final ok
