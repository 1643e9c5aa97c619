#!/bin/bash
# config benches for the README table (one GPU): RFT features (NT GEMM), CSR dense sketch,
# FJLT sampled, ADMM, KRR, LSRN, CG KRR; each step time-limited, results appended to gpurun_out/configs.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/configs.jsonl
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > $OUT/cfg_$name.log 2>&1; local rc=$?;
        grep '^{' $OUT/cfg_$name.log | sed "s/^{/{\"bench_name\": \"$name\", /" | tee -a $OUT/configs.jsonl; return $rc; }
run features_f32 python benchmarks/bench_features.py --dtype f32 || exit 1
run features_bf16 python benchmarks/bench_features.py --dtype bf16 || exit 1
run csr_sketch python benchmarks/csr_sketch_bench.py || exit 1
run fjlt python benchmarks/bench_fjlt.py || exit 1
run admm python benchmarks/bench_admm.py || exit 1
run admm_bf16 python benchmarks/bench_admm.py --cache-dtype bf16 --iters 10 || exit 1
run krr python benchmarks/bench_krr.py || exit 1
run krr_cg python benchmarks/krr_cg.py || exit 1
run lsrn python benchmarks/bench_lsrn.py || exit 1
