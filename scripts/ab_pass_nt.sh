#!/bin/bash
# A/B of the fused pass's LDS-DMA cache policy (SL_PASS_NT codes, rsvd_pass.hip
# P5Tiles::nt): the pass kernel alone (bench_pass.py, forward / reverse walks,
# nt variants) and the whole headline call (bench.py), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 python benchmarks/bench_pass.py --variants 0,512,256,768 --finals 0,1 --reps 15 > $OUT/ab_pass_nt_kernel.jsonl 2>&1 || exit 1
cat $OUT/ab_pass_nt_kernel.jsonl
for r in 1 2; do
  for c in ${CODES:-0 1 3 5}; do
    SL_PASS_NT=$c timeout -k 10 200 python bench.py --steps 40 --warmup 10 > $OUT/ab_nt_$c.log 2>&1 || exit 1
    python - "$c" "$r" $OUT/ab_nt_$c.log <<'PY' | tee -a $OUT/ab_pass_nt_bench.jsonl
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().split("\n")[-1])
print(json.dumps({"nt_code": int(sys.argv[1]), "round": int(sys.argv[2]), "ms_per_step": d["ms_per_step"],
                  "median": d["step_ms"]["median"], "min": d["step_ms"]["min"], "ok": d["check"]["ok"]}))
PY
  done
done
