#!/bin/bash
# A/B of an environment knob on the headline call: bench.py under
# rocprofv3 --kernel-trace for each value (interleaved rounds), then the
# median duration of the kernels whose name matches $PAT per run.
# usage: VAR=SL_XM_REV VALS="0 1" PAT=k_xm_pipe bash scripts/ab_env_prof.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$ROOT/gpurun_out/ab_env; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for r in 1 2; do
  for v in $VALS; do
    export $VAR=$v
    timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/${v}_$r -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $OUT/${v}_$r.log 2>&1 || exit 1
    python3 - "$OUT/${v}_$r" "$PAT" "$v" "$r" "$OUT/${v}_$r.log" <<'PY' | tee -a $OUT/summary.jsonl
import csv, glob, json, statistics, sys
d, pat, v, r, log = sys.argv[1:]
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
ts = [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in csv.DictReader(open(f)) if pat in x["Kernel_Name"]]
b = [json.loads(l) for l in open(log) if l.startswith("{\"metric\"")][0]
print(json.dumps({"var": v, "round": int(r), "kernel": pat, "n": len(ts), "median_us": round(statistics.median(ts) / 1e3, 2),
                  "min_us": round(min(ts) / 1e3, 2), "bench_ms": b["ms_per_step"], "ok": b["check"]["ok"]}))
PY
  done
done
