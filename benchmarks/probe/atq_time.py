"""Median time of sl_ts_atq (W = A^T Q, f32 / f64 A, f64 W) by row length:
does the 128-B alignment of A's rows matter for this product too?"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from libskylark_amd.ops import _lib  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_ts_atq_workspace", [i64, i64, i32, i32], C.c_int64)
_lib.register("sl_ts_atq", [vp, i64, i64, i64, vp, i32, vp, i32, vp, i32, vp])
_lib.register("sl_ts_set_atq_bf16", [i32], None)
BS = int(os.environ.get("SL_ATQ_BF16", "1"))   # split form on / off (A/B)
_lib.require().sl_ts_set_atq_bf16(BS)
_lib.register("sl_ts_set_az_align", [i32], None)
ALIGN = int(os.environ.get("SL_AZ_ALIGN", "1"))   # alignment classes (shared knob with Y = A Z)
_lib.require().sl_ts_set_az_align(ALIGN)
dev = torch.device("cuda")
CASES = ((torch.float32, 1_000_000, 1000, 40), (torch.float32, 1_000_000, 1024, 40),
                    (torch.float32, 250_000, 4000, 40), (torch.float32, 1_000_000, 1000, 16),
                    (torch.float32, 1_000_000, 1024, 16), (torch.float64, 500_000, 1000, 16),
                    (torch.float64, 500_000, 1024, 16), (torch.float64, 200_000, 5000, 40))
if len(sys.argv) > 1 and sys.argv[1] == "one":   # one case (PMC passes)
    CASES = CASES[:1]
if len(sys.argv) > 1 and sys.argv[1] == "k128":   # 64 < k <= 128
    CASES = ((torch.float32, 1_000_000, 1000, 128), (torch.float32, 1_000_000, 1000, 96), (torch.float32, 250_000, 4000, 128))
if len(sys.argv) > 1 and sys.argv[1] == "k64":   # 48 < k <= 64
    CASES = ((torch.float32, 1_000_000, 1000, 64), (torch.float32, 1_000_000, 1000, 56), (torch.float32, 250_000, 4000, 64))
for dt, m, n, k in CASES:
    A = torch.randn(m, n, device=dev, dtype=dt)
    Q = torch.randn(m, k, device=dev, dtype=dt)
    code = 0 if dt == torch.float32 else 1
    ws = torch.empty(int(_lib.require().sl_ts_atq_workspace(m, n, k, code)), dtype=torch.uint8, device=dev)
    W = torch.empty(n, k, device=dev, dtype=torch.float64)
    st = vp(torch.cuda.current_stream().cuda_stream)
    ts = []
    for _ in range(9):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("sl_ts_atq", vp(A.data_ptr()), m, n, n, vp(Q.data_ptr()), k, vp(W.data_ptr()), k, vp(ws.data_ptr()),
                  code, st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[2:])
    us = 1e3 * ts[len(ts) // 2]
    print(json.dumps({"dtype": str(dt)[6:], "m": m, "n": n, "k": k, "split": BS, "align": ALIGN, "us": round(us, 1),
                      "TBps": round(A.numel() * A.element_size() / us / 1e6, 2)}), flush=True)
    del A, Q, ws
    torch.cuda.empty_cache()
