"""Median time of sl_ts_az (Y = A Z, f32 / f64) on 1e6 x 1000 f32 (and 2e5 x
5000 f64) for several k: separates the memory stream from the per-column-tile
work (probe for the general engine's products)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from libskylark_amd.ops import _lib  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_ts_az", [vp, i64, i64, i64, vp, i32, vp, i64, i32, vp])
_lib.register("sl_ts_set_az_bf16", [i32], None)
_lib.register("sl_ts_set_az_align", [i32], None)
ALIGN = int(os.environ.get("SL_AZ_ALIGN", "1"))   # row-alignment classes on / off (A/B)
_lib.require().sl_ts_set_az_align(ALIGN)
dev = torch.device("cuda")
cases = [(torch.float32, 1_000_000, 1000), (torch.float64, 200_000, 5000)]
KS = (8, 16, 32, 40, 48, 64)
if len(sys.argv) > 1 and sys.argv[1] == "shapes":   # row-length sweep at one k
    cases = [(torch.float32, 1_000_000, 1000), (torch.float32, 1_000_000, 1024), (torch.float32, 250_000, 4000),
             (torch.float32, 125_000, 8000), (torch.float64, 500_000, 1000), (torch.float64, 125_000, 4000)]
    KS = (16,)
for dt, m, n in cases:
    A = torch.randn(m, n, device=dev, dtype=dt)
    for k in KS:
        for bs in ((1, 0) if dt == torch.float32 and k <= 48 else (1,)):
            _lib.require().sl_ts_set_az_bf16(bs)
            Z = torch.randn(n, k, device=dev, dtype=dt)
            Y = torch.empty(m, k, device=dev, dtype=dt)
            st = vp(torch.cuda.current_stream().cuda_stream)
            ts = []
            for _ in range(9):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.call("sl_ts_az", vp(A.data_ptr()), m, n, n, vp(Z.data_ptr()), k, vp(Y.data_ptr()), k,
                          0 if dt == torch.float32 else 1, st)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts = sorted(ts[2:])
            us = 1e3 * ts[len(ts) // 2]
            print(json.dumps({"dtype": str(dt)[6:], "m": m, "n": n, "k": k, "split": bs, "align": ALIGN, "us": round(us, 1),
                              "TBps": round(A.numel() * A.element_size() / us / 1e6, 2)}), flush=True)
    _lib.require().sl_ts_set_az_bf16(1)
    del A
    torch.cuda.empty_cache()
