"""Median time of sl_ts_gram_w (G = X^T X, 64 < k <= 128, f64 products) on
the general engine's shapes: f32 1e6 x 128 and f64 2e5 x 128 (probe for the
library A/B in scripts/ab_lib_cmd.sh)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from libskylark_amd.ops import _lib  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_ts_gram_w", [vp, i32, i64, i32, i64, vp, i32, vp, vp])
L = _lib.require()
L.sl_ts_gram64_workspace.argtypes = [i64, i32]
L.sl_ts_gram64_workspace.restype = i64
dev = torch.device("cuda")
for dt, code, m in ((torch.float32, 0, 1_000_000), (torch.float64, 1, 200_000)):
    k = 128
    X = torch.randn(m, k, device=dev, dtype=dt)
    G = torch.empty(k, k, device=dev, dtype=torch.float64)
    ws = torch.empty(L.sl_ts_gram64_workspace(m, k) // 8 + 1, device=dev, dtype=torch.float64)
    st = vp(torch.cuda.current_stream().cuda_stream)
    ts = []
    for _ in range(12):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("sl_ts_gram_w", vp(X.data_ptr()), code, m, k, k, vp(G.data_ptr()), k, vp(ws.data_ptr()), st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[2:])
    ref = X.double().t() @ X.double()
    err = float((G - ref).abs().max() / ref.abs().max())
    print(json.dumps({"dtype": str(dt).split(".")[-1], "m": m, "k": k, "ms": round(ts[len(ts) // 2], 4),
                      "ms_min": round(ts[0], 4), "rel_err": err}), flush=True)
