"""Median time of sl_ts_gram64 (f64 X^T X, k <= 64, matrix cores) on the f64
general engine's iterate (2e5 x 40) and a k = 64 case (probe for
scripts/ab_lib_cmd.sh)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from libskylark_amd.ops import _lib  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_ts_gram64", [vp, i64, i32, i64, vp, i32, vp, vp])
L = _lib.require()
L.sl_ts_gram64_workspace.argtypes = [i64, i32]
L.sl_ts_gram64_workspace.restype = i64
dev = torch.device("cuda")
for m, k in ((200_000, 40), (1_000_000, 64)):
    X = torch.randn(m, k, device=dev, dtype=torch.float64)
    G = torch.empty(k, k, device=dev, dtype=torch.float64)
    ws = torch.empty(L.sl_ts_gram64_workspace(m, k) // 8 + 1, device=dev, dtype=torch.float64)
    st = vp(torch.cuda.current_stream().cuda_stream)
    ts = []
    for _ in range(12):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("sl_ts_gram64", vp(X.data_ptr()), m, k, k, vp(G.data_ptr()), k, vp(ws.data_ptr()), st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[2:])
    ref = X.t() @ X
    print(json.dumps({"m": m, "k": k, "us": round(1e3 * ts[len(ts) // 2], 1),
                      "rel_err": float((G - ref).abs().max() / ref.abs().max())}), flush=True)
