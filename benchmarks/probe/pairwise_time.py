"""Median time of the pairwise L1 / exp-semigroup kernel Gram (distance_kernels.hip
sl_pairwise_map) on 8192 x 8192 points of dimension 512, f32 (probe for
scripts/ab_lib_cmd.sh)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from libskylark_amd.ops import _lib  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_pairwise_map", [vp, vp, vp, i32, i64, i64, i64, i64, i64, i64, i32, C.c_double, vp])
dev = torch.device("cuda")
m = n = 8192
d = 512
X = torch.randn(m, d, device=dev)
Y = torch.randn(n, d, device=dev)
K = torch.empty(m, n, device=dev)
st = vp(torch.cuda.current_stream().cuda_stream)
for mode in (0, 1):
    ts = []
    for _ in range(8):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("sl_pairwise_map", vp(X.data_ptr()), vp(Y.data_ptr()), vp(K.data_ptr()), 0, m, n, d, d, d, n, mode,
                  0.0, st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[2:])
    ref = torch.cdist(X[:64].double(), Y[:64].double(), p=1) if mode == 0 else None
    err = float((K[:64, :64].double() - ref).abs().max() / ref.abs().max()) if ref is not None else None
    print(json.dumps({"mode": mode, "m": m, "n": n, "d": d, "ms": round(ts[len(ts) // 2], 3), "rel_err": err}),
          flush=True)
