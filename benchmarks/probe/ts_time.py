"""Median times of the general engine's two products (rsvd_stream.hip
sl_ts_az / sl_ts_atq) on the bench shapes: f32 1e6 x 1000 and f64 2e5 x 5000
at k = 40 and k = 128 (10 launches each); one JSON line per case."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from libskylark_amd.ops import _lib  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
L = _lib.require()
_lib.register("sl_ts_az", [vp, i64, i64, i64, vp, i32, vp, i64, i32, vp])
_lib.register("sl_ts_atq_workspace", [i64, i64, i32, i32], C.c_int64)
_lib.register("sl_ts_atq", [vp, i64, i64, i64, vp, i32, vp, i32, vp, i32, vp])
dev = torch.device("cuda")
st = vp(torch.cuda.current_stream().cuda_stream)


def med(f, reps=10):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


for m, n, dt, code in ((1_000_000, 1000, torch.float32, 0), (200_000, 5000, torch.float64, 1)):
    A = torch.randn(m, n, device=dev, dtype=dt)
    for k in (40, 128):
        Z = torch.randn(n, k, device=dev, dtype=dt)
        Y = torch.empty(m, k, device=dev, dtype=dt)
        W = torch.empty(n, k, device=dev, dtype=torch.float64)
        ws = torch.empty(int(L.sl_ts_atq_workspace(m, n, k, code)), dtype=torch.uint8, device=dev)
        az = med(lambda: _lib.call("sl_ts_az", _lib.ptr(A), m, n, n, _lib.ptr(Z), k, _lib.ptr(Y), k, code, st))
        atq = med(lambda: _lib.call("sl_ts_atq", _lib.ptr(A), m, n, n, _lib.ptr(Y), k, _lib.ptr(W), k, _lib.ptr(ws),
                                    code, st))
        ref = (A[:4096].double() @ Z.double())
        err = float((Y[:4096].double() - ref).abs().max() / ref.abs().max())
        print(json.dumps({"dtype": str(dt).split(".")[-1], "m": m, "n": n, "k": k, "az_ms": round(az, 4),
                          "atq_ms": round(atq, 4), "az_rel_err": err}), flush=True)
    del A
    torch.cuda.empty_cache()
