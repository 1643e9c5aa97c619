"""Three launches each of the general engine's two products (rsvd_stream.hip
sl_ts_az / sl_ts_atq) on 1e6 x 1000 f32 (or --f64: 2e5 x 5000), k = 40: a
short target for rocprofv3 --pmc counter passes."""
import ctypes as C
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
f64 = "--f64" in sys.argv
m, n, dt, code = (200_000, 5000, torch.float64, 1) if f64 else (1_000_000, 1000, torch.float32, 0)
k = 40
dev = torch.device("cuda")
st = vp(torch.cuda.current_stream().cuda_stream)
A = torch.randn(m, n, device=dev, dtype=dt)
Z = torch.randn(n, k, device=dev, dtype=dt)
Y = torch.empty(m, k, device=dev, dtype=dt)
W = torch.empty(n, k, device=dev, dtype=torch.float64)
ws = torch.empty(int(L.sl_ts_atq_workspace(m, n, k, code)), dtype=torch.uint8, device=dev)
for _ in range(3):
    _lib.call("sl_ts_az", _lib.ptr(A), m, n, n, _lib.ptr(Z), k, _lib.ptr(Y), k, code, st)
    _lib.call("sl_ts_atq", _lib.ptr(A), m, n, n, _lib.ptr(Y), k, _lib.ptr(W), k, _lib.ptr(ws), code, st)
torch.cuda.synchronize()
print("ok")
