"""Diagnostic: W / Y column errors of pass variants against fp64 (one block and more)."""
import ctypes as C
import sys

import torch

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
from libskylark_amd.ops import _lib
_lib.require()
_lib.register("sl_rsvd_pass", [vp, i64, i64, i64, vp, i32, vp, vp, i64, i32, i32, vp])
_lib.register("sl_rsvd_pass_workspace", [i64, i64, i32], C.c_int64)
_lib.register("sl_rsvd_reduce", [vp, i64, i64, i32, vp, i32, i32, vp, i32, vp])
dev = torch.device("cuda")
for (m, n, k) in [(16, 1000, 40), (16, 512, 20), (16, 520, 33), (4097, 1000, 40)]:
    g = torch.Generator(device=dev).manual_seed(1)
    A = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16)
    Zt = torch.randn(k, n, device=dev, generator=g).to(torch.bfloat16)
    ws = torch.zeros(int(_lib.require().sl_rsvd_pass_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    st = vp(torch.cuda.current_stream().cuda_stream)
    y = A.double() @ Zt.double().t()
    Wref = A.double().t() @ y
    mag = A.double().abs().t() @ y.abs()
    for final in (0, 2):
        for v in (0, 64, 128, 32):
            W = torch.empty(n, k, device=dev, dtype=torch.float64)
            Y = torch.full((m, k), float("nan"), device=dev)
            _lib.call("sl_rsvd_pass", vp(A.data_ptr()), m, n, n, vp(Zt.data_ptr()), k, vp(ws.data_ptr()),
                      vp(Y.data_ptr()) if final else None, k, final, v, st)
            _lib.call("sl_rsvd_reduce", vp(ws.data_ptr()), m, n, k, vp(W.data_ptr()), 1, k, None, k, st)
            torch.cuda.synchronize()
            err = ((W - Wref).abs() / mag)
            cols = err.max(0).values
            msg = f"m={m} n={n} k={k} final={final} v={v} Wmax={float(err.max()):.2e} Wbadcols={[i for i in range(k) if cols[i] > 1e-4]}"
            if final:
                ye = ((Y.double() - y).abs() / (A.double().abs() @ Zt.double().abs().t())).max(0).values
                msg += f" Ymax={float(ye.max()):.2e} Ybadcols={[i for i in range(k) if ye[i] > 1e-4]}"
            print(msg)
            sys.stdout.flush()
