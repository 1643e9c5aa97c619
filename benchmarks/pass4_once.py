"""Run the v4 fused randSVD pass (rsvd_pass.hip) + its slab reduce N times on
the headline shape, for rocprofv3 --pmc counter runs.
usage: pass4_once.py [final=0|2] [reps=10]
(final 0: the inter-pass form; final 2: the last pass, Y stored, its fp64
Gram a separate kernel afterwards -- what the engine runs)"""
from __future__ import annotations

import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import _lib, rng  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_rsvd_pass", [vp, i64, i64, i64, vp, i32, vp, vp, i64, i32, i32, vp])
_lib.register("sl_rsvd_pass_workspace", [i64, i64, i32], C.c_int64)
_lib.register("sl_rsvd_reduce", [vp, i64, i64, i32, vp, i32, i32, vp, i32, vp])


def main():
    final = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    m, n, k = 1_000_000, 1000, 40
    dev = torch.device("cuda")
    lib = _lib.require()
    A = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
    Q, _ = torch.linalg.qr(torch.randn(n, k, device=dev, dtype=torch.float64))
    Zt = Q.t().contiguous().to(torch.bfloat16)
    KP = ((k + 15) // 16) * 16
    ws = torch.empty(int(lib.sl_rsvd_pass_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    W = torch.empty(n, k, device=dev, dtype=torch.float64)
    Y = torch.empty(m, KP, device=dev)
    st = vp(torch.cuda.current_stream().cuda_stream)
    for _ in range(reps):
        _lib.call("sl_rsvd_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt), k, _lib.ptr(ws),
                  _lib.ptr(Y) if final else None, KP, final, 0, st)
        _lib.call("sl_rsvd_reduce", _lib.ptr(ws), m, n, k, _lib.ptr(W), 1, k, None, k, st)
    torch.cuda.synchronize()
    print("ok", final, reps)


if __name__ == "__main__":
    main()
