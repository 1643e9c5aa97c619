"""Median time of the U = Y M pass (k_xm_pipe: Y m x k f32 contiguous, M k x k2)
on the headline's shape (1e6 x 40 -> 1e6 x 20) and a k2 = 40 case; the grid
cap comes from SL_XM_PIPE_GRID (read once per process)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from libskylark_amd.ops import _lib, tallskinny  # noqa: E402,F401

vp = C.c_void_p
dev = torch.device("cuda")
for m, k, k2 in ((1_000_000, 40, 20), (1_000_000, 40, 40)):
    Y = torch.randn(m, k, device=dev)
    M = torch.randn(k, k2, device=dev)
    U = torch.empty(m, k2, device=dev)
    st = vp(torch.cuda.current_stream().cuda_stream)
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("sl_tsk_f32_xm", vp(Y.data_ptr()), m, k, k, vp(M.data_ptr()), k2, vp(U.data_ptr()), k2,
                  None, None, st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[3:])
    err = float((U - Y @ M).abs().max())
    print(json.dumps({"grid_cap": os.environ.get("SL_XM_PIPE_GRID", "2048"), "m": m, "k": k, "k2": k2,
                      "us": round(1e3 * ts[len(ts) // 2], 1), "max_err": err}), flush=True)
