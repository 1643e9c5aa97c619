"""Cholesky inverse (sl_wave_la.hpp): variant 0 = one wave, 1 = the rows of
the elimination over 4 waves (default), us per call (200 back-to-back launches, so the
~1.5 us launch boundary is included) and the max error of R^-T G R^-1 - I."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from libskylark_amd.ops import _lib  # noqa: E402

vp = C.c_void_p
_lib.require()
_lib.register("sl_chol_inv_wave", [vp, C.c_int, C.c_int, vp, vp, vp])
_lib.require().sl_chol_inv_set_variant.argtypes = [C.c_int]
dev = torch.device("cuda:0")
for k in (40, 48, 32, 64):
    g = torch.Generator().manual_seed(1)
    X = torch.randn(2000, k, generator=g, dtype=torch.float64) * torch.logspace(0, -3, k, dtype=torch.float64)
    G = (X.t() @ X).to(dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    R = torch.empty(k, k, dtype=torch.float64, device=dev)
    s = vp(torch.cuda.current_stream().cuda_stream)
    for v in (0, 1, 2, 3, 4, 5):
        _lib.require().sl_chol_inv_set_variant(v)
        f = lambda: _lib.call("sl_chol_inv_wave", _lib.ptr(G), k, k, _lib.ptr(R), _lib.ptr(st), s)  # noqa: E731
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            f()
        e1.record()
        torch.cuda.synchronize()
        err = float((R.t() @ G @ R - torch.eye(k, dtype=torch.float64, device=dev)).abs().max())
        print(json.dumps({"k": k, "variant": ["one_wave", "rows_over_4_waves", "pairs_4_waves", "pairs_8_waves", "quads_4_waves", "quads_8_waves"][v], "us": round(e0.elapsed_time(e1) * 1e3 / 200, 2),
                          "orth_err": err, "status": int(st.item())}))
