"""A/B of the Y = A Z product's prefetch depth (rsvd_stream.hip k_ts_az:
2 A groups in flight per wave with two workgroups per CU, or 4 with one):
f32 1e6 x 1000 and f64 2e5 x 5000 at k = 40, interleaved, plus the max
relative difference of the two results.  (The PD = 4 variant and its
sl_ts_set_az_pd knob were removed after this A/B found no difference:
profiles/r6/az_prefetch_depth_ab.jsonl.)"""
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
L.sl_ts_set_az_pd.argtypes = [i32]
dev = torch.device("cuda")
st = vp(torch.cuda.current_stream().cuda_stream)
for m, n, dt, code in ((1_000_000, 1000, torch.float32, 0), (200_000, 5000, torch.float64, 1)):
    k = 40
    A = torch.randn(m, n, device=dev, dtype=dt)
    Z = torch.randn(n, k, device=dev, dtype=dt)
    Ys = {}
    for rnd in range(3):
        for pd in (2, 4):
            L.sl_ts_set_az_pd(pd)
            Y = torch.empty(m, k, device=dev, dtype=dt)
            f = lambda: _lib.call("sl_ts_az", _lib.ptr(A), m, n, n, _lib.ptr(Z), k, _lib.ptr(Y), k, code, st)  # noqa: E731
            f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            Ys[pd] = Y
            print(json.dumps({"dtype": str(dt).split(".")[-1], "m": m, "n": n, "k": k, "pd": pd, "round": rnd,
                              "ms": round(e0.elapsed_time(e1) / 10, 4)}), flush=True)
    d = float(((Ys[2] - Ys[4]).abs().max() / Ys[2].abs().max()))
    print(json.dumps({"dtype": str(dt).split(".")[-1], "max_rel_diff_pd2_pd4": d}), flush=True)
    del A, Z, Ys
    torch.cuda.empty_cache()
L.sl_ts_set_az_pd(2)
