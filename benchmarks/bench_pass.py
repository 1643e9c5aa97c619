"""Fused randSVD pass A/B on the headline shape (1e6 x 1000 bf16, k = 40):
sl_rsvd_pass variants (0 = forward walk, 256 = backward walk, 64/128 = y-wave
priority) for each form (final 0:
inter, 1: + Y + fp64 Gram, 2: + Y), timed with events, variants interleaved
so clock drift hits all of them alike.  One JSON line per (variant, form)."""
import argparse
import os
import sys
import ctypes as C
import json

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1_000_000)
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--k", type=int, default=40)
    ap.add_argument("--variants", default="0,256")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--finals", default="0,1,2")
    ap.add_argument("--prev", type=int, default=-1,
                    help="run an untimed forward inter pass right before each timed one "
                         "(MALL reuse A/B: variant 256 = reverse walk)")
    a = ap.parse_args()
    from libskylark_amd.ops import _lib
    _lib.require()
    _lib.register("sl_rsvd_pass", [vp, i64, i64, i64, vp, i32, vp, vp, i64, i32, i32, vp])
    _lib.register("sl_rsvd_pass_workspace", [i64, i64, i32], C.c_int64)
    m, n, k = a.m, a.n, a.k
    dev = torch.device("cuda")
    A = torch.randn(m, n, device=dev).to(torch.bfloat16)
    Zt = torch.linalg.qr(torch.randn(n, k, device=dev))[0].t().contiguous().to(torch.bfloat16)
    ws = torch.zeros(int(_lib.require().sl_rsvd_pass_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    Y = torch.empty(m, k, device=dev)
    st = vp(torch.cuda.current_stream().cuda_stream)
    variants = [int(v) for v in a.variants.split(",")]
    res = {}
    for rep in range(a.reps + 2):
        for final in [int(f) for f in a.finals.split(",")]:
            for v in variants:
                if a.prev >= 0:
                    _lib.call("sl_rsvd_pass", vp(A.data_ptr()), m, n, n, vp(Zt.data_ptr()), k, vp(ws.data_ptr()),
                              None, k, 0, a.prev, st)
                    torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.call("sl_rsvd_pass", vp(A.data_ptr()), m, n, n, vp(Zt.data_ptr()), k, vp(ws.data_ptr()),
                          vp(Y.data_ptr()) if final else None, k, final, v, st)
                e1.record()
                torch.cuda.synchronize()
                if rep >= 2:
                    res.setdefault((v, final), []).append(e0.elapsed_time(e1) * 1e3)
    for (v, final), ts in sorted(res.items()):
        ts.sort()
        med = ts[len(ts) // 2]
        print(json.dumps({"variant": v, "final": final, "us_median": round(med, 1), "us_min": round(ts[0], 1),
                          "TBps_median": round(m * n * 2 / med / 1e6, 2), "m": m, "n": n, "k": k, "prev": a.prev}))


if __name__ == "__main__":
    main()
