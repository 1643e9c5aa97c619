"""A/B of the fused tall-skinny pass: v1 (tsk_kernels.hip) vs the software-
pipelined v2 (tsk2_kernels.hip).  Checks v2 against v1 and an fp64 torch
reference first (ragged m, several n/k), then times both on the headline
shape (1e6 x 1000 bf16, k = 40) for the intermediate and final variants.

usage: python benchmarks/tsk_v2_bench.py [--reps 10] [--json out.jsonl]"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import _lib, rng, tallskinny as T  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64


def call(ver, A, Zt, k, W, G, Y, ws, flags):
    m, n = A.shape
    st = vp(torch.cuda.current_stream().cuda_stream)
    lib = _lib.require()
    if ver in (1, 11, 12, 13, 15, 17):
        lib.sl_tsk_set_x(0 if ver == 1 else ver - 10)
    if ver == 3:
        _lib.call("sl_tsk3_fused_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt), k, _lib.ptr(W),
                  _lib.ptr(G) if G is not None else None, _lib.ptr(Y) if Y is not None else None,
                  0 if Y is None else Y.stride(0), _lib.ptr(ws), ws.numel(), flags, st)
    elif ver in (1, 11, 12, 13, 15, 17):
        _lib.call("sl_tsk_fused_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt), k, _lib.ptr(W),
                  _lib.ptr(G) if G is not None else None, _lib.ptr(Y) if Y is not None else None,
                  0 if Y is None else Y.stride(0), _lib.ptr(ws), flags, st)
    else:
        _lib.call("sl_tsk2_fused_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt), k, _lib.ptr(W),
                  _lib.ptr(G) if G is not None else None, _lib.ptr(Y) if Y is not None else None,
                  0 if Y is None else Y.stride(0), _lib.ptr(ws), ws.numel(), flags, st)


def check(m, n, k, dev, out):
    A = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    rng.fill_random(A, D.Normal(), 7, 0, ir=n, ic=1)
    Z = torch.randn(n, k, device=dev, dtype=torch.float64) / n ** 0.5
    Zt = Z.t().to(torch.bfloat16).contiguous()
    Ad = A.double()
    Yr = Ad @ Zt.t().double()
    Wr = Ad.t() @ Yr
    Gr = Yr.t() @ Yr
    ws = torch.zeros(T.fused_workspace_bytes(m, n, k), dtype=torch.uint8, device=dev)
    res = {}
    for name, flags, keep_y, g64 in (("inter", 3, False, False), ("final_g64", 4, True, True),
                                     ("exact", 0, False, False), ("exact_y", 0, True, False)):
        for ver in (1, 11, 13, 15, 17):
            if ver == 3 and name in ("exact", "exact_y"):
                continue   # v3 forms every Gram in f64 (final_g64 covers it)
            W = torch.zeros(n, k, device=dev)
            G = torch.zeros(k, k, device=dev, dtype=torch.float64 if g64 else torch.float32)
            Y = torch.zeros(m, k, device=dev) if keep_y else None
            call(ver, A, Zt, k, W, G, Y, ws, flags)
            torch.cuda.synchronize()
            ew = float((W.double() - Wr).norm() / Wr.norm())
            eg = float((G.double() - Gr).norm() / Gr.norm()) if not (flags & 1) else 0.0
            ey = float((Y.double() - Yr).norm() / Yr.norm()) if Y is not None else 0.0
            res[(name, ver)] = (ew, eg, ey)
            rec = {"check": name, "ver": ver, "m": m, "n": n, "k": k, "errW": ew, "errG": eg, "errY": ey}
            out.append(rec)
            print(json.dumps(rec), flush=True)
    ok = True
    for (name, ver), e2 in res.items():
        tolw = 2e-2 if (name == "inter" and ver in (1, 2, 11, 12, 13, 15, 17)) else 1e-4
        if not (e2[0] < tolw and e2[1] < 1e-4 and e2[2] < 1e-5):
            ok = False
            print(f"MISMATCH {name} ver={ver} m={m} n={n} k={k}: {e2}", flush=True)
    return ok


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default=None)
    ap.add_argument("--skip-check", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    lib = _lib.require()
    lib.sl_tsk2_set_tuning.argtypes = [i32, i32]
    lib.sl_tsk_set_ablate.argtypes = [i32]
    lib.sl_tsk_set_x.argtypes = [i32]
    lib.sl_tsk3_set_tuning.argtypes = [i32]
    out = []
    ok = True
    if not a.skip_check:
        for (m, n, k) in ((100003, 1000, 40), (65536 + 7, 512, 16), (50001, 256, 32), (4099, 1000, 48), (10, 64, 8)):
            ok = check(m, n, k, dev, out) and ok
    m, n = 1_000_000, 1000
    A = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
    nbytes = m * n * 2
    for k in (40, 32):
        Zt = (torch.randn(k, n, device=dev) / 30).to(torch.bfloat16)
        ws = torch.empty(T.fused_workspace_bytes(m, n, k), dtype=torch.uint8, device=dev)
        W = torch.empty(n, k, device=dev)
        G = torch.empty(k, k, device=dev, dtype=torch.float64)
        Y = torch.empty(m, k, device=dev)
        for name, flags, Yc in (("inter", 3, None), ("final_g64", 4, Y)):
            vers = [(11, 0), (13, 0), (15, 0), (17, 0), (15, 64), (17, 64)]
            for ver, ab in vers:
                if ver in (1, 11, 12, 13, 15, 17):
                    lib.sl_tsk_set_ablate(ab)
                elif ver == 2:
                    lib.sl_tsk2_set_tuning(1, ab)
                else:
                    lib.sl_tsk3_set_tuning(ab)
                t = timeit(lambda: call(ver, A, Zt, k, W, G, Yc, ws, flags), a.reps)
                rec = {"case": name, "k": k, "ver": ver, "nt": bool(ab & 64), "us": round(t * 1e6, 1),
                       "GBps": round(nbytes / t / 1e9, 1)}
                out.append(rec)
                print(json.dumps(rec), flush=True)
        lib.sl_tsk3_set_tuning(0)
    lib.sl_tsk_set_ablate(0)
    lib.sl_tsk_set_x(0)
    lib.sl_tsk2_set_tuning(2, 0)
    if a.json:
        with open(a.json, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")
    print("ALL_OK" if ok else "CHECK_FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
