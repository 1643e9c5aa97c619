"""General-precision device randSVD engine (rsvd_general.hip) at the
reference's precisions and sizes: 1e6 x 1000 f32 and
2e5 x 5000 f64, plus k = 128 -- the whole call on the device (rocBLAS passes,
one-wave small algebra, f64 core; hand-written f32 / f64 products for
k <= 64), timed with HIP events over
repeated cold calls (a fresh sketch seed per call).  Prints one JSON line per
case: ms per call, effective HBM traffic of the passes (2 (q + 1) reads of A),
and the relative error of the leading singular values against a reference
(the singular values of A from its f64 Gram; the planted values are reported
too).

Reference: nla/svd.hpp:222-318 (ApproximateSVD), :71-149 (power iteration)."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import libskylark_amd as sk  # noqa: E402
from libskylark_amd.nla import svd as S  # noqa: E402


def planted(m, n, r, dtype, dev, seed=0):
    """A = U diag(s) V^T + tiny noise, built on the device panel by panel."""
    g = torch.Generator(device=dev).manual_seed(seed)
    U, _ = torch.linalg.qr(torch.randn(m, r, device=dev, dtype=torch.float64, generator=g))
    V, _ = torch.linalg.qr(torch.randn(n, r, device=dev, dtype=torch.float64, generator=g))
    s = 100.0 * 0.85 ** torch.arange(r, device=dev, dtype=torch.float64)
    A = torch.empty(m, n, device=dev, dtype=dtype)
    step = max(1, (1 << 27) // n)
    for i in range(0, m, step):
        blk = (U[i:i + step] * s) @ V.t()
        blk += 1e-6 * torch.randn(blk.shape, device=dev, dtype=torch.float64, generator=g)
        A[i:i + step] = blk.to(dtype)
    return A, s


BIG = 1
SPLIT = 1
AZB = None
AZA = None
NO_REF = False   # --no-ref: skip the f64 reference (kernel traces of the engine alone)


def run(m, n, rank, q, dtype, sketch="FJLT", reps=5):
    dev = torch.device("cuda")
    A, s_true = planted(m, n, max(2 * rank, 32), dtype, dev)
    prm = sk.nla.ApproximateSVDParams(num_iterations=q, sketch=sketch)
    ctx = sk.Context(seed=11)
    U, s, V = sk.nla.approximate_svd(A, rank, ctx, prm)       # plan + first call
    torch.cuda.synchronize()
    plan = [p for p in S._PLANS.values() if p.Aref() is A][0]
    times = []
    for i in range(reps):
        ctx = sk.Context(seed=1000 + i)                         # cold: a new sketch every call
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        U, s, V = sk.nla.approximate_svd(A, rank, ctx, prm)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    times.sort()
    ms = times[len(times) // 2]
    es = A.element_size()
    bytes_passes = 2 * (q + 1) * m * n * es
    # reference: the singular values of A itself (planted + noise), from the
    # f64 Gram A^T A summed over row chunks (the planted s alone is off by the
    # noise for the trailing wanted values)
    if NO_REF:
        print(json.dumps({"case": f"{m}x{n} {str(dtype).split('.')[-1]} rank {rank} q {q} {sketch}",
                          "engine": type(plan).__name__, "native": getattr(plan, "native", None),
                          "ms": round(ms, 3), "ms_min": round(times[0], 3),
                          "pass_traffic_GBps": round(bytes_passes / (ms * 1e-3) / 1e9, 1)}), flush=True)
        del A, U, V
        S._PLANS.clear()
        torch.cuda.empty_cache()
        return
    G = torch.zeros(n, n, device=A.device, dtype=torch.float64)
    step = max(1, (1 << 26) // n)
    for i in range(0, m, step):
        Ac = A[i:i + step].double()
        G += Ac.t() @ Ac
    s_ref = torch.linalg.eigvalsh(G).flip(0)[:rank].clamp_min(0).sqrt()
    del G
    err = float(((s.double() - s_ref).abs() / s_ref).max())
    err_planted = float(((s.double() - s_true[:rank]).abs() / s_true[:rank]).max())
    k = max(rank, min(n, 2 * rank))
    out = {"case": f"{m}x{n} {str(dtype).split('.')[-1]} rank {rank} (k {k}) q {q} {sketch}", "big": BIG, "bf16_split": SPLIT, "az_bf16": AZB, "az_align": AZA,
           "engine": type(plan).__name__, "native": getattr(plan, "native", None), "ms": round(ms, 3), "ms_min": round(times[0], 3),
           "pass_traffic_GBps": round(bytes_passes / (ms * 1e-3) / 1e9, 1), "max_rel_err_s": err,
           "max_rel_err_s_vs_planted": err_planted}
    print(json.dumps(out), flush=True)
    del A, U, V
    S._PLANS.clear()
    torch.cuda.empty_cache()


CASES = {
    "f32": lambda reps: run(1_000_000, 1000, 20, 2, torch.float32, reps=reps),
    "f64": lambda reps: run(200_000, 5000, 20, 2, torch.float64, reps=reps),
    "f64k128": lambda reps: run(200_000, 5000, 64, 1, torch.float64, reps=reps),   # k = 128
    "f32k128": lambda reps: run(1_000_000, 1000, 64, 1, torch.float32, reps=reps),
    "bf16": lambda reps: run(1_000_000, 1000, 20, 2, torch.bfloat16, reps=reps),  # the fused engine, for comparison
    "bf16w": lambda reps: run(500_000, 4000, 20, 2, torch.bfloat16, reps=reps),   # n > 1024: the general engine
}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="f32,f64,f64k128,bf16")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--big", type=int, default=1, help="0: rocBLAS products past k = 64 (A/B)")
    ap.add_argument("--bf16-split", type=int, default=1, help="0: bf16 A^T [Q_hi Q_lo] as one product (A/B)")
    ap.add_argument("--az-align", type=int, default=None, help="Y = A Z row-alignment classes on (1) / off (0)")
    ap.add_argument("--az-bf16", type=int, default=None, help="f32 Y = A Z on the exact bf16 split (1) or f32 MFMA (0)")
    a = ap.parse_args()
    import ctypes
    from libskylark_amd.ops import _lib
    _lib.require().sl_rsvd_gen_set_big.argtypes = [ctypes.c_int]
    _lib.require().sl_rsvd_gen_set_big(a.big)
    _lib.require().sl_rsvd_gen_set_bf16_split.argtypes = [ctypes.c_int]
    _lib.require().sl_rsvd_gen_set_bf16_split(a.bf16_split)
    if a.az_align is not None:
        _lib.require().sl_ts_set_az_align.argtypes = [ctypes.c_int]
        _lib.require().sl_ts_set_az_align(a.az_align)
    if a.az_bf16 is not None:
        _lib.require().sl_ts_set_az_bf16.argtypes = [ctypes.c_int]
        _lib.require().sl_ts_set_az_bf16(a.az_bf16)
    global NO_REF, BIG, SPLIT, AZB, AZA
    AZB = a.az_bf16
    AZA = a.az_align
    NO_REF = a.no_ref
    BIG = a.big
    SPLIT = a.bf16_split
    for c in a.cases.split(","):
        CASES[c](a.reps)


if __name__ == "__main__":
    main()
