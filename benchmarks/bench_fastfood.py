"""Fastfood (FastGaussianRFT) features for large N, rowwise, timed three ways
("Fastfood at N = 8192, S = 16384 timed against its
dense-W path"):
  fused     fastfood.hip: one launch per call, (row, block) workgroups, both
            DCTs + Pi + G + Sm + cosine in LDS
  pipeline  the previous GPU path: per block two rocFFT pipelines (pre pass,
            R2C, post gather) + torch scale + concat, then the epilogue pass
  denseW    the realised S x N operator through the fused MFMA feature GEMM
            (gemm_nt.hip, f32-exact 3-term bf16 split, cosine epilogue)
Synthetic Gaussian rows; one JSON line per (path, m)."""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=8192)
    ap.add_argument("--S", type=int, default=16384)
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--paths", default="fused,pipeline,denseW")
    a = ap.parse_args()
    import libskylark_amd as sk
    from libskylark_amd.ops import fused as F
    from libskylark_amd.sketch import ROWWISE
    dev = torch.device("cuda")
    X = torch.randn(a.m, a.N, device=dev) / math.sqrt(a.N)
    T = sk.sketch.FastGaussianRFT(a.N, a.S, sigma=3.0, context=sk.Context(7))
    out = {}
    for p in a.paths.split(","):
        if p == "fused":
            fn = lambda: T._fused_apply(X, None, epi=True)  # noqa: E731
        elif p == "apply":
            fn = lambda: T.apply(X, dim=ROWWISE)  # noqa: E731   (what the library picks)
        elif p == "pipeline":
            fn = lambda: T._post(T._features_pre_gpu(X, ROWWISE), ROWWISE)  # noqa: E731
        else:
            T.DENSE_MAX_N = a.N   # instance knob: allow realising W at this N
            W = F.SplitW(T.realize_W(torch.float64, dev).float())
            fn = lambda: F.feature_gemm(X, W, ROWWISE, shifts=T.shifts.to(dev), outscale=T.outscale,  # noqa: E731
                                        epi=F.EPI_COS)
        ms = timed(fn, a.reps)
        out[p] = fn().float()
        rec = {"path": p, "N": a.N, "S": a.S, "m": a.m, "ms": round(ms, 3),
               "rows_per_s": round(a.m / (ms * 1e-3), 1)}
        if p != "fused" and "fused" in out:
            rec["max_abs_diff_vs_fused"] = float((out[p] - out["fused"]).abs().max())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
