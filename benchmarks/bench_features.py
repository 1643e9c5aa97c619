"""Random-feature / dense-sketch throughput: fused MFMA GEMM + epilogue
(``feature_gemm.hip``) vs the unfused path (realised W + torch GEMM +
separate epilogue pass).  Default shape = BASELINE config 4's feature map:
Gaussian RFT of 1e6 x 512 synthetic data to 4096 features (rowwise, f32).

usage: python benchmarks/bench_features.py [--rows 1e6] [--dim 512] [--S 4096]
       [--sketch GaussianRFT|JLT|ExpSemigroupRLT] [--dtype f32|bf16] [--columnwise]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e6)
    ap.add_argument("--dim", type=int, default=512)
    ap.add_argument("--S", type=int, default=4096)
    ap.add_argument("--sketch", default="GaussianRFT")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--columnwise", action="store_true")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--modes", default="fused,unfused")
    a = ap.parse_args(argv)
    import libskylark_amd as sk
    dev = torch.device("cuda")
    m, d = int(a.rows), a.dim
    dt = torch.float32 if a.dtype == "f32" else torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(3)
    X = torch.rand(m, d, generator=g, device=dev, dtype=torch.float32).to(dt)
    if a.columnwise:
        X = X.t()                      # d x m view (examples as columns, reference layout)
    dim = 0 if a.columnwise else 1
    kw = {"sigma": 10.0} if "RFT" in a.sketch else ({"beta": 0.1} if "RLT" in a.sketch else {})
    T = getattr(sk.sketch, a.sketch)(d, a.S, context=sk.Context(1), **kw)
    res = {}
    for mode in a.modes.split(","):
        os.environ["SKH_FUSED_SKETCH"] = "1" if mode == "fused" else "0"
        for _ in range(a.warmup):
            Z = T.apply(X, dim=dim)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            Z = T.apply(X, dim=dim)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        res[mode] = {"ms": round(ms, 3), "features_per_s": round(m * a.S / (ms / 1e3), 1),
                     "tflops": round(2.0 * m * d * a.S / (ms / 1e3) / 1e12, 1)}
        res[mode + "_checksum"] = float(Z.double().abs().sum().item())
        del Z
        torch.cuda.empty_cache()
    out = {"metric": f"{a.sketch} feature map ms ({'columnwise' if a.columnwise else 'rowwise'})",
           "config": {"rows": m, "dim": d, "S": a.S, "dtype": a.dtype}, **res}
    if "fused" in res and "unfused" in res:
        out["speedup"] = round(res["unfused"]["ms"] / res["fused"]["ms"], 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
