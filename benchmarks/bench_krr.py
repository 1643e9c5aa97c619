"""BASELINE config 4 (KRR half): Gaussian random Fourier features + kernel
ridge regression on 1e6 x 512 synthetic examples per GPU
(``ml.approximate_kernel_ridge``: fused MFMA feature map, fp64 normal
equations [Z^T Z | Z^T Y] -- one RCCL all-reduce across ranks -- and a
Cholesky solve).  One warm-up solve, then the timed one; phases via
SKH_PROFILE-style synchronised timers.

usage: python benchmarks/bench_krr.py [--rows 1e6] [--dim 512] [--features 4096]
       torchrun --nproc-per-node N --master-addr 127.0.0.1 benchmarks/bench_krr.py
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
    ap.add_argument("--features", type=int, default=4096)
    ap.add_argument("--lam", type=float, default=1e-2)
    ap.add_argument("--compare-f64", type=int, default=1,
                    help="also solve with the all-fp64 Gram (SKH_KRR_F64_GRAM=1) and report the weight difference")
    a = ap.parse_args(argv)
    import libskylark_amd as sk
    from libskylark_amd import ml
    from libskylark_amd.parallel import DistMatrix, init_distributed
    comm = init_distributed()
    dev = torch.device("cuda", torch.cuda.current_device())
    m, d = int(a.rows), a.dim
    g = torch.Generator(device=dev).manual_seed(1 + comm.rank)
    X = torch.randn(m, d, generator=g, device=dev)
    w = torch.randn(d, 1, generator=torch.Generator(device=dev).manual_seed(7), device=dev) / d ** 0.5
    Y = torch.sin(X @ w) + 0.01 * torch.randn(m, 1, generator=g, device=dev)
    k = ml.Gaussian(d, sigma=float(d) ** 0.5)
    Xd = DistMatrix(X, (m * comm.size, d), "VC_STAR", comm) if comm.size > 1 else X
    Yd = DistMatrix(Y, (m * comm.size, 1), "VC_STAR", comm) if comm.size > 1 else Y
    res = []
    for rep in range(2):
        torch.cuda.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        S, W = ml.approximate_kernel_ridge(k, Xd, Yd, a.lam, a.features, context=sk.Context(3))
        torch.cuda.synchronize()
        res.append(time.perf_counter() - t0)
    extra = {}
    if a.compare_f64:
        os.environ["SKH_KRR_F64_GRAM"] = "1"
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, W64 = ml.approximate_kernel_ridge(k, Xd, Yd, a.lam, a.features, context=sk.Context(3))
        torch.cuda.synchronize()
        extra["f64_gram_s"] = round(time.perf_counter() - t0, 4)
        os.environ["SKH_KRR_F64_GRAM"] = "0"
        extra["w_rel_diff_vs_f64_gram"] = float((W.double() - W64.double()).norm() / W64.double().norm())
    # training fit on a sample (features of the first 100k local rows)
    Zs = S.apply(X[:100000], dim=sk.sketch.ROWWISE)
    pred = Zs.double() @ W.double().to(dev)
    rel = float((pred - Y[:100000].double()).norm() / Y[:100000].double().norm())
    t = torch.tensor(res, dtype=torch.float64, device=dev)
    comm.all_reduce_max(t)
    if comm.rank == 0:
        print(json.dumps({"metric": "RFT + KRR training wall-clock (approximate_kernel_ridge)",
                          "value": round(float(t[1]), 4), "unit": "s", "higher_is_better": False,
                          "n_gpus": comm.size, "scaling": "weak", "cold_first_run_s": round(float(t[0]), 4),
                          "train_rel_residual_sample": round(rel, 5), **extra,
                          "config": {"rows_per_gpu": m, "dim": d, "features": a.features, "lam": a.lam,
                                     "kernel": "gaussian", "dtype": "f32 features, normal equations: Z^T Z from exact bf16 split products (f32 sums per 8192 rows, f64 across), Z^T Y and the solve in f64"}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
