"""FasterKernelRidge CG iteration cost on the GPU:
CG on (K + lam I) A = Y with the random-feature Woodbury preconditioner
(reference ml/krr.hpp:452-541, algorithms/Krylov/CG.hpp:24-163) on an
n-point Gaussian Gram, device-scalar CG (sl_cg_*) against the torch-op
iteration, plus the kernel launches per CG iteration counted with the torch
profiler on a small system (operator GEMV and preconditioner included).

usage: python benchmarks/krr_cg.py [n] [d] [s]"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import libskylark_amd as sk  # noqa: E402
from libskylark_amd.algorithms import krylov as K  # noqa: E402
from libskylark_amd.algorithms.operators import DenseOp  # noqa: E402
from libskylark_amd.ml import krr  # noqa: E402
from libskylark_amd.ops import krylov_native as kn  # noqa: E402


def launches_per_iter(op, Yl, P, iters=20):
    from torch.profiler import ProfilerActivity, profile
    p = K.KrylovIterParams(tolerance=1e-30, iter_lim=iters, check_every=iters)
    K.cg(op, Yl, params=p, M=P)      # warm
    torch.cuda.synchronize()
    counts = []
    for n_it in (iters, 2 * iters):
        p = K.KrylovIterParams(tolerance=1e-30, iter_lim=n_it, check_every=n_it)
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            K.cg(op, Yl, params=p, M=P)
            torch.cuda.synchronize()
        counts.append(sum(1 for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA))
    return (counts[1] - counts[0]) / iters


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    s = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    X = torch.randn(n, d, generator=g).to(dev)
    Y = torch.randn(n, 1, generator=g).to(dev)
    ker = sk.ml.kernel("gaussian", d, 4.0)
    lam = 1e-2
    t0 = time.perf_counter()
    Kg = ker.symmetric_gram(X)
    Kg.diagonal().add_(lam)
    torch.cuda.synchronize()
    t_gram = time.perf_counter() - t0
    op = DenseOp(Kg)
    P = krr.FeatureMapPrecond(ker, lam, X, s, sk.Context(seed=3))
    out = {"n": n, "d": d, "s": s, "dtype": str(Kg.dtype), "gram_s": round(t_gram, 3)}
    for name, enabled in (("native", True), ("torch_ops", False)):
        kn.ENABLED = enabled
        try:
            for ce in (1, 10):
                p = K.KrylovIterParams(tolerance=1e-30, iter_lim=20, check_every=ce)
                K.cg(op, Y, params=p, M=P)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                K.cg(op, Y, params=p, M=P)
                torch.cuda.synchronize()
                out[f"{name}_ms_per_iter_check{ce}"] = round((time.perf_counter() - t0) / 20 * 1e3, 3)
        finally:
            kn.ENABLED = True
    # launch counts on a small system (same code path, operator + precond included)
    m = 4096
    Ks = ker.symmetric_gram(X[:m])
    Ks.diagonal().add_(lam)
    ops = DenseOp(Ks)
    Ps = krr.FeatureMapPrecond(ker, lam, X[:m], 64, sk.Context(seed=3))
    try:
        for name, enabled in (("native", True), ("torch_ops", False)):
            kn.ENABLED = enabled
            out[f"{name}_launches_per_iter_precond"] = launches_per_iter(ops, Y[:m], Ps)
            out[f"{name}_launches_per_iter_noprecond"] = launches_per_iter(ops, Y[:m], K.IdPrecond())
    except Exception as e:  # noqa: BLE001 - profiler unavailable
        out["launch_count_error"] = repr(e)[:200]
    finally:
        kn.ENABLED = True
    # FasterKernelRidge solves to convergence at the reference's defaults
    # (ml/krr.hpp:39-41: tolerance 1e-3, iter_lim 1000; code -1 = converged):
    # iterations and wall-clock (preconditioner setup included) per feature count
    print(json.dumps(out), flush=True)
    for s_pc in (s, 2048, 4096):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Pc = krr.FeatureMapPrecond(ker, lam, X, s_pc, sk.Context(seed=3))
        torch.cuda.synchronize()
        t_pc = time.perf_counter() - t0
        p = K.KrylovIterParams(tolerance=1e-3, iter_lim=1000, check_every=5)
        t0 = time.perf_counter()
        A, code = K.cg(op, Y, params=p, M=Pc)
        torch.cuda.synchronize()
        t_cg = time.perf_counter() - t0
        rec = {"bench": "faster_kernel_ridge_solve", "n": n, "d": d, "features": s_pc, "lam": lam,
               "tolerance": 1e-3, "code": code, "converged": code == -1,
               "iterations": getattr(p, "iterations", None), "precond_setup_s": round(t_pc, 3),
               "cg_s": round(t_cg, 3), "total_s": round(t_pc + t_cg, 3),
               "relres": float((op.matmul(A) - Y).norm() / Y.norm())}
        print(json.dumps(rec), flush=True)
        del Pc, A
        torch.cuda.empty_cache()
    # the same solve over kernel widths / regularisations: sigma ~ the median
    # pairwise distance (sqrt(2 d) = 8 for d = 32) and larger lambda give the
    # random-feature preconditioner a spectrum it captures
    del op, Kg
    torch.cuda.empty_cache()
    for sigma, lam2 in ((4.0, 1e-1), (8.0, 1e-2), (8.0, 1e-1), (8.0, 1.0)):
        ker2 = sk.ml.kernel("gaussian", d, sigma)
        Kg2 = ker2.symmetric_gram(X)
        Kg2.diagonal().add_(lam2)
        op2 = DenseOp(Kg2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Pc = krr.FeatureMapPrecond(ker2, lam2, X, 4096, sk.Context(seed=3))
        torch.cuda.synchronize()
        t_pc = time.perf_counter() - t0
        p = K.KrylovIterParams(tolerance=1e-3, iter_lim=1000, check_every=5)
        t0 = time.perf_counter()
        A, code = K.cg(op2, Y, params=p, M=Pc)
        torch.cuda.synchronize()
        t_cg = time.perf_counter() - t0
        rec = {"bench": "faster_kernel_ridge_solve", "n": n, "d": d, "sigma": sigma, "features": 4096, "lam": lam2,
               "tolerance": 1e-3, "code": code, "converged": code == -1,
               "iterations": getattr(p, "iterations", None), "precond_setup_s": round(t_pc, 3),
               "cg_s": round(t_cg, 3), "total_s": round(t_pc + t_cg, 3),
               "relres": float((op2.matmul(A) - Y).norm() / Y.norm())}
        print(json.dumps(rec), flush=True)
        del Pc, A, op2, Kg2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
