"""FasterKernelRidge at small lambda: CG on (K + lam I) A
= Y, n = 1e5 Gaussian Gram (d = 32, sigma = 4), lam = 1e-2, tolerance 1e-3,
iteration limit 1000 (reference ml/krr.hpp:39-41 defaults), with the
reference's random-feature Woodbury preconditioner against the Nystrom one
(KrrParams.precond = "nystrom"), per preconditioner size: iterations,
preconditioner setup and CG wall-clock, relres.

usage: python benchmarks/krr_precond_ab.py [n]"""
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    d, sigma, lam = 32, 4.0, 1e-2
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    X = torch.randn(n, d, generator=g).to(dev)
    Y = torch.randn(n, 1, generator=g).to(dev)
    ker = sk.ml.kernel("gaussian", d, sigma)
    Kg = ker.symmetric_gram(X)
    Kg.diagonal().add_(lam)
    op = DenseOp(Kg)
    for kind, s in (("features", 4096), ("nystrom", 512), ("nystrom", 1024), ("nystrom", 2048), ("nystrom", 4096)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if kind == "features":
            P = krr.FeatureMapPrecond(ker, lam, X, s, sk.Context(seed=3))
        else:
            P = krr.NystromPrecond(Kg, lam, s, n, 0, sk.Context(seed=3))
        torch.cuda.synchronize()
        t_pc = time.perf_counter() - t0
        p = K.KrylovIterParams(tolerance=1e-3, iter_lim=1000, check_every=5)
        t0 = time.perf_counter()
        A, code = K.cg(op, Y, params=p, M=P)
        torch.cuda.synchronize()
        t_cg = time.perf_counter() - t0
        print(json.dumps({"bench": "fkrr_precond", "precond": kind, "size": s, "n": n, "d": d, "sigma": sigma,
                          "lam": lam, "tolerance": 1e-3, "converged": code == -1,
                          "iterations": getattr(p, "iterations", None), "precond_setup_s": round(t_pc, 3),
                          "cg_s": round(t_cg, 3), "total_s": round(t_pc + t_cg, 3),
                          "relres": float((op.matmul(A) - Y).norm() / Y.norm())}), flush=True)
        del P, A
        torch.cuda.empty_cache()
    # end to end through the public entry point
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    A = sk.ml.faster_kernel_ridge(ker, X, Y, lam, 2048, sk.Context(seed=3), params=krr.KrrParams(precond="nystrom"))
    torch.cuda.synchronize()
    Kg2 = ker.symmetric_gram(X)
    Kg2.diagonal().add_(lam)
    print(json.dumps({"bench": "faster_kernel_ridge", "precond": "nystrom", "size": 2048, "n": n, "lam": lam,
                      "total_s_incl_gram": round(time.perf_counter() - t0, 3),
                      "relres": float((Kg2 @ A - Y).norm() / Y.norm())}), flush=True)


if __name__ == "__main__":
    main()
