"""The regression framework: exact (QR / SNE / SVD), sketched (CWT/JLT
sketch-and-solve) and accelerated (Blendenpik / LSRN) l2 regression solvers on
one problem (reference examples/regression.cpp,
algorithms/regression/*).
"""
import argparse

import torch

from _common import Timer, device

import libskylark_amd as sk
from libskylark_amd import algorithms as alg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=10000)
    ap.add_argument("--n", type=int, default=50)
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    dev = device(a.device)
    ctx = sk.Context(5)
    A = sk.base.GaussianMatrix(a.m, a.n, ctx, device=dev)
    b = A @ torch.ones(a.n, 1, dtype=A.dtype, device=dev) + 0.1 * sk.base.GaussianMatrix(a.m, 1, ctx, device=dev)
    prob = alg.RegressionProblem(A, "l2")
    for tag in ("qr", "sne", "svd"):
        with Timer(f"exact solver [{tag}]"):
            x = alg.RegressionSolver(prob, tag).solve(b)
        print(f"  residual {float((A @ x.view(-1, 1) - b).norm()):.4f}")
    for sk_name in ("CWT", "JLT"):
        with Timer(f"sketched solver [{sk_name}, t=4n]"):
            x = alg.SketchedRegressionSolver(prob, ctx, sk_name, 4 * a.n).solve(b)
        print(f"  residual {float((A @ x.view(-1, 1) - b).norm()):.4f}")
    for tag in ("blendenpik", "lsrn", "simplified_blendenpik"):
        with Timer(f"accelerated solver [{tag}]"):
            x = alg.AcceleratedRegressionSolver(prob, ctx, tag).solve(b)
            x = x[0] if isinstance(x, tuple) else x     # (x, krylov return code)
        print(f"  residual {float((A @ x.view(-1, 1) - b).norm()):.4f}")


if __name__ == "__main__":
    main()
