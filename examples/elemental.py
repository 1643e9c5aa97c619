"""Sketch-and-solve least squares with several sketches, comparing residuals
with the exact solution (reference examples/elemental.cpp and the
"Elemental Sketch" notebook: m=2000, n=30, t=100 with JLT / CWT).
"""
import argparse

import torch

from _common import Timer, device

import libskylark_amd as sk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=2000)
    ap.add_argument("--n", type=int, default=30)
    ap.add_argument("--t", type=int, default=100)
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    dev = device(a.device)
    ctx = sk.Context(123)
    A = sk.base.GaussianMatrix(a.m, a.n, ctx, device=dev)
    b = sk.base.GaussianMatrix(a.m, 1, ctx, device=dev)
    with Timer("exact least squares"):
        x = torch.linalg.lstsq(A.cpu(), b.cpu()).solution.to(dev)
    print(f"  residual {float((A @ x - b).norm()):.2f}")
    for name in ("JLT", "CWT", "FJLT", "SJLT"):
        S = getattr(sk.sketch, name)(a.m, a.t, context=ctx)
        with Timer(f"{name} sketch-and-solve (t={a.t})"):
            SA, Sb = S * A, S * b
            xs = torch.linalg.lstsq(SA.cpu(), Sb.cpu()).solution.to(dev)
        print(f"  residual {float((A @ xs - b).norm()):.2f}")


if __name__ == "__main__":
    main()
