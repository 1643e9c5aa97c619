"""Approximate (sketch-and-solve, FJLT) and faster (Blendenpik: sketched QR
preconditioner + LSQR) least squares vs the exact solve (reference
examples/least_squares.cpp, nla/least_squares.hpp).
"""
import argparse

import torch

from _common import Timer, device

import libskylark_amd as sk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=20000)
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--cond", type=float, default=1e4)
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    dev = device(a.device)
    ctx = sk.Context(23234)
    U, _ = torch.linalg.qr(sk.base.GaussianMatrix(a.m, a.n, ctx, device=dev))
    V, _ = torch.linalg.qr(sk.base.GaussianMatrix(a.n, a.n, ctx, device=dev))
    s = torch.logspace(0, -torch.log10(torch.tensor(a.cond)).item(), a.n, dtype=torch.float64, device=dev)
    A = (U * s) @ V.t()
    b = sk.base.GaussianMatrix(a.m, 1, ctx, device=dev)
    with Timer("exact (QR)"):
        x = torch.linalg.lstsq(A.cpu(), b.cpu()).solution.to(dev)
    r0 = float((A @ x - b).norm())
    print(f"  residual {r0:.6f}")
    with Timer("approximate (FJLT sketch-and-solve)"):
        xa = sk.nla.approximate_least_squares(A, b, ctx)
    print(f"  residual {float((A @ xa.view(-1, 1) - b).norm()):.6f}")
    with Timer("faster (Blendenpik + LSQR)"):
        xf = sk.nla.faster_least_squares(A, b, ctx)
    print(f"  residual {float((A @ xf.view(-1, 1) - b).norm()):.6f}  (exact {r0:.6f})")


if __name__ == "__main__":
    main()
