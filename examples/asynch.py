"""AsyRGS, CG and AsyFCG on a sparse SPD system (reference
examples/asynch.cpp: the same three solvers, tolerances and sweep limits).
"""
import argparse

import torch

from _common import Timer, device

import libskylark_amd as sk
from libskylark_amd import algorithms as alg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    dev = device(a.device)
    ctx = sk.Context(23234)
    # sparse SPD: shifted 2-D Laplacian-like matrix
    n = a.n
    i = torch.arange(n)
    rows = torch.cat([i, i[1:], i[:-1], i[32:], i[:-32]])
    cols = torch.cat([i, i[:-1], i[1:], i[:-32], i[32:]])
    vals = torch.cat([torch.full((n,), 4.5), -torch.ones(2 * (n - 1) + 2 * (n - 32))]).double()
    A = torch.sparse_coo_tensor(torch.stack([rows, cols]), vals, (n, n)).coalesce().to_sparse_csr().to(dev)
    b = sk.base.GaussianMatrix(n, 1, ctx, device=dev)

    with Timer("Using AsyRGS"):
        x, code = alg.asy_rgs(A, b, None, ctx, alg.AsyIterParams(tolerance=1e-3, syn_sweeps=5, sweeps_lim=2000,
                                                                am_i_printing=True, log_level=1))
    print(f"  code {code} relres {float((A @ x - b).norm() / b.norm()):.2e}")
    with Timer("Using CG"):
        x, code = alg.cg(A, b, None, alg.KrylovIterParams(tolerance=1e-3, iter_lim=2000, res_print=30,
                                                          am_i_printing=True, log_level=1))
    print(f"  code {code} relres {float((A @ x - b).norm() / b.norm()):.2e}")
    with Timer("Using FCG (high accuracy)"):
        x, code = alg.asy_fcg(A, b, None, ctx, alg.AsyIterParams(tolerance=1e-8, sweeps_lim=2, syn_sweeps=0,
                                                                iter_lim=200, am_i_printing=True, log_level=1))
    print(f"  code {code} relres {float((A @ x - b).norm() / b.norm()):.2e}")


if __name__ == "__main__":
    main()
