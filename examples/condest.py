"""Condition-number estimation of a sparse matrix (reference
examples/condest.cpp: CondEst with iter_lim 10000 on an HDF5 sparse matrix;
here a synthetic sparse matrix with a known spectrum, or --libsvm FILE).
"""
import argparse

import torch

from _common import Timer, device

import libskylark_amd as sk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=3000)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--libsvm", default=None, help="read the matrix from a LIBSVM file instead")
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    dev = device(a.device)
    ctx = sk.Context(23234)
    if a.libsvm:
        X, _ = sk.io.read_libsvm(a.libsvm)
        A = X.to(dev)
    else:
        D = sk.base.GaussianMatrix(a.m, a.n, ctx, device=dev)
        D = D * torch.logspace(0, -3, a.n, dtype=torch.float64, device=dev)
        D[torch.rand(a.m, a.n, device=dev) > 0.3] = 0
        A = D.to_sparse_csr()
    p = sk.nla.CondEstParams(am_i_printing=True, log_level=1, iter_lim=10000)
    with Timer("CondEst"):
        res = sk.nla.condest(A, ctx, p)
    print(f"Condition number = {res.cond:.4e} sigma_max = {res.sigma_max:.4e} sigma_min = {res.sigma_min:.4e}")


if __name__ == "__main__":
    main()
