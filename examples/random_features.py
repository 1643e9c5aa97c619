"""Random Fourier features of a dataset (reference
examples/random_features.cpp: read LIBSVM, apply GaussianRFT with --seed,
--sigma and --numfeatures, write the features as LIBSVM).  Without an input
file a synthetic dataset is used; on a GPU the fused MFMA feature kernel runs.
"""
import argparse

import torch

from _common import Timer, device

import libskylark_amd as sk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("input", nargs="?")
    ap.add_argument("output", nargs="?")
    ap.add_argument("--seed", "-s", type=int, default=38734)
    ap.add_argument("--sigma", "-x", type=float, default=10.0)
    ap.add_argument("--numfeatures", "-f", type=int, default=1000)
    ap.add_argument("--rows", type=int, default=10000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    dev = device(a.device)
    ctx = sk.Context(a.seed)
    if a.input:
        X, Y = sk.io.read_libsvm(a.input)
        X = X.to_dense() if X.layout != torch.strided else X
    else:
        X = sk.base.UniformMatrix(a.rows, a.dim, ctx)
        Y = torch.zeros(a.rows)
    X = X.to(dev, torch.float32)
    T = sk.sketch.GaussianRFT(X.shape[1], a.numfeatures, sigma=a.sigma, context=ctx)
    with Timer(f"GaussianRFT {tuple(X.shape)} -> {a.numfeatures} features"):
        Z = T / X            # rowwise: one feature vector per example
    print(f"  features {tuple(Z.shape)}; kernel approx error on 5 pairs: "
          f"{float(((Z[:5] @ Z[5:10].t()) - torch.exp(-torch.cdist(X[:5], X[5:10]) ** 2 / (2 * a.sigma ** 2))).abs().max()):.3f}")
    if a.output:
        sk.io.write_libsvm(a.output, Z.cpu().double(), Y)
        print(f"  wrote {a.output}")


if __name__ == "__main__":
    main()
