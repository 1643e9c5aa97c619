"""A short FasterKernelRidge CG run (n = 1e5 Gaussian Gram, 512-feature
preconditioner, 10 iterations) for a kernel-level profile of one iteration:
`rocprofv3 --kernel-trace --stats -- python3 benchmarks/krr_iter_profile.py`."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libskylark_amd as sk  # noqa: E402
from libskylark_amd.algorithms import krylov as K  # noqa: E402
from libskylark_amd.algorithms.operators import DenseOp  # noqa: E402
from libskylark_amd.ml import krr  # noqa: E402


def main():
    n, d, s = 100_000, 32, 512
    g = torch.Generator(device="cpu").manual_seed(0)
    X = torch.randn(n, d, generator=g).cuda()
    Y = torch.randn(n, 1, generator=g).cuda()
    ker = sk.ml.kernel("gaussian", d, 4.0)
    Kg = ker.symmetric_gram(X)
    Kg.diagonal().add_(1e-2)
    P = krr.FeatureMapPrecond(ker, 1e-2, X, s, sk.Context(seed=3))
    p = K.KrylovIterParams(tolerance=1e-30, iter_lim=10, check_every=10)
    K.cg(DenseOp(Kg), Y, params=p, M=P)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
