"""Fused Fastfood kernel (fastfood.hip) for large N: per (row, block) the B
flip, two orthonormal DCT-IIs (in-LDS Stockham FFTs), the permutation and G
scale, Sm and the cosine epilogue in one launch -- against the fp64 CPU
definition of the same draws (reference sketch/FRFT_Elemental.hpp:72-160)."""
import math

import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.sketch import ROWWISE

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,S,m", [(8192, 16384, 37), (1024, 3000, 50), (2048, 2048, 9), (16384, 5000, 3)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fastfood_fused_matches_fp64(N, S, m, dt):
    g = torch.Generator().manual_seed(N + S)
    X = (torch.randn(m, N, generator=g, dtype=torch.float64) / math.sqrt(N)).to(dt)
    T = sk.sketch.FastGaussianRFT(N, S, sigma=3.0, context=sk.Context(7))
    assert T._fused_ok(X.cuda(), ROWWISE)
    # linear part vs the fp64 CPU composition of the same draws
    pre = T._features_pre(X.cuda(), ROWWISE).double().cpu()
    ref = T._features_pre(X.double(), ROWWISE)
    scale = ref.abs().max().item()
    err = (pre - ref).abs().max().item() / scale
    assert err < 2e-5, err
    # full map (fused cosine epilogue) vs the CPU map
    Z = T.apply(X.cuda(), dim=ROWWISE).double().cpu()
    Zr = T.apply(X.double(), dim=ROWWISE)
    assert Z.shape == (m, S)
    assert (Z - Zr).abs().max().item() < 2e-4 * math.sqrt(2.0 / S) * 10


def test_fastfood_fused_row_range():
    """out_rows (a feature range spanning two blocks) on the fused path."""
    N, S, m = 4096 * 2, 20000, 5
    X = torch.randn(m, N, dtype=torch.float64) / math.sqrt(N)
    T = sk.sketch.FastGaussianRFT(N, S, sigma=2.0, context=sk.Context(3))
    part = T._features_pre(X.float().cuda(), ROWWISE, out_rows=(7000, 17000)).double().cpu()
    full = T._features_pre(X, ROWWISE)[:, 7000:17000]
    assert (part - full).abs().max().item() / full.abs().max().item() < 2e-5
