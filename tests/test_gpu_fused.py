"""Fused dense-sketch / random-feature / kernel-Gram maps on the NT GEMM (gemm_nt.hip, sl_gemm_nt_map) vs fp64
torch references of the same op."""
import math

import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.ops import fused as F

pytestmark = pytest.mark.gpu


def _ref(A, W, dim, sc=None, sh=None, outscale=1.0, epi=F.EPI_NONE):
    X = A.double().cpu()
    X = X if dim == 1 else X.t()
    Z = X @ W.double().cpu().t()
    if epi == F.EPI_COS:
        Z = outscale * torch.cos(Z * (sc.double().cpu() if sc is not None else 1.0) + sh.double().cpu())
    elif epi == F.EPI_EXPNEG:
        Z = outscale * torch.exp(-Z)
    else:
        Z = outscale * Z
    return Z if dim == 1 else Z.t()


@pytest.mark.parametrize("adt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("dim", [0, 1])
@pytest.mark.parametrize("epi", [F.EPI_NONE, F.EPI_COS, F.EPI_EXPNEG])
def test_feature_gemm_matches_fp64(dev, adt, dim, epi):
    torch.manual_seed(0)
    M, K, NF = 1037, 301, 259          # tails in every dimension
    A = torch.randn(M, K) if dim == 1 else torch.randn(K, M)
    if epi == F.EPI_EXPNEG:
        A = A.abs() * 0.01
    W = torch.randn(NF, K) / math.sqrt(K)
    if epi == F.EPI_EXPNEG:
        W = W.abs()
    sc = torch.rand(NF) + 0.5
    sh = torch.rand(NF) * 2 * math.pi
    Ad = A.to(dev, adt)
    Wd = F.SplitW(W.to(dev))
    out = F.feature_gemm(Ad, Wd, dim, scales=sc if epi == F.EPI_COS else None,
                         shifts=sh if epi == F.EPI_COS else None, outscale=0.7, epi=epi)
    assert out.shape == ((M, NF) if dim == 1 else (NF, M))
    ref = _ref(Ad, W, dim, sc, sh, 0.7, epi)
    # f32-class: |err| <~ 2^-16 * sum|a w| (plus v_cos on the reduced argument)
    mag = (Ad.double().cpu().abs() if dim == 1 else Ad.double().cpu().abs().t()) @ W.abs().double().t()
    if dim == 0:
        mag = mag.t()
    tol = 4e-5 * float(mag.max()) + 2e-6
    err = (out.double().cpu() - ref).abs().max().item()
    assert err < tol, (err, tol)


@pytest.mark.parametrize("adt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(1000, 301, 500), (2048, 512, 1024), (777, 64, 4096)])
@pytest.mark.parametrize("epi", [F.EPI_NONE, F.EPI_COS])
def test_feature_gemm_large_tiles_match_fp64(dev, adt, shape, epi):
    """256 x 128-tile LDS-DMA variant (row-major output, feature tiles in
    multiples of 4 x 128): ragged rows / features / K against fp64, ."""
    torch.manual_seed(3)
    M, K, NF = shape
    A = torch.randn(M, K)
    W = torch.randn(NF, K) / math.sqrt(K)
    sc = torch.rand(NF) + 0.5
    sh = torch.rand(NF) * 2 * math.pi
    Ad = A.to(dev, adt)
    Wd = F.SplitW(W.to(dev))
    kw = dict(scales=sc if epi == F.EPI_COS else None, shifts=sh if epi == F.EPI_COS else None, outscale=0.7, epi=epi)
    out = F.feature_gemm(Ad, Wd, 1, **kw)
    ref = _ref(Ad, W, 1, sc, sh, 0.7, epi)
    mag = Ad.double().cpu().abs() @ W.abs().double().t()
    tol = 4e-5 * float(mag.max()) + 2e-6
    assert (out.double().cpu() - ref).abs().max().item() < tol


def test_feature_gemm_transposed_view_and_unaligned(dev):
    torch.manual_seed(1)
    M, K, NF = 700, 77, 130
    base = torch.randn(M, K + 3, device=dev)
    A = base[:, 1:K + 1]                   # unaligned rows -> staged copy
    W = torch.randn(NF, K)
    out = F.feature_gemm(A, F.SplitW(W.to(dev)), 1)
    ref = A.double().cpu() @ W.double().t()
    assert (out.double().cpu() - ref).abs().max().item() < 1e-4 * ref.abs().max().item()
    At = torch.randn(M, K, device=dev).t()  # columnwise input that is a transposed view
    out0 = F.feature_gemm(At, F.SplitW(W.to(dev)), 0)
    ref0 = W.double() @ At.double().cpu()
    assert (out0.double().cpu() - ref0).abs().max().item() < 1e-4 * ref0.abs().max().item()


@pytest.mark.parametrize("name", ["JLT", "CT", "SJLT"])
@pytest.mark.parametrize("dim", [0, 1])
def test_dense_sketch_fused_vs_explicit(dev, name, dim):
    N, S, M = 900, 300, 500
    T = getattr(sk.sketch, name)(N, S, context=sk.Context(11))
    P = T.realize(torch.float64)
    A = torch.randn(N, M, dtype=torch.float64) if dim == 0 else torch.randn(M, N, dtype=torch.float64)
    Ad = A.to(dev, torch.float32)
    assert F.fused_ok(Ad, dim, N, S)
    out = T.apply(Ad, dim=dim).double().cpu()
    ref = P @ Ad.double().cpu() if dim == 0 else Ad.double().cpu() @ P.t()
    mag = float((P.abs() @ A.abs() if dim == 0 else A.abs() @ P.abs().t()).max())
    assert (out - ref).abs().max().item() < 3e-5 * mag


@pytest.mark.parametrize("name,kw", [("GaussianRFT", {"sigma": 3.0}), ("LaplacianRFT", {"sigma": 3.0}),
                                     ("MaternRFT", {"nu": 1.5, "l": 3.0}), ("GaussianQRFT", {"sigma": 3.0}),
                                     ("ExpSemigroupRLT", {"beta": 0.5}), ("ExpSemigroupQRLT", {"beta": 0.5}),
                                     ("FastGaussianRFT", {"sigma": 3.0}), ("FastMaternRFT", {"nu": 1.5, "l": 3.0})])
@pytest.mark.parametrize("dim", [0, 1])
def test_feature_maps_fused_vs_cpu(dev, name, kw, dim):
    N, S, M = 64, 384, 1000
    T = getattr(sk.sketch, name)(N, S, context=sk.Context(5), **kw)
    g = torch.Generator().manual_seed(2)
    A = torch.rand(N, M, generator=g, dtype=torch.float64) if dim == 0 else \
        torch.rand(M, N, generator=g, dtype=torch.float64)
    ref = T.apply(A, dim=dim)                     # CPU fp64 path (GEMM + separate epilogue)
    Ad = A.to(dev, torch.float32)
    assert F.fused_ok(Ad, dim, N, S)
    out = T.apply(Ad, dim=dim).double().cpu()
    assert out.shape == ref.shape
    # f32-class argument error scales with the feature's frequency norm
    # (Cauchy / Levy frequencies are heavy tailed, so some arguments are huge)
    W = T.realize_W(torch.float64)
    bound = W.abs().sum(1) * float(A.abs().max())
    if getattr(T, "scales", None) is not None:
        bound = bound * T.scales.double().cpu()
    tol = T.outscale * (5e-5 * bound + 1e-4)   # 3-term split product: ~2^-16 of sum|a w|
    err = (out - ref).abs()
    err = err.max(dim=1 - dim).values
    assert bool((err <= tol).all()), float((err - tol).max())


@pytest.mark.parametrize("dim", [0, 1])
def test_fjlt_direct_fused_vs_explicit(dev, dim):
    N, S, M = 700, 120, 300
    T = sk.sketch.FJLT(N, S, context=sk.Context(9))
    P = T.realize(torch.float64)
    A = torch.randn(N, M, dtype=torch.float64) if dim == 0 else torch.randn(M, N, dtype=torch.float64)
    Ad = A.to(dev, torch.float32)
    out = T.apply(Ad, dim=dim).double().cpu()
    ref = P @ Ad.double().cpu() if dim == 0 else Ad.double().cpu() @ P.t()
    assert (out - ref).abs().max().item() < 3e-5 * float(ref.abs().max())


def test_feature_map_large_output_nt_stores(dev):
    """GaussianRFT rowwise on 4160 x 512 f32 -> 4096 features: a 68 MB f32
    output at K = 3 x 512 (the f32-exact split), where the NT GEMM's auto rule
    turns on non-temporal C stores; against the CPU fp64 path."""
    N, S, M = 512, 4096, 4160
    T = sk.sketch.GaussianRFT(N, S, context=sk.Context(21), sigma=8.0)
    g = torch.Generator().manual_seed(4)
    A = torch.rand(M, N, generator=g, dtype=torch.float64)
    ref = T.apply(A, dim=1)
    Ad = A.to(dev, torch.float32)
    assert F.fused_ok(Ad, 1, N, S)
    out = T.apply(Ad, dim=1)
    assert out.numel() * out.element_size() >= 64 << 20
    W = T.realize_W(torch.float64)
    bound = W.abs().sum(1) * float(A.abs().max())
    if getattr(T, "scales", None) is not None:
        bound = bound * T.scales.double().cpu()
    tol = T.outscale * (5e-5 * bound + 1e-4)
    err = (out.double().cpu() - ref).abs().max(dim=0).values
    assert bool((err <= tol).all()), float((err - tol).max())
