"""GPU numerics for the ML / solver native kernels vs fp64 torch references."""
import math

import pytest
import torch

import libskylark_amd as sk
from libskylark_amd import ml

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("m,n,d", [(1, 1, 1), (70, 130, 33), (257, 64, 100)])
def test_pairwise_kernels(dev, dt, m, n, d):
    g = torch.Generator().manual_seed(m + n + d)
    X = torch.rand(m, d, generator=g, dtype=torch.float64)
    Y = torch.rand(n, d, generator=g, dtype=torch.float64)
    for k, ref in [(ml.Laplacian(d, 3.0), torch.exp(-(X[:, None] - Y[None]).abs().sum(-1) / 3.0)),
                   (ml.ExpSemigroup(d, 0.1), torch.exp(-0.1 * torch.sqrt(X[:, None] + Y[None]).sum(-1)))]:
        K = k.gram(X.to(dev, dt), Y=Y.to(dev, dt))
        tol = 1e-4 if dt == torch.float32 else 1e-10
        torch.testing.assert_close(K.double().cpu(), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_gemm_kernels(dev, dt):
    g = torch.Generator().manual_seed(0)
    X = torch.randn(300, 20, generator=g, dtype=torch.float64)
    Y = torch.randn(200, 20, generator=g, dtype=torch.float64)
    tol = 2e-4 if dt == torch.float32 else 1e-10
    kg = ml.Gaussian(20, 3.0)
    ref = torch.exp(-torch.cdist(X, Y) ** 2 / 18.0)
    torch.testing.assert_close(kg.gram(X.to(dev, dt), Y=Y.to(dev, dt)).double().cpu(), ref, rtol=tol, atol=tol)
    kp = ml.Polynomial(20, 2, 1.0, 0.1)
    ref = (0.1 * X @ Y.t() + 1.0) ** 2
    torch.testing.assert_close(kp.gram(X.to(dev, dt), Y=Y.to(dev, dt)).double().cpu(), ref, rtol=tol, atol=tol)


def test_asyrgs_native(dev):
    n = 2000
    T = torch.diag(torch.full((n,), 4.0, dtype=torch.float64))
    T -= torch.diag(torch.ones(n - 1, dtype=torch.float64), 1) + torch.diag(torch.ones(n - 1, dtype=torch.float64), -1)
    b = torch.randn(n, 3, dtype=torch.float64)
    X, code = sk.algorithms.asy_rgs(T.to_sparse_csr().to(dev), b.to(dev), context=sk.Context(3),
                                    params=sk.algorithms.AsyIterParams(tolerance=1e-9, sweeps_lim=300))
    assert code == -1
    assert float((T @ X.cpu() - b).norm() / b.norm()) < 1e-8


def test_krr_and_admm_on_gpu(dev):
    g = torch.Generator().manual_seed(1)
    X = torch.randn(2000, 8, generator=g, dtype=torch.float64)
    Y = torch.sin(X[:, :1])
    k = ml.Gaussian(8, 2.0)
    A = ml.faster_kernel_ridge(k, X.to(dev), Y.to(dev), 0.1, 256, sk.Context(2),
                               params=ml.KrrParams(tolerance=1e-10, iter_lim=300))
    Ar = ml.kernel_ridge(k, X, Y, 0.1)
    torch.testing.assert_close(A.cpu(), Ar, rtol=1e-5, atol=1e-6)
    lab = (X[:, 0] > 0).to(torch.float64) * 2 - 1
    s = ml.BlockADMMSolver("hinge", "l2", 0.01, 512, kernel=k, context=sk.Context(3))
    s.set_maxiter(20)
    model = s.train(X.to(dev).float(), lab.to(dev), regression=False, log=None)
    pred, _ = model.predict(X.to(dev).float())
    assert float((pred.cpu() == lab).double().mean()) > 0.95


def test_lsqr_on_gpu(dev):
    g = torch.Generator().manual_seed(0)
    A = torch.randn(5000, 50, generator=g, dtype=torch.float64)
    B = torch.randn(5000, 2, generator=g, dtype=torch.float64)
    X, code = sk.algorithms.lsqr(A.to(dev), B.to(dev),
                                 params=sk.algorithms.KrylovIterParams(tolerance=1e-13, iter_lim=300))
    torch.testing.assert_close(X.cpu(), torch.linalg.lstsq(A, B).solution, rtol=1e-8, atol=1e-8)
    Xf = sk.nla.faster_least_squares(A.to(dev), B.to(dev), sk.Context(1))
    torch.testing.assert_close(Xf.cpu(), torch.linalg.lstsq(A, B).solution, rtol=1e-7, atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["gaussian", "polynomial"])
def test_fused_gram_epilogue(dev, kind):
    """Large Gram matrices take the fused MFMA + epilogue kernel (EPI_GAUSS /
    EPI_POLY): compare with the fp64 definition."""
    from libskylark_amd.ml import kernels as KM
    g = torch.Generator().manual_seed(4)
    m, n, d = 3000, 2000, 64
    X = torch.randn(m, d, generator=g, dtype=torch.float64) / d ** 0.5
    Y = torch.randn(n, d, generator=g, dtype=torch.float64) / d ** 0.5
    if kind == "gaussian":
        k = ml.Gaussian(d, sigma=0.8)
        ref = torch.exp(-torch.cdist(X, Y) ** 2 / (2 * 0.8 ** 2))
    elif kind == "polynomial":
        k = ml.Polynomial(d, q=3, c=1.0, gamma=0.5)
        ref = (0.5 * X @ Y.t() + 1.0) ** 3
    assert m * n >= KM.FUSED_GRAM_MIN
    K = k.gram(X.float().to(dev), Y=Y.float().to(dev)).double().cpu()
    err = float((K - ref).abs().max() / ref.abs().max())
    assert err < 1e-4, err


def test_ata_pass_bf16_storage(dev):
    """One-pass A^T D / A X / A^T (A Y) with A stored as bf16 (the BlockADMM
    feature cache): exact bf16 values widened to f32, f32 products and sums --
    compared with fp64 of the same (rounded) operand."""
    from libskylark_amd.ops import normal_eq
    g = torch.Generator(device=dev).manual_seed(7)
    m, n = 50_001, 1024
    A = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16)
    Ad = A.double()
    D = torch.randn(m, 4, device=dev, generator=g)
    X = torch.randn(n, 4, device=dev, generator=g)
    assert normal_eq.native_ok(A, 4)
    W, Yo = normal_eq.dual(A, D, X)
    torch.testing.assert_close(W.double(), Ad.t() @ D.double(), rtol=2e-4, atol=2e-3)
    torch.testing.assert_close(Yo.double(), Ad @ X.double(), rtol=2e-4, atol=2e-3)
    W2, Y2 = normal_eq.ata(A, X, want_y=True)
    ay = Ad @ X.double()
    torch.testing.assert_close(Y2.double(), ay, rtol=2e-4, atol=2e-3)
    ref = Ad.t() @ Y2.double()   # W from the f32 y the kernel formed
    torch.testing.assert_close(W2.double(), ref, rtol=2e-4, atol=2e-2)


def test_admm_bf16_feature_cache_matches_f32(dev):
    """BlockADMM with the feature blocks cached as bf16: same classification
    accuracy and a training objective within 1% of the f32 cache."""
    g = torch.Generator().manual_seed(5)
    X = torch.randn(20000, 16, generator=g, dtype=torch.float64)
    lab = ((X[:, 0] + 0.5 * X[:, 1]) > 0).to(torch.float64) * 2 - 1
    k = ml.Gaussian(16, 3.0)
    res = {}
    for cd in (None, torch.bfloat16):
        s = ml.BlockADMMSolver("hinge", "l2", 0.01, 1024, kernel=k, NumFeaturePartitions=2, context=sk.Context(3))
        s.set_cache_transform(True)
        s.set_cache_dtype(cd)
        s.set_maxiter(15)
        model = s.train(X.to(dev).float(), lab.to(dev), regression=False, log=None)
        pred, _ = model.predict(X.to(dev).float())
        res[cd] = (float((pred.cpu() == lab).double().mean()), s.history[-1]["objective"] if s.history else None,
                   model.coef.double().cpu())
    (a32, o32, w32), (a16, o16, w16) = res[None], res[torch.bfloat16]
    assert a32 > 0.95 and abs(a16 - a32) < 0.005
    if o32 is not None:
        assert abs(o16 - o32) <= 0.01 * abs(o32)
    assert float((w16 - w32).norm() / w32.norm()) < 0.02


@pytest.mark.parametrize("loss,regression,ncls", [("squared", True, 1), ("lad", True, 1), ("hinge", False, 2),
                                                  ("hinge", False, 3), ("logistic", False, 3)])
def test_admm_native_prox_matches_torch(dev, loss, regression, ncls):
    """The fused per-iteration passes (admm_kernels.hip: prox, consensus
    updates, loss sums) against the torch element-wise chain they replace:
    same coefficients and objective history up to f32 rounding."""
    g = torch.Generator().manual_seed(11)
    X = torch.randn(12000, 12, generator=g, dtype=torch.float64)
    if regression:
        Y = X[:, 0] - 0.3 * X[:, 2] + 0.05 * torch.randn(12000, generator=g, dtype=torch.float64)
    else:
        s = X[:, 0] + 0.5 * X[:, 1]
        Y = torch.bucketize(s, torch.tensor([-0.4, 0.4], dtype=torch.float64)) if ncls == 3 else (s > 0).double() * 2 - 1
        Y = Y.double()
    k = ml.Gaussian(12, 3.0)
    res = {}
    for nat in (True, False):
        sol = ml.BlockADMMSolver(loss, "l2", 0.01, 512, kernel=k, NumFeaturePartitions=2, context=sk.Context(4))
        sol.native_prox = nat
        sol.set_cache_transform(True)
        sol.set_maxiter(8)
        model = sol.train(X.to(dev).float(), Y.to(dev), regression=regression, log=None)
        res[nat] = (model.coef.double().cpu(), [h["objective"] for h in sol.history])
    (w1, h1), (w0, h0) = res[True], res[False]
    assert float((w1 - w0).norm() / w0.norm()) < 2e-3, float((w1 - w0).norm() / w0.norm())
    for a, b in zip(h1, h0):
        assert abs(a - b) <= 2e-3 * abs(b) + 1e-6, (h1, h0)


def test_feature_map_precond_f32_apply_matches_f64(dev):
    """The GPU preconditioner application (f32 one-pass dual kernel + streaming
    GEMV) against the f64 Woodbury product, and CG converging to the same
    kernel-ridge solution with it."""
    from libskylark_amd.algorithms import krylov as K
    from libskylark_amd.algorithms.operators import DenseOp
    from libskylark_amd.ml import krr
    g = torch.Generator().manual_seed(3)
    X = torch.randn(6000, 10, generator=g).to(dev)
    B = torch.randn(6000, 1, generator=g).to(dev)
    ker = ml.kernel("gaussian", 10, 3.0)
    P = krr.FeatureMapPrecond(ker, 0.1, X, 256, sk.Context(7))
    assert P._v32 is not None
    got = P.apply(B)
    V = P.V
    ref = B.double() / P.lam - V @ (V.t() @ B.double())
    assert float((got.double() - ref).norm() / ref.norm()) < 1e-5
    Kg = ker.symmetric_gram(X)
    Kg.diagonal().add_(0.1)
    p = K.KrylovIterParams(tolerance=1e-6, iter_lim=500, check_every=5)
    A32, code = K.cg(DenseOp(Kg), B, params=p, M=P)
    P._v32 = None                       # the f64 application
    p = K.KrylovIterParams(tolerance=1e-6, iter_lim=500, check_every=5)
    A64, code64 = K.cg(DenseOp(Kg), B, params=p, M=P)
    assert code == -1 and code64 == -1
    assert float((A32 - A64).norm() / A64.norm()) < 1e-4


@pytest.mark.parametrize("blocks", [1, 4])
@pytest.mark.parametrize("n,s", [(20000, 512), (9000, 300), (777, 64)])
def test_krr_split_gram_matches_fp64(dev, n, s, blocks, monkeypatch):
    """Z^T Z of f32 features from the exact three-plane bf16 split (gemm_nt.hip
    k_split3_t + two NT GEMMs per row chunk, f32 sums per chunk, f64 across)
    against the fp64 product, ragged last chunk included (reference
    ml/krr.hpp:94-196 forms Z^T Z in the features' precision); blocks > 1:
    the block-upper-triangle products mirrored (s = 512 only; the others fall
    back to the full products)."""
    from libskylark_amd.ml import krr as K
    monkeypatch.setattr(K, "SPLIT_GRAM_ROWS", 4096)
    monkeypatch.setattr(K, "SPLIT_GRAM_BLOCKS", blocks)
    g = torch.Generator(device=dev).manual_seed(n)
    Z = torch.cos(torch.randn(n, s, generator=g, device=dev) * 3.0) * (2.0 / s) ** 0.5
    G = torch.zeros(s, s, dtype=torch.float64, device=dev)
    K._gram_split(Z, G)
    ref = Z.double().t() @ Z.double()
    rel = float((G - ref).abs().max() / ref.abs().max())
    assert rel < 1e-5, rel   # f32 sums over <= 4 x 4096 exact products per chunk: ~2^-24 sqrt(K)
    assert torch.equal(G, G.t()) or float((G - G.t()).abs().max() / ref.abs().max()) < 1e-6


def test_krr_ridge_split_matches_fp64_gram(dev, monkeypatch):
    """approximate_kernel_ridge's weights with the split Gram against the
    all-fp64 normal equations on the same features."""
    import libskylark_amd as sk
    from libskylark_amd import ml
    g = torch.Generator(device=dev).manual_seed(5)
    X = torch.randn(30000, 64, generator=g, device=dev)
    Y = torch.sin(X[:, :1]) + 0.01 * torch.randn(30000, 1, generator=g, device=dev)
    k = ml.Gaussian(64, sigma=8.0)
    _, W = ml.approximate_kernel_ridge(k, X, Y, 1e-2, 512, context=sk.Context(3))
    monkeypatch.setenv("SKH_KRR_F64_GRAM", "1")
    _, W64 = ml.approximate_kernel_ridge(k, X, Y, 1e-2, 512, context=sk.Context(3))
    rel = float((W.double() - W64.double()).norm() / W64.double().norm())
    assert rel < 1e-4, rel
