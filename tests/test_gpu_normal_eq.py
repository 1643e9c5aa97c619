"""One-pass ``A^T (A Y)`` kernel (ata_kernels.hip) against an fp64 torch
reference, and the normal-form LSQR / Chebyshev iterations built on it
against the classic two-product iterations."""
import math

import pytest
import torch

from libskylark_amd.algorithms import krylov as K
from libskylark_amd.ops import normal_eq


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(10007, 100, 1), (10007, 1000, 4), (4099, 2048, 4), (20001, 3000, 2),
                                   (7, 5000, 1), (30011, 5000, 1), (513, 6144, 1), (1, 257, 2)])
def test_ata_pass_vs_fp64(dev, m, n, k):
    g = torch.Generator().manual_seed(m + n + k)
    A = torch.randn(m, n, generator=g)
    Y = torch.randn(n, k, generator=g)
    Ag = A.to(dev)
    assert normal_eq.native_ok(Ag, k)
    W, AY = normal_eq.ata(Ag, Y.to(dev), want_y=True)
    torch.cuda.synchronize()
    Yr = A.double() @ Y.double()
    Wr = A.double().t() @ Yr
    ew = float((W.double().cpu() - Wr).norm() / Wr.norm())
    ey = float((AY.double().cpu() - Yr).norm() / Yr.norm())
    assert ew < 1e-5 and ey < 1e-5, (ew, ey)
    W2, none = normal_eq.ata(Ag, Y.to(dev), want_y=False)
    assert none is None
    assert torch.equal(W2, W)   # deterministic: fixed slab order


@pytest.mark.gpu
def test_ata_strided_rows(dev):
    """lda > n (a column slice of a wider matrix)."""
    g = torch.Generator().manual_seed(3)
    big = torch.randn(5000, 1200, generator=g)
    A = big.to(dev)[:, :1000]
    Y = torch.randn(1000, 2, generator=g)
    W, _ = normal_eq.ata(A, Y.to(dev))
    Wr = big[:, :1000].double().t() @ (big[:, :1000].double() @ Y.double())
    assert float((W.double().cpu() - Wr).norm() / Wr.norm()) < 1e-5


@pytest.mark.gpu
def test_normal_form_krylov_matches_classic(dev):
    from libskylark_amd.algorithms.regression import _build_precond
    g = torch.Generator().manual_seed(0)
    m, n = 40000, 300
    A = (torch.randn(m, n, generator=g) * torch.logspace(0, -4, n)).to(dev)
    x = torch.randn(n, 1, generator=g).to(dev)
    b = A @ x + 1e-3 * torch.randn(m, 1, generator=g).to(dev)
    S = torch.randn(4 * n, m, generator=g).to(dev) / math.sqrt(4 * n)
    P, _ = _build_precond(S @ A, "qr")
    t = 4 * n
    al = math.sqrt(2 * math.log(2e6) / t)
    sU = math.sqrt(t) / ((1 - al) * math.sqrt(t) - math.sqrt(n))
    sL = math.sqrt(t) / ((1 + al) * math.sqrt(t) + math.sqrt(n))
    out = {}
    for fused in (False, True):
        p = K.KrylovIterParams(tolerance=1e-6, iter_lim=200, fused_normal=fused, check_every=5)
        Xc = K.chebyshev_ls(A, b, sL, sU, p, P)
        Xl, code = K.lsqr(A, b, params=p, R=P)
        out[fused] = (Xc, Xl, code)
    assert out[True][2] in (-2, -3)
    for i in (0, 1):
        d = float((out[True][i] - out[False][i]).norm() / out[False][i].norm())
        assert d < 1e-3, (i, d)
    r = float((A @ out[True][0] - b).norm() / (A @ out[False][0] - b).norm())
    assert abs(r - 1) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k,with_x", [(10007, 1024, 4, True), (5003, 1024, 4, False), (20001, 3000, 2, True),
                                          (999, 5000, 1, False), (3, 300, 2, True)])
def test_dual_pass_vs_fp64(dev, m, n, k, with_x):
    g = torch.Generator().manual_seed(m * 7 + k)
    A = torch.randn(m, n, generator=g)
    Dt = torch.randn(k, m, generator=g)           # given as k x m: the kernel reads its transpose
    X = torch.randn(n, k, generator=g) if with_x else None
    W, Y = normal_eq.dual(A.to(dev), Dt.to(dev).t(), X.to(dev) if with_x else None)
    torch.cuda.synchronize()
    Wr = A.double().t() @ Dt.double().t()
    assert float((W.double().cpu() - Wr).norm() / Wr.norm()) < 1e-5
    if with_x:
        Yr = A.double() @ X.double()
        assert float((Y.double().cpu() - Yr).norm() / Yr.norm()) < 1e-5
    else:
        assert Y is None


@pytest.mark.gpu
def test_admm_one_pass_matches_four_products(dev):
    """BlockADMM with the two fused Z passes per block is as accurate as the
    four-product iteration: both f32 runs against an f64 run of the same
    iteration (ADMM's (Z^T Z + I)^-1 step amplifies f32 rounding, so the two
    f32 paths differ from each other at about the level they differ from f64)."""
    import libskylark_amd as sk
    from libskylark_amd import ml
    g = torch.Generator(device=dev).manual_seed(1)
    m, d = 20000, 32
    lab = torch.randint(0, 3, (m,), generator=g, device=dev)
    centers = torch.randn(3, d, generator=torch.Generator(device=dev).manual_seed(9), device=dev)
    X = centers[lab] + 0.5 * torch.randn(m, d, generator=g, device=dev)
    res = {}
    for name, one_pass, dt in (("f64", False, torch.float64), ("f32_4", False, torch.float32),
                               ("f32_fused", True, torch.float32)):
        kern = ml.Gaussian(d, sigma=float(d) ** 0.5)
        s = ml.BlockADMMSolver("squared", "l2", 1e-3, 512, kernel=kern, NumFeaturePartitions=2, context=sk.Context(5))
        s.set_cache_transform(True)
        s.set_maxiter(6)
        s.one_pass = one_pass
        model = s.train(X.to(dt), lab.double(), regression=False, log=None, dtype=dt)
        res[name] = (model.coef.clone(), [h["objective"] for h in s.history])
    ref = res["f64"][0]
    e4 = float((res["f32_4"][0] - ref).norm() / ref.norm())
    ef = float((res["f32_fused"][0] - ref).norm() / ref.norm())
    assert ef <= 3 * e4 + 1e-6, (ef, e4)
    for a, b in zip(res["f64"][1], res["f32_fused"][1]):
        assert abs(a - b) <= 1e-3 * abs(a)


@pytest.mark.gpu
@pytest.mark.parametrize("cond", [1e4, 1e6])
def test_normal_form_lsqr_unpreconditioned_ill_conditioned(dev, cond):
    """the n-space recurrence of normal-form LSQR on an
    UNpreconditioned ill-conditioned A.  The default for an identity
    preconditioner is the classic form; the explicitly requested fused form
    (refreshed every 16 iterations) must still end at a residual within 1 %
    of the classic one and not report a better stop than classic."""
    g = torch.Generator().manual_seed(int(math.log10(cond)))
    m, n = 20000, 200
    U, _ = torch.linalg.qr(torch.randn(m, n, generator=g, dtype=torch.float64))
    Vq, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    s = torch.logspace(0, -math.log10(cond), n, dtype=torch.float64)
    A = ((U * s) @ Vq.t()).float().to(dev)
    b = (A @ torch.randn(n, 1, generator=g).to(dev)) + 1e-4 * torch.randn(m, 1, generator=g).to(dev)
    from libskylark_amd.algorithms import operators as O
    assert O.DenseOp(A).has_fused_normal(1)
    pd = K.KrylovIterParams(tolerance=1e-8, iter_lim=400)
    Xd, cd = K.lsqr(A, b, params=pd)
    pc = K.KrylovIterParams(tolerance=1e-8, iter_lim=400, fused_normal=False)
    Xc, cc = K.lsqr(A, b, params=pc)
    pf = K.KrylovIterParams(tolerance=1e-8, iter_lim=400, fused_normal=True)
    Xf, cf = K.lsqr(A, b, params=pf)
    # default == classic for the identity preconditioner
    assert torch.equal(Xd, Xc) and cd == cc
    rc = float((A @ Xc - b).norm())
    rf = float((A @ Xf - b).norm())
    assert rf <= 1.01 * rc, (rf, rc, cf, cc)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k,with_d", [(50000, 1024, 4, True), (50000, 1024, 4, False), (20000, 512, 2, True),
                                          (30000, 304, 1, True), (20003, 1000, 8, False), (4096, 16, 3, True)])
def test_pass_mfma_matches_fp64(m, n, k, with_d):
    """The fused pass's EXT form (rsvd_pass.hip sl_rsvd_pass_ext, BlockADMM's
    bf16-cache passes): Y = A X from X's bf16 hi / lo planes, W = A^T Y or
    A^T D with the long operand as bf16 hi + lo -- against fp64 products of the
    same bf16 A (partial last row block, n not a multiple of 32, k = 1..8)."""
    from libskylark_amd.ops import normal_eq as NE
    g = torch.Generator(device="cuda").manual_seed(m + n + k)
    A = (torch.randn(m, n, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    X = torch.randn(n, k, device="cuda", generator=g)
    D = None
    if with_d:
        Db = torch.randn(k, m, device="cuda", generator=g)
        D = Db.t()                       # column-major m x k, as BlockADMM's Dp.t()
    assert NE.mfma_ok(A, k, D)
    W, Y = NE.pass_mfma(A, X, D)
    Ad = A.double()
    Yr = Ad @ X.double()
    torch.testing.assert_close(Y.double(), Yr, rtol=0, atol=1e-5 * float((Ad.abs() @ X.double().abs()).max()))
    L = D.double() if with_d else Y.double()
    Wr = Ad.t() @ L
    tol = 3e-5 * float((Ad.abs().t() @ L.abs()).max())
    torch.testing.assert_close(W.double(), Wr, rtol=0, atol=tol)
