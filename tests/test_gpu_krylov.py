"""Native Krylov vector kernels (krylov_kernels.hip) vs torch fp64 references,
and the device-scalar LSQR against the torch-op LSQR on the same problem."""
import math

import pytest
import torch

from libskylark_amd.algorithms import krylov as K
from libskylark_amd.ops import krylov_native as kn


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,dt", [(100003, 1, torch.float32), (5000, 3, torch.float64), (777, 40, torch.float32),
                                    (1, 64, torch.float64), (65536, 17, torch.float32)])
def test_colsumsq_coldot_axpby(dev, m, k, dt):
    g = torch.Generator().manual_seed(m + k)
    X = torch.randn(m, k, generator=g, dtype=torch.float64)
    Y = torch.randn(m, k, generator=g, dtype=torch.float64)
    Xd, Yd = X.to(dev, dt), Y.to(dev, dt)
    tol = 1e-5 if dt == torch.float32 else 1e-12
    ref = (Xd.double() ** 2).sum(0)
    assert torch.allclose(kn.colsumsq(Xd), ref, rtol=tol)
    assert torch.allclose(kn.coldot(Xd, Yd), (Xd.double() * Yd.double()).sum(0), rtol=tol, atol=tol * m)
    a = torch.randn(k, generator=g, dtype=torch.float64).to(dev)
    b = torch.randn(k, generator=g, dtype=torch.float64).to(dev)
    want = (a * Xd.double() + b * Yd.double())
    s2 = kn.axpby_colsumsq(Xd, Yd, a, b)
    assert torch.allclose(Yd.double(), want, rtol=tol, atol=tol)
    assert torch.allclose(s2, (Yd.double() ** 2).sum(0), rtol=tol)
    kn.colscale(Yd, s2.sqrt(), inv=True)
    assert torch.allclose(Yd.double().norm(dim=0), torch.ones(k, dtype=torch.float64, device=dev), rtol=1e-4)
    # strided view (column slice of a wider matrix)
    Wd = torch.randn(m, k + 5, device=dev, dtype=dt)[:, 2:2 + k]
    assert torch.allclose(kn.colsumsq(Wd), (Wd.double() ** 2).sum(0), rtol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
def test_native_lsqr_matches_torch_lsqr(dev, fused):
    from libskylark_amd.algorithms.regression import _build_precond
    g = torch.Generator().manual_seed(11)
    m, n, k = 30000, 200, 2
    A = (torch.randn(m, n, generator=g) * torch.logspace(0, -3, n)).to(dev)
    B = torch.randn(m, k, generator=g).to(dev)
    S = torch.randn(4 * n, m, generator=g).to(dev) / math.sqrt(4 * n)
    P, _ = _build_precond(S @ A, "qr")
    p = K.KrylovIterParams(tolerance=1e-6, iter_lim=100, fused_normal=fused, check_every=4)
    Xn, cn = K.lsqr(A, B, params=p, R=P)
    kn.ENABLED = False
    try:
        Xt, ct = K.lsqr(A, B, params=p, R=P)
    finally:
        kn.ENABLED = True
    assert cn in (-2, -3) and ct in (-2, -3)
    rn = (A @ Xn - B).norm() / B.norm()
    rt = (A @ Xt - B).norm() / B.norm()
    assert abs(float(rn / rt) - 1) < 1e-4
    assert float((Xn - Xt).norm() / Xt.norm()) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("nr,nc,k,dt", [(1000, 1000, 1, torch.float32), (5000, 5000, 2, torch.float32),
                                        (333, 777, 5, torch.float64), (64, 3, 8, torch.float32)])
def test_thin_gemm(dev, nr, nc, k, dt):
    g = torch.Generator().manual_seed(nr + k)
    M = torch.randn(nr, nc, generator=g, dtype=torch.float64)
    X = torch.randn(nc, k, generator=g, dtype=torch.float64)
    Md, Xd = M.to(dev, dt), X.to(dev, dt)
    assert kn.thin_gemm_ok(Md, Xd)
    Y = kn.thin_gemm(Md, Xd)
    ref = Md.double() @ Xd.double()
    tol = 1e-6 if dt == torch.float32 else 1e-13
    assert float((Y.double() - ref).norm() / ref.norm()) < tol


@pytest.mark.gpu
def test_dense_operator_native_products(dev):
    from libskylark_amd.algorithms.operators import DenseOp
    g = torch.Generator().manual_seed(2)
    A = torch.randn(50001, 700, generator=g)
    X = torch.randn(700, 3, generator=g)
    Yv = torch.randn(50001, 3, generator=g)
    op = DenseOp(A.to(dev))
    AX = op.matmul(X.to(dev)).double().cpu()
    AtY = op.rmatmul(Yv.to(dev)).double().cpu()
    assert float((AX - A.double() @ X.double()).norm() / AX.norm()) < 1e-5
    assert float((AtY - A.double().t() @ Yv.double()).norm() / AtY.norm()) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,density,k,vdt", [(20000, 3000, 5e-4, 1, torch.float32), (5000, 8000, 0.01, 3, torch.float64),
                                               (1000, 500, 0.2, 20, torch.float32), (77, 33, 0.3, 40, torch.float64)])
def test_csr_spmm_and_sparse_operator(dev, m, n, density, k, vdt):
    from libskylark_amd.algorithms.operators import SparseOp
    from libskylark_amd.ops import spmm
    g = torch.Generator().manual_seed(m + k)
    nnz = max(1, int(m * n * density))
    idx = torch.stack([torch.randint(0, m, (nnz,), generator=g), torch.randint(0, n, (nnz,), generator=g)])
    A = torch.sparse_coo_tensor(idx, torch.randn(nnz, generator=g, dtype=torch.float64), (m, n)).coalesce()
    Ad = A.to_dense()
    Acsr = A.to(vdt).to_sparse_csr().to(dev)
    X = torch.randn(n, k, generator=g, dtype=torch.float64)
    Yv = torch.randn(m, k, generator=g, dtype=torch.float64)
    tol = 1e-5 if vdt == torch.float32 else 1e-12
    got = spmm.csr_mm(Acsr, X.to(dev)).double().cpu()
    assert float((got - Ad @ X).norm() / (Ad @ X).norm()) < tol
    op = SparseOp(Acsr)
    got_t = op.rmatmul(Yv.to(dev)).double().cpu()
    assert float((got_t - Ad.t() @ Yv).norm() / (Ad.t() @ Yv).norm()) < tol


def _spd(n, k, dt, dev, seed):
    g = torch.Generator().manual_seed(seed)
    Q, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    A = (Q * torch.logspace(0, 3, n, dtype=torch.float64)) @ Q.t()
    B = torch.randn(n, k, generator=g, dtype=torch.float64)
    return A.to(dev, dt), B.to(dev, dt)


@pytest.mark.gpu
@pytest.mark.parametrize("dt,k,precond,flexible", [(torch.float64, 3, False, False), (torch.float64, 1, True, False),
                                                   (torch.float32, 40, False, False), (torch.float64, 2, True, True),
                                                   (torch.float64, 5, False, True)])
def test_native_cg_matches_torch_cg(dev, dt, k, precond, flexible):
    """Device-scalar (flexible) CG (sl_cg_*: last-block reductions, no host
    sync but the stop flags) against the torch-op iteration on the same SPD
    system (reference algorithms/Krylov/CG.hpp:24-163, FlexibleCG.hpp)."""
    n = 600
    A, B = _spd(n, k, dt, dev, 7 + k)
    M = K.MatPrecond(torch.diag(1.0 / torch.diagonal(A))) if precond else None
    tol = 1e-10 if dt == torch.float64 else 1e-4
    p = K.KrylovIterParams(tolerance=tol, iter_lim=3000, check_every=5)
    f = K.flexible_cg if flexible else K.cg
    Xn, cn = f(A, B, params=p, M=M)
    kn.ENABLED = False
    try:
        Xt, ct = f(A, B, params=p, M=M)
    finally:
        kn.ENABLED = True
    assert cn == -1 and ct == -1
    rn = ((A.double() @ Xn.double() - B.double()).norm(dim=0) / B.double().norm(dim=0)).max()
    assert float(rn) < (1e-9 if dt == torch.float64 else 5e-3)
    assert float((Xn.double() - Xt.double()).norm() / Xt.double().norm()) < (1e-7 if dt == torch.float64 else 1e-2)
