"""GPU-resident small linear algebra (k <= 64; the Cholesky inverse to k = 128) vs fp64 torch references."""
import math
import pytest
import torch

from libskylark_amd.ops import small_la as SL

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k", [1, 7, 16, 17, 33, 40, 48, 64])
def test_chol_inv(dev, k):
    X = torch.randn(3 * k + 5, k, dtype=torch.float64)
    G = X.t() @ X
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    R, Ri, Ri32 = SL.chol_inv(G.to(dev), st)
    assert int(st) == 0
    Rr = torch.linalg.cholesky(G).t()
    torch.testing.assert_close(R.cpu(), Rr, rtol=1e-10, atol=1e-10)
    torch.testing.assert_close(Ri.cpu() @ Rr, torch.eye(k, dtype=torch.float64), rtol=1e-9, atol=1e-9)
    torch.testing.assert_close(Ri32.cpu().double(), Ri.cpu(), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("k", [1, 7, 16, 17, 33, 40, 41, 48, 64, 65, 96, 97, 120, 128])
def test_chol_inv_wave(dev, k):
    """One-wave register Cholesky inverse (the randSVD boundary kernel) vs
    LAPACK: R^{-1} R = I to the attainable ~eps cond(G)."""
    g = torch.Generator().manual_seed(k)
    X = torch.randn(3 * k + 5, k, generator=g, dtype=torch.float64) @ torch.diag(torch.logspace(0, 3, k,
                                                                                               dtype=torch.float64))
    G = X.t() @ X
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    Ri = SL.chol_inv_wave(G.to(dev), st).cpu()
    assert int(st) == 0
    Rr = torch.linalg.cholesky(G).t()
    assert float(torch.tril(Ri, -1).abs().max()) == 0.0
    e_ref = float((torch.linalg.inv(Rr).t() @ G @ torch.linalg.inv(Rr) - torch.eye(k, dtype=torch.float64)).abs().max())
    e = float((Ri.t() @ G @ Ri - torch.eye(k, dtype=torch.float64)).abs().max())
    assert e <= max(8 * e_ref, 1e-12), (e, e_ref)
    torch.testing.assert_close(Ri, torch.linalg.inv(Rr), rtol=1e-8, atol=1e-8 * float(Ri.abs().max()))


@pytest.mark.parametrize("k,dep", [(12, 5), (100, 77)])
def test_chol_inv_wave_drops_dependent_direction(dev, k, dep):
    g = torch.Generator().manual_seed(3)
    W = torch.randn(400, k, generator=g, dtype=torch.float64)
    W[:, dep] = 2.0 * W[:, 2]
    G = W.t() @ W
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    Ri = SL.chol_inv_wave(G.to(dev), st).cpu()
    assert int(st) & 1
    assert float(Ri[:, dep].abs().max()) == 0.0 and float(Ri[dep, :].abs().max()) == 0.0
    Q = W @ Ri
    keep = [j for j in range(k) if j != dep]
    torch.testing.assert_close(Q[:, keep].t() @ Q[:, keep], torch.eye(k - 1, dtype=torch.float64), atol=1e-8, rtol=0)


def test_chol_inv_flags_breakdown(dev):
    G = torch.zeros(5, 5, dtype=torch.float64, device=dev)
    G[0, 0] = 1
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    SL.chol_inv(G, st)
    assert int(st) == 1


@pytest.mark.parametrize("n,k", [(1000, 40), (64, 64), (300, 3)])
def test_cholqr2_device(dev, n, k):
    W = torch.randn(n, k, device=dev) @ torch.diag(torch.logspace(0, 2, k, device=dev))
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    Q, R = SL.cholqr2(W, st, want_r=True)
    assert int(st) == 0
    torch.testing.assert_close(Q.double().t() @ Q.double(), torch.eye(k, dtype=torch.float64, device=dev),
                               atol=2e-6, rtol=0)
    torch.testing.assert_close(Q.double() @ R, W.double(), rtol=1e-5, atol=1e-4 * float(W.abs().max()))


def test_small_matmul(dev):
    A = torch.randn(33, 17, dtype=torch.float64, device=dev)
    B = torch.randn(17, 9, dtype=torch.float64, device=dev)
    C, C32 = SL.small_matmul(A, B, want32=True)
    torch.testing.assert_close(C, A @ B)
    torch.testing.assert_close(C32, (A @ B).float())


@pytest.mark.parametrize("k,r", [(40, 20), (7, 3), (64, 64), (48, 10)])
@pytest.mark.parametrize("spread", [1.0, 1e-12])
def test_sym_eig_topr_vs_lapack(dev, k, r, spread):
    g = torch.Generator().manual_seed(k)
    Q, _ = torch.linalg.qr(torch.randn(k, k, generator=g, dtype=torch.float64))
    lam = torch.logspace(0, math.log10(spread), k, dtype=torch.float64) if spread != 1.0 else \
        torch.rand(k, generator=g, dtype=torch.float64) + 0.1
    C = (Q * lam) @ Q.t()
    out = SL.sym_eig_topr(C.to(dev), r, sqrt=True).cpu()
    V, s = out[:k * r].view(k, r), out[k * r:]
    ref = torch.sort(torch.linalg.eigvalsh(C), descending=True).values[:r]
    # backward stable: |lambda - lambda_lapack| ~ eps * ||C||
    assert ((s * s - ref).abs().max() / lam.max()) < 1e-13, (s * s - ref).abs().max()
    # eigenvector residuals
    res = (C @ V - V * (s * s)).norm(dim=0) / lam.max()
    assert res.max() < 1e-10
    assert torch.allclose(V.t() @ V, torch.eye(r, dtype=torch.float64), atol=1e-10)


def test_sym_eig_repeated_eigenvalues(dev):
    k = 32
    C = torch.diag(torch.tensor([2.0] * 16 + [1.0] * 16, dtype=torch.float64))
    g = torch.Generator().manual_seed(0)
    Q, _ = torch.linalg.qr(torch.randn(k, k, generator=g, dtype=torch.float64))
    C = Q @ C @ Q.t()
    out = SL.sym_eig_topr(C.to(dev), 20).cpu()
    lam = out[k * 20:]
    assert torch.allclose(lam[:16], torch.full((16,), 2.0, dtype=torch.float64), atol=1e-12)
    assert torch.allclose(lam[16:], torch.full((4,), 1.0, dtype=torch.float64), atol=1e-12)


def test_sym_eig_converges_in_few_sweeps(dev):
    k = 40
    g = torch.Generator().manual_seed(3)
    X = torch.randn(1000, k, generator=g, dtype=torch.float64)
    C = X.t() @ X
    sweeps = torch.zeros(1, dtype=torch.int32, device=dev)
    SL.sym_eig_topr(C.to(dev), 20, sweeps=sweeps)
    assert 2 <= int(sweeps.item()) <= 12


def _eig_check(C, out, k, r):
    V, lam = out[:k * r].view(k, r), out[k * r:]
    ref = torch.sort(torch.linalg.eigvalsh(C), descending=True).values[:r]
    nrm = float(torch.linalg.eigvalsh(C).abs().max())
    assert float((lam - ref).abs().max()) / nrm < 4e-13, (lam - ref).abs().max()
    res = (C @ V - V * lam).norm(dim=0) / nrm
    assert float(res.max()) < 1e-10, res.max()
    assert torch.allclose(V.t() @ V, torch.eye(r, dtype=torch.float64), atol=1e-10)


@pytest.mark.parametrize("k,r", [(40, 20), (7, 3), (64, 32), (48, 10), (2, 1), (1, 1), (3, 3), (33, 32), (40, 40),
                                 (64, 64), (17, 16)])
@pytest.mark.parametrize("kind", ["uniform", "logspace", "planted", "gram", "indefinite"])
def test_sym_eig_tridiag_vs_lapack(dev, k, r, kind):
    """Device tridiagonal eigensolver (Householder + multisection + twisted
    factorisation) against LAPACK: eigenvalues to eps ||C||, residuals,
    orthogonality, and no host-fallback flag on well-separated spectra."""
    g = torch.Generator().manual_seed(k * 7 + r)
    Q, _ = torch.linalg.qr(torch.randn(k, k, generator=g, dtype=torch.float64))
    if kind == "uniform":
        lam = torch.rand(k, generator=g, dtype=torch.float64) + 0.1
    elif kind == "logspace":
        lam = torch.logspace(0, -12, k, dtype=torch.float64)
    elif kind == "planted":
        lam = (1000.0 * 0.9 ** torch.arange(k, dtype=torch.float64)) ** 2
    elif kind == "indefinite":
        lam = torch.randn(k, generator=g, dtype=torch.float64) * 3
    else:
        X = torch.randn(1000, k, generator=g, dtype=torch.float64)
        C = X.t() @ X
        lam = None
    if lam is not None:
        C = (Q * lam) @ Q.t()
        C = 0.5 * (C + C.t())
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    out = SL.sym_eig_tridiag(C.to(dev), r, status=st).cpu()
    assert int(st.item()) == 0
    _eig_check(C, out, k, r)
    # sqrt packing as the randSVD plan consumes it
    out2 = SL.sym_eig_tridiag(C.to(dev), r, sqrt=True).cpu()
    lam2 = out[k * r:]
    torch.testing.assert_close(out2[k * r:], lam2.clamp_min(0).sqrt(), rtol=4e-16, atol=0)


def test_sym_eig_tridiag_close_cluster(dev):
    """Relative gaps 1e-6 inside the top block: re-orthogonalised, no fallback."""
    k, r = 40, 20
    g = torch.Generator().manual_seed(5)
    Q, _ = torch.linalg.qr(torch.randn(k, k, generator=g, dtype=torch.float64))
    lam = torch.linspace(10, 1, k, dtype=torch.float64)
    lam[3:6] = torch.tensor([7.11, 7.11 - 1e-6 * 10, 7.11 - 2e-6 * 10], dtype=torch.float64)
    C = (Q * lam) @ Q.t()
    C = 0.5 * (C + C.t())
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    out = SL.sym_eig_tridiag(C.to(dev), r, status=st).cpu()
    assert int(st.item()) == 0
    V, lv = out[:k * r].view(k, r), out[k * r:]
    assert torch.allclose(V.t() @ V, torch.eye(r, dtype=torch.float64), atol=1e-10)
    ref = torch.sort(torch.linalg.eigvalsh(C), descending=True).values[:r]
    assert float((lv - ref).abs().max()) < 1e-12 * 10
    # the cluster's invariant subspace is right even if its basis is not LAPACK's
    res = (C @ V - V * lv).norm(dim=0) / 10
    assert float(res.max()) < 1e-8


@pytest.mark.parametrize("case", ["repeated", "low_rank", "nan"])
def test_sym_eig_tridiag_flags_host_fallback(dev, case):
    k, r = 32, 20
    g = torch.Generator().manual_seed(9)
    Q, _ = torch.linalg.qr(torch.randn(k, k, generator=g, dtype=torch.float64))
    if case == "repeated":
        lam = torch.tensor([2.0] * 16 + [1.0] * 16, dtype=torch.float64)
    else:
        lam = torch.cat([torch.linspace(5, 1, 10, dtype=torch.float64), torch.zeros(k - 10, dtype=torch.float64)])
    C = (Q * lam) @ Q.t()
    if case == "nan":
        C = (Q * (torch.rand(k, generator=g, dtype=torch.float64) + 1)) @ Q.t()
        C[3, 4] = float("nan")
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    SL.sym_eig_tridiag(C.to(dev), r, status=st, sqrt=True)
    assert int(st.item()) & 1
