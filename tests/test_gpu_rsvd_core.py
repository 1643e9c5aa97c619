"""Device small linear algebra of the randSVD engine (rsvd_core.hip) against
fp64 numpy references, through the pass-boundary kernel on an all-reduced
[W; G] buffer (sl_rsvd_boundary, the multi-rank form): the CholeskyQR
inverse between passes and the next pass operand, the fp64 core (Cholesky
of Y^T Y, C = Rt^-T H Rt^-1, tridiagonal eigensolver, factors), V = W N (sl_rsvd_make_v),
pivot dropping, numerically repeated core eigenvalues (Jacobi fallback)."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64


@pytest.fixture(scope="module")
def L():
    from libskylark_amd.ops import _lib
    _lib.require()
    _lib.register("sl_rsvd_bnd_workspace", [i32], C.c_int64)
    _lib.register("sl_rsvd_boundary", [i32, i32, i32, i32, vp, vp, vp, i32, vp, vp, vp, vp, vp,
                                       vp, vp, vp, vp, vp])
    _lib.register("sl_rsvd_make_v", [vp, i32, i32, i32, vp, i32, vp, vp, vp, vp])
    return _lib


def _p(t):
    return vp(t.data_ptr()) if t is not None else None


def _graded(n, k, lo, hi, seed):
    g = np.random.RandomState(seed)
    Q1, _ = np.linalg.qr(g.randn(n, k))
    Q2, _ = np.linalg.qr(g.randn(k, k))
    return (Q1 * np.logspace(hi, lo, k)) @ Q2.T


def _ws(L, k, dev):
    return torch.zeros(int(L.require().sl_rsvd_bnd_workspace(k)), dtype=torch.uint8, device=dev)


def _wg(W, Gy=None):
    n, k = W.shape
    WG = torch.zeros((n + k) * k, dtype=torch.float64, device="cuda")
    WG[: n * k] = torch.from_numpy(np.ascontiguousarray(W).ravel()).to("cuda")
    if Gy is not None:
        WG[n * k:] = torch.from_numpy(np.ascontiguousarray(Gy).ravel()).to("cuda")
    return WG


def _inter(L, WG, n, k, ws, Rinv, Zt, st, s):
    L.call("sl_rsvd_boundary", 0, n, k, 0, _p(WG), _p(ws), _p(st), 1, _p(Rinv), _p(Zt),
           None, None, None, None, None, None, None, s)


def _final(L, WG, n, k, r, ws, M, N, s64, st, s):
    L.call("sl_rsvd_boundary", 1, n, k, r, _p(WG), _p(ws), _p(st), 1, None, None,
           _p(M), _p(N), _p(s64), None, None, None, None, s)


@pytest.mark.parametrize("n,k", [(1000, 40), (64, 17), (1024, 48), (16, 1)])
def test_inter_la_is_cholesky_inverse(L, n, k):
    dev = torch.device("cuda")
    W = _graded(n, k, 0, 5, n + k)
    WG = _wg(W)
    ws = _ws(L, k, dev)
    Rinv = torch.empty(k, k, dtype=torch.float64, device=dev)
    Zt = torch.empty(k, n, dtype=torch.bfloat16, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    s = vp(torch.cuda.current_stream().cuda_stream)
    for _ in range(2):   # the ticket counter is reset for the next launch
        _inter(L, WG, n, k, ws, Rinv, Zt, st, s)
    torch.cuda.synchronize()
    assert int(st[0]) == 0
    Ri = Rinv.cpu().numpy()
    assert np.abs(np.tril(Ri, -1)).max() == 0.0
    H = W.T @ W
    R = np.linalg.cholesky(H).T
    # CholeskyQR loses ~eps cond(H) of orthogonality (cond(H) = 1e10 here):
    # hold the device factor to LAPACK's own residual, not to an absolute 1e-9
    e_ref = np.abs(np.linalg.inv(R).T @ H @ np.linalg.inv(R) - np.eye(k)).max()
    assert np.abs(Ri.T @ H @ Ri - np.eye(k)).max() <= max(4 * e_ref, 1e-12)
    np.testing.assert_allclose(Ri, np.linalg.inv(R), rtol=1e-5, atol=1e-6 * np.abs(Ri).max())
    # next pass operand: Z^T = (W R^-1)^T in bf16
    Zr = (W @ Ri).T
    np.testing.assert_allclose(Zt.double().cpu().numpy(), Zr, atol=8e-3 * np.abs(Zr).max())


def test_inter_la_drops_dependent_direction(L):
    dev = torch.device("cuda")
    n, k = 200, 12
    W = _graded(n, k, 0, 2, 3)
    W[:, 5] = W[:, 2] * 2.0          # exactly dependent column
    WG = _wg(W)
    ws = _ws(L, k, dev)
    Rinv = torch.empty(k, k, dtype=torch.float64, device=dev)
    Zt = torch.empty(k, n, dtype=torch.bfloat16, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    _inter(L, WG, n, k, ws, Rinv, Zt, st, vp(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert int(st[0]) & 1
    Ri = Rinv.cpu().numpy()
    assert np.abs(Ri[:, 5]).max() == 0.0
    Q = W @ Ri
    keep = [j for j in range(k) if j != 5]
    np.testing.assert_allclose(Q[:, keep].T @ Q[:, keep], np.eye(k - 1), atol=1e-8)


@pytest.mark.parametrize("n,k,r", [(1000, 40, 20), (96, 17, 5), (512, 48, 48)])
def test_final_la_matches_fp64_core(L, n, k, r):
    dev = torch.device("cuda")
    g = np.random.RandomState(k)
    W = _graded(n, k, -1, 4, 7 * k)
    Yg = g.randn(4 * k, k) @ np.diag(np.logspace(0, 2, k))
    Gy = Yg.T @ Yg
    Wd, WG = torch.from_numpy(W).to(dev), _wg(W, Gy)
    ws = _ws(L, k, dev)
    M = torch.empty(k, r, device=dev)
    N = torch.empty(k, r, dtype=torch.float64, device=dev)
    s64 = torch.empty(r, dtype=torch.float64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    s = vp(torch.cuda.current_stream().cuda_stream)
    # reference: C = Rt^-T H Rt^-1, eigenpairs descending
    Rt = np.linalg.cholesky(Gy).T
    Rti = np.linalg.inv(Rt)
    Cm = Rti.T @ (W.T @ W) @ Rti
    ev, Ub = np.linalg.eigh(0.5 * (Cm + Cm.T))
    ev, Ub = ev[::-1][:r], Ub[:, ::-1][:, :r]
    outs = []
    for _ in range(3):   # replays: the worker count / consumed count handshake advances
        _final(L, WG, n, k, r, ws, M, N, s64, st, s)
        torch.cuda.synchronize()
        assert int(st[0]) & ~1 == 0, int(st[0])
        sv = s64.cpu().numpy()
        np.testing.assert_allclose(sv, np.sqrt(ev), rtol=1e-9, atol=1e-9 * np.sqrt(ev[0]))
        # M = Rt^-1 Ub_r up to column signs
        Mr = Rti @ Ub
        Mn = M.double().cpu().numpy()
        sg = np.sign(np.sum(Mn * Mr, axis=0))
        np.testing.assert_allclose(Mn * sg, Mr, atol=1e-5 * np.abs(Mr).max())
        # N = M S^-1: columns of well-resolved values (sigma >= 1e-3 sigma_1),
        # each to its own scale (the trailing ones of a cond-1e5 core are not
        # determined to 1e-5 by any fp64 eigensolver)
        Nr, Nn = Mr / np.sqrt(ev), N.cpu().numpy() * sg
        for c in np.nonzero(np.sqrt(ev) >= 1e-3 * np.sqrt(ev[0]))[0]:
            np.testing.assert_allclose(Nn[:, c], Nr[:, c], atol=1e-5 * np.abs(Nr[:, c]).max())
        outs.append(sv)
    # V = W N
    Vt = torch.empty(n, r, device=dev)
    s32 = torch.empty(r, device=dev)
    L.call("sl_rsvd_make_v", _p(Wd), n, k, k, _p(N), r, _p(Vt), _p(s64), _p(s32), s)
    torch.cuda.synchronize()
    Vr = W @ N.cpu().numpy()
    np.testing.assert_allclose(Vt.double().cpu().numpy(), Vr, atol=1e-6 * np.abs(Vr).max())
    np.testing.assert_allclose(s32.cpu().numpy(), outs[-1].astype(np.float32))


def test_final_core_repeated_eigenvalues_fall_back_to_jacobi(L):
    """A core with an exactly repeated top eigenvalue (equal singular values)
    defeats the twisted factorisation; the boundary re-solves it by Jacobi and
    still returns an orthonormal basis of the eigenspace."""
    dev = torch.device("cuda")
    n, k, r = 256, 16, 8
    g = np.random.RandomState(3)
    Q1, _ = np.linalg.qr(g.randn(n, k))
    Q2, _ = np.linalg.qr(g.randn(k, k))
    sv = np.array([5.0] * 4 + list(np.linspace(3, 1, k - 4)))
    W = (Q1 * sv) @ Q2.T              # W^T W = Q2 diag(sv^2) Q2^T: 4-fold repeated top eigenvalue
    Gy = np.eye(k)
    WG = _wg(W, Gy)
    ws = _ws(L, k, dev)
    M = torch.empty(k, r, device=dev)
    N = torch.empty(k, r, dtype=torch.float64, device=dev)
    s64 = torch.empty(r, dtype=torch.float64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    _final(L, WG, n, k, r, ws, M, N, s64, st, vp(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    np.testing.assert_allclose(s64.cpu().numpy(), sv[:r], rtol=1e-10)
    Mn = M.double().cpu().numpy()        # Rt = I: M = Ub_r, orthonormal columns
    np.testing.assert_allclose(Mn.T @ Mn, np.eye(r), atol=1e-6)
    C = W.T @ W
    np.testing.assert_allclose(C @ Mn, Mn * (s64.cpu().numpy() ** 2), atol=1e-5 * 25)
