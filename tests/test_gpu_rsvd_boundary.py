"""The fused pass-boundary kernel of the randSVD engine (rsvd_core.hip
k_boundary, sl_rsvd_boundary) on a reduced [W; G] buffer: Gram + Cholesky
inverse + Z^T between passes, the fp64 core + V = W N after the last --
against fp64 numpy references of the same algebra (reference nla/svd.hpp:
71-149 re-orthonormalisation, :278-317 the core SVD); the replay contract
(ticket reset, generation advance, status store vs OR)."""
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
    return _lib


def _p(t):
    return vp(t.data_ptr()) if t is not None else None


def _graded(n, k, lo, hi, seed):
    g = np.random.RandomState(seed)
    Q1, _ = np.linalg.qr(g.randn(n, k))
    Q2, _ = np.linalg.qr(g.randn(k, k))
    return (Q1 * np.logspace(hi, lo, k)) @ Q2.T


@pytest.mark.parametrize("n,k", [(1000, 40), (64, 17), (1024, 48), (16, 1), (1000, 48)])
def test_boundary_inter(L, n, k):
    dev = torch.device("cuda")
    W = _graded(n, k, 0, 4, n + k)
    WG = torch.zeros((n + k) * k, dtype=torch.float64, device=dev)
    WG[: n * k] = torch.from_numpy(W.ravel()).to(dev)
    bws = torch.zeros(int(L.require().sl_rsvd_bnd_workspace(k)), dtype=torch.uint8, device=dev)
    Rinv = torch.empty(k, k, dtype=torch.float64, device=dev)
    Zt = torch.empty(k, n, dtype=torch.bfloat16, device=dev)
    st = torch.full((1,), 99, dtype=torch.int32, device=dev)
    s = vp(torch.cuda.current_stream().cuda_stream)
    for it in range(3):   # ticket reset / generation advance across launches
        L.call("sl_rsvd_boundary", 0, n, k, 0, _p(WG), _p(bws), _p(st), 0, _p(Rinv), _p(Zt),
               None, None, None, None, None, None, None, s)
    torch.cuda.synchronize()
    assert int(st[0]) == 0          # stored (status_or = 0), not OR-ed into 99
    sync = bws[:256].view(torch.int32).cpu().numpy()
    assert sync[0] == 0 and sync[16] == 3
    H = W.T @ W
    R = np.linalg.cholesky(H).T
    Ri = Rinv.cpu().numpy()
    assert np.abs(np.tril(Ri, -1)).max() == 0.0
    e_ref = np.abs(np.linalg.inv(R).T @ H @ np.linalg.inv(R) - np.eye(k)).max()
    # CholeskyQR: orthogonality to ~eps cond(H); a different (blocked) Gram
    # summation order than LAPACK moves it by a small factor
    assert np.abs(Ri.T @ H @ Ri - np.eye(k)).max() <= max(8 * e_ref, 1e-12)
    Zr = (W @ Ri).T
    np.testing.assert_allclose(Zt.double().cpu().numpy(), Zr, atol=8e-3 * np.abs(Zr).max())


@pytest.mark.parametrize("n,k,r", [(1000, 40, 20), (96, 17, 5), (512, 48, 48)])
def test_boundary_final(L, n, k, r):
    dev = torch.device("cuda")
    g = np.random.RandomState(k)
    W = _graded(n, k, -1, 4, 7 * k)
    Yg = g.randn(4 * k, k) @ np.diag(np.logspace(0, 2, k))
    Gy = Yg.T @ Yg
    WG = torch.zeros((n + k) * k, dtype=torch.float64, device=dev)
    WG[: n * k] = torch.from_numpy(W.ravel()).to(dev)
    WG[n * k:] = torch.from_numpy(Gy.ravel()).to(dev)
    bws = torch.zeros(int(L.require().sl_rsvd_bnd_workspace(k)), dtype=torch.uint8, device=dev)
    M = torch.empty(k, r, device=dev)
    N = torch.empty(k, r, dtype=torch.float64, device=dev)
    s64 = torch.empty(r, dtype=torch.float64, device=dev)
    st = torch.full((1,), 1, dtype=torch.int32, device=dev)
    V = torch.empty(n, r, device=dev)
    s32 = torch.empty(r, device=dev)
    s = vp(torch.cuda.current_stream().cuda_stream)
    for _ in range(2):
        L.call("sl_rsvd_boundary", 1, n, k, r, _p(WG), _p(bws), _p(st), 1, None, None,
               _p(M), _p(N), _p(s64), None, _p(V), _p(s32), None, s)
    torch.cuda.synchronize()
    assert int(st[0]) == 1, int(st[0])   # OR-ed into the preset pivot bit, nothing else
    Rt = np.linalg.cholesky(Gy).T
    Rti = np.linalg.inv(Rt)
    Cm = Rti.T @ (W.T @ W) @ Rti
    ev, Ub = np.linalg.eigh(0.5 * (Cm + Cm.T))
    ev, Ub = ev[::-1][:r], Ub[:, ::-1][:, :r]
    sv = s64.cpu().numpy()
    np.testing.assert_allclose(sv, np.sqrt(ev), rtol=1e-9, atol=1e-9 * np.sqrt(ev[0]))
    Mr = Rti @ Ub
    Mn = M.double().cpu().numpy()
    sg = np.sign(np.sum(Mn * Mr, axis=0))
    np.testing.assert_allclose(Mn * sg, Mr, atol=1e-5 * np.abs(Mr).max())
    # V = W N with the device N (its own column signs)
    Vr = W @ N.cpu().numpy()
    np.testing.assert_allclose(V.double().cpu().numpy(), Vr, atol=1e-6 * np.abs(Vr).max())
    np.testing.assert_allclose(s32.cpu().numpy(), sv.astype(np.float32))


def test_boundary_rejects_bad_shapes(L):
    from libskylark_amd.ops import _lib
    dev = torch.device("cuda")
    WG = torch.zeros(8, dtype=torch.float64, device=dev)
    bws = torch.zeros(int(L.require().sl_rsvd_bnd_workspace(4)), dtype=torch.uint8, device=dev)
    fn = _lib.require().sl_rsvd_boundary
    # n % 8 != 0, k > 48: refused before any launch
    assert fn(0, 20, 4, 0, _p(WG), _p(bws), None, 0, None, None, None, None, None, None,
              None, None, None, None) != 0
    assert fn(0, 64, 49, 0, _p(WG), _p(bws), None, 0, None, None, None, None, None, None,
              None, None, None, None) != 0
