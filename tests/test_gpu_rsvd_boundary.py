"""The fused pass-boundary kernel of the randSVD engine (rsvd_core.hip
k_boundary, sl_rsvd_boundary): slab reduce + Gram + Cholesky inverse + Z^T
between passes, and slab reduce + the fp64 core + V = W N after the last --
against fp64 numpy references of the same algebra (reference nla/svd.hpp:
71-149 re-orthonormalisation, :278-317 the core SVD), from the pass slabs
(single rank) and from an all-reduced [W; G] buffer (multi-rank form)."""
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
    _lib.register("sl_rsvd_pass_grid", [i64], C.c_int)
    _lib.register("sl_rsvd_pass_workspace", [i64, i64, i32], C.c_int64)
    _lib.register("sl_rsvd_boundary", [i32, vp, i64, i32, i32, i32, vp, vp, vp, i32, vp, vp, vp, vp, vp, i32,
                                       vp, vp, vp, vp, vp, vp, vp])
    return _lib


def _p(t):
    return vp(t.data_ptr()) if t is not None else None


def _graded(n, k, lo, hi, seed):
    g = np.random.RandomState(seed)
    Q1, _ = np.linalg.qr(g.randn(n, k))
    Q2, _ = np.linalg.qr(g.randn(k, k))
    return (Q1 * np.logspace(hi, lo, k)) @ Q2.T


def _slabs(L, m, n, k, W, Gy, seed):
    """A pass workspace whose W slabs sum to W and G slabs to Gy (f32 / f64
    parts; W's f32 rounding is returned as the exact sum)."""
    grid = int(L.require().sl_rsvd_pass_grid(m))
    nbytes = int(L.require().sl_rsvd_pass_workspace(m, n, k))
    ws = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    g = np.random.RandomState(seed)
    parts = (g.rand(grid, n, k) + 0.5)
    parts /= parts.sum(0, keepdims=True)
    Ws = (parts * W[None]).astype(np.float32)
    wv = ws[: grid * n * k * 4].view(torch.float32).view(grid, n, k)
    wv.copy_(torch.from_numpy(Ws))
    off = (grid * n * k * 4 + 255) & ~255
    gparts = g.rand(grid, k, k) + 0.5
    gparts /= gparts.sum(0, keepdims=True)
    Gs = gparts * Gy[None]
    gv = ws[off: off + grid * k * k * 8].view(torch.float64).view(grid, k, k)
    gv.copy_(torch.from_numpy(Gs))
    return ws, Ws.astype(np.float64).sum(0), Gs.sum(0), grid


@pytest.mark.parametrize("from_slabs", [True, False])
@pytest.mark.parametrize("n,k,m", [(1000, 40, 1_000_000), (64, 17, 800), (1024, 48, 50_000), (16, 1, 16)])
def test_boundary_inter(L, n, k, m, from_slabs):
    dev = torch.device("cuda")
    W = _graded(n, k, 0, 4, n + k)
    WG = torch.zeros((n + k) * k, dtype=torch.float64, device=dev)
    if from_slabs:
        ws, Wsum, _, _ = _slabs(L, m, n, k, W, np.eye(k), 5)
    else:
        ws, Wsum = None, W
        WG[: n * k] = torch.from_numpy(W.ravel()).to(dev)
    bws = torch.zeros(int(L.require().sl_rsvd_bnd_workspace(k)), dtype=torch.uint8, device=dev)
    Rinv = torch.empty(k, k, dtype=torch.float64, device=dev)
    Zt = torch.empty(k, n, dtype=torch.bfloat16, device=dev)
    st = torch.full((1,), 99, dtype=torch.int32, device=dev)
    s = vp(torch.cuda.current_stream().cuda_stream)
    for it in range(3):   # ticket reset / generation advance across launches
        L.call("sl_rsvd_boundary", 0, _p(ws), m, n, k, 0, _p(WG), _p(bws), _p(st), 0, _p(Rinv), _p(Zt),
               None, None, None, 0, None, None, None, None, None, None, s)
    torch.cuda.synchronize()
    assert int(st[0]) == 0          # stored (status_or = 0), not OR-ed into 99
    np.testing.assert_allclose(WG[: n * k].cpu().numpy().reshape(n, k), Wsum, rtol=1e-12, atol=1e-12 * np.abs(Wsum).max())
    sync = bws[:256].view(torch.int32).cpu().numpy()
    assert sync[0] == 0 and sync[16] == 3
    H = Wsum.T @ Wsum
    R = np.linalg.cholesky(H).T
    Ri = Rinv.cpu().numpy()
    assert np.abs(np.tril(Ri, -1)).max() == 0.0
    e_ref = np.abs(np.linalg.inv(R).T @ H @ np.linalg.inv(R) - np.eye(k)).max()
    # CholeskyQR: orthogonality to ~eps cond(H); a different (blocked) Gram
    # summation order than LAPACK moves it by a small factor
    assert np.abs(Ri.T @ H @ Ri - np.eye(k)).max() <= max(8 * e_ref, 1e-12)
    Zr = (Wsum @ Ri).T
    np.testing.assert_allclose(Zt.double().cpu().numpy(), Zr, atol=8e-3 * np.abs(Zr).max())


@pytest.mark.parametrize("from_slabs", [True, False])
@pytest.mark.parametrize("n,k,r,m", [(1000, 40, 20, 1_000_000), (96, 17, 5, 3000), (512, 48, 48, 20_000)])
def test_boundary_final(L, n, k, r, m, from_slabs):
    dev = torch.device("cuda")
    g = np.random.RandomState(k)
    W = _graded(n, k, -1, 4, 7 * k)
    Yg = g.randn(4 * k, k) @ np.diag(np.logspace(0, 2, k))
    Gy = Yg.T @ Yg
    WG = torch.zeros((n + k) * k, dtype=torch.float64, device=dev)
    if from_slabs:
        ws, Wsum, Gsum, _ = _slabs(L, m, n, k, W, Gy, 9)
    else:
        ws, Wsum, Gsum = None, W, Gy
        WG[: n * k] = torch.from_numpy(W.ravel()).to(dev)
        WG[n * k:] = torch.from_numpy(Gy.ravel()).to(dev)
    bws = torch.zeros(int(L.require().sl_rsvd_bnd_workspace(k)), dtype=torch.uint8, device=dev)
    M = torch.empty(k, r, device=dev)
    N = torch.empty(k, r, dtype=torch.float64, device=dev)
    s64 = torch.empty(r, dtype=torch.float64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    V = torch.empty(n, r, device=dev)
    s32 = torch.empty(r, device=dev)
    s = vp(torch.cuda.current_stream().cuda_stream)
    for _ in range(2):
        L.call("sl_rsvd_boundary", 1, _p(ws), m, n, k, r, _p(WG), _p(bws), _p(st), 1, None, None,
               _p(M), _p(N), _p(s64), 0, None, None, None, _p(V), _p(s32), None, s)
    torch.cuda.synchronize()
    assert int(st[0]) & ~1 == 0, int(st[0])
    np.testing.assert_allclose(WG[n * k:].cpu().numpy().reshape(k, k), Gsum, rtol=1e-12, atol=1e-12 * np.abs(Gsum).max())
    Rt = np.linalg.cholesky(Gsum).T
    Rti = np.linalg.inv(Rt)
    Cm = Rti.T @ (Wsum.T @ Wsum) @ Rti
    ev, Ub = np.linalg.eigh(0.5 * (Cm + Cm.T))
    ev, Ub = ev[::-1][:r], Ub[:, ::-1][:, :r]
    sv = s64.cpu().numpy()
    np.testing.assert_allclose(sv, np.sqrt(ev), rtol=1e-9, atol=1e-9 * np.sqrt(ev[0]))
    Mr = Rti @ Ub
    Mn = M.double().cpu().numpy()
    sg = np.sign(np.sum(Mn * Mr, axis=0))
    np.testing.assert_allclose(Mn * sg, Mr, atol=1e-5 * np.abs(Mr).max())
    # V = W N with the device N (its own column signs)
    Vr = Wsum @ N.cpu().numpy()
    np.testing.assert_allclose(V.double().cpu().numpy(), Vr, atol=1e-6 * np.abs(Vr).max())
    np.testing.assert_allclose(s32.cpu().numpy(), sv.astype(np.float32))
