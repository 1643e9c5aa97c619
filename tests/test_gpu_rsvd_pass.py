"""The fused bf16 randSVD pass (rsvd_pass.hip) against fp64 torch references
of the same op: y = A Z, W = A^T y' and, in the last pass (final = 1), the
stored Y = y' (the bf16 hi + lo pair of y) and its fp64 Gram formed in-pass
from exact bf16 products.  Ragged row counts exercise the clamped last block;
k in {8, 20, 40} covers one, two and three 16-column tiles."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64


@pytest.fixture(scope="module")
def L():
    from libskylark_amd.ops import _lib
    _lib.require()
    _lib.register("sl_rsvd_pass", [vp, i64, i64, i64, vp, i32, vp, vp, i64, i32, i32, vp])
    _lib.register("sl_rsvd_pass_workspace", [i64, i64, i32], C.c_int64)
    _lib.register("sl_rsvd_reduce", [vp, i64, i64, i32, vp, i32, i32, vp, i32, vp])
    return _lib


@pytest.mark.parametrize("m,n,k", [(100_003, 1000, 40), (70_001, 512, 20), (33_333, 256, 8), (4_097, 1000, 40),
                                   (257, 1024, 48), (9_999, 520, 33), (100, 16, 1)])
@pytest.mark.parametrize("final", [0, 1, 2])
@pytest.mark.parametrize("variant", [0, 256])
def test_pass_matches_fp64(L, m, n, k, final, variant, ldy_pad=0):
    """variant 0: the pass walking row blocks forward; 256: backwards (the
    engine's odd passes, MALL reuse)."""
    if variant == 256 and (m, n, k) not in ((100_003, 1000, 40), (4_097, 1000, 40), (9_999, 520, 33)):
        pytest.skip("reverse walk on a subset of shapes")
    _run_pass(L, m, n, k, final, variant, ldy_pad)


def test_pass_strided_y(L):
    """ldy != k: the stored Y goes out as 4-B elements (not float4 rows)."""
    _run_pass(L, 20_011, 1000, 40, 1, 0, 5)


def _run_pass(L, m, n, k, final, variant, ldy_pad):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(m + k)
    A = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16)
    # a graded Z: y columns of very different scale (the Gram's dynamic range)
    Q, _ = torch.linalg.qr(torch.randn(n, k, device=dev, dtype=torch.float64, generator=g))
    Zt = (Q * torch.logspace(0, -3, k, device=dev, dtype=torch.float64)).t().contiguous().to(torch.bfloat16)
    ws = torch.zeros(int(L.require().sl_rsvd_pass_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    W = torch.empty(n, k, device=dev, dtype=torch.float64)
    G = torch.zeros(k, k, device=dev, dtype=torch.float64)
    Yfull = torch.full((m, k + ldy_pad), float("nan"), device=dev)
    Y = Yfull[:, :k]
    st = vp(torch.cuda.current_stream().cuda_stream)
    L.call("sl_rsvd_pass", vp(A.data_ptr()), m, n, n, vp(Zt.data_ptr()), k, vp(ws.data_ptr()),
           vp(Y.data_ptr()) if final else None, k + ldy_pad, final, variant, st)
    L.call("sl_rsvd_reduce", vp(ws.data_ptr()), m, n, k, vp(W.data_ptr()), 1, k,
           vp(G.data_ptr()) if final == 1 else None, k, st)
    torch.cuda.synchronize()

    Ad, Zd = A.double(), Zt.double().t()
    y = Ad @ Zd
    # y: f32 MFMA sums of exact bf16 products
    mag = A.double().abs() @ Zd.abs()
    if final:
        assert torch.isfinite(Y).all()
        if ldy_pad:
            assert torch.isnan(Yfull[:, k:]).all()   # the padding columns are never written
        # Y = bf16 hi + lo pair of the f32 y: within 2^-16 |y| of y
        assert ((Y.double() - y).abs() <= 2.0 ** -16 * y.abs() + 2e-6 * mag).all()
        Yd = Y.double()
    else:
        Yd = y
    # W = A^T y' with y' the stored pair (f32 accumulation over m rows)
    Wref = Ad.t() @ (Yd if final else y)
    wmag = Ad.abs().t() @ Yd.abs()
    assert ((W - Wref).abs() <= 5e-5 * wmag + 1e-30).all(), float(((W - Wref).abs() / wmag).max())
    if final == 1:
        Gref = Yd.t() @ Yd
        d = Gref.diagonal().sqrt()
        rel = ((G - Gref).abs() / torch.outer(d, d)).max().item()
        # per 16-row block the 64 exact products are summed in f32 (2^-24
        # relative to the block's sum of |products|), blocks in f64: bounded by
        # ~2^-23 sqrt(G_ii G_jj), far below that for many blocks
        assert rel < 1.2e-7, rel
        if m > 50_000:
            assert rel < 1e-8, rel
        assert torch.equal(G, G.t())
