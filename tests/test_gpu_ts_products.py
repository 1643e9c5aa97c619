"""Hand-written tall-skinny products of the general-precision randSVD engine
(rsvd_stream.hip) against fp64 torch references of the same ops:
Y = A Z and W = A^T Q in A's precision (f32 / f64 matrix cores; f32 Y = A Z
with 16 < k <= 48 on the exact three-plane bf16 split), the f64
helpers X M, X^T X and the one-workgroup k x k product.  Ragged shapes cover
partial row blocks / row quads, n not a multiple of the column group, lda > n
and an lda that rules out 16-B vector loads (scalar path)."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
F32, F64 = 0, 1   # SL_F32 / SL_F64 (sl_common.hpp SlDtype)


@pytest.fixture(scope="module")
def L():
    from libskylark_amd.ops import _lib
    _lib.require()
    _lib.register("sl_ts_az", [vp, i64, i64, i64, vp, i32, vp, i64, i32, vp])
    _lib.register("sl_ts_atq_workspace", [i64, i64, i32, i32], C.c_int64)
    _lib.register("sl_ts_atq", [vp, i64, i64, i64, vp, i32, vp, i32, vp, i32, vp])
    _lib.register("sl_ts_xm64", [vp, i64, i32, i64, vp, i32, vp, i64, i32, vp])
    _lib.register("sl_ts_gram64_workspace", [i64, i32], C.c_int64)
    _lib.register("sl_ts_gram64", [vp, i64, i32, i64, vp, i32, vp, vp])
    _lib.register("sl_ts_small", [i32, i32, i32, i32, i32, vp, i32, vp, i32, vp, i32, vp])
    _lib.register("sl_ts_gram_w", [vp, i32, i64, i32, i64, vp, i32, vp, vp])
    return _lib


def _st():
    return vp(torch.cuda.current_stream().cuda_stream)


# (300_007, 200, 24, 4): whole-block rounds then the stream-K tail of k_ts_az
SHAPES = [(100_003, 1000, 40, 0), (4_097, 1000, 40, 8), (777, 37, 20, 0), (129, 16, 1, 0), (2_500, 530, 64, 3),
          (20_000, 5000, 40, 0), (64, 2049, 33, 0), (300_007, 200, 24, 4),
          # 64 < k <= 128: six / eight column tiles (512-thread az, one vector per wave in atq)
          (50_001, 1000, 128, 0), (3_001, 530, 65, 3), (20_000, 5000, 96, 0), (7_777, 300, 111, 4)]


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("m,n,k,pad", SHAPES)
def test_az_and_atq(L, dt, m, n, k, pad):
    if dt == torch.float32 and n == 5000 and m > 10_000:
        m = 5_000
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(m + n + k)
    lda = n + pad
    Afull = torch.randn(m, lda, device=dev, dtype=dt, generator=g)
    A = Afull[:, :n]
    Z = torch.randn(n, k, device=dev, dtype=dt, generator=g)
    Y = torch.full((m, k), float("nan"), device=dev, dtype=dt)
    code = F32 if dt == torch.float32 else F64
    L.call("sl_ts_az", vp(Afull.data_ptr()), m, n, lda, vp(Z.data_ptr()), k, vp(Y.data_ptr()), k, code, _st())
    Q = torch.randn(m, k, device=dev, dtype=dt, generator=g)
    ws = torch.zeros(int(L.require().sl_ts_atq_workspace(m, n, k, code)), dtype=torch.uint8, device=dev)
    W = torch.full((n, k), float("nan"), device=dev, dtype=torch.float64)
    L.call("sl_ts_atq", vp(Afull.data_ptr()), m, n, lda, vp(Q.data_ptr()), k, vp(W.data_ptr()), k,
           vp(ws.data_ptr()), code, _st())
    torch.cuda.synchronize()
    Ad = A.double()
    eps = 1.2e-7 if dt == torch.float32 else 2.3e-16
    yref = Ad @ Z.double()
    ymag = Ad.abs() @ Z.double().abs()
    assert torch.isfinite(Y).all()
    # one f32 / f64 rounding per product in a k-ordered chain: |err| <= ~n eps sum|a b|
    assert ((Y.double() - yref).abs() <= 4 * eps * (n ** 0.5 + 4) * ymag + 1e-300).all(), \
        float(((Y.double() - yref).abs() / ymag).max())
    wref = Ad.t() @ Q.double()
    wmag = Ad.abs().t() @ Q.double().abs()
    assert torch.isfinite(W).all()
    assert ((W - wref).abs() <= 4 * eps * (m ** 0.5 + 4) * wmag + 1e-300).all(), \
        float(((W - wref).abs() / wmag).max())


@pytest.mark.parametrize("m,n,k,pad", [sh for sh in SHAPES if 16 < sh[2] <= 48])
def test_az_f32_mfma_form(L, m, n, k, pad):
    """f32 Y = A Z with 16 < k <= 48 on the f32 matrix-core form (the A/B knob
    sl_ts_set_az_bf16(0); the default exact three-plane bf16 split is what
    test_az_and_atq checks): the same error bound, and stream-K cut blocks
    still bit-reproducible."""
    dev = torch.device("cuda")
    L.register("sl_ts_set_az_bf16", [i32], None)
    g = torch.Generator(device=dev).manual_seed(m + n + k + 1)
    lda = n + pad
    Afull = torch.randn(m, lda, device=dev, generator=g)
    A = Afull[:, :n]
    Z = torch.randn(n, k, device=dev, generator=g)
    outs = []
    try:
        L.require().sl_ts_set_az_bf16(0)
        for _ in range(2):
            Y = torch.full((m, k), float("nan"), device=dev)
            L.call("sl_ts_az", vp(Afull.data_ptr()), m, n, lda, vp(Z.data_ptr()), k, vp(Y.data_ptr()), k, F32, _st())
            outs.append(Y)
        torch.cuda.synchronize()
    finally:
        L.require().sl_ts_set_az_bf16(1)
    Y = outs[0]
    assert torch.isfinite(Y).all() and torch.equal(outs[0], outs[1])
    Ad = A.double()
    yref = Ad @ Z.double()
    ymag = Ad.abs() @ Z.double().abs()
    assert ((Y.double() - yref).abs() <= 4 * 1.2e-7 * (n ** 0.5 + 4) * ymag).all(), \
        float(((Y.double() - yref).abs() / ymag).max())


@pytest.mark.parametrize("dt,m,n,lda,k", [
    (torch.float32, 300_007, 1000, 1000, 40),   # 4000-B rows: four alignment classes, stream-K tail
    (torch.float64, 300_007, 1000, 1000, 40),   # 8000-B rows: two classes
    (torch.float64, 60_001, 5000, 5000, 20),
    (torch.float32, 5_000, 100, 104, 24),       # one chunk per row block
    (torch.float32, 50_001, 1000, 1000, 128),   # eight column tiles, eight waves
    (torch.float32, 3, 1000, 1000, 16)])         # fewer rows than a tile's classes
def test_az_alignment_classes(L, dt, m, n, lda, k):
    """Y = A Z with rows grouped by 128-B alignment class and the column
    groups shifted to whole cache lines (row pitch not a multiple of 128 B):
    within the product's error bound, bit-reproducible, and equal in bound to
    the unshifted form (sl_ts_set_az_align(0))."""
    dev = torch.device("cuda")
    L.register("sl_ts_set_az_align", [i32], None)
    g = torch.Generator(device=dev).manual_seed(m + n + k + 7)
    Afull = torch.randn(m, lda, device=dev, dtype=dt, generator=g)
    A = Afull[:, :n]
    Z = torch.randn(n, k, device=dev, dtype=dt, generator=g)
    code = F32 if dt == torch.float32 else F64
    outs = []
    try:
        for al in (1, 1, 0):
            L.require().sl_ts_set_az_align(al)
            Y = torch.full((m, k), float("nan"), device=dev, dtype=dt)
            L.call("sl_ts_az", vp(Afull.data_ptr()), m, n, lda, vp(Z.data_ptr()), k, vp(Y.data_ptr()), k, code, _st())
            outs.append(Y)
        torch.cuda.synchronize()
    finally:
        L.require().sl_ts_set_az_align(1)
    assert torch.isfinite(outs[0]).all() and torch.equal(outs[0], outs[1])
    Ad = A.double()
    yref = Ad @ Z.double()
    ymag = Ad.abs() @ Z.double().abs()
    eps = 1.2e-7 if dt == torch.float32 else 2.3e-16
    for Y in (outs[0], outs[2]):
        assert ((Y.double() - yref).abs() <= 4 * eps * (n ** 0.5 + 4) * ymag).all(), \
            float(((Y.double() - yref).abs() / ymag).max())


@pytest.mark.parametrize("m,n,k,lda", [(100_003, 1000, 40, 1000), (300_007, 200, 24, 204), (4_097, 1000, 33, 1008),
                                       (20_011, 1020, 40, 1020), (77, 104, 17, 104), (2, 1000, 48, 1000),
                                       (50_001, 1000, 64, 1000), (3_001, 200, 50, 200),
                                       (50_001, 1000, 128, 1000), (4_001, 300, 80, 304), (999, 104, 111, 104)])
def test_atq_f32_forms(L, m, n, k, lda):
    """f32 W = A^T Q for 16 < k <= 128 on both forms: the exact three-plane
    bf16 split (default, k_ts_atq_bs; ragged slices, a two-row operand) and
    the f32 matrix-core kernel (sl_ts_set_atq_bf16(0)), each within the f32
    product's error bound."""
    dev = torch.device("cuda")
    L.register("sl_ts_set_atq_bf16", [i32], None)
    g = torch.Generator(device=dev).manual_seed(m + n + k + 3)
    Afull = torch.randn(m, lda, device=dev, generator=g)
    A = Afull[:, :n]
    Q = torch.randn(m, k, device=dev, generator=g)
    ws = torch.zeros(int(L.require().sl_ts_atq_workspace(m, n, k, F32)), dtype=torch.uint8, device=dev)
    outs = []
    try:
        for bs in (1, 0):
            L.require().sl_ts_set_atq_bf16(bs)
            W = torch.full((n, k), float("nan"), device=dev, dtype=torch.float64)
            L.call("sl_ts_atq", vp(Afull.data_ptr()), m, n, lda, vp(Q.data_ptr()), k, vp(W.data_ptr()), k,
                   vp(ws.data_ptr()), F32, _st())
            torch.cuda.synchronize()
            outs.append(W)
    finally:
        L.require().sl_ts_set_atq_bf16(1)
    Ad = A.double()
    wref = Ad.t() @ Q.double()
    wmag = Ad.abs().t() @ Q.double().abs()
    for W in outs:
        assert torch.isfinite(W).all()
        assert ((W - wref).abs() <= 4 * 1.2e-7 * (m ** 0.5 + 4) * wmag).all(), float(((W - wref).abs() / wmag).max())


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_az_stream_k_deterministic(L, dt):
    """Row blocks cut by a stream-K range boundary are summed from two atomic
    partials: repeated calls must agree bit for bit."""
    dev = torch.device("cuda")
    m, n, k = 200_000, 777, 40
    A = torch.randn(m, n + 1, device=dev, dtype=dt)[:, :n]
    Z = torch.randn(n, k, device=dev, dtype=dt)
    code = F32 if dt == torch.float32 else F64
    outs = []
    for _ in range(3):
        Y = torch.full((m, k), float("nan"), device=dev, dtype=dt)
        L.call("sl_ts_az", vp(A.data_ptr()), m, n, n + 1, vp(Z.data_ptr()), k, vp(Y.data_ptr()), k, code, _st())
        outs.append(Y)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    ref = A.double() @ Z.double()
    tol = 1e-4 if dt == torch.float32 else 1e-12
    assert torch.allclose(outs[0].double(), ref, rtol=tol, atol=tol * ref.abs().max().item())


@pytest.mark.parametrize("m,n,k", [(100_003, 1000, 40), (2_500, 530, 64), (777, 37, 20)])
def test_atq_one_vector_variant(L, m, n, k):
    """A^T Q with one vector per wave and row (two workgroups per CU)."""
    dev = torch.device("cuda")
    _lib = L
    _lib.register("sl_ts_set_atq_av", [i32], None)
    try:
        _lib.require().sl_ts_set_atq_av(1)
        for dt, code in ((torch.float32, F32), (torch.float64, F64)):
            A = torch.randn(m, n, device=dev, dtype=dt)
            Q = torch.randn(m, k, device=dev, dtype=dt)
            ws = torch.zeros(int(_lib.require().sl_ts_atq_workspace(m, n, k, code)), dtype=torch.uint8, device=dev)
            W = torch.full((n, k), float("nan"), device=dev, dtype=torch.float64)
            _lib.call("sl_ts_atq", vp(A.data_ptr()), m, n, n, vp(Q.data_ptr()), k, vp(W.data_ptr()), k,
                      vp(ws.data_ptr()), code, _st())
            torch.cuda.synchronize()
            ref = A.double().t() @ Q.double()
            tol = 1e-4 if dt == torch.float32 else 1e-12
            assert torch.allclose(W, ref, rtol=tol, atol=tol * ref.abs().max().item())
    finally:
        _lib.require().sl_ts_set_atq_av(2)


def test_unaligned_lda_scalar_path(L):
    """lda = n + 1 (odd): 16-B loads are not allowed, the scalar path runs."""
    dev = torch.device("cuda")
    m, n, k = 3_001, 301, 24
    for dt, code in ((torch.float32, F32), (torch.float64, F64)):
        Afull = torch.randn(m, n + 1, device=dev, dtype=dt)
        Z = torch.randn(n, k, device=dev, dtype=dt)
        Y = torch.empty(m, k, device=dev, dtype=dt)
        L.call("sl_ts_az", vp(Afull.data_ptr()), m, n, n + 1, vp(Z.data_ptr()), k, vp(Y.data_ptr()), k, code, _st())
        ws = torch.zeros(int(L.require().sl_ts_atq_workspace(m, n, k, code)), dtype=torch.uint8, device=dev)
        W = torch.empty(n, k, device=dev, dtype=torch.float64)
        L.call("sl_ts_atq", vp(Afull.data_ptr()), m, n, n + 1, vp(Y.data_ptr()), k, vp(W.data_ptr()), k,
               vp(ws.data_ptr()), code, _st())
        torch.cuda.synchronize()
        Ad = Afull[:, :n].double()
        yref = Ad @ Z.double()
        tol = 1e-4 if dt == torch.float32 else 1e-12
        assert torch.allclose(Y.double(), yref, rtol=tol, atol=tol * yref.abs().max().item())
        wref = Ad.t() @ Y.double()
        assert torch.allclose(W, wref, rtol=tol, atol=tol * wref.abs().max().item())


@pytest.mark.parametrize("rows,k,k2", [(200_001, 40, 40), (1000, 40, 20), (77, 64, 64), (5, 3, 1)])
def test_xm64_gram64(L, rows, k, k2):
    dev = torch.device("cuda")
    X = torch.randn(rows, k, device=dev, dtype=torch.float64)
    M = torch.randn(k, k2, device=dev, dtype=torch.float64)
    for code, dt in ((F64, torch.float64), (F32, torch.float32)):
        out = torch.empty(rows, k2, device=dev, dtype=dt)
        L.call("sl_ts_xm64", vp(X.data_ptr()), rows, k, k, vp(M.data_ptr()), k2, vp(out.data_ptr()), k2, code, _st())
        torch.cuda.synchronize()
        ref = X @ M
        tol = 1e-12 if dt == torch.float64 else 1e-6
        assert torch.allclose(out.double(), ref, rtol=tol, atol=tol * ref.abs().max().item())
    ws = torch.zeros(int(L.require().sl_ts_gram64_workspace(rows, k)), dtype=torch.uint8, device=dev)
    G = torch.empty(k, k, device=dev, dtype=torch.float64)
    L.call("sl_ts_gram64", vp(X.data_ptr()), rows, k, k, vp(G.data_ptr()), k, vp(ws.data_ptr()), _st())
    torch.cuda.synchronize()
    ref = X.t() @ X
    assert torch.allclose(G, ref, rtol=1e-12, atol=1e-12 * ref.abs().max().item())
    assert torch.equal(G, G.t())


@pytest.mark.parametrize("rows,k,ldx", [(200_001, 128, 128), (5000, 100, 104), (3, 65, 65), (777, 128, 130)])
def test_gram_wide(L, rows, k, ldx):
    """X^T X for 64 < k <= 128 (pair-split matrix-core Gram) vs fp64 torch,
    f64 and f32 X, padded row stride; exactly symmetric."""
    dev = torch.device("cuda")
    Xp = torch.randn(rows, ldx, device=dev, dtype=torch.float64)
    for code, dt in ((F64, torch.float64), (F32, torch.float32)):
        Xs = Xp.to(dt)
        X = Xs[:, :k]
        ws = torch.zeros(int(L.require().sl_ts_gram64_workspace(rows, k)), dtype=torch.uint8, device=dev)
        G = torch.empty(k, k, device=dev, dtype=torch.float64)
        L.call("sl_ts_gram_w", vp(Xs.data_ptr()), code, rows, k, ldx, vp(G.data_ptr()), k, vp(ws.data_ptr()), _st())
        torch.cuda.synchronize()
        Xd = X.double()
        ref = Xd.t() @ Xd
        assert torch.allclose(G, ref, rtol=1e-12, atol=1e-12 * ref.abs().max().item())
        assert torch.equal(G, G.t())


def test_small(L):
    dev = torch.device("cuda")
    A = torch.randn(40, 40, device=dev, dtype=torch.float64)
    B = torch.randn(40, 20, device=dev, dtype=torch.float64)
    for ta in (0, 1):
        C_ = torch.empty(40, 20, device=dev, dtype=torch.float64)
        L.call("sl_ts_small", ta, 0, 40, 20, 40, vp(A.data_ptr()), 40, vp(B.data_ptr()), 20, vp(C_.data_ptr()), 20,
               _st())
        torch.cuda.synchronize()
        ref = (A.t() if ta else A) @ B
        assert torch.allclose(C_, ref, rtol=1e-13, atol=1e-12)


@pytest.mark.parametrize("mr,nc,kd", [(128, 128, 128), (100, 77, 128), (65, 130, 33), (128, 40, 128)])
def test_small_tiled(L, mr, nc, kd):
    """op(A) op(B) past 64 (the 64 < k <= 128 core): the 32 x 32-tile form,
    all four transpose combinations, padded leading dimensions."""
    dev = torch.device("cuda")
    for ta in (0, 1):
        for tb in (0, 1):
            Ab = torch.randn(*((kd, mr + 3) if ta else (mr, kd + 3)), device=dev, dtype=torch.float64)
            Bb = torch.randn(*((nc, kd + 5) if tb else (kd, nc + 5)), device=dev, dtype=torch.float64)
            A = Ab[:, :mr] if ta else Ab[:, :kd]
            B = Bb[:, :kd] if tb else Bb[:, :nc]
            C_ = torch.full((mr, nc + 2), 7.0, device=dev, dtype=torch.float64)
            L.call("sl_ts_small", ta, tb, mr, nc, kd, vp(A.data_ptr()), Ab.stride(0), vp(B.data_ptr()), Bb.stride(0),
                   vp(C_.data_ptr()), C_.stride(0), _st())
            torch.cuda.synchronize()
            ref = (A.t() if ta else A) @ (B.t() if tb else B)
            assert torch.allclose(C_[:, :nc], ref, rtol=1e-13, atol=1e-12)
            assert torch.all(C_[:, nc:] == 7.0)
