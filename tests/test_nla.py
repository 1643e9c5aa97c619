"""Randomized SVD / power iteration / fused pass: reconstruction and accuracy."""
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.ops import tallskinny


def _lowrank(m, n, r, decay=0.5, noise=1e-3, seed=0, dtype=torch.float64):
    g = torch.Generator().manual_seed(seed)
    U, _ = torch.linalg.qr(torch.randn(m, n, generator=g, dtype=torch.float64))
    V, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    s = torch.tensor([decay ** i for i in range(n)], dtype=torch.float64) * 10
    s[r:] *= noise
    return ((U * s) @ V.t()).to(dtype), s


@pytest.mark.parametrize("sketch", ["JLT", "FJLT", "CWT"])
@pytest.mark.parametrize("iters", [0, 2])
def test_approximate_svd_tall(sketch, iters):
    A, s0 = _lowrank(2000, 120, 10, decay=0.7)
    U, s, V = sk.nla.approximate_svd(A, 10, context=sk.Context(1),
                                     params=sk.nla.ApproximateSVDParams(num_iterations=iters, sketch=sketch))
    assert U.shape == (2000, 10) and V.shape == (120, 10)
    torch.testing.assert_close(s, s0[:10], rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(U.t() @ U, torch.eye(10, dtype=U.dtype), atol=1e-8, rtol=0)
    R = (U * s) @ V.t()
    assert float((A - R).norm() / A.norm()) < 1e-2


def test_approximate_svd_wide():
    A, s0 = _lowrank(1500, 100, 8, decay=0.6)
    At = A.t().contiguous()
    U, s, V = sk.nla.approximate_svd(At, 8, params=sk.nla.ApproximateSVDParams(num_iterations=1))
    assert U.shape == (100, 8) and V.shape == (1500, 8)
    torch.testing.assert_close(s, s0[:8], rtol=1e-2, atol=1e-2)


def test_rank_check():
    with pytest.raises(sk.base.exceptions.InvalidParametersError):
        sk.nla.approximate_svd(torch.randn(10, 5, dtype=torch.float64), 6)


def test_fused_pass_torch_path():
    A = torch.randn(5000, 64, dtype=torch.float64)
    Z = torch.randn(64, 12, dtype=torch.float64)
    W, G, Y = tallskinny.fused_pass(A, Z, keep_y=True)
    Yr = A @ Z
    torch.testing.assert_close(Y, Yr)
    torch.testing.assert_close(W, A.t() @ Yr)
    torch.testing.assert_close(G, Yr.t() @ Yr)


def test_symmetric_svd():
    A, s0 = _lowrank(300, 300, 6, decay=0.5)
    Asym = A @ A.t()
    V, w = sk.nla.approximate_symmetric_svd(Asym, 6, params=sk.nla.ApproximateSVDParams(num_iterations=2))
    torch.testing.assert_close(w, (s0[:6] ** 2), rtol=1e-3, atol=1e-6)


def _indefinite(n, spec):
    g = torch.Generator().manual_seed(11)
    Q, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    return (Q * torch.tensor(spec, dtype=torch.float64)) @ Q.t()


@pytest.mark.parametrize("uplo", ["L", "U"])
def test_symmetric_svd_reads_one_triangle(uplo):
    """Only the uplo triangle is read (the other holds garbage); eigenvalues are
    ordered by signed value, descending (reference El::DESCENDING)."""
    n = 120
    spec = [50.0, -45.0, 30.0, -20.0, 10.0] + [1e-3] * (n - 5)
    S = _indefinite(n, spec)
    junk = torch.randn(n, n, dtype=torch.float64) * 100
    A = torch.tril(S) + torch.triu(junk, 1) if uplo == "L" else torch.triu(S) + torch.tril(junk, -1)
    V, w = sk.nla.approximate_symmetric_svd(A, 5, context=sk.Context(4),
                                            params=sk.nla.ApproximateSVDParams(num_iterations=3), uplo=uplo)
    # the 2 r = 10 Ritz values hold the 5 dominant |lambda|; sorted by signed
    # value the top 5 are 50, 30, 10 and two from the 1e-3 cluster
    torch.testing.assert_close(w[:3], torch.tensor([50.0, 30.0, 10.0], dtype=torch.float64), rtol=1e-6, atol=1e-6)
    assert (w[3:] - 1e-3).abs().max() < 1e-4
    # eigenvectors of the full symmetric matrix
    torch.testing.assert_close(S @ V[:, :3], V[:, :3] * w[:3], rtol=1e-6, atol=1e-5)
    # sparse input, same triangle semantics
    Vs, ws = sk.nla.approximate_symmetric_svd(A.to_sparse_csr(), 5, context=sk.Context(4),
                                              params=sk.nla.ApproximateSVDParams(num_iterations=3), uplo=uplo)
    torch.testing.assert_close(ws, w, rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_approximate_svd_gpu_bf16(dev):
    A, s0 = _lowrank(20000, 256, 12, decay=0.7)
    Ab = A.to(dev, torch.bfloat16)
    ref_s = torch.linalg.svdvals(Ab.double())[:12].cpu()
    U, s, V = sk.nla.approximate_svd(Ab, 12, context=sk.Context(2),
                                     params=sk.nla.ApproximateSVDParams(num_iterations=2, sketch="FJLT"))
    torch.testing.assert_close(s.double().cpu(), ref_s, rtol=2e-3, atol=2e-3)
    I = torch.eye(12, device=dev)
    torch.testing.assert_close(U.t().float() @ U.float(), I, atol=1e-4, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(70001, 1000, 40), (5000, 512, 64), (3000, 136, 9), (33, 64, 16)])
def test_tsk_matmul_native(dev, m, n, k):
    A = torch.randn(m, n, device=dev).to(torch.bfloat16)
    Z = torch.randn(n, k, device=dev, dtype=torch.float64)
    assert tallskinny._native_ok(A, k)
    Y = tallskinny.matmul(A, Z)
    Yr = A.double() @ Z
    torch.testing.assert_close(Y.double(), Yr, rtol=1e-4, atol=1e-4 * float(Yr.abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(70001, 1000, 40), (4099, 512, 64), (1000, 72, 3), (17, 1024, 48)])
def test_fused_pass_native_shapes(dev, shape):
    m, n, k = shape
    A = torch.randn(m, n, device=dev).to(torch.bfloat16)
    Z = torch.randn(n, k, device=dev) / 30
    assert tallskinny._native_ok(A, k)
    W, G, Y = tallskinny.fused_pass(A, Z, keep_y=True)
    Ad = A.double()
    Yr = Ad @ Z.to(torch.bfloat16).double()
    torch.testing.assert_close(Y.double(), Yr, rtol=1e-4, atol=1e-4 * float(Yr.abs().max()))
    Wr = Ad.t() @ Yr
    torch.testing.assert_close(W.double(), Wr, rtol=1e-3, atol=1e-4 * float(Wr.abs().max()))
    Gr = Yr.t() @ Yr
    torch.testing.assert_close(G.double(), Gr, rtol=1e-3, atol=1e-5 * float(Gr.abs().max()))
    W2, G2, Y2 = tallskinny.fused_pass(A, Z, keep_y=False)
    assert Y2 is None
    torch.testing.assert_close(W2, W)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(70001, 1000, 40), (4099, 512, 64), (1000, 72, 3), (17, 1024, 48), (33, 64, 16)])
def test_fused_pass_native_gram64(dev, shape):
    """In-pass f64 Gram of the stored f32 Y equals the f64 Gram of that Y
    (exact f32 products, f64 sums) — the numbers the separate gram64 pass gave."""
    m, n, k = shape
    A = torch.randn(m, n, device=dev).to(torch.bfloat16)
    Z = torch.randn(n, k, device=dev) / 30
    W, G, Y = tallskinny.fused_pass(A, Z, keep_y=True, gram64=True)
    assert G.dtype == torch.float64 and G.shape == (k, k)
    Yd = Y.double()
    Gr = Yd.t() @ Yd
    torch.testing.assert_close(G, Gr, rtol=1e-12, atol=1e-12 * float(Gr.abs().max()))
    torch.testing.assert_close(G, tallskinny.gram64(Y), rtol=1e-12, atol=1e-12 * float(Gr.abs().max()))
    W0, _, Y0 = tallskinny.fused_pass(A, Z, keep_y=True, gram=False)
    torch.testing.assert_close(W, W0, rtol=0, atol=0)
    torch.testing.assert_close(Y, Y0, rtol=0, atol=0)
    # rows walked last-to-first: the same Y bit for bit, W / G up to the order
    # of the per-workgroup partial sums
    Wr, Gr2, Yr2 = tallskinny.fused_pass(A, Z, keep_y=True, gram64=True, reverse=True)
    torch.testing.assert_close(Yr2, Y, rtol=0, atol=0)
    torch.testing.assert_close(Gr2, G, rtol=1e-12, atol=1e-12 * float(Gr.abs().max()))
    torch.testing.assert_close(Wr, W, rtol=1e-5, atol=1e-5 * float(W.abs().max()))
    Wi, _, _ = tallskinny.fused_pass(A, Z, keep_y=False, gram=False, exact=False)
    Wir, _, _ = tallskinny.fused_pass(A, Z, keep_y=False, gram=False, exact=False, reverse=True)
    torch.testing.assert_close(Wir, Wi, rtol=1e-5, atol=1e-5 * float(Wi.abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("native", [False, True])
def test_fused_pass_gpu_bf16(dev, native):
    old = tallskinny.USE_NATIVE
    tallskinny.USE_NATIVE = native
    try:
        m, n, k = 70001, 1000, 40
        A = torch.randn(m, n, device=dev).to(torch.bfloat16)
        Z = torch.randn(n, k, device=dev) / 30
        W, G, Y = tallskinny.fused_pass(A, Z, keep_y=True)
        Ad = A.double()
        Yr = Ad @ Z.to(torch.bfloat16).double()
        torch.testing.assert_close(Y.double(), Yr, rtol=1e-4, atol=1e-4 * float(Yr.abs().max()))
        Wr = Ad.t() @ Yr
        torch.testing.assert_close(W.double(), Wr, rtol=1e-3, atol=1e-4 * float(Wr.abs().max()))
        Gr = Yr.t() @ Yr
        torch.testing.assert_close(G.double(), Gr, rtol=1e-3, atol=1e-5 * float(Gr.abs().max()))
    finally:
        tallskinny.USE_NATIVE = old


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,k2", [(1000003, 40, 20), (5000, 64, 64), (77, 5, 3)])
def test_f32_xm_native(dev, m, k, k2):
    g = torch.Generator(device=dev).manual_seed(m + k)
    Y = torch.randn(m, k, device=dev, generator=g)
    M = torch.randn(k, k2, device=dev, generator=g)
    Q, G = tallskinny.f32_xm(Y, M, store=True, gram=True)
    Qr = Y.double() @ M.double()
    torch.testing.assert_close(Q.double(), Qr, rtol=1e-4, atol=1e-4)

    def rel(a, b):  # f32 accumulation: error ~ eps * sum |terms|, so compare in norm
        return float((a.double() - b).norm() / b.norm())
    assert rel(G, Qr.t() @ Qr) < 1e-5
    _, G1 = tallskinny.f32_xm(Y, None, store=False, gram=True)
    assert rel(G1, Y.double().t() @ Y.double()) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,k2", [(1000003, 40, 20), (5001, 64, 64), (31, 8, 3), (70000, 16, 40), (100, 24, 33)])
def test_f32_xm_store_native(dev, m, k, k2):
    """Store-only Q = Y M (the contiguous pipelined kernel) == fp64 torch."""
    g = torch.Generator(device=dev).manual_seed(m + k2)
    Y = torch.randn(m, k, device=dev, generator=g)
    M = torch.randn(k, k2, device=dev, generator=g)
    Q, G = tallskinny.f32_xm(Y, M, store=True, gram=False)
    assert G is None and Q.shape == (m, k2)
    Qr = Y.double() @ M.double()
    torch.testing.assert_close(Q.double(), Qr, rtol=1e-5, atol=1e-5 * float(Qr.abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("m,k,ld", [(1000003, 40, 40), (5000, 64, 64), (77, 5, 5), (4099, 17, 24), (3, 33, 33)])
def test_gram64_native(dev, m, k, ld):
    """fp64 Gram of f32 Y on the f64 matrix cores == fp64 torch (to ~eps64)."""
    g = torch.Generator(device=dev).manual_seed(m + k)
    Yf = torch.randn(m, ld, device=dev, generator=g)
    Y = Yf[:, :k]
    G = tallskinny.gram64(Y)
    Yd = Y.double()
    Gr = sum(Yd[i:i + 8192].t() @ Yd[i:i + 8192] for i in range(0, m, 8192))  # short fp64 chains
    assert G.dtype == torch.float64 and G.shape == (k, k)
    assert float((G - Gr).norm() / Gr.norm()) < 1e-12
    assert float((G - G.t()).abs().max()) <= 1e-14 * float(Gr.abs().max())


def _fullrank_decaying(m, n, decay, seed):
    g = torch.Generator().manual_seed(seed)
    U0, _ = torch.linalg.qr(torch.randn(m, n, generator=g))
    V0, _ = torch.linalg.qr(torch.randn(n, n, generator=g))
    s0 = 100.0 * decay ** torch.arange(n, dtype=torch.float32)
    return (U0 * s0) @ V0.t()


@pytest.mark.gpu
@pytest.mark.parametrize("sketch", ["FJLT", "JLT"])
def test_approximate_svd_device_plan_full_path(dev, sketch):
    """Full-rank input (no CholeskyQR breakdown): the device plan runs end to
    end -- fused passes, fp64 Gram, chol_inv, svd_core / svd_finish, graph
    capture and replay -- and is not replaced by the host fallback."""
    from libskylark_amd.nla import svd as SV
    A = _fullrank_decaying(20000, 256, 0.9, 5).to(dev, torch.bfloat16)
    ref = torch.linalg.svd(A.double(), full_matrices=False)
    p = sk.nla.ApproximateSVDParams(num_iterations=2, sketch=sketch)
    SV._PLANS.clear()
    outs = []
    for _ in range(3):                       # eager, capture, replay
        U, s, V = sk.nla.approximate_svd(A, 10, context=sk.Context(3), params=p)
        outs.append((U, s, V))
    plans = list(SV._PLANS.values())
    assert len(plans) == 1 and plans[0].calls == 3 and plans[0].graph_built()
    for U, s, V in outs:
        torch.testing.assert_close(s.double(), ref.S[:10], rtol=1e-2, atol=0)
        torch.testing.assert_close(s[:3].double(), ref.S[:3], rtol=1e-4, atol=0)
        I = torch.eye(10, device=dev, dtype=torch.float64)
        torch.testing.assert_close(U.double().t() @ U.double(), I, atol=1e-5, rtol=0)
        torch.testing.assert_close(V.double().t() @ V.double(), I, atol=1e-4, rtol=0)
        # leading singular vectors match the exact ones (up to sign)
        cu = (U[:, :3].double() * ref.U[:, :3]).sum(0).abs()
        cv = (V[:, :3].double() * ref.Vh[:3].t()).sum(0).abs()
        assert float(cu.min()) > 0.999 and float(cv.min()) > 0.999
    torch.testing.assert_close(outs[2][1], outs[1][1], rtol=1e-6, atol=0)


@pytest.mark.gpu
def test_approximate_svd_graph_replay_matches_eager(dev):
    """The hipGraph-replayed device plan gives the eager result (same context)."""
    g = torch.Generator().manual_seed(4)
    U0, _ = torch.linalg.qr(torch.randn(20000, 12, generator=g))
    V0, _ = torch.linalg.qr(torch.randn(256, 12, generator=g))
    s0 = torch.linspace(50, 5, 12)
    A = ((U0 * s0) @ V0.t()).to(dev, torch.bfloat16)
    p = sk.nla.ApproximateSVDParams(num_iterations=2, sketch="FJLT")
    outs = []
    for _ in range(4):  # call 1 eager, call 2 captures, calls 3-4 replay
        U, s, V = sk.nla.approximate_svd(A, 8, context=sk.Context(9), params=p)
        outs.append((U.cpu(), s.cpu(), V.cpu()))
    for U, s, V in outs[1:]:
        torch.testing.assert_close(s, outs[0][1], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(U.abs(), outs[0][0].abs(), rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(V.abs(), outs[0][2].abs(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(outs[0][1], s0[:8], rtol=2e-2, atol=2e-2)
    # a different sketch (fresh context) still gives the same top spectrum
    _, s2, _ = sk.nla.approximate_svd(A, 8, context=sk.Context(10), params=p)
    torch.testing.assert_close(s2.cpu(), s0[:8], rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("sketch,tol", [("JLT", 1e-5), ("FJLT", 1e-3)])
def test_approximate_svd_engine_matches_host_path(dev, sketch, tol):
    """The C++ engine (device CholeskyQRs, fp64 core, device Jacobi, no host
    round trip) gives the host-driven path's answer (LAPACK SVD of the core):
    same spectrum, same leading subspaces, on eager, capture and replay calls.
    FJLT samples its k = 20 DCT frequencies of n = 256 with replacement: on a
    repeat the engine drops the dependent direction (status bit 1, k - 1
    columns) where the host path's Householder fallback keeps an arbitrary
    one, so the trailing values agree to 1e-3 there, not 1e-5."""
    from libskylark_amd.nla import svd as SV
    A = _fullrank_decaying(20000, 256, 0.9, 5).to(dev, torch.bfloat16)
    p = sk.nla.ApproximateSVDParams(num_iterations=2, sketch=sketch)
    SV._PLANS.clear()
    for _ in range(3):                       # eager, capture, replay
        U, s, V = sk.nla.approximate_svd(A, 10, context=sk.Context(3), params=p)
    st = SV.last_device_status()
    assert st & ~SV.ST_PIVOT == 0
    if sketch == "JLT":
        assert st == 0
    # host-driven reference: same sketch / same context, no engine
    old = SV._engine_ok
    SV._engine_ok = lambda *a: False
    try:
        Uh, sh, Vh = sk.nla.approximate_svd(A, 10, context=sk.Context(3), params=p)
    finally:
        SV._engine_ok = old
    torch.testing.assert_close(s.double(), sh.double(), rtol=tol, atol=0)
    torch.testing.assert_close((U.double().t() @ Uh.double()).abs().diagonal()[:8],
                               torch.ones(8, dtype=torch.float64, device=dev), atol=10 * tol, rtol=0)
    torch.testing.assert_close((V.double().t() @ Vh.double()).abs().diagonal()[:8],
                               torch.ones(8, dtype=torch.float64, device=dev), atol=10 * tol, rtol=0)


