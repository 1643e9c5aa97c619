"""HIP kernel numerics on the MI355X vs plain PyTorch fp32/fp64 references."""
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.ops import _lib

pytestmark = pytest.mark.gpu


def test_native_library_is_loaded():
    lib = _lib.require()
    assert lib.sl_version() >= 1


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
@pytest.mark.parametrize("dim", [0, 1])
def test_cwt_dense_gpu_vs_explicit(dev, dtype, dim):
    N, S, M = 3000, 257, 333
    T = sk.sketch.CWT(N, S, context=sk.Context(7))
    P = T.realize(torch.float64)
    A = torch.randn(N, M, dtype=torch.float64) if dim == 0 else torch.randn(M, N, dtype=torch.float64)
    Ad = A.to(dev, dtype)
    out = T.apply(Ad, dim=dim).double().cpu()
    Aq = Ad.double().cpu()
    ref = P @ Aq if dim == 0 else Aq @ P.t()
    tol = 1e-10 if dtype == torch.float64 else 1e-4 * float(ref.abs().max())
    torch.testing.assert_close(out, ref, atol=tol, rtol=1e-4)


@pytest.mark.parametrize("dim", [0, 1])
@pytest.mark.parametrize("vdt", [torch.float32, torch.float64])
def test_cwt_csr_gpu_vs_explicit(dev, dim, vdt):
    N, S, M = 5000, 300, 700
    T = sk.sketch.MMT(N, S, context=sk.Context(3))
    P = T.realize(torch.float64)
    A = torch.randn(N, M, dtype=torch.float64)
    A[torch.rand(N, M) > 0.05] = 0
    if dim == 1:
        A = A.t().contiguous()
    As = A.to(vdt).to_sparse_csr().to(dev)
    out = T.apply(As, dim=dim, sparse_output=False)
    assert out.dtype == vdt                      # f64 values accumulate in f64 (ds_add_f64)
    out = out.double().cpu()
    Aq = A.to(vdt).double()
    ref = P @ Aq if dim == 0 else Aq @ P.t()
    rel = 1e-12 if vdt == torch.float64 else 1e-4
    torch.testing.assert_close(out, ref, atol=rel * float(ref.abs().max()), rtol=rel)


@pytest.mark.parametrize("dim", [0, 1])
@pytest.mark.parametrize("vdt", [torch.float32, torch.float64])
@pytest.mark.parametrize("density", [0.002, 0.005, 0.05])
def test_cwt_csr_sparse_out_native(dev, dim, vdt, density):
    """hash_sparse_out.hip (sort-free CSR -> CSR) vs the generic coalesce
    route: same sparsity pattern and values; rowwise row lengths ~8 / ~20 / ~200
    exercise the 8/16/32 sorting networks and the generic fallback beyond 32."""
    from libskylark_amd.ops import hash_sketch as H
    N, S, M = 4000, 64, 700
    T = sk.sketch.CWT(N, S, context=sk.Context(5))
    A = torch.randn(N, M, dtype=torch.float64)
    A[torch.rand(N, M) > density] = 0
    if dim == 1:
        A = A.t().contiguous()
    As = A.to(vdt).to_sparse_csr().to(dev)
    As = torch.sparse_csr_tensor(As.crow_indices(), As.col_indices(), As.values(), As.shape)
    out = T.apply(As, dim=dim, sparse_output=True)
    ref = H._csr_sparse_out_generic(T._hd, As, dim)
    assert out.layout == torch.sparse_csr and out.shape == ref.shape
    assert torch.equal(out.crow_indices().cpu(), ref.crow_indices().cpu().to(torch.int64))
    assert torch.equal(out.col_indices().cpu(), ref.col_indices().cpu().to(torch.int64))
    tol = 1e-12 if vdt == torch.float64 else 1e-4
    torch.testing.assert_close(out.values().cpu(), ref.values().cpu(), rtol=tol, atol=tol)
    assert out.values().dtype == vdt


@pytest.mark.parametrize("dim", [0, 1])
def test_jlt_gpu_vs_cpu(dev, dim):
    N, S, M = 2048, 128, 96
    T = sk.sketch.JLT(N, S, context=sk.Context(11))
    A = torch.randn(N, M, dtype=torch.float64) if dim == 0 else torch.randn(M, N, dtype=torch.float64)
    cpu = T.apply(A, dim=dim)
    gpu64 = T.apply(A.to(dev), dim=dim).cpu()
    torch.testing.assert_close(gpu64, cpu, rtol=1e-10, atol=1e-10)
    gpu32 = T.apply(A.float().to(dev), dim=dim).double().cpu()
    torch.testing.assert_close(gpu32, cpu, rtol=1e-3, atol=1e-3 * float(cpu.abs().max()))


def test_rft_epilogue_gpu(dev):
    d, s = 64, 512
    T = sk.sketch.GaussianRFT(d, s, sigma=2.0, context=sk.Context(1))
    X = torch.randn(d, 200, dtype=torch.float64)
    torch.testing.assert_close((T * X.to(dev)).cpu(), T * X, rtol=1e-9, atol=1e-9)
    Tm = sk.sketch.MaternRFT(d, s, nu=1.5, l=2.0, context=sk.Context(1))
    torch.testing.assert_close((Tm / X.t().contiguous().to(dev)).cpu(), Tm / X.t().contiguous(), rtol=1e-9, atol=1e-9)
    Tr = sk.sketch.ExpSemigroupRLT(d, s, beta=0.5, context=sk.Context(2))
    Xp = X.abs()
    torch.testing.assert_close((Tr * Xp.to(dev)).cpu(), Tr * Xp, rtol=1e-8, atol=1e-10)


def test_fjlt_gpu(dev):
    for s in (40, 400):
        T = sk.sketch.FJLT(1000, s, context=sk.Context(5))
        A = torch.randn(1000, 64, dtype=torch.float64)
        torch.testing.assert_close((T * A.to(dev)).cpu(), T.realize() @ A, rtol=1e-8, atol=1e-8)


def test_fastfood_and_ppt_gpu(dev):
    X = torch.randn(32, 50, dtype=torch.float64)
    for T in (sk.sketch.FastGaussianRFT(32, 100, sigma=1.0, context=sk.Context(3)),
              sk.sketch.PPT(32, 128, q=3, context=sk.Context(3))):
        torch.testing.assert_close((T * X.to(dev)).cpu(), T * X, rtol=1e-8, atol=1e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("N,S", [(1, 1), (1000, 40), (4099, 17)])
def test_dct2_rows_native(dev, N, S):
    from libskylark_amd.ops import fut
    rows = torch.randint(0, N, (S,))
    rows[0] = 0
    d = torch.randint(0, 2, (N,)).double() * 2 - 1
    ref = fut.dct2_rows_matrix(N, rows, dtype=torch.float64, d=d, scale=1.7)
    for tr in (False, True):
        got = fut.dct2_rows_matrix(N, rows, dtype=torch.float64, device=dev, d=d, scale=1.7, transpose=tr)
        torch.testing.assert_close(got.cpu(), ref.t() if tr else ref, rtol=1e-12, atol=1e-12)
    got32 = fut.dct2_rows_matrix(N, rows, dtype=torch.float32, device=dev, d=d, scale=1.7, transpose=True)
    torch.testing.assert_close(got32.cpu().double(), ref.t(), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("N,S", [(1000, 40), (257, 13)])
def test_fjlt_operator_from_device_params_matches_sketch(dev, N, S):
    from libskylark_amd.ops import fut as F
    ctx = sk.Context(38734, counter=77)
    T = sk.sketch.FJLT(N, S, context=ctx.copy())
    ref = T.realize(torch.float64, transpose=True)
    prm = torch.tensor([ctx.seed, ctx.counter, ctx.counter + N], dtype=torch.int64, device=dev)
    out = torch.empty(N, S, dtype=torch.float64, device=dev)
    F.fjlt_operator(prm, S, N, (N / S) ** 0.5, out, transpose=True)
    torch.testing.assert_close(out.cpu(), ref, atol=1e-12, rtol=1e-12)


@pytest.mark.parametrize("cond,dt", [(1e3, torch.float32), (1e10, torch.float64)])
def test_lsrn_gpu_preconditioner_paths(dev, cond, dt):
    """Cholesky-QR + explicit R^-1 for well-conditioned sketches, Householder +
    triangular solves for ill-conditioned ones: both solve the problem."""
    import libskylark_amd as sk
    from libskylark_amd.algorithms import AcceleratedRegressionSolver, KrylovIterParams, RegressionProblem
    torch.manual_seed(0)
    m, n = 20000, 300
    U, _ = torch.linalg.qr(torch.randn(m, n, dtype=torch.float64, device=dev))
    s = torch.logspace(0, -torch.log10(torch.tensor(cond)).item(), n, dtype=torch.float64, device=dev)
    A = ((U * s) @ torch.linalg.qr(torch.randn(n, n, dtype=torch.float64, device=dev))[0]).to(dt)
    x = torch.randn(n, 1, device=dev, dtype=dt)
    b = A @ x
    solver = AcceleratedRegressionSolver(RegressionProblem(A), sk.Context(3), method="lsrn", precond="qr",
                                         params=KrylovIterParams(tolerance=1e-6, iter_lim=400))
    X, code = solver.solve(b)
    res = float((A @ X.to(A.dtype) - b).norm() / b.norm())
    assert res < 1e-4, (res, code)


@pytest.mark.parametrize("dim,backend", [(0, "gemm_nt"), (0, "hipblaslt"), (1, None)])
@pytest.mark.parametrize("block", [0, 1000, 1003])
@pytest.mark.parametrize("M", [333, 512])
def test_dense_sketch_bf16x2_panels(dev, dim, backend, block, M, monkeypatch):
    """LSRN's internal sketch: bf16-realised S panels times the
    bf16 hi/lo split of f32 A in reused buffers; equals S_bf16 @ A to ~2^-16
    for one or many panels (block 1003: ragged).  Columnwise: the NT form
    (transposed split planes, C2 += P HL^T) on the hand-written NT GEMM's
    accumulate path (M = 512: 16-B aligned C rows, the preloaded-C
    epilogue; 333: the per-element path) or on hipBLASLt; rowwise: the NN
    form (16-B alignment fallback for column slices)."""
    from libskylark_amd.ops import dense_sketch as DS
    from libskylark_amd.sketch import params
    if backend is not None:
        monkeypatch.setattr(DS, "LSRN_GEMM", backend)
    N, S = 4100, 96
    T = sk.sketch.JLT(N, S, context=sk.Context(21))
    A = torch.randn(N, M, device=dev) if dim == 0 else torch.randn(M, N, device=dev)
    old = params.get_blocksize()
    params.set_blocksize(block)
    try:
        out = DS.apply_dense(A, dim, dist=T.dist, seed=T.entries.seed, base=T.entries.base, S=S, N=N,
                             scale=T.scale, precision="bf16x2")
    finally:
        params.set_blocksize(old)
    Sb = DS.realize_panel(T.dist, T.entries.seed, T.entries.base, S, (0, S), (0, N), scale=T.scale,
                          dtype=torch.bfloat16, device=dev).double()
    ref = Sb @ A.double() if dim == 0 else A.double() @ Sb.t()
    torch.testing.assert_close(out.double(), ref, rtol=0, atol=2e-5 * float(ref.abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("shape,view,dt", [((20000, 1000), "row", torch.bfloat16), ((333, 1001), "row", torch.float32),
                                           ((1000, 77), "col", torch.bfloat16), ((513, 1200), "slice", torch.bfloat16),
                                           ((4097, 1), "row", torch.float32), ((1, 4097), "row", torch.bfloat16)])
def test_fill_normal_fast_lines_bitwise(dev, shape, view, dt):
    """The vectorised N(0,1) line kernel reproduces the generic fill bit for
    bit: the same logical matrix filled into a strided view with no unit
    stride (which only the generic kernel serves) holds the same bits."""
    from libskylark_amd.base import distributions as D
    from libskylark_amd.ops import rng

    def make():
        if view == "col":
            return torch.empty(shape[1], shape[0], dtype=dt, device=dev).t()
        if view == "slice":
            return torch.empty(shape[0], shape[1] + 40, dtype=dt, device=dev)[:, 3:3 + shape[1]]
        return torch.empty(shape, dtype=dt, device=dev)
    fast = make()
    rng.fill_random(fast, D.Normal(), 1234, 77, r0=5, c0=11, ir=1, ic=50021, scale=0.3)
    gen = torch.empty(shape[0], 2 * shape[1], dtype=dt, device=dev)[:, ::2]   # strides (2 cols, 2)
    if shape[0] == 1 or shape[1] == 1:
        gen = torch.empty(2 * shape[0], 2 * shape[1], dtype=dt, device=dev)[::2, ::2]
    rng.fill_random(gen, D.Normal(), 1234, 77, r0=5, c0=11, ir=1, ic=50021, scale=0.3)
    torch.cuda.synchronize()
    it = torch.int16 if dt == torch.bfloat16 else torch.int32
    assert torch.equal(fast.contiguous().view(it), gen.contiguous().view(it))


@pytest.mark.gpu
@pytest.mark.parametrize("vdt", [torch.float32, torch.float64])
def test_cwt_csr_deterministic_mode(dev, vdt):
    """Deterministic mode: int64 fixed-point accumulation gives bit-identical
    results across runs, within f32/f64 rounding of the fp64 reference."""
    from libskylark_amd.sketch import params
    g = torch.Generator().manual_seed(5)
    N, m, S = 20000, 3000, 256
    nnz = N * 12
    rows = torch.randint(0, N, (nnz,), generator=g)
    cols = torch.randint(0, m, (nnz,), generator=g)
    v = torch.randn(nnz, generator=g, dtype=torch.float64) * torch.exp(2 * torch.randn(nnz, generator=g,
                                                                                      dtype=torch.float64))
    A = torch.sparse_coo_tensor(torch.stack([rows, cols]), v, (N, m)).coalesce().to_sparse_csr()
    sk_ = sk.sketch.CWT(N, S, context=sk.Context(3))
    Ad = A.to(vdt).to(dev)
    ref = sk_.apply(A.to_dense(), dim=sk.sketch.COLUMNWISE)     # CPU fp64 index_add reference
    try:
        params.set_deterministic(True)
        outs = [sk_.apply(Ad, dim=sk.sketch.COLUMNWISE, sparse_output=False).cpu() for _ in range(3)]
    finally:
        params.set_deterministic(False)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    err = float((outs[0].double() - ref).norm() / ref.norm())
    assert err < (1e-6 if vdt == torch.float32 else 1e-12), err
    fast = sk_.apply(Ad, dim=sk.sketch.COLUMNWISE, sparse_output=False).cpu()
    assert float((fast.double() - ref).norm() / ref.norm()) < (1e-6 if vdt == torch.float32 else 1e-12)


@pytest.mark.gpu
def test_cwt_csr_rowwise_atomic_free(dev):
    """Rowwise CSR with short rows runs one lane per row (no atomics): repeated
    runs are bitwise identical and match the fp64 reference."""
    g = torch.Generator().manual_seed(6)
    m, N, S = 5000, 20000, 512
    nnz = m * 8
    rows = torch.randint(0, m, (nnz,), generator=g)
    cols = torch.randint(0, N, (nnz,), generator=g)
    A = torch.sparse_coo_tensor(torch.stack([rows, cols]), torch.randn(nnz, generator=g), (m, N)).coalesce()
    A = A.to_sparse_csr()
    sk_ = sk.sketch.CWT(N, S, context=sk.Context(4))
    ref = sk_.apply(A.to_dense().double(), dim=sk.sketch.ROWWISE)
    o1 = sk_.apply(A.to(dev), dim=sk.sketch.ROWWISE, sparse_output=False).cpu()
    o2 = sk_.apply(A.to(dev), dim=sk.sketch.ROWWISE, sparse_output=False).cpu()
    assert torch.equal(o1, o2)
    assert float((o1.double() - ref).norm() / ref.norm()) < 1e-6
