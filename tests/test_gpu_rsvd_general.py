"""General-precision device randSVD engine (rsvd_general.hip): f32 / f64 / bf16
operands of any width, k up to 128, the whole call on the device -- against
fp64 numpy SVDs of the same operand (reference nla/svd.hpp:222-318, double by
default).  f32 / f64 with k <= 64 run only hand-written kernels (matrix-core
products rsvd_stream.hip, one-wave small algebra); 64 < k <= 128 the same
products at six / eight column tiles with the core on rocSOLVER syevd; bf16
with n > 1024 keeps library GEMMs."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _planted(m, n, r, decay=0.8, noise=1e-7, seed=0):
    g = np.random.RandomState(seed)
    U0, _ = np.linalg.qr(g.randn(m, r))
    V0, _ = np.linalg.qr(g.randn(n, r))
    sig = 100.0 * decay ** np.arange(r)
    return (U0 * sig) @ V0.T + noise * g.randn(m, n)


def _check(A64, U, s, V, rank, rtol_s, tol_orth, tol_res):
    sv = np.linalg.svd(A64, compute_uv=False)[:rank]
    s = s.double().cpu().numpy()
    np.testing.assert_allclose(s, sv, rtol=rtol_s, atol=rtol_s * sv[0])
    Ud, Vd = U.double().cpu().numpy(), V.double().cpu().numpy()
    assert np.abs(Ud.T @ Ud - np.eye(rank)).max() < tol_orth
    assert np.abs(Vd.T @ Vd - np.eye(rank)).max() < tol_orth
    res = np.linalg.norm(A64 @ Vd - Ud * s) / np.linalg.norm(s)
    assert res < tol_res, res


@pytest.mark.parametrize("dtype,m,n,rank,q,sketch", [
    (torch.float64, 6000, 700, 10, 2, "FJLT"),
    (torch.float64, 3000, 2500, 12, 1, "JLT"),
    (torch.float32, 20000, 512, 10, 2, "FJLT"),
    (torch.float32, 4096, 3000, 8, 2, "CT"),
    (torch.bfloat16, 8192, 1536, 10, 2, "FJLT"),   # n > 1024: beyond the fused engine
])
def test_general_engine_vs_numpy(dtype, m, n, rank, q, sketch):
    import libskylark_amd as sk
    from libskylark_amd.nla import svd as S
    A64 = _planted(m, n, max(rank + 4, 16), noise=1e-7)
    A = torch.from_numpy(A64).to("cuda", dtype)
    if dtype == torch.bfloat16:
        A64 = A.double().cpu().numpy()   # the operand the engine sees
    prm = sk.nla.ApproximateSVDParams(num_iterations=q, sketch=sketch, check=True)
    U, s, V = sk.nla.approximate_svd(A, rank, sk.Context(seed=5), prm)
    plan = [p for p in S._PLANS.values() if p.Aref() is A][0]
    assert isinstance(plan, S._GenPlan)
    assert plan.native == (dtype != torch.bfloat16)   # no rocBLAS for f32 / f64 at k <= 64
    assert U.dtype == (torch.float64 if dtype == torch.float64 else torch.float32)
    tol = {torch.float64: (1e-9, 1e-10, 1e-6), torch.float32: (1e-4, 1e-4, 1e-3),
           torch.bfloat16: (2e-2, 2e-3, 5e-2)}[dtype]
    _check(A64, U, s, V, rank, *tol)


def test_general_engine_k_above_64_uses_rocsolver():
    """k = 2 r = 100 > 64: the products on the hand-written kernels at eight
    column tiles, the Cholesky inverses on the two-waves-per-row register
    kernel, the core by rocSOLVER syevd."""
    import libskylark_amd as sk
    A64 = _planted(5000, 800, 60, decay=0.95, noise=1e-9, seed=2)
    A = torch.from_numpy(A64).cuda()
    prm = sk.nla.ApproximateSVDParams(num_iterations=2, sketch="JLT", check=True)
    U, s, V = sk.nla.approximate_svd(A, 50, sk.Context(seed=1), prm)
    _check(A64, U, s, V, 50, 1e-8, 1e-10, 1e-6)


def test_general_engine_f32_k_above_64_odd_width():
    """f32, rank 55 -> k = 110 (seven column tiles padded to eight) on an odd
    row width (n = 777: the scalar-load paths of the products), against fp64
    numpy; the library-GEMM form of the same plan (sl_rsvd_gen_set_big(0))
    agrees to f32 roundoff."""
    import libskylark_amd as sk
    from libskylark_amd.ops import _lib
    A64 = _planted(7000, 777, 64, decay=0.93, noise=1e-7, seed=6)
    A = torch.from_numpy(A64).to("cuda", torch.float32)
    A64 = A.double().cpu().numpy()
    prm = sk.nla.ApproximateSVDParams(num_iterations=1, sketch="JLT", check=True)
    U, s, V = sk.nla.approximate_svd(A, 55, sk.Context(seed=12), prm)
    _check(A64, U, s, V, 55, 1e-4, 1e-4, 1e-3)
    lib = _lib.require()
    lib.sl_rsvd_gen_set_big(0)
    try:
        A2 = A.clone()   # a fresh plan, created with the knob off
        U2, s2, V2 = sk.nla.approximate_svd(A2, 55, sk.Context(seed=12), prm)
    finally:
        lib.sl_rsvd_gen_set_big(1)
    np.testing.assert_allclose(s.cpu().numpy(), s2.cpu().numpy(), rtol=1e-5, atol=1e-5 * float(s[0]))


def test_general_engine_matches_host_path_f64():
    """Same sketch stream, same algorithm: the device engine and the host-driven
    path (CPU tensor) agree to fp64 roundoff on a well-conditioned problem."""
    import libskylark_amd as sk
    A64 = _planted(3000, 400, 12, noise=1e-6, seed=3)
    prm = sk.nla.ApproximateSVDParams(num_iterations=1, sketch="JLT")
    Ug, sg, Vg = sk.nla.approximate_svd(torch.from_numpy(A64).cuda(), 8, sk.Context(seed=9), prm)
    Uc, sc, Vc = sk.nla.approximate_svd(torch.from_numpy(A64), 8, sk.Context(seed=9), prm)
    np.testing.assert_allclose(sg.cpu().numpy(), sc.numpy(), rtol=1e-10)
    np.testing.assert_allclose(np.abs(Vg.cpu().numpy()), np.abs(Vc.numpy()), atol=1e-8)


def test_general_engine_bf16_k_above_64():
    """bf16 A with rank 40 (k = 80 > 64): Y is kept in f32 and its Gram staged
    in f64 pieces through the plan workspace -- sized for bf16 too (it was
    sized for f32 only, and this call wrote past the plan allocation)."""
    import libskylark_amd as sk
    from libskylark_amd.nla import svd as S
    A64 = _planted(6000, 1536, 48, decay=0.9, noise=1e-6, seed=4)
    A = torch.from_numpy(A64).to("cuda", torch.bfloat16)
    A64 = A.double().cpu().numpy()
    prm = sk.nla.ApproximateSVDParams(num_iterations=2, sketch="FJLT", check=True)
    U, s, V = sk.nla.approximate_svd(A, 40, sk.Context(seed=3), prm)
    plan = [p for p in S._PLANS.values() if p.Aref() is A][0]
    assert isinstance(plan, S._GenPlan) and plan.k == 80
    _check(A64, U, s, V, 40, 2e-2, 2e-3, 5e-2)


def test_general_engine_rank_deficient_f32():
    """f32 operand of exact rank 15 < k = 40: the CholeskyQR factors drop the
    null directions (pivot dropping) and the top-10 SVD still matches numpy,
    as the host path's TSQR fallback does on the same operand."""
    import libskylark_amd as sk
    g = np.random.RandomState(11)
    A64 = (g.randn(5000, 15) * (10.0 * 0.8 ** np.arange(15))) @ g.randn(15, 600)
    A = torch.from_numpy(A64).to("cuda", torch.float32)
    A64 = A.double().cpu().numpy()
    prm = sk.nla.ApproximateSVDParams(num_iterations=2, sketch="JLT")
    U, s, V = sk.nla.approximate_svd(A, 10, sk.Context(seed=2), prm)
    _check(A64, U, s, V, 10, 1e-4, 1e-4, 1e-3)
    Uc, sc, Vc = sk.nla.approximate_svd(torch.from_numpy(A64), 10, sk.Context(seed=2), prm)
    np.testing.assert_allclose(s.double().cpu().numpy(), sc.double().numpy(), rtol=1e-4)


def test_general_engine_f64_graded_k128_matches_host():
    """f64, graded spectrum (0.9^i over 128 values + noise), rank 64 -> k =
    128 (library small algebra): the device engine agrees with the host-driven
    path (CPU f64, same sketch stream, explicit QR re-orthonormalisation) to
    far below the algorithm's own approximation error, so what accuracy the
    call has at k = 128 is the randomised algorithm's, not lost numerically
    (the eigen-whitening of an ill-conditioned Gram).  Parity with the
    reference's El::SVD of the same Rayleigh-Ritz core: pinned by the host
    path's own tests."""
    import libskylark_amd as sk
    from libskylark_amd.nla import svd as S
    g = np.random.RandomState(21)
    m, n = 4000, 700
    U0, _ = np.linalg.qr(g.randn(m, 128))
    V0, _ = np.linalg.qr(g.randn(n, 128))
    A64 = (U0 * (100.0 * 0.9 ** np.arange(128))) @ V0.T + 1e-8 * g.randn(m, n)
    prm = sk.nla.ApproximateSVDParams(num_iterations=1, sketch="JLT", check=True)
    A = torch.from_numpy(A64).cuda()
    Ug, sg, Vg = sk.nla.approximate_svd(A, 64, sk.Context(seed=8), prm)
    plan = [p for p in S._PLANS.values() if p.Aref() is A][0]
    assert isinstance(plan, S._GenPlan) and plan.k == 128 and not plan.native
    Uc, sc, Vc = sk.nla.approximate_svd(torch.from_numpy(A64), 64, sk.Context(seed=8), prm)
    sg, sc = sg.cpu().numpy(), sc.numpy()
    np.testing.assert_allclose(sg, sc, rtol=1e-9, atol=1e-9 * sc[0])
    # and the approximation itself: the top 64 of 128 graded values
    sv = np.linalg.svd(A64, compute_uv=False)[:64]
    np.testing.assert_allclose(sg, sv, rtol=1e-6)
    Vd = Vg.cpu().numpy()
    assert np.abs(Vd.T @ Vd - np.eye(64)).max() < 1e-10


def test_general_engine_f64_k_le_64_native_graded():
    """f64 graded spectrum at k = 64 on the hand-written path: singular values
    to 1e-9 of numpy's, orthonormal factors to 1e-10."""
    import libskylark_amd as sk
    from libskylark_amd.nla import svd as S
    g = np.random.RandomState(22)
    m, n = 20000, 900
    U0, _ = np.linalg.qr(g.randn(m, 64))
    V0, _ = np.linalg.qr(g.randn(n, 64))
    A64 = (U0 * (100.0 * 0.85 ** np.arange(64))) @ V0.T + 1e-10 * g.randn(m, n)
    A = torch.from_numpy(A64).cuda()
    prm = sk.nla.ApproximateSVDParams(num_iterations=2, sketch="FJLT", check=True)
    U, s, V = sk.nla.approximate_svd(A, 32, sk.Context(seed=4), prm)
    plan = [p for p in S._PLANS.values() if p.Aref() is A][0]
    assert plan.k == 64 and plan.native
    _check(A64, U, s, V, 32, 1e-9, 1e-10, 1e-7)
