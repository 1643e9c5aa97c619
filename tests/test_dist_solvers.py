"""Distributed exact least-squares solvers (TSQR / Gram; no gather of A) and
the distributed symmetric randomized eigensolver equal their one-process
answers (gloo, CPU ranks).  Reference: ``El::qr::ExplicitTS`` for [VC,*]
(``base/QR.hpp:11-36``), ``linearl2_regression_solver_Elemental.hpp:23-631``,
``ApproximateSymmetricSVD`` any-variants (``nla/svd.hpp:396-506``)."""
import pytest
import torch

from mp_utils import run_distributed


def _solver_worker(rank, world, layout):
    import libskylark_amd as sk
    from libskylark_amd.algorithms import regression as R
    from libskylark_amd.parallel.comm import world as W
    from libskylark_amd.parallel.distmatrix import DistMatrix
    comm = W()
    g = torch.Generator().manual_seed(3)
    m, n = 203, 9
    A = torch.randn(m, n, generator=g, dtype=torch.float64)
    b = torch.randn(m, 2, generator=g, dtype=torch.float64)
    ref = torch.linalg.lstsq(A, b).solution
    D = DistMatrix.from_global(A, layout, comm, block=(16, 4) if layout == "MC_MR" else None)
    Bd = DistMatrix.from_global(b, "VC_STAR", comm)
    for method in ("qr", "sne", "ne", "svd"):
        comm.bytes_sent = 0
        s = R.RegressionSolver(R.RegressionProblem(D), method)
        for rhs in (b, Bd):
            x = s.solve(rhs)
            torch.testing.assert_close(x, ref, rtol=1e-8, atol=1e-9)
        x1 = s.solve(b[:, 0])
        torch.testing.assert_close(x1, ref[:, 0], rtol=1e-8, atol=1e-9)
    return True


@pytest.mark.parametrize("world,layout", [(4, "VC_STAR"), (8, "MC_MR"), (3, "STAR_VC")])
def test_exact_solvers_distributed(world, layout):
    run_distributed(_solver_worker, world, layout)


def _symsvd_worker(rank, world):
    import libskylark_amd as sk
    from libskylark_amd.parallel.comm import world as W
    from libskylark_amd.parallel.distmatrix import DistMatrix
    comm = W()
    n = 90
    g = torch.Generator().manual_seed(5)
    Q, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    spec = torch.tensor([40.0, -30.0, 20.0, 10.0] + [0.01] * (n - 4), dtype=torch.float64)
    S = (Q * spec) @ Q.t()
    A = torch.tril(S) + torch.triu(torch.full((n, n), 7.0, dtype=torch.float64), 1)   # junk above
    params = sk.nla.ApproximateSVDParams(num_iterations=3)
    V0, w0 = sk.nla.approximate_symmetric_svd(A, 3, context=sk.Context(9), params=params, uplo="L")
    for layout in ("VC_STAR", "MC_MR"):
        D = DistMatrix.from_global(A, layout, comm)
        V, w = sk.nla.approximate_symmetric_svd(D, 3, context=sk.Context(9), params=params, uplo="L")
        torch.testing.assert_close(w, w0, rtol=1e-8, atol=1e-8)
        torch.testing.assert_close(V.to_global().abs(), V0.abs(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(w0, torch.tensor([40.0, 20.0, 10.0], dtype=torch.float64), rtol=1e-6, atol=1e-6)
    return True


@pytest.mark.parametrize("world", [2, 4])
def test_symmetric_svd_distributed(world):
    run_distributed(_symsvd_worker, world)


def _lsrn_worker(rank, world):
    import libskylark_amd as sk
    from libskylark_amd.algorithms.krylov import KrylovIterParams
    from libskylark_amd.parallel.comm import world as W
    from libskylark_amd.parallel.distmatrix import DistMatrix
    comm = W()
    g = torch.Generator().manual_seed(5)
    m, n = 1600, 12
    U, _ = torch.linalg.qr(torch.randn(m, n, generator=g, dtype=torch.float64))
    V, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    A = (U * torch.logspace(0, 3, n, dtype=torch.float64)) @ V.t()       # cond 1e3
    b = torch.randn(m, 2, generator=g, dtype=torch.float64)
    ref = torch.linalg.lstsq(A, b).solution
    D = DistMatrix.from_global(A, "VC_STAR", comm)
    Bd = DistMatrix.from_global(b, "VC_STAR", comm)
    p = KrylovIterParams(tolerance=1e-12, iter_lim=300)
    comm.bytes_sent = 0
    xl = sk.nla.lsrn_least_squares(D, Bd, sk.Context(2), params=p)
    # A is never gathered: the traffic is the t x n sketch reduction plus
    # n-sized Krylov reductions, well under one rank's share of A
    assert comm.bytes_sent < A.numel() * 8 // world, comm.bytes_sent
    x1 = sk.nla.lsrn_least_squares(A, b, sk.Context(2), params=p)
    for x in (xl, x1):
        x = x.to_global() if hasattr(x, "to_global") else x
        r = float((A @ x - b).norm() / (A @ ref - b).norm())
        assert r < 1 + 1e-8, r
    return True


def test_lsrn_distributed_world8():
    """LSRN (JLT sketch of the row-sharded A -> one t x n all-reduce, QR/SVD
    preconditioner, preconditioned Krylov with all-reduced n-vectors) on 8
    ranks reaches the least-squares optimum like the one-process solve
    (reference accelerated_linearl2_regression_solver_Elemental.hpp:531-616)."""
    assert all(run_distributed(_lsrn_worker, 8))
