"""2-D block-sparse distribution (CombBLAS SpParMat analogue) at world 4 (2 x 2)
and 6 (2 x 3) on gloo/CPU: COO assembly through one all-to-all, A X / A^T Y
with the grid-row / grid-column reductions, and hash / dense / generic
sketches of the distributed matrix against single-process results
(reference ``base/detail/combblas_mixed_gemm.hpp``,
``sketch/hash_transform_CombBLAS.hpp``)."""
import pytest
import torch

from mp_utils import run_distributed


def _matrix(m, n, density=0.08, seed=3):
    g = torch.Generator().manual_seed(seed)
    D = torch.randn(m, n, generator=g, dtype=torch.float64)
    D[torch.rand(m, n, generator=g) > density] = 0.0
    return D


def _worker(rank, world, m, n, block, what):
    import libskylark_amd as sk
    from libskylark_amd.parallel.comm import world as W
    from libskylark_amd.parallel.dist_sparse2d import COLUMNWISE, ROWWISE, DistSparse2D
    from libskylark_amd.parallel.distmatrix import Grid
    comm = W()
    grid = Grid.default(comm)
    A = _matrix(m, n)
    if what == "assemble":
        # every rank contributes a scattered, overlapping share of the triples
        coo = A.to_sparse().coalesce()
        r, c = coo.indices()
        v = coo.values()
        pick = torch.arange(r.numel()) % world == rank
        # split each picked value in two halves (duplicates must be summed)
        rr = torch.cat([r[pick], r[pick]])
        cc = torch.cat([c[pick], c[pick]])
        vv = torch.cat([0.25 * v[pick], 0.75 * v[pick]])
        M = DistSparse2D.from_local_coo(rr, cc, vv, (m, n), comm, grid, block)
        assert M.nnz() == coo.values().numel()
        assert torch.allclose(M.to_global(), A, atol=1e-14)
        return True
    M = DistSparse2D.from_global(A.to_sparse_csr(), comm, grid, block)
    assert torch.equal(M.to_global(), A)
    if what == "products":
        g = torch.Generator().manual_seed(9)
        X = torch.randn(n, 5, generator=g, dtype=torch.float64)
        Y = torch.randn(m, 3, generator=g, dtype=torch.float64)
        AX = M.matmul(X)
        assert torch.allclose(AX, (A @ X)[M.rows], atol=1e-12)
        assert torch.allclose(M.gather_rows(AX), A @ X, atol=1e-12)
        AtY = M.rmatmul(Y)
        assert torch.allclose(AtY, (A.t() @ Y)[M.cols], atol=1e-12)
        assert torch.allclose(M.gather_cols(AtY), A.t() @ Y, atol=1e-12)
        return True
    S = 7
    ctx = sk.Context(11)
    for kind in ("CWT", "WZT", "JLT", "FJLT"):
        for dim in (COLUMNWISE, ROWWISE):
            N = m if dim == COLUMNWISE else n
            T = {"CWT": lambda: sk.sketch.CWT(N, S, context=ctx),
                 "WZT": lambda: sk.sketch.WZT(N, S, p=1.5, context=ctx),
                 "JLT": lambda: sk.sketch.JLT(N, S, context=ctx),
                 "FJLT": lambda: sk.sketch.FJLT(N, S, context=ctx)}[kind]()
            ref = T.apply(A, dim=dim)
            ref = ref.to_dense() if ref.layout != torch.strided else ref
            got = T.apply(M, dim=dim) if kind == "CWT" else M.sketch(T, dim)
            want = ref[:, M.cols] if dim == COLUMNWISE else ref[M.rows]
            assert got.shape == want.shape, (kind, dim, got.shape, want.shape)
            assert torch.allclose(got, want, atol=1e-10), (kind, dim, (got - want).abs().max())
    return True


@pytest.mark.parametrize("world,m,n,block", [(4, 53, 41, (5, 4)), (6, 47, 38, (3, 7)), (4, 20, 16, (64, 64))])
@pytest.mark.parametrize("what", ["assemble", "products", "sketch"])
def test_dist_sparse2d(world, m, n, block, what):
    assert all(run_distributed(_worker, world, m, n, block, what))


def test_dist_sparse2d_single_process():
    from libskylark_amd.parallel.comm import Comm
    from libskylark_amd.parallel.dist_sparse2d import DistSparse2D
    from libskylark_amd.parallel.distmatrix import Grid
    A = _matrix(30, 12)
    comm = Comm(None)
    M = DistSparse2D.from_global(A, comm, Grid(comm), (4, 4))
    X = torch.randn(12, 2, dtype=torch.float64)
    assert torch.allclose(M.matmul(X), A @ X, atol=1e-12)
    assert torch.equal(M.to_global(), A)


def _lsqr_worker(rank, world):
    from libskylark_amd.algorithms import krylov
    from libskylark_amd.parallel.comm import world as W
    from libskylark_amd.parallel.dist_sparse2d import DistSparse2D
    from libskylark_amd.parallel.distmatrix import Grid
    comm = W()
    A = _matrix(90, 12, density=0.3, seed=4)
    A += torch.eye(90, 12, dtype=torch.float64)          # full column rank
    B = torch.randn(90, 2, generator=torch.Generator().manual_seed(5), dtype=torch.float64)
    M = DistSparse2D.from_global(A.to_sparse_csr(), comm, Grid.default(comm), (7, 5))
    params = krylov.KrylovIterParams(tolerance=1e-12, iter_lim=300)
    X, code = krylov.lsqr(M, B, params=params)
    ref = torch.linalg.lstsq(A, B).solution
    assert torch.allclose(X, ref, atol=1e-8), (X - ref).abs().max()
    return True


@pytest.mark.parametrize("world", [4, 6])
def test_lsqr_on_2d_sparse(world):
    assert all(run_distributed(_lsqr_worker, world))
