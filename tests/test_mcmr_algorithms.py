"""[MC,MR] algorithms at world 4 (2 x 2) and 6 (2 x 3) on gloo/CPU: SUMMA with
its super-panel loop, and the three dense-sketch panel algorithms (inner
panel, outer panel, panel-matrix with a reduce-scatter) columnwise and
rowwise, against the single-process results (reference
``sketch/dense_transform_Elemental_mc_mr.hpp:87-656``, Elemental SUMMA)."""
import pytest
import torch

from mp_utils import run_distributed


def _summa_worker(rank, world, m, K, n, blockA, blockB):
    from libskylark_amd.base import blas as B
    from libskylark_amd.parallel.comm import world as W
    from libskylark_amd.parallel.distmatrix import DistMatrix, Grid
    comm = W()
    grid = Grid.default(comm)
    g = torch.Generator().manual_seed(1)
    A = torch.randn(m, K, generator=g, dtype=torch.float64)
    Bm = torch.randn(K, n, generator=g, dtype=torch.float64)
    DA = DistMatrix.from_global(A, "MC_MR", comm, grid=grid, block=blockA)
    DB = DistMatrix.from_global(Bm, "MC_MR", comm, grid=grid, block=blockB)
    C = B.Gemm("N", "N", 1.0, DA, DB)
    ref = DistMatrix.from_global(A @ Bm, "MC_MR", comm, grid=grid, block=C.block)
    assert C.layout == "MC_MR" and C.local.shape == ref.local.shape
    assert torch.allclose(C.local, ref.local, atol=1e-10), (C.local - ref.local).abs().max()
    return True


@pytest.mark.parametrize("world,m,K,n,bA,bB", [(4, 37, 53, 29, (5, 4), (4, 6)), (6, 40, 61, 33, (3, 7), (2, 5)),
                                                (4, 16, 8, 12, (4, 4), (4, 4))])
def test_summa_panel_loop(world, m, K, n, bA, bB):
    assert all(run_distributed(_summa_worker, world, m, K, n, bA, bB))


def _sketch_worker(rank, world, algo, dim, kind):
    import libskylark_amd as sk
    from libskylark_amd.parallel.comm import world as W
    from libskylark_amd.parallel.distmatrix import DistMatrix, Grid
    from libskylark_amd.sketch import params
    comm = W()
    grid = Grid.default(comm)
    N, w, S = 240, 14, 10
    g = torch.Generator().manual_seed(2)
    A = torch.randn(N, w, generator=g, dtype=torch.float64) if dim == 0 else \
        torch.randn(w, N, generator=g, dtype=torch.float64)
    if kind == "JLT":
        T = sk.sketch.JLT(N, S, context=sk.Context(5))
    else:
        T = sk.sketch.GaussianRFT(N, S, sigma=3.0, context=sk.Context(5))
    ref = T.apply(A, dim=dim)
    D = DistMatrix.from_global(A, "MC_MR", comm, grid=grid, block=(7, 3) if dim == 0 else (3, 7))
    from libskylark_amd.parallel import dist_sketch as DS
    called = []
    for name in ("_inner_panel", "_outer_panel", "_panel_matrix"):
        orig = getattr(DS, name)
        setattr(DS, name, (lambda f, nm: (lambda *a, **k: (called.append(nm), f(*a, **k))[1]))(orig, name))
    params.set_mc_mr_algorithm(algo)
    try:
        R = T.apply(D, dim=dim)
    finally:
        params.set_mc_mr_algorithm("auto")
    want = {"inner": "_inner_panel", "outer": "_outer_panel" if dim == 0 else "_panel_matrix",
            "panel": "_panel_matrix"}.get(algo)
    if want is not None:
        assert called == [want], called
    full = R.to_global() if isinstance(R, DistMatrix) else R
    assert torch.allclose(full, ref, atol=1e-10), (full - ref).abs().max()
    return True


@pytest.mark.parametrize("algo", ["inner", "outer", "panel", "auto"])
@pytest.mark.parametrize("dim", [0, 1])
def test_mc_mr_sketch_algorithms(algo, dim):
    assert all(run_distributed(_sketch_worker, 4, algo, dim, "JLT"))


@pytest.mark.parametrize("dim", [0, 1])
def test_mc_mr_feature_map_panel_reduce_scatter(dim):
    assert all(run_distributed(_sketch_worker, 6, "panel", dim, "RFT"))
