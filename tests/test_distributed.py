"""Multi-process (gloo, CPU) tests of the distributed paths: every layout x
sketch family equals the local result; comm primitives; distributed randSVD,
LSQR and least squares equal their single-process answers.

The reference tests these by running its C++/Python suites under mpirun
(SURVEY.md 4); here ranks are spawned processes on 127.0.0.1.
"""
import pytest
import torch

from mp_utils import run_distributed

LAYOUTS = ["VC_STAR", "VR_STAR", "STAR_VC", "STAR_VR", "MC_MR", "CIRC_CIRC", "STAR_STAR"]
SKETCHES = [("JLT", {}), ("CT", {"C": 2.0}), ("CWT", {}), ("MMT", {}), ("FJLT", {}), ("GaussianRFT", {"sigma": 2.0}),
            ("PPT", {"q": 2, "c": 1.0, "gamma": 0.5}), ("FastGaussianRFT", {"sigma": 2.0})]


def _world():
    from libskylark_amd.parallel.comm import world
    return world()


def _sketch_worker(rank, world):
    import libskylark_amd as sk
    from libskylark_amd.parallel.distmatrix import DistMatrix
    comm = _world()
    g = torch.Generator().manual_seed(0)
    A = torch.randn(37, 23, generator=g, dtype=torch.float64)
    bad = []
    for name, kw in SKETCHES:
        cls = sk.sketch.base.sketch_class(name)
        for dim, n, s in ((sk.sketch.COLUMNWISE, 37, 16), (sk.sketch.ROWWISE, 23, 16)):
            S = cls(n, s, context=sk.Context(5), **kw)
            ref = S.apply(A, dim=dim)
            for lay in LAYOUTS:
                D = DistMatrix.from_global(A, lay, comm)
                out = S.apply(D, dim=dim)
                got = out.to_global() if isinstance(out, DistMatrix) else out
                if not torch.allclose(got, ref, rtol=1e-9, atol=1e-9):
                    bad.append((name, dim, lay, float((got - ref).abs().max())))
    assert not bad, bad


@pytest.mark.parametrize("world", [2, 3])
def test_dist_sketch_equals_local(world):
    run_distributed(_sketch_worker, world)


def _comm_worker(rank, world):
    from libskylark_amd.parallel.comm import balanced_counts
    comm = _world()
    t = torch.full((3,), float(rank + 1))
    comm.all_reduce(t)
    assert t.tolist() == [sum(range(1, world + 1))] * 3
    counts = balanced_counts(10, world)
    mine = torch.arange(sum(counts[:rank]), sum(counts[:rank + 1]), dtype=torch.float64)[:, None]
    assert comm.all_gather_v(mine, counts)[:, 0].tolist() == list(range(10))
    full = torch.arange(10, dtype=torch.float64)[:, None] * (rank + 1)
    rs = comm.reduce_scatter_v(full, counts)
    tot = sum(range(1, world + 1))
    assert rs[:, 0].tolist() == [tot * v for v in range(sum(counts[:rank]), sum(counts[:rank + 1]))]
    sends = [torch.full((r + 1, 2), float(rank * 10 + r)) for r in range(world)]
    recv = comm.all_to_all_v(sends)
    for src, rt in enumerate(recv):
        assert rt.shape == (rank + 1, 2) and float(rt[0, 0]) == src * 10 + rank
    b = torch.tensor([float(rank)])
    comm.broadcast(b, root=world - 1)
    assert float(b) == world - 1
    sub = comm.split(rank % 2)
    assert sub.size == len([r for r in range(world) if r % 2 == rank % 2])


@pytest.mark.parametrize("world", [2, 3])
def test_comm_primitives(world):
    run_distributed(_comm_worker, world)


def _svd_worker(rank, world):
    import libskylark_amd as sk
    from libskylark_amd.parallel.distmatrix import DistMatrix
    comm = _world()
    g = torch.Generator().manual_seed(1)
    U0, _ = torch.linalg.qr(torch.randn(400, 6, generator=g, dtype=torch.float64))
    V0, _ = torch.linalg.qr(torch.randn(50, 6, generator=g, dtype=torch.float64))
    s0 = torch.tensor([9.0, 7, 5, 3, 2, 1], dtype=torch.float64)
    A = (U0 * s0) @ V0.t()
    p = sk.nla.ApproximateSVDParams(num_iterations=2)
    U, s, V = sk.nla.approximate_svd(DistMatrix.from_global(A, "VC_STAR", comm), 6, sk.Context(3), p)
    torch.testing.assert_close(s, s0, rtol=1e-8, atol=1e-8)
    Ug = U.to_global() if isinstance(U, DistMatrix) else U
    torch.testing.assert_close((Ug * s) @ V.t(), A, rtol=1e-7, atol=1e-7)
    # LSQR / Blendenpik over row-distributed A == local solution
    B = torch.randn(400, 2, generator=g, dtype=torch.float64)
    Ad = DistMatrix.from_global(A + 0.1 * torch.eye(400, 50, dtype=torch.float64), "VC_STAR", comm)
    Al = Ad.to_global()
    X, code = sk.algorithms.lsqr(Ad, B, params=sk.algorithms.KrylovIterParams(tolerance=1e-14, iter_lim=500))
    torch.testing.assert_close(X, torch.linalg.lstsq(Al, B).solution, rtol=1e-7, atol=1e-7)
    Xf = sk.nla.faster_least_squares(Ad, B, sk.Context(4))
    torch.testing.assert_close(Xf, torch.linalg.lstsq(Al, B).solution, rtol=1e-7, atol=1e-7)


def test_dist_randsvd_and_lsqr():
    run_distributed(_svd_worker, 2)


def _krr_worker(rank, world):
    import libskylark_amd as sk
    from libskylark_amd import ml
    from libskylark_amd.parallel.distmatrix import DistMatrix
    comm = _world()
    g = torch.Generator().manual_seed(2)
    X = torch.randn(120, 3, generator=g, dtype=torch.float64)
    Y = torch.sin(X[:, :1])
    k = ml.Gaussian(3, 1.0)
    Xd = DistMatrix.from_global(X, "VC_STAR", comm)
    p = ml.KrrParams(tolerance=1e-11, iter_lim=500)
    A_loc = ml.faster_kernel_ridge(k, Xd, Y, 0.1, 40, sk.Context(1), params=p)
    A = comm.all_gather_v(A_loc.contiguous(), Xd.row_counts())
    torch.testing.assert_close(A, ml.kernel_ridge(k, X, Y, 0.1), rtol=1e-7, atol=1e-8)
    S, W = ml.approximate_kernel_ridge(k, Xd, Y, 0.1, 64, sk.Context(2))
    S2, W2 = ml.approximate_kernel_ridge(k, X, Y, 0.1, 64, sk.Context(2))
    torch.testing.assert_close(W, W2, rtol=1e-9, atol=1e-9)


def test_dist_krr():
    run_distributed(_krr_worker, 2)


def _outer_panel_worker(rank, world):
    import libskylark_amd as sk
    from libskylark_amd.parallel.distmatrix import DistMatrix
    from libskylark_amd.parallel import dist_sketch as DS
    comm = _world()
    g = torch.Generator().manual_seed(1)
    A = torch.randn(30, 11, generator=g, dtype=torch.float64)
    bad = []
    for S, blk in ((60, None), (60, (4, 3)), (8, None)):
        T = sk.sketch.JLT(30, S, context=sk.Context(2))
        ref = T.apply(A, dim=0)
        D = DistMatrix.from_global(A, "MC_MR", comm, block=blk)
        used_outer = DS._use_outer_panel(T, D, 0, "linear")
        got = T.apply(D, dim=0).to_global()
        if not torch.allclose(got, ref, rtol=1e-10, atol=1e-10):
            bad.append((S, blk, used_outer))
        if S == 60 and not used_outer:
            bad.append(("outer not selected", S))
        if S == 8 and used_outer:
            bad.append(("outer selected", S))
    sk.sketch.params.set_factor(1000)     # the knob moves the selection
    if DS._use_outer_panel(sk.sketch.JLT(30, 60, context=sk.Context(2)), DistMatrix.from_global(A, "MC_MR", comm), 0,
                           "linear"):
        bad.append("factor ignored")
    sk.sketch.params.set_factor(20)
    assert not bad, bad


def test_mc_mr_outer_panel_equals_local():
    run_distributed(_outer_panel_worker, 4)


def test_blocksize_knob_keeps_results():
    import libskylark_amd as sk
    A = torch.randn(500, 7, dtype=torch.float64)
    T = sk.sketch.JLT(500, 40, context=sk.Context(4))
    ref = T * A
    sk.sketch.params.set_blocksize(37)
    try:
        assert torch.allclose(T * A, ref, rtol=1e-12, atol=1e-12)
    finally:
        sk.sketch.params.set_blocksize(0)
