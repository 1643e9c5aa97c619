"""Layout redistribution at world = 8 (a 2 x 4 grid, gloo on CPU): every
(src, dst) layout pair reproduces the global matrix exactly, and the
all-to-all moves at most a rank's own shard (the reference
redistributes implicitly inside Elemental, e.g. ``A1_VC_STAR = A1`` in
``sketch/dense_transform_Elemental_mc_mr.hpp:287``)."""
import pytest
import torch

from mp_utils import run_distributed

LAYOUTS = ["VC_STAR", "STAR_VC", "MC_MR", "CIRC_CIRC", "STAR_STAR"]


def _redist_worker(rank, world, m, n, block):
    from libskylark_amd.parallel.comm import world as W
    from libskylark_amd.parallel.distmatrix import DistMatrix, Grid
    comm = W()
    grid = Grid.default(comm)
    A = torch.arange(m * n, dtype=torch.float64).view(m, n)
    bad = []
    for src in LAYOUTS:
        D = DistMatrix.from_global(A, src, comm, grid=grid if src == "MC_MR" else None,
                                   block=block if src == "MC_MR" else None)
        for dst in LAYOUTS:
            comm.bytes_sent = 0
            R = D.redistribute(dst, grid=grid if dst == "MC_MR" else None, block=block if dst == "MC_MR" else None)
            sent = comm.bytes_sent
            ref = DistMatrix.from_global(A, dst, comm, grid=R.grid, block=R.block)
            if R.local.shape != ref.local.shape or not torch.equal(R.local, ref.local):
                bad.append((src, dst, "values"))
            # a rank sends at most its own shard, except towards replication
            if dst != "STAR_STAR" and src != "STAR_STAR":
                own = D.local.numel() * D.local.element_size()
                if sent > own:
                    bad.append((src, dst, "bytes", sent, own))
            if src == "STAR_STAR" and sent:
                bad.append((src, dst, "replicated source communicated", sent))
    assert not bad, bad
    return grid.pr, grid.pc


@pytest.mark.parametrize("m,n,block", [(53, 29, None), (64, 40, (4, 3)), (37, 11, (1, 1))])
def test_redistribute_world8(m, n, block):
    res = run_distributed(_redist_worker, 8, m, n, block)
    assert res[0] == (2, 4)


def _mcmr_bytes_worker(rank, world):
    """[MC,MR] -> [VC,*] of a tall matrix: bytes per rank <= m n / p (own shard)."""
    from libskylark_amd.parallel.comm import world as W
    from libskylark_amd.parallel.distmatrix import DistMatrix
    comm = W()
    m, n = 4096, 96
    D = DistMatrix.random((m, n), "MC_MR", comm, seed=3, dtype=torch.float32, block=(128, 12))
    comm.bytes_sent = 0
    R = D.redistribute("VC_STAR")
    sent = comm.bytes_sent
    assert sent <= m * n * 4 // world
    # the row shard equals the globally indexed random matrix
    ref = DistMatrix.random((m, n), "VC_STAR", comm, seed=3, dtype=torch.float32)
    assert torch.equal(R.local, ref.local)
    # second call reuses the cached plan and gives the same bytes
    comm.bytes_sent = 0
    R2 = D.redistribute("VC_STAR")
    assert comm.bytes_sent == sent and torch.equal(R2.local, R.local)
    return sent


def test_mcmr_to_vcstar_bytes_bounded():
    sent = run_distributed(_mcmr_bytes_worker, 8)
    assert max(sent) <= 4096 * 96 * 4 // 8


def _rs_worker(rank, world):
    from libskylark_amd.parallel.comm import world as W
    comm = W()
    counts = [3, 1, 0, 2, 5, 1, 1, 2][:world]
    tot = sum(counts)
    full = torch.arange(tot * 2, dtype=torch.float64).view(tot, 2) * (rank + 1)
    comm.bytes_sent = 0
    out = comm.reduce_scatter_v(full, counts)
    s = sum(range(1, world + 1))
    off = sum(counts[:rank])
    assert torch.equal(out, torch.arange(tot * 2, dtype=torch.float64).view(tot, 2)[off:off + counts[rank]] * s)
    # padded reduce-scatter: never an all-reduce of the whole operand
    assert comm.bytes_sent <= max(counts) * 2 * 8 * world


def test_reduce_scatter_unequal_world8():
    run_distributed(_rs_worker, 8)


def _svd_mcmr_worker(rank, world):
    """randSVD of a [MC,MR] operand on a 2 x 4 grid == single-process randSVD;
    U comes back in A's [MC,MR] layout (reference UType follows A)."""
    import libskylark_amd as sk
    from libskylark_amd.parallel.comm import world as W
    from libskylark_amd.parallel.distmatrix import DistMatrix
    comm = W()
    g = torch.Generator().manual_seed(1)
    m, n, r = 600, 40, 5
    A = (torch.randn(m, r, generator=g, dtype=torch.float64) * torch.tensor([50., 30., 20., 10., 5.], dtype=torch.float64)) \
        @ torch.randn(r, n, generator=g, dtype=torch.float64) + 0.01 * torch.randn(m, n, generator=g, dtype=torch.float64)
    params = sk.nla.ApproximateSVDParams(num_iterations=2)
    U0, s0, V0 = sk.nla.approximate_svd(A, r, context=sk.Context(7), params=params)
    D = DistMatrix.from_global(A, "MC_MR", comm, block=(16, 8))
    U, s, V = sk.nla.approximate_svd(D, r, context=sk.Context(7), params=params)
    assert isinstance(U, DistMatrix) and U.layout == "MC_MR" and U.shape == (m, r)
    torch.testing.assert_close(s, s0, rtol=1e-9, atol=1e-9)
    torch.testing.assert_close(V.abs(), V0.abs(), rtol=1e-7, atol=1e-9)
    torch.testing.assert_close(U.to_global().abs(), U0.abs(), rtol=1e-7, atol=1e-9)
    # wide operand: U follows A's layout, V is gathered
    Dw = DistMatrix.from_global(A.t().contiguous(), "MC_MR", comm, block=(8, 16))
    Uw, sw, Vw = sk.nla.approximate_svd(Dw, r, context=sk.Context(7), params=params)
    assert isinstance(Uw, DistMatrix) and Uw.layout == "MC_MR" and Uw.shape == (n, r)
    assert torch.is_tensor(Vw) and Vw.shape == (m, r)
    torch.testing.assert_close(sw, s0, rtol=1e-9, atol=1e-9)
    # 8 x 1 grid (bench.py's strong-scaling grid for a tall-skinny A): the
    # cyclic row tiles are read in place -- only the small (n + k) x k
    # reductions touch the wire, never a share of A
    from libskylark_amd.parallel.distmatrix import Grid
    g81 = Grid.default(comm, world)
    D8 = DistMatrix.from_global(A, "MC_MR", comm, grid=g81, block=(16, 8))
    def _no_a2a(*a, **k):
        raise AssertionError("the 8 x 1 grid must not redistribute A")
    a2a, comm.all_to_all_v = comm.all_to_all_v, _no_a2a
    try:
        U8, s8, V8 = sk.nla.approximate_svd(D8, r, context=sk.Context(7), params=params)
    finally:
        comm.all_to_all_v = a2a
    assert isinstance(U8, DistMatrix) and U8.layout == "MC_MR" and U8.grid is g81 and U8.shape == (m, r)
    assert U8.local.shape == (D8.local.shape[0], r)
    torch.testing.assert_close(s8, s0, rtol=1e-9, atol=1e-9)
    torch.testing.assert_close(V8.abs(), V0.abs(), rtol=1e-7, atol=1e-9)
    torch.testing.assert_close(U8.to_global().abs(), U0.abs(), rtol=1e-7, atol=1e-9)


def test_randsvd_mcmr_world8():
    run_distributed(_svd_mcmr_worker, 8)


def _bench_matrix_worker(rank, world):
    """bench.py's planted matrix: [MC,MR] tiles on 8 ranks == the one-rank matrix."""
    import importlib.util
    import os
    from libskylark_amd.parallel.comm import Comm, world as W
    from libskylark_amd.parallel.distmatrix import DistMatrix, Grid
    spec = importlib.util.spec_from_file_location(
        "bench", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    comm = W()
    dev = torch.device("cpu")
    m, n = 300, 48
    D = bench.planted_matrix((m, n), "MC_MR", comm, dev, Grid.default(comm), (32, 8))
    full = bench.planted_matrix((m, n), "VC_STAR", Comm.single(), dev)
    assert torch.equal(D.to_global(), full.local)
    return True


def test_bench_planted_matrix_world8():
    run_distributed(_bench_matrix_worker, 8)
