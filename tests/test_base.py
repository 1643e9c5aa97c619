"""Base layer: sparse containers, random matrices, cross-type BLAS, params.

Oracles follow the reference's unit tests: mixed sparse/dense GEMM in all
four orientations vs the dense product (tests/unit/MixedGemmTest.cpp:51-169),
distributed sparse Gemm vs dense (DistSparseTest.cpp:132-276), random
matrices identical across distributions (base/random_matrices.hpp global
indexing), and "distributed == local" for every distributed product.
"""
import io
import json

import numpy as np
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.base import blas as B
from libskylark_amd.base.sparse import DistSparseMatrix, GraphAdapter, SparseMatrix
from mp_utils import run_distributed


def _rand_sparse(m, n, density=0.2, seed=0):
    g = torch.Generator().manual_seed(seed)
    D = torch.randn(m, n, generator=g, dtype=torch.float64)
    D[torch.rand(m, n, generator=g) > density] = 0
    return D


# ------------------------------------------------------------- sparse
def test_sparse_set_sums_duplicates_and_transposes():
    S = SparseMatrix(4, 3).set([(0, 0, 1.0), (2, 1, 2.0), (0, 0, 3.0), (3, 2, -1.0)])
    assert S.nonzeros() == 3 and S.shape == (4, 3)
    D = torch.zeros(4, 3, dtype=torch.float64)
    D[0, 0], D[2, 1], D[3, 2] = 4.0, 2.0, -1.0
    assert torch.equal(S.to_dense(), D)
    assert torch.equal(S.transpose().to_dense(), D.t())
    assert torch.equal(S.to_torch("csr").to_dense(), D)
    assert S.copy() == S and S.copy() is not S


def test_sparse_attach_detach_scipy_roundtrip():
    import scipy.sparse as sp
    D = _rand_sparse(30, 20)
    M = sp.csc_matrix(D.numpy())
    S = SparseMatrix.from_scipy(M)
    assert torch.equal(S.to_dense(), D)
    assert (S.to_scipy() != M).nnz == 0
    T = SparseMatrix.from_torch(D)
    assert T == S
    ptr, idx, val = T.detach()
    assert T.nonzeros() == 0 and val.numel() == S.nonzeros()
    U = SparseMatrix().attach(ptr, idx, val, 30, 20, own=False)
    assert not U.owns_data() and U == S


def test_graph_adapter():
    A = SparseMatrix(3, 3).set([(0, 1, 1.0), (1, 0, 1.0), (2, 1, 1.0)])
    G = GraphAdapter(A)
    assert G.num_vertices() == 3
    assert G.degrees().tolist() == [1, 2, 0]
    assert sorted(G.neighbors(1).tolist()) == [0, 2]


# ------------------------------------------------------ random matrices
def test_random_matrix_global_indexing_and_counter():
    ctx = sk.Context(11)
    G = sk.base.GaussianMatrix(17, 9, ctx)
    assert ctx.counter == 17 * 9
    G2 = sk.base.GaussianMatrix(17, 9, sk.Context(11))
    assert torch.equal(G, G2)
    U = sk.base.UniformMatrix(50, 40, sk.Context(3), a=-2.0, b=2.0)
    assert float(U.min()) >= -2 and float(U.max()) <= 2
    with pytest.raises(sk.base.UnsupportedBaseOperation):
        sk.base.UniformMatrix(3, 3, sparse=True)


# ----------------------------------------------------------------- BLAS
@pytest.mark.parametrize("oA,oB", [("N", "N"), ("T", "N"), ("N", "T"), ("T", "T")])
@pytest.mark.parametrize("sparse_side", ["A", "B", "none"])
def test_gemm_mixed_orientations(oA, oB, sparse_side):
    A = _rand_sparse(12, 9, seed=1)
    Bm = _rand_sparse(9, 7, seed=2)
    A = A if oA == "N" else A.t().contiguous()
    Bm = Bm if oB == "N" else Bm.t().contiguous()
    ref = (A.t() if oA == "T" else A) @ (Bm.t() if oB == "T" else Bm)
    Ao = SparseMatrix.from_torch(A) if sparse_side == "A" else A
    Bo = SparseMatrix.from_torch(Bm) if sparse_side == "B" else Bm
    C = torch.ones_like(ref)
    out = B.Gemm(oA, oB, 2.0, Ao, Bo, 0.5, C)
    torch.testing.assert_close(out, 2.0 * ref + 0.5, rtol=1e-12, atol=1e-12)


def test_gemv_symm_trsm_qr_axpy_views():
    g = torch.Generator().manual_seed(4)
    A = torch.randn(8, 5, generator=g, dtype=torch.float64)
    x = torch.randn(5, generator=g, dtype=torch.float64)
    torch.testing.assert_close(B.Gemv("N", 1.0, A, x), A @ x)
    S = torch.randn(5, 5, generator=g, dtype=torch.float64)
    Sym = torch.tril(S) + torch.tril(S, -1).t()
    X = torch.randn(5, 3, generator=g, dtype=torch.float64)
    torch.testing.assert_close(B.Symm("L", "L", 1.0, torch.tril(S), X), Sym @ X)
    R = torch.triu(torch.randn(5, 5, generator=g, dtype=torch.float64)) + 5 * torch.eye(5, dtype=torch.float64)
    Y = torch.randn(5, 3, generator=g, dtype=torch.float64)
    Z = Y.clone()
    B.Trsm("L", "U", "N", "N", 1.0, R, Z)
    torch.testing.assert_close(R @ Z, Y)
    Q = A.clone()
    B.ExplicitUnitary(Q)
    torch.testing.assert_close(Q.t() @ Q, torch.eye(5, dtype=torch.float64), atol=1e-12, rtol=0)
    Yc = torch.zeros(8, 5, dtype=torch.float64)
    B.Axpy(torch.arange(5, dtype=torch.float64), A, Yc)
    torch.testing.assert_close(Yc, A * torch.arange(5, dtype=torch.float64))
    assert torch.equal(B.ColumnView(A, 1, 2), A[:, 1:3]) and torch.equal(B.RowView(A, 2, 3), A[2:5])
    assert B.Height(A) == 8 and B.Width(A) == 5
    torch.testing.assert_close(B.RowDot(A, A), (A * A).sum(1))


def test_computed_matrix_materialises_in_gemm():
    class Ones(B.ComputedMatrix):
        def height(self):
            return 4

        def width(self):
            return 3

        def materialize(self):
            return torch.ones(4, 3, dtype=torch.float64)

    X = torch.randn(3, 2, dtype=torch.float64)
    torch.testing.assert_close(B.Gemm("N", "N", 1.0, Ones(), X), torch.ones(4, 3, dtype=torch.float64) @ X)


def test_params_json_and_print_matrix():
    p = sk.base.Params(am_i_printing=True, log_level=2, prefix="[t] ", debug_level=2)
    q = sk.base.Params.from_json(p.to_json())
    assert q.log_level == 2 and q.prefix == "[t] "
    buf = io.StringIO()
    p.log_stream = buf
    p.log(1, "hello")
    p.log(3, "hidden")
    p.print_matrix(torch.eye(2), "I")
    out = buf.getvalue()
    assert "[t] hello" in out and "hidden" not in out and "I (2 x 2" in out
    assert json.loads(p.to_json())["debug_level"] == 2


# ---------------------------------------------------------- distributed
def _dist_blas_worker(rank, world):
    from libskylark_amd.parallel.distmatrix import DistMatrix
    from libskylark_amd.parallel.comm import world as W
    comm = W()
    g = torch.Generator().manual_seed(7)
    A = torch.randn(23, 6, generator=g, dtype=torch.float64)
    Bm = torch.randn(23, 4, generator=g, dtype=torch.float64)
    M = torch.randn(6, 5, generator=g, dtype=torch.float64)
    bad = []
    # [VC,*]^T [VC,*] -> [*,*]
    C = B.Gemm("T", "N", 1.0, DistMatrix.from_global(A, "VC_STAR", comm), DistMatrix.from_global(Bm, "VC_STAR", comm))
    if not torch.allclose(C.local, A.t() @ Bm):
        bad.append("tn")
    # [VC,*] [*,*] -> [VC,*]
    C = B.Gemm("N", "N", 1.0, DistMatrix.from_global(A, "VC_STAR", comm), M)
    if not torch.allclose(C.to_global(), A @ M):
        bad.append("nn-local")
    # [*,VC] [VC,*] -> [*,*]
    C = B.Gemm("N", "N", 1.0, DistMatrix.from_global(A.t().contiguous(), "STAR_VC", comm),
               DistMatrix.from_global(Bm, "VC_STAR", comm))
    if not torch.allclose(C.local, A.t() @ Bm):
        bad.append("star_vc x vc_star")
    # SUMMA [MC,MR] x [MC,MR]
    P = torch.randn(13, 11, generator=g, dtype=torch.float64)
    Q = torch.randn(11, 9, generator=g, dtype=torch.float64)
    for blk in (None, (2, 3)):
        Pd = DistMatrix.from_global(P, "MC_MR", comm, block=blk)
        Qd = DistMatrix.from_global(Q, "MC_MR", comm, block=(3, 2) if blk else None)
        C = B.Gemm("N", "N", 1.0, Pd, Qd)
        if not torch.allclose(C.to_global(), P @ Q):
            bad.append(("summa", blk))
    # general path: A^T of [MC,MR] times [MC,MR]
    C = B.Gemm("T", "N", 1.0, DistMatrix.from_global(A, "MC_MR", comm), DistMatrix.from_global(Bm, "MC_MR", comm))
    got = C.to_global() if isinstance(C, DistMatrix) else C
    if not torch.allclose(got, A.t() @ Bm):
        bad.append("general")
    # Gemv with all-reduce, ExplicitUnitary (TSQR), Trsm right on [VC,*]
    x = torch.randn(23, generator=g, dtype=torch.float64)
    y = B.Gemv("T", 1.0, DistMatrix.from_global(A, "VC_STAR", comm), DistMatrix.from_global(x.view(-1, 1), "VC_STAR", comm))
    if not torch.allclose(y.local.view(-1), A.t() @ x):
        bad.append("gemv")
    Ad = DistMatrix.from_global(A, "VC_STAR", comm)
    B.ExplicitUnitary(Ad)
    Qg = Ad.to_global()
    if not torch.allclose(Qg.t() @ Qg, torch.eye(6, dtype=torch.float64), atol=1e-12):
        bad.append("tsqr")
    # distributed sparse matrix from updates queued on every rank (duplicates summed)
    D = _rand_sparse(19, 8, seed=3)
    nz = D.nonzero()
    S = DistSparseMatrix(19, 8, "VC_STAR", comm)
    for t, (i, j) in enumerate(nz.tolist()):
        if t % world == rank:              # each entry queued by one rank, in halves
            S.queue_update(i, j, float(D[i, j]) / 2)
            S.queue_update(i, j, float(D[i, j]) / 2)
    Sd = S.finalize()
    if S.nonzeros() != nz.shape[0]:
        bad.append(("nnz", S.nonzeros(), nz.shape[0]))
    if not torch.allclose(Sd.to_global() if Sd.local.layout == torch.strided else
                          DistMatrix(Sd.local.to_dense(), Sd.shape, Sd.layout, comm).to_global(), D):
        bad.append("dist sparse")
    C = B.Gemm("T", "N", 1.0, Sd, DistMatrix.from_global(torch.ones(19, 2, dtype=torch.float64), "VC_STAR", comm))
    if not torch.allclose(C.local, D.t() @ torch.ones(19, 2, dtype=torch.float64)):
        bad.append("sparse tn")
    Sc = DistSparseMatrix(19, 8, "STAR_VR", comm)
    if rank == 0:
        Sc.queue_update(nz[:, 0], nz[:, 1], D[nz[:, 0], nz[:, 1]])
    Scd = Sc.finalize()
    full = DistMatrix(Scd.local.to_dense(), Scd.shape, Scd.layout, comm).to_global()
    if not torch.allclose(full, D):
        bad.append("star_vr sparse")
    # random matrices: every layout holds the same entries
    ref = sk.base.GaussianMatrix(14, 10, sk.Context(9))
    for lay in ("VC_STAR", "STAR_VC", "MC_MR", "STAR_STAR"):
        R = sk.base.GaussianMatrix(14, 10, sk.Context(9), layout=lay, comm=comm)
        if not torch.allclose(R.to_global(), ref.to(R.local.dtype)):
            bad.append(("random", lay))
    assert not bad, bad


@pytest.mark.parametrize("world", [2, 4])
def test_distributed_blas_and_sparse(world):
    run_distributed(_dist_blas_worker, world)
