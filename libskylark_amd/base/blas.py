"""Cross-type dense / sparse / distributed BLAS: ``Gemm``, ``Gemv``, ``Symm``,
``Trsm``, explicit-Q ``QR``, ``Axpy``, views, ``DenseCopy``, shape queries.

Reference: ``base/Gemm.hpp:19-583`` (local dense, sparse x dense in all four
orientations, ``[VC,*]^T [VC,*] -> [*,*]`` by local GEMM + all-reduce
(``:84-103``), ``[VC,*] [*,*] -> [VC,*]`` communication-free, computed
matrices materialised on demand ``:541-583``), ``base/Gemv.hpp`` (all-reduce
of ``A^T x``, ``:59``), ``base/Symm.hpp`` (sparse-local, sparse ``[VC,*]``
with broadcasts ``:217-222``), ``base/Trsm.hpp``, ``base/QR.hpp:11-36``
(``ExplicitUnitary``, TSQR for ``[VC,*]``), ``base/basic.hpp:48-70``
(``Axpy`` incl. per-column alphas), ``base/viewing.hpp``, ``base/copy.hpp``,
``base/query.hpp``.

Operands: torch tensors (dense or sparse CSR/CSC/COO, any device),
:class:`~libskylark_amd.base.sparse.SparseMatrix`,
:class:`~libskylark_amd.parallel.DistMatrix` (dense or sparse local shard),
and :class:`ComputedMatrix`.  Orientation flags follow Elemental:
``"N"`` (normal), ``"T"`` (transpose), ``"C"`` (adjoint; = T for real data).

MI355X mapping: local products are hipBLASLt GEMMs / hipSPARSE SpMM through
torch on the tensor's device; distributed products need exactly one RCCL
collective (all-reduce of the ``k x n`` result for ``[VC,*]^T [VC,*]``, an
all-gather of the replicated operand for ``[MC,MR]`` SUMMA panels), sized so
the big operand never moves.
"""
from __future__ import annotations

import torch

from .exceptions import DimensionMismatchError, UnsupportedBaseOperation


# ------------------------------------------------------------------ helpers
class ComputedMatrix:
    """Lazily materialised matrix (``base/computed_matrix.hpp:17-26``):
    sub-classes implement ``height``, ``width`` and ``materialize``."""

    def height(self) -> int:
        raise NotImplementedError

    def width(self) -> int:
        raise NotImplementedError

    def materialize(self) -> torch.Tensor:
        raise NotImplementedError


def _is_dist(X):
    from ..parallel.distmatrix import DistMatrix
    return isinstance(X, DistMatrix)


def _as_tensor(X):
    from .sparse import SparseMatrix
    if isinstance(X, ComputedMatrix):
        return X.materialize()
    if isinstance(X, SparseMatrix):
        return X.to_torch("csr")
    return X


def _op(X: torch.Tensor, o: str) -> torch.Tensor:
    o = o.upper()
    if o == "N":
        return X
    if o in ("T", "C"):
        if X.layout == torch.strided:
            Xt = X.t()
            return Xt.conj() if (o == "C" and X.is_complex()) else Xt
        return X.t()   # sparse: transpose view (CSR <-> CSC)
    raise ValueError(f"orientation must be N, T or C (got {o})")


def _mm(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """Local product with sparse operands allowed on either side."""
    if A.layout != torch.strided and B.layout != torch.strided:
        return torch.sparse.mm(A, B.to_dense()) if A.layout != torch.sparse_csc else torch.sparse.mm(
            A.to_sparse_csr(), B.to_dense())
    if A.layout != torch.strided:
        A = A if A.layout in (torch.sparse_csr, torch.sparse_coo) else A.to_sparse_csr()
        return torch.sparse.mm(A, B)
    if B.layout != torch.strided:
        Bt = B.t()
        Bt = Bt if Bt.layout in (torch.sparse_csr, torch.sparse_coo) else Bt.to_sparse_csr()
        return torch.sparse.mm(Bt, A.t()).t()
    return A @ B


def Height(X) -> int:
    if isinstance(X, ComputedMatrix):
        return X.height()
    return int(X.shape[0])


def Width(X) -> int:
    if isinstance(X, ComputedMatrix):
        return X.width()
    return int(X.shape[1])


# ---------------------------------------------------------------------- Gemm
def Gemm(oA: str, oB: str, alpha, A, B, beta=0.0, C=None):
    """``C = alpha op(A) op(B) + beta C`` across operand types; returns C.

    Distributed cases (reference ``base/Gemm.hpp`` / ``dist_mixed_gemm.hpp``):

    * ``[VC,*]^T [VC,*] -> [*,*]``: local GEMM + one all-reduce;
    * ``[VC,*] [*,*] -> [VC,*]`` (and local replicated B): no communication;
    * ``[*,VC] [VC,*] -> [*,*]``: local GEMM + all-reduce;
    * ``[MC,MR] x [MC,MR] -> [MC,MR]``: SUMMA over row / column panels;
    * anything else: redistribute to a supported pairing (all-to-all)."""
    if _is_dist(A) or _is_dist(B) or _is_dist(C):
        return _gemm_dist(oA, oB, alpha, A, B, beta, C)
    A, B = _as_tensor(A), _as_tensor(B)
    P = _mm(_op(A, oA), _op(B, oB))
    if P.layout != torch.strided:
        P = P.to_dense()
    if alpha != 1.0:
        P = P * alpha
    if C is None:
        return P
    if C.shape != P.shape:
        raise DimensionMismatchError(f"Gemm: C is {tuple(C.shape)}, product is {tuple(P.shape)}")
    if beta == 0.0:
        C.copy_(P)
    else:
        C.mul_(beta).add_(P.to(C.dtype))
    return C


def _gemm_dist(oA, oB, alpha, A, B, beta, C):
    from ..parallel.distmatrix import DistMatrix, is_col_dist, is_row_dist
    tA, tB = oA.upper() != "N", oB.upper() != "N"
    dA, dB = _is_dist(A), _is_dist(B)
    comm = (A if dA else B).comm
    out = None
    if dA and dB and is_row_dist(A.layout) and is_row_dist(B.layout) and tA and not tB:
        # [VC,*]^T [VC,*] -> [*,*]: local partial + all-reduce (base/Gemm.hpp:84-103)
        P = _mm(_op(_as_tensor(A.local), "T"), _as_tensor(B.local))
        P = (P.to_dense() if P.layout != torch.strided else P).contiguous()
        comm.all_reduce(P)
        out = DistMatrix(P, (A.shape[1], B.shape[1]), "STAR_STAR", comm)
    elif dA and is_row_dist(A.layout) and not tA and (not dB or B.layout == "STAR_STAR"):
        # [VC,*] [*,*] -> [VC,*]: communication free
        Bl = _op(_as_tensor(B.local if dB else B), oB)
        P = _mm(_as_tensor(A.local), Bl)
        P = P.to_dense() if P.layout != torch.strided else P
        out = DistMatrix(P, (A.shape[0], Bl.shape[1]), A.layout, comm)
    elif dA and dB and is_col_dist(A.layout) and is_row_dist(B.layout) and not tA and not tB:
        # [*,VC] [VC,*] -> [*,*]: contraction over the distributed index
        P = _mm(_as_tensor(A.local), _as_tensor(B.local))
        P = (P.to_dense() if P.layout != torch.strided else P).contiguous()
        comm.all_reduce(P)
        out = DistMatrix(P, (A.shape[0], B.shape[1]), "STAR_STAR", comm)
    elif dA and dB and A.layout == "MC_MR" and B.layout == "MC_MR" and not tA and not tB:
        out = _summa(A, B)
    elif dA and dB and A.layout == "STAR_STAR" and B.layout == "STAR_STAR":
        P = _mm(_op(_as_tensor(A.local), oA), _op(_as_tensor(B.local), oB))
        out = DistMatrix(P.to_dense() if P.layout != torch.strided else P,
                         (P.shape[0], P.shape[1]), "STAR_STAR", comm)
    elif dA and not dB and A.layout == "STAR_STAR":
        P = _mm(_op(_as_tensor(A.local), oA), _op(_as_tensor(B), oB))
        out = DistMatrix(P.to_dense() if P.layout != torch.strided else P, tuple(P.shape), "STAR_STAR", comm)
    else:
        # general: bring operands to a supported pairing
        if dA and A.local.layout != torch.strided:
            raise UnsupportedBaseOperation(f"Gemm {oA}{oB} with sparse {A.layout} operand")
        if tA and dA and not is_row_dist(A.layout):
            return _gemm_dist(oA, oB, alpha, A.redistribute("VC_STAR"), B, beta, C)
        if not tA and dA and not is_row_dist(A.layout) and A.layout != "STAR_STAR":
            return _gemm_dist(oA, oB, alpha, A.redistribute("VC_STAR"), B, beta, C)
        if dB and B.layout != "STAR_STAR" and not (tA and is_row_dist(B.layout)):
            return _gemm_dist(oA, oB, alpha, A, B.redistribute("STAR_STAR"), beta, C)
        if tA and dB and not is_row_dist(B.layout):
            return _gemm_dist(oA, oB, alpha, A, B.redistribute("VC_STAR"), beta, C)
        if not dA:
            A = DistMatrix(_as_tensor(A), tuple(A.shape), "STAR_STAR", comm)
            return _gemm_dist(oA, oB, alpha, A, B, beta, C)
        if not dB:
            B = DistMatrix(_as_tensor(B), tuple(B.shape), "STAR_STAR", comm)
            return _gemm_dist(oA, oB, alpha, A, B, beta, C)
        raise UnsupportedBaseOperation(f"Gemm {oA}{oB} {A.layout} x {getattr(B, 'layout', 'local')}")
    if alpha != 1.0:
        out.local = out.local * alpha
    if C is None:
        return out
    Cd = C if _is_dist(C) else None
    if Cd is not None and Cd.layout != out.layout:
        out = out.redistribute(Cd.layout, Cd.grid, Cd.block)
    target = Cd.local if Cd is not None else C
    if beta == 0.0:
        target.copy_(out.local)
    else:
        target.mul_(beta).add_(out.local.to(target.dtype))
    return C


def _summa(A, B):
    """``[MC,MR] x [MC,MR] -> [MC,MR]`` on the pr x pc grid: SUMMA (Elemental's
    ``Gemm`` for this layout; reference call sites e.g. ``ml/krr.hpp:423``).

    The inner dimension K is walked in super-panels of ``L = lcm(pr, pc)``
    consecutive K-blocks: every process column owns L / pc blocks of A's
    super-panel and every process row L / pr blocks of B's, so one
    all-gather in the row communicator (A: m/pr x L bK) and one in the
    column communicator (B: L bK x n/pc) bring rank (r, c) exactly the
    operands of its local update ``C_rc += A[R_r, panel] B[panel, C_c]``.
    Memory per rank is one super-panel of each operand (O(m/pr L bK)), not
    whole block rows; the collective volume is SUMMA's m K / pr + K n / pc."""
    import math as _m
    from ..parallel.distmatrix import DistMatrix, _cyclic_blocks
    m, K = A.shape
    K2, n = B.shape
    if K != K2:
        raise DimensionMismatchError("Gemm: inner dimensions differ")
    g = A.grid
    bK = A.block[1]
    if B.grid is not g or B.layout != "MC_MR" or B.block[0] != bK:
        B = B.redistribute("MC_MR", grid=g, block=(bK, B.block[1]))
    dev = A.local.device
    dt = torch.promote_types(A.dtype, B.dtype)
    Aloc = A.local.to(dt)
    Bloc = B.local.to(dt)
    C = torch.zeros(Aloc.shape[0], Bloc.shape[1], dtype=dt, device=dev)
    L = g.pr * g.pc // _m.gcd(g.pr, g.pc)
    nblk = (K + bK - 1) // bK
    # local column offsets of A's K-blocks (this process column) / row offsets of B's
    a_off, off = {}, 0
    for s0, e0 in _cyclic_blocks(K, bK, g.pc, g.mycol):
        a_off[s0 // bK] = (off, e0 - s0)
        off += e0 - s0
    b_off, off = {}, 0
    for s0, e0 in _cyclic_blocks(K, bK, g.pr, g.myrow):
        b_off[s0 // bK] = (off, e0 - s0)
        off += e0 - s0
    for j0 in range(0, nblk, L):
        blocks = list(range(j0, min(nblk, j0 + L)))
        # A super-panel: process column c contributes its blocks j (j % pc == c), in order
        mineA = [a_off[j] for j in blocks if j % g.pc == g.mycol]
        pieceA = torch.cat([Aloc[:, o:o + w] for o, w in mineA], 1) if mineA else Aloc[:, :0]
        cntA = [sum(min(K, (j + 1) * bK) - j * bK for j in blocks if j % g.pc == c) for c in range(g.pc)]
        GA = g.row_comm.all_gather_v(pieceA.contiguous(), cntA, 1) if g.pc > 1 else pieceA
        # B super-panel: process row r contributes its blocks j (j % pr == r)
        mineB = [b_off[j] for j in blocks if j % g.pr == g.myrow]
        pieceB = torch.cat([Bloc[o:o + w] for o, w in mineB], 0) if mineB else Bloc[:0]
        cntB = [sum(min(K, (j + 1) * bK) - j * bK for j in blocks if j % g.pr == r) for r in range(g.pr)]
        GB = g.col_comm.all_gather_v(pieceB.contiguous(), cntB, 0) if g.pr > 1 else pieceB
        # gathered order is owner-major; put both operands in K order
        posA, o = {}, 0
        for c in range(g.pc):
            for j in blocks:
                if j % g.pc == c:
                    w = min(K, (j + 1) * bK) - j * bK
                    posA[j] = (o, w)
                    o += w
        posB, o = {}, 0
        for r in range(g.pr):
            for j in blocks:
                if j % g.pr == r:
                    w = min(K, (j + 1) * bK) - j * bK
                    posB[j] = (o, w)
                    o += w
        Ap = torch.cat([GA[:, posA[j][0]:posA[j][0] + posA[j][1]] for j in blocks], 1)
        Bp = torch.cat([GB[posB[j][0]:posB[j][0] + posB[j][1]] for j in blocks], 0)
        C += Ap @ Bp
    return DistMatrix(C, (m, n), "MC_MR", A.comm, grid=g, block=(A.block[0], B.block[1]))


def Gemv(oA: str, alpha, A, x, beta=0.0, y=None):
    """``y = alpha op(A) x + beta y``; ``[VC,*]^T x`` all-reduces (``base/Gemv.hpp:59``)."""
    xx = x if (hasattr(x, "dim") and x.dim() == 2) or _is_dist(x) else x.reshape(-1, 1)
    yy = None
    if y is not None:
        yy = y if (hasattr(y, "dim") and y.dim() == 2) or _is_dist(y) else y.view(-1, 1)
    r = Gemm(oA, "N", alpha, A, xx, beta, yy)
    if y is not None:
        return y
    if _is_dist(r):
        return r
    return r.reshape(-1) if not (hasattr(x, "dim") and x.dim() == 2) else r


def Symm(side: str, uplo: str, alpha, A, B, beta=0.0, C=None):
    """``C = alpha A B + beta C`` (side L) or ``alpha B A`` (side R) with
    symmetric A stored in its ``uplo`` triangle (``base/Symm.hpp``)."""
    if _is_dist(A):
        Af = A.to_global()
    else:
        Af = _as_tensor(A)
    if Af.layout != torch.strided:
        Af = Af.to_dense()
    tri = torch.tril(Af) if uplo.upper() == "L" else torch.triu(Af)
    S = tri + tri.t() - torch.diag(torch.diagonal(Af))
    if side.upper() == "L":
        return Gemm("N", "N", alpha, S, B, beta, C) if not _is_dist(B) else _dist_left(S, alpha, B, beta, C)
    return Gemm("N", "N", alpha, B, S, beta, C)


def _dist_left(S, alpha, B, beta, C):
    """Replicated symmetric S times a distributed B (all-gather B once)."""
    from ..parallel.distmatrix import DistMatrix
    Bf = B.to_global()
    P = alpha * (S.to(Bf.dtype) @ Bf)
    out = DistMatrix.from_global(P, B.layout, B.comm, B.grid, B.block)
    if C is None:
        return out
    C.local.mul_(beta).add_(out.local)
    return C


def Trsm(side: str, uplo: str, orient: str, diag: str, alpha, A, B):
    """Triangular solve in place on B: ``op(A) X = alpha B`` (side L) or
    ``X op(A) = alpha B`` (side R) (``base/Trsm.hpp``); A replicated."""
    Af = A.to_global() if _is_dist(A) else _as_tensor(A)
    upper = uplo.upper() == "U"
    unit = diag.upper() == "U"
    if orient.upper() != "N":
        Af, upper = Af.t(), not upper
    Bt = B.local if _is_dist(B) else B
    if side.upper() == "L":
        if _is_dist(B) and B.layout not in ("STAR_STAR", "STAR_VC", "STAR_VR"):
            raise UnsupportedBaseOperation("Trsm left needs the rows of B replicated")
        X = torch.linalg.solve_triangular(Af.to(Bt.dtype), alpha * Bt, upper=upper, left=True, unitriangular=unit)
    else:
        if _is_dist(B) and B.layout not in ("STAR_STAR", "VC_STAR", "VR_STAR"):
            raise UnsupportedBaseOperation("Trsm right needs the columns of B replicated")
        X = torch.linalg.solve_triangular(Af.to(Bt.dtype), alpha * Bt, upper=upper, left=False, unitriangular=unit)
    Bt.copy_(X)
    return B


def ExplicitUnitary(A):
    """Overwrite A with the Q factor of its QR (``base/QR.hpp:11-36``): TSQR for
    ``[VC,*]`` (one all-gather of the k x k R factors), Householder locally."""
    from . import linalg as L
    if _is_dist(A):
        from ..parallel.distmatrix import is_row_dist
        if not is_row_dist(A.layout):
            B = A.redistribute("VC_STAR")
            ExplicitUnitary(B)
            A.local.copy_(B.redistribute(A.layout, A.grid, A.block).local)
            return A
        Q, _ = L.tsqr(A.local, A.comm)
        A.local.copy_(Q.to(A.local.dtype))
        return A
    Q, _ = torch.linalg.qr(A)
    A.copy_(Q)
    return A


def QR(A):
    """(Q, R) with Q explicit (distributed ``[VC,*]``: TSQR)."""
    from . import linalg as L
    if _is_dist(A):
        from ..parallel.distmatrix import DistMatrix
        B = A if A.layout in ("VC_STAR", "VR_STAR") else A.redistribute("VC_STAR")
        Q, R = L.tsqr(B.local, B.comm)
        return DistMatrix(Q.to(B.local.dtype), B.shape, B.layout, B.comm), R
    return torch.linalg.qr(A)


# ---------------------------------------------------------------- basic ops
def Axpy(alpha, X, Y):
    """``Y += alpha X``; ``alpha`` may be a per-column vector (``base/basic.hpp:48-70``)."""
    Xl = X.local if _is_dist(X) else X
    Yl = Y.local if _is_dist(Y) else Y
    if isinstance(alpha, torch.Tensor) and alpha.numel() > 1:
        Yl.add_(Xl * alpha.to(Yl.device, Yl.dtype).view(1, -1))
    else:
        Yl.add_(Xl, alpha=float(alpha))
    return Y


def Scale(alpha, X):
    (X.local if _is_dist(X) else X).mul_(alpha)
    return X


def ColumnView(X, j0: int, width: int):
    """Columns ``[j0, j0+width)`` as a view (``base/viewing.hpp``)."""
    if _is_dist(X):
        from ..parallel.distmatrix import is_row_dist
        if not is_row_dist(X.layout) and X.layout != "STAR_STAR":
            raise UnsupportedBaseOperation("ColumnView of a column-distributed matrix")
        return X.like(X.local[:, j0:j0 + width], (X.shape[0], width))
    return X[:, j0:j0 + width]


def RowView(X, i0: int, height: int):
    if _is_dist(X):
        from ..parallel.distmatrix import is_col_dist
        if not is_col_dist(X.layout) and X.layout != "STAR_STAR":
            raise UnsupportedBaseOperation("RowView of a row-distributed matrix")
        return X.like(X.local[i0:i0 + height], (height, X.shape[1]))
    return X[i0:i0 + height]


def DenseCopy(X) -> torch.Tensor:
    """Dense copy of a sparse operand (``base/copy.hpp:20-30``)."""
    from .sparse import SparseMatrix
    if isinstance(X, SparseMatrix):
        return X.to_dense()
    if isinstance(X, torch.Tensor) and X.layout != torch.strided:
        return X.to_dense()
    if _is_dist(X) and X.local.layout != torch.strided:
        return X.like(X.local.to_dense())
    return X.clone() if isinstance(X, torch.Tensor) else X


def RowDot(X, Y) -> torch.Tensor:
    """Row-wise dot products (``base/inner.hpp`` RowDot); row-distributed
    operands need no communication."""
    Xl = X.local if _is_dist(X) else X
    Yl = Y.local if _is_dist(Y) else Y
    return (Xl * Yl).sum(1)


__all__ = ["ComputedMatrix", "Gemm", "Gemv", "Symm", "Trsm", "ExplicitUnitary", "QR", "Axpy", "Scale",
           "ColumnView", "RowView", "DenseCopy", "RowDot", "Height", "Width"]
