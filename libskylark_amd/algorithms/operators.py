"""Linear-operator adapters for the iterative solvers.

The reference's solvers are templated on Elemental / sparse matrix types and
call ``base::Gemm`` / ``base::Symm`` / ``base::ColumnNrm2`` (which contain the
all-reduces, ``base/Gemm.hpp:84-103``, ``base/inner.hpp``).  Here an
:class:`Operator` hides the layout:

* "long" vectors live on the row side of A (m x k); for a row-distributed A
  ([VC,*]) they are row-distributed too and inner products all-reduce k
  scalars;
* "short" vectors live on the column side (n x k) and are replicated on every
  GPU; ``A^T U`` is a local GEMM plus ONE all-reduce of n x k.

Dense (torch, any device), sparse CSR (torch) and DistMatrix [VC,*] inputs
are supported; anything with ``matmul``/``rmatmul`` methods passes through.
"""
from __future__ import annotations

import torch

from ..ops.spmm import csr_transpose as _csr_transpose

from ..ops import krylov_native as _kn
from ..parallel.comm import Comm
from ..parallel.distmatrix import DistMatrix


class Operator:
    distributed = False

    def __init__(self, shape, dtype, device, comm: Comm | None = None):
        self.shape = tuple(shape)
        self.dtype = dtype
        self.device = device
        self.comm = comm or Comm(None)

    # y = A x (x short/replicated, y long/distributed)
    def matmul(self, X):
        raise NotImplementedError

    # x = A^T y (y long/distributed, x short/replicated)
    def rmatmul(self, Y):
        raise NotImplementedError

    # column 2-norms / dots of LONG vectors (all-reduce when distributed); on
    # the GPU one native streaming pass each (ops/krylov_native.py, f64 sums)
    def long_colnorm(self, U):
        if _kn.ok(U):
            s = _kn.colsumsq(U)
            if self.distributed:
                self.comm.all_reduce(s)
            return s.sqrt().to(U.dtype)
        s = (U * U).sum(0)
        if self.distributed:
            self.comm.all_reduce(s)
        return s.sqrt()

    def long_coldot(self, U, V):
        if _kn.ok(U) and isinstance(V, torch.Tensor) and V.shape == U.shape and V.is_cuda:
            s = _kn.coldot(U, V)
            if self.distributed:
                self.comm.all_reduce(s)
            return s.to(U.dtype)
        s = (U * V).sum(0)
        if self.distributed:
            self.comm.all_reduce(s)
        return s

    @staticmethod
    def short_colnorm(X):
        if _kn.ok(X):
            return _kn.colsumsq(X).sqrt().to(X.dtype)
        return (X * X).sum(0).sqrt()

    def long_like(self, B):
        return B

    def local_rows(self):
        return self.shape[0]

    # (A^T A X, A X or None); operators with a one-pass kernel override this
    def normal(self, X, want_y: bool = False):
        Y = self.matmul(X)
        return self.rmatmul(Y), (Y if want_y else None)

    def has_fused_normal(self, k: int) -> bool:
        return False


class DenseOp(Operator):
    def __init__(self, A: torch.Tensor, compute_dtype=None):
        cdt = compute_dtype or (A.dtype if A.dtype in (torch.float32, torch.float64) else torch.float32)
        super().__init__(A.shape, cdt, A.device)
        self.A = A

    def matmul(self, X):
        if self.A.dtype in (torch.bfloat16, torch.float16):
            from ..ops import tallskinny as T
            return T.matmul(self.A, X, out_dtype=self.dtype)
        if X.dim() == 2 and self.has_fused_normal(X.shape[1]):
            # A X from the one-pass kernel (its A^T A X byproduct is discarded):
            # ~6 TB/s against ~2.4 TB/s for the library GEMV on tall f32 A
            from ..ops import normal_eq
            return normal_eq.ata(self.A, X, want_y=True)[1]
        from ..ops import normal_eq
        if (X.dim() == 1 or X.shape[1] == 1) and normal_eq.gemv_ok(self.A, 1) and self.A.shape[1] > 6144:
            # rows too wide for the one-pass kernel (a stored kernel Gram), one
            # right-hand side: the streaming GEMV, 6.25 vs 5.46 TB/s for the
            # library at n = 1e5 (k = 2, 4: the library is as fast or faster,
            # profiles/r5/gemv_v1.jsonl)
            return normal_eq.gemv(self.A, X)
        return self.A @ X.to(self.A.dtype)

    def rmatmul(self, Y):
        if Y.dim() == 2 and self.A.dtype == torch.float32 and self.has_fused_normal(Y.shape[1]) \
                and Y.shape[0] == self.A.shape[0]:
            # A^T Y as the dual pass with D = Y (one read of A; the transposed
            # library GEMV ran at ~1 TB/s)
            from ..ops import normal_eq
            return normal_eq.dual(self.A, Y.to(torch.float32))[0]
        if self.A.dtype in (torch.bfloat16, torch.float16):
            hi = Y.to(self.A.dtype)
            lo = (Y - hi.to(Y.dtype)).to(self.A.dtype)
            if self.A.is_cuda:
                return (torch.mm(self.A.t(), hi, out_dtype=torch.float32) +
                        torch.mm(self.A.t(), lo, out_dtype=torch.float32)).to(self.dtype)
            return (self.A.t().float() @ (hi.float() + lo.float())).to(self.dtype)
        return self.A.t() @ Y.to(self.A.dtype)

    def has_fused_normal(self, k: int) -> bool:
        from ..ops import normal_eq
        return normal_eq.native_ok(self.A, k)

    def normal(self, X, want_y: bool = False):
        if self.has_fused_normal(X.shape[1]):
            from ..ops import normal_eq
            W, Y = normal_eq.ata(self.A, X, want_y)
            return W.to(self.dtype), (Y.to(self.dtype) if Y is not None else None)
        return super().normal(X, want_y)


class SparseOp(Operator):
    def __init__(self, A: torch.Tensor):
        vdt = A.values().dtype
        super().__init__(A.shape, vdt if vdt in (torch.float32, torch.float64) else torch.float32, A.device)
        self.A = A
        self._At = None

    def matmul(self, X):
        from ..ops import spmm
        if X.dim() == 2 and spmm.ok(self.A, X):
            return spmm.csr_mm(self.A, X)
        return torch.sparse.mm(self.A, X.to(self.dtype))

    def rmatmul(self, Y):
        # the CSR of A^T is built once per operator (deterministic sums; an
        # atomic scatter A^T Y would not be)
        if self._At is None:
            self._At = _csr_transpose(self.A)
        from ..ops import spmm
        if Y.dim() == 2 and spmm.ok(self._At, Y):
            return spmm.csr_mm(self._At, Y)
        return torch.sparse.mm(self._At, Y.to(self.dtype))


class DistRowOp(Operator):
    """A distributed as [VC,*] row blocks (local shard m_loc x n)."""

    distributed = True

    def __init__(self, D: DistMatrix):
        if D.layout not in ("VC_STAR", "VR_STAR"):
            D = D.redistribute("VC_STAR")
        loc = D.local
        inner = SparseOp(loc) if loc.layout == torch.sparse_csr else DenseOp(loc)
        super().__init__(D.shape, inner.dtype, loc.device, D.comm)
        self.D = D
        self.inner = inner
        self.distributed = D.comm.size > 1

    def matmul(self, X):
        return self.inner.matmul(X)

    def rmatmul(self, Y):
        out = self.inner.rmatmul(Y).contiguous()
        if self.distributed:
            self.comm.all_reduce(out)
        return out

    def local_rows(self):
        return self.D.local.shape[0]

    def has_fused_normal(self, k: int) -> bool:
        return self.inner.has_fused_normal(k)

    def normal(self, X, want_y: bool = False):
        """Local one-pass A_loc^T (A_loc X) + ONE all-reduce of n x k."""
        W, Y = self.inner.normal(X, want_y)
        W = W.contiguous()
        if self.distributed:
            self.comm.all_reduce(W)
        return W, Y

    def long_like(self, B):
        # B may be given globally (replicated m x k) or already as the local shard
        if isinstance(B, DistMatrix):
            return B.redistribute("VC_STAR").local
        if B.shape[0] == self.shape[0] and self.D.local.shape[0] != self.shape[0]:
            s, e = self.D.row_range()
            return B[s:e]
        return B


class DistSymOp(DistRowOp):
    """Square symmetric A held as [VC,*] row blocks, for CG-type solvers where
    every vector is "long" (row-distributed like A): ``A P`` all-gathers the
    n x k direction block (one collective per iteration) and multiplies the
    local row block; ``A^T`` is ``A``."""

    def matmul(self, X):
        if self.distributed:
            counts = self.D.row_counts()
            X = self.comm.all_gather_v(X.contiguous(), counts, dim=0)
        return self.inner.matmul(X)

    rmatmul = matmul


class Sparse2DOp(Operator):
    """A held as 2-D block-sparse tiles (:class:`~..parallel.dist_sparse2d.DistSparse2D`,
    the CombBLAS SpParMat analogue; reference ``base/detail/combblas_mixed_gemm.hpp``).

    Long vectors are the row block ``R_r`` of the grid row (replicated along
    it), short vectors are replicated: ``A X`` = tile SpMM + one all-reduce in
    the grid row; ``A^T Y`` = tile SpMM placed at the tile's columns + ONE
    world all-reduce (every tile contributes exactly once).  Long-vector
    norms/dots reduce over the grid column (the ranks that partition the
    rows)."""

    def __init__(self, M):
        vdt = M.local.values().dtype
        super().__init__(M.shape, vdt if vdt in (torch.float32, torch.float64) else torch.float32,
                         M.local.device, M.grid.col_comm)
        self.M = M
        self.distributed = M.comm.size > 1
        self._cols = None

    def matmul(self, X):
        return self.M.matmul(X)

    def rmatmul(self, Y):
        M = self.M
        part = M._spmm(M._transposed(), Y.contiguous())
        if self._cols is None:
            self._cols = M.cols.to(part.device)
        out = torch.zeros(M.shape[1], part.shape[1], dtype=part.dtype, device=part.device)
        out.index_copy_(0, self._cols, part)
        if self.distributed:
            M.comm.all_reduce(out)
        return out

    def local_rows(self):
        return self.M.rows.numel()

    def long_like(self, B):
        if B.shape[0] == self.shape[0] and self.M.rows.numel() != self.shape[0]:
            return B.index_select(0, self.M.rows.to(B.device))
        return B


class CallableOp(Operator):
    def __init__(self, obj):
        super().__init__(obj.shape, getattr(obj, "dtype", torch.float64), getattr(obj, "device", None),
                         getattr(obj, "comm", None))
        self.obj = obj
        self.distributed = getattr(obj, "distributed", False)

    def matmul(self, X):
        return self.obj.matmul(X)

    def rmatmul(self, Y):
        return self.obj.rmatmul(Y)


def as_operator(A) -> Operator:
    if isinstance(A, Operator):
        return A
    if isinstance(A, DistMatrix):
        return DistRowOp(A)
    if type(A).__name__ == "DistSparse2D":
        return Sparse2DOp(A)
    if isinstance(A, torch.Tensor):
        if A.layout != torch.strided:
            return SparseOp(A.to_sparse_csr() if A.layout != torch.sparse_csr else A)
        return DenseOp(A)
    if hasattr(A, "matmul") and hasattr(A, "rmatmul"):
        return CallableOp(A)
    import numpy as np
    if isinstance(A, np.ndarray):
        return DenseOp(torch.from_numpy(A))
    raise TypeError(f"cannot build an operator from {type(A)}")
