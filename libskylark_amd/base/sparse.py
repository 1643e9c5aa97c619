"""Sparse matrices: local CSC container and row/column-distributed sparse
matrices built from queued updates.

Reference:
  * ``base/sparse_matrix.hpp:25-318`` — ``sparse_matrix_t``: CSC arrays with
    attach/detach ownership, ``set(coords)`` building the CSC and SUMMING
    duplicate coordinates (``:158-211``), ``Transpose`` (``:321-364``),
    ``Copy`` (``:367-382``), equality;
  * ``base/sparse_dist_matrix.hpp:46-389`` — distributed sparse matrix with
    queued updates and ``finalize()`` (local CSC + an all-reduce of the
    non-zero count, ``:140-182``); ``[VC,*]`` (rows) and ``[*,VR]`` (columns)
    specialisations (``base/sparse_vc_star_matrix.hpp:19-52``,
    ``base/sparse_star_vr_matrix.hpp:15-48``);
  * ``base/graph_adapters.hpp:6-27`` — CSC viewed as an adjacency structure.

MI355X design: the arrays are torch tensors on any device (int32 or int64
indices); compute (sketching, SpMM) consumes them as torch CSR/CSC tensors,
the form the native CountSketch kernels and hipSPARSE-backed torch ops take.
The distributed container is a thin builder: ``finalize()`` returns a
:class:`~libskylark_amd.parallel.DistMatrix` whose local shard is a CSR
tensor, so every distributed sketch / GEMM path accepts it unchanged.
Contiguous row (column) blocks replace the reference's element-cyclic
``[VC,*]`` (``[*,VR]``) ownership.
"""
from __future__ import annotations

import numpy as np
import torch

from .exceptions import DimensionMismatchError, InvalidParametersError


def _coalesce_csc(rows, cols, vals, m, n, index_dtype):
    """CSC arrays from (row, col, val) triples, duplicates summed, rows sorted."""
    rows = torch.as_tensor(rows, dtype=torch.int64)
    cols = torch.as_tensor(cols, dtype=torch.int64, device=rows.device)
    vals = torch.as_tensor(vals, device=rows.device)
    if rows.numel():
        if int(rows.min()) < 0 or int(rows.max()) >= m or int(cols.min()) < 0 or int(cols.max()) >= n:
            raise InvalidParametersError("sparse set: coordinate out of range")
    key = cols * m + rows
    key, order = torch.sort(key)
    vals = vals[order]
    uniq, inv = torch.unique_consecutive(key, return_inverse=True)
    summed = torch.zeros(uniq.numel(), dtype=vals.dtype, device=vals.device).index_add_(0, inv, vals)
    c = uniq // m
    r = uniq - c * m
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=rows.device)
    indptr[1:] = torch.bincount(c, minlength=n).cumsum(0)
    return indptr.to(index_dtype), r.to(index_dtype), summed


class SparseMatrix:
    """Local sparse matrix in CSC form (``sparse_matrix_t``).

    ``indptr`` (width+1), ``indices`` (row of each non-zero, sorted within a
    column) and ``values``.  ``attach`` adopts caller arrays (optionally not
    owned: ``detach`` hands them back); ``set`` builds from coordinates and
    sums duplicates like the reference."""

    def __init__(self, height: int = 0, width: int = 0, dtype=torch.float64, index_dtype=torch.int32,
                 device=None):
        self._m, self._n = int(height), int(width)
        self.index_dtype = index_dtype
        self.indptr = torch.zeros(self._n + 1, dtype=index_dtype, device=device)
        self.indices = torch.zeros(0, dtype=index_dtype, device=device)
        self.values = torch.zeros(0, dtype=dtype, device=device)
        self._owned = True

    # ---------------------------------------------------------------- shape
    def height(self) -> int:
        return self._m

    def width(self) -> int:
        return self._n

    @property
    def shape(self):
        return (self._m, self._n)

    def nonzeros(self) -> int:
        return int(self.values.numel())

    nnz = nonzeros

    @property
    def dtype(self):
        return self.values.dtype

    @property
    def device(self):
        return self.values.device

    # ------------------------------------------------------------ building
    def attach(self, indptr, indices, values, height: int, width: int, own: bool = True):
        indptr, indices, values = (torch.as_tensor(x) for x in (indptr, indices, values))
        if indptr.numel() != width + 1 or indices.numel() != values.numel():
            raise DimensionMismatchError("attach: inconsistent CSC arrays")
        if int(indptr[-1]) != values.numel():
            raise DimensionMismatchError("attach: indptr[-1] != nnz")
        self._m, self._n = int(height), int(width)
        self.indptr, self.indices, self.values = indptr, indices, values
        self.index_dtype = indices.dtype
        self._owned = bool(own)
        return self

    def detach(self):
        """Release the arrays (reference ``detach``): returns (indptr, indices, values)."""
        out = (self.indptr, self.indices, self.values)
        self.__init__(0, 0, self.values.dtype, self.index_dtype, self.values.device)
        return out

    def owns_data(self) -> bool:
        return self._owned

    def set(self, coords, height: int | None = None, width: int | None = None):
        """Build from ``coords`` = iterable of (row, col, value) (or three arrays);
        duplicate coordinates are summed (``sparse_matrix_t::set``)."""
        if height is not None:
            self._m = int(height)
        if width is not None:
            self._n = int(width)
        if isinstance(coords, (tuple, list)) and len(coords) == 3 and not np.isscalar(coords[0]) and \
                hasattr(coords[0], "__len__") and len(coords[0]) != 3:
            r, c, v = coords
        else:
            arr = list(coords)
            r = [int(t[0]) for t in arr]
            c = [int(t[1]) for t in arr]
            v = [float(t[2]) for t in arr]
        v = torch.as_tensor(v, dtype=self.values.dtype)
        dev = self.values.device
        self.indptr, self.indices, self.values = (x.to(dev) for x in _coalesce_csc(
            torch.as_tensor(r), torch.as_tensor(c), v, self._m, self._n, self.index_dtype))
        self._owned = True
        return self

    # ---------------------------------------------------------- conversion
    @classmethod
    def from_torch(cls, T: torch.Tensor, index_dtype=torch.int32):
        if T.layout == torch.strided:
            T = T.to_sparse_csc()
        elif T.layout != torch.sparse_csc:
            T = T.to_sparse_coo().coalesce().to_sparse_csc()
        S = cls(T.shape[0], T.shape[1], T.dtype, index_dtype, T.device)
        return S.attach(T.ccol_indices().to(index_dtype), T.row_indices().to(index_dtype), T.values(),
                        T.shape[0], T.shape[1])

    @classmethod
    def from_scipy(cls, M, index_dtype=torch.int32):
        import scipy.sparse as sp
        M = sp.csc_matrix(M)
        M.sort_indices()
        S = cls(M.shape[0], M.shape[1], torch.from_numpy(M.data).dtype, index_dtype)
        return S.attach(torch.from_numpy(M.indptr).to(index_dtype), torch.from_numpy(M.indices).to(index_dtype),
                        torch.from_numpy(M.data.copy()), M.shape[0], M.shape[1])

    def to_torch(self, layout: str = "csr", device=None) -> torch.Tensor:
        """As a torch sparse tensor (``"csr"`` for the compute kernels, or ``"csc"``)."""
        T = torch.sparse_csc_tensor(self.indptr.to(torch.int64), self.indices.to(torch.int64), self.values,
                                    size=self.shape)
        if layout == "csr":
            T = T.to_sparse_coo().coalesce().to_sparse_csr() if self.nonzeros() else \
                torch.sparse_csr_tensor(torch.zeros(self._m + 1, dtype=torch.int64), torch.zeros(0, dtype=torch.int64),
                                        torch.zeros(0, dtype=self.dtype), size=self.shape)
        return T.to(device) if device is not None else T

    def to_scipy(self):
        import scipy.sparse as sp
        return sp.csc_matrix((self.values.cpu().numpy(), self.indices.cpu().numpy(), self.indptr.cpu().numpy()),
                             shape=self.shape)

    def to_dense(self) -> torch.Tensor:
        """``DenseCopy`` (reference ``base/copy.hpp:20-30``)."""
        out = torch.zeros(self.shape, dtype=self.dtype, device=self.device)
        if self.nonzeros():
            cols = torch.repeat_interleave(torch.arange(self._n, device=self.device),
                                           (self.indptr[1:] - self.indptr[:-1]).to(torch.int64))
            out.index_put_((self.indices.to(torch.int64), cols), self.values, accumulate=True)
        return out

    # --------------------------------------------------------- operations
    def transpose(self) -> "SparseMatrix":
        """``Transpose`` (reference ``:321-364``): the CSC of A^T."""
        cols = torch.repeat_interleave(torch.arange(self._n, device=self.device),
                                       (self.indptr[1:] - self.indptr[:-1]).to(torch.int64))
        out = SparseMatrix(self._n, self._m, self.dtype, self.index_dtype, self.device)
        out.indptr, out.indices, out.values = (x.to(self.device) for x in _coalesce_csc(
            cols, self.indices.to(torch.int64), self.values, self._n, self._m, self.index_dtype))
        return out

    T = property(transpose)

    def copy(self) -> "SparseMatrix":
        out = SparseMatrix(self._m, self._n, self.dtype, self.index_dtype, self.device)
        return out.attach(self.indptr.clone(), self.indices.clone(), self.values.clone(), self._m, self._n)

    def to(self, device=None, dtype=None) -> "SparseMatrix":
        out = SparseMatrix(self._m, self._n, dtype or self.dtype, self.index_dtype, device or self.device)
        return out.attach(self.indptr.to(device), self.indices.to(device), self.values.to(device=device, dtype=dtype),
                          self._m, self._n)

    def structure_equal(self, other: "SparseMatrix") -> bool:
        return self.shape == other.shape and torch.equal(self.indptr.cpu().long(), other.indptr.cpu().long()) and \
            torch.equal(self.indices.cpu().long(), other.indices.cpu().long())

    def __eq__(self, other) -> bool:
        return isinstance(other, SparseMatrix) and self.structure_equal(other) and \
            torch.equal(self.values.cpu(), other.values.cpu())

    def __repr__(self):
        return f"SparseMatrix({self._m}x{self._n}, nnz={self.nonzeros()}, {self.dtype}, {self.device})"


class DistSparseMatrix:
    """Distributed sparse matrix assembled from queued global updates.

    ``layout`` ``"VC_STAR"`` (rows split in contiguous blocks over the ranks)
    or ``"STAR_VR"`` (columns split).  Any rank may queue any entry; entries
    owned by other ranks are routed to them by one all-to-all in
    :meth:`finalize`, duplicates are summed, and the result is a
    :class:`DistMatrix` whose local shard is a CSR tensor on ``device``."""

    def __init__(self, height: int, width: int, layout: str = "VC_STAR", comm=None, dtype=torch.float64,
                 device=None):
        from ..parallel.comm import world
        from ..parallel.distmatrix import canon
        self.shape = (int(height), int(width))
        self.layout = canon(layout)
        if self.layout not in ("VC_STAR", "VR_STAR", "STAR_VC", "STAR_VR"):
            raise InvalidParametersError("DistSparseMatrix supports [VC,*] / [*,VR] style layouts")
        self.comm = comm or world()
        self.dtype = dtype
        self.device = device
        self._queue = ([], [], [])
        self._nnz = None

    def queue_update(self, i, j, v):
        """Queue A[i, j] += v (scalars or equal-length arrays; global indices)."""
        self._queue[0].append(torch.as_tensor(i, dtype=torch.int64).reshape(-1))
        self._queue[1].append(torch.as_tensor(j, dtype=torch.int64).reshape(-1))
        self._queue[2].append(torch.as_tensor(v, dtype=self.dtype).reshape(-1))

    def finalize(self):
        """Route queued entries to their owners, sum duplicates; returns the
        DistMatrix (sparse CSR local shard).  Collective."""
        from ..parallel.comm import balanced_offsets
        from ..parallel.distmatrix import DistMatrix, is_row_dist
        c = self.comm
        m, n = self.shape
        q = self._queue
        I = torch.cat(q[0]) if q[0] else torch.zeros(0, dtype=torch.int64)
        J = torch.cat(q[1]) if q[1] else torch.zeros(0, dtype=torch.int64)
        V = torch.cat(q[2]) if q[2] else torch.zeros(0, dtype=self.dtype)
        self._queue = ([], [], [])
        rowdist = is_row_dist(self.layout)
        offs = torch.tensor(balanced_offsets(m if rowdist else n, c.size), dtype=torch.int64)
        key = I if rowdist else J
        owner = torch.searchsorted(offs[1:], key, right=True) if key.numel() else key
        if c.size > 1:
            order = torch.argsort(owner, stable=True)
            I, J, V, owner = I[order], J[order], V[order], owner[order]
            counts = torch.bincount(owner, minlength=c.size).tolist()
            cdev = c.collective_device()
            rI = c.all_to_all_v(list(torch.split(I.to(cdev), counts)))
            rJ = c.all_to_all_v(list(torch.split(J.to(cdev), counts)))
            rV = c.all_to_all_v(list(torch.split(V.to(cdev), counts)))
            I, J, V = torch.cat(rI).cpu(), torch.cat(rJ).cpu(), torch.cat(rV).cpu()
        lo, hi = int(offs[c.rank]), int(offs[c.rank + 1])
        if rowdist:
            lm, ln, li, lj = hi - lo, n, I - lo, J
        else:
            lm, ln, li, lj = m, hi - lo, I, J - lo
        indptr, rows, vals = _coalesce_csc(li, lj, V, lm, ln, torch.int64)
        local = SparseMatrix(lm, ln, self.dtype, torch.int64).attach(indptr, rows, vals, lm, ln)
        csr = local.to_torch("csr", self.device)
        nnz = torch.tensor([local.nonzeros()], dtype=torch.int64)
        if c.size > 1:
            nnz = c.all_reduce(nnz.to(c.collective_device())).cpu()
        self._nnz = int(nnz[0])
        return DistMatrix(csr, self.shape, self.layout, c)

    def nonzeros(self) -> int:
        """Global non-zero count (after :meth:`finalize`; all-reduced there)."""
        if self._nnz is None:
            raise InvalidParametersError("nonzeros() before finalize()")
        return self._nnz


class GraphAdapter:
    """Adjacency view of a square sparse matrix (``base/graph_adapters.hpp``):
    vertex ``v``'s neighbours are the row indices of column ``v``."""

    def __init__(self, A: SparseMatrix):
        if A.height() != A.width():
            raise DimensionMismatchError("graph adapter needs a square matrix")
        self.A = A
        self._ptr = A.indptr.cpu().to(torch.int64)
        self._idx = A.indices.cpu().to(torch.int64)

    def num_vertices(self) -> int:
        return self.A.width()

    def degree(self, v: int) -> int:
        return int(self._ptr[v + 1] - self._ptr[v])

    def neighbors(self, v: int) -> torch.Tensor:
        return self._idx[self._ptr[v]:self._ptr[v + 1]]

    def degrees(self) -> torch.Tensor:
        return self._ptr[1:] - self._ptr[:-1]


__all__ = ["SparseMatrix", "DistSparseMatrix", "GraphAdapter"]
