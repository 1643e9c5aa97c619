"""2-D block-sparse distribution: the CombBLAS ``SpParMat`` analogue.

Reference: ``base/detail/combblas_mixed_gemm.hpp:26-368`` (sparse x dense
products on a 2-D process grid) and ``sketch/hash_transform_CombBLAS.hpp``
(CountSketch of a CombBLAS matrix).  An ``m x n`` sparse matrix lives on the
``pr x pc`` grid of :class:`~.distmatrix.Grid` in block-cyclic tiles: rank
(r, c) holds rows ``R_r`` and columns ``C_c`` (blocks of ``block`` =
``(br, bc)``) as one local CSR tile (local row / column indices in
block-cyclic order).  MI355X mapping:

* assembly from arbitrary per-rank COO triples is ONE all-to-all of
  (row, col, value) to the owners (CombBLAS builds SpParMat the same way);
* ``A X`` for a replicated thin ``X``: local CSR SpMM on the tile (native
  ``ops/spmm.py`` kernel on the GPU), then one reduce-scatter-free all-reduce
  inside the grid row (the partial row blocks of the same ``R_r``);
  ``A^T Y`` symmetric inside the grid column;
* sketches along the row dimension: the tile's partial sketch over its rows
  (hash transforms scatter-add with global row indices, dense transforms
  realise only the columns of S for the tile's rows), then one all-reduce in
  the grid-column communicator -- the result is replicated down each grid
  column, column-distributed across grid columns (``[*, MR]``).
"""
from __future__ import annotations

import torch

from ..ops.spmm import csr_transpose as _csr_transpose

from .comm import Comm
from .distmatrix import Grid, _cyclic_blocks

COLUMNWISE, ROWWISE = 0, 1


def _positions(n, b, p, me):
    """Global indices owned by coordinate ``me`` in local order (int64 tensor)."""
    return torch.tensor([i for s, e in _cyclic_blocks(n, b, p, me) for i in range(s, e)], dtype=torch.int64)


def _owner(idx: torch.Tensor, b: int, p: int):
    """(owner coordinate, local position) of global indices under block-cyclic (b, p)."""
    blk = idx // b
    own = blk % p
    local = (blk // p) * b + idx % b
    return own, local


class DistSparse2D:
    """Sparse ``m x n`` matrix in 2-D block-cyclic CSR tiles."""

    def __init__(self, local: torch.Tensor, shape, grid: Grid, block=(1, 1)):
        self.local = local                      # CSR tile (|R_r| x |C_c|)
        self.shape = (int(shape[0]), int(shape[1]))
        self.grid = grid
        self.comm: Comm = grid.comm
        self.block = (int(block[0]), int(block[1]))
        m, n = self.shape
        self.rows = _positions(m, self.block[0], grid.pr, grid.myrow)
        self.cols = _positions(n, self.block[1], grid.pc, grid.mycol)
        self._At = None

    # ------------------------------------------------------------ assembly
    @classmethod
    def from_local_coo(cls, rows, cols, vals, shape, comm: Comm, grid: Grid | None = None, block=(64, 64),
                       device=None):
        """Assemble from this rank's (global row, global col, value) triples
        (any rank may hold any entries; duplicates are summed): one all-to-all
        to the tile owners."""
        grid = grid or Grid.default(comm)
        br, bc = int(block[0]), int(block[1])
        rows = torch.as_tensor(rows, dtype=torch.int64)
        cols = torch.as_tensor(cols, dtype=torch.int64)
        vals = torch.as_tensor(vals)
        orow, lrow = _owner(rows, br, grid.pr)
        ocol, lcol = _owner(cols, bc, grid.pc)
        dest = orow + ocol * grid.pr            # column-major grid rank
        order = torch.argsort(dest, stable=True)
        counts = torch.bincount(dest, minlength=comm.size).tolist()
        trip = torch.stack([lrow[order].to(torch.float64), lcol[order].to(torch.float64),
                            vals[order].to(torch.float64)], 1)
        sends = list(torch.split(trip, counts))
        got = torch.cat(comm.all_to_all_v(sends), 0) if comm.size > 1 else trip
        m, n = int(shape[0]), int(shape[1])
        nr = int(_positions(m, br, grid.pr, grid.myrow).numel())
        nc = int(_positions(n, bc, grid.pc, grid.mycol).numel())
        vdt = vals.dtype if vals.dtype in (torch.float32, torch.float64) else torch.float64
        if got.numel():
            idx = got[:, :2].t().to(torch.int64)
            coo = torch.sparse_coo_tensor(idx, got[:, 2].to(vdt), (nr, nc)).coalesce()
        else:
            coo = torch.sparse_coo_tensor(torch.zeros(2, 0, dtype=torch.int64), torch.zeros(0, dtype=vdt), (nr, nc))
        local = coo.to_sparse_csr()
        if device is not None:
            local = local.to(device)
        return cls(local, (m, n), grid, (br, bc))

    @classmethod
    def from_global(cls, A: torch.Tensor, comm: Comm, grid: Grid | None = None, block=(64, 64)):
        """Every rank holds the global sparse (or dense) A; keep this rank's tile."""
        grid = grid or Grid.default(comm)
        coo = (A if A.layout != torch.strided else A.to_sparse()).to_sparse_coo().coalesce()
        r, c = coo.indices()
        v = coo.values()
        orow, _ = _owner(r, int(block[0]), grid.pr)
        ocol, _ = _owner(c, int(block[1]), grid.pc)
        keep = (orow == grid.myrow) & (ocol == grid.mycol)
        # only local entries: the all-to-all inside from_local_coo then moves nothing
        return cls.from_local_coo(r[keep], c[keep], v[keep], A.shape, comm, grid, block, device=A.device)

    def to_global(self) -> torch.Tensor:
        """Dense global matrix on every rank (tests / small problems)."""
        m, n = self.shape
        coo = self.local.to_sparse_coo().coalesce()
        li, lj = coo.indices()
        gi, gj = self.rows.to(li.device)[li], self.cols.to(lj.device)[lj]
        full = torch.zeros(m, n, dtype=coo.values().dtype, device=coo.values().device)
        full.index_put_((gi, gj), coo.values(), accumulate=True)
        self.comm.all_reduce(full)
        return full

    def nnz(self) -> int:
        t = torch.tensor([self.local.values().numel()], dtype=torch.int64)
        self.comm.all_reduce(t)
        return int(t.item())

    # ------------------------------------------------------------ products
    def _spmm(self, T: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
        from ..ops import spmm
        if X.dim() == 2 and spmm.ok(T, X):
            return spmm.csr_mm(T, X)
        return torch.sparse.mm(T, X.to(T.values().dtype))

    def matmul(self, X: torch.Tensor) -> torch.Tensor:
        """``(A X)[R_r]`` (|R_r| x k) for a replicated ``X`` (n x k): local SpMM
        with ``X[C_c]`` plus one all-reduce in the grid-row communicator."""
        Xc = X.index_select(0, self.cols.to(X.device)).contiguous()
        Y = self._spmm(self.local, Xc).contiguous()
        if self.grid.pc > 1:
            self.grid.row_comm.all_reduce(Y)
        return Y

    def rmatmul(self, Y: torch.Tensor) -> torch.Tensor:
        """``(A^T Y)[C_c]`` (|C_c| x k) for a replicated ``Y`` (m x k): SpMM with the
        tile's transposed CSR (built once) plus one all-reduce in the grid column."""
        Yr = Y.index_select(0, self.rows.to(Y.device)).contiguous()
        X = self._spmm(self._transposed(), Yr).contiguous()
        if self.grid.pr > 1:
            self.grid.col_comm.all_reduce(X)
        return X

    def gather_rows(self, Yr: torch.Tensor) -> torch.Tensor:
        """Replicated m x k from the grid-row-replicated blocks ``Yr`` = (A X)[R_r]."""
        m = self.shape[0]
        full = torch.zeros(m, Yr.shape[1], dtype=Yr.dtype, device=Yr.device)
        if self.grid.mycol == 0:
            full.index_copy_(0, self.rows.to(Yr.device), Yr)
        self.comm.all_reduce(full)
        return full

    def gather_cols(self, Xc: torch.Tensor, axis: int = 0) -> torch.Tensor:
        """Replicated global array from blocks ``Xc`` indexed by this rank's columns
        (replicated down each grid column) along ``axis``."""
        n = self.shape[1]
        shape = list(Xc.shape)
        shape[axis] = n
        full = torch.zeros(shape, dtype=Xc.dtype, device=Xc.device)
        if self.grid.myrow == 0:
            full.index_copy_(axis, self.cols.to(Xc.device), Xc)
        self.comm.all_reduce(full)
        return full

    # ------------------------------------------------------------ sketches
    def _transposed(self):
        if self._At is None:
            self._At = _csr_transpose(self.local)
        return self._At

    def sketch(self, sk, dim: int = COLUMNWISE) -> torch.Tensor:
        """Columnwise ``S A`` (S x n) or rowwise ``A S^T`` (m x S) of the whole
        matrix; returns this rank's block: columns ``C_c`` of ``S A`` (S x |C_c|,
        replicated down the grid column) or rows ``R_r`` of ``A S^T``
        (|R_r| x S, replicated along the grid row).

        Hash sketches scatter-add the tile's nonzeros with their global
        indices; dense sketches realise only the operator columns of the
        tile's indices and run one local SpMM; both finish with ONE all-reduce
        in the grid-column (columnwise) or grid-row (rowwise) communicator.
        Any other transform falls back to assembling the tile's full
        columns (rows) inside that communicator and applying it locally."""
        cw = dim == COLUMNWISE
        comm = self.grid.col_comm if cw else self.grid.row_comm
        nshare = self.grid.pr if cw else self.grid.pc
        v = self.local.values()
        dev = v.device
        wdt = torch.float64 if v.dtype == torch.float64 else torch.float32
        S = sk.getsketchdim()
        gidx = (self.rows if cw else self.cols).to(dev)
        if hasattr(sk, "row_idx") and hasattr(sk, "row_value"):
            coo = self.local.to_sparse_coo().coalesce()
            li, lj = coo.indices()
            lidx, oidx = (li, lj) if cw else (lj, li)
            g = gidx[lidx]
            out = torch.zeros(S, (self.cols if cw else self.rows).numel(), dtype=wdt, device=dev)
            out.index_put_((sk.row_idx.to(dev)[g], oidx), sk.row_value.to(dev, wdt)[g] * coo.values().to(wdt),
                           accumulate=True)
        elif getattr(sk, "entries", None) is not None and hasattr(sk, "realize"):
            n_sk = self.shape[0] if cw else self.shape[1]
            b = self.block[0] if cw else self.block[1]
            p, me = (self.grid.pr, self.grid.myrow) if cw else (self.grid.pc, self.grid.mycol)
            # S x |tile dim|: operator columns of this tile's indices, block by block
            P = torch.cat([sk.realize(wdt, dev, cols=(s0, e0)) for s0, e0 in _cyclic_blocks(n_sk, b, p, me)]
                          or [torch.zeros(S, 0, dtype=wdt, device=dev)], 1)
            T = self._transposed() if cw else self.local
            if T.values().dtype != wdt:
                T = T.to(wdt)
            out = self._spmm(T, P.t().contiguous()).t().contiguous()     # S x |other|
        else:
            # generic transform: whole columns (rows) of the tile's block, then local apply
            full = torch.zeros(self.shape[0] if cw else self.shape[1],
                               (self.cols if cw else self.rows).numel(), dtype=wdt, device=dev)
            D = self.local.to_dense().to(wdt)
            full.index_copy_(0, gidx, D if cw else D.t().contiguous())
            if nshare > 1:
                comm.all_reduce(full)
            out = sk.apply(full, dim=0)
            return out if cw else out.t().contiguous()
        if nshare > 1:
            comm.all_reduce(out)
        return out if cw else out.t().contiguous()
