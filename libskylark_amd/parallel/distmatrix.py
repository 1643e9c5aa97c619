"""Distributed dense matrices over one process per GPU.

Replaces Elemental's ``DistMatrix<T, U, V>`` family (reference type names in
``utility/types.hpp:8-70``).  Layouts:

=============  ======================  =====================================
layout         Elemental analogue      storage on rank r
=============  ======================  =====================================
``STAR_STAR``  ``[*,*]`` (Shared)      whole matrix (replicated)
``CIRC_CIRC``  ``[CIRC,CIRC]`` (Root)  whole matrix on rank 0, empty elsewhere
``VC_STAR``    ``[VC,*]``              contiguous row block r (1-D rows)
``VR_STAR``    ``[VR,*]``              same as VC_STAR (alias)
``STAR_VC``    ``[*,VC]``              contiguous column block r
``STAR_VR``    ``[*,VR]``              same as STAR_VC (alias)
``MC_MR``      ``[MC,MR]``             2-D block-cyclic tiles over a pr x pc grid
=============  ======================  =====================================

MI355X-first choices: 1-D layouts use *contiguous* blocks (coalesced,
one GEMM per shard) instead of element-cyclic ones; because every random
sketch entry is indexed by GLOBAL coordinates, results are independent of the
layout and of the GPU count (the reference's "distributed == local" test
invariant, ``tests/unit/DenseSketchApplyElementalTest.cpp:52-101``).  The 2-D
layout is block-cyclic with tile ``(mb, nb)`` (default: one tile per rank,
i.e. plain 2-D block) and carries row / column sub-communicators (the
analogues of Elemental's MC / MR communicators).
"""
from __future__ import annotations

import math

import torch

from .comm import balanced_counts, Comm, balanced_offsets, world

LAYOUTS = ("STAR_STAR", "CIRC_CIRC", "VC_STAR", "VR_STAR", "STAR_VC", "STAR_VR", "MC_MR")
ALIASES = {"SharedMatrix": "STAR_STAR", "RootMatrix": "CIRC_CIRC", "DistMatrix": "MC_MR",
           "DistMatrix_VC_STAR": "VC_STAR", "DistMatrix_VR_STAR": "VR_STAR",
           "DistMatrix_STAR_VC": "STAR_VC", "DistMatrix_STAR_VR": "STAR_VR",
           "[*,*]": "STAR_STAR", "[CIRC,CIRC]": "CIRC_CIRC", "[VC,*]": "VC_STAR", "[VR,*]": "VR_STAR",
           "[*,VC]": "STAR_VC", "[*,VR]": "STAR_VR", "[MC,MR]": "MC_MR"}


def canon(layout: str) -> str:
    layout = ALIASES.get(layout, layout)
    if layout not in LAYOUTS:
        raise ValueError(f"unknown layout {layout}")
    return layout


def is_row_dist(layout):
    return layout in ("VC_STAR", "VR_STAR")


def is_col_dist(layout):
    return layout in ("STAR_VC", "STAR_VR")


class Grid:
    """pr x pc process grid with row/column sub-communicators (created collectively)."""

    _cache = {}

    def __init__(self, comm: Comm, pr: int | None = None):
        p = comm.size
        if pr is None:
            pr = int(math.sqrt(p))
            while p % pr:
                pr -= 1
        self.pr, self.pc = pr, p // pr
        self.comm = comm
        self.myrow = comm.rank % self.pr      # column-major rank -> (row, col), like Elemental
        self.mycol = comm.rank // self.pr
        # ranks with the same grid column form a "column communicator" (vary over rows: MC)
        self.col_comm = comm.split(self.mycol, self.myrow)
        self.row_comm = comm.split(self.myrow, self.mycol)

    @classmethod
    def default(cls, comm: Comm | None = None, pr=None):
        comm = comm or world()
        key = (id(comm.group), comm.size, pr)
        g = cls._cache.get(key)
        if g is None:
            g = cls(comm, pr)
            cls._cache[key] = g
        return g


def _cyclic_blocks(n: int, b: int, p: int, me: int):
    """Global [start, end) ranges of the tiles owned by coordinate me."""
    out = []
    nblk = (n + b - 1) // b
    for k in range(me, nblk, p):
        out.append((k * b, min(n, (k + 1) * b)))
    return out


class DistMatrix:
    """A distributed ``m x n`` matrix: local shard + global shape + layout."""

    def __init__(self, local: torch.Tensor, shape, layout: str = "VC_STAR", comm: Comm | None = None,
                 grid: Grid | None = None, block=None):
        self.layout = canon(layout)
        self.comm = comm or world()
        self.shape = (int(shape[0]), int(shape[1]))
        self.local = local
        self.grid = grid
        self.block = block
        if self.layout == "MC_MR":
            self.grid = grid or Grid.default(self.comm)
            if block is None:
                self.block = (max(1, -(-self.shape[0] // self.grid.pr)), max(1, -(-self.shape[1] // self.grid.pc)))

    # ----------------------------------------------------------- geometry
    @property
    def height(self):
        return self.shape[0]

    @property
    def width(self):
        return self.shape[1]

    @property
    def dtype(self):
        return self.local.dtype

    @property
    def device(self):
        return self.local.device

    def row_range(self, rank=None):
        rank = self.comm.rank if rank is None else rank
        off = balanced_offsets(self.shape[0], self.comm.size)
        return off[rank], off[rank + 1]

    def col_range(self, rank=None):
        rank = self.comm.rank if rank is None else rank
        off = balanced_offsets(self.shape[1], self.comm.size)
        return off[rank], off[rank + 1]

    def row_counts(self):
        """Rows held by every rank, for the 1-D row layouts ([VC,*]/[VR,*])."""
        return balanced_counts(self.shape[0], self.comm.size)

    def row_blocks(self, rank=None):
        """Global row ranges held by ``rank`` (default: this rank), in local order."""
        rank = self.comm.rank if rank is None else rank
        if self.layout in ("STAR_STAR", "STAR_VC", "STAR_VR"):
            return [(0, self.shape[0])]
        if self.layout == "CIRC_CIRC":
            return [(0, self.shape[0])] if rank == 0 else []
        if is_row_dist(self.layout):
            return [self.row_range(rank)]
        g = self.grid
        return _cyclic_blocks(self.shape[0], self.block[0], g.pr, rank % g.pr)

    def col_blocks(self, rank=None):
        rank = self.comm.rank if rank is None else rank
        if self.layout in ("STAR_STAR", "VC_STAR", "VR_STAR"):
            return [(0, self.shape[1])]
        if self.layout == "CIRC_CIRC":
            return [(0, self.shape[1])] if rank == 0 else []
        if is_col_dist(self.layout):
            return [self.col_range(rank)]
        g = self.grid
        return _cyclic_blocks(self.shape[1], self.block[1], g.pc, rank // g.pr)

    def local_shape(self, rank=None):
        return (sum(e - s for s, e in self.row_blocks(rank)), sum(e - s for s, e in self.col_blocks(rank)))

    # ----------------------------------------------------- construction
    @classmethod
    def empty(cls, shape, layout="VC_STAR", comm=None, dtype=torch.float32, device=None, grid=None, block=None):
        d = cls(torch.empty(0), shape, layout, comm, grid, block)
        d.local = torch.empty(d.local_shape(), dtype=dtype, device=device)
        return d

    @classmethod
    def zeros(cls, shape, layout="VC_STAR", comm=None, dtype=torch.float32, device=None, grid=None, block=None):
        d = cls.empty(shape, layout, comm, dtype, device, grid, block)
        d.local.zero_()
        return d

    @classmethod
    def from_global(cls, A: torch.Tensor, layout="VC_STAR", comm=None, grid=None, block=None):
        """Build from a matrix every rank holds (slices locally; no communication)."""
        d = cls(torch.empty(0), tuple(A.shape), layout, comm, grid, block)
        rb, cb = d.row_blocks(), d.col_blocks()
        if not rb or not cb:
            d.local = torch.empty(d.local_shape(), dtype=A.dtype, device=A.device)
            return d
        rows = torch.cat([A[s:e] for s, e in rb], 0) if len(rb) > 1 else A[rb[0][0]:rb[0][1]]
        d.local = torch.cat([rows[:, s:e] for s, e in cb], 1) if len(cb) > 1 else rows[:, cb[0][0]:cb[0][1]]
        d.local = d.local.contiguous()
        return d

    @classmethod
    def random(cls, shape, layout="VC_STAR", comm=None, dist=None, seed=0, base=0, dtype=torch.float32,
               device=None, grid=None, block=None, scale=1.0):
        """Random matrix realised shard-locally from global indices (reference
        ``GaussianMatrix``/``UniformMatrix``, ``base/random_matrices.hpp:23-171``)."""
        from ..base import distributions as D
        from ..ops import rng
        dist = dist or D.Normal()
        d = cls.empty(shape, layout, comm, dtype, device, grid, block)
        ro = 0
        for rs, re in d.row_blocks():
            co = 0
            for cs, ce in d.col_blocks():
                view = d.local[ro:ro + re - rs, co:co + ce - cs]
                rng.fill_random(view, dist, seed, base, r0=rs, c0=cs, ir=1, ic=shape[0], scale=scale)
                co += ce - cs
            ro += re - rs
        return d

    # ------------------------------------------------------- conversion
    def to_global(self) -> torch.Tensor:
        """Replicated copy of the whole matrix on every rank (all-gather)."""
        return self.redistribute("STAR_STAR").local

    def redistribute(self, layout: str, grid=None, block=None, out: torch.Tensor | None = None) -> "DistMatrix":
        """Return this matrix in another layout.

        Replicated sources are sliced locally (no communication).  Every other
        pair is ONE ``all_to_all_single``: rank s sends rank d exactly the
        entries (rows(s) & rows(d)) x (cols(s) & cols(d)), packed row-major, so
        a rank puts at most its own shard on the wire (``[*,*]`` targets
        excepted, which are all-gathers by definition; ``[CIRC,CIRC]`` is a
        gather / scatter through rank 0).  The pack / unpack index plans are
        cached per geometry, so a repeated redistribution (e.g. the ``[MC,MR]``
        -> ``[VC,*]`` step inside randSVD) issues only device gathers, the
        collective and device scatters.  Replaces Elemental's implicit
        redistributions (``A1_VC_STAR = A1``, ``[*,VC]`` <->
        ``[VC,*]`` in FJLT_Elemental.hpp:150, RFUT_Elemental.hpp:335, ...).

        ``out``: optional destination buffer (this rank's shard shape) reused
        by callers that redistribute the same operand repeatedly."""
        layout = canon(layout)
        if layout == self.layout and (layout != "MC_MR" or (grid in (None, self.grid) and block in (None, self.block))):
            return self
        c = self.comm
        dst = DistMatrix(torch.empty(0, dtype=self.local.dtype, device=self.local.device), self.shape, layout, c,
                         grid, block)
        if self.layout == "STAR_STAR":
            return DistMatrix.from_global(self.local, layout, c, dst.grid, dst.block)
        if c.size == 1 or _same_storage_cached(self, dst):
            # identical local storage (e.g. any layout on one rank): no copy
            return DistMatrix(self.local, self.shape, layout, c, dst.grid, dst.block)
        if is_row_dist(self.layout) and layout == "STAR_STAR":
            counts = [self.row_range(r)[1] - self.row_range(r)[0] for r in range(c.size)]
            return DistMatrix(c.all_gather_v(self.local.contiguous(), counts, 0), self.shape, layout, c)
        if is_col_dist(self.layout) and layout == "STAR_STAR":
            counts = [self.col_range(r)[1] - self.col_range(r)[0] for r in range(c.size)]
            return DistMatrix(c.all_gather_v(self.local.contiguous(), counts, 1), self.shape, layout, c)
        plan = _redist_plan(self, dst)
        dst.local = plan.run(self.local, c, out)
        return dst

    def _same_storage(self, other: "DistMatrix") -> bool:
        """True when every rank stores exactly the same global entries in the
        same order under both layouts (checked for all ranks: a collective-free
        decision every rank takes identically)."""
        for r in range(self.comm.size):
            if _merge(self.row_blocks(r)) != _merge(other.row_blocks(r)) or \
                    _merge(self.col_blocks(r)) != _merge(other.col_blocks(r)):
                return False
        return True

    def _assemble_global(self) -> torch.Tensor:
        """Whole matrix on every rank (an all-gather; for diagnostics)."""
        return self.redistribute("STAR_STAR").local

    # ---------------------------------------------------------- helpers
    def __repr__(self):
        return f"DistMatrix({self.shape}, {self.layout}, local={tuple(self.local.shape)}, rank={self.comm.rank}/{self.comm.size})"

    def like(self, local: torch.Tensor, shape=None) -> "DistMatrix":
        return DistMatrix(local, shape or self.shape, self.layout, self.comm, self.grid, self.block)


def _merge(ranges):
    """Coalesce adjacent [s, e) ranges."""
    out = []
    for s, e in ranges:
        if e <= s:
            continue
        if out and out[-1][1] == s:
            out[-1] = (out[-1][0], e)
        else:
            out.append((s, e))
    return out


def _intersect(a, b):
    """Intersection of two sorted lists of disjoint [s, e) ranges."""
    out, i, j = [], 0, 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append((s, e))
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def _local_positions(owned, sub):
    """Positions, in the local storage whose global index ranges are
    ``owned`` (local order = concatenation), of the global ranges ``sub``
    (each inside one owned range).  Returns ``(start, length)`` when they are
    one contiguous run, else an int64 numpy array."""
    import bisect
    import numpy as np
    starts = [s for s, _ in owned]
    pref = [0]
    for s, e in owned:
        pref.append(pref[-1] + e - s)
    runs = []
    for s, e in sub:
        i = bisect.bisect_right(starts, s) - 1
        p = pref[i] + s - owned[i][0]
        if runs and runs[-1][0] + runs[-1][1] == p:
            runs[-1] = (runs[-1][0], runs[-1][1] + e - s)
        else:
            runs.append((p, e - s))
    if len(runs) <= 1:
        return runs[0] if runs else (0, 0)
    return np.concatenate([np.arange(p, p + n, dtype=np.int64) for p, n in runs])


class _RedistPlan:
    """Pack / exchange / unpack schedule of one (src geometry, dst geometry)
    pair on this rank.  Index maps live on the data's device."""

    def __init__(self, src: DistMatrix, dst: DistMatrix, device):
        c = src.comm
        me = c.rank
        self.dst_shape = dst.local_shape(me)
        sr, sc = src.row_blocks(me), src.col_blocks(me)
        dr, dc = dst.row_blocks(me), dst.col_blocks(me)
        self.send, self.recv = [], []
        for d in range(c.size):
            ri = _intersect(sr, dst.row_blocks(d))
            ci = _intersect(sc, dst.col_blocks(d))
            nr, nc = sum(e - s for s, e in ri), sum(e - s for s, e in ci)
            self.send.append(None if nr * nc == 0 else
                             (self._idx(_local_positions(sr, ri), device), self._idx(_local_positions(sc, ci), device),
                              nr, nc))
        for s_ in range(c.size):
            ri = _intersect(src.row_blocks(s_), dr)
            ci = _intersect(src.col_blocks(s_), dc)
            nr, nc = sum(e - s for s, e in ri), sum(e - s for s, e in ci)
            self.recv.append(None if nr * nc == 0 else
                             (self._idx(_local_positions(dr, ri), device), self._idx(_local_positions(dc, ci), device),
                              nr, nc))

    @staticmethod
    def _idx(pos, device):
        if isinstance(pos, tuple):
            return slice(pos[0], pos[0] + pos[1])
        return torch.from_numpy(pos).to(device)

    @staticmethod
    def _take(X, ri, ci):
        X = X[ri] if isinstance(ri, slice) else X.index_select(0, ri)
        return X[:, ci] if isinstance(ci, slice) else X.index_select(1, ci)

    @staticmethod
    def _put(X, ri, ci, P):
        if isinstance(ri, slice) and isinstance(ci, slice):
            X[ri, ci] = P
        elif isinstance(ri, slice):
            X[ri].index_copy_(1, ci, P)
        elif isinstance(ci, slice):
            X.index_copy_(0, ri, P) if (ci.start == 0 and ci.stop == X.shape[1]) else X[:, ci].index_copy_(0, ri, P)
        else:
            X.index_put_((ri[:, None], ci[None, :]), P)

    def run(self, local: torch.Tensor, comm, out: torch.Tensor | None = None) -> torch.Tensor:
        dt, dev = local.dtype, local.device
        sends = []
        for d, e in enumerate(self.send):
            if e is None:
                sends.append(torch.empty(0, dtype=dt, device=dev))
            else:
                ri, ci, nr, nc = e
                sends.append(self._take(local, ri, ci).reshape(-1))
        rcounts = [0 if e is None else e[2] * e[3] for e in self.recv]
        recvs = comm.all_to_all_v(sends, recv_counts=rcounts)
        if out is None or tuple(out.shape) != tuple(self.dst_shape) or out.dtype != dt or out.device != dev:
            out = torch.empty(self.dst_shape, dtype=dt, device=dev)
        for e, P in zip(self.recv, recvs):
            if e is not None:
                ri, ci, nr, nc = e
                self._put(out, ri, ci, P.view(nr, nc))
        return out


_PLANS: dict = {}
_SAME: dict = {}


def _same_storage_cached(src: DistMatrix, dst: DistMatrix) -> bool:
    key = (_geom_key(src), _geom_key(dst), src.comm.size)
    v = _SAME.get(key)
    if v is None:
        if len(_SAME) >= 256:
            _SAME.clear()
        v = _SAME[key] = src._same_storage(dst)
    return v


def _geom_key(A: DistMatrix):
    g = A.grid
    return (A.layout, A.shape, None if g is None else (g.pr, g.pc), A.block)


def _redist_plan(src: DistMatrix, dst: DistMatrix) -> _RedistPlan:
    key = (_geom_key(src), _geom_key(dst), src.comm.rank, src.comm.size, id(src.comm.group), str(src.local.device))
    p = _PLANS.get(key)
    if p is None:
        if len(_PLANS) >= 32:
            _PLANS.pop(next(iter(_PLANS)))
        p = _PLANS[key] = _RedistPlan(src, dst, src.local.device)
    return p


def vc_star(A_local: torch.Tensor, m: int, comm: Comm | None = None) -> DistMatrix:
    return DistMatrix(A_local, (m, A_local.shape[1]), "VC_STAR", comm)
