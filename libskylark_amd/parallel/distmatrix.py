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

    def row_blocks(self):
        """Global row ranges held locally (in local order)."""
        if self.layout in ("STAR_STAR", "STAR_VC", "STAR_VR"):
            return [(0, self.shape[0])]
        if self.layout == "CIRC_CIRC":
            return [(0, self.shape[0])] if self.comm.rank == 0 else []
        if is_row_dist(self.layout):
            return [self.row_range()]
        g = self.grid
        return _cyclic_blocks(self.shape[0], self.block[0], g.pr, g.myrow)

    def col_blocks(self):
        if self.layout in ("STAR_STAR", "VC_STAR", "VR_STAR"):
            return [(0, self.shape[1])]
        if self.layout == "CIRC_CIRC":
            return [(0, self.shape[1])] if self.comm.rank == 0 else []
        if is_col_dist(self.layout):
            return [self.col_range()]
        g = self.grid
        return _cyclic_blocks(self.shape[1], self.block[1], g.pc, g.mycol)

    def local_shape(self):
        return (sum(e - s for s, e in self.row_blocks()), sum(e - s for s, e in self.col_blocks()))

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

    def redistribute(self, layout: str, grid=None, block=None) -> "DistMatrix":
        layout = canon(layout)
        if layout == self.layout and (layout != "MC_MR" or (grid in (None, self.grid) and block in (None, self.block))):
            return self
        c = self.comm
        m, n = self.shape
        # fast paths
        if self.layout in ("VC_STAR", "VR_STAR") and layout == "STAR_STAR":
            counts = [self.row_range(r)[1] - self.row_range(r)[0] for r in range(c.size)]
            return DistMatrix(c.all_gather_v(self.local.contiguous(), counts, 0), self.shape, layout, c)
        if self.layout in ("STAR_VC", "STAR_VR") and layout == "STAR_STAR":
            counts = [self.col_range(r)[1] - self.col_range(r)[0] for r in range(c.size)]
            return DistMatrix(c.all_gather_v(self.local.contiguous(), counts, 1), self.shape, layout, c)
        if self.layout in ("VC_STAR", "VR_STAR") and layout in ("VC_STAR", "VR_STAR"):
            return DistMatrix(self.local, self.shape, layout, c)
        if self.layout in ("STAR_VC", "STAR_VR") and layout in ("STAR_VC", "STAR_VR"):
            return DistMatrix(self.local, self.shape, layout, c)
        if self.layout in ("VC_STAR", "VR_STAR") and layout in ("STAR_VC", "STAR_VR"):
            # all-to-all: send to rank q my rows restricted to q's columns
            sends = [self.local[:, slice(*self.col_range(q))].contiguous() for q in range(c.size)]
            recvs = c.all_to_all_v([s.reshape(-1) for s in sends])
            rows = [self.row_range(q) for q in range(c.size)]
            cs, ce = self.col_range()
            parts = [r.view(e - s, ce - cs) for r, (s, e) in zip(recvs, rows)]
            return DistMatrix(torch.cat(parts, 0), self.shape, layout, c)
        if self.layout in ("STAR_VC", "STAR_VR") and layout in ("VC_STAR", "VR_STAR"):
            sends = [self.local[slice(*self.row_range(q))].contiguous() for q in range(c.size)]
            recvs = c.all_to_all_v([s.reshape(-1) for s in sends])
            cols = [self.col_range(q) for q in range(c.size)]
            rs, re = self.row_range()
            parts = [r.view(re - rs, e - s) for r, (s, e) in zip(recvs, cols)]
            return DistMatrix(torch.cat(parts, 1), self.shape, layout, c)
        if layout == "CIRC_CIRC":
            full = self.to_global()
            loc = full if c.rank == 0 else torch.empty(0, 0, dtype=full.dtype, device=full.device)
            return DistMatrix(loc, self.shape, layout, c)
        if self.layout == "CIRC_CIRC":
            if c.rank == 0:
                buf = self.local.contiguous()
                meta = torch.tensor([1], device=buf.device)
            else:
                buf = torch.empty(self.shape, dtype=self.local.dtype, device=self.local.device)
            c.broadcast(buf, 0)
            return DistMatrix.from_global(buf, layout, c, grid, block)
        # general path: assemble the global matrix from every rank's tiles
        full = self._assemble_global()
        return DistMatrix.from_global(full, layout, c, grid, block)

    def _assemble_global(self) -> torch.Tensor:
        c = self.comm
        if self.layout == "STAR_STAR":
            return self.local
        m, n = self.shape
        full = torch.zeros(m, n, dtype=self.local.dtype, device=self.local.device)
        ro = 0
        for rs, re in self.row_blocks():
            co = 0
            for cs, ce in self.col_blocks():
                full[rs:re, cs:ce] = self.local[ro:ro + re - rs, co:co + ce - cs]
                co += ce - cs
            ro += re - rs
        if self.layout == "CIRC_CIRC":
            return c.broadcast(full, 0)
        return c.all_reduce(full)

    # ---------------------------------------------------------- helpers
    def __repr__(self):
        return f"DistMatrix({self.shape}, {self.layout}, local={tuple(self.local.shape)}, rank={self.comm.rank}/{self.comm.size})"

    def like(self, local: torch.Tensor, shape=None) -> "DistMatrix":
        return DistMatrix(local, shape or self.shape, self.layout, self.comm, self.grid, self.block)


def vc_star(A_local: torch.Tensor, m: int, comm: Comm | None = None) -> DistMatrix:
    return DistMatrix(A_local, (m, A_local.shape[1]), "VC_STAR", comm)
