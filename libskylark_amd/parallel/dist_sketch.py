"""Distributed sketch application over :class:`DistMatrix`.

Reference: the per-layout ``dense_transform_Elemental_*`` /
``hash_transform_Elemental*`` / ``*_Elemental.hpp`` specialisations and their
collective call sites.  MI355X-native communication plan:

* sketched dimension NOT distributed (``[*,VC]`` columnwise, ``[VC,*]``
  rowwise, ``[*,*]``): every GPU sketches its own columns/rows — no
  communication at all (the random entries are indexed globally);
* sketched dimension distributed (``[VC,*]`` columnwise, ``[*,VC]`` rowwise):
  each GPU computes the partial product of its shard (RNG-GEMM / CountSketch
  kernel), then ONE collective: all-reduce (→ ``[*,*]``), reduce (→
  ``[CIRC,CIRC]``) or reduce-scatter (→ same 1-D layout).  Non-linear feature
  maps (RFT/RLT) reduce the linear part first and apply the cos/exp epilogue
  after;
* ``[MC,MR]``: partial products over each tile, summed inside the grid-column
  communicator (the reference's ``panel_matrix_gemm`` reduce-scatter,
  ``sketch/dense_transform_Elemental_mc_mr.hpp:545-615``);
* transforms that need the whole sketched dimension on one GPU (FFT-based
  FJLT, Fastfood, PPT) redistribute with one all-to-all first.
"""
from __future__ import annotations

import torch

from ..base.exceptions import DimensionMismatchError
from .distmatrix import DistMatrix, canon, is_col_dist, is_row_dist

COLUMNWISE, ROWWISE = 0, 1


def _kind(sk):
    name = sk.sketch_type
    if name in ("PPT", "FastGaussianRFT", "FastMaternRFT"):
        return "local_only"
    if hasattr(sk, "linear_local_shard"):
        return "feature"
    if name == "FJLT":
        from ..sketch.fjlt import DIRECT_MAX_S
        return "linear" if sk.getsketchdim() <= DIRECT_MAX_S else "local_only"
    if name == "UST":
        return "local_only"
    return "linear"


def _sketched_dim_local(layout, dim):
    if layout in ("STAR_STAR", "CIRC_CIRC"):
        return True
    return is_col_dist(layout) if dim == COLUMNWISE else is_row_dist(layout)


def _local_full_apply(sk, A: DistMatrix, dim):
    S = sk.getsketchdim()
    if A.layout == "CIRC_CIRC" and A.comm.rank != 0:
        shape = (S, A.shape[1]) if dim == COLUMNWISE else (A.shape[0], S)
        return DistMatrix(torch.empty(0, 0, dtype=A.local.dtype, device=A.local.device), shape, "CIRC_CIRC", A.comm)
    loc = sk.apply(A.local, None, dim)
    if not isinstance(loc, torch.Tensor):
        loc = torch.as_tensor(loc)
    if loc.layout != torch.strided:
        loc = loc.to_dense()
    shape = (S, A.shape[1]) if dim == COLUMNWISE else (A.shape[0], S)
    return DistMatrix(loc, shape, A.layout, A.comm, A.grid, None if A.layout != "MC_MR" else A.block)


def dist_apply(sk, A: DistMatrix, SA=None, dim=COLUMNWISE, out_layout: str | None = None):
    N, S = sk.getindim(), sk.getsketchdim()
    if A.shape[dim] != N:
        raise DimensionMismatchError(f"Sketched dimension is incorrect (input): {A.shape[dim]} != {N}")
    if isinstance(SA, DistMatrix):
        out_layout = SA.layout
    out_layout = canon(out_layout or A.layout)
    kind = _kind(sk)
    out_shape = (S, A.shape[1]) if dim == COLUMNWISE else (A.shape[0], S)

    if _sketched_dim_local(A.layout, dim):
        R = _local_full_apply(sk, A, dim)
    elif kind == "local_only":
        tmp = A.redistribute("STAR_VC" if dim == COLUMNWISE else "VC_STAR")
        R = _local_full_apply(sk, tmp, dim)
    else:
        R = _partial_and_reduce(sk, A, dim, kind, out_layout, out_shape)
    if R.layout != out_layout:
        R = R.redistribute(out_layout)
    if isinstance(SA, DistMatrix):
        SA.local = R.local
        return SA
    return R


def _partial(sk, A: DistMatrix, dim, kind):
    """Sum of the linear part over this rank's blocks along the sketched dim."""
    blocks_d = A.row_blocks() if dim == COLUMNWISE else A.col_blocks()
    fn = sk.linear_local_shard if kind == "feature" else sk.apply_local_shard
    out = None
    off = 0
    for s, e in blocks_d:
        blk = A.local[off:off + e - s] if dim == COLUMNWISE else A.local[:, off:off + e - s]
        off += e - s
        part = fn(blk, dim, s)
        out = part if out is None else out + part
    if out is None:
        S = sk.getsketchdim()
        other = A.local.shape[1] if dim == COLUMNWISE else A.local.shape[0]
        shape = (S, other) if dim == COLUMNWISE else (other, S)
        dt = torch.float64 if A.local.dtype == torch.float64 else torch.float32
        out = torch.zeros(shape, dtype=dt, device=A.local.device)
    return out.contiguous()


def _use_outer_panel(sk, A: DistMatrix, dim, kind) -> bool:
    """Outer-panel vs panel-matrix for a columnwise dense sketch of an [MC,MR]
    matrix (reference selector ``dense_transform_Elemental_mc_mr.hpp:617-656``):
    gathering the input panel (N x m/pc per grid column) beats reducing the
    output panel (S x m/pc) when S exceeds factor * N / 20 (equal collective
    volumes at the default factor)."""
    from ..sketch import params
    from ..sketch.dense import DenseSketch
    if kind != "linear" or dim != COLUMNWISE or not isinstance(sk, DenseSketch):
        return False
    if A.local.layout != torch.strided or A.grid.pr == 1:
        return False
    N, S = sk.getindim(), sk.getsketchdim()
    return S * 20 > N * params.get_factor()


def _outer_panel(sk, A: DistMatrix, out_shape):
    """All-gather A's rows inside the grid column, then every rank realises
    only ITS output rows of S over the full N: no reduction of the output."""
    from .distmatrix import _cyclic_blocks
    g = A.grid
    N, S = sk.getindim(), sk.getsketchdim()
    counts, order = [], []
    for r in range(g.pr):
        blk = _cyclic_blocks(N, A.block[0], g.pr, r)
        counts.append(sum(e - s for s, e in blk))
        order.extend(i for s, e in blk for i in range(s, e))
    G = g.col_comm.all_gather_v(A.local.contiguous(), counts, 0)
    full = torch.empty_like(G)
    full[torch.tensor(order, device=G.device)] = G
    R = DistMatrix(torch.empty(0), out_shape, "MC_MR", A.comm, g, (max(1, -(-S // g.pr)), A.block[1]))
    parts = [sk.apply_local_shard(full, COLUMNWISE, 0, out_rows=(s, e)) for s, e in R.row_blocks()]
    if parts:
        R.local = torch.cat(parts, 0).contiguous()
    else:
        dt = torch.float64 if A.local.dtype == torch.float64 else torch.float32
        R.local = torch.zeros(0, full.shape[1], dtype=dt, device=full.device)
    return R


def _partial_and_reduce(sk, A: DistMatrix, dim, kind, out_layout, out_shape):
    c = A.comm
    part = _partial(sk, A, dim, kind)
    finish = (lambda X, rows=None: sk.finish_features(X, dim, rows)) if kind == "feature" else None
    S = sk.getsketchdim()

    if A.layout == "MC_MR" and _use_outer_panel(sk, A, dim, kind):
        return _outer_panel(sk, A, out_shape)
    if A.layout == "MC_MR":
        g = A.grid
        # the sketched dimension is spread over grid rows (columnwise: sum over
        # the grid-column communicator) or grid columns (rowwise: grid-row comm)
        (g.col_comm if dim == COLUMNWISE else g.row_comm).all_reduce(part)
        if finish is not None:
            part = finish(part)
        if dim == COLUMNWISE:
            R = DistMatrix(torch.empty(0), out_shape, "MC_MR", c, g, (A.block[0] if A.block else None, A.block[1]))
            R.block = (max(1, -(-S // g.pr)), A.block[1])
            rows = R.row_blocks()
            R.local = torch.cat([part[s:e] for s, e in rows], 0) if rows else part[:0]
        else:
            R = DistMatrix(torch.empty(0), out_shape, "MC_MR", c, g, (A.block[0], max(1, -(-S // g.pc))))
            cols = R.col_blocks()
            R.local = torch.cat([part[:, s:e] for s, e in cols], 1) if cols else part[:, :0]
        R.local = R.local.contiguous()
        return R

    if out_layout == "CIRC_CIRC":
        c.reduce(part, 0)
        if c.rank == 0:
            if finish is not None:
                part = finish(part)
            return DistMatrix(part, out_shape, "CIRC_CIRC", c)
        return DistMatrix(torch.empty(0, 0, dtype=part.dtype, device=part.device), out_shape, "CIRC_CIRC", c)

    sdim_out = 0 if dim == COLUMNWISE else 1  # which output dim has extent S
    same_1d = (dim == COLUMNWISE and is_row_dist(out_layout)) or (dim == ROWWISE and is_col_dist(out_layout))
    if same_1d and finish is None:
        from .comm import balanced_counts
        counts = balanced_counts(S, c.size)
        loc = c.reduce_scatter_v(part, counts, sdim_out)
        return DistMatrix(loc, out_shape, out_layout, c)
    c.all_reduce(part)
    if finish is not None:
        part = finish(part)
    return DistMatrix(part, out_shape, "STAR_STAR", c)
