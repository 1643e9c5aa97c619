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
from .distmatrix import DistMatrix, _cyclic_blocks, canon, is_col_dist, is_row_dist

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


def _mc_mr_algorithm(sk, A: DistMatrix, dim, kind) -> str:
    """Panel algorithm for a sketch of an [MC,MR] matrix: ``params.mc_mr_algorithm``
    forces one ("inner" / "outer" / "panel"); "auto" takes the reference's
    inner-panel regime (both output dimensions below 1/factor of the sketched
    one, ``dense_transform_Elemental_mc_mr.hpp:640-656``) and otherwise the
    collective-volume rule of :func:`_use_outer_panel`."""
    from ..sketch import params
    forced = params.get_mc_mr_algorithm()
    if kind != "linear" or A.local.layout != torch.strided:
        return "panel"
    if forced != "auto":
        if forced == "outer" and not (dim == COLUMNWISE and A.grid.pr > 1):
            return "panel"
        return forced
    N = A.shape[0] if dim == COLUMNWISE else A.shape[1]
    width = A.shape[1] if dim == COLUMNWISE else A.shape[0]
    S, f = sk.getsketchdim(), params.get_factor()
    if S * f <= N and width * f <= N:
        return "inner"
    return "outer" if _use_outer_panel(sk, A, dim, kind) else "panel"


def _owner_order(n, b, p):
    """(counts per coordinate, global indices in coordinate-major order) of a
    block-cyclic distribution of n entries in blocks of b over p coordinates."""
    counts, order = [], []
    for r in range(p):
        blk = _cyclic_blocks(n, b, p, r)
        counts.append(sum(e - s for s, e in blk))
        order.extend(i for s, e in blk for i in range(s, e))
    return counts, order


def _panel_matrix(part, sk, A: DistMatrix, dim, out_shape, finish):
    """Panel-matrix algorithm: this rank's partial product over its tiles of
    the sketched dimension, then ONE reduce-scatter inside the grid-column
    (columnwise) or grid-row (rowwise) communicator straight into the output's
    block-cyclic rows / columns (reference ``panel_matrix_gemm`` with
    ``AxpyContract``, ``dense_transform_Elemental_mc_mr.hpp:545-615``)."""
    g = A.grid
    c = A.comm
    S = sk.getsketchdim()
    if dim == COLUMNWISE:
        comm, p, me = g.col_comm, g.pr, g.myrow
        bS = max(1, -(-S // g.pr))
        block = (bS, A.block[1])
    else:
        comm, p, me = g.row_comm, g.pc, g.mycol
        bS = max(1, -(-S // g.pc))
        block = (A.block[0], bS)
    counts, order = _owner_order(S, bS, p)
    sdim = 0 if dim == COLUMNWISE else 1
    if order != list(range(S)):
        part = part.index_select(sdim, torch.tensor(order, device=part.device))
    loc = comm.reduce_scatter_v(part.contiguous(), counts, sdim) if p > 1 else part
    if finish is not None:
        pieces, off = [], 0
        for s0, e0 in _cyclic_blocks(S, bS, p, me):
            blk = loc[off:off + e0 - s0] if dim == COLUMNWISE else loc[:, off:off + e0 - s0]
            pieces.append(finish(blk, (s0, e0)))
            off += e0 - s0
        if pieces:
            loc = torch.cat(pieces, sdim)
    return DistMatrix(loc.contiguous(), out_shape, "MC_MR", c, g, block)


def _inner_panel(sk, A: DistMatrix, dim, out_shape):
    """Inner-panel algorithm (reference ``inner_panel_gemm``,
    ``dense_transform_Elemental_mc_mr.hpp:211-326``): the input is
    redistributed once to a 1-D layout over the WHOLE grid along the sketched
    dimension (one all-to-all), every rank contracts its slice for a panel of
    b sketch rows, and the small panel x width partial is reduce-scattered over
    the whole grid straight into the output's [MC,MR] tiles.  Memory per rank:
    one b x N_loc panel of S."""
    from ..sketch import params
    g = A.grid
    c = A.comm
    S = sk.getsketchdim()
    if dim == COLUMNWISE:
        A1 = A.redistribute("VC_STAR")
        width = A.shape[1]
    else:
        A1 = A.redistribute("STAR_VC")
        width = A.shape[0]
    (s_in, e_in), = A1.row_blocks() if dim == COLUMNWISE else A1.col_blocks()
    block = (max(1, -(-S // g.pr)), A.block[1]) if dim == COLUMNWISE else (A.block[0], max(1, -(-S // g.pc)))
    R = DistMatrix(torch.empty(0), out_shape, "MC_MR", c, g, block)
    b = params.get_blocksize() or S
    # destination tiles of every rank of the grid: (its sketch rows, its width cols)
    dest = []
    for rk in range(c.size):
        dest.append((R.row_blocks(rk) if dim == COLUMNWISE else R.col_blocks(rk),
                     R.col_blocks(rk) if dim == COLUMNWISE else R.row_blocks(rk)))
    pieces = []
    for p0 in range(0, S, b):
        p1 = min(S, p0 + b)
        part = sk.apply_local_shard(A1.local, dim, s_in, out_rows=(p0, p1))   # (p1-p0) x width (col) / width x .. (row)
        if dim == ROWWISE:
            part = part.t()
        part = part.contiguous()
        sends, counts = [], []
        for srows, wcols in dest:
            ri = [i - p0 for s0, e0 in srows for i in range(max(s0, p0), min(e0, p1))]
            ci = [j for s0, e0 in wcols for j in range(s0, e0)]
            if ri and ci:
                t = part.index_select(0, torch.tensor(ri, device=part.device)).index_select(
                    1, torch.tensor(ci, device=part.device))
            else:
                t = part.new_zeros(0)
            sends.append(t.reshape(-1))
            counts.append(t.numel())
        flat = torch.cat(sends) if sends else part.new_zeros(0)
        mine = c.reduce_scatter_v(flat, counts, 0) if c.size > 1 else flat
        myrows = [i for s0, e0 in dest[c.rank][0] for i in range(max(s0, p0), min(e0, p1))]
        mycols = sum(e0 - s0 for s0, e0 in dest[c.rank][1])
        pieces.append(mine.view(len(myrows), mycols))
    loc = torch.cat(pieces, 0) if pieces else torch.zeros(0, 0)
    R.local = (loc if dim == COLUMNWISE else loc.t()).contiguous()
    return R


def _partial_and_reduce(sk, A: DistMatrix, dim, kind, out_layout, out_shape):
    c = A.comm
    if A.layout == "MC_MR":
        algo = _mc_mr_algorithm(sk, A, dim, kind)
        if algo == "inner":
            return _inner_panel(sk, A, dim, out_shape)
        if algo == "outer" and dim == COLUMNWISE:
            return _outer_panel(sk, A, out_shape)
    part = _partial(sk, A, dim, kind)
    finish = (lambda X, rows=None: sk.finish_features(X, dim, rows)) if kind == "feature" else None
    S = sk.getsketchdim()

    if A.layout == "MC_MR":
        return _panel_matrix(part, sk, A, dim, out_shape, finish)

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
