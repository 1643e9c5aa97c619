"""python-skylark ``skylark.elemhelper`` (``python-skylark/skylark/elemhelper.py``):
build distributed matrices entry by entry or from a replicated local one.

``layout`` is one of :data:`~.parallel.distmatrix.LAYOUTS` (the reference's
Elemental distribution types); every rank computes only its own entries."""
from __future__ import annotations

import torch

from .parallel.comm import world
from .parallel.distmatrix import DistMatrix, Grid, _merge


def create_distributed_matrix(m: int, n: int, f, layout: str = "MC_MR", comm=None, dtype=torch.float64,
                              device=None, grid=None, block=None) -> DistMatrix:
    """DistMatrix with entry (i, j) = f(i, j).  ``f`` may be vectorised: it is
    called once with broadcastable global index tensors (i as a column, j
    as a row) and falls back to a per-entry loop if that fails."""
    comm = comm or world()
    if layout == "MC_MR" and grid is None:
        grid = Grid.default(comm)
    D = DistMatrix.empty((m, n), layout, comm, dtype=dtype, device=device, grid=grid, block=block)
    rows = [i for s, e in _merge(D.row_blocks()) for i in range(s, e)]
    cols = [j for s, e in _merge(D.col_blocks()) for j in range(s, e)]
    I = torch.tensor(rows, dtype=torch.int64)[:, None]
    J = torch.tensor(cols, dtype=torch.int64)[None, :]
    try:
        vals = torch.as_tensor(f(I, J), dtype=dtype)
        vals = vals.expand(len(rows), len(cols))
    except Exception:  # noqa: BLE001 - scalar-only f
        vals = torch.tensor([[float(f(i, j)) for j in cols] for i in rows], dtype=dtype).reshape(len(rows), len(cols))
    D.local.copy_(vals.to(D.local.device))
    return D


create_elemental_matrix = create_distributed_matrix


def local2distributed(A, layout: str = "MC_MR", comm=None, grid=None, block=None) -> DistMatrix:
    """DistMatrix of a matrix replicated on every rank (each keeps its part)."""
    A = torch.as_tensor(A)
    comm = comm or world()
    if layout == "MC_MR" and grid is None:
        grid = Grid.default(comm)
    return DistMatrix.from_global(A, layout, comm, grid=grid, block=block)
