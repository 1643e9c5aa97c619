"""Random dense matrices realised from GLOBAL indices.

Reference ``base/random_matrices.hpp:23-171``: ``RandomMatrix`` fills a local
or distributed matrix with iid samples indexed by the global (row, column)
position, so every distribution of the same matrix holds the same entries;
``GaussianMatrix`` / ``UniformMatrix`` are the common cases, and
``UniformMatrix`` for sparse matrices throws by design (``:157-171``).

Entry (i, j) of an m x n matrix is stream slot ``base + i + j*m`` (column-major,
as the reference's Elemental global index), drawn by the Threefry fill kernel
on the tensor's device; the context advances by ``m*n`` slots.
"""
from __future__ import annotations

import torch

from . import distributions as D
from .context import Context
from .exceptions import UnsupportedBaseOperation


def RandomMatrix(m: int, n: int, dist: D.Distribution, context: Context | None = None, *,
                 dtype=torch.float64, device=None, layout: str | None = None, comm=None, grid=None,
                 block=None, scale: float = 1.0, sparse: bool = False):
    """``m x n`` matrix of iid ``dist`` samples; local tensor, or a DistMatrix
    when ``layout`` is given (realised shard-locally, no communication)."""
    from .. import default_context
    from ..ops import rng
    if sparse:
        raise UnsupportedBaseOperation("random sparse matrices are not supported (reference behaviour)")
    ctx = context if context is not None else default_context()
    base = ctx.counter
    ctx.counter += m * n
    if layout is not None:
        from ..parallel.distmatrix import DistMatrix
        return DistMatrix.random((m, n), layout, comm, dist, ctx.seed, base, dtype, device, grid, block, scale)
    out = torch.empty(m, n, dtype=dtype, device=device)
    rng.fill_random(out, dist, ctx.seed, base, r0=0, c0=0, ir=1, ic=m, scale=scale,
                    precise=dtype == torch.float64)
    return out


def GaussianMatrix(m: int, n: int, context: Context | None = None, **kw):
    """iid N(0, 1) entries (``GaussianMatrix``, reference ``:132``)."""
    return RandomMatrix(m, n, D.Normal(), context, **kw)


def UniformMatrix(m: int, n: int, context: Context | None = None, a: float = 0.0, b: float = 1.0, **kw):
    """iid U(a, b) entries (``UniformMatrix``, reference ``:148``)."""
    return RandomMatrix(m, n, D.Uniform(a, b), context, **kw)


__all__ = ["RandomMatrix", "GaussianMatrix", "UniformMatrix"]
