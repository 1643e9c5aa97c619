"""Dense sketches: JLT (Gaussian) and CT (Cauchy).

Reference: ``sketch/JLT_data.hpp:17-78`` (scale ``sqrt(1/S)``, ``N*S`` normals
allocated lazily), ``sketch/CT_data.hpp:20-91`` (scale ``C/S``, ``N*S``
Cauchy samples), engine ``sketch/dense_transform_*``.
"""
from __future__ import annotations

import math

import torch

from ..base import distributions as D
from ..ops import dense_sketch as _ds
from ..ops import fused as _fused
from .base import COLUMNWISE, SketchTransform, register


class DenseSketch(SketchTransform):
    """S x N matrix with iid entries ``scale * dist`` realised from the stream."""

    dist = D.Normal()
    linear_shards = True   # S A = sum over row blocks of A of S[:, blk] A[blk] (streaming, distribution)

    def _scale(self) -> float:
        raise NotImplementedError

    precision = "exact"   # "bf16x2": bf16-rounded S on MFMA (see ops.dense_sketch.apply_dense)

    def _build(self, ctx):
        self.scale = self._scale()
        self.entries = ctx.allocate_random_samples_array(self._N * self._S, self.dist)

    def set_precision(self, precision: str):
        """"exact" (default) or "bf16x2" (fast internal sketches; GPU fp32 inputs)."""
        self.precision = precision
        return self

    # global realisation helpers (used by tests, nla and the distributed layer)
    def realize(self, dtype=torch.float64, device=None, rows=None, cols=None) -> torch.Tensor:
        r = rows or (0, self._S)
        c = cols or (0, self._N)
        return _ds.realize_panel(self.dist, self.entries.seed, self.entries.base, self._S, r, c,
                                 scale=self.scale, dtype=dtype, device=device,
                                 precise=dtype == torch.float64)

    def _apply_dense(self, A, dim, in_offset: int = 0, out_rows=None):
        k = A.shape[dim]
        i0, i1 = out_rows if out_rows is not None else (0, self._S)
        if _fused.fused_ok(A, dim, k, i1 - i0):
            # W block realised once (f64 sampler -> f32 -> bf16 hi/lo) and cached
            # on the device; one MFMA launch per apply (ops/fused.py)
            if getattr(self, "_wcache", None) is None:
                self._wcache = _fused.WCache()
            W = self._wcache.get((str(A.device), i0, i1, in_offset, k), lambda: self.realize(
                torch.float64, A.device, rows=(i0, i1), cols=(in_offset, in_offset + k)).float())
            return _fused.feature_gemm(A, W, dim, use_lo=self.precision != "bf16x2")
        return _ds.apply_dense(A, dim, dist=self.dist, seed=self.entries.seed, base=self.entries.base,
                               S=self._S, N=self._N, scale=self.scale, in_offset=in_offset,
                               out_rows=out_rows, precision=self.precision)

    def _apply_sparse(self, A, dim, sparse_out):
        return _ds.apply_sparse(A, dim, dist=self.dist, seed=self.entries.seed, base=self.entries.base,
                                S=self._S, N=self._N, scale=self.scale)

    # distributed hook: partial product of a shard along the sketched dim
    def apply_local_shard(self, A_local, dim, in_offset, out_rows=None):
        if A_local.layout == torch.sparse_csr:
            if out_rows is None:
                # panels of exactly this shard's sketch columns (no densification)
                return _ds.apply_sparse(A_local, dim, dist=self.dist, seed=self.entries.seed,
                                        base=self.entries.base, S=self._S, N=self._N, scale=self.scale,
                                        in_offset=in_offset)
            A_local = A_local.to_dense()
        return self._apply_dense(A_local, dim, in_offset=in_offset, out_rows=out_rows)


@register
class JLT(DenseSketch):
    """Johnson-Lindenstrauss transform: Gaussian S with scale sqrt(1/S)."""

    sketch_type = "JLT"
    dist = D.Normal()

    def _scale(self):
        return math.sqrt(1.0 / self._S)


@register
class CT(DenseSketch):
    """Cauchy transform (l1 embedding): Cauchy S with scale C/S."""

    sketch_type = "CT"
    dist = D.Cauchy()

    def __init__(self, n, s, C=1.0, context=None):
        self._C = float(C)
        super().__init__(n, s, context)

    def _scale(self):
        return self._C / self._S

    def _extra_params(self):
        return {"C": self._C}

    @classmethod
    def _params_from_dict(cls, d):
        return {"C": float(d["C"])}


@register
class SJLT(DenseSketch):
    """Sparse Johnson-Lindenstrauss transform (Achlioptas 2003; Li, Hastie,
    Church 2006): entries ``±sqrt(1/(density*S))`` with probability
    ``density/2`` each, zero otherwise, so ``E[S^T S] = I``.

    Reference: ``python-skylark/skylark/sketch.py:303-338`` (pure-Python
    only there; its ``_S`` construction refers to undefined names and omits
    the ``1/sqrt(S)`` scale its JLT uses — here entries follow the same
    counter layout as JLT, ``base + j*S + i``, so the operator is realisable
    lazily and shard-locally like every dense sketch).
    """

    sketch_type = "SJLT"

    def __init__(self, n, s, density=1.0 / 3.0, context=None):
        self._density = float(density)
        if not 0.0 < self._density <= 1.0:
            from ..base.exceptions import InvalidParametersError
            raise InvalidParametersError("SJLT density must be in (0, 1]")
        self.dist = D.SparseSign(self._density)
        super().__init__(n, s, context)

    def _scale(self):
        return math.sqrt(1.0 / self._S)

    def _extra_params(self):
        return {"density": self._density}

    @classmethod
    def _params_from_dict(cls, d):
        return {"density": float(d.get("density", 1.0 / 3.0))}


SparseJLT = SJLT

__all__ = ["JLT", "CT", "SJLT", "SparseJLT", "DenseSketch", "COLUMNWISE"]
