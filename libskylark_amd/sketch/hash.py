"""Hashing sketches: CWT (CountSketch), MMT (Meng-Mahoney), WZT (Woodruff-Zhang).

Reference data classes: ``sketch/hash_transform_data.hpp:21-104`` (draw order:
``N`` bucket indices uniform in ``[0, S-1]``, then ``N`` values),
``sketch/CWT_data.hpp`` (values ±1), ``sketch/MMT_data.hpp`` (Cauchy values),
``sketch/WZT_data.hpp:27-130`` (``N`` Exp(1) draws then ``N`` Rademacher signs:
value ``±(1/E)^(1/p)``, ``p`` in [1, 2]).
"""
from __future__ import annotations

import torch

from ..base import distributions as D
from ..base.exceptions import InvalidParametersError
from ..ops import hash_sketch as _hs
from .base import SketchTransform, register


class HashSketch(SketchTransform):
    supports_sparse_output = True  # sparse in -> sparse out by default (reference: output ctor = input's)
    linear_shards = True           # S A = sum over row blocks (streaming, distribution)
    value_dist = D.Rademacher()

    def _draw_values(self, ctx) -> torch.Tensor:
        return ctx.generate_random_samples_array(self._N, self.value_dist)

    def _build(self, ctx):
        self.row_idx = ctx.generate_random_samples_array(self._N, D.UniformInt(0, self._S - 1),
                                                         dtype=torch.int64)
        self.row_value = self._draw_values(ctx)
        self._hd = _hs.HashData(self.row_idx, self.row_value, self._S)

    # explicit operator (tests use it as the oracle, reference test_utils.hpp:14-35)
    def realize(self, dtype=torch.float64) -> torch.Tensor:
        P = torch.zeros(self._S, self._N, dtype=dtype)
        P[self.row_idx, torch.arange(self._N)] = self.row_value.to(dtype)
        return P

    def _apply_dense(self, A, dim, in_offset: int = 0, out_rows=None):
        return _hs.apply_dense(self._hd, A, dim, in_offset=in_offset)

    def _apply_sparse(self, A, dim, sparse_out):
        if sparse_out:
            return _hs.apply_csr_sparse_out(self._hd, A, dim)
        return _hs.apply_csr_dense_out(self._hd, A, dim)

    def apply_local_shard(self, A_local, dim, in_offset, out_rows=None):
        if A_local.layout == torch.sparse_csr:
            return _hs.apply_csr_dense_out(self._hd, A_local, dim, in_offset=in_offset)
        return _hs.apply_dense(self._hd, A_local, dim, in_offset=in_offset)


@register
class CWT(HashSketch):
    """Clarkson-Woodruff transform (CountSketch): values ±1."""

    sketch_type = "CWT"
    value_dist = D.Rademacher()


@register
class MMT(HashSketch):
    """Meng-Mahoney transform: Cauchy values (l1 subspace embedding)."""

    sketch_type = "MMT"
    value_dist = D.Cauchy()


@register
class WZT(HashSketch):
    """Woodruff-Zhang transform for l_p, p in [1, 2]: values ±(1/E)^(1/p)."""

    sketch_type = "WZT"

    def __init__(self, n, s, p=1.0, context=None):
        p = float(p)
        if p < 1.0 or p > 2.0:
            raise InvalidParametersError("WZT parameter p has to be in (1, 2)")
        self._p = p
        super().__init__(n, s, context)

    def _draw_values(self, ctx):
        e = ctx.generate_random_samples_array(self._N, D.Exponential())
        sign = ctx.generate_random_samples_array(self._N, D.Rademacher())
        return sign * torch.pow(1.0 / e, 1.0 / self._p)

    def _extra_params(self):
        return {"P": self._p}

    @classmethod
    def _params_from_dict(cls, d):
        return {"p": float(d.get("P", d.get("p", 1.0)))}


CountSketch = CWT
