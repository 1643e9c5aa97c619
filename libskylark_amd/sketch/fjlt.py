"""FJLT (fast JL / SRHT-style), RFUT and UST.

Reference: ``sketch/FJLT_data.hpp:19-94`` (RFUT data: ``N`` Rademacher for D,
then ``S`` uniform ints in [0, N) with replacement), apply
``sketch/FJLT_Elemental.hpp:144-171``: ``SA = sqrt(N/S) * P * F * D * A``;
``sketch/RFUT_data.hpp:20-51``; ``sketch/UST_data.hpp:75-100`` (with
replacement: ``S`` ints; without: inside-out Fisher-Yates with one
``uniform_int(0, i)`` draw per i, N draws), UST applies without scaling.

MI355X design: when the number of samples is small (``S <= 256``) the
sampled rows of ``F*D`` are realised explicitly (``S x N``) and applied as an
MFMA GEMM — one streaming pass over A; otherwise the rocFFT DCT pipeline
(D-scale, FFT, twiddle, gather) is used.
"""
from __future__ import annotations

import math

import torch

from ..base import distributions as D
from ..ops import fut as _fut
from ..ops import rng as _rng
from ..utils.devcache import device_copy
from .base import COLUMNWISE, SketchTransform, register

DIRECT_MAX_S = 256


class RFUT:
    """Random fast unitary transform ``F * D`` (not a registered sketch type;
    used by FJLT and Blendenpik).  ``fut`` in {"DCT", "DHT", "WHT"}."""

    def __init__(self, N: int, context, fut: str = "DCT"):
        self.N = N
        self.fut = fut
        self.D = context.generate_random_samples_array(N, D.Rademacher())

    def apply(self, A: torch.Tensor, dim: int = COLUMNWISE) -> torch.Tensor:
        if (self.fut == "DCT" and A.is_cuda and A.dtype in (torch.float32, torch.bfloat16) and A.dim() == 2
                and A.stride(1) == 1 and self.N >= 2):
            # native pipeline with every frequency kept: D-scale + reorder pass,
            # rocFFT R2C, twiddle/scale pass (3 HBM passes instead of ~7)
            if getattr(self, "_all", None) is None or self._all.device != A.device:
                self._all = torch.arange(self.N, dtype=torch.int64, device=A.device)
            return _fut.fjlt_sampled(A, dim, self.D, self._all, 1.0)
        d = device_copy(self.D, A.device, torch.float64 if A.dtype == torch.float64 else torch.float32)
        X = A * (d[:, None] if dim == COLUMNWISE else d[None, :])
        return _fut.FUTS[self.fut][0](X, dim)

    def apply_inverse(self, A: torch.Tensor, dim: int = COLUMNWISE) -> torch.Tensor:
        d = device_copy(self.D, A.device, torch.float64 if A.dtype == torch.float64 else torch.float32)
        X = _fut.FUTS[self.fut][1](A, dim)
        return X * (d[:, None] if dim == COLUMNWISE else d[None, :])


@register
class FJLT(SketchTransform):
    sketch_type = "FJLT"

    def _build(self, ctx):
        self.rfut = RFUT(self._N, ctx, "DCT")
        self.samples = ctx.generate_random_samples_array(self._S, D.UniformInt(0, self._N - 1),
                                                         dtype=torch.int64)
        self.scale = math.sqrt(self._N / self._S)
        self._W = {}

    def realize(self, dtype=torch.float64, device=None, transpose: bool = False) -> torch.Tensor:
        """Explicit ``S x N`` operator ``sqrt(N/S) P F D`` (``transpose``: its N x S transpose)."""
        return _fut.dct2_rows_matrix(self._N, self.samples, dtype=dtype, device=device, d=self.rfut.D,
                                     scale=self.scale, transpose=transpose)

    def _operator(self, device, dtype):
        key = (str(device), dtype)
        if key not in self._W:
            self._W[key] = self.realize(dtype=dtype, device=device)
        return self._W[key]

    def _apply_dense(self, A, dim, in_offset=0, out_rows=None):
        cdt = A.dtype if A.dtype in (torch.float32, torch.float64, torch.bfloat16, torch.float16) else torch.float32
        if self._S <= DIRECT_MAX_S:
            from ..ops import fused as _fused
            k = A.shape[dim]
            if _fused.fused_ok(A, dim, k, self._S):
                # explicit sqrt(N/S) P F D on the fused bf16x3 MFMA GEMM
                if getattr(self, "_wcache", None) is None:
                    self._wcache = _fused.WCache()
                Wf = self._wcache.get((str(A.device), in_offset, k), lambda: self.realize(
                    torch.float64, A.device)[:, in_offset:in_offset + k].float())
                return _fused.feature_gemm(A, Wf, dim)
            W = self._operator(A.device, cdt)
            k = A.shape[dim]
            Wl = W[:, in_offset:in_offset + k]
            if dim == COLUMNWISE:
                out = torch.matmul(Wl, A.to(cdt))
            else:
                out = torch.matmul(A.to(cdt), Wl.t())
            return out.float() if cdt in (torch.bfloat16, torch.float16) else out
        if in_offset != 0:
            raise ValueError("FFT-based FJLT needs the full sketched dimension on one device")
        out = _fut.fjlt_sampled(A, dim, self.rfut.D, self.samples, self.scale)
        return out.to(torch.float64) if A.dtype == torch.float64 else out

    def apply_local_shard(self, A_local, dim, in_offset, out_rows=None):
        if A_local.layout == torch.sparse_csr:
            A_local = A_local.to_dense()
        if in_offset == 0 and A_local.shape[dim] == self._N:
            return self._apply_dense(A_local, dim)
        return self._apply_dense(A_local, dim, in_offset=in_offset)


def _fisher_yates_prefix(ctx, N: int, S: int):
    """S distinct indices of [0, N): S steps of the backward Fisher-Yates
    shuffle in native code (``sl_ust_noreplace_host``, O(S) time and memory);
    reserves N counter slots like the reference (``sketch/UST_data.hpp:81-100``)."""
    import ctypes as C
    from ..ops import _lib
    seed, base = ctx.seed, ctx.counter
    ctx.counter += N
    out = torch.empty(S, dtype=torch.int64)
    _lib.call("sl_ust_noreplace_host", _lib.ptr(out), C.c_uint64(seed), C.c_uint64(base), N, S)
    return out


@register
class UST(SketchTransform):
    """Uniform sampling transform (row/column selection, unscaled)."""

    sketch_type = "UST"

    def __init__(self, n, s, replace=True, context=None):
        self._replace = bool(replace)
        super().__init__(n, s, context)

    def _build(self, ctx):
        if self._replace:
            self.samples = ctx.generate_random_samples_array(self._S, D.UniformInt(0, self._N - 1),
                                                             dtype=torch.int64)
        else:
            if self._S > self._N:
                from ..base.exceptions import InvalidParametersError
                raise InvalidParametersError("UST without replacement needs S <= N")
            self.samples = _fisher_yates_prefix(ctx, self._N, self._S)

    def realize(self, dtype=torch.float64):
        P = torch.zeros(self._S, self._N, dtype=dtype)
        P[torch.arange(self._S), self.samples] = 1
        return P

    def _apply_dense(self, A, dim, in_offset=0, out_rows=None):
        idx = device_copy(self.samples, A.device)
        return A.index_select(dim, idx)

    def _apply_sparse(self, A, dim, sparse_out):
        idx = self.samples.to(A.device)
        coo = A.to_sparse_coo().coalesce()
        out = coo.index_select(dim, idx).coalesce()
        return out.to_sparse_csr() if sparse_out else out.to_dense()

    supports_sparse_output = True

    def _extra_params(self):
        return {"replace": self._replace}

    @classmethod
    def _params_from_dict(cls, d):
        r = d.get("replace", True)
        if isinstance(r, str):
            r = r.lower() == "true"
        return {"replace": bool(r)}


@register
class NURST(SketchTransform):
    """Non-uniform random sampling transform: ``S`` indices drawn with
    replacement from the probability vector ``p`` over ``[0, N)``
    (reference pure-Python ``NURST``, ``python-skylark/skylark/sketch.py:906-933``).

    Draws: ``S`` uniform(0,1) slots of the context stream, mapped through the
    inverse CDF of ``p`` (so the indices are reproducible from the context,
    unlike the reference's scipy draw).  ``p`` is normalised; it is stored in
    the serialised form.
    """

    sketch_type = "NURST"
    supports_sparse_output = True

    def __init__(self, n, s, p=None, context=None):
        import numpy as np
        if p is None:
            raise ValueError("NURST needs a probability vector p")
        p = np.asarray(p.cpu().numpy() if isinstance(p, torch.Tensor) else p, dtype=np.float64).reshape(-1)
        if p.shape[0] != int(n):
            from ..base.exceptions import InvalidParametersError
            raise InvalidParametersError("size of probability array should be exactly n")
        if (p < 0).any() or p.sum() <= 0:
            from ..base.exceptions import InvalidParametersError
            raise InvalidParametersError("p must be a non-negative, non-zero vector")
        self._p = p / p.sum()
        super().__init__(n, s, context)

    def _build(self, ctx):
        import numpy as np
        u = ctx.generate_random_samples_array(self._S, D.Uniform(0.0, 1.0)).cpu().numpy()
        cdf = np.cumsum(self._p)
        cdf[-1] = 1.0
        idx = np.searchsorted(cdf, u, side="right")
        self.samples = torch.from_numpy(np.minimum(idx, self._N - 1).astype(np.int64))

    realize = UST.realize
    _apply_dense = UST._apply_dense
    _apply_sparse = UST._apply_sparse

    def _extra_params(self):
        return {"p": [float(x) for x in self._p]}

    @classmethod
    def _params_from_dict(cls, d):
        return {"p": d["p"]}


URST = UST
UniformSampler = UST
NonUniformSampler = NURST
FastJLT = FJLT
