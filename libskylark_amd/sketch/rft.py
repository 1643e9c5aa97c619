"""Random-feature maps: RFT / QRFT (random Fourier), RLT / QRLT (random Laplace).

Reference:
  * ``sketch/RFT_data.hpp:25-354``: W = dense transform with scale ``inscale``
    (Gaussian: N(0,1)/sigma; Laplacian: Cauchy/sigma; Matérn: N(0,1)/l with
    per-feature scales ``sqrt(2 nu / chi2_{2nu})``), ``S`` shifts U(0, 2pi),
    outscale ``sqrt(2/S)``; apply ``Z = outscale*cos(scales*(W A) + shifts)``
    (``sketch/RFT_Elemental.hpp:83-160``).  Draw order: W (N*S slots, lazy),
    shifts (S), Matérn chi-squared (S).
  * ``sketch/QRFT_data.hpp``: W entries are distribution quantiles of a leaped
    Halton sequence of dimension N+1; shift_i = 2pi * coordinate(skip+i, N).
    Row i of W is QMC point ``skip + i`` (coordinate j = input dim j).
  * ``sketch/RLT_data.hpp``: ``Z = sqrt(1/S) * exp(-(W A))`` with W Lévy,
    scale ``beta^2/2``; QRLT with the Lévy quantile ``scale/(2 erfcinv(p)^2)``.

MI355X: W A is the RNG-panel MFMA GEMM of ``ops.dense_sketch``; the
cos/exp epilogue is one fused element-wise HIP pass (``sl_feature_epilogue``).
"""
from __future__ import annotations

import ctypes as C
import math

import torch

from ..base import distributions as D
from ..base import quasirand as Q
from ..ops import _lib
from ..ops import dense_sketch as _ds
from ..ops import fused as _fused
from .base import COLUMNWISE, SketchTransform, register

_lib.register("sl_feature_epilogue", [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_void_p,
                                      C.c_void_p, C.c_double, C.c_int, C.c_int, C.c_void_p])

EPI_COS, EPI_EXP = 0, 1


def feature_epilogue(X: torch.Tensor, scales, shifts, outscale: float, feature_dim: int, mode: int):
    """In-place ``X = outscale*cos(scales*X + shifts)`` (mode 0) or ``outscale*exp(-X)``."""
    if X.is_cuda:
        if X.stride(1) != 1:
            raise ValueError("feature_epilogue expects row-major X")
        sc = scales.to(X.device, torch.float64).contiguous() if scales is not None else None
        sh = shifts.to(X.device, torch.float64).contiguous() if shifts is not None else None
        _lib.call("sl_feature_epilogue", _lib.ptr(X), _lib.dtype_code(X.dtype), X.shape[0], X.shape[1],
                  X.stride(0), _lib.ptr(sc) if sc is not None else None,
                  _lib.ptr(sh) if sh is not None else None, float(outscale), int(feature_dim), int(mode),
                  C.c_void_p(_lib.stream_of(X)))
        return X
    shape = (-1, 1) if feature_dim == 0 else (1, -1)
    if mode == EPI_COS:
        z = X if scales is None else X * scales.to(X.dtype).view(shape)
        X.copy_(outscale * torch.cos(z + shifts.to(X.dtype).view(shape)))
    else:
        X.copy_(outscale * torch.exp(-X))
    return X


class _FeatureMap(SketchTransform):
    mode = EPI_COS

    def _features_pre(self, A, dim, in_offset=0, out_rows=None):
        raise NotImplementedError

    def _post(self, X, dim, out_rows=None):
        i0, i1 = out_rows if out_rows is not None else (0, self._S)
        sc = self.scales[i0:i1] if getattr(self, "scales", None) is not None else None
        sh = self.shifts[i0:i1] if getattr(self, "shifts", None) is not None else None
        if not X.is_contiguous():
            X = X.contiguous()
        return feature_epilogue(X, sc, sh, self.outscale, 0 if dim == COLUMNWISE else 1, self.mode)

    def _apply_dense(self, A, dim, in_offset=0, out_rows=None):
        k = A.shape[dim]
        i0, i1 = out_rows if out_rows is not None else (0, self._S)
        dense_ok = hasattr(self, "realize_W") and self._N <= getattr(self, "DENSE_MAX_N", self._N)
        if dense_ok and in_offset == 0 and k == self._N and _fused.fused_ok(A, dim, k, i1 - i0):
            # GEMM + cos/exp epilogue in one MFMA launch (ops/fused.py)
            if getattr(self, "_wcache", None) is None:
                self._wcache = _fused.WCache()
            W = self._wcache.get((str(A.device), i0, i1),
                                 lambda: self.realize_W(torch.float64, A.device)[i0:i1].float())
            sc = self.scales[i0:i1] if getattr(self, "scales", None) is not None else None
            sh = self.shifts[i0:i1] if getattr(self, "shifts", None) is not None else None
            epi = _fused.EPI_COS if self.mode == EPI_COS else _fused.EPI_EXPNEG
            return _fused.feature_gemm(A, W, dim, scales=sc, shifts=sh, outscale=self.outscale, epi=epi)
        return self._post(self._features_pre(A, dim, in_offset, out_rows), dim, out_rows)

    def _apply_sparse(self, A, dim, sparse_out):
        return self._apply_dense(A.to_dense(), dim)

    # distributed: a feature map is nonlinear, so the linear part is summed
    # across shards first (linear_local_shard) and the epilogue applied after.
    def linear_local_shard(self, A_local, dim, in_offset, out_rows=None):
        if A_local.layout == torch.sparse_csr:
            A_local = A_local.to_dense()
        return self._features_pre(A_local, dim, in_offset, out_rows)

    def finish_features(self, X, dim, out_rows=None):
        return self._post(X, dim, out_rows)


class _RFT(_FeatureMap):
    """Random Fourier features over a lazily realised dense W."""

    dist = D.Normal()

    def _inscale(self):
        raise NotImplementedError

    def _build(self, ctx):
        self.inscale = self._inscale()
        self.outscale = math.sqrt(2.0 / self._S)
        self.W = ctx.allocate_random_samples_array(self._N * self._S, self.dist)
        self.shifts = ctx.generate_random_samples_array(self._S, D.Uniform(0.0, 2 * math.pi))
        self.scales = None

    def realize_W(self, dtype=torch.float64, device=None):
        return _ds.realize_panel(self.dist, self.W.seed, self.W.base, self._S, (0, self._S),
                                 (0, self._N), scale=self.inscale, dtype=dtype, device=device,
                                 precise=dtype == torch.float64)

    def _features_pre(self, A, dim, in_offset=0, out_rows=None):
        return _ds.apply_dense(A, dim, dist=self.dist, seed=self.W.seed, base=self.W.base, S=self._S,
                               N=self._N, scale=self.inscale, in_offset=in_offset, out_rows=out_rows)


@register
class GaussianRFT(_RFT):
    """Random Fourier features of the Gaussian kernel exp(-|x-y|^2 / (2 sigma^2))."""

    sketch_type = "GaussianRFT"
    dist = D.Normal()

    def __init__(self, n, s, sigma=1.0, context=None):
        self._sigma = float(sigma)
        super().__init__(n, s, context)

    def _inscale(self):
        return 1.0 / self._sigma

    def _extra_params(self):
        return {"sigma": self._sigma}

    @classmethod
    def _params_from_dict(cls, d):
        return {"sigma": float(d["sigma"])}


@register
class LaplacianRFT(GaussianRFT):
    """Random Fourier features of the Laplacian kernel exp(-|x-y|_1 / sigma)."""

    sketch_type = "LaplacianRFT"
    dist = D.Cauchy()


@register
class MaternRFT(_RFT):
    """Random Fourier features of the Matérn kernel (multivariate-t sampling)."""

    sketch_type = "MaternRFT"
    dist = D.Normal()

    def __init__(self, n, s, nu=1.5, l=1.0, context=None):  # noqa: E741
        self._nu, self._l = float(nu), float(l)
        super().__init__(n, s, context)

    def _inscale(self):
        return 1.0 / self._l

    def _build(self, ctx):
        super()._build(ctx)
        chi = ctx.generate_random_samples_array(self._S, D.ChiSquared(2 * self._nu))
        self.scales = torch.sqrt(2.0 * self._nu / chi)

    def _extra_params(self):
        return {"nu": self._nu, "l": self._l}

    @classmethod
    def _params_from_dict(cls, d):
        return {"nu": float(d["nu"]), "l": float(d["l"])}


# ------------------------------------------------------------------- QMC
def _normal_quantile(u):
    return math.sqrt(2.0) * torch.erfinv(2 * u - 1)


def _cauchy_quantile(u):
    return torch.tan(math.pi * (u - 0.5))


def _levy_quantile(u, scale=1.0):
    v = torch.erfinv(1 - u)  # erfc^{-1}(u)
    return scale / (2 * v * v)


class _QMCMap(_FeatureMap):
    quantile = staticmethod(_normal_quantile)
    seq_extra = 1  # QRFT uses dimension N+1 (last coordinate -> shifts)

    def __init__(self, n, s, sigma=1.0, skip=0, sequence=None, context=None):
        self._sigma = float(sigma)
        self._skip = int(skip)
        self._sequence = sequence or Q.LeapedHaltonSequence(n + self.seq_extra)
        super().__init__(n, s, context)

    def _build(self, ctx):
        # QMC features draw nothing from the random stream.
        self._setup()
        self._Wcache = {}

    def _points(self):
        return self._sequence.block(self._skip, self._S, self._N + self.seq_extra)

    def realize_W(self, dtype=torch.float64, device=None):
        key = (str(device), dtype)
        if key not in self._Wcache:
            P = self._points()[:, :self._N].clamp(1e-16, 1 - 1e-16)
            W = self.inscale * self.quantile(P)
            self._Wcache[key] = W.to(device=device, dtype=dtype)
        return self._Wcache[key]

    def _features_pre(self, A, dim, in_offset=0, out_rows=None):
        cdt = A.dtype if A.dtype in (torch.float32, torch.float64) else torch.float32
        W = self.realize_W(cdt, A.device)
        i0, i1 = out_rows if out_rows is not None else (0, self._S)
        k = A.shape[dim]
        Wl = W[i0:i1, in_offset:in_offset + k]
        return Wl @ A.to(cdt) if dim == COLUMNWISE else A.to(cdt) @ Wl.t()

    def _extra_params(self):
        return {"sigma": self._sigma, "skip": self._skip, "sequence": self._sequence.to_dict()}

    @classmethod
    def _params_from_dict(cls, d):
        seq = Q.from_dict(d["sequence"]) if "sequence" in d else None
        return {"sigma": float(d.get("sigma", 1.0)), "skip": int(d.get("skip", 0)), "sequence": seq}


@register
class GaussianQRFT(_QMCMap):
    sketch_type = "GaussianQRFT"
    quantile = staticmethod(_normal_quantile)

    def _setup(self):
        self.inscale = 1.0 / self._sigma
        self.outscale = math.sqrt(2.0 / self._S)
        self.scales = None
        self.shifts = 2 * math.pi * self._points()[:, self._N].clone()


@register
class LaplacianQRFT(GaussianQRFT):
    sketch_type = "LaplacianQRFT"
    quantile = staticmethod(_cauchy_quantile)


@register
class ExpSemigroupRLT(_RFT):
    """Random Laplace features of the exponential-semigroup kernel
    exp(-beta * sum_i sqrt(x_i + y_i))."""

    sketch_type = "ExpSemigroupRLT"
    dist = D.Levy()
    mode = EPI_EXP

    def __init__(self, n, s, beta=1.0, context=None):
        self._beta = float(beta)
        super().__init__(n, s, context)

    def _inscale(self):
        return self._beta * self._beta / 2

    def _build(self, ctx):
        self.inscale = self._inscale()
        self.outscale = math.sqrt(1.0 / self._S)
        self.W = ctx.allocate_random_samples_array(self._N * self._S, self.dist)
        self.shifts = None
        self.scales = None

    def _extra_params(self):
        return {"beta": self._beta}

    @classmethod
    def _params_from_dict(cls, d):
        return {"beta": float(d["beta"])}


@register
class ExpSemigroupQRLT(_QMCMap):
    sketch_type = "ExpSemigroupQRLT"
    quantile = staticmethod(_levy_quantile)
    mode = EPI_EXP
    seq_extra = 0

    def __init__(self, n, s, beta=1.0, skip=0, sequence=None, context=None):
        self._beta = float(beta)
        super().__init__(n, s, sigma=1.0, skip=skip, sequence=sequence, context=context)

    def _setup(self):
        self.inscale = self._beta * self._beta / 2
        self.outscale = math.sqrt(1.0 / self._S)
        self.scales = None
        self.shifts = None

    def _extra_params(self):
        return {"beta": self._beta, "skip": self._skip, "sequence": self._sequence.to_dict()}

    @classmethod
    def _params_from_dict(cls, d):
        seq = Q.from_dict(d["sequence"]) if "sequence" in d else None
        return {"beta": float(d["beta"]), "skip": int(d.get("skip", 0)), "sequence": seq}
