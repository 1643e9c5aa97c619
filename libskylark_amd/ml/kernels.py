"""Positive-definite kernels: Gram matrices and random-feature maps.

Reference ``ml/kernels.hpp:12-1289`` (``kernel_t`` with ``gram`` /
``symmetric_gram`` / ``create_rft`` / ``create_qrft`` / ``to_ptree``, the six
kernels and ``kernel_container_t``) and ``python-skylark/skylark/ml/kernels.py``
(``kernel()`` factory, ``Kernel.gram(X, K, dirX, dirY, Y)``, ``rft(s, subtype)``).

MI355X layout: data points are ROWS of a row-major ``(n, d)`` tensor (the
Python API's default ``dirX="rows"``); ``"columns"`` inputs are transposed
views.  On the GPU:

* linear / polynomial / Gaussian Grams are ``X Y^T`` on hipBLASLt (fp32/fp64)
  followed by ONE in-place native epilogue pass (``sl_gram_map``: distance
  from cached squared row norms, clamp, exp / pow);
* Laplacian and exp-semigroup Grams are not GEMM-shaped: the native
  ``sl_pairwise_map`` kernel (64x64 LDS tiles, fused ``exp(-D/sigma)``)
  computes them in one pass without materialising the distance matrix;
* GPU ops require the native library (no silent fallback); CPU tensors use
  plain torch.

Distributed inputs (``DistMatrix`` with row layouts) produce the row block
``K[rows_local, :]`` against an all-gathered ``Y`` (``gram_dist``).
"""
from __future__ import annotations

import json
import math

import torch

from ..base.context import Context
from ..base.exceptions import InvalidParametersError, UnsupportedError
from ..ops import _lib as L
from ..parallel.distmatrix import DistMatrix
from .. import sketch as SK

VERSION = "0.1.0"

_PW_L1, _PW_SEMIGROUP = 0, 1
_GM_GAUSSIAN, _GM_POLY = 0, 1

L.register("sl_pairwise_map", [L.vp, L.vp, L.vp, L.i32, L.i64, L.i64, L.i64, L.i64, L.i64, L.i64,
                               L.i32, L.f64, L.vp])
L.register("sl_gram_map", [L.vp, L.i32, L.i64, L.i64, L.i64, L.vp, L.vp, L.i32, L.f64, L.f64, L.f64, L.vp])


def _points(X, direction: str) -> torch.Tensor:
    """Return a row-major (n_points, d) view of X (``direction`` as in the reference)."""
    if isinstance(X, DistMatrix):
        X = X.local
    if not isinstance(X, torch.Tensor):
        import numpy as np
        if hasattr(X, "toarray"):
            X = X.toarray()
        X = torch.from_numpy(np.asarray(X))
    if X.is_sparse or X.layout != torch.strided:
        X = X.to_dense()
    d = _dir(direction)
    return X if d == "rows" else X.t()


def _dir(direction) -> str:
    if direction in (0, "columns", "COLUMNS", "cols"):
        return "columns"
    if direction in (1, "rows", "ROWS"):
        return "rows"
    raise InvalidParametersError(f"direction must be rows/columns, got {direction!r}")


def _work_dtype(*ts):
    dt = torch.promote_types(ts[0].dtype, ts[-1].dtype)
    return dt if dt in (torch.float32, torch.float64) else torch.float32


def _native_ok(X: torch.Tensor) -> bool:
    if not X.is_cuda:
        return False
    L.require()
    return True


def _pairwise(X: torch.Tensor, Y: torch.Tensor, mode: int, scale: float) -> torch.Tensor:
    dt = _work_dtype(X, Y)
    X = X.to(dt).contiguous()
    Y = Y.to(dt).contiguous()
    m, n = X.shape[0], Y.shape[0]
    if _native_ok(X):
        K = torch.empty(m, n, dtype=dt, device=X.device)
        L.call("sl_pairwise_map", L.ptr(X), L.ptr(Y), L.ptr(K), L.dtype_code(dt), m, n, X.shape[1],
               X.stride(0), Y.stride(0), K.stride(0), mode, float(scale), L.stream_of(X))
        return K
    if mode == _PW_L1:
        D = torch.cdist(X, Y, p=1)
    else:
        D = torch.empty(m, n, dtype=dt)
        bs = max(1, (1 << 24) // max(1, X.shape[1] * n))
        for i in range(0, m, bs):
            D[i:i + bs] = torch.sqrt((X[i:i + bs, None, :] + Y[None, :, :]).abs()).sum(-1)
    return torch.exp(-scale * D) if scale > 0 else D


# Gram matrices at least this large (m * n entries) on the GPU take the fused
# path: one MFMA kernel computes X Y^T (bf16x3 split operands, ~1e-5 relative
# in the inner products) and applies the kernel map in its epilogue, instead
# of an f32 library GEMM plus a second pass over K (sl_gram_map)
FUSED_GRAM_MIN = 1 << 22


def _gemm_map_fused(X, Y, kind, a, c, q, symmetric):
    from ..ops import fused as F
    if not (X.is_cuda and X.dtype == torch.float32 and F.enabled()):
        return None
    m, d = X.shape
    n = Y.shape[0]
    if m * n < FUSED_GRAM_MIN or n * d > F.MAX_W_ELEMS or kind not in (_GM_GAUSSIAN, _GM_POLY):
        return None
    W = F.SplitW(Y)
    if kind == _GM_GAUSSIAN:
        xn = (X * X).sum(1)
        yn = xn if symmetric else (Y * Y).sum(1)
        return F.feature_gemm(X, W, 1, scales=torch.full((n,), 2.0 * a, device=X.device),
                              shifts=-a * yn, rowterm=-a * xn, epi=F.EPI_GAUSS)
    if kind == _GM_POLY:
        return F.feature_gemm(X, W, 1, scales=torch.full((n,), float(a), device=X.device),
                              shifts=torch.full((n,), float(c), device=X.device), p0=float(q), epi=F.EPI_POLY)
    return None


def _gemm_map(X: torch.Tensor, Y: torch.Tensor, kind: int, a: float, c: float = 0.0, q: float = 1.0,
              symmetric: bool = False) -> torch.Tensor:
    dt = _work_dtype(X, Y)
    if dt == torch.float32:
        Kf = _gemm_map_fused(X.to(dt).contiguous(), (X if symmetric else Y).to(dt).contiguous(), kind, a, c, q,
                             symmetric)
        if Kf is not None:
            return Kf
    X = X.to(dt)
    Y = X if symmetric else Y.to(dt)
    K = X @ Y.t()
    if kind < 0:
        return K
    xn = (X * X).sum(1)
    yn = xn if symmetric else (Y * Y).sum(1)
    if _native_ok(K):
        xn, yn = xn.contiguous(), yn.contiguous()
        L.call("sl_gram_map", L.ptr(K), L.dtype_code(dt), K.shape[0], K.shape[1], K.stride(0), L.ptr(xn),
               L.ptr(yn), kind, float(a), float(c), float(q), L.stream_of(K))
        return K
    if kind == _GM_GAUSSIAN:
        D = (xn[:, None] + yn[None, :] - 2.0 * K).clamp_min_(0)
        return torch.exp(-a * D)
    return (a * K + c) ** q


class Kernel:
    """Base kernel (reference ``kernel_t``)."""

    kernel_type = "abstract"

    def __init__(self, d: int):
        self._N = int(d)

    # ----------------------------------------------------------- interface
    def get_dim(self) -> int:
        return self._N

    @property
    def d(self) -> int:
        return self._N

    def _gram_rows(self, X: torch.Tensor, Y: torch.Tensor, symmetric: bool) -> torch.Tensor:
        raise NotImplementedError

    def gram(self, X, K=None, dirX="rows", dirY="rows", Y=None) -> torch.Tensor:
        """K[i, j] = k(x_i, y_j) (python-skylark ``Kernel.gram`` signature;
        ``Y=None`` means ``Y = X``).  If ``K`` is given it is filled in place."""
        sym = Y is None
        if sym:
            Y, dirY = X, dirX
        if isinstance(X, DistMatrix) or isinstance(Y, DistMatrix):
            out = gram_dist(self, X, Y, dirX, dirY)
        else:
            Xr, Yr = _points(X, dirX), _points(Y, dirY)
            self._check(Xr, Yr)
            out = self._gram_rows(Xr, Yr, sym)
        if K is not None:
            K.copy_(out)
            return K
        return out

    def symmetric_gram(self, X, direction="rows", uplo: str = "L") -> torch.Tensor:
        """Full symmetric Gram k(X, X) (the reference fills one triangle; both are filled here)."""
        Xr = _points(X, direction)
        self._check(Xr, Xr)
        return self._gram_rows(Xr, Xr, True)

    def _check(self, X, Y):
        if X.shape[1] != self._N or Y.shape[1] != self._N:
            raise InvalidParametersError(f"{self.kernel_type} kernel of dim {self._N}: got points of dim "
                                         f"{X.shape[1]} and {Y.shape[1]}")

    def create_rft(self, S: int, fast: bool = False, context: Context | None = None):
        """Random feature map of size ``S`` whose inner products approximate k
        (reference ``create_rft(S, regular|fast_feature_transform_tag, context)``)."""
        raise UnsupportedError(f"random features not available for {self.kernel_type} kernel")

    def create_qrft(self, S: int, sequence=None, skip: int = 0, context: Context | None = None):
        raise UnsupportedError(f"quasi-random features not available for {self.kernel_type} kernel")

    def rft(self, s, subtype=None, context: Context | None = None, **kw):
        """python-skylark spelling: ``subtype`` None/'regular' or 'fast'
        (Laplacian/ExpSemiGroup also accept 'quasi')."""
        if subtype == "quasi":
            return self.create_qrft(s, context=context, **kw)
        return self.create_rft(s, fast=(subtype == "fast"), context=context)

    def qrft_sequence_dim(self) -> int:
        return self._N

    # ----------------------------------------------------- serialization
    def _params(self) -> dict:
        return {}

    def to_dict(self) -> dict:
        d = {"skylark_object_type": "kernel", "skylark_version": VERSION, "kernel_type": self.kernel_type}
        d.update(self._params())
        d["N"] = self._N
        return d

    to_ptree = to_dict

    def to_json(self) -> str:
        return json.dumps(self.to_dict())

    def __repr__(self):
        p = ", ".join(f"{k}={v}" for k, v in self._params().items())
        return f"{type(self).__name__}(d={self._N}{', ' + p if p else ''})"

    def __eq__(self, other):
        return isinstance(other, Kernel) and self.to_dict() == other.to_dict()

    __hash__ = object.__hash__


class Linear(Kernel):
    """k(x, y) = x^T y (reference ``linear_t`` ``:156-316``)."""
    kernel_type = "linear"

    def _gram_rows(self, X, Y, symmetric):
        return _gemm_map(X, Y, -1, 0.0, symmetric=symmetric)

    def create_rft(self, S, fast=False, context=None):
        raise UnsupportedError("linear kernel has no random feature map (use the identity)")


class Gaussian(Kernel):
    """k(x, y) = exp(-|x - y|^2 / (2 sigma^2)) (reference ``gaussian_t`` ``:320-493``)."""
    kernel_type = "gaussian"

    def __init__(self, d, sigma):
        super().__init__(d)
        self._sigma = float(sigma)

    @property
    def sigma(self):
        return self._sigma

    def _params(self):
        return {"sigma": self._sigma}

    def _gram_rows(self, X, Y, symmetric):
        return _gemm_map(X, Y, _GM_GAUSSIAN, 1.0 / (2.0 * self._sigma ** 2), symmetric=symmetric)

    def create_rft(self, S, fast=False, context=None):
        cls = SK.FastGaussianRFT if fast else SK.GaussianRFT
        return cls(self._N, S, self._sigma, context=context)

    def create_qrft(self, S, sequence=None, skip=0, context=None):
        return SK.GaussianQRFT(self._N, S, self._sigma, skip=skip, sequence=sequence, context=context)


class Polynomial(Kernel):
    """k(x, y) = (gamma x^T y + c)^q (reference ``polynomial_t`` ``:495-668``).
    Random features: PPT (TensorSketch), used for both regular and fast."""
    kernel_type = "polynomial"

    def __init__(self, d, q=3, c=0.0, gamma=1.0):
        super().__init__(d)
        self._q, self._c, self._gamma = int(q), float(c), float(gamma)

    def _params(self):
        return {"q": self._q, "c": self._c, "gamma": self._gamma}

    def _gram_rows(self, X, Y, symmetric):
        return _gemm_map(X, Y, _GM_POLY, self._gamma, self._c, self._q, symmetric=symmetric)

    def create_rft(self, S, fast=False, context=None):
        return SK.PPT(self._N, S, self._q, self._c, self._gamma, context=context)


class Laplacian(Kernel):
    """k(x, y) = exp(-|x - y|_1 / sigma) (reference ``laplacian_t`` ``:671-840``)."""
    kernel_type = "laplacian"

    def __init__(self, d, sigma):
        super().__init__(d)
        self._sigma = float(sigma)

    def _params(self):
        return {"sigma": self._sigma}

    def _gram_rows(self, X, Y, symmetric):
        return _pairwise(X, Y, _PW_L1, 1.0 / self._sigma)

    def create_rft(self, S, fast=False, context=None):
        if fast:
            raise UnsupportedError("fast feature transform has not been implemented for the laplacian kernel")
        return SK.LaplacianRFT(self._N, S, self._sigma, context=context)

    def create_qrft(self, S, sequence=None, skip=0, context=None):
        return SK.LaplacianQRFT(self._N, S, self._sigma, skip=skip, sequence=sequence, context=context)


class ExpSemigroup(Kernel):
    """k(x, y) = exp(-beta sum_i sqrt(x_i + y_i)) on non-negative data
    (reference ``expsemigroup_t`` ``:843-1010``; symmetric_gram is not
    special-cased there — here it is simply the full Gram)."""
    kernel_type = "expsemigroup"

    def __init__(self, d, beta):
        super().__init__(d)
        self._beta = float(beta)

    def _params(self):
        return {"beta": self._beta}

    def _gram_rows(self, X, Y, symmetric):
        return _pairwise(X, Y, _PW_SEMIGROUP, self._beta)

    def create_rft(self, S, fast=False, context=None):
        if fast:
            raise UnsupportedError("fast feature transform has not been implemented for expsemigroup kernel")
        return SK.ExpSemigroupRLT(self._N, S, self._beta, context=context)

    def create_qrft(self, S, sequence=None, skip=0, context=None):
        return SK.ExpSemigroupQRLT(self._N, S, self._beta, skip=skip, sequence=sequence, context=context)


class Matern(Kernel):
    """Matérn kernel, features only (reference ``matern_t`` ``:1013-1160``:
    gram/symmetric_gram throw).  Here the Gram is implemented too, for the
    half-integer orders with closed forms (nu = 0.5, 1.5, 2.5); other orders
    raise as in the reference."""
    kernel_type = "matern"

    def __init__(self, d, nu, l):  # noqa: E741
        super().__init__(d)
        self._nu, self._l = float(nu), float(l)

    def _params(self):
        return {"nu": self._nu, "l": self._l}

    def _gram_rows(self, X, Y, symmetric):
        D2 = _gemm_map(X, Y, -1, 0.0, symmetric=symmetric)
        xn = (X.to(D2.dtype) ** 2).sum(1)
        yn = xn if symmetric else (Y.to(D2.dtype) ** 2).sum(1)
        r = (xn[:, None] + yn[None, :] - 2 * D2).clamp_min_(0).sqrt_() / self._l
        if self._nu == 0.5:
            return torch.exp(-r)
        if self._nu == 1.5:
            a = math.sqrt(3) * r
            return (1 + a) * torch.exp(-a)
        if self._nu == 2.5:
            a = math.sqrt(5) * r
            return (1 + a + a * a / 3) * torch.exp(-a)
        raise UnsupportedError("gram has not yet been implemented for matern kernel with this nu")

    def create_rft(self, S, fast=False, context=None):
        cls = SK.FastMaternRFT if fast else SK.MaternRFT
        return cls(self._N, S, self._nu, self._l, context=context)


ExpSemiGroup = ExpSemigroup

_KERNELS = {c.kernel_type: c for c in (Linear, Gaussian, Polynomial, Laplacian, ExpSemigroup, Matern)}


def kernel(kerneltype: str, *args, **kw) -> Kernel:
    """Kernel factory (python-skylark ``kernel(kerneltype, *args)``): first arg is d."""
    if not isinstance(kerneltype, str):
        raise ValueError("kerneltype must be a string")
    cls = _KERNELS.get(kerneltype.lower())
    if cls is None:
        raise ValueError("kerneltype not recognized")
    return cls(*args, **kw)


def kernel_from_dict(d) -> Kernel:
    """Rebuild from the JSON/ptree form (reference ``kernel_container_t(ptree)``);
    accepts boost's all-strings encoding."""
    if isinstance(d, str):
        d = json.loads(d)
    t = d["kernel_type"]
    N = int(d["N"])
    if t == "linear":
        return Linear(N)
    if t in ("gaussian", "laplacian"):
        return _KERNELS[t](N, float(d["sigma"]))
    if t == "polynomial":
        return Polynomial(N, int(d["q"]), float(d["c"]), float(d["gamma"]))
    if t == "expsemigroup":
        return ExpSemigroup(N, float(d["beta"]))
    if t == "matern":
        return Matern(N, float(d["nu"]), float(d["l"]))
    raise InvalidParametersError(f"unknown kernel_type {t}")


KernelContainer = kernel_from_dict


def gram_dist(k: Kernel, X, Y, dirX="rows", dirY="rows") -> torch.Tensor | DistMatrix:
    """Gram for row-distributed data.  ``X`` a [VC,*]/[VR,*] DistMatrix of points:
    each rank computes ``K[rows_local, :]`` against the all-gathered ``Y``
    (one all-gather of n x d, then a purely local GEMM/pairwise kernel); the
    result is a [VC,*] DistMatrix of shape (m, n)."""
    if _dir(dirX) != "rows" or (isinstance(Y, DistMatrix) and _dir(dirY) != "rows"):
        raise UnsupportedError("distributed Gram expects points as rows ([VC,*] layouts)")
    if isinstance(X, DistMatrix):
        Xd = X if X.layout in ("VC_STAR", "VR_STAR") else X.redistribute("VC_STAR")
        Yl = Y.to_global() if isinstance(Y, DistMatrix) else _points(Y, dirY)
        Kl = k._gram_rows(Xd.local, Yl.to(Xd.local.device), False)
        return DistMatrix(Kl, (Xd.shape[0], Yl.shape[0]), Xd.layout, Xd.comm)
    Yd = Y if Y.layout in ("VC_STAR", "VR_STAR") else Y.redistribute("VC_STAR")
    Xl = _points(X, dirX)
    Kt = k._gram_rows(Yd.local, Xl.to(Yd.local.device), False)
    return DistMatrix(Kt.t().contiguous(), (Xl.shape[0], Yd.shape[0]), "STAR_VC", Yd.comm)


def Gram(dirX, dirY, k: Kernel, X, Y):
    """Reference-order free function ``Gram(dirX, dirY, k, X, Y, K)``."""
    return k.gram(X, dirX=dirX, dirY=dirY, Y=Y)


def SymmetricGram(uplo, direction, k: Kernel, X):
    return k.symmetric_gram(X, direction, uplo)
