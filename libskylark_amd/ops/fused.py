"""Fused dense-sketch / random-feature GEMM (``_native/src/feature_gemm.hip``).

``Z = outscale * epi(scale_f * (A W^T)[r, f] + shift_f)`` in one launch on
bf16 MFMA: f32 inputs are split once into bf16 hi + lo planes (one streaming
pass, ``sl_split_bf16``) and the realised sketching matrix W is held as a
bf16 hi + lo pair, so the 3-term product is f32-class accurate
(|err| ~ 2^-16 of sum |a w|) at 3/16 of the bf16 MFMA cost.

Used by the dense transforms (JLT / CT / SJLT, ``epi = none``) and the
feature maps (RFT / QRFT ``cos``, RLT / QRLT ``exp(-x)``) whenever the
sketched dimension is small enough for W (``S x N``) to be realised once and
cached on the device (``MAX_W_ELEMS``); tall sketched dimensions stream W
panels through ``ops.dense_sketch`` instead.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _lib

EPI_NONE, EPI_COS, EPI_EXPNEG, EPI_GAUSS, EPI_POLY = 0, 1, 2, 3, 4
BN, BK = 128, 32
MAX_W_ELEMS = 1 << 26          # W (S x N) realised whole up to 64 M entries (256 MB as hi+lo)

_lib.register("sl_feature_gemm", [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64,
                                  C.c_void_p, C.c_void_p, C.c_int64, C.c_int64,
                                  C.c_void_p, C.c_void_p, C.c_float, C.c_int,
                                  C.c_void_p, C.c_int, C.c_int64, C.c_int, C.c_void_p])
_lib.register("sl_feature_gemm2", [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64,
                                   C.c_void_p, C.c_void_p, C.c_int64, C.c_int64,
                                   C.c_void_p, C.c_void_p, C.c_float, C.c_int,
                                   C.c_void_p, C.c_int, C.c_int64, C.c_int, C.c_void_p, C.c_float, C.c_void_p])
_lib.register("sl_split_bf16", [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                C.c_void_p])
_lib.register("sl_split_bf16_2", [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                  C.c_int64, C.c_void_p])


def enabled() -> bool:
    return os.environ.get("SKH_FUSED_SKETCH", "1") != "0"


def fused_ok(A: torch.Tensor, dim: int, k: int, nf: int) -> bool:
    """Can (and should) ``A`` (dense, on a GPU) take the fused kernel?"""
    if not (enabled() and isinstance(A, torch.Tensor) and A.is_cuda and A.dim() == 2
            and A.layout == torch.strided and A.dtype in (torch.float32, torch.bfloat16)):
        return False
    if k <= 0 or nf <= 0 or nf * k > MAX_W_ELEMS or not _lib.available():
        return False
    if dim == 1:
        return True
    # columnwise needs A^T row-major: free if A is a transposed view, else a copy
    # that only pays off when the product is wide enough to be compute bound
    return A.t().is_contiguous() or nf >= 256


class SplitW:
    """A realised S x N block of W as zero-padded bf16 hi/lo planes."""

    __slots__ = ("hi", "lo", "nf", "k", "ldw", "cat")

    def __init__(self, W: torch.Tensor):
        nf, k = W.shape
        npad = -(-nf // BN) * BN
        ldw = -(-k // BK) * BK
        Wf = torch.zeros(npad, ldw, dtype=torch.float32, device=W.device)
        Wf[:nf, :k] = W
        self.hi = Wf.to(torch.bfloat16)
        self.lo = (Wf - self.hi.float()).to(torch.bfloat16)
        self.nf, self.k, self.ldw = nf, k, ldw
        self.cat = {}

    def concat(self, terms):
        """``[W_t1 | W_t2 | ...]`` (nf x n kp, kp = k rounded up to 64): the
        B operand of a multi-term product as ONE NT GEMM over the
        concatenated K (``terms``: "h" / "l" per term)."""
        key = tuple(terms)
        B = self.cat.get(key)
        if B is None:
            kp = -(-self.k // 64) * 64
            B = torch.zeros(self.nf, len(terms) * kp, dtype=torch.bfloat16, device=self.hi.device)
            for i, t in enumerate(terms):
                B[:, i * kp:i * kp + self.k] = (self.hi if t == "h" else self.lo)[:self.nf, :self.k]
            self.cat[key] = B
        return B


def split_planes(X: torch.Tensor):
    """Row-major bf16 operand planes for the kernel: ``(hi, lo, ld)`` with
    ``ld`` a multiple of 32 and zero padding.  f32 input -> hi + lo (one
    ``sl_split_bf16`` streaming pass; x = hi + lo to ~2^-17); bf16 input ->
    the data itself (lo = None), copied only when its rows are not padded."""
    m, k = X.shape
    ld = -(-k // BK) * BK
    dev = X.device
    if X.dtype == torch.bfloat16:
        if X.stride(1) == 1 and X.stride(0) == ld and X.data_ptr() % 16 == 0 and ld == k:
            return X, None, ld
        buf = torch.zeros(m, ld, dtype=torch.bfloat16, device=dev)
        buf[:, :k] = X
        return buf, None, ld
    if X.stride(1) != 1:
        X = X.contiguous()
    hi = torch.empty(m, ld, dtype=torch.bfloat16, device=dev)
    lo = torch.empty(m, ld, dtype=torch.bfloat16, device=dev)
    _lib.call("sl_split_bf16", _lib.ptr(X), m, k, X.stride(0), _lib.ptr(hi), _lib.ptr(lo), ld,
              C.c_void_p(_lib.stream_of(X)))
    return hi, lo, ld


def feature_gemm(A: torch.Tensor, W: SplitW, dim: int, *, scales=None, shifts=None,
                 outscale: float = 1.0, epi: int = EPI_NONE, out_dtype=torch.float32,
                 use_lo: bool = True, rowterm=None, p0: float = 0.0) -> torch.Tensor:
    """Columnwise (dim 0: A is K x m -> Z is nf x m) or rowwise (dim 1: A is
    m x K -> Z is m x nf) fused product with W^T and the epilogue."""
    X = A if dim == 1 else A.t()
    m, k = X.shape
    if k != W.k:
        raise ValueError(f"feature_gemm: inner dimension {k} != {W.k}")
    if dim == 1 and epi in (EPI_NONE, EPI_COS) and rowterm is None and _gemm_nt_ok(X):
        return _feature_gemm_nt(X, W, scales, shifts, outscale, epi, out_dtype, use_lo)
    hi, lo, ld = split_planes(X)
    dev = A.device
    if dim == 1:
        out = torch.empty(m, W.nf, dtype=out_dtype, device=dev)
        ldo, out_t = W.nf, 0
    else:
        out = torch.empty(W.nf, m, dtype=out_dtype, device=dev)
        ldo, out_t = m, 1
    sc = scales.to(device=dev, dtype=torch.float32).contiguous() if scales is not None else None
    sh = shifts.to(device=dev, dtype=torch.float32).contiguous() if shifts is not None else None
    if W.ldw != ld:
        raise ValueError("feature_gemm: W and A planes must share the padded inner dimension")
    rt = rowterm.to(device=dev, dtype=torch.float32).contiguous() if rowterm is not None else None
    _lib.call("sl_feature_gemm2", _lib.ptr(hi), _lib.ptr(lo) if lo is not None else None, m, k, ld,
              _lib.ptr(W.hi), _lib.ptr(W.lo) if use_lo else None, W.nf, W.ldw,
              _lib.ptr(sc) if sc is not None else None, _lib.ptr(sh) if sh is not None else None,
              float(outscale), int(epi), _lib.ptr(out), _lib.dtype_code(out_dtype), ldo, out_t,
              _lib.ptr(rt) if rt is not None else None, float(p0), C.c_void_p(_lib.stream_of(out)))
    return out


# rowwise linear / cosine maps on the 256 x 256 NT GEMM (gemm_nt.hip) with
# the hi / lo terms concatenated along K (one launch, no per-term passes)
def _gemm_nt_ok(X):
    return X.stride(1) == 1 and X.dtype in (torch.float32, torch.bfloat16)


def _feature_gemm_nt(X, W, scales, shifts, outscale, epi, out_dtype, use_lo):
    """``[X_h | X_l | X_h] [W_h | W_h | W_l]^T`` (f32 X; bf16 X: ``[X | X]
    [W_h | W_l]^T``, or one term without W's lo plane) with the epilogue."""
    from . import gemm as _g
    m, k = X.shape
    kp = -(-k // 64) * 64
    if X.dtype == torch.float32:
        ta, tb = ("h", "l", "h"), ("h", "h", "l")
        if not use_lo:
            ta, tb = ("h", "l"), ("h", "h")
    else:
        ta, tb = (("h", "h"), ("h", "l")) if use_lo else (("h",), ("h",))
    Ap = torch.empty(m, len(ta) * kp, dtype=torch.bfloat16, device=X.device)
    if X.dtype == torch.float32:
        Xc = X if X.stride(0) % 4 == 0 and X.data_ptr() % 16 == 0 else X.contiguous()
        _lib.call("sl_split_bf16_2", _lib.ptr(Xc), m, k, Xc.stride(0), _lib.ptr(Ap), _lib.ptr(Ap[:, kp:]), kp,
                  Ap.stride(0), C.c_void_p(_lib.stream_of(X)))
        if len(ta) == 3:
            Ap[:, 2 * kp:].copy_(Ap[:, :kp])
    else:
        Ap[:, :k] = X
        if kp > k:
            Ap[:, k:kp].zero_()
        for i in range(1, len(ta)):
            Ap[:, i * kp:(i + 1) * kp].copy_(Ap[:, :kp])
    B = W.concat(tb)
    out = torch.empty(m, W.nf, dtype=out_dtype, device=X.device)
    if epi == EPI_COS:
        sc = scales if scales is not None else torch.ones(W.nf, device=X.device)
        sh = shifts if shifts is not None else torch.zeros(W.nf, device=X.device)
        return _g.gemm_nt(Ap, B, out=out, alpha=outscale, cos_scales=sc.to(X.device), cos_shifts=sh.to(X.device))
    return _g.gemm_nt(Ap, B, out=out, alpha=outscale)


class WCache:
    """Per-sketch LRU cache of realised, split W blocks keyed by device and
    window.  Bounded (``MAX_ENTRIES`` blocks, ``MAX_BYTES`` of planes): a
    streamed or sharded apply touches one window per panel, and keeping them
    all would grow to the whole realised S."""

    MAX_ENTRIES = 8
    MAX_BYTES = 1 << 30

    def __init__(self):
        self._d = {}

    @staticmethod
    def _bytes(w):
        return w.hi.numel() * w.hi.element_size() * 2

    def get(self, key, make):
        w = self._d.pop(key, None)
        if w is None:
            w = SplitW(make())
        self._d[key] = w                      # most recently used last
        total = sum(self._bytes(v) for v in self._d.values())
        while len(self._d) > 1 and (len(self._d) > self.MAX_ENTRIES or total > self.MAX_BYTES):
            old = self._d.pop(next(iter(self._d)))
            total -= self._bytes(old)
        return w

    def clear(self):
        self._d.clear()


# kept for the dense_sketch hook
def dense_sketch_fused_ok(A, dim, s, k, m) -> bool:
    return False
