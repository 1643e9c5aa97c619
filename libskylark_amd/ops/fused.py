"""Fused dense-sketch / random-feature / kernel-Gram GEMM on the 256 x 256
bf16 NT GEMM (``_native/src/gemm_nt.hip``, ``sl_gemm_nt_map``).

``Z = outscale * map(scale_f * (A W^T)[r, f] + shift_f)`` in one launch on
bf16 MFMA: f32 inputs are split once into bf16 hi + lo planes (one streaming
pass) and the realised sketching matrix W is held as a bf16 hi + lo pair; the
3-term product ``Ah Wh + Al Wh + Ah Wl`` goes in as ONE GEMM over the terms
concatenated along K (f32-class accuracy, |err| ~ 2^-16 of sum |a w|).
Rowwise maps (dim 1) compute ``X W^T`` with the features along the output
columns; columnwise maps (dim 0) compute ``W X^T`` with the features along
the output rows (the kernel's FROW epilogue), no transposed copy of Z.

Used by the dense transforms (JLT / CT / SJLT, ``map = none``), the feature
maps (RFT / QRFT ``cos``, RLT / QRLT ``exp(-x)``) and the Gaussian /
polynomial kernel Grams (``ml.kernels``) whenever W (``S x N``) is small
enough to realise once and cache on the device (``MAX_W_ELEMS``); tall
sketched dimensions stream W panels through ``ops.dense_sketch`` instead.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from . import _lib

EPI_NONE, EPI_COS, EPI_EXPNEG, EPI_GAUSS, EPI_POLY = 0, 1, 2, 3, 4
BN, BK = 128, 32                # SplitW padding of W (rows, K)
MAX_W_ELEMS = 1 << 26          # W (S x N) realised whole up to 64 M entries (256 MB as hi+lo)

_lib.register("sl_gemm_nt_map", [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int,
                                 C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_float,
                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_void_p])
_lib.register("sl_split_bf16", [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                C.c_void_p])
_lib.register("sl_split_bf16_2", [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                  C.c_int64, C.c_void_p])
_lib.register("sl_split_bf16_t", [C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_void_p, C.c_void_p, C.c_int,
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


def _x_terms(X: torch.Tensor, use_lo: bool):
    """The data operand as bf16 terms concatenated along K: ``(P, terms_W)``
    with ``P = [X_h | X_l | X_h]`` (f32 X; ``[X_h | X_l]`` without W's lo
    plane) or ``[X | X]`` / ``[X]`` (bf16 X), each term ``kp`` wide (k
    rounded up to 64, zero padded), and the matching W terms."""
    m, k = X.shape
    kp = -(-k // 64) * 64
    dev = X.device
    if X.dtype == torch.float32:
        ta, tb = (("h", "l", "h"), ("h", "h", "l")) if use_lo else (("h", "l"), ("h", "h"))
    else:
        ta, tb = (("h", "h"), ("h", "l")) if use_lo else (("h",), ("h",))
    P = torch.empty(m, len(ta) * kp, dtype=torch.bfloat16, device=dev)
    st = C.c_void_p(_lib.stream_of(X))
    if X.dtype == torch.float32:
        if X.stride(1) != 1 and X.stride(0) == 1 and X.t().stride(0) % 4 == 0:
            # X = A^T of a row-major A (k x m): the transposing split reads A directly
            At = X.t()
            _lib.call("sl_split_bf16_t", _lib.ptr(At), k, m, At.stride(0), _lib.ptr(P), _lib.ptr(P[:, kp:]), kp,
                      P.stride(0), st)
        else:
            Xc = X if (X.stride(1) == 1 and X.stride(0) % 4 == 0 and X.data_ptr() % 16 == 0) else X.contiguous()
            _lib.call("sl_split_bf16_2", _lib.ptr(Xc), m, k, Xc.stride(0), _lib.ptr(P), _lib.ptr(P[:, kp:]), kp,
                      P.stride(0), st)
        if len(ta) == 3:
            P[:, 2 * kp:].copy_(P[:, :kp])
    else:
        P[:, :k] = X
        if kp > k:
            P[:, k:kp].zero_()
        for i in range(1, len(ta)):
            P[:, i * kp:(i + 1) * kp].copy_(P[:, :kp])
    return P, tb


def feature_gemm(A: torch.Tensor, W: SplitW, dim: int, *, scales=None, shifts=None,
                 outscale: float = 1.0, epi: int = EPI_NONE, out_dtype=torch.float32,
                 use_lo: bool = True, rowterm=None, p0: float = 0.0) -> torch.Tensor:
    """Columnwise (dim 0: A is K x m -> Z is nf x m) or rowwise (dim 1: A is
    m x K -> Z is m x nf) fused product with W^T and the map; ``rowterm`` is
    the per-data-point term of the Gaussian Gram."""
    X = A if dim == 1 else A.t()
    m, k = X.shape
    if k != W.k:
        raise ValueError(f"feature_gemm: inner dimension {k} != {W.k}")
    P, tb = _x_terms(X, use_lo)
    B = W.concat(tb)
    dev = A.device
    sc = scales.to(device=dev, dtype=torch.float32).contiguous() if scales is not None else None
    sh = shifts.to(device=dev, dtype=torch.float32).contiguous() if shifts is not None else None
    rt = rowterm.to(device=dev, dtype=torch.float32).contiguous() if rowterm is not None else None
    if dim == 1:
        out = torch.empty(m, W.nf, dtype=out_dtype, device=dev)
        Aop, Bop, M, N = P, B, m, W.nf
    else:
        out = torch.empty(W.nf, m, dtype=out_dtype, device=dev)
        Aop, Bop, M, N = B, P, W.nf, m
    _lib.call("sl_gemm_nt_map", _lib.ptr(Aop), Aop.stride(0), _lib.ptr(Bop), Bop.stride(0), M, N, P.shape[1],
              _lib.ptr(out), out.stride(0), _lib.dtype_code(out_dtype), int(epi), int(dim == 0), float(outscale),
              _lib.ptr(sc) if sc is not None else None, _lib.ptr(sh) if sh is not None else None,
              _lib.ptr(rt) if rt is not None else None, float(p0), C.c_void_p(_lib.stream_of(out)))
    return out


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

