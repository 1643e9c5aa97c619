"""Native column reductions and fused LSQR updates (``krylov_kernels.hip``).

Tall-skinny blocks (rows x k, k <= 64, f32/f64, unit column stride) on the
GPU: per-column sums of squares / dots in one streaming pass with f64
accumulation (two launches), ``Y = a X + b Y`` fused with the new column
norms, and LSQR's steps 4-12 (Givens rotation, X / W updates, |W| and every
scalar recurrence) in two launches with all scalars device resident.
Reference: ``algorithms/Krylov/LSQR.hpp:113-248``, ``base/inner.hpp:22-170``.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

vp, i32, i64, f64 = C.c_void_p, C.c_int, C.c_int64, C.c_double
_lib.register("sl_krylov_ws_bytes", [i32], C.c_int64)
_lib.register("sl_colred", [vp, i64, vp, i64, i64, i32, i32, i32, vp, i32, vp, vp])
_lib.register("sl_axpby_red", [vp, i64, vp, i64, i64, i32, i32, vp, f64, vp, f64, vp, i32, vp, vp, vp, vp])
_lib.register("sl_lsqr_setstate", [vp, i32, vp, i32, vp])
_lib.register("sl_rows_gemm", [vp, i64, i64, i64, vp, i64, i32, vp, i64, i32, vp])
_lib.register("sl_colscale", [vp, i64, i64, i32, i32, vp, i32, vp])
_lib.register("sl_lsqr_nstate", [], C.c_int)
_lib.register("sl_lsqr_step", [vp, i64, vp, i64, vp, i64, i64, i32, i32, vp, vp, f64, f64, i32, vp, vp])

_WS: dict = {}
ENABLED = True     # tests flip this to run the torch reference path on the GPU

# LSQR scalar-state rows (krylov_kernels.hip enum)
(S_ALPHA, S_BETA, S_RHOBAR, S_PHIBAR, S_NRMA, S_SQD, S_CNDA, S_NRMX, S_SQX, S_CS2, S_SN2, S_ZZ, S_NRMAR0, S_STAG,
 S_RHO, S_PHI, S_THETA, S_NRMAR) = range(18)


def ok(*ts) -> bool:
    """Native path applies: CUDA, f32/f64, 2-D with unit column stride, 1 <= k <= 64."""
    if not ENABLED or not _lib.available():
        return False
    for t in ts:
        if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype in (torch.float32, torch.float64)
                and t.dim() == 2 and t.stride(1) == 1 and 1 <= t.shape[1] <= 64):
            return False
    return True


def _ws(dev, k):
    nb = int(_lib.require().sl_krylov_ws_bytes(k))
    key = str(dev)
    w = _WS.get(key)
    if w is None or w.numel() < nb:
        w = _WS[key] = torch.empty(nb, dtype=torch.uint8, device=dev)
    return w


def _st(t):
    return vp(_lib.stream_of(t))


def colsumsq(X: torch.Tensor) -> torch.Tensor:
    """Per-column sum of squares (f64 k-vector)."""
    m, k = X.shape
    out = torch.empty(k, dtype=torch.float64, device=X.device)
    _lib.call("sl_colred", _lib.ptr(X), X.stride(0), None, 0, m, k, _lib.dtype_code(X.dtype), 0, _lib.ptr(out), 0,
              _lib.ptr(_ws(X.device, k)), _st(X))
    return out


def coldot(X: torch.Tensor, Y: torch.Tensor) -> torch.Tensor:
    """Per-column dot products (f64 k-vector)."""
    m, k = X.shape
    if Y.dtype != X.dtype:
        Y = Y.to(X.dtype)
    if Y.stride(1) != 1:
        Y = Y.contiguous()
    out = torch.empty(k, dtype=torch.float64, device=X.device)
    _lib.call("sl_colred", _lib.ptr(X), X.stride(0), _lib.ptr(Y), Y.stride(0), m, k, _lib.dtype_code(X.dtype), 1,
              _lib.ptr(out), 0, _lib.ptr(_ws(X.device, k)), _st(X))
    return out


def axpby(X: torch.Tensor, Y: torch.Tensor, a=None, sa: float = 1.0, b=None, sb: float = 1.0, d=None,
          red: int = 0, st: torch.Tensor | None = None):
    """In place ``Y = (sa a .* X + sb b .* Y) ./ d`` with per-column f64 device
    scalars (None: a = 1, b = 0, d = 1).  ``red``: 0 nothing; 1 return the new
    Y's column sums of squares; 2 / 3 set the LSQR state ``st`` (beta and the
    |A| estimate / alpha) from |Y| (single rank)."""
    m, k = Y.shape
    if X.dtype != Y.dtype:
        X = X.to(Y.dtype)
    if X.stride(1) != 1:
        X = X.contiguous()
    out = torch.empty(k, dtype=torch.float64, device=Y.device) if red == 1 else None

    def p(v):
        return _lib.ptr(v) if v is not None else None
    _lib.call("sl_axpby_red", _lib.ptr(X), X.stride(0), _lib.ptr(Y), Y.stride(0), m, k, _lib.dtype_code(Y.dtype),
              p(a), float(sa), p(b), float(sb), p(d), int(red), p(out), p(st), _lib.ptr(_ws(Y.device, k)), _st(Y))
    return out


def axpby_colsumsq(X: torch.Tensor, Y: torch.Tensor, a: torch.Tensor | None, b: torch.Tensor | None) -> torch.Tensor:
    """In place ``Y = a .* X + b .* Y``; returns the new Y's column sums of squares."""
    av = a.to(torch.float64).contiguous() if a is not None else None
    bv = b.to(torch.float64).contiguous() if b is not None else None
    return axpby(X, Y, av, 1.0, bv, 1.0, None, red=1)


def setstate(sums: torch.Tensor, st: torch.Tensor, mode: int):
    """LSQR state from all-reduced column sums of squares (1: beta + |A|, 2: alpha)."""
    k = st.shape[1]
    _lib.call("sl_lsqr_setstate", _lib.ptr(sums), k, _lib.ptr(st), int(mode), _st(st))


def colscale(Y: torch.Tensor, s: torch.Tensor, inv: bool = False) -> torch.Tensor:
    """In place ``Y[:, c] *= s[c]`` (``/= s[c]`` with ``inv``; zero divisor -> 0)."""
    m, k = Y.shape
    sv = s.to(torch.float64).contiguous()
    _lib.call("sl_colscale", _lib.ptr(Y), Y.stride(0), m, k, _lib.dtype_code(Y.dtype), _lib.ptr(sv), int(inv), _st(Y))
    return Y


def lsqr_state(k: int, device) -> torch.Tensor:
    return torch.zeros(int(_lib.require().sl_lsqr_nstate()), k, dtype=torch.float64, device=device)


def lsqr_step(X, W, Z, st, flags, tol: float, eps: float, max_stag: int):
    """LSQR steps 4-12: X, W updated in place, ``st`` advanced, ``flags`` (int32 k)
    set (1 S1, 2 S2, 4 S3, 8 stagnation)."""
    n, k = X.shape
    if Z.stride(1) != 1:
        Z = Z.contiguous()
    _lib.call("sl_lsqr_step", _lib.ptr(X), X.stride(0), _lib.ptr(W), W.stride(0), _lib.ptr(Z), Z.stride(0), n, k,
              _lib.dtype_code(X.dtype), _lib.ptr(st), _lib.ptr(flags), float(tol), float(eps), int(max_stag),
              _lib.ptr(_ws(X.device, k)), _st(X))


def thin_gemm_ok(M: torch.Tensor, X: torch.Tensor) -> bool:
    return (ENABLED and _lib.available() and M.is_cuda and X.is_cuda and M.dim() == 2 and X.dim() == 2
            and M.dtype == X.dtype and M.dtype in (torch.float32, torch.float64) and M.stride(1) == 1
            and X.stride(1) == 1 and 1 <= X.shape[1] <= 8 and M.shape[1] == X.shape[0])


def thin_gemm(M: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    """``M @ X`` for a row-major M and a thin X (<= 8 columns): one wave per row."""
    nr, nc = M.shape
    k = X.shape[1]
    Y = torch.empty(nr, k, dtype=M.dtype, device=M.device)
    _lib.call("sl_rows_gemm", _lib.ptr(M), M.stride(0), nr, nc, _lib.ptr(X), X.stride(0), k, _lib.ptr(Y),
              Y.stride(0), _lib.dtype_code(M.dtype), _st(M))
    return Y


# ------------------------------------------------------------------ CG / FCG
_lib.register("sl_cg_nstate", [], C.c_int)
_lib.register("sl_cg_dot", [vp, i64, vp, i64, vp, i64, i64, i32, i32, i32, vp, vp, vp, vp])
_lib.register("sl_cg_p", [vp, i64, vp, i64, i64, i32, i32, vp, f64, vp])
_lib.register("sl_cg_xr", [vp, i64, vp, i64, vp, i64, vp, i64, i64, i32, i32, i32, vp, vp, f64, vp, vp, vp])

# CG scalar-state rows (krylov_kernels.hip enum)
C_RHO, C_RHO0, C_ALPHA, C_BETA, C_PQ, C_RR, C_NRMB = range(7)


class CGState:
    """Device state of a (flexible) CG run: per-column f64 scalars, the
    reduction workspace, the last-block ticket counter and the stop flags."""

    def __init__(self, k: int, device):
        L = _lib.require()
        self.k = k
        self.st = torch.zeros(int(L.sl_cg_nstate()), k, dtype=torch.float64, device=device)
        self.ws = torch.empty(2 * int(L.sl_krylov_ws_bytes(k)), dtype=torch.uint8, device=device)
        self.counter = torch.zeros(4, dtype=torch.int32, device=device)
        self.flags = torch.zeros(k, dtype=torch.int32, device=device)


def _c(t):
    return t if t.stride(1) == 1 else t.contiguous()


def cg_dot(X: torch.Tensor, Y: torch.Tensor, mode: int, cs: CGState, Y2: torch.Tensor | None = None):
    """Column dots finished on the device into the CG state (see sl_cg_dot)."""
    m, k = X.shape
    Y = _c(Y.to(X.dtype))
    Y2 = _c(Y2.to(X.dtype)) if Y2 is not None else None
    _lib.call("sl_cg_dot", _lib.ptr(X), X.stride(0), _lib.ptr(Y), Y.stride(0),
              _lib.ptr(Y2) if Y2 is not None else None, Y2.stride(0) if Y2 is not None else 0, m, k,
              _lib.dtype_code(X.dtype), int(mode), _lib.ptr(cs.st), _lib.ptr(cs.ws), _lib.ptr(cs.counter), _st(X))


def cg_p(Z: torch.Tensor, P: torch.Tensor, cs: CGState, sb: float = 1.0):
    """In place ``P = Z + sb * beta .* P``."""
    m, k = P.shape
    Z = _c(Z.to(P.dtype))
    _lib.call("sl_cg_p", _lib.ptr(Z), Z.stride(0), _lib.ptr(P), P.stride(0), m, k, _lib.dtype_code(P.dtype),
              _lib.ptr(cs.st), float(sb), _st(P))


def cg_xr(X, P, R, Q, cs: CGState, idp: bool, tol: float):
    """In place ``X += alpha P``, ``R -= alpha Q``; |R|^2, stop flags and (idp)
    rho / beta into the state."""
    m, k = X.shape
    Q = _c(Q.to(X.dtype))
    _lib.call("sl_cg_xr", _lib.ptr(X), X.stride(0), _lib.ptr(P), P.stride(0), _lib.ptr(R), R.stride(0), _lib.ptr(Q),
              Q.stride(0), m, k, _lib.dtype_code(X.dtype), int(bool(idp)), _lib.ptr(cs.st), _lib.ptr(cs.flags),
              float(tol), _lib.ptr(cs.ws), _lib.ptr(cs.counter), _st(X))
