"""Streaming tall-skinny products over a row shard of A (the randSVD / LSQR hot path).

For ``A`` (m x n, m >> n) and a skinny ``Z`` (n x k) the randomized SVD needs,
per power iteration, ``Y = A Z`` and ``A^T Y`` (and ``Y^T Y`` to
orthonormalise).  Those are bandwidth-bound (k ~ 40: ~40 flop per A element)
so the only thing that matters is how many times A streams through HBM.

``fused_pass`` reads A ONCE and returns ``W = A^T (A Z)``, ``G = (A Z)^T (A Z)``
(and optionally ``Y = A Z``): the row block's ``y = A_blk Z`` never leaves
the chip.  This halves the HBM traffic of subspace iteration.  On gfx950 it
is the hand-written MFMA kernel ``sl_tsk_fused_pass`` (bf16 A, bf16-hi/lo
split operands, f32 accumulation); elsewhere a chunked torch composition
with the same semantics.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_tsk_fused_pass", [vp, i64, i64, i64, vp, i32, vp, vp, vp, i64, vp, i32, vp])
_lib.register("sl_tsk_fused_workspace", [i64, i64, i32], C.c_int64)
_lib.register("sl_tsk_matmul", [vp, i64, i64, i64, vp, i32, vp, i64, i32, vp])

# rows per chunk in the torch fallback (bounds the y temporary)
CHUNK_ROWS = 1 << 16
USE_NATIVE = True


def _native_ok(A: torch.Tensor, k: int) -> bool:
    if not (USE_NATIVE and A.is_cuda and A.dtype == torch.bfloat16 and k <= 64):
        return False
    if A.stride(1) != 1 or A.shape[1] % 8 or A.stride(0) % 8 or A.shape[1] < 8:
        return False
    n = A.shape[1]
    if n > 1024 or (n > 512 and k > 48):
        return False
    lib = _lib.load()
    return lib is not None and hasattr(lib, "sl_tsk_fused_pass")


def _split_bf16(X: torch.Tensor):
    hi = X.to(torch.bfloat16)
    lo = (X - hi.to(X.dtype)).to(torch.bfloat16)
    return hi, lo


class FusedWorkspace:
    """Per-device scratch for the native fused pass (partial slabs)."""

    def __init__(self):
        self.buf = {}

    def get(self, device, nbytes):
        key = str(device)
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.empty(nbytes, dtype=torch.uint8, device=device)
            self.buf[key] = b
        return b


_WS = FusedWorkspace()


def fused_pass(A: torch.Tensor, Z: torch.Tensor, keep_y: bool = False, gram: bool = True,
               exact: bool = True, ws: torch.Tensor | None = None, gram64: bool = False,
               zt: torch.Tensor | None = None, wg_out: torch.Tensor | None = None, reverse: bool = False):
    """Return ``(W, G, Y)`` with ``Y = A Z``, ``W = A^T Y`` (n x k), ``G = Y^T Y`` (k x k).

    W and G are float32 (A bf16/fp32) or float64 (A fp64); Y is float32/64 or
    None.  Partial over this shard only — the caller all-reduces W and G.
    ``gram=False`` skips G (returns None); ``exact=False`` lets the native
    kernel form W from bf16-rounded y (intermediate power iterations only
    orthonormalise W, so a 2^-9 relative perturbation is harmless there).
    ``gram64=True`` (with ``keep_y`` and ``exact``) forms G from the f32 ``Y``
    with f64 products and f64 accumulation inside the same pass (the fp64
    Gram a CholeskyQR of an ill-conditioned ``Y`` needs; same numbers as
    :func:`gram64` of the returned ``Y`` up to summation order).

    Native-path extras (randSVD device plan): ``zt`` is ``Z`` already in the
    kernel's bf16 ``k x n`` layout (``Z`` may then be None); ``wg_out`` is an
    f64 ``(n + k) x k`` buffer that receives ``[W; G]`` directly (with
    ``gram64``), returned as ``W`` and ``G`` views; ``reverse`` walks the rows
    last-to-first (alternating directions over repeated passes re-reads the
    tail a previous pass left in the Infinity Cache).
    """
    m, n = A.shape
    k = Z.shape[1] if Z is not None else zt.shape[0]
    if _native_ok(A, k):
        return _fused_native(A, Z, keep_y, gram, exact, ws, gram64, zt, wg_out, reverse)
    if Z is None:
        Z = zt.t().float()
    wdt = torch.float64 if A.dtype == torch.float64 else torch.float32
    # low-precision A: Z is rounded to A's dtype (as the MFMA kernel does) and
    # the products are formed in f32
    Zc = Z.to(A.dtype).to(wdt) if A.dtype in (torch.bfloat16, torch.float16) else Z.to(wdt)
    W = torch.zeros(n, k, dtype=wdt, device=A.device)
    G = torch.zeros(k, k, dtype=torch.float64, device=A.device)
    Ys = [] if keep_y else None
    for r0 in range(0, m, CHUNK_ROWS):
        Ab = A[r0:r0 + CHUNK_ROWS]
        y = torch.matmul(Ab.to(wdt), Zc)
        if A.dtype in (torch.bfloat16, torch.float16):
            yh, yl = _split_bf16(y)
            if A.is_cuda:
                W += torch.mm(Ab.t(), yh, out_dtype=torch.float32) + torch.mm(Ab.t(), yl, out_dtype=torch.float32)
            else:
                W += Ab.t().float() @ (yh.float() + yl.float())
        else:
            W += torch.matmul(Ab.t().to(wdt), y)
        G += (y.double().t() @ y.double()) if gram64 else (y.t() @ y).double()
        if keep_y:
            Ys.append(y)
    Y = torch.cat(Ys, 0) if keep_y and Ys else (torch.zeros(0, k, dtype=wdt, device=A.device) if keep_y else None)
    if wg_out is not None:
        wg_out[:n].copy_(W)
        wg_out[n:].copy_(G)
        return wg_out[:n], wg_out[n:], Y
    return W, G, Y


def fused_workspace_bytes(m: int, n: int, k: int) -> int:
    return max(int(_lib.require().sl_tsk_fused_workspace(m, n, k)), 16)


def f32_workspace_bytes(m: int) -> int:
    return int(_lib.require().sl_tsk_f32_workspace(m))


def _fused_native(A: torch.Tensor, Z: torch.Tensor | None, keep_y: bool, gram: bool = True, exact: bool = True,
                  ws: torch.Tensor | None = None, gram64: bool = False, zt: torch.Tensor | None = None,
                  wg_out: torch.Tensor | None = None, reverse: bool = False):
    m, n = A.shape
    dev = A.device
    if zt is not None:
        k = zt.shape[0]
        if zt.dtype != torch.bfloat16 or tuple(zt.shape) != (k, n) or zt.stride(1) != 1 or zt.stride(0) != n:
            raise ValueError("fused_pass: zt must be a contiguous bf16 k x n tensor")
        Zb = zt
    else:
        k = Z.shape[1]
        Zb = Z.t().to(torch.bfloat16).contiguous()  # Zt layout (k x n)
    g64 = bool(gram64 and gram and keep_y and exact)
    flags = (0 if gram else 1) | (0 if exact else 2) | (4 if g64 else 0) | (32 if reverse else 0)
    if wg_out is not None:
        # f64 W straight into wg_out[:n]; with the in-pass fp64 Gram also G
        # into wg_out[n:] (gram=False leaves that block to the caller)
        if not (g64 or not gram) or wg_out.dtype != torch.float64 or tuple(wg_out.shape) != (n + k, k) \
                or not wg_out.is_contiguous():
            raise ValueError("fused_pass: wg_out needs gram64 (or gram=False) and a contiguous f64 (n + k) x k buffer")
        W, G = wg_out[:n], wg_out[n:]
        flags |= 16
    else:
        W = torch.empty(n, k, dtype=torch.float32, device=dev)
        G = torch.empty(k, k, dtype=torch.float64 if g64 else torch.float32, device=dev)
    Y = torch.empty(m, k, dtype=torch.float32, device=dev) if keep_y else None
    if ws is None:
        ws = _WS.get(dev, fused_workspace_bytes(m, n, k))
    _lib.call("sl_tsk_fused_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zb), k, _lib.ptr(W), _lib.ptr(G),
              _lib.ptr(Y) if Y is not None else None, 0 if Y is None else Y.stride(0), _lib.ptr(ws),
              flags, vp(_lib.stream_of(A)))
    return W, (G if G.dtype == torch.float64 else G.double()) if gram else None, Y


_lib.register("sl_tsk_f32_xm", [vp, i64, i32, i64, vp, i32, vp, i64, vp, vp, vp])
_lib.register("sl_tsk_f32_workspace", [i64], C.c_int64)
_WS32 = FusedWorkspace()


def f32_xm(Y: torch.Tensor, M: torch.Tensor | None = None, store: bool = True, gram: bool = False,
           ws: torch.Tensor | None = None):
    """``Q = Y M`` (``M=None``: ``Q = Y``) for tall f32 ``Y`` (k, k2 <= 64).

    Returns ``(Q or None, G or None)`` with ``G = Q^T Q`` in float64 (partial
    over this shard).  Native streaming kernel on GPU, torch on CPU.
    """
    m, k = Y.shape
    k2 = k if M is None else M.shape[1]
    if Y.is_cuda and Y.dtype == torch.float32 and k <= 64 and k2 <= 64 and Y.stride(1) == 1 and _lib.available():
        Mc = None if M is None else M.to(device=Y.device, dtype=torch.float32).contiguous()
        out = torch.empty(m, k2, dtype=torch.float32, device=Y.device) if (store and M is not None) else None
        G = torch.empty(k2, k2, dtype=torch.float64, device=Y.device) if gram else None
        if gram and ws is None:
            ws = _WS32.get(Y.device, f32_workspace_bytes(m))
        _lib.call("sl_tsk_f32_xm", _lib.ptr(Y), m, k, Y.stride(0), _lib.ptr(Mc) if Mc is not None else None, k2,
                  _lib.ptr(out) if out is not None else None, out.stride(0) if out is not None else 0,
                  _lib.ptr(G) if G is not None else None, _lib.ptr(ws) if ws is not None else None,
                  vp(_lib.stream_of(Y)))
        return (out if M is not None else (Y if store else None)), G
    Q = Y if M is None else Y @ M.to(Y.dtype)
    G = None
    if gram:
        from ..base.linalg import gram as _g
        G = _g(Q, None)
    return (Q if store else None), G


_lib.register("sl_tsk_f32_xm_bf16t", [vp, i64, i32, i64, vp, i32, vp, i64, vp])


def f32_xm_bf16t(Y: torch.Tensor, M: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """``(Y M)^T`` as a contiguous bf16 ``k2 x m`` tensor (the fused pass's Zt
    operand layout) in one launch; torch on CPU."""
    m, k = Y.shape
    k2 = M.shape[1]
    if out is None:
        out = torch.empty(k2, m, dtype=torch.bfloat16, device=Y.device)
    if Y.is_cuda and Y.dtype == torch.float32 and Y.stride(1) == 1 and k <= 64 and k2 <= 64 and _lib.available():
        Mc = M.to(device=Y.device, dtype=torch.float32).contiguous()
        _lib.call("sl_tsk_f32_xm_bf16t", _lib.ptr(Y), m, k, Y.stride(0), _lib.ptr(Mc), k2, _lib.ptr(out),
                  out.stride(0), vp(_lib.stream_of(Y)))
        return out
    out.copy_((Y.float() @ M.float()).t())
    return out


_lib.register("sl_tsk_gram64", [vp, i64, i32, i64, vp, vp, vp])
_lib.register("sl_tsk_gram64_workspace", [i64, i32], C.c_int64)


def gram64_workspace_bytes(m: int, k: int) -> int:
    return int(_lib.require().sl_tsk_gram64_workspace(m, k))


def gram64(Y: torch.Tensor, ws: torch.Tensor | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """``G = Y^T Y`` in float64 for tall f32 ``Y`` (k <= 64), partial over this
    shard: fp64 products and sums on the f64 matrix cores, so one fp64
    CholeskyQR of ``Y`` from this ``G`` is as orthogonal as CholeskyQR2 with an
    f32 second Gram.  Torch (fp64) on CPU."""
    m, k = Y.shape
    if Y.is_cuda and Y.dtype == torch.float32 and k <= 64 and Y.stride(1) == 1 and _lib.available():
        G = out if out is not None else torch.empty(k, k, dtype=torch.float64, device=Y.device)
        if not (G.dtype == torch.float64 and G.is_contiguous() and tuple(G.shape) == (k, k)):
            raise ValueError("gram64: out must be a contiguous f64 k x k tensor")
        if ws is None:
            ws = _WS32.get(Y.device, gram64_workspace_bytes(m, k))
        _lib.call("sl_tsk_gram64", _lib.ptr(Y), m, k, Y.stride(0), _lib.ptr(G), _lib.ptr(ws), vp(_lib.stream_of(Y)))
        return G
    Yd = Y.double()
    return Yd.t() @ Yd


def matmul(A: torch.Tensor, Z: torch.Tensor, out_dtype=torch.float32) -> torch.Tensor:
    """``Y = A Z`` streaming (A bf16 m x n, Z n x k small) with f32 output."""
    if _native_ok(A, Z.shape[1]) and hasattr(_lib.require(), "sl_tsk_matmul"):
        m, n = A.shape
        k = Z.shape[1]
        hi, lo = _split_bf16(Z.float())
        Zs = torch.cat([hi.t(), lo.t()], 0).contiguous()  # [Z_hi^T; Z_lo^T] (2k x n)
        Y = torch.empty(m, k, dtype=torch.float32, device=A.device)
        _lib.call("sl_tsk_matmul", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zs), k, _lib.ptr(Y), Y.stride(0), 1,
                  vp(_lib.stream_of(A)))
        return Y.to(out_dtype)
    if A.dtype in (torch.bfloat16, torch.float16):
        hi, lo = _split_bf16(Z.float())
        return (torch.matmul(A, hi).float() + torch.matmul(A, lo).float()).to(out_dtype)
    return torch.matmul(A, Z.to(A.dtype)).to(out_dtype)
