"""One-pass ``A^T (A Y)`` for tall f32 (or bf16-stored) operators (``ata_kernels.hip``).

Used by the Krylov solvers (LSQR, Chebyshev) so that an iteration reads A
once instead of twice (reference loops ``algorithms/Krylov/LSQR.hpp:113-248``,
``Chebyshev.hpp:18-85``).  Falls back to two products where the kernel does
not apply (CPU, f64, sparse, wide n, k > 4).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_ata_pass", [vp, i64, i64, i64, vp, i32, vp, vp, i64, vp, vp])
_lib.register("sl_ata_workspace", [i64, i32], C.c_int64)
_lib.register("sl_ata_pass2", [vp, i64, i64, i64, vp, i32, vp, vp, i64, vp, i64, i64, vp, vp])
_lib.register("sl_ata_pass3", [vp, i32, i64, i64, i64, vp, i32, vp, vp, i64, vp, i64, i64, vp, vp, i32])
_lib.register("sl_gemv_rows_f32", [vp, i64, i64, i64, vp, i32, vp, i64, vp])
_lib.register("sl_rsvd_pass_ext", [vp, i64, i64, i64, vp, i32, vp, vp, i64, vp, i64, i32, vp])
_lib.register("sl_rsvd_pass_workspace", [i64, i64, i32], C.c_int64)
_lib.register("sl_rsvd_reduce_z", [vp, i64, i64, i32, vp, i32, i32, vp, i32, vp, vp])
_DT = {torch.float32: 0, torch.bfloat16: 2}   # SlDtype codes of the stored A

_WS: dict = {}


def native_ok(A: torch.Tensor, k: int) -> bool:
    """f32 A, or a bf16-stored A (e.g. BlockADMM's bf16 feature cache: the
    kernel widens each element to f32, products and sums stay f32)."""
    if not (isinstance(A, torch.Tensor) and A.is_cuda and A.dtype in _DT and A.dim() == 2
            and A.layout == torch.strided and A.stride(1) == 1 and _lib.available()):
        return False
    n = A.shape[1]
    J = -(-n // 256)
    if n > 6144 or k not in (1, 2, 4) or (J > 8 and k == 4) or (J > 16 and k > 1):
        return False
    return True


def _ws(A, n, k):
    """Slab workspace per (device, stream): launches on different streams
    (side-stream overlap, concurrent solvers) never share scratch."""
    nb = int(_lib.require().sl_ata_workspace(n, k))
    key = (str(A.device), torch.cuda.current_stream(A.device).cuda_stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < nb:
        ws = _WS[key] = torch.empty(nb, dtype=torch.uint8, device=A.device)
    return ws


def dual(A: torch.Tensor, D: torch.Tensor, X: torch.Tensor | None = None, y_out: torch.Tensor | None = None):
    """``(A^T D, A X or None)`` from ONE read of A (m x n): D is m x k (any
    strides, e.g. the transpose of a k x m block), X n x k.  The BlockADMM pair
    ``{Z Wbar, Z^T d}`` (``ml/BlockADMM.hpp:400-498``).  ``y_out`` (m x k f32,
    contiguous): A X is ADDED into it (and returned) instead of a new tensor."""
    k = D.shape[1]
    if X is not None and X.shape[1] != k:
        raise ValueError("dual: X and D need the same number of columns")
    if native_ok(A, k) and D.dtype == torch.float32 and D.is_cuda:
        m, n = A.shape
        W = torch.empty(n, k, dtype=torch.float32, device=A.device)
        Xc = X.to(torch.float32).contiguous() if X is not None else None
        acc = y_out is not None and X is not None
        Yo = y_out if acc else (torch.empty(m, k, dtype=torch.float32, device=A.device) if X is not None else None)
        _lib.call("sl_ata_pass3", _lib.ptr(A), _DT[A.dtype], m, n, A.stride(0),
                  _lib.ptr(Xc) if Xc is not None else None, k, _lib.ptr(W), _lib.ptr(Yo) if Yo is not None else None,
                  k, _lib.ptr(D), D.stride(0), D.stride(1), _lib.ptr(_ws(A, n, k)), vp(_lib.stream_of(A)), int(acc))
        return W, Yo
    Af = A.float() if A.dtype == torch.bfloat16 else A
    AX = Af @ X.to(Af.dtype) if X is not None else None
    if AX is not None and y_out is not None:
        AX = y_out.add_(AX)
    return Af.t() @ D.to(Af.dtype), AX


def ata(A: torch.Tensor, Y: torch.Tensor, want_y: bool = False, y_out: torch.Tensor | None = None):
    """``(A^T (A Y), A Y or None)`` for the local block A (m x n) and Y (n x k).
    Partial over a row shard: the caller all-reduces the first result.
    ``y_out`` (m x k f32, contiguous, with want_y): A Y is ADDED into it."""
    k = Y.shape[1]
    if native_ok(A, k):
        m, n = A.shape
        Yc = Y.to(torch.float32).contiguous()
        W = torch.empty(n, k, dtype=torch.float32, device=A.device)
        acc = y_out is not None and want_y
        Yo = y_out if acc else (torch.empty(m, k, dtype=torch.float32, device=A.device) if want_y else None)
        _lib.call("sl_ata_pass3", _lib.ptr(A), _DT[A.dtype], m, n, A.stride(0), _lib.ptr(Yc), k, _lib.ptr(W),
                  _lib.ptr(Yo) if Yo is not None else None, k, None, 0, 0, _lib.ptr(_ws(A, n, k)),
                  vp(_lib.stream_of(A)), int(acc))
        return W, Yo
    Af = A.float() if A.dtype == torch.bfloat16 else A
    AY = Af @ Y.to(Af.dtype)
    WW = Af.t() @ AY
    if want_y and y_out is not None:
        AY = y_out.add_(AY)
    return WW, (AY if want_y else None)


def gemv_ok(A: torch.Tensor, k: int) -> bool:
    """Can ``A @ X`` (X with k columns) take the wide-row streaming GEMV
    (gemv_kernels.hip)?  f32 on the GPU, k in {1, 2, 4}, rows 16-B aligned."""
    return (isinstance(A, torch.Tensor) and A.is_cuda and A.dtype == torch.float32 and A.dim() == 2
            and A.stride(1) == 1 and A.shape[1] % 4 == 0 and A.stride(0) % 4 == 0 and A.data_ptr() % 16 == 0
            and k in (1, 2, 4) and _lib.available())


def gemv(A: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    """``A @ X`` (A m x n f32, X n or n x k) by one streaming read of A:
    every workgroup owns 4 rows, X is re-read from L2 (transposed to k x n)."""
    vec = X.dim() == 1
    X2 = X[:, None] if vec else X
    m, n = A.shape
    k = X2.shape[1]
    Xt = X2.to(torch.float32).t().contiguous()
    if Xt.data_ptr() % 16:
        # a contiguous view at an unaligned storage offset passes through
        # .contiguous() unchanged; the kernel reads X in 16-B pieces
        Xt = Xt.clone()
    Y = torch.empty(m, k, dtype=torch.float32, device=A.device)
    _lib.call("sl_gemv_rows_f32", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Xt), k, _lib.ptr(Y), Y.stride(0),
              C.c_void_p(_lib.stream_of(A)))
    return Y[:, 0] if vec else Y


# ------------------------------------------------------------ matrix-core form
def mfma_ok(A: torch.Tensor, k: int, D: torch.Tensor | None = None) -> bool:
    """Can the fused pass's EXT form (rsvd_pass.hip sl_rsvd_pass_ext) take this
    bf16 A (n <= 1024 columns) with k <= 8 right-hand sides (and D)?"""
    if not (isinstance(A, torch.Tensor) and A.is_cuda and A.dtype == torch.bfloat16 and A.dim() == 2
            and A.stride(1) == 1 and A.stride(0) % 8 == 0 and A.shape[1] % 8 == 0 and 16 <= A.shape[1] <= 1024
            and 1 <= k <= 8 and A.data_ptr() % 16 == 0 and _lib.available()):
        return False
    if D is not None:
        m = A.shape[0]
        return (D.is_cuda and D.dtype == torch.float32 and D.shape == (m, k) and D.stride(0) == 1
                and D.stride(1) % 4 == 0 and D.stride(1) >= m and D.data_ptr() % 16 == 0 and m % 16 == 0)
    return True


def pass_mfma(A: torch.Tensor, X: torch.Tensor, D: torch.Tensor | None = None):
    """``(W, Y)`` with ``Y = A X`` (m x k f32) and ``W = A^T Y`` -- or ``W =
    A^T D`` when D is given -- from ONE read of the bf16 A on the matrix
    cores: the randSVD fused pass (LDS-DMA ring, MFMA) with X entering as its
    bf16 hi / lo planes (products exact, f32 sums) and the long operand of
    the W product as bf16 hi + lo (~2^-17 relative).  BlockADMM's two
    passes per feature block over its bf16 cache (reference
    ml/BlockADMM.hpp:400-498); the VALU widening kernel (``dual`` / ``ata``)
    is issue-bound on bf16 (3.4-3.6 TB/s)."""
    m, n = A.shape
    k = X.shape[1]
    Xf = X.to(torch.float32)
    hi = Xf.to(torch.bfloat16)
    lo = (Xf - hi.float()).to(torch.bfloat16)
    Zt2 = torch.cat([hi.t(), lo.t()]).contiguous()            # 2k x n
    lib = _lib.require()
    nb = int(lib.sl_rsvd_pass_workspace(m, n, k))
    key = ("mfma", str(A.device), torch.cuda.current_stream(A.device).cuda_stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < nb:
        ws = _WS[key] = torch.empty(nb, dtype=torch.uint8, device=A.device)
    Y = torch.empty(m, k, dtype=torch.float32, device=A.device)
    st = vp(_lib.stream_of(A))
    _lib.call("sl_rsvd_pass_ext", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt2), k, _lib.ptr(ws), _lib.ptr(Y), k,
              _lib.ptr(D) if D is not None else None, D.stride(1) if D is not None else 0, 0, st)
    W = torch.empty(n, k, dtype=torch.float32, device=A.device)
    _lib.call("sl_rsvd_reduce_z", _lib.ptr(ws), m, n, k, _lib.ptr(W), 0, k, None, 0, None, st)
    return W, Y
