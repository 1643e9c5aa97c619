"""Hand-written bf16 NT GEMM on MFMA (``gemm_nt.hip``): ``C = epi(A B^T)``
for K-contiguous bf16 ``A`` (M x K) and ``B`` (N x K), f32 accumulation.

Used for the dense-sketch panel products (LSRN's t x N sketch of a tall
block, ``ops/dense_sketch.py``) and the random-feature map with its cosine
epilogue (reference ``sketch/dense_transform_data.hpp:79-152``,
``sketch/RFT_Elemental.hpp:83-160``).  K must be a multiple of 64; the
helpers below zero-pad.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_gemm_nt_bf16", [vp, i64, vp, i64, i32, i32, i32, vp, i64, i32, i32, i32, C.c_float, vp, vp, vp])
_lib.register("sl_split_bf16_t", [vp, i32, i32, i64, vp, vp, i32, i64, vp])
_lib.register("sl_gemm_nt_set_nt_store", [i32], None)


def set_nt_store(mode: int) -> None:
    """C-store cache policy of the NT GEMM: -1 auto (non-temporal stores for
    C >= 64 MiB at K <= 2048, the default), 0 always default, 1 always
    non-temporal.  Process-wide (an A/B and test knob)."""
    _lib.require().sl_gemm_nt_set_nt_store(int(mode))

BK = 64


def ok(A: torch.Tensor, B: torch.Tensor) -> bool:
    return (A.is_cuda and B.is_cuda and A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16
            and A.dim() == 2 and B.dim() == 2 and A.shape[1] == B.shape[1] and A.stride(1) == 1
            and B.stride(1) == 1 and A.stride(0) % 8 == 0 and B.stride(0) % 8 == 0 and A.shape[1] % BK == 0
            and A.data_ptr() % 16 == 0 and B.data_ptr() % 16 == 0 and _lib.available())


def gemm_nt(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor | None = None, *, alpha: float = 1.0,
            accumulate: bool = False, out_dtype: torch.dtype = torch.float32,
            cos_scales: torch.Tensor | None = None, cos_shifts: torch.Tensor | None = None) -> torch.Tensor:
    """``out (+)= alpha A B^T``, or the feature map
    ``out = alpha cos(cos_scales * (A B^T) + cos_shifts)`` (per output column)
    when ``cos_scales`` / ``cos_shifts`` are given."""
    if not ok(A, B):
        raise ValueError("gemm_nt: needs K-contiguous bf16 CUDA operands, K % 64 == 0, 16-B aligned rows")
    M, K = A.shape
    N = B.shape[0]
    if out is None:
        if accumulate:
            raise ValueError("gemm_nt: accumulate needs out")
        out = torch.empty(M, N, dtype=out_dtype, device=A.device)
    if out.stride(1) != 1 or out.dtype not in (torch.float32, torch.bfloat16) or tuple(out.shape) != (M, N):
        raise ValueError("gemm_nt: out must be a row-major M x N f32 / bf16 view")
    epi = 1 if (cos_scales is not None or cos_shifts is not None) else 0
    sc = cos_scales.float().contiguous() if cos_scales is not None else None
    sh = cos_shifts.float().contiguous() if cos_shifts is not None else None
    _lib.call("sl_gemm_nt_bf16", _lib.ptr(A), A.stride(0), _lib.ptr(B), B.stride(0), M, N, K, _lib.ptr(out),
              out.stride(0), _lib.dtype_code(out.dtype), int(bool(accumulate)), epi, float(alpha),
              vp(sc.data_ptr()) if sc is not None else None, vp(sh.data_ptr()) if sh is not None else None,
              vp(_lib.stream_of(A)))
    return out
