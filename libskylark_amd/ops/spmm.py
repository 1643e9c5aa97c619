"""CSR sparse x thin dense products on the GPU (``spmm_kernels.hip``).

``csr_mm(A, X)`` = A X for a CSR tensor A and a thin dense X (row-major);
A^T X runs the same kernel on the CSR of A^T (built once by the caller,
``algorithms/operators.py::SparseOp``).  Reference: ``base/Gemm.hpp:212-494``.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_csr_spmm", [vp, vp, i32, vp, i32, i64, vp, i64, i32, vp, i64, i32, vp])


def _group_for(avg: float) -> int:
    if avg >= 48:
        return 64
    if avg >= 12:
        return 16
    if avg >= 3:
        return 4
    return 1


def ok(A: torch.Tensor, X: torch.Tensor) -> bool:
    return (_lib.available() and A.is_cuda and A.layout == torch.sparse_csr and X.is_cuda and X.dim() == 2
            and A.values().dtype in (torch.float32, torch.float64) and X.shape[0] == A.shape[1]
            and X.shape[1] >= 1)


def csr_mm(A: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    """A X (values dtype) for CSR A on the GPU."""
    vals = A.values()
    vdt = vals.dtype
    rp = A.crow_indices()
    if rp.dtype != torch.int64:
        rp = rp.to(torch.int64)
    ci = A.col_indices()
    idx32 = 1 if ci.dtype == torch.int32 else 0
    if ci.dtype not in (torch.int32, torch.int64):
        ci, idx32 = ci.to(torch.int64), 0
    Xc = X.to(vdt)
    if Xc.stride(1) != 1:
        Xc = Xc.contiguous()
    m = A.shape[0]
    k = X.shape[1]
    Y = torch.empty(m, k, dtype=vdt, device=X.device)
    avg = vals.numel() / max(1, m)
    _lib.call("sl_csr_spmm", _lib.ptr(rp), _lib.ptr(ci), idx32, _lib.ptr(vals.contiguous()), _lib.dtype_code(vdt), m,
              _lib.ptr(Xc), Xc.stride(0), k, _lib.ptr(Y), Y.stride(0), _group_for(avg), vp(_lib.stream_of(X)))
    return Y
