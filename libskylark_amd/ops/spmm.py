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
_lib.register("sl_csr_transpose_workspace", [i64, i64], i64)
_lib.register("sl_csr_transpose", [vp, vp, i32, vp, i32, i64, i64, i64, vp, vp, vp, vp, i64, vp])


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


def csr_transpose(A: torch.Tensor) -> torch.Tensor:
    """CSR of A^T (sorted column indices), on A's device: ``csr_transpose.hip``
    (one stable radix sort of (column, position) over the column bits, a
    gather, binary-searched column pointers) on the GPU, torch's COO coalesce
    elsewhere."""
    nnz = A.values().numel()
    if (A.is_cuda and _lib.available() and nnz < (1 << 31) and max(A.shape) < (1 << 31)
            and A.values().dtype in (torch.float32, torch.float64)):
        import ctypes as C
        rp = A.crow_indices().to(torch.int64)
        ci = A.col_indices()
        if ci.dtype not in (torch.int32, torch.int64):
            ci = ci.to(torch.int64)
        vals = A.values().contiguous()
        m, n = A.shape
        ws_bytes = int(_lib.require().sl_csr_transpose_workspace(nnz, n))
        if ws_bytes > 0:
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=A.device)
            colptr = torch.empty(n + 1, dtype=torch.int64, device=A.device)
            orow = torch.empty(nnz, dtype=torch.int32, device=A.device)
            oval = torch.empty(nnz, dtype=vals.dtype, device=A.device)
            _lib.call("sl_csr_transpose", _lib.ptr(rp), _lib.ptr(ci), 1 if ci.dtype == torch.int32 else 0,
                      _lib.ptr(vals), _lib.dtype_code(vals.dtype), m, n, nnz, _lib.ptr(colptr), _lib.ptr(orow),
                      _lib.ptr(oval), _lib.ptr(ws), ws_bytes, C.c_void_p(_lib.stream_of(vals)))
            return torch.sparse_csr_tensor(colptr.to(torch.int32), orow, oval, (n, m))
    coo = A.to_sparse_coo()
    idx = coo.indices()
    return torch.sparse_coo_tensor(idx.flip(0), coo.values(), (A.shape[1], A.shape[0])).coalesce().to_sparse_csr()
