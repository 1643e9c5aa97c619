"""GPU-resident small dense linear algebra (k <= 64) for iteration loops.

CholeskyQR2 of replicated n x k iterates and Cholesky/inverse of k x k Grams
without any host synchronisation: Grams and products via the MFMA kernels
of ``tsk_f32_kernels.hip``, the k x k factorisation by one workgroup
(``small_la.hip``).  Failures are flagged in a device status word that the
caller checks once, at the end.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from . import tallskinny as T

vp, i32 = C.c_void_p, C.c_int
_lib.register("sl_small_chol_inv", [vp, i32, i32, vp, vp, vp, vp, vp])
_lib.register("sl_small_matmul", [vp, vp, vp, i32, i32, i32, vp, vp])
_lib.register("sl_sym_eig_topr", [vp, i32, i32, i32, vp, i32, i32, vp, vp])


def sym_eig_topr(C: torch.Tensor, r: int, out: torch.Tensor | None = None, sqrt: bool = False,
                 max_sweeps: int = 30, sweeps: torch.Tensor | None = None):
    """Top-``r`` eigenpairs (descending) of a symmetric k x k (k <= 64) matrix
    by device Jacobi: returns ``out`` (f64, k*r + r) = [V_r row-major, lambda_r]
    (``sqrt(max(lambda, 0))`` with ``sqrt``), all on C's device, no host sync."""
    k = C.shape[0]
    C = C.to(torch.float64).contiguous()
    if out is None:
        out = torch.empty(k * r + r, dtype=torch.float64, device=C.device)
    _lib.call("sl_sym_eig_topr", _lib.ptr(C), k, k, r, _lib.ptr(out), int(bool(sqrt)), int(max_sweeps),
              _lib.ptr(sweeps) if sweeps is not None else None, vp(_lib.stream_of(C)))
    return out


_lib.register("sl_sym_eig_tridiag", [vp, i32, i32, i32, vp, i32, vp, vp])


def sym_eig_tridiag(C: torch.Tensor, r: int, out: torch.Tensor | None = None, sqrt: bool = False,
                    status: torch.Tensor | None = None, ldc: int | None = None):
    """Top-``r`` eigenpairs (descending) of a symmetric k x k matrix (k <= 64,
    r <= k) in one launch: Householder tridiagonalisation on one wave,
    multisection on division-free Sturm counts, twisted-factorisation
    eigenvectors, back-transform (``sym_eig.hip`` on ``sl_wave_la.hpp``).  Output packed as :func:`sym_eig_topr`; ``status`` (int32)
    gets bit 1 when the result must be recomputed on the host (near-repeated
    eigenvalues, non-finite data or a vanishing r-th eigenvalue).  ``C`` may be
    any f64 device buffer holding the matrix with row stride ``ldc``."""
    k = int(C.shape[0]) if ldc is None else int(ldc)
    if ldc is None:
        C = C.to(torch.float64).contiguous()
    if out is None:
        out = torch.empty(k * r + r, dtype=torch.float64, device=C.device)
    _lib.call("sl_sym_eig_tridiag", _lib.ptr(C), k, k, r, _lib.ptr(out), int(bool(sqrt)),
              _lib.ptr(status) if status is not None else None, vp(_lib.stream_of(C)))
    return out


_lib.register("sl_chol_inv_wave", [vp, i32, i32, vp, vp, vp])


def chol_inv_wave(G: torch.Tensor, status: torch.Tensor | None = None) -> torch.Tensor:
    """R^{-1} (upper, f64) of G = R^T R (k <= 128) by the register
    kernel the randSVD boundaries use; dropped pivots (<= 1e-13 max G_ii) give
    zero rows / columns and set status bit 1."""
    k = G.shape[0]
    G = G.to(torch.float64).contiguous()
    X = torch.empty(k, k, dtype=torch.float64, device=G.device)
    _lib.call("sl_chol_inv_wave", _lib.ptr(G), k, k, _lib.ptr(X), _lib.ptr(status) if status is not None else None,
              vp(_lib.stream_of(G)))
    return X


def chol_inv(G: torch.Tensor, status: torch.Tensor | None = None):
    """R (upper, G = R^T R), R^{-1} (f64) and R^{-1} as f32, all on G's device."""
    k = G.shape[0]
    G = G.to(torch.float64).contiguous()
    R = torch.empty(k, k, dtype=torch.float64, device=G.device)
    Ri = torch.empty_like(R)
    Ri32 = torch.empty(k, k, dtype=torch.float32, device=G.device)
    _lib.call("sl_small_chol_inv", _lib.ptr(G), k, k, _lib.ptr(R), _lib.ptr(Ri), _lib.ptr(Ri32),
              _lib.ptr(status) if status is not None else None, vp(_lib.stream_of(G)))
    return R, Ri, Ri32


def small_matmul(A: torch.Tensor, B: torch.Tensor, want32: bool = False):
    A = A.to(torch.float64).contiguous()
    B = B.to(torch.float64).contiguous()
    m, kk = A.shape
    n = B.shape[1]
    Cm = torch.empty(m, n, dtype=torch.float64, device=A.device)
    C32 = torch.empty(m, n, dtype=torch.float32, device=A.device) if want32 else None
    _lib.call("sl_small_matmul", _lib.ptr(A), _lib.ptr(B), _lib.ptr(Cm), m, kk, n,
              _lib.ptr(C32) if C32 is not None else None, vp(_lib.stream_of(A)))
    return (Cm, C32) if want32 else Cm


def cholqr(W: torch.Tensor, status: torch.Tensor | None = None, ws: torch.Tensor | None = None,
           zt_out: torch.Tensor | None = None):
    """One CholeskyQR step (basis of the column space, orthonormal to ~eps*cond(W)):
    enough to re-condition an intermediate power-iteration block.  With
    ``zt_out`` (bf16 k x n) Q is written there transposed, in the fused pass's
    operand layout, and returned in that form."""
    W = W.float().contiguous()
    _, G1 = T.f32_xm(W, None, store=False, gram=True, ws=ws)
    _, _, R1i = chol_inv(G1, status)
    if zt_out is not None:
        return T.f32_xm_bf16t(W, R1i, zt_out)
    Q, _ = T.f32_xm(W, R1i, store=True)
    return Q


def cholqr2(W: torch.Tensor, status: torch.Tensor | None = None, want_r: bool = False):
    """Orthonormal basis of the columns of a replicated f32 n x k matrix (CholeskyQR2).

    With ``want_r`` also returns the f64 triangular factor ``R = R2 R1``
    (``W = Q R``)."""
    W = W.float().contiguous()
    _, G1 = T.f32_xm(W, None, store=False, gram=True)
    R1, _, R1i = chol_inv(G1, status)
    Q1, G2 = T.f32_xm(W, R1i, store=True, gram=True)
    R2, _, R2i = chol_inv(G2, status)
    Q, _ = T.f32_xm(Q1, R2i, store=True)
    if want_r:
        return Q, small_matmul(R2, R1)
    return Q
