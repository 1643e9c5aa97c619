"""Asynchronous randomized Gauss-Seidel (AsyRGS) and AsyFCG.

Reference: ``algorithms/asynch/AsyRGS.hpp:82-236`` (sweeps of n random
coordinate updates, synchronising every ``syn_sweeps`` sweeps for a residual
test; returns -1 on convergence, -6 otherwise), ``asy_iter_params.hpp``,
``AsyFCG.hpp`` (flexible CG preconditioned by AsyRGS sweeps),
``asynch/precond.hpp``.

GPU: ``sl_asyrgs`` (one wavefront per coordinate update, f64 atomics).  The
coordinate sequence is drawn from the context stream exactly like the
reference (``sweeps * n`` uniform ints per synchronisation); on the CPU the
same sequence is applied sequentially.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from ..base import distributions as D
from ..ops import _lib
from .krylov import KrylovIterParams, Precond, flexible_cg

vp, i32, i64, u64 = C.c_void_p, C.c_int, C.c_int64, C.c_uint64
_lib.register("sl_asyrgs", [vp, vp, i32, vp, i32, i64, vp, vp, i32, u64, u64, i64, vp])
_lib.register("sl_asyrgs_host", [vp, vp, vp, i64, vp, vp, i32, u64, u64, i64])


@dataclass
class AsyIterParams:
    tolerance: float = 1e-3
    syn_sweeps: int = 10
    sweeps_lim: int = 100
    iter_lim: int = 20
    iter_res_print: int = 1
    am_i_printing: bool = False
    log_level: int = 0
    prefix: str = ""


asy_iter_params_t = AsyIterParams


def _csr(A: torch.Tensor):
    if A.layout != torch.sparse_csr:
        A = A.to_sparse_csr() if A.layout != torch.strided else A.to_sparse_csr()
    return A


def _sweep(A: torch.Tensor, Bt: torch.Tensor, Xt: torch.Tensor, seed: int, base: int, nsteps: int):
    n = A.shape[0]
    k = Bt.shape[1]
    rp = A.crow_indices().to(torch.int64).contiguous()
    ci = A.col_indices().contiguous()
    vals = A.values().contiguous()
    if Xt.is_cuda:
        idx32 = 1 if ci.dtype == torch.int32 else 0
        if ci.dtype not in (torch.int32, torch.int64):
            ci, idx32 = ci.to(torch.int64), 0
        if vals.dtype not in (torch.float32, torch.float64):
            vals = vals.double()
        _lib.call("sl_asyrgs", _lib.ptr(rp), _lib.ptr(ci), idx32, _lib.ptr(vals), _lib.dtype_code(vals.dtype), n,
                  _lib.ptr(Bt), _lib.ptr(Xt), k, u64(seed), u64(base), nsteps, vp(_lib.stream_of(Xt)))
    else:
        _lib.call("sl_asyrgs_host", _lib.ptr(rp), _lib.ptr(ci.to(torch.int64).contiguous()),
                  _lib.ptr(vals.double().contiguous()), n, _lib.ptr(Bt), _lib.ptr(Xt), k, u64(seed), u64(base), nsteps)


def asy_rgs(A, B: torch.Tensor, X: torch.Tensor | None = None, context=None,
            params: AsyIterParams | None = None):
    """Solve ``A X = B`` (A sparse SPD, CSR) by asynchronous randomized
    Gauss-Seidel.  Returns ``(X, code)`` (-1 converged, -6 sweep limit)."""
    from .. import default_context
    ctx = context if context is not None else default_context()
    params = params or AsyIterParams()
    A = _csr(A)
    n = A.shape[0]
    vec = B.dim() == 1
    Bt = (B[:, None] if vec else B).to(torch.float64).contiguous()
    k = Bt.shape[1]
    Xt = torch.zeros(n, k, dtype=torch.float64, device=Bt.device) if X is None else \
        (X[:, None] if X.dim() == 1 else X).to(torch.float64).contiguous().clone()
    nrmb = Bt.norm(dim=0)
    left = params.sweeps_lim
    code = -6
    Ad = A.to(torch.float64) if A.values().dtype != torch.float64 else A
    while left > 0:
        sweeps = min(params.syn_sweeps, left) if params.syn_sweeps > 0 else left
        arr = ctx.allocate_random_samples_array(sweeps * n, D.UniformInt(0, n - 1))
        _sweep(A, Bt, Xt, arr.seed, arr.base, sweeps * n)
        left -= sweeps
        if params.tolerance > 0:
            Rr = Bt - torch.sparse.mm(Ad, Xt)
            res = Rr.norm(dim=0)
            if params.am_i_printing and params.log_level >= 2:
                print(f"{params.prefix}AsyRGS: Relres = {float(res.norm() / nrmb.norm()):.2e}")
            if bool((res < params.tolerance * nrmb).all()):
                code = -1
                break
    out = Xt[:, 0] if vec else Xt
    if X is not None:
        X.copy_(out.to(X.dtype))
    return out.to(B.dtype if B.dtype in (torch.float32, torch.float64) else torch.float64), code


AsyRGS = asy_rgs


class AsyRGSPrecond(Precond):
    """``z = M(r)``: ``sweeps_lim`` asynchronous sweeps on ``A z = r`` from z = 0
    (reference ``algorithms/asynch/precond.hpp``) — a variable preconditioner,
    hence used with flexible CG."""

    def __init__(self, A, context, sweeps: int):
        self.A = _csr(A)
        self.ctx = context
        self.sweeps = sweeps

    def apply(self, R):
        n = self.A.shape[0]
        Rt = R.to(torch.float64).contiguous()
        Zt = torch.zeros_like(Rt)
        arr = self.ctx.allocate_random_samples_array(self.sweeps * n, D.UniformInt(0, n - 1))
        _sweep(self.A, Rt, Zt, arr.seed, arr.base, self.sweeps * n)
        return Zt.to(R.dtype)

    apply_adjoint = apply


def asy_fcg(A, B, X=None, context=None, params: AsyIterParams | None = None):
    """Flexible CG preconditioned with AsyRGS sweeps (reference ``AsyFCG.hpp:8-28``)."""
    from .. import default_context
    ctx = context if context is not None else default_context()
    params = params or AsyIterParams()
    A = _csr(A)
    kp = KrylovIterParams(tolerance=params.tolerance, iter_lim=params.iter_lim, res_print=params.iter_res_print,
                          am_i_printing=params.am_i_printing, log_level=params.log_level)
    Bv = B if B.dim() == 2 else B[:, None]
    op_A = A.to(torch.float64) if A.values().dtype != torch.float64 else A
    Xs, code = flexible_cg(op_A, Bv.to(torch.float64), None, kp, AsyRGSPrecond(A, ctx, params.sweeps_lim))
    return (Xs if B.dim() == 2 else Xs[:, 0]), code


AsyFCG = asy_fcg
