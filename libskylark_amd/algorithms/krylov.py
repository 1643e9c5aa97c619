"""Krylov solvers: block LSQR, block CG, flexible CG, Chebyshev semi-iteration.

Reference: ``algorithms/Krylov/LSQR.hpp:21-255`` (Paige-Saunders LSQR with a
right preconditioner; return codes -2 S1 convergence, -3 S2, -4 ill
conditioning, -5 stagnation, -6 iteration limit), ``CG.hpp:24-163`` (-1
convergence, -6 limit), ``FlexibleCG.hpp``, ``Chebyshev.hpp:18-85``,
``precond.hpp:14-118``, ``krylov_iter_params.hpp:8-29``.

All k right-hand sides advance together; every per-column scalar lives in a
length-k device tensor, so an iteration is a handful of fused element-wise
ops, one ``A Z`` and one ``A^T U`` (+ one all-reduce of n x k when A is
row-distributed) and a host synchronisation only every ``check_every``
iterations (the convergence test).

Normal form (LSQR and Chebyshev, ``KrylovIterParams.fused_normal``): both
methods only ever need ``A^T`` of the NEW long vector, which is a linear
combination of ``A Z`` and vectors whose ``A^T`` image is already known, so the
recurrences are carried in n-space:

* LSQR: ``U' = (A Z - alpha U) / beta``  =>  ``A^T U' = (A^T A Z - alpha A^T U) / beta``;
* Chebyshev: ``R' = R - alpha A PV``     =>  ``A^T R' = A^T R - alpha A^T A PV``;

and ``(A^T A Z, A Z)`` comes from ONE streaming read of A (``ops/normal_eq.py``,
``ata_kernels.hip``), halving the HBM traffic of an iteration (A is read
twice per iteration in the reference, ``LSQR.hpp:113-248``,
``Chebyshev.hpp:18-85``).  The carried ``A^T U`` is replaced by the exact
product every ``refresh_every`` iterations to bound the drift.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from ..ops import krylov_native as _kn
from .operators import Operator, as_operator


@dataclass
class KrylovIterParams:
    tolerance: float = 1e-14
    iter_lim: int = 100
    res_print: int = 10
    am_i_printing: bool = False
    log_level: int = 0
    prefix: str = ""
    check_every: int = 1     # convergence test every N iterations (host sync)
    # normal-form iteration: one fused ``A^T (A Z)`` pass per iteration instead
    # of ``A Z`` then ``A^T U`` (None = when the operator has the kernel); the
    # n-space recurrence for A^T U is recomputed exactly every ``refresh_every``
    # iterations (0 = never; None = 16 for LSQR, whose recurrence divides by
    # beta, and never for Chebyshev, where a refresh costs two passes)
    fused_normal: bool | None = None
    refresh_every: int | None = None


krylov_iter_params_t = KrylovIterParams


# ------------------------------------------------------------ preconditioners
class Precond:
    """In-place/out-of-place preconditioner P: ``apply(X) = P X``, ``apply_adjoint(X) = P^T X``."""

    is_id = False

    def apply(self, X):
        raise NotImplementedError

    def apply_adjoint(self, X):
        raise NotImplementedError


class IdPrecond(Precond):
    is_id = True

    def apply(self, X):
        return X

    def apply_adjoint(self, X):
        return X


class MatPrecond(Precond):
    """``P X = N X`` for an explicit (replicated) matrix N (reference mat_precond_t)."""

    def __init__(self, N: torch.Tensor):
        self.N = N
        self._cast = {}

    def _get(self, dtype, t):
        # cast (and transposed copy) made once per dtype: a transposed GEMV
        # operand made hipBLASLt pick a ~20x slower kernel
        key = (dtype, t)
        if key not in self._cast:
            M = self.N.to(dtype)
            self._cast[key] = M.t().contiguous() if t else M
        return self._cast[key]

    def apply(self, X):
        return _thin(self._get(X.dtype, False), X)

    def apply_adjoint(self, X):
        return _thin(self._get(X.dtype, True), X)


class TriInversePrecond(Precond):
    """``P X = R^{-1} X`` for triangular R (reference tri_inverse_precond_t).

    With ``Rinv`` given (the explicit inverse, formed once) every application
    is a GEMV/GEMM instead of a triangular solve: on the MI355X a 5000 x 5000
    ``trsv`` is latency bound at ~1.9 ms per call, the GEMV streams R^{-1} in
    ~40 us, and a Krylov loop applies the preconditioner twice per iteration."""

    def __init__(self, R: torch.Tensor, upper: bool = True, Rinv: torch.Tensor | None = None):
        self.R = R
        self.upper = upper
        self.Rinv = Rinv
        self._cast = {}

    def _inv(self, dtype, t=False):
        # cast and transposed copy made once per dtype (a transposed GEMV
        # operand made hipBLASLt pick a ~20x slower kernel: 318 us vs 15 us)
        key = (dtype, t)
        if key not in self._cast:
            M = self.Rinv.to(dtype)
            self._cast[key] = M.t().contiguous() if t else M
        return self._cast[key]

    def apply(self, X):
        if self.Rinv is not None:
            return _thin(self._inv(X.dtype), X)
        return torch.linalg.solve_triangular(self.R.to(X.dtype), X, upper=self.upper)

    def apply_adjoint(self, X):
        if self.Rinv is not None:
            return _thin(self._inv(X.dtype, True), X)
        return torch.linalg.solve_triangular(self.R.to(X.dtype).t(), X, upper=not self.upper)


def _thin(M, X):
    """M @ X; a thin right-hand side (<= 8 columns) on the GPU goes through the
    one-wave-per-row kernel (``sl_rows_gemm``)."""
    if X.dim() == 2 and _kn.thin_gemm_ok(M, X):
        return _kn.thin_gemm(M, X)
    return M @ X


class CallablePrecond(Precond):
    def __init__(self, f, ft=None):
        self.f, self.ft = f, ft or f

    def apply(self, X):
        return self.f(X)

    def apply_adjoint(self, X):
        return self.ft(X)


def _eps(dtype):
    return 32 * torch.finfo(dtype).eps


def _clamp_tol(tol, dtype):
    eps = _eps(dtype)
    if tol < eps:
        return eps
    if tol >= 1.0:
        return 1 - eps
    return tol


def _log(params, msg):
    if params.am_i_printing:
        print(f"{params.prefix}{msg}")


# -------------------------------------------------------------------- LSQR
def lsqr(A, B, X=None, params: KrylovIterParams | None = None, R: Precond | None = None):
    """Solve ``min ||A X - B||_F`` column by column (block LSQR).

    Returns ``(X, code)`` with the reference's codes (-2/-3 converged,
    -4 ill-conditioned, -5 stagnation, -6 iteration limit).
    """
    op: Operator = as_operator(A)
    params = params or KrylovIterParams()
    R = R or IdPrecond()
    m, n = op.shape
    dt = op.dtype if op.dtype in (torch.float32, torch.float64) else torch.float32
    dev = op.device
    U = op.long_like(B).to(dt).clone()
    if U.dim() == 1:
        U = U[:, None]
    k = U.shape[1]
    tol = _clamp_tol(params.tolerance, dt)
    eps = _eps(dt)
    iter_lim = params.iter_lim if params.iter_lim >= 0 else max(20, 2 * min(m, n))
    X = torch.zeros(n, k, dtype=dt, device=dev) if X is None else X.to(dt)

    fused = params.fused_normal
    if fused is None:
        # the n-space recurrence T = (G - alpha T) / beta scales its error by
        # alpha / beta every step: only on by default for a preconditioned
        # (well-conditioned) system, where that ratio stays near one
        fused = op.has_fused_normal(k) and not isinstance(R, IdPrecond)
    refresh = 16 if params.refresh_every is None else max(0, int(params.refresh_every))
    beta = op.long_colnorm(U)
    U = U / beta.clamp_min(torch.finfo(dt).tiny)
    T = op.rmatmul(U).to(dt)       # A^T U (carried in n-space in normal form)
    V = R.apply_adjoint(T)
    alpha = op.short_colnorm(V)
    V = V / alpha.clamp_min(torch.finfo(dt).tiny)
    Z = R.apply(V.clone())
    W = Z.clone()
    nrm_a = torch.zeros(k, dtype=dt, device=dev)
    cnd_a = torch.zeros_like(nrm_a)
    sq_d = torch.zeros_like(nrm_a)
    nrm_r = beta.clone()
    nrm_x = torch.zeros_like(nrm_a)
    sq_x = torch.zeros_like(nrm_a)
    nrm_ar_0 = alpha * beta
    phibar = beta.clone()
    rhobar = alpha.clone()
    cs2 = -torch.ones_like(nrm_a)
    sn2 = torch.zeros_like(nrm_a)
    zz = torch.zeros_like(nrm_a)
    stag = torch.zeros(k, dtype=torch.int32, device=dev)
    max_n_stag = 3
    if bool((nrm_ar_0 == 0).all()):
        return X, -1
    code = -6
    if _kn.ok(U, V) and n > 0:
        return _lsqr_native(op, params, R, U, V, X, alpha, beta, fused, refresh, T, tol, eps, iter_lim, max_n_stag)
    code = -6
    for itn in range(iter_lim):
        # 1. U = A Z - alpha U, beta = |U|
        if fused:
            G, AZ = op.normal(Z, want_y=True)
            U = AZ.to(dt) - alpha * U
        else:
            U = op.matmul(Z).to(dt) - alpha * U
        beta = op.long_colnorm(U)
        U = U / beta
        # 2. norm(A) estimate
        nrm_a = torch.sqrt(nrm_a * nrm_a + alpha * alpha + beta * beta)
        # 3. V = P^T A^T U - beta V
        if not fused or (refresh and (itn + 1) % refresh == 0):
            T = op.rmatmul(U).to(dt)
        else:
            T = (G.to(dt) - alpha * T) / beta
        V = R.apply_adjoint(T) - beta * V
        alpha = op.short_colnorm(V)
        V = V / alpha
        Z = R.apply(V.clone())
        # 4. Givens rotation
        rho = torch.sqrt(rhobar * rhobar + beta * beta)
        cs = rhobar / rho
        sn = beta / rho
        theta = sn * alpha
        rhobar = -cs * alpha
        phi = cs * phibar
        phibar = sn * phibar
        # 5. X, W updates
        X = X + (phi / rho) * W
        W = Z - (theta / rho) * W
        # 6-7. residual estimates
        nrm_r = phibar
        nrm_ar = torch.abs(phibar * alpha * cs)
        s1 = nrm_ar < tol * nrm_ar_0
        s2 = nrm_ar < eps * nrm_a * nrm_r
        # 9. condition estimate
        nrm_w = op.short_colnorm(W)
        sq_d = sq_d + (nrm_w * nrm_w) / (rho * rho)
        cnd_a = nrm_a * torch.sqrt(sq_d)
        s3 = cnd_a > 1.0 / eps
        # 11. stagnation
        stagnating = torch.abs(phi / rho) * nrm_w < eps * nrm_x
        stag = torch.where(stagnating, stag + 1, torch.zeros_like(stag))
        s5 = stag >= max_n_stag
        # 12. norm(X) estimate
        delta = sn2 * rho
        gambar = -cs2 * rho
        rhs = phi - delta * zz
        zbar = rhs / gambar
        nrm_x = torch.sqrt(sq_x + zbar * zbar)
        gamma = torch.sqrt(gambar * gambar + theta * theta)
        cs2 = gambar / gamma
        sn2 = theta / gamma
        zz = rhs / gamma
        sq_x = sq_x + zz * zz
        if (itn + 1) % params.check_every == 0 or itn == iter_lim - 1:
            flags = torch.stack([s1.all(), s2.all(), s3.any(), s5.any()]).tolist()
            if params.log_level >= 2 and itn % max(1, params.res_print) == 0:
                _log(params, f"LSQR: Iteration {itn}: {nrm_ar.max().item():.3e}")
            if flags[0]:
                _log(params, "LSQR: Convergence (S1)!")
                code = -2
                break
            if flags[1]:
                _log(params, "LSQR: Convergence (S2)!")
                code = -3
                break
            if flags[2]:
                _log(params, "LSQR: Stopping (S3)!")
                code = -4
                break
            if flags[3]:
                _log(params, "LSQR: Stagnation.")
                code = -5
                break
    else:
        _log(params, "LSQR: No convergence within iteration limit.")
    return X, code


def _lsqr_native(op, params, R, U, V, X, alpha, beta, fused, refresh, T, tol, eps, iter_lim, max_n_stag):
    """GPU LSQR with device-resident scalars: per iteration the operator
    product(s), one fused ``U = A Z - alpha U`` + |U| pass, the preconditioner,
    one fused ``V = P^T A^T U - beta V`` + |V| pass, and LSQR steps 4-12 in two
    launches (``sl_lsqr_step``); the stop flags are read every
    ``params.check_every`` iterations."""
    k = U.shape[1]
    dt = U.dtype
    st = _kn.lsqr_state(k, U.device)
    a64, b64 = alpha.to(torch.float64), beta.to(torch.float64)
    st[_kn.S_ALPHA], st[_kn.S_BETA] = a64, b64
    st[_kn.S_RHOBAR], st[_kn.S_PHIBAR] = a64, b64
    st[_kn.S_NRMAR0] = a64 * b64
    st[_kn.S_CS2] = -1.0
    flags = torch.zeros(k, dtype=torch.int32, device=U.device)
    U = U.contiguous()
    V = V.contiguous()
    Z = R.apply(V.clone()).to(dt).contiguous()
    W = Z.clone()
    X = X.to(dt).contiguous()
    sA, sB = st[_kn.S_ALPHA], st[_kn.S_BETA]
    T = T.to(dt).contiguous()
    code = -6
    for itn in range(iter_lim):
        # 1-2. U = (A Z - alpha U) / beta, beta = |U|, |A| estimate (old alpha, new beta)
        if fused:
            G, AZ = op.normal(Z, want_y=True)
        else:
            AZ = op.matmul(Z)
        if op.distributed:
            sums = _kn.axpby(AZ, U, b=sA, sb=-1.0, red=1)
            op.comm.all_reduce(sums)
            _kn.setstate(sums, st, 1)
        else:
            _kn.axpby(AZ, U, b=sA, sb=-1.0, red=2, st=st)
        _kn.colscale(U, sB, inv=True)
        # 3. V = (P^T A^T U - beta V) / alpha
        if not fused or (refresh and (itn + 1) % refresh == 0):
            T = op.rmatmul(U).to(dt).contiguous()
        else:
            _kn.axpby(G, T, b=sA, sb=-1.0, d=sB)           # T = (G - alpha T) / beta
        PT = R.apply_adjoint(T)
        _kn.axpby(PT, V, b=sB, sb=-1.0, red=3, st=st)
        _kn.colscale(V, sA, inv=True)
        Z = V.clone() if R.is_id else R.apply(V).to(dt).contiguous()
        # 4-12. Givens, X / W updates, |W|, estimates, stop flags
        _kn.lsqr_step(X, W, Z, st, flags, tol, eps, max_n_stag)
        if (itn + 1) % params.check_every == 0 or itn == iter_lim - 1:
            f = flags.cpu()
            if params.log_level >= 2 and itn % max(1, params.res_print) == 0:
                _log(params, f"LSQR: Iteration {itn}: {st[_kn.S_NRMAR].max().item():.3e}")
            if bool(((f & 1) != 0).all()):
                _log(params, "LSQR: Convergence (S1)!")
                code = -2
                break
            if bool(((f & 2) != 0).all()):
                _log(params, "LSQR: Convergence (S2)!")
                code = -3
                break
            if bool(((f & 4) != 0).any()):
                _log(params, "LSQR: Stopping (S3)!")
                code = -4
                break
            if bool(((f & 8) != 0).any()):
                _log(params, "LSQR: Stagnation.")
                code = -5
                break
    else:
        _log(params, "LSQR: No convergence within iteration limit.")
    return X, code


def LSQR(A, B, X, params=None, R=None) -> int:
    """Reference-style in-place interface: X is overwritten, the code returned."""
    Xs, code = lsqr(A, B, None, params, R)
    X.copy_(Xs.to(X.dtype))
    return code


# ---------------------------------------------------------------------- CG
def cg(A, B, X=None, params: KrylovIterParams | None = None, M: Precond | None = None, uplo: str = "L"):
    """Preconditioned block CG for SPD ``A`` (n x n).  Returns ``(X, code)``:
    -1 converged, -6 iteration limit (reference ``CG.hpp``)."""
    op = as_operator(A)
    params = params or KrylovIterParams()
    M = M or IdPrecond()
    dt = op.dtype if op.dtype in (torch.float32, torch.float64) else torch.float32
    Bv = op.long_like(B).to(dt)
    if Bv.dim() == 1:
        Bv = Bv[:, None]
    k = Bv.shape[1]
    tol = _clamp_tol(params.tolerance, dt)
    # X lives where B does (row-distributed for a DistSymOp)
    X = torch.zeros_like(Bv) if X is None else op.long_like(X).to(dt).clone()
    Rr = Bv - op.matmul(X).to(dt)
    if _kn.ok(Bv) and not op.distributed:
        return _cg_native(op, Bv, X, Rr, params, M, tol, flexible=False)
    nrmb = op.long_colnorm(Bv)
    ressqr = op.long_coldot(Rr, Rr)
    P = torch.zeros_like(Rr)
    rho0 = None
    code = -6
    for itn in range(params.iter_lim):
        if not M.is_id:
            Z = M.apply(Rr)
            rho = op.long_coldot(Rr, Z)
        else:
            Z = Rr
            rho = ressqr
        beta = torch.zeros_like(rho) if rho0 is None else rho / rho0
        P = beta * P + Z
        Q = op.matmul(P).to(dt)
        alpha = rho / op.long_coldot(P, Q)
        X = X + alpha * P
        Rr = Rr - alpha * Q
        rho0 = rho
        ressqr = op.long_coldot(Rr, Rr)
        if (itn + 1) % params.check_every == 0:
            conv = int((ressqr.sqrt() < tol * nrmb).sum())
            if params.log_level >= 2 and itn % max(1, params.res_print) == 0:
                relres = float(ressqr.sum().sqrt() / nrmb.pow(2).sum().sqrt())
                _log(params, f"CG: Iteration {itn}, Relres = {relres:.2e}, {conv} rhs converged")
            if conv == k:
                _log(params, "CG: Convergence!")
                code = -1
                break
    else:
        _log(params, "CG: No convergence within iteration limit.")
    params.iterations = itn + 1 if params.iter_lim > 0 else 0   # iterations run (reporting)
    return X, code


def _cg_native(op, Bv, X, Rr, params, M, tol, flexible: bool):
    """Single-GPU (flexible) CG with device-resident scalars
    (``krylov_kernels.hip``: every column reduction finished by its pass's last
    block).  Per iteration, besides ``A P`` and the preconditioner:
    CG 3 launches (``P = R + beta P``; ``P.Q`` -> alpha; ``X += alpha P``,
    ``R -= alpha Q``, ``|R|`` -> rho, beta, flags), 4 with a preconditioner
    (``R.Z`` -> rho, beta first); flexible CG 4 (``Q_prev.Z`` -> beta,
    ``P = Z - beta P``, ``P.Q`` and ``P.R`` -> alpha, the X / R update).  The
    stop flags reach the host every ``check_every`` iterations."""
    k = Bv.shape[1]
    dt = Bv.dtype
    cs = _kn.CGState(k, Bv.device)
    X = X.contiguous()
    R = Rr.contiguous()
    cs.st[_kn.C_NRMB] = _kn.colsumsq(Bv).sqrt()
    idp = M.is_id and not flexible
    if idp:
        cs.st[_kn.C_RHO] = _kn.colsumsq(R)
    P = torch.zeros_like(R)
    Q = None
    name = "FlexibleCG" if flexible else "CG"
    code = -6
    for itn in range(params.iter_lim):
        if flexible:
            Z = M.apply(R).to(dt)
            if itn == 0:
                P.copy_(Z)
            else:
                _kn.cg_dot(Q, Z, 2, cs)          # beta = Q_prev . Z / pq_prev
                _kn.cg_p(Z, P, cs, -1.0)         # P = Z - beta P
        elif idp:
            _kn.cg_p(R, P, cs)                   # P = R + beta P
        else:
            Z = M.apply(R).to(dt)
            _kn.cg_dot(R, Z, 1, cs)              # rho, beta
            _kn.cg_p(Z, P, cs)
        Q = op.matmul(P).to(dt)
        if Q.stride(1) != 1:
            Q = Q.contiguous()
        if flexible:
            _kn.cg_dot(P, Q, 3, cs, Y2=R)        # pq, alpha = P.R / pq
        else:
            _kn.cg_dot(P, Q, 0, cs)              # alpha = rho / P.Q
        _kn.cg_xr(X, P, R, Q, cs, idp, tol)
        if (itn + 1) % params.check_every == 0 or itn == params.iter_lim - 1:
            conv = int(cs.flags.sum())
            if params.log_level >= 2 and itn % max(1, params.res_print) == 0:
                relres = float(cs.st[_kn.C_RR].sum().sqrt() / cs.st[_kn.C_NRMB].pow(2).sum().sqrt())
                _log(params, f"{name}: Iteration {itn}, Relres = {relres:.2e}, {conv} rhs converged")
            if conv == k:
                _log(params, f"{name}: Convergence!")
                code = -1
                break
    else:
        _log(params, f"{name}: No convergence within iteration limit.")
    params.iterations = itn + 1 if params.iter_lim > 0 else 0   # iterations run (reporting)
    return X, code


def CG(uplo, A, B, X, params=None, M=None) -> int:
    Xs, code = cg(A, B, None, params, M, uplo)
    X.copy_(Xs.to(X.dtype))
    return code


def flexible_cg(A, B, X=None, params: KrylovIterParams | None = None, M: Precond | None = None):
    """Flexible CG (Notay): tolerates a variable preconditioner (e.g. AsyRGS sweeps).
    Reference ``algorithms/Krylov/FlexibleCG.hpp:23-153``.  Returns ``(X, code)``."""
    op = as_operator(A)
    params = params or KrylovIterParams()
    M = M or IdPrecond()
    dt = op.dtype if op.dtype in (torch.float32, torch.float64) else torch.float32
    Bv = op.long_like(B).to(dt)
    if Bv.dim() == 1:
        Bv = Bv[:, None]
    k = Bv.shape[1]
    n = op.shape[0]
    tol = _clamp_tol(params.tolerance, dt)
    X = torch.zeros(n, k, dtype=dt, device=Bv.device) if X is None else X.to(dt).clone()
    Rr = Bv - op.matmul(X).to(dt)
    if _kn.ok(Bv) and not op.distributed:
        return _cg_native(op, Bv, X, Rr, params, M, tol, flexible=True)
    nrmb = op.long_colnorm(Bv)
    Ps, Qs, PQs = [], [], []
    code = -6
    for itn in range(params.iter_lim):
        Z = M.apply(Rr)
        P = Z.clone()
        # orthogonalise against the previous direction (truncation m_max = 1, as the reference)
        if Ps:
            beta = op.long_coldot(Qs[-1], Z) / PQs[-1]
            P = P - beta * Ps[-1]
        Q = op.matmul(P).to(dt)
        pq = op.long_coldot(P, Q)
        alpha = op.long_coldot(P, Rr) / pq
        X = X + alpha * P
        Rr = Rr - alpha * Q
        Ps, Qs, PQs = [P], [Q], [pq]
        if (itn + 1) % params.check_every == 0:
            nrmr = op.long_colnorm(Rr)
            conv = int((nrmr < tol * nrmb).sum())
            if conv == k:
                _log(params, "FlexibleCG: Convergence!")
                code = -1
                break
    return X, code


def chebyshev_ls(A, B, sigma_L: float, sigma_U: float, params: KrylovIterParams | None = None,
                 P: Precond | None = None):
    """Chebyshev semi-iteration for least squares given singular value bounds of
    ``A P`` (LSRN).  Reference ``algorithms/Krylov/Chebyshev.hpp:18-85``.
    No inner products: one ``A^T R`` and one ``A V`` per iteration, or one
    fused ``A^T A PV`` in normal form (the exact ``A^T (B - A X)`` is re-formed
    every ``params.refresh_every`` iterations, two passes)."""
    op = as_operator(A)
    params = params or KrylovIterParams()
    P = P or IdPrecond()
    dt = op.dtype if op.dtype in (torch.float32, torch.float64) else torch.float32
    Rr = op.long_like(B).to(dt).clone()
    if Rr.dim() == 1:
        Rr = Rr[:, None]
    k = Rr.shape[1]
    n = op.shape[1]
    tol = _clamp_tol(params.tolerance, dt)
    its = (math.log(tol) - math.log(2)) / math.log((sigma_U - sigma_L) / (sigma_U + sigma_L)) + 1
    d = (sigma_U * sigma_U + sigma_L * sigma_L) / 2
    c = (sigma_U * sigma_U - sigma_L * sigma_L) / 2
    X = torch.zeros(n, k, dtype=dt, device=Rr.device)
    V = None  # search direction in the preconditioned (y = P^{-1} x) space
    fused = params.fused_normal
    if fused is None:
        fused = op.has_fused_normal(k)
    refresh = 0 if params.refresh_every is None else max(0, int(params.refresh_every))
    T = op.rmatmul(Rr).to(dt) if fused else None     # A^T R carried in n-space
    B0 = Rr if fused and refresh else None
    alpha = beta = 0.0
    i = 0
    while i < its:
        if i == 0:
            beta, alpha = 0.0, 1.0 / d
        elif i == 1:
            beta = (c * c) / (d * d * 2)
            alpha = 1 / (d - c * c / (2 * d))
        else:
            beta = alpha * alpha * c * c / 4.0
            alpha = 1 / (d - alpha * c * c / 4.0)
        if fused:
            if refresh and i > 0 and i % refresh == 0:
                T = op.rmatmul(B0 - op.matmul(X).to(dt)).to(dt)
            AR = P.apply_adjoint(T)
        else:
            AR = P.apply_adjoint(op.rmatmul(Rr).to(dt))
        V = AR if V is None else beta * V + AR
        PV = P.apply(V)
        X = X + alpha * PV
        if fused:
            T = T - alpha * op.normal(PV)[0].to(dt)
        else:
            Rr = Rr - alpha * op.matmul(PV).to(dt)
        i += 1
    return X


ChebyshevLS = chebyshev_ls
FlexibleCG = flexible_cg
