"""Condition-number estimation with certificates (Avron, Druinsky, Toledo).

Reference ``nla/CondEst.hpp:17-302``: ``powerits`` (300) power iterations
for sigma_max with left/right certificate vectors; an LSQR run on
``A x = A xhat`` (xhat Gaussian) tracking the forward error ``d = xhat - x``,
whose Rayleigh quotient ``|A d| / |d|`` certifies sigma_min; stopping tests
C1 (residual), C2 (forward error below tau), C3 (singular), C4 (adjust c1);
finally the singular values of the Lanczos bidiagonal R (LAPACK ``dbdsqr``
there, ``scipy.linalg.svdvals`` of the bidiagonal here) give a second
sigma_min estimate.  Return codes: -1 cond = 1, -2 C1, -3 C2, -4 C3, -6 limit.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from ..algorithms.operators import as_operator
from ..base import distributions as D
from ..base.context import Context
from ..ops import rng


def _erfinv(x):
    from scipy.special import erfinv
    return float(erfinv(x))


_EM = float(np.finfo(np.float64).eps)


@dataclass
class CondEstParams:
    iter_lim: int = 1000
    powerits: int = 300
    c1: float = 8 * _EM
    c2: float = 1e-3
    c3: float = 64.0 / _EM
    c4: float = math.sqrt(_EM)
    c1t: float = 4 * _EM
    am_i_printing: bool = False
    log_level: int = 0
    prefix: str = ""


condest_params_t = CondEstParams


@dataclass
class CondEstResult:
    cond: float
    sigma_max: float
    v_max: torch.Tensor
    u_max: torch.Tensor
    sigma_min: float
    sigma_min_c: float
    v_min: torch.Tensor
    u_min: torch.Tensor
    code: int = -6


def _gauss(n, ctx, dtype, device):
    arr = ctx.allocate_random_samples_array(n, D.Normal())
    out = torch.empty(n, 1, dtype=dtype, device=device)
    rng.fill_random(out, D.Normal(), arr.seed, arr.base, ir=1, ic=n, precise=True)
    return out


def condest(A, context: Context | None = None, params: CondEstParams | None = None,
            check_every: int = 8) -> CondEstResult:
    """Device-resident: every scalar of the recurrences is a 0-d device tensor
    and the stopping tests are read back once per ``check_every`` iterations
    (the state of the iteration the reference would stop at is restored from a
    short per-iteration history, so the result does not depend on
    ``check_every``).  With a one-pass normal kernel for A (f32 dense,
    ``ops/normal_eq.py``) the power iterations read A once each and the Lanczos
    step does ``(A^T A v, A v)`` in one pass plus the ``A d`` certificate
    product: two reads of A per iteration instead of three."""
    from .. import default_context
    ctx = context if context is not None else default_context()
    p = params or CondEstParams()
    op = as_operator(A)
    m, n = op.shape
    dt = torch.float64
    dev = op.device
    fused = op.has_fused_normal(1)

    def Av(x):
        return op.matmul(x.to(op.dtype)).to(dt)

    def Atv(u):
        return op.rmatmul(u.to(op.dtype)).to(dt)

    def lnorm(u):
        return op.long_colnorm(u)[0]

    # --- sigma_max by power iteration (normalised every step, no host sync)
    v_max = _gauss(n, ctx, dt, dev)
    v_max = v_max / v_max.norm()
    for _ in range(p.powerits):
        v_max = op.normal(v_max.to(op.dtype))[0].to(dt) if fused else Atv(Av(v_max))
        v_max = v_max / v_max.norm()
    u_max = Av(v_max)
    sigma_max_t = lnorm(u_max)
    u_max = u_max / sigma_max_t
    sigma_max = float(sigma_max_t)

    xhat = _gauss(n, ctx, dt, dev)
    nrm_xhat = float(xhat.norm())
    tau = math.sqrt(2) * _erfinv(p.c2) / nrm_xhat
    xhat = xhat / nrm_xhat
    b = Av(xhat)
    nrm_b = lnorm(b)
    beta = nrm_b
    u = b / beta
    Atu = Atv(u)
    alpha = Atu.norm()
    v = Atu / alpha
    x = torch.zeros(n, 1, dtype=dt, device=dev)
    w = v.clone()
    phibar, rhobar = beta, alpha
    T = p.iter_lim if p.iter_lim >= 0 else max(20, 2 * min(m, n))
    Tlim = T
    Rdiag, Rsub = [], []
    c1 = torch.tensor(p.c1, dtype=dt, device=dev)
    c1t = torch.tensor(p.c1t, dtype=dt, device=dev)
    sig_min = sigma_max_t.clone()
    u_min, v_min = u_max.clone(), v_max.clone()
    retval = -6
    theta = None
    itn = 0
    hist, flags = [], []          # per-iteration (sig_min, v_min, u_min) / stopping flags since the last check
    refresh = 16
    while itn < T:
        if fused:
            G, AvV = op.normal(v.to(op.dtype), want_y=True)
            u = AvV.to(dt) - alpha * u
            beta = lnorm(u)
            u = u / beta
            Atu = Atv(u) if (itn + 1) % refresh == 0 else (G.to(dt) - alpha * Atu) / beta
        else:
            u = Av(v) - alpha * u
            beta = lnorm(u)
            u = u / beta
            Atu = Atv(u)
        v = Atu - beta * v
        alpha = v.norm()
        v = v / alpha
        rho = torch.sqrt(rhobar * rhobar + beta * beta)
        Rdiag.append(rho)
        if itn > 0:
            Rsub.append(theta)
        cs, sn = rhobar / rho, beta / rho
        theta = sn * alpha
        rhobar = -cs * alpha
        phi = cs * phibar
        phibar = sn * phibar
        x = x + (phi / rho) * w
        w = v - (theta / rho) * w
        d = xhat - x
        nrm_d = d.norm()
        Ad = Av(d)
        nrm_ad = lnorm(Ad)
        better = nrm_ad <= sig_min * nrm_d
        sig_min = torch.where(better, nrm_ad / nrm_d, sig_min)
        v_min = torch.where(better, d, v_min)
        u_min = torch.where(better, Ad / nrm_ad, u_min)
        c1 = torch.where((c1 != c1t) & (sig_min / sigma_max <= p.c4), c1t, c1)
        nrm_x = x.norm()
        flags.append(torch.stack([nrm_d == 0, nrm_ad <= c1 * (sigma_max * nrm_x + nrm_b), nrm_d <= tau,
                                  sigma_max / sig_min >= p.c3]))
        hist.append((sig_min, v_min, u_min))
        if p.am_i_printing and p.log_level >= 2:
            print(f"{p.prefix}CondEst: Iteration {itn} sigma_min = {float(sig_min)} "
                  f"cond = {sigma_max / float(sig_min)}")
        itn += 1
        if itn % check_every == 0 or itn >= T:
            F = torch.stack(flags).cpu().tolist()      # one host sync per check
            first = itn - len(F)
            for i, (zero_d, f1, f2, f3) in enumerate(F):
                it_i = first + i
                if it_i >= T:
                    break
                if zero_d:
                    return CondEstResult(1.0, sigma_max, v_max, u_max, sigma_max, sigma_max, v_max, u_max, -1)
                if T == Tlim and f1:
                    T, retval = int(1.25 * it_i + 1), -2
                if T == Tlim and f2:
                    T, retval = int(1.25 * it_i + 1), -3
                if T == Tlim and f3:
                    T, retval = int(1.25 * it_i + 1), -4
            if itn > T:      # overshoot past the stop iteration: restore its state
                sig_min, v_min, u_min = hist[T - 1 - first]
                del Rdiag[T:]
                del Rsub[max(0, T - 1):]
                itn = T
            flags, hist = [], []
    # sigma_min of the Lanczos bidiagonal R
    from scipy.linalg import svdvals
    N = len(Rdiag)
    Rd = torch.stack(Rdiag).cpu().numpy() if N else np.zeros(0)
    Rs = torch.stack(Rsub).cpu().numpy() if len(Rsub) else np.zeros(0)
    Rm = np.diag(Rd) + (np.diag(Rs, 1) if N > 1 else 0)
    sigma_min_c = float(sig_min)
    sigma_min_R = float(svdvals(Rm)[-1]) if N else sigma_min_c
    sigma_min = min(sigma_min_c, sigma_min_R)
    return CondEstResult(sigma_max / sigma_min, sigma_max, v_max, u_max, sigma_min, sigma_min_c, v_min, u_min,
                         retval)


CondEst = condest
