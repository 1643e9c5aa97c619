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


def condest(A, context: Context | None = None, params: CondEstParams | None = None) -> CondEstResult:
    from .. import default_context
    ctx = context if context is not None else default_context()
    p = params or CondEstParams()
    op = as_operator(A)
    m, n = op.shape
    dt = torch.float64
    dev = op.device

    def Av(x):
        return op.matmul(x.to(op.dtype)).to(dt)

    def Atv(u):
        return op.rmatmul(u.to(op.dtype)).to(dt)

    def lnorm(u):
        return float(op.long_colnorm(u)[0])

    # --- sigma_max by power iteration (normalised every step)
    v_max = _gauss(n, ctx, dt, dev)
    v_max = v_max / v_max.norm()
    for _ in range(p.powerits):
        u = Av(v_max)
        v_max = Atv(u)
        v_max = v_max / v_max.norm()
    u_max = Av(v_max)
    sigma_max = lnorm(u_max)
    u_max = u_max / sigma_max
    sigma_min = sigma_max
    u_min, v_min = u_max.clone(), v_max.clone()

    xhat = _gauss(n, ctx, dt, dev)
    nrm_xhat = float(xhat.norm())
    tau = math.sqrt(2) * _erfinv(p.c2) / nrm_xhat
    xhat = xhat / nrm_xhat
    b = Av(xhat)
    nrm_b = lnorm(b)
    u = b.clone()
    beta = lnorm(u)
    u = u / beta
    v = Atv(u)
    alpha = float(v.norm())
    v = v / alpha
    x = torch.zeros(n, 1, dtype=dt, device=dev)
    w = v.clone()
    phibar, rhobar = beta, alpha
    T = p.iter_lim if p.iter_lim >= 0 else max(20, 2 * min(m, n))
    Tlim = T
    Rdiag, Rsub = [], []
    c1 = p.c1
    retval = -6
    theta = 0.0
    itn = 0
    while itn < T:
        u = Av(v) - alpha * u
        beta = lnorm(u)
        u = u / beta
        v = Atv(u) - beta * v
        alpha = float(v.norm())
        v = v / alpha
        rho = math.sqrt(rhobar * rhobar + beta * beta)
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
        nrm_d = float(d.norm())
        if nrm_d == 0.0:
            return CondEstResult(1.0, sigma_max, v_max, u_max, sigma_max, sigma_max, v_max, u_max, -1)
        Ad = Av(d)
        nrm_ad = lnorm(Ad)
        if nrm_ad <= sigma_min * nrm_d:
            sigma_min = nrm_ad / nrm_d
            v_min = d.clone()
            u_min = Ad / nrm_ad
        if c1 != p.c1t and sigma_min / sigma_max <= p.c4:
            c1 = p.c1t
        nrm_x = float(x.norm())
        if T == Tlim and nrm_ad <= c1 * (sigma_max * nrm_x + nrm_b):
            T, retval = int(1.25 * itn + 1), -2
        if T == Tlim and nrm_d <= tau:
            T, retval = int(1.25 * itn + 1), -3
        if T == Tlim and sigma_max / sigma_min >= p.c3:
            T, retval = int(1.25 * itn + 1), -4
        if p.am_i_printing and p.log_level >= 2:
            print(f"{p.prefix}CondEst: Iteration {itn} sigma_min = {sigma_min} cond = {sigma_max / sigma_min}")
        itn += 1
    # sigma_min of the Lanczos bidiagonal R
    from scipy.linalg import svdvals
    N = len(Rdiag)
    Rm = np.diag(np.array(Rdiag)) + (np.diag(np.array(Rsub), 1) if N > 1 else 0)
    sigma_min_R = float(svdvals(Rm)[-1]) if N else sigma_min
    sigma_min_c = sigma_min
    if sigma_min_R < sigma_min:
        sigma_min = sigma_min_R
    return CondEstResult(sigma_max / sigma_min, sigma_max, v_max, u_max, sigma_min, sigma_min_c, v_min, u_min,
                         retval)


CondEst = condest
