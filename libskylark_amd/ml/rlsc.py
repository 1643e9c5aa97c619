"""Regularised least-squares classification (reference ``ml/rlsc.hpp:45-311``).

Each KRR variant is wrapped: labels are dummy-coded (±1 one-vs-rest, codes in
order of first appearance, :mod:`.coding`), the multi-output ridge problem
is solved, and ``rcoding`` is returned so predictions can be decoded by
arg-max (:func:`.coding.dummy_decode` / the model classes).
"""
from __future__ import annotations

from .coding import dummy_coding
from .krr import (KrrParams, approximate_kernel_ridge, faster_kernel_ridge, kernel_ridge,
                  large_scale_kernel_ridge, sketched_approximate_kernel_ridge, _Data)

rlsc_params_t = KrrParams


def _code(L, X, direction):
    data = _Data(X, direction)
    Y, _, rcoding = dummy_coding(L, dtype=data.local.dtype if data.local.dtype.is_floating_point else None,
                                 device=data.local.device)
    return Y, rcoding


def kernel_rlsc(k, X, L, lam, direction="rows", params=None):
    """Returns ``(A, rcoding)``."""
    Y, rc = _code(L, X, direction)
    return kernel_ridge(k, X, Y, lam, direction, params), rc


def approximate_kernel_rlsc(k, X, L, lam, s, context=None, direction="rows", params=None):
    """Returns ``(S, W, rcoding)``."""
    Y, rc = _code(L, X, direction)
    S, W = approximate_kernel_ridge(k, X, Y, lam, s, context, direction, params)
    return S, W, rc


def sketched_approximate_kernel_rlsc(k, X, L, lam, s, t=-1, context=None, direction="rows", params=None):
    """Returns ``(scale_maps, transforms, W, rcoding)``."""
    Y, rc = _code(L, X, direction)
    return (*sketched_approximate_kernel_ridge(k, X, Y, lam, s, t, context, direction, params), rc)


def faster_kernel_rlsc(k, X, L, lam, s, context=None, direction="rows", params=None):
    """Returns ``(A, rcoding)``."""
    Y, rc = _code(L, X, direction)
    return faster_kernel_ridge(k, X, Y, lam, s, context, direction, params), rc


def large_scale_kernel_rlsc(k, X, L, lam, s, context=None, direction="rows", params=None):
    """Returns ``(scale_maps, transforms, W, rcoding)``."""
    Y, rc = _code(L, X, direction)
    return (*large_scale_kernel_ridge(k, X, Y, lam, s, context, direction, params), rc)


KernelRLSC = kernel_rlsc
ApproximateKernelRLSC = approximate_kernel_rlsc
SketchedApproximateKernelRLSC = sketched_approximate_kernel_rlsc
FasterKernelRLSC = faster_kernel_rlsc
LargeScaleKernelRLSC = large_scale_kernel_rlsc
