"""Least squares entry points (reference ``nla/least_squares.hpp``).

* :func:`approximate_least_squares` — sketch-and-solve with FJLT, sketch size
  ``4n`` by default, QR solve of the sketched problem (``:42-184``);
* :func:`faster_least_squares` — Blendenpik (QR-preconditioned LSQR) to full
  accuracy (``:237-314``, C API ``sl_faster_least_squares``);
* :func:`lsrn_least_squares` — LSRN (JLT sketch, SVD preconditioner,
  Chebyshev / LSQR), the north-star "LSRN sketch-and-solve" configuration.

``A`` may be a dense or sparse local tensor or a row-distributed DistMatrix
([VC,*]); ``orientation="adjoint"`` solves the under-determined problem
``min ||x|| s.t. A^T x = b`` by working on ``A^T``.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..algorithms.krylov import KrylovIterParams
from ..algorithms.regression import (AcceleratedRegressionSolver, RegressionProblem,
                                     SketchedRegressionSolver)
from ..base.context import Context
from ..parallel.distmatrix import DistMatrix


@dataclass
class FasterLSParams:
    am_i_printing: bool = False
    log_level: int = 0
    prefix: str = ""
    debug_level: int = 0
    tolerance: float = 1e-14
    iter_lim: int = 100

    @classmethod
    def from_dict(cls, d):
        keys = cls.__dataclass_fields__.keys()
        return cls(**{k: v for k, v in d.items() if k in keys})


faster_ls_params_t = FasterLSParams


def _orient(A, orientation):
    if orientation in ("normal", "NORMAL", 0):
        return A
    if isinstance(A, DistMatrix):
        g = A.redistribute("STAR_VC")
        return DistMatrix(g.local.t().contiguous(), (A.shape[1], A.shape[0]), "VC_STAR", A.comm)
    return A.t()


def approximate_least_squares(A, B, context: Context | None = None, orientation: str = "normal",
                              sketch_size: int | None = None, sketch_type: str = "FJLT"):
    """Sketch-and-solve: ``argmin ||S A x - S b||`` (FJLT sketch, s = 4n)."""
    A = _orient(A, orientation)
    prob = RegressionProblem(A)
    solver = SketchedRegressionSolver(prob, context, sketch_type=sketch_type,
                                      sketch_size=sketch_size or 4 * prob.n, exact="qr")
    return solver.solve(B)


def faster_least_squares(A, B, context: Context | None = None, orientation: str = "normal",
                         params: FasterLSParams | None = None):
    """Blendenpik-accelerated LSQR to (near) machine accuracy.  Returns X."""
    params = params or FasterLSParams()
    A = _orient(A, orientation)
    kp = KrylovIterParams(tolerance=params.tolerance, iter_lim=params.iter_lim, am_i_printing=params.am_i_printing,
                          log_level=params.log_level, prefix=params.prefix)
    solver = AcceleratedRegressionSolver(RegressionProblem(A), context, method="blendenpik", params=kp)
    X, _ = solver.solve(B)
    return X


def lsrn_least_squares(A, B, context: Context | None = None, params: KrylovIterParams | None = None,
                       oversample: int = 4, precond: str = "auto"):
    """LSRN: JLT sketch (t = oversample * n), SVD (or equivalent-spectrum QR)
    preconditioner, Chebyshev or LSQR.  ``precond="auto"``: SVD for n <= 2000,
    QR (same preconditioned singular values, much cheaper) above."""
    n = A.shape[1]
    if precond == "auto":
        precond = "svd" if n <= 2000 else "qr"
    solver = AcceleratedRegressionSolver(RegressionProblem(A), context, method="lsrn", precond=precond,
                                         params=params or KrylovIterParams(tolerance=1e-10, iter_lim=200),
                                         oversample=oversample)
    X, _ = solver.solve(B)
    return X


ApproximateLeastSquares = approximate_least_squares
FasterLeastSquares = faster_least_squares
