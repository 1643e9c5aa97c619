"""Linear least-squares regression: problem, exact, sketched and accelerated solvers.

Reference (``algorithms/regression/``):
  * ``regression_problem_t<A, linear_tag, l2_tag, no_reg_tag>``
    (``regression_problem.hpp:57-83``);
  * exact solvers ``qr_l2_solver_tag`` / ``sne_l2_solver_tag`` (semi-normal
    equations) / ``ne_l2_solver_tag`` / ``svd_l2_solver_tag`` /
    ``iterative_l2_solver_tag<lsqr_tag>``
    (``linearl2_regression_solver_Elemental.hpp:23-631``, ``..._Krylov.hpp``);
  * ``sketched_regression_solver_t`` (sketch-and-solve:
    ``sketched_regression_solver_Elemental.hpp:19-215`` — we sketch B, not the
    reference's ``SB`` typo at :110);
  * ``accelerated_regression_solver_t`` with ``blendenpik_tag`` (RFUT-DCT +
    uniform row sampling, t = 4n, QR preconditioner, ``dtrcon`` condition
    check with up to 3 retries then an SVD-solver fallback, LSQR),
    ``simplified_blendenpik_tag<Transform>`` (any sketch, LSQR) and
    ``lsrn_tag`` (JLT t = 4n, SVD preconditioner, Chebyshev when the
    singular-value bounds are tight enough, else LSQR)
    (``accelerated_linearl2_regression_solver_Elemental.hpp:1-624``).

Row-distributed problems (DistMatrix [VC,*]) keep A sharded: the sketch is a
partial product per GPU plus one all-reduce, the small factorisations are
redundant on every GPU, LSQR/Chebyshev use the distributed operator.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..base.context import Context
from ..base.exceptions import InvalidParametersError
from ..parallel.distmatrix import DistMatrix
from ..utils.timer import PROFILER
from .krylov import IdPrecond, KrylovIterParams, MatPrecond, TriInversePrecond, chebyshev_ls, lsqr
from .operators import as_operator


class RegressionProblem:
    """``min_x || A x - b ||_2`` (linear, l2 loss, no regulariser)."""

    def __init__(self, A, loss: str = "l2", regularizer: str | None = None):
        if loss not in ("l2", "linear_l2"):
            raise InvalidParametersError("only linear l2 regression problems are supported (as the reference)")
        if regularizer not in (None, "none"):
            raise InvalidParametersError("regularised linear regression is not supported (as the reference)")
        self.A = A
        self.m, self.n = (A.shape if not isinstance(A, DistMatrix) else A.shape)

    @property
    def input_matrix(self):
        return self.A


regression_problem_t = RegressionProblem


def _local_dense(A):
    """A local (non-distributed) operand as a dense tensor."""
    if A.layout != torch.strided:
        return A.to_dense()
    return A


def _wdt(A):
    dt = A.dtype if not isinstance(A, DistMatrix) else A.local.dtype
    return torch.float64 if dt == torch.float64 else torch.float32


class RegressionSolver:
    """Exact solvers: ``method`` in {"qr", "sne", "ne", "svd", "lsqr"}.

    A row-distributed DistMatrix (any layout; non-row layouts are brought to
    ``[VC,*]`` by one all-to-all) is never gathered: "qr", "sne" and "svd"
    factor it by TSQR (reference ``El::qr::ExplicitTS`` for ``[VC,*]``,
    ``base/QR.hpp:11-36``) -- a local Householder QR per GPU plus one
    all-gather of the n x n R factors -- "ne" by the all-reduced Gram, and the
    right-hand side enters only through ``Q^T b`` / ``A^T b`` (one all-reduce
    of n x k).  The n x n factorisations are redundant on every rank."""

    def __init__(self, problem: RegressionProblem, method: str = "qr", params: KrylovIterParams | None = None):
        self.problem = problem
        self.method = method.lower()
        self.params = params or KrylovIterParams()
        A = problem.A
        if self.method == "lsqr":
            return
        if self.method not in ("qr", "sne", "ne", "svd"):
            raise InvalidParametersError(f"unknown exact solver {method}")
        self.dist = isinstance(A, DistMatrix)
        if self.dist:
            D = A if A.layout in ("VC_STAR", "VR_STAR") else A.redistribute("VC_STAR")
            self.D, self.comm = D, D.comm
            Ad = D.local.to(torch.float64)
        else:
            self.comm = None
            Ad = _local_dense(A).to(torch.float64)
        from ..base import linalg as L
        if self.method in ("qr", "sne", "svd"):
            if self.dist:
                self.Q, self.R = L.tsqr(Ad, self.comm)
            else:
                self.Q, self.R = torch.linalg.qr(Ad, mode="reduced")
            if self.method == "sne":
                self.Ad, self.Q = Ad, None
            elif self.method == "svd":
                Ur, self.s, self.Vh = torch.linalg.svd(self.R, full_matrices=False)
                self.Ur = Ur
        else:
            self.Ad = Ad
            G = Ad.t() @ Ad
            if self.dist:
                self.comm.all_reduce(G)
            self.L = torch.linalg.cholesky(G)

    def _rhs_local(self, b):
        """Rows of b matching this rank's rows of A (fp64, 2-D)."""
        if isinstance(b, DistMatrix):
            if self.dist:
                bb = b if b.layout in ("VC_STAR", "VR_STAR") else b.redistribute("VC_STAR")
                return bb.local
            return b.to_global()
        if self.dist:
            r0, r1 = self.D.row_range()
            return b[r0:r1]
        return b

    def _reduce(self, X):
        if self.dist:
            self.comm.all_reduce(X)
        return X

    def solve(self, b):
        A = self.problem.A
        vec = (b.dim() == 1) if isinstance(b, torch.Tensor) else False
        if self.method == "lsqr":
            X, _ = lsqr(A, b[:, None] if vec else b, params=self.params)
            return X[:, 0] if vec else X
        B = self._rhs_local(b)
        B2 = (B[:, None] if B.dim() == 1 else B).to(torch.float64).to(self._dev())
        if self.method == "qr":
            X = torch.linalg.solve_triangular(self.R, self._reduce(self.Q.t() @ B2), upper=True)
        elif self.method == "sne":
            # semi-normal equations R^T R x = A^T b
            y = torch.linalg.solve_triangular(self.R.t(), self._reduce(self.Ad.t() @ B2), upper=False)
            X = torch.linalg.solve_triangular(self.R, y, upper=True)
        elif self.method == "ne":
            X = torch.cholesky_solve(self._reduce(self.Ad.t() @ B2), self.L)
        else:
            tol = self.s.max() * max(self.problem.m, self.problem.n) * torch.finfo(torch.float64).eps
            sinv = torch.where(self.s > tol, 1.0 / self.s, torch.zeros_like(self.s))
            X = self.Vh.t() @ (sinv[:, None] * (self.Ur.t() @ self._reduce(self.Q.t() @ B2)))
        return X[:, 0] if vec else X

    def _dev(self):
        for name in ("Q", "R", "Ad"):
            t = getattr(self, name, None)
            if isinstance(t, torch.Tensor):
                return t.device
        return None


regression_solver_t = RegressionSolver


def _sketch_rows(sketch_type: str, m: int, t: int, ctx: Context, **kw):
    from .. import sketch as S
    cls = S.sketch_class(sketch_type)
    return cls(m, t, context=ctx, **kw)


def _apply_columnwise(sk, A):
    """S A (t x n, replicated) for local or [VC,*]-distributed A."""
    if isinstance(A, DistMatrix):
        from ..parallel.dist_sketch import dist_apply
        return dist_apply(sk, A, None, 0, out_layout="STAR_STAR").local
    out = sk.apply(A, None, 0)
    return out.to_dense() if isinstance(out, torch.Tensor) and out.layout != torch.strided else out


class SketchedRegressionSolver:
    """Sketch-and-solve: ``x = argmin ||S A x - S b||`` with an exact solver on the sketch."""

    def __init__(self, problem: RegressionProblem, context: Context | None = None, sketch_type: str = "JLT",
                 sketch_size: int | None = None, exact: str = "qr", **sketch_params):
        from .. import default_context
        ctx = context if context is not None else default_context()
        self.problem = problem
        t = sketch_size or 4 * problem.n
        self.S = _sketch_rows(sketch_type, problem.m, t, ctx, **sketch_params)
        SA = _apply_columnwise(self.S, problem.A)
        self.inner = RegressionSolver(RegressionProblem(SA), exact)

    def solve(self, b):
        vec = (b.dim() == 1) if isinstance(b, torch.Tensor) else False
        bb = b[:, None] if vec else b
        Sb = _apply_columnwise(self.S, bb)
        x = self.inner.solve(Sb)
        return x[:, 0] if vec else x


sketched_regression_solver_t = SketchedRegressionSolver


def _utcondest(R: torch.Tensor) -> float:
    """1-norm condition estimate of an upper-triangular matrix (LAPACK dtrcon)."""
    from scipy.linalg import lapack
    rc, info = lapack.dtrcon(R.detach().double().cpu().numpy(), norm="1", uplo="U", diag="N")
    return float("inf") if rc == 0 else 1.0 / rc


def _on_gpu(A) -> bool:
    loc = A.local if isinstance(A, DistMatrix) else A
    return isinstance(loc, torch.Tensor) and loc.is_cuda and loc.dtype == torch.float32


CHOLQR_MAX_COND = 1e7     # fp64 Gram squares the condition number: keep kappa(R)^2 eps64 << 1


def _tri_inv_upper(R: torch.Tensor, block: int = 1024) -> torch.Tensor:
    """R^{-1} of an upper-triangular R, one column block at a time (column
    block j of R^{-1} only involves the leading j1 x j1 block of R; blocking
    also bounds the BLAS trsm workspace, which failed to allocate for a single
    5000-column right-hand side on the MI355X)."""
    n = R.shape[0]
    Rinv = torch.zeros_like(R)
    for j0 in range(0, n, block):
        j1 = min(n, j0 + block)
        E = torch.zeros(j1, j1 - j0, dtype=R.dtype, device=R.device)
        E[j0:j1] = torch.eye(j1 - j0, dtype=R.dtype, device=R.device)
        Rinv[:j1, j0:j1] = torch.linalg.solve_triangular(R[:j1, :j1], E, upper=True)
    return Rinv


def _cholqr_r(SA: torch.Tensor):
    """(R, R^{-1}) of the sketch SA = Q R by fp64 Cholesky of the Gram on the
    GPU (one f64 GEMM of t x n^2 flops + an n^3/3 Cholesky + a triangular
    inverse, all on the matrix cores), or None when the Gram is not safely
    SPD: then the caller falls back to Householder QR.  The guard is the exact
    1-norm condition number of R computed from R^{-1} (which the explicit
    preconditioner needs anyway)."""
    X = SA.to(torch.float64)
    G = X.t() @ X
    L, info = torch.linalg.cholesky_ex(G)
    if int(info) != 0:
        return None
    R = L.t().contiguous()
    Rinv = _tri_inv_upper(R)
    kappa = float(torch.linalg.matrix_norm(R, 1) * torch.linalg.matrix_norm(Rinv, 1))
    if not (kappa < CHOLQR_MAX_COND):
        return None
    return R, Rinv


def _build_precond(SA: torch.Tensor, kind: str):
    if kind == "qr":
        if SA.is_cuda and SA.shape[1] >= 256:
            rr = _cholqr_r(SA)
            if rr is not None:
                return TriInversePrecond(rr[0], upper=True, Rinv=rr[1]), rr[0]
        _, R = torch.linalg.qr(SA.to(torch.float64), mode="r")
        Rinv = None
        if SA.is_cuda and SA.shape[1] >= 256:
            # explicit inverse only while it stays accurate (its error grows like
            # kappa(R) eps); ill-conditioned R keeps the backward-stable solves
            Rinv = _tri_inv_upper(R)
            kappa = float(torch.linalg.matrix_norm(R, 1) * torch.linalg.matrix_norm(Rinv, 1))
            if not (kappa < CHOLQR_MAX_COND):
                Rinv = None
        return TriInversePrecond(R, upper=True, Rinv=Rinv), R
    SA = SA.to(torch.float64)
    U, s, Vh = torch.linalg.svd(SA, full_matrices=False)
    tol = s.max() * max(SA.shape) * torch.finfo(torch.float64).eps
    sinv = torch.where(s > tol, 1.0 / s, torch.zeros_like(s))
    return MatPrecond(Vh.t() * sinv[None, :]), None


class AcceleratedRegressionSolver:
    """Sketch-preconditioned iterative least squares.

    ``method``: "blendenpik" (RFUT-DCT row mixing + uniform sampling, QR
    precond, condition check/retries, LSQR), "simplified_blendenpik" (any
    ``transform``), "lsrn" (JLT, SVD precond, Chebyshev/LSQR).
    """

    def __init__(self, problem: RegressionProblem, context: Context | None = None, method: str = "blendenpik",
                 precond: str = "qr", transform: str = "FJLT", sketch_size: int | None = None,
                 params: KrylovIterParams | None = None, oversample: int = 4, lowp_sketch: bool = True):
        from .. import default_context
        ctx = context if context is not None else default_context()
        self.problem = problem
        self.method = method.lower()
        self.params = params or KrylovIterParams()
        m, n = problem.m, problem.n
        t = sketch_size or oversample * n
        A = problem.A
        self.use_lsqr = True
        self.fallback = None
        if self.method == "blendenpik":
            self.precond = None
            for _ in range(3):
                sk = _sketch_rows("FJLT", m, t, ctx)
                SA = _apply_columnwise(sk, A)
                P, R = _build_precond(SA, "qr")
                if _utcondest(R) < 1e14:
                    self.precond = P
                    break
            if self.precond is None:  # reference: fall back to an exact SVD solver
                self.fallback = RegressionSolver(problem, "svd")
        elif self.method == "simplified_blendenpik":
            sk = _sketch_rows(transform, m, t, ctx)
            self.precond, _ = _build_precond(_apply_columnwise(sk, A), precond)
        elif self.method == "lsrn":
            delta = 1e-6
            with PROFILER.phase("lsrn.sketch"):
                sk = _sketch_rows("JLT", m, t, ctx)
                if _on_gpu(A) and lowp_sketch:
                    sk.set_precision("bf16x2")  # S rounded to bf16: still a Gaussian-like sketch
                SA = _apply_columnwise(sk, A)
            # LSRN's N = V S^{-1} (precond="svd") and R^{-1} from SA = QR ("qr") give
            # preconditioned operators with identical singular values, so the
            # Chebyshev bounds below hold for both; QR is far cheaper for large n.
            with PROFILER.phase("lsrn.precond"):
                self.precond, _ = _build_precond(SA, precond)
            alpha = math.sqrt(2 * math.log(2.0 / delta) / t)
            if alpha >= 1 - math.sqrt(n / t):
                self.use_lsqr = True
            else:
                self.use_lsqr = False
                self.sigma_U = math.sqrt(t) / ((1 - alpha) * math.sqrt(t) - math.sqrt(n))
                self.sigma_L = math.sqrt(t) / ((1 + alpha) * math.sqrt(t) + math.sqrt(n))
        else:
            raise InvalidParametersError(f"unknown accelerated method {method}")

    def solve(self, b):
        if self.fallback is not None:
            return self.fallback.solve(b), -1
        vec = (b.dim() == 1) if isinstance(b, torch.Tensor) else False
        bb = b[:, None] if vec else b
        with PROFILER.phase("regression.krylov"):
            if self.use_lsqr:
                X, code = lsqr(self.problem.A, bb, params=self.params, R=self.precond)
            else:
                X = chebyshev_ls(self.problem.A, bb, self.sigma_L, self.sigma_U, self.params, self.precond)
                code = -6
        return (X[:, 0] if vec else X), code


accelerated_regression_solver_t = AcceleratedRegressionSolver
