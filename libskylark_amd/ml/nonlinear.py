"""Kernel regularized-least-squares estimators of the Python package
(reference ``python-skylark/skylark/ml/nonlinear.py``: ``rls``,
``sketchrls``, ``nystromrls``, ``sketchpcr``; ``ml/distances.py``).

All four share one shape: build a feature matrix, solve a small SPD system
(Cholesky on the device holding the data), keep what prediction needs.
Examples are ROWS of ``X``.  Multiclass problems are one-vs-rest on a ±1
dummy coding (:func:`.coding.dummy_coding`), decoded back to the original
label values.

* :class:`RLS` — exact kernel ridge: ``(K + lam I) alpha = Y`` on the full
  Gram (native Gram kernels on the GPU).
* :class:`SketchRLS` — random features ``Z = X S^T`` (the kernel's RFT, the
  fused MFMA feature GEMM on the GPU), ``(Z^T Z + lam I) W = Z^T Y``.
* :class:`NystromRLS` — ``s`` landmark rows drawn by a non-uniform sampler
  (uniform or ridge-leverage probabilities), features ``k(X, L) U`` with
  ``U = V diag(1/sqrt(evals))`` of ``k(L, L) + eps I``.
* :class:`SketchPCR` — principal-component regression on random features:
  the dominant ``rank``-dimensional subspace of ``Z`` is found from a
  ``t``-row CountSketch of ``Z`` (R of its QR, then the SVD of R), so only a
  ``t x s`` matrix is factorised; optional ``samplesize`` row subsampling
  for the subspace.  (The reference calls ``nla.lowrank.approximate_
  domsubspace_basis``, which its package does not ship; this is our own
  sketch-based construction of the same quantities ``Z, S, R, V``.)
"""
from __future__ import annotations

import torch

from ..base.context import Context
from ..base.exceptions import InvalidParametersError
from .coding import dummy_coding, dummy_decode


def euclidean(X, Y):
    """Squared distances ``D[i, j] = |Y_i - X_j|^2`` (t x m; reference
    ``ml/distances.py:24``).  Dense or sparse operands."""
    def sq(M):
        if M.layout != torch.strided:
            M = M.to_dense()
        return M
    Xd, Yd = sq(X), sq(Y)
    nx = (Xd * Xd).sum(dim=1)
    ny = (Yd * Yd).sum(dim=1)
    return ny[:, None] + nx[None, :] - 2.0 * (Yd @ Xd.t())


def _targets(Y, multiclass, dtype, device):
    if multiclass:
        T, _, rcoding = dummy_coding(Y, 1.0, -1.0, dtype=dtype, device=device)
        return T, rcoding
    T = torch.as_tensor(Y, dtype=dtype, device=device)
    return (T[:, None] if T.dim() == 1 else T), None


def _decode(P, rcoding):
    if rcoding is None:
        return P[:, 0] if P.shape[1] == 1 else P
    return dummy_decode(P, rcoding)


def _spd_solve(A, B):
    L, info = torch.linalg.cholesky_ex(A)
    if int(info) != 0:
        return torch.linalg.solve(A, B)
    return torch.cholesky_solve(B, L)


def _ctx(context):
    return context if context is not None else Context(0)


def _feat(rft, X):
    """Rowwise application: m x s features of the m examples."""
    return rft / X


class RLS:
    """Exact kernel RLS (reference ``rls``)."""

    def __init__(self, kernel):
        self._kernel = kernel
        self.model = {}

    def train(self, X, Y, regularization=1.0, multiclass=True, zerobased=False):
        K = self._kernel.gram(X)
        T, rc = _targets(Y, multiclass, K.dtype, K.device)
        K.diagonal().add_(float(regularization))
        alpha = _spd_solve(K, T)
        self.model = {"kernel": self._kernel, "alpha": alpha, "regularization": regularization, "data": X,
                      "multiclass": multiclass, "zerobased": zerobased, "rcoding": rc}
        return self

    def decision_function(self, Xt):
        K = self._kernel.gram(Xt, Y=self.model["data"])
        return K @ self.model["alpha"].to(K.dtype)

    def predict(self, Xt):
        return _decode(self.decision_function(Xt), self.model["rcoding"])


class SketchRLS:
    """Random-features kernel RLS (reference ``sketchrls``)."""

    def __init__(self, kernel, context: Context | None = None):
        self._kernel = kernel
        self._ctx = _ctx(context)
        self.model = {}

    def train(self, X, Y, random_features=100, regularization=1.0, multiclass=True, zerobased=False,
              subtype=None):
        self._rft = self._kernel.rft(random_features, subtype, context=self._ctx)
        Z = _feat(self._rft, X)
        T, rc = _targets(Y, multiclass, Z.dtype, Z.device)
        A = Z.t() @ Z
        A.diagonal().add_(float(regularization))
        W = _spd_solve(A, Z.t() @ T)
        self.model = {"kernel": self._kernel, "rft": self._rft, "weights": W, "random_features": random_features,
                      "regularization": regularization, "multiclass": multiclass, "zerobased": zerobased,
                      "rcoding": rc}
        return self

    def decision_function(self, Xt):
        Z = _feat(self._rft, Xt)
        return Z @ self.model["weights"].to(Z.dtype)

    def predict(self, Xt):
        return _decode(self.decision_function(Xt), self.model["rcoding"])


class NystromRLS:
    """Nyström kernel RLS (reference ``nystromrls``): ``probdist`` is
    'uniform' or 'leverages' (ridge leverage scores ``diag(K (K + lam I)^-1)``,
    which needs the full Gram: small problems only)."""

    def __init__(self, kernel, context: Context | None = None):
        self._kernel = kernel
        self._ctx = _ctx(context)
        self.model = {}

    def train(self, X, Y, random_features=100, regularization=1.0, probdist="uniform", multiclass=True,
              zerobased=False, eps=1e-8):
        from ..sketch import NURST
        m = X.shape[0]
        if probdist == "uniform":
            p = torch.full((m,), 1.0 / m, dtype=torch.float64)
        elif probdist == "leverages":
            K = self._kernel.gram(X).to(torch.float64)
            Kr = K.clone()
            Kr.diagonal().add_(float(regularization))
            p = torch.linalg.solve(Kr, K).diagonal().clamp_min(0).cpu()
        else:
            raise InvalidParametersError(f"Unknown probability distribution strategy {probdist!r}")
        SX = NURST(m, random_features, p, context=self._ctx) * X
        if SX.layout != torch.strided:
            SX = SX.to_dense()
        Kll = self._kernel.gram(SX)
        Kll.diagonal().add_(eps)
        evals, evecs = torch.linalg.eigh(Kll)
        U = evecs / evals.clamp_min(eps).sqrt()[None, :]
        Z = self._kernel.gram(X, Y=SX) @ U
        T, rc = _targets(Y, multiclass, Z.dtype, Z.device)
        A = Z.t() @ Z
        A.diagonal().add_(float(regularization))
        W = _spd_solve(A, Z.t() @ T)
        self.model = {"kernel": self._kernel, "weights": W, "random_features": random_features,
                      "regularization": regularization, "multiclass": multiclass, "zerobased": zerobased,
                      "SX": SX, "U": U, "rcoding": rc}
        return self

    def decision_function(self, Xt):
        Z = self._kernel.gram(Xt, Y=self.model["SX"]) @ self.model["U"]
        return Z @ self.model["weights"].to(Z.dtype)

    def predict(self, Xt):
        return _decode(self.decision_function(Xt), self.model["rcoding"])


def approximate_domsubspace_basis(X, rank: int, s: int, t: int, kernel, subtype=None, context=None):
    """Dominant ``rank``-dimensional subspace of the random-feature matrix
    ``Z = X S^T`` (S: ``s`` features of ``kernel``).  Returns ``(Q, S, R, V)``
    with ``Q = Z R^-1 V`` (m x rank, orthonormal up to the sketch's
    distortion), ``R`` (s x s upper triangular) from the QR of a ``t``-row
    CountSketch of ``Z`` and ``V`` the top-``rank`` left singular vectors of
    ``R``.  ``t >= s`` is required for ``R`` to be invertible."""
    from ..sketch import CWT
    ctx = _ctx(context)
    if t < s:
        raise InvalidParametersError("sketch size t must be >= number of features s")
    S = kernel.rft(s, subtype, context=ctx)
    Z = _feat(S, X)
    PZ = CWT(Z.shape[0], t, context=ctx) * Z
    R = torch.linalg.qr(PZ, mode="r")[1]
    # a zero diagonal entry (rank-deficient features) would make R singular
    d = R.diagonal()
    tiny = d.abs() <= 1e-12 * d.abs().max()
    if bool(tiny.any()):
        R = R + torch.diag(torch.where(tiny, 1e-12 * d.abs().max(), torch.zeros_like(d)))
    Ur, _, _ = torch.linalg.svd(R)
    V = Ur[:, :rank]
    Q = torch.linalg.solve_triangular(R, V, upper=True, left=True)
    Q = Z @ Q
    return Q, S, R, V


class SketchPCR:
    """Random-features principal-component regression (reference ``sketchpcr``)."""

    def __init__(self, kernel, context: Context | None = None):
        self._kernel = kernel
        self._ctx = _ctx(context)
        self.model = {}

    def train(self, X, Y, rank, s=None, t=None, samplesize=None, multiclass=True, zerobased=False, subtype=None):
        from ..sketch import UST
        s = 2 * rank if s is None else s
        t = 2 * s if t is None else t
        Xs = X if samplesize is None else UST(X.shape[0], samplesize, context=self._ctx) * X
        if Xs.layout != torch.strided:
            Xs = Xs.to_dense()
        Q, S, R, V = approximate_domsubspace_basis(Xs, rank, s, t, self._kernel, subtype, self._ctx)
        T, rc = _targets(Y, multiclass, Q.dtype, Q.device)
        if samplesize is not None:
            Q = _feat(S, X) @ torch.linalg.solve_triangular(R, V, upper=True)
        # least squares on the (nearly orthonormal) basis; exactly Q^T T when Q is orthonormal
        w0 = torch.linalg.lstsq(Q.cpu(), T.cpu()).solution.to(Q.device)
        W = torch.linalg.solve_triangular(R, V @ w0, upper=True)
        self._rft = S
        self.model = {"kernel": self._kernel, "rft": S, "weights": W, "s": s, "t": t, "rank": rank,
                      "multiclass": multiclass, "zerobased": zerobased, "rcoding": rc}
        return self

    def decision_function(self, Xt):
        Z = _feat(self._rft, Xt)
        return Z @ self.model["weights"].to(Z.dtype)

    def predict(self, Xt):
        return _decode(self.decision_function(Xt), self.model["rcoding"])


# python-skylark spellings
rls, sketchrls, nystromrls, sketchpcr = RLS, SketchRLS, NystromRLS, SketchPCR
