"""Cross-layout linear algebra on tensors and DistMatrix shards.

Reference: ``base/Gemm.hpp`` (``[VC,*]^T [VC,*] -> [*,*]`` via local GEMM +
all-reduce, ``:84-103``), ``base/inner.hpp`` (Nrm2 / ColumnNrm2 / ColumnDot
with one all-reduce of k scalars), ``base/QR.hpp:11-36`` (explicit Q,
``El::qr::ExplicitTS`` = TSQR for ``[VC,*]``), ``base/distance.hpp``
(Euclidean / L1 / exp-semigroup distance matrices), ``base/basic.hpp``.

Small factorisations (k x k, n x k with n <= a few thousand) are done
redundantly on every GPU in fp64 — cheap with 288 GB of HBM per GPU and it
removes a broadcast from every Krylov / power iteration.
"""
from __future__ import annotations

import torch

from ..parallel.comm import Comm


def _c(comm):
    return comm if comm is not None else Comm()


# ------------------------------------------------------------- products
GRAM_CHUNK = 1 << 16


def gram(Y_local: torch.Tensor, comm: Comm | None = None, dtype=torch.float64) -> torch.Tensor:
    """``Y^T Y`` for a row-distributed Y (all-reduced, replicated k x k, float64).

    f32 inputs are multiplied in f32 on the matrix cores in row chunks whose
    partial Grams are accumulated in f64 (an f64 GEMM over a million rows
    is ~50x slower on MI355X and buys nothing here)."""
    if Y_local.dtype == torch.float64:
        G = Y_local.t() @ Y_local
    else:
        Yf = Y_local if Y_local.dtype == torch.float32 else Y_local.float()
        G = torch.zeros(Yf.shape[1], Yf.shape[1], dtype=torch.float64, device=Yf.device)
        for r0 in range(0, Yf.shape[0], GRAM_CHUNK):
            Yc = Yf[r0:r0 + GRAM_CHUNK]
            G += (Yc.t() @ Yc).double()
    return _c(comm).all_reduce(G.contiguous())


def gemm_tn(A_local: torch.Tensor, B_local: torch.Tensor, comm: Comm | None = None) -> torch.Tensor:
    """``A^T B`` for row-distributed A, B (reference base::Gemm [VC,*]^T[VC,*] -> [*,*])."""
    C = A_local.t() @ B_local
    return _c(comm).all_reduce(C.contiguous())


def column_nrm2(X_local: torch.Tensor, comm: Comm | None = None, distributed: bool = True) -> torch.Tensor:
    """Column 2-norms of a row-distributed matrix (one all-reduce of k scalars)."""
    sq = (X_local.double() ** 2).sum(0) if X_local.dtype != torch.float64 else (X_local ** 2).sum(0)
    if distributed:
        _c(comm).all_reduce(sq)
    return sq.sqrt()


def column_dot(X_local, Y_local, comm: Comm | None = None, distributed: bool = True):
    d = (X_local.double() * Y_local.double()).sum(0)
    if distributed:
        _c(comm).all_reduce(d)
    return d


def nrm2(X_local, comm: Comm | None = None, distributed: bool = True):
    s = (X_local.double() ** 2).sum().reshape(1)
    if distributed:
        _c(comm).all_reduce(s)
    return float(s.sqrt())


# ------------------------------------------------------------------ QR
def cholesky_qr(Y_local: torch.Tensor, comm: Comm | None = None, shift: float = 0.0):
    """One CholeskyQR step: ``Q = Y R^{-1}``, ``R = chol(Y^T Y)``; returns (Q, R) or None on failure."""
    G = gram(Y_local, comm)
    if shift:
        G = G + shift * torch.eye(G.shape[0], dtype=G.dtype, device=G.device) * G.diagonal().max()
    L, info = torch.linalg.cholesky_ex(G)
    if int(info) != 0:
        return None
    R = L.t()
    Q = torch.linalg.solve_triangular(R.to(Y_local.dtype), Y_local, upper=True, left=False)
    return Q, R


def cholesky_qr2(Y_local: torch.Tensor, comm: Comm | None = None):
    """CholeskyQR2 (two passes) with a shifted first pass fallback; TSQR if both fail."""
    r1 = cholesky_qr(Y_local, comm)
    if r1 is None:
        r1 = cholesky_qr(Y_local, comm, shift=1e-12 * Y_local.shape[0])
        if r1 is None:
            return tsqr(Y_local, comm)
    Q1, R1 = r1
    r2 = cholesky_qr(Q1, comm)
    if r2 is None:
        return tsqr(Y_local, comm)
    Q2, R2 = r2
    return Q2, R2 @ R1


def tsqr(Y_local: torch.Tensor, comm: Comm | None = None):
    """Tall-skinny QR for a row-distributed matrix (reference El::qr::ExplicitTS).

    Local Householder QR on every GPU, all-gather of the k x k R factors,
    redundant QR of the stacked R's, local update of Q.
    """
    c = _c(comm)
    k = Y_local.shape[1]
    wd = torch.float64
    Yd = Y_local.to(wd)
    if Yd.shape[0] >= k:
        Q1, R1 = torch.linalg.qr(Yd, mode="reduced")
    else:  # short shard: pad R to k x k
        Q1, R1 = torch.linalg.qr(Yd, mode="complete")
        Q1 = torch.cat([Q1, torch.zeros(Yd.shape[0], k - Q1.shape[1], dtype=wd, device=Yd.device)], 1)[:, :k]
        R1 = torch.cat([R1, torch.zeros(k - R1.shape[0], k, dtype=wd, device=Yd.device)], 0)
    if c.size == 1:
        Q, R = Q1, R1
    else:
        Rs = c.all_gather(R1.contiguous(), 0)  # (p*k) x k
        Q2, R = torch.linalg.qr(Rs, mode="reduced")
        Q = Q1 @ Q2[c.rank * k:(c.rank + 1) * k]
    # sign convention: positive diagonal of R
    s = torch.sign(torch.diagonal(R))
    s[s == 0] = 1
    return (Q * s[None, :]).to(Y_local.dtype), s[:, None] * R


def orthonormalize(Y_local, comm: Comm | None = None, method: str = "cholqr2"):
    if method == "tsqr":
        return tsqr(Y_local, comm)[0]
    return cholesky_qr2(Y_local, comm)[0]


# -------------------------------------------------------------- distances
def euclidean_distance_matrix(X: torch.Tensor, Y: torch.Tensor, columns: bool = True) -> torch.Tensor:
    """Squared Euclidean distances between columns (or rows) of X and Y
    (reference ``base/distance.hpp:44-78``: ``|x|^2 + |y|^2 - 2 x^T y``)."""
    if not columns:
        X, Y = X.t(), Y.t()
    xn = (X * X).sum(0)
    yn = (Y * Y).sum(0)
    D = xn[:, None] + yn[None, :] - 2.0 * (X.t() @ Y)
    return D.clamp_min_(0)


def l1_distance_matrix(X: torch.Tensor, Y: torch.Tensor, columns: bool = True) -> torch.Tensor:
    if not columns:
        X, Y = X.t(), Y.t()
    return torch.cdist(X.t().contiguous(), Y.t().contiguous(), p=1)


def expsemigroup_distance_matrix(X: torch.Tensor, Y: torch.Tensor, columns: bool = True) -> torch.Tensor:
    """``D_ij = sum_k sqrt(x_ki + y_kj)`` (reference ``base/distance.hpp:385-418``)."""
    if not columns:
        X, Y = X.t(), Y.t()
    out = torch.empty(X.shape[1], Y.shape[1], dtype=X.dtype, device=X.device)
    bs = max(1, (1 << 24) // max(1, X.shape[0] * Y.shape[1]))
    for i in range(0, X.shape[1], bs):
        xi = X[:, i:i + bs]
        out[i:i + bs] = torch.sqrt((xi[:, :, None] + Y[:, None, :]).abs()).sum(0)
    return out


def symmetric_entrywise_map(D, fn, uplo="L"):
    return fn(D)
