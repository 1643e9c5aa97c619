"""Losses with proximal operators (reference ``algorithms/regression/loss.hpp:7-446``).

Every loss provides ``evaluate(O, Y)`` (total loss over the k x n output
matrix O and targets Y — a label vector for the classification losses) and
``proxoperator(X, lambda, Y)`` returning ``argmin_Z loss(Z, Y) + 1/(2 lambda)
||Z - X||^2``.  All operations are element-wise / per-example GPU kernels
(torch); the logistic prox runs a batched Newton iteration (one example per
column) entirely on the device.
"""
from __future__ import annotations

import torch


class Loss:
    name = "loss"

    def evaluate(self, O: torch.Tensor, Y: torch.Tensor) -> float:
        return float(self.evaluate_t(O, Y))

    def evaluate_t(self, O: torch.Tensor, Y: torch.Tensor) -> torch.Tensor:
        """The loss as a 0-d device tensor (no host synchronisation)."""
        raise NotImplementedError

    def proxoperator(self, X: torch.Tensor, lam: float, Y: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError


def _targets_matrix(Y, k, like):
    """Y (n labels in [0,k) or k x n real targets) -> k x n matrix."""
    if Y.dim() == 2:
        return Y.to(like.dtype)
    if k == 1:
        return Y.to(like.dtype)[None, :]
    T = -torch.ones(k, Y.shape[0], dtype=like.dtype, device=like.device)
    T[Y.long(), torch.arange(Y.shape[0], device=like.device)] = 1.0
    return T


class SquaredLoss(Loss):
    """0.5 ||O - Y||^2 (regression)."""
    name = "squared"

    def evaluate_t(self, O, Y):
        T = _targets_matrix(Y, O.shape[0], O)
        return 0.5 * ((O - T) ** 2).sum()

    def proxoperator(self, X, lam, Y):
        T = _targets_matrix(Y, X.shape[0], X)
        return (X + lam * T) / (1.0 + lam)


class LADLoss(Loss):
    """||O - Y||_1 (least absolute deviations)."""
    name = "lad"

    def evaluate_t(self, O, Y):
        T = _targets_matrix(Y, O.shape[0], O)
        return (O - T).abs().sum()

    def proxoperator(self, X, lam, Y):
        T = _targets_matrix(Y, X.shape[0], X)
        D = X - T
        return T + torch.sign(D) * torch.clamp(D.abs() - lam, min=0)


class HingeLoss(Loss):
    """Multiclass hinge sum_i max(0, 1 - y_ij o_ij) with ±1 one-vs-rest coding."""
    name = "hinge"

    def evaluate_t(self, O, Y):
        T = _targets_matrix(Y, O.shape[0], O)
        return torch.clamp(1 - T * O, min=0).sum()

    def proxoperator(self, X, lam, Y):
        T = _targets_matrix(Y, X.shape[0], X)
        # prox of max(0, 1 - t z): case split on t x
        tx = T * X
        Z = torch.where(tx >= 1, X, torch.where(tx <= 1 - lam, X + lam * T, T))
        return Z


class LogisticLoss(Loss):
    """Multinomial logistic: sum_j [ log sum_c exp(o_cj) - o_{y_j, j} ]."""
    name = "logistic"

    def evaluate_t(self, O, Y):
        y = Y.long() if Y.dim() == 1 else Y.argmax(0)
        return (torch.logsumexp(O, 0) - O[y, torch.arange(O.shape[1], device=O.device)]).sum()

    def proxoperator(self, X, lam, Y, iters: int = 30, tol: float = 1e-10):
        """Per-example Newton iteration with backtracking (reference logexp prox,
        ``loss.hpp:364-424``), batched over columns on the device."""
        y = Y.long() if Y.dim() == 1 else Y.argmax(0)
        k, n = X.shape
        E = torch.zeros_like(X)
        E[y, torch.arange(n, device=X.device)] = 1.0
        Z = X.clone()

        def obj(Z):
            return lam * (torch.logsumexp(Z, 0) - (E * Z).sum(0)) + 0.5 * ((Z - X) ** 2).sum(0)

        for it in range(iters):
            P = torch.softmax(Z, 0)
            g = lam * (P - E) + (Z - X)
            # Hessian = I + lam (diag(p) - p p^T): solve per column (Sherman-Morrison)
            dvec = 1.0 + lam * P
            u = g / dvec
            w = P / dvec
            coef = (lam * (P * u).sum(0)) / (1.0 - lam * (P * w).sum(0))
            step = u + coef * w
            f0 = obj(Z)
            t = torch.ones(n, dtype=X.dtype, device=X.device)
            for _ in range(20):
                Zn = Z - t * step
                ok = obj(Zn) <= f0 - 1e-4 * t * (g * step).sum(0)
                if bool(ok.all()):
                    break
                t = torch.where(ok, t, t * 0.5)
            Z = Z - t * step
            if it % 5 == 4 and float(g.abs().max()) < tol:   # host sync only every 5 Newton steps
                break
        return Z


LOSSES = {"squared": SquaredLoss, "lad": LADLoss, "hinge": HingeLoss, "logistic": LogisticLoss}


def make_loss(name):
    """Reference CLI codes: 0 squared, 1 lad, 2 hinge, 3 logistic (ml/options.hpp)."""
    if isinstance(name, int):
        name = ["squared", "lad", "hinge", "logistic"][name]
    return LOSSES[name.lower()]()
