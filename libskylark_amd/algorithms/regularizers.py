"""Regularisers with proximal operators (reference ``algorithms/regression/regularizers.hpp:8-100``)."""
from __future__ import annotations

import torch


class Regularizer:
    name = "none"

    def evaluate(self, W: torch.Tensor) -> float:
        return float(self.evaluate_t(W))

    def evaluate_t(self, W: torch.Tensor) -> torch.Tensor:
        """The penalty as a 0-d device tensor (no host synchronisation)."""
        return torch.zeros((), dtype=W.dtype, device=W.device)

    def proxoperator(self, W: torch.Tensor, lam: float) -> torch.Tensor:
        return W


class NoRegularizer(Regularizer):
    pass


class L2Regularizer(Regularizer):
    """0.5 ||W||_F^2 ; prox = shrinkage W / (1 + lambda)."""
    name = "l2"

    def evaluate_t(self, W):
        return 0.5 * (W * W).sum()

    def proxoperator(self, W, lam):
        return W / (1.0 + lam)


class L1Regularizer(Regularizer):
    """||W||_1 ; prox = soft thresholding."""
    name = "l1"

    def evaluate_t(self, W):
        return W.abs().sum()

    def proxoperator(self, W, lam):
        return torch.sign(W) * torch.clamp(W.abs() - lam, min=0)


REGULARIZERS = {"none": NoRegularizer, "l2": L2Regularizer, "l1": L1Regularizer}


def make_regularizer(name):
    """Reference CLI codes: 0 none, 1 l2, 2 l1."""
    if isinstance(name, int):
        name = ["none", "l2", "l1"][name]
    return REGULARIZERS[name.lower()]()
