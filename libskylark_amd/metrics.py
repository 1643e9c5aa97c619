"""Prediction metrics used by the python-skylark examples
(``skylark.metrics.classification_accuracy`` in
``python-skylark/skylark/ml/nonlinear.py`` docstrings; the reference package
does not ship the module itself)."""
from __future__ import annotations

import numpy as np
import torch


def _host(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().double().numpy().reshape(-1)
    return np.asarray(v, dtype=np.float64).reshape(-1)


def classification_accuracy(predictions, labels) -> float:
    """Percentage of predictions equal to the labels."""
    p, y = _host(predictions), _host(labels)
    if p.shape != y.shape:
        raise ValueError(f"predictions ({p.shape[0]}) and labels ({y.shape[0]}) differ in length")
    return 100.0 * float((p == y).mean()) if p.size else 0.0


def rmse(predictions, targets) -> float:
    p, y = _host(predictions), _host(targets)
    return float(np.sqrt(np.mean((p - y) ** 2))) if p.size else 0.0


def relative_error(predictions, targets) -> float:
    """``|p - y| / |y|`` (2-norms), the regression error printed by the CLIs."""
    p, y = _host(predictions), _host(targets)
    return float(np.linalg.norm(p - y) / max(np.linalg.norm(y), np.finfo(float).tiny))
