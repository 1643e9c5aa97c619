"""python-skylark ``skylark.ml.utils`` (``python-skylark/skylark/ml/utils.py``):
indicator coding of class labels and its decoding, on tensors."""
from __future__ import annotations

import numpy as np
import torch


def dummycoding(Y, K: int | None = None, zerobased: bool = False, dtype=torch.float64, device=None) -> torch.Tensor:
    """n x K indicator matrix (1 at the label's column) of labels 1..K (or
    0..K-1 with ``zerobased``); K is inferred from the largest label if None."""
    y = torch.as_tensor(np.asarray(Y, dtype=np.int64) if not isinstance(Y, torch.Tensor) else Y).reshape(-1)
    y = y.to(torch.int64)
    if not zerobased:
        y = y - 1
    if y.numel() and int(y.min()) < 0:
        raise ValueError("dummycoding: label below the first class")
    n = int(y.max()) + 1 if K is None else int(K)
    out = torch.zeros(y.numel(), n, dtype=dtype, device=device)
    out[torch.arange(y.numel(), device=out.device), y.to(out.device)] = 1.0
    return out


def dummydecode(pred, zerobased: bool = False) -> torch.Tensor:
    """Labels from per-class scores (argmax over columns), 1-based unless ``zerobased``."""
    p = torch.as_tensor(pred) if not isinstance(pred, torch.Tensor) else pred
    lab = torch.argmax(p, dim=1)
    return lab if zerobased else lab + 1
