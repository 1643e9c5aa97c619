"""Dummy (one-vs-rest ±1) coding of class labels (reference ``ml/coding.hpp:7-146``).

Codes are assigned in order of FIRST APPEARANCE of each label (as the
reference does), not sorted.  For row-distributed labels the label vector is
all-gathered first (the reference copies to [*,*]) so every rank agrees on
the coding.
"""
from __future__ import annotations

import torch

from ..parallel.distmatrix import DistMatrix


def _labels_host(L):
    if isinstance(L, DistMatrix):
        L = L.to_global()
    if isinstance(L, torch.Tensor):
        return L.reshape(-1).detach().cpu().tolist()
    import numpy as np
    return np.asarray(L).reshape(-1).tolist()


def _canon(v):
    f = float(v)
    return int(f) if f.is_integer() else f


def dummy_coding(L, pval: float = 1.0, nval: float = -1.0, orientation: str = "normal", dtype=torch.float64,
                 device=None):
    """Return ``(Y, coding, rcoding)``: Y is n x c (``orientation="normal"``)
    or c x n ("adjoint") with ``pval`` at the label's code and ``nval``
    elsewhere; ``coding`` maps label -> column, ``rcoding`` column -> label."""
    labels = [_canon(v) for v in _labels_host(L)]
    coding, rcoding = {}, []
    for lab in labels:
        if lab not in coding:
            coding[lab] = len(rcoding)
            rcoding.append(lab)
    if device is None and isinstance(L, torch.Tensor):
        device = L.device
    idx = torch.tensor([coding[lab] for lab in labels], dtype=torch.long, device=device)
    Y = torch.full((len(labels), len(rcoding)), float(nval), dtype=dtype, device=device)
    Y[torch.arange(len(labels), device=device), idx] = float(pval)
    if orientation.lower() in ("adjoint", "transpose", "columns"):
        Y = Y.t().contiguous()
    return Y, coding, rcoding


def dummy_decode(Y: torch.Tensor, rcoding, orientation: str = "normal"):
    """Label of the max entry per example (rows for "normal", columns for "adjoint")."""
    if orientation.lower() in ("adjoint", "transpose", "columns"):
        Y = Y.t()
    idx = Y.argmax(dim=1).cpu().tolist()
    return [rcoding[i] for i in idx]


DummyCoding = dummy_coding
DummyDecode = dummy_decode
