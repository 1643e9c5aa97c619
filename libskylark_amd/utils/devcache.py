"""Device copies of a sketch's host-resident operands (its random diagonal,
sample indices, hash tables), kept per source tensor OBJECT: a sketch is
applied many times and re-uploading e.g. a 1e6-entry Rademacher vector from
pageable host memory on every application cost ~0.3 ms of a 3.4 ms FJLT.

The cache holds a weak reference and the tensor's version counter, so a
tensor that died (its memory possibly reused) or was modified in place is
never served stale."""
from __future__ import annotations

import weakref

import torch

_COPIES: dict = {}
_MAX = 32


def version_of(t: torch.Tensor) -> int:
    """``t._version``, or -1 for an inference tensor (created under
    ``torch.inference_mode()``: it has no version counter, and it cannot be
    modified in place outside inference mode, so identity alone keys it)."""
    if t.is_inference():
        return -1
    return t._version


def device_copy(t: torch.Tensor, dev, dtype=None) -> torch.Tensor:
    """``t.to(device=dev, dtype=dtype).contiguous()``, uploaded once per
    (tensor object, version, device, dtype)."""
    dtype = dtype or t.dtype
    dev = torch.device(dev)
    if t.device == dev and t.dtype == dtype and t.is_contiguous():
        return t
    key = (id(t), str(dev), dtype)
    hit = _COPIES.get(key)
    if hit is not None and hit[0]() is t and hit[1] == version_of(t):
        return hit[2]
    out = t.to(device=dev, dtype=dtype).contiguous()
    if len(_COPIES) >= _MAX:
        _COPIES.pop(next(iter(_COPIES)))
    _COPIES[key] = (weakref.ref(t), version_of(t), out)
    return out
