"""Quasi-Monte-Carlo sequences (reference ``base/quasirand.hpp:9-113``).

``LeapedHaltonSequence(d, leap)``: ``coordinate(idx, i) =
RadicalInverse(prime(i), idx * leap)`` with the reference's 1-based radical
inverse (``idx + 1``) and ``prime(0) = 2``; default ``leap = prime(d)``.
Serialised as ``{"skylark_object_type": "qmc_sequence", "sequence_type":
"leaped halton", "d": .., "leap": ..}``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from .. import __version__


def primes(n: int) -> np.ndarray:
    """First n primes (prime(0) = 2)."""
    if n <= 0:
        return np.zeros(0, dtype=np.int64)
    limit = max(16, int(n * (np.log(n + 2) + np.log(np.log(n + 3)) + 3)))
    while True:
        sieve = np.ones(limit + 1, dtype=bool)
        sieve[:2] = False
        for i in range(2, int(limit ** 0.5) + 1):
            if sieve[i]:
                sieve[i * i::i] = False
        ps = np.nonzero(sieve)[0]
        if len(ps) >= n:
            return ps[:n].astype(np.int64)
        limit *= 2


def prime(i: int) -> int:
    return int(primes(i + 1)[i])


def radical_inverse(base: int, idx: int) -> float:
    r, m, res = 0.0, 1.0 / base, idx + 1
    while res > 0:
        r += m * (res % base)
        res //= base
        m /= base
    return r


class LeapedHaltonSequence:
    sequence_type = "leaped halton"

    def __init__(self, d: int, leap: int | None = None):
        self.d = int(d)
        self.leap = int(leap) if leap is not None and leap != -1 else prime(self.d)

    def coordinate(self, idx: int, i: int) -> float:
        return radical_inverse(prime(i), idx * self.leap)

    def block(self, start: int, n: int, dims: int, device=None) -> torch.Tensor:
        """Points ``start .. start+n-1``, coordinates ``0 .. dims-1`` (n x dims, float64)."""
        from ..ops import _lib
        ps = torch.from_numpy(primes(dims))
        out = torch.empty(n, dims, dtype=torch.float64)
        # RadicalInverse(p, idx*leap) with the 1-based offset folded in: native
        # kernel computes RI(p, k) for k = (skip + i) * leap; we add 1 here.
        vals = np.empty((n, dims))
        idx = (np.arange(start, start + n, dtype=np.int64) * self.leap + 1)
        for j, p in enumerate(primes(dims)):
            vals[:, j] = _ri_vec(int(p), idx)
        out = torch.from_numpy(vals)
        return out.to(device) if device is not None else out

    def to_dict(self) -> dict:
        return {"skylark_object_type": "qmc_sequence", "skylark_version": __version__,
                "sequence_type": self.sequence_type, "d": self.d, "leap": self.leap}

    @classmethod
    def from_dict(cls, d: dict):
        return cls(int(d["d"]), int(d["leap"]))


def _ri_vec(base: int, ks: np.ndarray) -> np.ndarray:
    """Vectorised radical inverse of integer array ks (already 1-based)."""
    r = np.zeros(ks.shape, dtype=np.float64)
    m = 1.0 / base
    res = ks.copy()
    while np.any(res > 0):
        r += m * (res % base)
        res //= base
        m /= base
    return r


def from_dict(d: dict):
    if d.get("sequence_type", "leaped halton") != "leaped halton":
        raise ValueError(f"unknown QMC sequence {d.get('sequence_type')}")
    return LeapedHaltonSequence.from_dict(d)
