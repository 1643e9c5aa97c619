"""Random-stream context (reference ``base/context.hpp:19-183``).

A :class:`Context` is ``(seed, counter)``.  Every random allocation reserves
``size`` consecutive counter slots and advances the counter, so all ranks that
issue the same sequence of allocations stay in sync *without communication*
(the reference's key reproducibility invariant).  The arrays themselves are
lazy: :class:`RandomSamplesArray` only records ``(seed, base, size,
distribution)`` and realises entries on demand, on the host or on a GPU.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import __version__
from . import distributions as D


class Context:
    """Holds the random-stream state ``(seed, counter)``."""

    def __init__(self, seed: int = 0, counter: int = 0):
        self.seed = int(seed)
        self.counter = int(counter)

    # ---------------------------------------------------------- allocation
    def allocate_random_samples_array(self, size: int, dist: "D.Distribution") -> "RandomSamplesArray":
        arr = RandomSamplesArray(self.seed, self.counter, int(size), dist)
        self.counter += int(size)
        return arr

    def generate_random_samples_array(self, size: int, dist: "D.Distribution",
                                      device=None, dtype=torch.float64) -> torch.Tensor:
        """Reserve and immediately realise ``size`` samples as a 1-D tensor."""
        arr = self.allocate_random_samples_array(size, dist)
        return arr.realize(device=device, dtype=dtype)

    def allocate_random_array(self, size: int) -> "RandomSamplesArray":
        return self.allocate_random_samples_array(size, D.UniformInt(0, 2**31 - 1))

    def random_value(self, dist: "D.Distribution") -> float:
        v = self.generate_random_samples_array(1, dist)
        return float(v[0])

    def random_int(self) -> int:
        return int(self.generate_random_samples_array(1, D.UniformInt(0, 2**31 - 1), dtype=torch.int64)[0])

    def get_counter(self) -> int:
        return self.counter

    def copy(self) -> "Context":
        return Context(self.seed, self.counter)

    # ------------------------------------------------------- serialization
    def to_dict(self) -> dict:
        return {"skylark_object_type": "context", "skylark_version": __version__,
                "seed": self.seed, "counter": self.counter}

    to_ptree = to_dict

    def to_json(self) -> str:
        return json.dumps(self.to_dict())

    @classmethod
    def from_dict(cls, d: dict) -> "Context":
        return cls(int(d["seed"]), int(d["counter"]))

    @classmethod
    def from_json(cls, s: str) -> "Context":
        return cls.from_dict(json.loads(s))

    def __repr__(self):
        return f"Context(seed={self.seed}, counter={self.counter})"

    def __eq__(self, other):
        return isinstance(other, Context) and (self.seed, self.counter) == (other.seed, other.counter)


@dataclass
class RandomSamplesArray:
    """Lazy, random-access array of samples (reference ``base/randgen.hpp:17-122``).

    Entry ``i`` is ``dist`` applied to Threefry-2x64-13 at counter
    ``base + i`` keyed by ``seed``.  Realisation never needs the other
    entries, so a shard can be produced locally on any device.
    """

    seed: int
    base: int
    size: int
    dist: "D.Distribution" = field(default_factory=lambda: D.Normal())

    def __len__(self):
        return self.size

    def realize(self, start: int = 0, count: int | None = None, device=None,
                dtype=torch.float64, scale: float = 1.0) -> torch.Tensor:
        """Materialise entries ``[start, start+count)`` as a 1-D tensor."""
        from ..ops import rng as _rng
        count = self.size - start if count is None else int(count)
        if start < 0 or start + count > self.size:
            raise IndexError("random samples array: index out of range")
        if dtype in (torch.int64, torch.int32):
            if not isinstance(self.dist, D.UniformInt):
                raise TypeError("integer realisation requires a UniformInt distribution")
            out = _rng.random_int(self.seed, self.base + start, count, self.dist.lo, self.dist.hi,
                                  device=device)
            return out.to(dtype)
        out = torch.empty(count, dtype=dtype, device=device)
        _rng.fill_random(out.view(count, 1), self.dist, self.seed, self.base + start,
                         ir=1, ic=0, scale=scale, precise=True)
        return out

    def __getitem__(self, i: int):
        if isinstance(self.dist, D.UniformInt):
            return int(self.realize(i, 1, dtype=torch.int64)[0])
        return float(self.realize(i, 1)[0])

    def to_numpy(self) -> np.ndarray:
        if isinstance(self.dist, D.UniformInt):
            return self.realize(dtype=torch.int64).numpy()
        return self.realize().numpy()
