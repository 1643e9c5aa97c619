"""Sample distributions over the counter-based stream
(reference ``utility/distributions.hpp:17-141``).

Each class carries the native sampler id (``sl_rng.hpp`` ``enum Dist``) and
up to two parameters.  The samplers are documented in ``sl_rng.hpp``.
"""
from __future__ import annotations

from dataclasses import dataclass


class Distribution:
    code: int = -1
    p0: float = 0.0
    p1: float = 0.0

    def params(self):
        return float(self.p0), float(self.p1)


@dataclass
class Normal(Distribution):
    code = 0


@dataclass
class Cauchy(Distribution):
    code = 1


@dataclass
class Rademacher(Distribution):
    code = 2


@dataclass
class Uniform(Distribution):
    a: float = 0.0
    b: float = 1.0
    code = 3

    @property
    def p0(self):
        return self.a

    @property
    def p1(self):
        return self.b


@dataclass
class Exponential(Distribution):
    code = 4


@dataclass
class Levy(Distribution):
    """Standard Lévy: 1/Z^2 (= 1/Gamma(1/2, scale 2) of the reference)."""
    code = 5


@dataclass
class ChiSquared(Distribution):
    k: float = 1.0
    code = 6

    @property
    def p0(self):
        return self.k


@dataclass
class UniformInt(Distribution):
    lo: int = 0
    hi: int = 1
    code = 7

    @property
    def p0(self):
        return float(self.lo)

    @property
    def p1(self):
        return float(self.hi)


@dataclass
class WZTValue(Distribution):
    """±(1/E)^(1/p), E ~ Exp(1) (reference sketch/WZT_data.hpp:27-130)."""
    p: float = 1.0
    code = 8

    @property
    def p0(self):
        return self.p


@dataclass
class SparseSign(Distribution):
    """±1/sqrt(d) with probability d/2 each, 0 otherwise (sparse JL entries)."""
    density: float = 1.0 / 3.0
    code = 9

    @property
    def p0(self):
        return self.density
