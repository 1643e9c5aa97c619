"""Chebyshev spectral helpers (reference ``nla/spectral.hpp:17-92``), used by
the time-dependent PageRank of the graph module."""
from __future__ import annotations

import math

import torch


def chebyshev_points(N: int, a: float = -1.0, b: float = 1.0, dtype=torch.float64) -> torch.Tensor:
    """N Chebyshev (extrema) points mapped to [a, b], as the reference computes them."""
    s = (b - a) / 2.0
    M = N - 1
    x = torch.tensor([(math.cos(j * math.pi / M) + a + 1) * s for j in range(M + 1)], dtype=dtype)
    if M % 2 == 0:
        x[M // 2] = 0.0
    return x


def chebyshev_diff_matrix(N: int, a: float = -1.0, b: float = 1.0, dtype=torch.float64):
    """(D, X): Chebyshev differentiation matrix on N points and the points."""
    x = chebyshev_points(N, dtype=dtype)
    M = N - 1
    D = torch.empty(M + 1, M + 1, dtype=dtype)
    for j in range(M + 1):
        for i in range(M + 1):
            d = i - j
            v = 2.0 / (b - a)
            if i == 0 and j == 0:
                v *= (2.0 * M * M + 1.0) / 6.0
            elif i == M and j == M:
                v *= -(2.0 * M * M + 1.0) / 6.0
            else:
                if i == 0 or i == M:
                    v *= 2.0
                if j == 0 or j == M:
                    v /= 2.0
                if d == 0:
                    v *= -x[j] / (2.0 * (1 - x[j] * x[j]))
                elif d % 2 == 0:
                    v *= 1.0 / (x[i] - x[j])
                else:
                    v *= -1.0 / (x[i] - x[j])
            D[i, j] = v
    if a != -1 or b != 1:
        x = a + (x + 1.0) * (b - a) / 2.0
    return D, x


ChebyshevPoints = chebyshev_points
ChebyshevDiffMatrix = chebyshev_diff_matrix
