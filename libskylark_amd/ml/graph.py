"""Graph analytics: local community detection (TD-PPR) and spectral embeddings.

* :class:`SimpleGraph` — undirected, unweighted graph from an edge list /
  arc-list file (self loops and duplicate edges dropped, like the
  reference's ``simple_unweighted_graph_t`` in ``ml/skylark_community.cpp``),
  stored as CSR over dense vertex ids with a label <-> id map.
* :func:`time_dependent_ppr` / :func:`find_local_cluster` — reference
  ``ml/graph/local_computations.hpp:50-370``.  The collocation operator is
  built here (Chebyshev differentiation on [0, gamma], QR, pseudo-inverse,
  cached per (N, gamma)); the push loop and the sweep cut run in the native
  host library (``sl_td_ppr`` / ``sl_local_cluster``, C++).
* :func:`approximate_ase` — adjacency spectral embedding ``V sqrt(S)`` via
  :func:`..nla.approximate_symmetric_svd` (``spectral_embedding.hpp:11-92``).
"""
from __future__ import annotations

import ctypes as C
import math
from functools import lru_cache

import numpy as np
import torch

from ..base.context import Context
from ..ops import _lib as L

L.register("sl_td_ppr", [L.i64, L.vp, L.vp, L.vp, L.vp, L.i64, L.vp, L.i32, L.i32, L.f64, L.f64, L.vp, L.vp,
                         L.vp])
L.register("sl_local_cluster", [L.i64, L.vp, L.vp, L.i64, L.vp, L.i64, L.vp, L.i32, L.i32, L.f64, L.f64, L.i32,
                                L.vp, L.vp, L.vp])


class SimpleGraph:
    def __init__(self, edges, labels=None):
        """``edges``: (E, 2) array of vertex labels (any hashable ints)."""
        e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
        e = e[e[:, 0] != e[:, 1]]
        if labels is None:
            labels, inv = np.unique(e.reshape(-1), return_inverse=True)
            e = inv.reshape(-1, 2)
        else:
            labels = np.asarray(labels, dtype=np.int64)
            lut = {int(v): i for i, v in enumerate(labels)}
            e = np.vectorize(lut.__getitem__)(e) if e.size else e
        n = len(labels)
        sym = np.concatenate([e, e[:, ::-1]], axis=0)
        key = np.unique(sym[:, 0] * n + sym[:, 1])
        src, dst = key // n, key % n
        self.n = n
        self.labels = labels
        self.index = {int(v): i for i, v in enumerate(labels)}
        self.rowptr = np.zeros(n + 1, dtype=np.int64)
        np.add.at(self.rowptr, src + 1, 1)
        self.rowptr = np.cumsum(self.rowptr).astype(np.int64)
        self.col = dst.astype(np.int64)
        self.num_edges_ = int(len(self.col))

    @classmethod
    def from_file(cls, fname: str):
        """Arc-list text: one ``u v`` per line, ``#`` comments.  ``fname`` may
        be an fsspec URL (``hdfs://namenode/path``, ...), streamed line by line."""
        rows = []
        if "://" in fname:
            from ..io.remote import LineStreamer
            f = LineStreamer(fname)
        else:
            f = open(fname)
        with f:
            for line in f:
                if not line.strip() or line.startswith("#"):
                    continue
                t = line.split()
                rows.append((int(t[0]), int(t[1])))
        return cls(np.array(rows, dtype=np.int64).reshape(-1, 2))

    def num_vertices(self):
        return self.n

    def num_edges(self):
        """Twice the number of undirected edges (reference convention)."""
        return self.num_edges_

    def degree(self, v):
        i = self.index[int(v)]
        return int(self.rowptr[i + 1] - self.rowptr[i])

    def neighbors(self, v):
        i = self.index[int(v)]
        return [int(self.labels[j]) for j in self.col[self.rowptr[i]:self.rowptr[i + 1]]]

    def adjacency_matrix(self, dtype=torch.float64, device=None) -> torch.Tensor:
        """Sparse CSR adjacency in vertex-id order (``indexmap = labels``)."""
        vals = torch.ones(len(self.col), dtype=dtype)
        A = torch.sparse_csr_tensor(torch.from_numpy(self.rowptr), torch.from_numpy(self.col), vals,
                                    (self.n, self.n))
        return A.to(device) if device is not None else A


@lru_cache(maxsize=64)
def _min_n(epsilon: float, gamma: float) -> int:
    from scipy.special import iv
    minN = 10
    Cc = 20.0 * math.sqrt(minN) * math.exp(-gamma / 2)
    while Cc * iv(minN, gamma) * 0.8 ** minN > epsilon / (gamma * (1 + (2 / math.pi) * math.log(minN - 1))):
        minN += 1
    return minN


@lru_cache(maxsize=64)
def _collocation(N: int, gamma: float):
    """Row-major N x N operator (reference ``Dmap`` construction)."""
    from ..nla.spectral import chebyshev_diff_matrix
    D0, _ = chebyshev_diff_matrix(N, 0.0, gamma)
    D0 = D0.numpy() + np.eye(N)
    Q, R = np.linalg.qr(D0)
    D = np.zeros((N, N))
    D[N - 1, :] = Q[:, N - 1]
    R1 = np.linalg.pinv(R[:N - 1, :N - 1])
    D[:N - 1, :] = R1 @ Q[:, :N - 1].T
    return np.ascontiguousarray(D)


def _setup(alpha, gamma, epsilon, NX):
    minN = _min_n(float(epsilon), float(gamma))
    N = minN if minN % NX == 0 else (minN // NX + 1) * NX
    NR = N // NX
    from ..nla.spectral import chebyshev_points
    x1 = chebyshev_points(N, 0.0, gamma).numpy()
    x = np.array([x1[i * NR] for i in range(NX)])
    LC = 1 + (2 / math.pi) * math.log(N - 1)
    Cc = ((1 - alpha) * epsilon / ((1 - math.exp((alpha - 1) * gamma)) * LC)) if alpha < 1 else epsilon / (gamma * LC)
    return N, _collocation(N, float(gamma)), x, Cc


def _p(a):
    return C.c_void_p(a.ctypes.data)


def time_dependent_ppr(G: SimpleGraph, seeds: dict, alpha=0.85, gamma=5.0, epsilon=0.001, NX=4):
    """Returns ``(y, x)``: ``y`` maps vertex label -> NX values at times ``x``."""
    N, D, x, Cc = _setup(alpha, gamma, epsilon, NX)
    sid = np.array([G.index[int(v)] for v in seeds], dtype=np.int64)
    sval = np.array([float(v) for v in seeds.values()], dtype=np.float64)
    nodes = np.zeros(G.n, dtype=np.int64)
    y = np.zeros((G.n, NX), dtype=np.float64)
    nout = np.zeros(1, dtype=np.int64)
    L.call("sl_td_ppr", G.n, _p(G.rowptr), _p(G.col), _p(sid), _p(sval), len(sid), _p(D), N, NX, float(alpha),
           float(Cc), _p(nodes), _p(y), _p(nout))
    k = int(nout[0])
    return {int(G.labels[nodes[i]]): y[i].copy() for i in range(k)}, x


def find_local_cluster(G: SimpleGraph, seeds, alpha=0.85, gamma=5.0, epsilon=0.001, NX=4, recursive=False):
    """Returns ``(cluster_labels_set, conductance)``."""
    N, D, _, Cc = _setup(alpha, gamma, epsilon, NX)
    sid = np.array(sorted(G.index[int(v)] for v in seeds), dtype=np.int64)
    out = np.zeros(G.n, dtype=np.int64)
    ncl = np.zeros(1, dtype=np.int64)
    cond = np.zeros(1, dtype=np.float64)
    L.call("sl_local_cluster", G.n, _p(G.rowptr), _p(G.col), G.num_edges_, _p(sid), len(sid), _p(D), N, NX,
           float(alpha), float(Cc), int(recursive), _p(out), _p(ncl), _p(cond))
    return {int(G.labels[i]) for i in out[:int(ncl[0])]}, float(cond[0])


def approximate_ase(G: SimpleGraph, k: int, context: Context | None = None, params=None, device=None):
    """Adjacency spectral embedding: returns ``(X, indexmap)`` with X n x k."""
    from .. import nla
    A = G.adjacency_matrix(device=device)
    V, S = nla.approximate_symmetric_svd(A, k, context, params)
    X = V * S.abs().sqrt()[None, :]
    return X, list(int(v) for v in G.labels)


TimeDependentPPR = time_dependent_ppr
FindLocalCluster = find_local_cluster
ApproximateASE = approximate_ase
