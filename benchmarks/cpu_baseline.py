"""Host (CPU) baseline for the headline workload: the reference
publishes no number on "FJLT + randomized rank-20 SVD of 1e6 x 1e3 dense", so
this times the same algorithm -- the reference's ``ApproximateSVD``
(``nla/svd.hpp``: sketch, q power iterations with re-orthonormalisation, final
basis, small SVD) with an FJLT test matrix (``sketch/FJLT_Elemental.hpp``:
random signs, DCT, uniform row sample) -- in NumPy/SciPy on the host, the way
the reference's pure-Python fallbacks (``python-skylark/skylark/sketch.py``
``_ppyapply``) run it.  fp32 (NumPy has no bf16; fp32 GEMMs are the fastest
host path, so this is generous to the CPU).

usage: python benchmarks/cpu_baseline.py [--rows 1000000] [--cols 1000] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import scipy.fft
import scipy.linalg


def fjlt_test_matrix(n, k, rng):
    """n x k matrix Omega with A @ Omega = FJLT sketch of A's rows."""
    d = rng.choice(np.array([-1.0, 1.0], np.float32), n)
    H = scipy.fft.dct(np.eye(n, dtype=np.float32), norm="ortho", axis=0)   # orthonormal DCT-II
    rows = rng.integers(0, n, k)
    return (np.sqrt(n / k) * (H[rows] * d[None, :])).T.astype(np.float32)


def randsvd(A, rank, iters, rng):
    n = A.shape[1]
    k = 2 * rank
    Y = A @ fjlt_test_matrix(n, k, rng)
    Q, _ = np.linalg.qr(Y)
    for _ in range(iters):
        Z, _ = np.linalg.qr(A.T @ Q)
        Q, _ = np.linalg.qr(A @ Z)
    B = Q.T @ A
    Ub, s, Vt = scipy.linalg.svd(B, full_matrices=False)
    return (Q @ Ub)[:, :rank], s[:rank], Vt[:rank].T


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--rank", type=int, default=20)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rng = np.random.default_rng(1234)
    A = np.empty((a.rows, a.cols), np.float32)
    blk = 100_000
    for i in range(0, a.rows, blk):
        A[i:i + blk] = rng.standard_normal((min(blk, a.rows - i), a.cols), dtype=np.float32)
    randsvd(A, a.rank, a.iters, rng)          # warm-up (BLAS threads, page faults)
    ts = []
    for _ in range(a.steps):
        t = time.perf_counter()
        _, s, _ = randsvd(A, a.rank, a.iters, rng)
        ts.append(time.perf_counter() - t)
    ms = 1e3 * min(ts)
    row = {"metric": "randSVD wall-clock, host NumPy/SciPy baseline (same algorithm)", "ms_per_step": round(ms, 1),
           "bf16_equiv_GBps": round(a.rows * a.cols * 2 / (ms / 1e3) / 1e9, 2),
           "host_threads": os.cpu_count(), "dtype": "fp32",
           "config": {"rows": a.rows, "cols": a.cols, "rank": a.rank, "iters": a.iters, "sketch": "FJLT"},
           "top_singular_values": [round(float(x), 3) for x in s[:3]]}
    print(json.dumps(row))
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
