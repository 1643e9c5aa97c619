"""Microbenchmarks of the per-iteration small kernels of the randSVD step
(k x k Cholesky/inverse implementations, CholeskyQR2 of an n x k iterate)."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import statistics

import torch

from libskylark_amd.ops import _lib
from libskylark_amd.ops import small_la as SL


def timeit(fn, reps=50):
    ts = []
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda")
    _lib.require()
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    for k in (16, 40, 64):
        X = torch.randn(4 * k, k, dtype=torch.float64, device=dev)
        G = X.t() @ X
        us = timeit(lambda: SL.chol_inv(G, st))
        print(f"chol_inv k={k:2d} aug  {us:8.1f} us", flush=True)
        us = timeit(lambda: SL.chol_inv_wave(G, st))
        print(f"chol_inv k={k:2d} wave {us:8.1f} us", flush=True)
    W = torch.randn(1000, 40, device=dev)
    print(f"cholqr2 1000x40      {timeit(lambda: SL.cholqr2(W, st)):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
