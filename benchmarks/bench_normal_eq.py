"""One-pass A^T (A y) (ata_kernels.hip) vs the two-GEMV reference on LSRN's
per-GPU block (1.25e6 x 5e3 f32 = 25 GB): time and effective GB/s of A.

usage: python benchmarks/bench_normal_eq.py [--rows 1.25e6] [--cols 5000] [--reps 5]"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import normal_eq, rng  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1.25e6)
    ap.add_argument("--cols", type=int, default=5000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for m, n in ((int(a.rows), a.cols), (1_000_000, 1024), (1_000_000, 2048)):
        run(m, n, dev, a.reps)


def run(m, n, dev, reps):
    A = torch.empty(m, n, device=dev)
    rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
    gb = m * n * 4 / 1e9
    for k in (1, 2, 4):
        if not normal_eq.native_ok(A, k):
            continue
        y = torch.randn(n, k, device=dev)
        W, Y = normal_eq.ata(A, y, want_y=True)
        Yr = A @ y
        Wr = A.t() @ Yr
        err = float((W - Wr).norm() / Wr.norm())
        Dt = torch.randn(k, m, device=dev)
        for name, fn in (("fused_ata", lambda: normal_eq.ata(A, y)),
                         ("dual_AtD", lambda: normal_eq.dual(A, Dt.t())),
                         ("dual_AtD_AX", lambda: normal_eq.dual(A, Dt.t(), y)),
                         ("fused_ata_storeY", lambda: normal_eq.ata(A, y, want_y=True)),
                         ("torch_two_gemv", lambda: A.t() @ (A @ y))):
            t = timeit(fn, reps)
            print(json.dumps({"bench": "normal_eq", "variant": name, "m": m, "n": n, "k": k,
                              "ms": round(t * 1e3, 3), "GBps_of_A": round(gb / t, 1),
                              "rel_err_vs_torch": err}), flush=True)


if __name__ == "__main__":
    main()
