"""Kernel micro-benchmarks for the randSVD hot path (run on the GPU box).

Interleaved rounds in ONE process (CDNA HIP guide rule 24): for each variant
the median over rounds is reported, with the effective HBM bandwidth of the
bytes the kernel must move.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import argparse
import json
import statistics
import time

import torch

from libskylark_amd.base import distributions as D
from libskylark_amd.ops import _lib, rng, tallskinny


def timed(fn, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1_000_000)
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--k", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m, n, k = a.m, a.n, a.k
    A = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
    Z = torch.randn(n, k, device=dev) / 30
    Y = torch.randn(m, k, device=dev)
    Mx = torch.randn(k, k, device=dev)
    _lib.require()
    abytes = A.numel() * 2
    res = {}

    variants = {
        "fused": (None, lambda: tallskinny.fused_pass(A, Z), abytes),
        "fused_keepy": (None, lambda: tallskinny.fused_pass(A, Z, keep_y=True), abytes + m * k * 4),
        "matmul_zsplit": (None, lambda: tallskinny.matmul(A, Z), abytes + m * k * 4),
        "f32_gram_ident": (None, lambda: tallskinny.f32_xm(Y, None, store=False, gram=True), m * k * 4),
        "f32_gram_xm": (None, lambda: tallskinny.f32_xm(Y, Mx, store=False, gram=True), m * k * 4),
        "f32_xm_store20": (None, lambda: tallskinny.f32_xm(Y, Mx[:, :20].contiguous(), store=True), m * k * 4 + m * 20 * 4),
        "hipblaslt_A_Z_bf16": (None, lambda: torch.mm(A, Z.bfloat16(), out_dtype=torch.float32), abytes + m * k * 4),
        "hipblaslt_At_Y_bf16": (None, lambda: torch.mm(A.t(), Y.bfloat16(), out_dtype=torch.float32), abytes + m * k * 2),
        "copy_A": (None, lambda: A.clone(), 2 * abytes),
    }
    times = {name: [] for name in variants}
    for name, (pre, fn, _) in variants.items():  # warm-up
        if pre:
            pre()
        fn()
    for _ in range(a.rounds):
        for name, (pre, fn, _) in variants.items():
            if pre:
                pre()
            times[name].append(timed(fn))
    for name, (_, _, by) in variants.items():
        med = statistics.median(times[name])
        res[name] = {"median_us": round(med * 1e6, 1), "min_us": round(min(times[name]) * 1e6, 1),
                     "GBps": round(by / med / 1e9, 1)}
        print(f"{name:24s} {med*1e6:9.1f} us  {by/med/1e9:8.1f} GB/s")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"shape": [m, n, k], "results": res}, f, indent=1)


if __name__ == "__main__":
    main()
