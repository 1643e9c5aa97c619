"""Final-pass cost split: fused pass timed with / without the Y store and
with exact (hi + lo) vs hi-only W, G skipped as in the randSVD plan
(interleaved rounds, one process)."""
from __future__ import annotations

import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ctypes as C  # noqa: E402

import torch  # noqa: E402

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import _lib, rng, tallskinny  # noqa: E402,F401  (registers the sl_tsk_* signatures)


def main():
    m, n, k = 1_000_000, 1000, 40
    dev = torch.device("cuda")
    A = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
    Zt = (torch.randn(k, n, device=dev) / 30).to(torch.bfloat16)
    W = torch.empty(n, k, device=dev)
    G = torch.empty(k, k, device=dev)
    Y = torch.empty(m, k, device=dev)
    lib = _lib.require()
    ws = torch.empty(tallskinny.fused_workspace_bytes(m, n, k), dtype=torch.uint8, device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run(store, flags):
        _lib.call("sl_tsk_fused_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt), k, _lib.ptr(W), _lib.ptr(G),
                  _lib.ptr(Y) if store else None, k if store else 0, _lib.ptr(ws), flags, st)

    variants = {"store_exact": (1, 1), "store_hi": (1, 3), "nostore_exact": (0, 1), "nostore_hi": (0, 3)}
    res = {v: [] for v in variants}
    for v in variants.values():
        run(*v)
    for _ in range(7):
        for name, v in variants.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                run(*v)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / 5)
    for name, ts in res.items():
        med = statistics.median(ts)
        print(f"{name:14s} {med*1e6:8.1f} us  {m*n*2/med/1e9:7.1f} GB/s of A", flush=True)


if __name__ == "__main__":
    main()
