"""Normal realisation rate of a dense-sketch panel (LSRN: 2e4 x 13421 bf16,
column-major stream), vectorised line kernel vs the generic fill kernel.

usage: python benchmarks/bench_rng.py"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import _lib, rng  # noqa: E402


def main():
    lib = _lib.require()
    dev = torch.device("cuda")
    for dt, (t, b) in ((torch.bfloat16, (20000, 13421)), (torch.float32, (20000, 6710))):
        P = torch.empty(t, b, dtype=dt, device=dev)
        for fast in (0, 1):
            lib.sl_rng_set_fast_lines(fast)
            rng.fill_random(P, D.Normal(), 7, 0, r0=0, c0=0, ir=1, ic=20000)
            torch.cuda.synchronize()
            reps = 5
            t0 = time.perf_counter()
            for i in range(reps):
                rng.fill_random(P, D.Normal(), 7, 0, r0=0, c0=i * b, ir=1, ic=20000)
            torch.cuda.synchronize()
            dtm = (time.perf_counter() - t0) / reps
            print(json.dumps({"bench": "fill_normal", "kernel": "lines" if fast else "generic", "dtype": str(dt),
                              "shape": [t, b], "ms": round(dtm * 1e3, 3),
                              "Gsamples_per_s": round(t * b / dtm / 1e9, 1)}), flush=True)
    lib.sl_rng_set_fast_lines(1)


if __name__ == "__main__":
    main()
