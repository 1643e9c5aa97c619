"""Wide-row f32 GEMV (gemv_kernels.hip) against the library GEMV (torch) on a
stored kernel-Gram shape (default n = 1e5: 40 GB).  Prints one JSON line per
k.  usage: python benchmarks/bench_gemv.py [n]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libskylark_amd.ops import normal_eq  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    A = torch.empty(n, n, device="cuda")
    A.normal_()
    gb = A.numel() * 4 / 1e9
    for k in (1, 2, 4):
        X = torch.randn(n, k, device="cuda")
        ours = timeit(lambda: normal_eq.gemv(A, X))
        lib = timeit(lambda: A @ X)
        err = float((normal_eq.gemv(A, X) - A @ X).abs().max() / (A @ X).abs().max())
        print(json.dumps({"bench": "gemv_rows", "n": n, "k": k, "GB": round(gb, 1), "ours_ms": round(ours, 3),
                          "ours_TBps": round(gb / ours, 2), "lib_ms": round(lib, 3), "lib_TBps": round(gb / lib, 2),
                          "rel_diff": err}), flush=True)


if __name__ == "__main__":
    main()
