"""FJLT sketch with many samples on a tall f32 matrix (Blendenpik's t = 4n
sketch): the four-step sampled DCT (fjlt_fourstep.hip, the default), the
fused pre-pass + rocFFT rfft + sampled post-gather, and the torch DCT-II +
index_select composition.  Prints one JSON line per variant."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.ops import fut  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    m, n = int(os.environ.get("M", 1_000_000)), int(os.environ.get("NCOL", 1000))
    S = 4 * n
    dev = torch.device("cuda")
    A = torch.randn(m, n, device=dev)
    d = torch.where(torch.rand(m) < 0.5, -1.0, 1.0).double()
    smp = torch.randint(0, m, (S,))
    scale = (m / S) ** 0.5
    nbytes = m * n * 4

    def old():
        X = A * d.to(dev, torch.float32)[:, None]
        return fut.dct2(X, 0).index_select(0, smp.to(dev)) * scale

    def rfft():
        ok = fut.fourstep_ok
        fut.fourstep_ok = lambda *a: False
        try:
            return fut.fjlt_sampled(A, 0, d, smp, scale)
        finally:
            fut.fourstep_ok = ok

    def new():
        return fut.fjlt_fourstep(A, d, smp, scale)

    ref = old().double()
    only = os.environ.get("VARIANTS")
    for name, fn in (("torch_dct_gather", old), ("fused_rfft_sampled", rfft), ("fourstep_sampled", new)):
        if only and name not in only.split(","):
            continue
        err = float((fn().double() - ref).norm() / ref.norm())
        t = timeit(fn)
        print(json.dumps({"bench": "fjlt_sampled", "variant": name, "m": m, "n": n, "S": S, "ms": round(t * 1e3, 3),
                          "GBps_of_A": round(nbytes / t / 1e9, 1), "rel_diff_vs_torch": err}), flush=True)


if __name__ == "__main__":
    main()
