"""Ablation of the fused tall-skinny pass: time the kernel with steps removed
(runtime mask, so nothing is dead-code-eliminated) in interleaved rounds.
Results are wrong in ablated runs by design; only the timing matters."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ctypes as C
import statistics
import sys
import time

import torch

from libskylark_amd.base import distributions as D
from libskylark_amd.ops import _lib, rng, tallskinny  # noqa: F401  (registers the sl_tsk_* signatures)


def main():
    m, n, k = 1_000_000, 1000, int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda")
    lda = int(os.environ.get("LDA", n))   # padded leading dimension (elements)
    A = torch.empty(m, lda, dtype=torch.bfloat16, device=dev)[:, :n]
    rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
    Zt = (torch.randn(k, n, device=dev) / 30).to(torch.bfloat16)
    W = torch.empty(n, k, device=dev)
    G = torch.empty(k, k, device=dev)
    lib = _lib.require()
    ws = torch.empty(tallskinny.fused_workspace_bytes(m, n, k), dtype=torch.uint8, device=dev)
    lib.sl_tsk_set_ablate.argtypes = [C.c_int]
    lib.sl_tsk_set_nbuf.argtypes = [C.c_int]
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        _lib.call("sl_tsk_fused_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt), k, _lib.ptr(W), _lib.ptr(G),
                  None, 0, _lib.ptr(ws), flags[0], st)

    flags = [0]
    variants = {"full": 0, "k32_step3": 16, "hi_only": 32, "hi_only_nog": 40, "no_step1": 1, "no_step2": 2,
                "no_step3": 4, "no_step4": 8, "no_3_4": 12, "loads_only": 15,
                "loads_only_nt": 79, "full_nt": 64, "hi_only_nog_nt": 104}
    res = {v: [] for v in variants}
    for nb in (3, 4, 5):
        lib.sl_tsk_set_nbuf(nb)
        for name, ab in variants.items():
            lib.sl_tsk_set_ablate(ab)
            run()
    for _ in range(5):
        for nb in (4,):
            lib.sl_tsk_set_nbuf(nb)
            for name, ab in variants.items():
                lib.sl_tsk_set_ablate(ab)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5):
                    run()
                torch.cuda.synchronize()
                res[name].append((time.perf_counter() - t0) / 5)
    lib.sl_tsk_set_ablate(0)
    for name, ts in res.items():
        med = statistics.median(ts)
        print(f"{name:12s} {med*1e6:8.1f} us  {m*n*2/med/1e9:7.1f} GB/s")


if __name__ == "__main__":
    main()
