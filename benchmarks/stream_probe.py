"""Load-pipeline probe for the fused tall-skinny pass: leading dimension
(1000 vs 1024-padded rows), non-temporal LDS-DMA, ring depth, with the
compute steps ablated or not.  Timing only (ablated results are wrong)."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ctypes as C
import statistics
import time

import torch

from libskylark_amd.base import distributions as D
from libskylark_amd.ops import _lib, rng


def main():
    m, n, k = 1_000_000, 1000, 40
    dev = torch.device("cuda")
    lib = _lib.require()
    lib.sl_tsk_set_ablate.argtypes = [C.c_int]
    lib.sl_tsk_set_nbuf.argtypes = [C.c_int]
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    Zt = (torch.randn(k, n, device=dev) / 30).to(torch.bfloat16)
    W = torch.empty(n, k, device=dev)
    G = torch.empty(k, k, device=dev)
    ws = torch.empty(int(lib.sl_tsk_fused_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    mats = {}
    for ld in (1000, 1024):
        buf = torch.empty(m, ld, dtype=torch.bfloat16, device=dev)
        rng.fill_random(buf, D.Normal(), 1, 0, ir=ld, ic=1)
        mats[ld] = buf[:, :n]
    res = {}

    def run(A, flags):
        _lib.call("sl_tsk_fused_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt), k, _lib.ptr(W), _lib.ptr(G),
                  None, 0, _lib.ptr(ws), flags, st)

    cases = []
    for ld in (1000, 1024):
        for nt in (0, 64):
            for nb in (4, 5):
                for name, ab, fl in (("loads", 15, 0), ("inter", 0, 3), ("final", 0, 0)):
                    cases.append((f"ld{ld} nt{int(bool(nt))} nb{nb} {name}", ld, ab | nt, nb, fl))
    for c in cases:
        res[c[0]] = []
    for rep in range(4):
        for label, ld, ab, nb, fl in cases:
            lib.sl_tsk_set_nbuf(nb)
            lib.sl_tsk_set_ablate(ab)
            run(mats[ld], fl)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                run(mats[ld], fl)
            torch.cuda.synchronize()
            if rep:
                res[label].append((time.perf_counter() - t0) / 5)
    lib.sl_tsk_set_ablate(0)
    lib.sl_tsk_set_nbuf(4)
    for label, ts in res.items():
        med = statistics.median(ts)
        print(f"{label:28s} {med*1e6:8.1f} us  {m*n*2/med/1e12:6.2f} TB/s(useful)", flush=True)


if __name__ == "__main__":
    main()
