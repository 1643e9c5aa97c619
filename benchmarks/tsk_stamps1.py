"""Per-phase cycle breakdown of the v1 fused pass (diagnostic s_memtime build
``sl_tsk_stamp_pass``): average cycles per row block per phase over all waves.
usage: python benchmarks/tsk_stamps1.py"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import _lib, rng, tallskinny as T  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_tsk_stamp_pass", [vp, i64, i64, i64, vp, i32, vp, vp, vp, i32, vp])
PHASES = ["dma_wait", "step1", "partial_write_barrier1", "reduce_barrier2", "y_fragments", "step3_4"]


def main():
    m, n, k = 1_000_000, 1000, 40
    dev = torch.device("cuda")
    A = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
    Zt = (torch.randn(k, n, device=dev) / 30).to(torch.bfloat16)
    ws = torch.zeros(T.fused_workspace_bytes(m, n, k), dtype=torch.uint8, device=dev)
    Y = torch.empty(m, k, device=dev)
    dbg = torch.zeros(256 * 8 * 8, dtype=torch.int64, device=dev)
    st = vp(torch.cuda.current_stream().cuda_stream)
    for final in (0, 1):
        for _ in range(3):
            dbg.zero_()
            _lib.call("sl_tsk_stamp_pass", _lib.ptr(A), m, n, n, _lib.ptr(Zt), k, _lib.ptr(ws), _lib.ptr(Y),
                      _lib.ptr(dbg), final, st)
        torch.cuda.synchronize()
        d = dbg.view(256, 8, 8).double()
        blocks = d[:, :, 6].clamp_min(3) - 2
        per = (d[:, :, :6] / blocks[:, :, None]).mean(dim=(0, 1))
        rec = {"pass": "final_g64" if final else "inter", "cycles_per_block": {p: round(float(v), 1)
                                                                               for p, v in zip(PHASES, per)},
               "total": round(float(per.sum()), 1)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
