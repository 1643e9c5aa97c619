"""Per-phase cycle breakdown of the v2 fused pass (diagnostic s_memtime build):
average cycles per row block per phase, over all waves of all workgroups.
usage: python benchmarks/tsk_stamps.py"""
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
_lib.register("sl_tsk2_stamp_pass", [vp, i64, i64, i64, vp, i32, vp, i64, vp, vp, i32, i32, vp])
PHASES = ["wait_vm", "partial_sum", "barrier1", "steps3_4", "step1_publish", "barrier_end"]


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
        for ypb in (1, 2):
            for _ in range(3):
                dbg.zero_()
                _lib.call("sl_tsk2_stamp_pass", _lib.ptr(A), m, n, n, _lib.ptr(Zt), k, _lib.ptr(ws), ws.numel(),
                          _lib.ptr(Y), _lib.ptr(dbg), final, ypb, st)
            torch.cuda.synchronize()
            d = dbg.view(256, 8, 8).double()
            blocks = d[:, 0, 6].sum()
            per = (d[:, :, :6].sum(dim=(0, 1)) / (8 * (blocks - 2 * 256))).tolist()
            rec = {"final": final, "ypb": ypb, "cycles_per_block": {p: round(v, 1) for p, v in zip(PHASES, per)},
                   "total": round(sum(per), 1)}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
