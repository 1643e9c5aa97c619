"""Per-phase cycle stamps of the v4 fused pass (diagnostic build
benchmarks/native/libpass_stamps.so = rsvd_pass.hip with -DSL_PASS_STAMPS):
mean shader cycles per row block and wave for each phase, and the in-kernel
clock (s_memtime / s_memrealtime at 100 MHz)."""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import rng  # noqa: E402

PH = ["wait_dma", "step1+part", "barrierA", "reduce", "barrierB", "gram64", "step3"]


def main():
    m, n, k = 1_000_000, 1000, 40
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libpass_stamps.so"))
    vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
    lib.sl_rsvd_pass.argtypes = [vp, i64, i64, i64, vp, i32, vp, vp, i64, i32, i32, vp]
    lib.sl_rsvd_pass_workspace.argtypes = [i64, i64, i32]
    lib.sl_rsvd_pass_workspace.restype = i64
    lib.sl_rsvd_pass_grid.argtypes = [i64]
    dev = torch.device("cuda")
    A = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
    Q, _ = torch.linalg.qr(torch.randn(n, k, device=dev, dtype=torch.float64))
    Zt = Q.t().contiguous().to(torch.bfloat16)
    wsb = int(lib.sl_rsvd_pass_workspace(m, n, k))
    ws = torch.zeros(wsb + (1 << 20), dtype=torch.uint8, device=dev)
    grid = int(lib.sl_rsvd_pass_grid(m))
    scratch_off = wsb - 1024
    Y = torch.empty(m, 48, device=dev)
    st = vp(torch.cuda.current_stream().cuda_stream)
    for final in (0, 1):
        for variant in (0, 3):
            for _ in range(6):
                rc = lib.sl_rsvd_pass(vp(A.data_ptr()), m, n, n, vp(Zt.data_ptr()), k, vp(ws.data_ptr()),
                                      vp(Y.data_ptr()) if final else None, 48, final, variant, st)
                assert rc == 0, rc
            torch.cuda.synchronize()
            raw = ws[scratch_off + 256 * 8: scratch_off + 256 * 8 + grid * 8 * 10 * 8].view(torch.int64).view(grid * 8, 10)
            raw = raw.double().cpu()
            blocks = raw[:, 7].clamp_min(1)
            per = {PH[i]: round(float((raw[:, i] / blocks).mean()), 1) for i in range(7)}
            clock = float((raw[:, 8] / raw[:, 9]).median()) * 100.0
            per["total_per_block"] = round(float((raw[:, 8] / blocks).mean()), 1)
            print(json.dumps({"final": final, "nbuf": 3 if variant == 3 else 4, "clock_MHz": round(clock, 1),
                              "cycles_per_block": per}), flush=True)


if __name__ == "__main__":
    main()
