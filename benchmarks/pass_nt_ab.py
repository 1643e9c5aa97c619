"""A/B of the fused randSVD pass (rsvd_pass.hip) on the headline shape
(1e6 x 1000 bf16, k = 40): row stride 1000 (dense) vs 1024 (2 KiB-aligned
rows), and the LDS-DMA loads with / without the non-temporal hint (variant
bit 16).  Interleaved rounds of 10 passes, HIP-event timed; prints the
median us per pass and the effective read bandwidth of A."""
from __future__ import annotations

import ctypes as C
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.ops import _lib  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_rsvd_pass", [vp, i64, i64, i64, vp, i32, vp, vp, i64, i32, i32, vp])
_lib.register("sl_rsvd_pass_workspace", [i64, i64, i32], C.c_int64)


def main():
    m, n, k = 1_000_000, 1000, 40
    dev = torch.device("cuda")
    lib = _lib.require()
    base = torch.randn(m, 1024, device=dev).to(torch.bfloat16)
    Q, _ = torch.linalg.qr(torch.randn(n, k, device=dev, dtype=torch.float64))
    Zt = Q.t().contiguous().to(torch.bfloat16)
    ws = torch.empty(int(lib.sl_rsvd_pass_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    Y = torch.empty(m, k, device=dev)
    dense = base[:, :n].contiguous()
    st = vp(torch.cuda.current_stream().cuda_stream)
    cases = []
    if os.environ.get("FINAL_AB"):
        # same-box A/B of the last-pass forms: W only / + Y / + Y + in-pass Gram
        for final in (0, 2, 1):
            cases.append((1000, 0, final, dense))
    else:
        for lda in (1000, 1024):
            A = dense if lda == 1000 else base
            for nt in (0, 16):
                for final in (0, 1):
                    cases.append((lda, nt, final, A))
    times = {c[:3]: [] for c in cases}
    for rnd in range(5):
        for lda, nt, final, A in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                _lib.call("sl_rsvd_pass", _lib.ptr(A), m, n, lda, _lib.ptr(Zt), k, _lib.ptr(ws),
                          _lib.ptr(Y) if final else None, k, final, nt, st)
            e1.record()
            e1.synchronize()
            if rnd:
                times[(lda, nt, final)].append(e0.elapsed_time(e1) * 100.0)
    for (lda, nt, final), ts in times.items():
        us = statistics.median(ts)
        print(json.dumps({"lda": lda, "nt": bool(nt), "final": final, "us": round(us, 1),
                          "TBps": round(m * n * 2 / (us * 1e-6) / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
