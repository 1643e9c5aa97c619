"""Phase ablation of the fused pass (inter variant, flags 3, k = 40) on the
headline shape 1e6 x 1e3 bf16: time with step 1 (A Z), step 2 (cross-wave y
reduction + its 2 barriers) and/or step 3 (W += A^T y) switched off
(``sl_tsk_set_ablate`` bits 1 / 2 / 4; results are wrong, timing only)."""
from __future__ import annotations

import ctypes as C
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import _lib, rng, tallskinny  # noqa: E402,F401


def main():
    extra = int(sys.argv[1]) if len(sys.argv) > 1 else 0   # OR-ed into every setting (64: nt loads)
    m, n, k = 1_000_000, 1000, 40
    dev = torch.device("cuda")
    lib = _lib.require()
    lib.sl_tsk_set_ablate.argtypes = [C.c_int]
    A = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
    Zt = (torch.randn(k, n, device=dev) / 30).to(torch.bfloat16)
    W = torch.empty(n, k, device=dev)
    G = torch.empty(k, k, device=dev, dtype=torch.float64)
    Y = torch.empty(m, k, device=dev)
    ws = torch.empty(int(lib.sl_tsk_fused_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for case, flags, Yp in (("inter", 3, None), ("final_g64", 4, Y)):
        for ab in (0, 1, 2, 4, 1 | 2, 2 | 4, 1 | 4, 1 | 2 | 4, 8, 2 | 8):
            lib.sl_tsk_set_ablate(ab | extra)

            def run():
                _lib.call("sl_tsk_fused_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt), k, _lib.ptr(W),
                          _lib.ptr(G), _lib.ptr(Yp) if Yp is not None else None, 0 if Yp is None else Yp.stride(0),
                          _lib.ptr(ws), flags, st)
            run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(15):
                t0 = time.perf_counter()
                run()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            t = statistics.median(ts)
            print(json.dumps({"case": case, "ablate": ab, "extra": extra, "skip": [s for b, s in ((1, "step1"), (2, "reduce"),
                                                                                  (4, "step3"), (8, "gram"))
                                                                    if ab & b],
                              "us": round(t * 1e6, 1), "TBps": round(m * n * 2 / t / 1e12, 2)}), flush=True)
    lib.sl_tsk_set_ablate(0)


if __name__ == "__main__":
    main()
