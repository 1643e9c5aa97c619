"""Stage 2 of the four-step sampled DCT (fjlt_fourstep.hip) alone on the FJLT
bench shape (1e6 x 1000, S = 4000 samples: ~8000 frequencies over N2 = 500
groups): the MFMA kernel (variant 1) against the VALU kernel (variant 0),
outputs compared.  Prints one JSON line per variant."""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libskylark_amd.ops import fut  # noqa: E402


def main():
    N, m, S = 1_000_000, 1000, 4000
    smp = torch.randint(0, N, (S,))
    plan = fut._FourStepPlan(N, smp, torch.device("cuda"))
    Y = torch.randn(plan.N2 * plan.N1 * m * 2, device="cuda")
    L = fut._fs_lib()
    st = C.c_void_p(L.stream_of(Y))
    reps = int(os.environ.get("FS_REPS", 10))
    first = None
    for v in (1, 0):
        fut.set_fourstep_stage2(v)
        Zs = torch.zeros(plan.nslots * m * 2, device="cuda")
        if v:
            f = lambda: L.call("sl_fs_stage2", L.ptr(Y), plan.N1, plan.N2, m, L.ptr(plan.gptr_s),
                               L.ptr(plan.gk1_s), L.ptr(plan.gslot_s), L.ptr(Zs), L.ptr(plan.gord), st)
        else:
            f = lambda: L.call("sl_fs_stage2", L.ptr(Y), plan.N1, plan.N2, m, L.ptr(plan.gptr), L.ptr(plan.gk1),
                               L.ptr(plan.gslot), L.ptr(Zs), None, st)
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        rel = None if first is None else float((Zs - first).abs().max() / first.abs().max())
        first = Zs.clone() if first is None else first
        print(json.dumps({"bench": "fjlt_stage2", "variant": "mfma" if v else "valu", "N1": plan.N1, "N2": plan.N2,
                          "freqs": plan.nslots, "ms": round(ms, 3), "GBps_of_Y": round(Y.numel() * 4 / ms / 1e6, 1),
                          "maxrel_vs_mfma": rel}), flush=True)
    fut.set_fourstep_stage2(1)


if __name__ == "__main__":
    main()
