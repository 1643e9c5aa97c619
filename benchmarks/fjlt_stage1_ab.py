"""A/B and ablation builds of fjlt_fourstep.hip's stage 1 (FS_AB_LIBS =
"tag:path,..."), timed directly on the FJLT bench shape (1e6 x 1000 f32,
N1 x N2 = 1000 x 500).  Prints one JSON line per build."""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libskylark_amd.ops import _lib, fut  # noqa: E402


def main():
    N, m = 1_000_000, 1000
    A = torch.randn(N, m, device="cuda")
    d = (torch.randint(0, 2, (N,), device="cuda") * 2 - 1).double()
    N1, N2, rs = fut.fourstep_split(N)
    Y = torch.empty(N2 * N1 * m * 2, dtype=torch.float32, device="cuda")
    st = C.c_void_p(_lib.stream_of(A))
    # FS_PLANS="4-5-5-5,25-20": radix plans to time (default: the planner's)
    plans = [[int(r) for r in p.split("-")] for p in os.environ.get("FS_PLANS", "").split(",") if p] or [rs]
    runs = [(e, p) for e in os.environ.get("FS_AB_LIBS", "").split(",") if e for p in plans]
    for e, rs in runs:
        rplan = sum(r << (4 * i) for i, r in enumerate(rs))
        tag, path = e.split(":", 1)
        L = C.CDLL(path)
        f = lambda: L.sl_fs_stage1(C.c_void_p(A.data_ptr()), _lib.dtype_code(A.dtype), C.c_int64(A.stride(0)),
                                   C.c_int64(N), m, C.c_void_p(d.data_ptr()), N1, N2, C.c_uint64(rplan), len(rs),
                                   C.c_void_p(Y.data_ptr()), st)
        rc = f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        ref = Y[:4 * m].clone()
        print(json.dumps({"build": tag, "rc": rc, "checksum": float(ref.double().abs().sum()), "stage1_ms": round(ms, 3), "N1": N1, "N2": N2, "radices": rs}),
              flush=True)


if __name__ == "__main__":
    main()
