"""Stage 1 of the four-step sampled DCT (fjlt_fourstep.hip) alone, timed on
the FJLT bench shape (1e6 x 1000, N1 x N2 = 1000 x 500).  FS_DTYPE=bf16 for
bf16 input.  Prints one JSON line."""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libskylark_amd.ops import fut  # noqa: E402


def main():
    N, m = int(os.environ.get("FS_N", 1_000_000)), int(os.environ.get("FS_M", 1000))
    dt = torch.bfloat16 if os.environ.get("FS_DTYPE") == "bf16" else torch.float32
    A = torch.randn(N, m, device="cuda").to(dt)
    d = (torch.randint(0, 2, (N,), device="cuda") * 2 - 1).float()
    N1, N2, rs = fut.fourstep_split(N)
    rplan = sum(r << (4 * i) for i, r in enumerate(rs))
    Y = torch.empty(N2 * N1 * m * 2, dtype=torch.float32, device="cuda")
    L = fut._fs_lib()
    st = C.c_void_p(L.stream_of(A))
    reps = int(os.environ.get("FS_REPS", 10))
    f = lambda: L.call("sl_fs_stage1", L.ptr(A), L.dtype_code(A.dtype), A.stride(0), N, m, L.ptr(d), N1, N2,
                       C.c_uint64(rplan), len(rs), L.ptr(Y), st)
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    gb = (A.numel() * A.element_size() + Y.numel() * 4) / 1e9
    print(json.dumps({"bench": "fjlt_stage1", "dtype": str(dt).split(".")[-1], "N1": N1, "N2": N2, "radices": rs,
                      "ms": round(ms, 3), "GBps": round(gb / ms * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
