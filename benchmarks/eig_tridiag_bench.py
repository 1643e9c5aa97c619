"""Device k x k small LA of the randSVD core: the one-wave Cholesky inverse
and the tridiagonal top-r eigensolver (sl_wave_la.hpp) vs device Jacobi and
host LAPACK, microseconds per call (CUDA events over 200 back-to-back calls;
each call is one launch, so this includes the ~2 us launch boundary)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from libskylark_amd.ops import small_la as SL

dev = torch.device("cuda:0")


def timed(fn, n=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / n, 2)


out = []
for k, r in ((40, 20), (48, 24), (32, 16), (64, 32), (16, 8)):
    g = torch.Generator().manual_seed(1)
    X = torch.randn(2000, k, generator=g, dtype=torch.float64)
    C = (X.t() @ X).to(dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    o = torch.empty(k * r + r, dtype=torch.float64, device=dev)
    out.append({"k": k, "r": r, "impl": "tridiag_wave", "us": timed(lambda: SL.sym_eig_tridiag(C, r, out=o, status=st))})
    out.append({"k": k, "r": r, "impl": "jacobi", "us": timed(lambda: SL.sym_eig_topr(C, r, out=o), 20)})
    out.append({"k": k, "impl": "chol_inv_wave", "us": timed(lambda: SL.chol_inv_wave(C, st))})
    out.append({"k": k, "impl": "chol_inv_old", "us": timed(lambda: SL.chol_inv(C, st))})
    Ch = C.cpu()
    torch.set_num_threads(1)
    t = time.perf_counter()
    for _ in range(200):
        torch.linalg.eigh(Ch)
    out.append({"k": k, "r": r, "impl": "host_lapack_1thread", "us": round((time.perf_counter() - t) / 200 * 1e6, 2)})
    out.append({"k": k, "status": int(st.item())})
# an empty kernel's launch boundary, for reference
z = torch.zeros(1, device=dev)
out.append({"impl": "empty_kernel_launch", "us": timed(lambda: z.add_(0))})
for o_ in out:
    print(json.dumps(o_))
