"""Device k x k eigensolvers for the randSVD core (k = 40, r = 20): tridiagonal
path vs Jacobi vs host LAPACK, microseconds per call (CUDA events, 200 calls)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from libskylark_amd.ops import small_la as SL

dev = torch.device("cuda:0")
out = []
for k, r in ((40, 20), (64, 32), (20, 10)):
    g = torch.Generator().manual_seed(1)
    X = torch.randn(2000, k, generator=g, dtype=torch.float64)
    C = (X.t() @ X).to(dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    o = torch.empty(k * r + r, dtype=torch.float64, device=dev)
    for name, fn in (("tridiag", lambda: SL.sym_eig_tridiag(C, r, out=o, status=st)),
                     ("jacobi", lambda: SL.sym_eig_topr(C, r, out=o))):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append({"k": k, "r": r, "impl": name, "us": round(e0.elapsed_time(e1) * 1e3 / 200, 2)})
    Ch = C.cpu()
    torch.set_num_threads(1)
    t = time.perf_counter()
    for _ in range(200):
        torch.linalg.eigh(Ch)
    out.append({"k": k, "r": r, "impl": "host_lapack_1thread", "us": round((time.perf_counter() - t) / 200 * 1e6, 2)})
import ctypes
from libskylark_amd.ops import _lib
lib = _lib.require()
lib.sl_sym_eig_tridiag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
for k, r in ((40, 20), (64, 32)):
    g = torch.Generator().manual_seed(1)
    X = torch.randn(2000, k, generator=g, dtype=torch.float64)
    C = (X.t() @ X).to(dev)
    o = torch.empty(k * r + r, dtype=torch.float64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    stamps = torch.zeros(5, dtype=torch.int64, device=dev)
    for _ in range(3):
        lib.sl_sym_eig_tridiag_stamps(C.data_ptr(), k, k, r, o.data_ptr(), st.data_ptr(), stamps.data_ptr(),
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    t = stamps.cpu().tolist()
    out.append({"k": k, "r": r, "phase_cycles": {"tridiag": t[1] - t[0], "multisection": t[2] - t[1],
                                                 "vectors": t[3] - t[2], "backtransform": t[4] - t[3]}})
for o in out:
    print(json.dumps(o))
