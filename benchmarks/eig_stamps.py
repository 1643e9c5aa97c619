"""Phase stamps (shader clock, s_memtime) of the one-workgroup tridiagonal
eigensolver (sym_eig.hip on sl_wave_la.hpp): tridiagonalisation,
multisection, twisted vectors, MGS + residual check, back-transform.
Uses a diagnostic build (-DSL_EIG_STAMPS) made on the build host:
  hipcc -O3 -fPIC -shared -std=c++17 --offload-arch=gfx950 -DSL_EIG_STAMPS \\
        -I libskylark_amd/_native/include libskylark_amd/_native/src/sym_eig.hip \\
        benchmarks/native/stub_err.hip -o benchmarks/native/libeig_stamps.so"""
import ctypes as C
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "native", "libeig_stamps.so"))
vp, i32 = C.c_void_p, C.c_int
lib.sl_sym_eig_tridiag.argtypes = [vp, i32, i32, i32, vp, i32, vp, vp]
lib.sl_eig_stamps.argtypes = [vp]
dev = torch.device("cuda:0")
names = ["tridiag", "multisection", "vectors", "mgs+resid", "backtransform"]
for k, r in ((40, 20), (48, 24), (32, 16), (64, 32)):
    g = torch.Generator().manual_seed(1)
    X = torch.randn(2000, k, generator=g, dtype=torch.float64)
    Cm = (X.t() @ X).to(dev)
    o = torch.empty(k * r + r, dtype=torch.float64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    s = vp(torch.cuda.current_stream().cuda_stream)
    acc = [0.0] * 5
    sub = [0.0] * 5
    n = 20
    for it in range(n + 2):
        lib.sl_sym_eig_tridiag(vp(Cm.data_ptr()), k, k, r, vp(o.data_ptr()), 0, vp(st.data_ptr()), s)
        torch.cuda.synchronize()
        h = (C.c_ulonglong * 64)()
        lib.sl_eig_stamps(h)
        if it >= 2:
            for p in range(5):
                acc[p] += (h[p + 1] - h[p]) / n
                sub[p] += (h[11 + p] - h[10 + p]) / n
    print(json.dumps({"k": k, "r": r, "status": int(st.item()),
                      "phase_cycles": {nm: round(a) for nm, a in zip(names, acc)},
                      "tridiag_step10_cycles": {nm: round(a) for nm, a in
                                                zip(["s2+v+bcast", "p", "Kd", "w+bcast", "update"], sub)}}))
