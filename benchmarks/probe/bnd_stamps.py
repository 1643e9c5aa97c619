"""Phase timestamps of the headline call's pass-boundary kernels, read from a
library built with stamp writes in k_boundary (a probe build only; the
shipped source has none).  Runs the bench call several times, then prints
the last call's INTER (second) and FINAL boundary phases in microseconds
from the kernel's first workgroup start."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libskylark_amd as sk  # noqa: E402
from libskylark_amd.ops import _lib  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda")
A = bench.planted_matrix((1_000_000, 1000), "VC_STAR", None, dev) if hasattr(bench, "planted_matrix") else None
if A is None:
    A = torch.randn(1_000_000, 1000, device=dev).to(torch.bfloat16)
A = A.local if hasattr(A, "local") else A
prm = sk.nla.ApproximateSVDParams(num_iterations=2, sketch="FJLT")
for i in range(12):
    U, s, V = sk.nla.approximate_svd(A, 20, sk.Context(seed=100 + i), prm)
torch.cuda.synchronize()
L = _lib.require()
buf = (C.c_uint64 * 48)()
L.sl_bnd_stamps.argtypes = [C.c_void_p]
assert L.sl_bnd_stamps(C.cast(buf, C.c_void_p)) == 0
v = list(buf)
names = {0: "start(wg0)", 1: "last: ticket done", 2: "last: partials summed", 3: "last: cholesky done",
         4: "last: worker Rt^-1 in", 5: "core: C formed", 6: "core: tridiag done", 7: "core: eigvecs done",
         8: "last: core done", 9: "last: released", 10: "wg0: woke", 11: "wg0: rows done"}
for base, tag in ((0, "INTER"), (16, "FINAL")):
    t0 = v[base]
    out = {names[i]: round((v[base + i] - t0) * 0.01, 2) for i in range(12) if v[base + i] >= t0 and v[base + i]}
    print(json.dumps({"boundary": tag, "us_from_start": out}))
w0 = v[16]
print(json.dumps({"worker": {"chol start": round((v[32] - w0) * 0.01, 2), "chol done": round((v[33] - w0) * 0.01, 2)}}))
