"""A/B of the tridiagonalisation inside the device top-r eigensolver
(sl_sym_eig_tridiag): one wave (0) vs four waves (1, wg_tridiag), us per call
(200 back-to-back launches) and eigenpair accuracy against fp64 LAPACK, on a
Gram matrix and a graded matrix."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from libskylark_amd.ops import _lib  # noqa: E402
from libskylark_amd.ops import small_la as SL  # noqa: E402

_lib.require().sl_sym_eig_set_tri_variant.argtypes = [C.c_int]
_lib.require().sl_sym_eig_set_tri_variant.restype = None
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


for k, r in ((40, 20), (48, 24), (32, 16), (64, 32), (16, 8)):
    for kind in ("gram", "graded"):
        g = torch.Generator().manual_seed(k)
        X = torch.randn(2000, k, generator=g, dtype=torch.float64)
        if kind == "graded":
            X = X * torch.logspace(0, -6, k, dtype=torch.float64)
        Cm = X.t() @ X
        w, V = np.linalg.eigh(Cm.numpy())
        w, V = w[::-1][:r], V[:, ::-1][:, :r]
        Cd = Cm.to(dev)
        for v in (0, 1):
            _lib.require().sl_sym_eig_set_tri_variant(v)
            st = torch.zeros(1, dtype=torch.int32, device=dev)
            o = torch.empty(k * r + r, dtype=torch.float64, device=dev)
            us = timed(lambda: SL.sym_eig_tridiag(Cd, r, out=o, status=st))
            st.zero_()
            SL.sym_eig_tridiag(Cd, r, out=o, status=st)
            oc = o.cpu().numpy()
            lam, U = oc[k * r:], oc[:k * r].reshape(k, r)
            lerr = float(np.max(np.abs(lam - w)) / w[0])
            res = float(np.max(np.abs(Cm.numpy() @ U - U * lam)) / w[0])
            orth = float(np.max(np.abs(U.T @ U - np.eye(r))))
            print(json.dumps({"k": k, "r": r, "matrix": kind, "tri": ["one_wave", "four_waves"][v], "us": us,
                              "lam_err": lerr, "resid": res, "orth": orth, "status": int(st.item())}))
_lib.require().sl_sym_eig_set_tri_variant(-1)
