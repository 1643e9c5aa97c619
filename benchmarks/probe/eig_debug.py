"""Accuracy diagnostics of the one-wave eigensolver (diagnostic build, see
eig_stamps.py): the tridiagonal (d, e) of wave_tridiag against LAPACK's
eigenvalues of C (isolates the reduction from the multisection), and the
multisection eigenvalues of that tridiagonal against LAPACK on the same
(d, e).  Cases: the close-cluster and logspace spectra of tests/test_small_la."""
import ctypes as C
import json
import os

import numpy as np
import scipy.linalg as sla
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "native", "libeig_stamps.so"))
vp, i32 = C.c_void_p, C.c_int
lib.sl_tridiag_dbg.argtypes = [vp, i32, vp, vp]
dev = torch.device("cuda:0")


def case(name, k, lam, seed):
    g = torch.Generator().manual_seed(seed)
    Q, _ = torch.linalg.qr(torch.randn(k, k, generator=g, dtype=torch.float64))
    Cm = (Q * lam) @ Q.t()
    Cm = 0.5 * (Cm + Cm.t())
    K = 40 if k <= 40 else 64
    out = torch.zeros(4 * K + 8, dtype=torch.float64, device=dev)
    lib.sl_tridiag_dbg(vp(Cm.to(dev).data_ptr()), k, vp(out.data_ptr()), vp(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    d, e, lm = o[:K], o[K:2 * K], o[2 * K:2 * K + k]
    ref = np.sort(np.linalg.eigvalsh(Cm.numpy()))[::-1]
    # the padding (k < K) sits at -beta below the spectrum: keep the top k
    tri = np.sort(sla.eigvalsh_tridiagonal(d, e[:K - 1]))[::-1][:k]
    nrm = np.abs(ref).max()
    print(json.dumps({"case": name, "k": k,
                      "tridiag_vs_C": float(np.abs(tri - ref).max() / nrm),
                      "multisection_vs_tridiag": float(np.abs(lm - tri).max() / nrm),
                      "multisection_vs_C": float(np.abs(lm - ref).max() / nrm)}), flush=True)


lam = torch.linspace(10, 1, 40, dtype=torch.float64)
lam[3:6] = torch.tensor([7.11, 7.11 - 1e-5, 7.11 - 2e-5], dtype=torch.float64)
case("close_cluster", 40, lam, 5)
for k in (17, 33, 40, 64):
    case("logspace", k, torch.logspace(0, -12, k, dtype=torch.float64), k * 7 + k - 1)
case("uniform", 40, torch.rand(40, generator=torch.Generator().manual_seed(1), dtype=torch.float64) + 0.1, 3)
