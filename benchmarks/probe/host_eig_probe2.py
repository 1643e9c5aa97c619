"""Host-side cost of the randSVD k x k eigensolve block (k = 40, r = 20):
LAPACK drivers and the surrounding tensor bookkeeping, current code vs a
numpy-view version (the block sits on the randSVD critical path)."""
import time

import numpy as np
import scipy.linalg as sl
import torch

k, r = 40, 20
C = torch.randn(k, k, dtype=torch.float64)
C = C @ C.T
host = torch.cat([C.reshape(-1), torch.zeros(1, dtype=torch.float64)])
pin = torch.zeros(k * r + r, dtype=torch.float64)


def tm(f, n=300):
    f()
    t = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t) / n * 1e6


def cur():
    nt = torch.get_num_threads()
    Cm = host[:k * k].view(k, k)
    if not bool(torch.isfinite(Cm).all()):
        return
    torch.set_num_threads(1)
    evals, evecs = torch.linalg.eigh(Cm)
    torch.set_num_threads(nt)
    if not float(evals[k - r]) > 1e-30 * max(float(evals[-1]), 1e-300):
        return
    pin[:k * r].view(k, r).copy_(evecs[:, k - r:].flip(1))
    torch.sqrt(evals[k - r:].flip(0).clamp_min(0.0), out=pin[k * r:])


hn = host.numpy()
pn = pin.numpy()


def lean():
    Cm = hn[:k * k].reshape(k, k)
    if not np.isfinite(Cm).all():
        return
    w, v = sl.eigh(Cm, driver="evd", check_finite=False, overwrite_a=False)
    if not w[k - r] > 1e-30 * max(w[-1], 1e-300):
        return
    pn[:k * r].reshape(k, r)[:] = v[:, :k - r - 1:-1]
    np.sqrt(np.maximum(w[:k - r - 1:-1], 0.0), out=pn[k * r:])


def lean_torch():
    Cm = hn[:k * k].reshape(k, k)
    if not np.isfinite(Cm).all():
        return
    w, v = torch.linalg.eigh(torch.from_numpy(Cm))
    w, v = w.numpy(), v.numpy()
    if not w[k - r] > 1e-30 * max(w[-1], 1e-300):
        return
    pn[:k * r].reshape(k, r)[:] = v[:, :k - r - 1:-1]
    np.sqrt(np.maximum(w[:k - r - 1:-1], 0.0), out=pn[k * r:])


print("threads", torch.get_num_threads())
print("torch eigh only", tm(lambda: torch.linalg.eigh(C)))
print("current block", tm(cur))
print("lean scipy evd", tm(lean))
torch.set_num_threads(1)
print("lean torch (1 thread)", tm(lean_torch))
print("scipy evr top20", tm(lambda: sl.eigh(C.numpy(), subset_by_index=[20, 39], driver="evr", check_finite=False)))
print("scipy evd", tm(lambda: sl.eigh(C.numpy(), driver="evd", check_finite=False)))
