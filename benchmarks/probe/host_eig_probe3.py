"""Host k x k eigensolver options for the randSVD core (k = 40): per-call us."""
import json
import time

import numpy as np
import scipy.linalg as sl
import scipy.linalg.lapack as la
import torch

k = 40
g = np.random.default_rng(0)
X = g.standard_normal((2000, k))
C = X.T @ X


def tm(f, n=400):
    for _ in range(20):
        f()
    t = time.perf_counter()
    for _ in range(n):
        f()
    return round((time.perf_counter() - t) / n * 1e6, 2)


Ct = torch.from_numpy(C)
res = {"threads": torch.get_num_threads()}


def toggled():
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    torch.linalg.eigh(Ct)
    torch.set_num_threads(n)


res["torch_toggle"] = tm(toggled)
res["scipy_dsyevd"] = tm(lambda: la.dsyevd(C, compute_v=1, lower=0))
res["scipy_dsyevr"] = tm(lambda: la.dsyevr(C, compute_v=1, lower=0))
res["scipy_dsyev"] = tm(lambda: la.dsyev(C, compute_v=1, lower=0))
res["numpy_eigh"] = tm(lambda: np.linalg.eigh(C))
res["scipy_eigh_evd"] = tm(lambda: sl.eigh(C, driver="evd", check_finite=False))
torch.set_num_threads(1)
res["torch_1thread"] = tm(lambda: torch.linalg.eigh(Ct))
print(json.dumps(res))
