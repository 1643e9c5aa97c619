"""Host eigensolver cost for the randSVD k x k core (k = 40) on this CPU."""
import time
import numpy as np
import torch
import scipy.linalg.lapack as LA

X = np.random.randn(1000, 40)
C = X.T @ X
Ct = torch.from_numpy(C)


def timeit(fn, n=200):
    fn()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t) / n * 1e6


print("threads", torch.get_num_threads())
print("numpy eigh us", timeit(lambda: np.linalg.eigh(C)))
print("scipy dsyevd us", timeit(lambda: LA.dsyevd(C)))
print("scipy dsyevr us", timeit(lambda: LA.dsyevr(C, range="I", il=21, iu=40)))
n = torch.get_num_threads()
torch.set_num_threads(1)
print("torch eigh 1thr us", timeit(lambda: torch.linalg.eigh(Ct)))
torch.set_num_threads(n)
print("torch eigh nthr us", timeit(lambda: torch.linalg.eigh(Ct)))
