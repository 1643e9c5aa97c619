"""Phase times of approximate_kernel_ridge on 1e6 x 512 -> 4096 features
(config 4's KRR half): feature map, split Z^T Z, Z^T Y (fp64), the Cholesky
solve.  usage: python benchmarks/probe/krr_phases.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import libskylark_amd as sk  # noqa: E402
from libskylark_amd import ml  # noqa: E402
from libskylark_amd.ml import krr as K  # noqa: E402


def tm(f, it=2):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        out = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3, out


dev = torch.device("cuda")
m, d, s = 1_000_000, 512, 4096
g = torch.Generator(device=dev).manual_seed(1)
X = torch.randn(m, d, generator=g, device=dev)
Y = torch.randn(m, 1, generator=g, device=dev)
kern = ml.Gaussian(d, sigma=float(d) ** 0.5)
S = kern.create_rft(s, context=sk.Context(3))
res = {}
res["features_ms"], Z = tm(lambda: S.apply(X, dim=sk.sketch.ROWWISE))
G = torch.zeros(s, s, dtype=torch.float64, device=dev)
GY = torch.zeros(s, 1, dtype=torch.float64, device=dev)
for R in (4096, 8192, 16384):
    K.SPLIT_GRAM_ROWS = R
    res[f"split_gram_R{R}_ms"], _ = tm(lambda: K._gram_split(Z, G.zero_()))
K.SPLIT_GRAM_ROWS = 8192
from libskylark_amd.ops import normal_eq  # noqa: E402
res["zty_dual_ms"], _ = tm(lambda: normal_eq.dual(Z, Y))


def zty():
    out = torch.zeros(s, 1, dtype=torch.float64, device=dev)
    ch = (1 << 27) // (s + 1)
    for r0 in range(0, m, ch):
        out.addmm_(Z[r0:r0 + ch].double().t(), Y[r0:r0 + ch].double())
    return out


res["zty_f64_ms"], _ = tm(zty)
C = G.clone()
C.diagonal().add_(1e-2)
b = torch.randn(s, 1, dtype=torch.float64, device=dev)
res["chol_solve_ms"], _ = tm(lambda: torch.cholesky_solve(b, torch.linalg.cholesky(C)))
res["total_ridge_ms"], _ = tm(lambda: K._ridge(Z, Y, 1e-2))
print(json.dumps({k: round(v, 2) for k, v in res.items()}))
