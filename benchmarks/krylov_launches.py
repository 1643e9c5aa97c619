"""Kernel launches and time per Krylov iteration (LSQR / Chebyshev) on an
LSRN-shaped f32 problem, for the launch-count report of the device-resident
solvers.  Run under ``rocprofv3 --kernel-trace --stats`` to count launches:
the solver runs ``--iters`` iterations twice (``--reps 2``), so the per-
iteration launch count is the kernel total of the profile divided by
2 * iters (setup launches are amortised).

usage: python benchmarks/krylov_launches.py [--rows 1e6] [--cols 1000] [--iters 50] [--solver lsqr|cheb]"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e6)
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--solver", default="lsqr")
    ap.add_argument("--classic", action="store_true")
    a = ap.parse_args()
    from libskylark_amd.algorithms import krylov as K
    from libskylark_amd.algorithms.regression import _build_precond
    from libskylark_amd.base import distributions as D
    from libskylark_amd.ops import rng
    dev = torch.device("cuda")
    m, n = int(a.rows), a.cols
    A = torch.empty(m, n, device=dev)
    rng.fill_random(A, D.Normal(), 3, 0, ir=n, ic=1)
    A *= torch.logspace(0, -3, n, device=dev)
    b = torch.randn(m, 1, device=dev)
    S = torch.randn(4 * n, m, device=dev) / math.sqrt(4 * n)
    P, _ = _build_precond(S @ A, "qr")
    del S
    p = K.KrylovIterParams(tolerance=0.0, iter_lim=a.iters, check_every=a.iters,
                           fused_normal=False if a.classic else None)
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if a.solver == "lsqr":
            K.lsqr(A, b, params=p, R=P)
        else:
            K.chebyshev_ls(A, b, 0.5, 2.0, p, P)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"bench": "krylov_iteration", "solver": a.solver, "m": m, "n": n, "iters": a.iters,
                      "form": "classic" if a.classic else "normal", "ms_per_iter": round(min(ts) / a.iters * 1e3, 4),
                      "GBps_of_A_reads": None}), flush=True)


if __name__ == "__main__":
    main()
