"""BASELINE config 5: LSRN sketch-and-solve of an overdetermined least-squares
problem, 1e7 x 5e3 dense on 8 GPUs = 1.25e6 x 5e3 fp32 rows per GPU (weak
scaling, [VC,*] row blocks; the sketch partials and every Chebyshev/LSQR
product A^T r are one RCCL all-reduce).

Reports the sketch time (JLT t = 4n, bf16x2 MFMA panels), preconditioner time
(QR of the t x n sketch), solve time/iterations and the relative residual
against the planted solution.  Data: Gaussian A with geometrically scaled
columns (condition number ~cond), b = A x + 1e-3 noise.

usage: python benchmarks/bench_lsrn.py [--rows 1.25e6] [--cols 5000] [--cond 1e4]
       torchrun --nproc-per-node N --master-addr 127.0.0.1 benchmarks/bench_lsrn.py
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1.25e6)
    ap.add_argument("--cols", type=int, default=5000)
    ap.add_argument("--cond", type=float, default=1e4)
    ap.add_argument("--oversample", type=int, default=4)
    ap.add_argument("--tol", type=float, default=1e-6)
    ap.add_argument("--classic", action="store_true", help="two products per Krylov iteration (no fused A^T A pass)")
    ap.add_argument("--warmup", type=int, default=1, help="untimed full solves first (library init, kernel loads)")
    a = ap.parse_args(argv)
    import libskylark_amd as sk
    from libskylark_amd.algorithms import AcceleratedRegressionSolver, KrylovIterParams, RegressionProblem
    from libskylark_amd.base import distributions as D
    from libskylark_amd.ops import rng
    from libskylark_amd.parallel import DistMatrix, init_distributed
    comm = init_distributed()
    dev = torch.device("cuda", torch.cuda.current_device())
    m_loc, n = int(a.rows), a.cols
    m = m_loc * comm.size
    A_loc = torch.empty(m_loc, n, dtype=torch.float32, device=dev)
    rng.fill_random(A_loc, D.Normal(), seed=3, base=0, r0=comm.rank * m_loc, c0=0, ir=n, ic=1)
    colscale = torch.logspace(0, -torch.log10(torch.tensor(a.cond)).item(), n, device=dev)
    A_loc *= colscale
    x_true = torch.randn(n, 1, generator=torch.Generator(device=dev).manual_seed(5), device=dev)
    b_loc = A_loc @ x_true
    noise = torch.empty(m_loc, 1, device=dev)
    rng.fill_random(noise, D.Normal(), seed=4, base=0, r0=comm.rank * m_loc, c0=0, ir=1, ic=1)
    b_loc += 1e-3 * noise
    A = DistMatrix(A_loc, (m, n), "VC_STAR", comm) if comm.size > 1 else A_loc
    from libskylark_amd.utils.timer import PROFILER
    cold = None
    for rep in range(a.warmup + 1):
        if rep == a.warmup:
            PROFILER.reset()
        torch.cuda.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        solver = AcceleratedRegressionSolver(RegressionProblem(A), sk.Context(7), method="lsrn", precond="qr",
                                             oversample=a.oversample,
                                             params=KrylovIterParams(tolerance=a.tol, iter_lim=300,
                                                                             fused_normal=False if a.classic else None))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        X, code = solver.solve(b_loc)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if rep == 0 and a.warmup:
            cold = round(t2 - t0, 4)
        use_lsqr = solver.use_lsqr
        del solver
    r = (A_loc @ X.to(A_loc.dtype) - b_loc)
    st = torch.stack([(r * r).sum(), (b_loc * b_loc).sum()]).double()
    comm.all_reduce(st)
    xerr = float((X.to(x_true.dtype) - x_true).norm() / x_true.norm())
    tt = torch.tensor([t1 - t0, t2 - t1], dtype=torch.float64, device=dev)
    comm.all_reduce_max(tt)
    if comm.rank == 0:
        print(json.dumps({"metric": "LSRN least squares wall-clock (sketch + precond + solve)",
                          "value": round(float(tt.sum()), 4), "unit": "s", "higher_is_better": False,
                          "n_gpus": comm.size, "scaling": "weak",
                          "setup_s": round(float(tt[0]), 4), "solve_s": round(float(tt[1]), 4),
                          "warmup_runs": a.warmup, "cold_first_run_s": cold,
                          "method": "chebyshev" if not use_lsqr else "lsqr", "code": int(code),
                          "krylov_form": "classic" if a.classic else "normal (fused A^T A pass)",
                          "rel_residual": float((st[0] / st[1]).sqrt()), "rel_x_error": xerr,
                          "config": {"rows_per_gpu": m_loc, "cols": n, "cond": a.cond,
                                     "sketch": f"JLT t={a.oversample}n (bf16x2)", "precond": "QR of sketch",
                                     "dtype": "fp32"}}))
        if PROFILER.enabled:
            for name, r in PROFILER.report().items():
                print(f"[profile] {name}: {r['avg_s'] * 1e3:.2f} ms total ({r['calls']} calls)", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
