#!/usr/bin/env python
"""Headline benchmark: FJLT-sketched randomized rank-20 SVD of a dense bf16
1e6 x 1e3 matrix per GPU (BASELINE.json config 3: "FJLT + randomized rank-20
SVD of 1e6x1e3 dense bf16"), one process per GPU, A row-distributed
([VC,*]) over the N GPUs, RCCL all-reduces of the (n+k) x k pass results.

Scaling is WEAK: every GPU holds a 1e6 x 1e3 bf16 shard (2 GB), the global
matrix is (N*1e6) x 1e3.  One "step" = one complete ``approximate_svd``
(sketch + q=2 power iterations + final basis + small SVD), nothing cached
between steps except the input matrix.

metric value = aggregate sketch+apply throughput in GB/s = (bytes of the
global A) / (randSVD wall-clock);  ms_per_step = randSVD wall-clock.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1: torchrun --nproc-per-node N bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

METRIC = "sketch+apply GB/s and randSVD wall-clock on 1e6×1e3 dense, 1/2/4/8 MI355X"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=1_000_000, help="rows per GPU")
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--rank", type=int, default=20)
    ap.add_argument("--iters", type=int, default=2, help="power iterations")
    ap.add_argument("--sketch", default="FJLT")
    ap.add_argument("--native", type=int, default=1, help="use the fused HIP pass kernel")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)

    import libskylark_amd as sk
    from libskylark_amd.base import distributions as D
    from libskylark_amd.ops import rng, tallskinny
    from libskylark_amd.parallel import DistMatrix, init_distributed

    tallskinny.USE_NATIVE = bool(a.native)
    if not torch.cuda.is_available():
        print("bench.py needs a GPU", file=sys.stderr)
        return 2
    comm = init_distributed()
    if comm.size == 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    dev = torch.device("cuda", torch.cuda.current_device())
    N = comm.size
    m_loc, n = a.rows, a.cols
    m = m_loc * N

    # synthetic input: Gaussian entries realised from GLOBAL indices (each GPU
    # produces its own rows; identical to the single-GPU matrix for N = 1)
    A_loc = torch.empty(m_loc, n, dtype=torch.bfloat16, device=dev)
    rng.fill_random(A_loc, D.Normal(), seed=1234, base=0, r0=comm.rank * m_loc, c0=0, ir=n, ic=1)
    A = DistMatrix(A_loc, (m, n), "VC_STAR", comm)
    params = sk.nla.ApproximateSVDParams(num_iterations=a.iters, sketch=a.sketch)

    def step():
        ctx = sk.Context(seed=38734)
        return sk.nla.approximate_svd(A, a.rank, context=ctx, params=params)

    for _ in range(a.warmup):
        U, s, V = step()
    torch.cuda.synchronize()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        U, s, V = step()
    torch.cuda.synchronize()
    comm.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    comm.all_reduce_max(t)
    dt = float(t.item())
    ms = dt / a.steps * 1e3
    a_bytes = m * n * 2
    gbs = a_bytes / (ms / 1e3) / 1e9
    if comm.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(gbs, 2),
            "unit": "GB/s",
            "n_gpus": N,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (Gaussian bf16 matrix realised by the Threefry kernel; random-init sketch)",
            "config": {
                "model": f"FJLT + randomized rank-{a.rank} SVD (q={a.iters}) of dense bf16 {m_loc}x{n} per GPU",
                "global_batch": m,
                "seq_len": n,
                "parallelism": f"dp{N} ([VC,*] row blocks, RCCL all-reduce)",
            },
            "randsvd_ms": round(ms, 4),
            "top_singular_values": [round(float(x), 3) for x in s[:3].tolist()],
            "native_fused_pass": bool(tallskinny._native_ok(A_loc, 2 * a.rank)),
        }
        print(json.dumps(out))
        from libskylark_amd.utils.timer import PROFILER
        if PROFILER.enabled:
            for name, r in PROFILER.report().items():
                print(f"[profile] {name}: {r['avg_s'] * 1e3 / max(1, a.steps + a.warmup):.3f} ms/step "
                      f"({r['calls']} calls)", file=sys.stderr)
    if N > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
