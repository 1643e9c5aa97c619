#!/usr/bin/env python
"""Headline benchmark (BASELINE.json config 3): FJLT-sketched randomized
rank-20 SVD (q = 2 power iterations) of a dense bf16 1e6 x 1e3 matrix held
2-D block-cyclic ([MC,MR]) over the N GPUs of one node, one process per GPU,
RCCL over xGMI.

Scaling is STRONG by default: the GLOBAL matrix is 1e6 x 1e3 for every N.
The process grid is shaped for the operand: a tall-skinny 1e6 x 1e3 matrix
goes on an N x 1 grid of 4096-row tiles (``--grid-rows``; Elemental's
``Grid(comm, height)``), where every rank's cyclic row tiles already hold
whole rows, so randSVD reads them in place and the only traffic is the
(n + k) x k all-reduces.  A square-ish grid (2 x 4 at N = 8) would have to
move ~3/4 of A over xGMI on every call (~190 MB per rank, about 1 ms on the
point-to-point links -- more than the whole 8-GPU compute); for N > 1 that
grid is still timed, as the secondary key ``square_grid``.  One
"step" = one complete ``approximate_svd`` call on the [MC,MR] operand: (on
a grid with several columns, the one all-to-all that brings it to row
shards,) the FJLT sketch, q = 2 fused
power passes, the final basis pass, the small SVD and U returned in A's
[MC,MR] layout.  Every step draws a NEW sketch (``Context(seed=38734 + i)``)
and solves its k x k core from scratch: what carries over between steps is
only the input matrix, the engine's workspaces and its captured hipGraph.
``--scaling weak`` times 1e6 rows PER
GPU in [VC,*] instead; for N > 1 a short weak run is appended as a
secondary key.

The matrix is synthetic, planted low rank plus noise,
    A = U0 diag(sigma) V0^T + eps E,  sigma_i = 1000 * 0.9^i (i < 20),
every entry realised from its GLOBAL index by the Threefry kernel (so the
matrix is the same for every N and layout).  After the timed loop the run
checks the answer: orthogonality of U and ||A V - U S||_F / ||S||_F.

metric value = (bytes of the global bf16 A) / (randSVD wall-clock)  [GB/s];
ms_per_step  = randSVD wall-clock (max over ranks).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1: torchrun --nproc-per-node N bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

METRIC = "sketch+apply GB/s and randSVD wall-clock on 1e6×1e3 dense, 1/2/4/8 MI355X"
PLANT_RANK = 20


def planted_matrix(shape, layout, comm, dev, grid=None, block=None, seed=1234, eps=0.05):
    """bf16 DistMatrix A = U0 diag(sigma) V0^T + eps E from global indices."""
    from libskylark_amd.base import distributions as D
    from libskylark_amd.ops import rng
    from libskylark_amd.parallel.distmatrix import DistMatrix, _merge
    m, n = shape
    p = PLANT_RANK
    A = DistMatrix.empty(shape, layout, comm, dtype=torch.bfloat16, device=dev, grid=grid, block=block)
    sig = 1000.0 * 0.9 ** torch.arange(p, dtype=torch.float32, device=dev)
    rows, cols = _merge(A.row_blocks()), _merge(A.col_blocks())
    V0 = torch.empty(n, p, dtype=torch.float32, device=dev)
    rng.fill_random(V0, D.Normal(), seed + 2, 0, ir=p, ic=1, scale=1.0 / math.sqrt(n))
    ro = 0
    for rs, re in rows:
        for c0 in range(rs, re, 1 << 16):
            c1 = min(re, c0 + (1 << 16))
            U0 = torch.empty(c1 - c0, p, dtype=torch.float32, device=dev)
            rng.fill_random(U0, D.Normal(), seed + 1, 0, r0=c0, ir=p, ic=1, scale=1.0 / math.sqrt(m))
            co = 0
            for cs, ce in cols:
                T = torch.empty(c1 - c0, ce - cs, dtype=torch.float32, device=dev)
                rng.fill_random(T, D.Normal(), seed, 0, r0=c0, c0=cs, ir=n, ic=1, scale=eps)
                T.addmm_(U0 * sig, V0[cs:ce].t())
                A.local[ro + c0 - rs: ro + c1 - rs, co: co + ce - cs].copy_(T)
                co += ce - cs
        ro += re - rs
    return A


def check_answer(A, U, s, V, comm):
    """(max |U^T U - I|, ||A V - U S||_F / ||S||_F, sigma_1..3) with A, U distributed."""
    Avc = A.redistribute("VC_STAR")
    Uvc = U.redistribute("VC_STAR").local.double()
    G = Uvc.t() @ Uvc
    comm.all_reduce(G)
    orth = float((G - torch.eye(G.shape[0], dtype=G.dtype, device=G.device)).abs().max())
    R = Avc.local.float() @ V.float() - (Uvc * s.double()).float()
    r2 = torch.tensor([float((R.double() ** 2).sum())], dtype=torch.float64, device=R.device)
    comm.all_reduce(r2)
    resid = math.sqrt(float(r2)) / float(s.double().norm())
    return orth, resid


def run(a, comm, dev, scaling, square=False):
    import libskylark_amd as sk
    from libskylark_amd.ops import tallskinny
    from libskylark_amd.parallel.distmatrix import Grid
    N = comm.size
    n = a.cols
    if scaling == "strong":
        m = a.rows
        layout = a.layout
    else:
        m = a.rows * N
        layout = "VC_STAR"
    grid = None
    if layout == "MC_MR":
        pr = None if square else (a.grid_rows or N)
        grid = Grid.default(comm, pr)
    block = (a.tile_rows, a.tile_cols) if layout == "MC_MR" else None
    A = planted_matrix((m, n), layout, comm, dev, grid, block)
    torch.cuda.synchronize()
    params = sk.nla.ApproximateSVDParams(num_iterations=a.iters, sketch=a.sketch)
    ctr = [0]

    def step():
        # a fresh sketch every call
        ctr[0] += 1
        return sk.nla.approximate_svd(A, a.rank, context=sk.Context(seed=38734 + ctr[0]), params=params)

    primary = scaling == a.scaling and not square
    steps, warmup = (a.steps, a.warmup) if primary else (max(3, a.steps // 2), 2)
    for _ in range(warmup):
        U, s, V = step()
    # per-step device time from events recorded between the steps (no host
    # synchronisation inside the timed loop); the headline number is the
    # wall clock of all K steps, bracketed by barrier + synchronize
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    torch.cuda.synchronize()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(steps):
        U, s, V = step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    comm.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    comm.all_reduce_max(t)
    ms = float(t.item()) / steps * 1e3
    per = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    step_ms = {"min": round(per[0], 4), "median": round(per[len(per) // 2], 4), "max": round(per[-1], 4)}
    from libskylark_amd.nla.svd import last_device_status
    status = last_device_status(wait=True)
    # a one-shot all-reduce whose peer missed its bounded wait poisoned that
    # call's operand with NaN: never report a number from such a run.  Every
    # rank learns every rank's failure (check_collectives(agree=True)), every
    # rank must have run the same engine, and no rank may report a device
    # timeout; any of these makes the run an error (non-zero exit, reason in
    # the JSON line)
    errors = []
    try:
        comm.check_collectives(agree=True)
    except Exception as e:  # noqa: BLE001 - OneShotError (the same text on every rank)
        errors.append(f"{type(e).__name__}: {e}")
    if N > 1:
        from libskylark_amd.nla.svd import last_engine
        eng = comm.all_gather_object(last_engine())
        if len(set(eng)) > 1:
            errors.append(f"ranks ran different randSVD engines: {eng}")
        sts = comm.all_gather_object(int(status))
        late = [q for q, x in enumerate(sts) if x & 16]
        if late:
            errors.append(f"device engine timeout (status bit 16) on rank(s) {late}")
    orth, resid = check_answer(A, U, s, V, comm)
    red = "one-shot IPC all-reduces" if getattr(comm, "_oneshot", None) else "RCCL all-reduces"
    if grid is not None:
        how = "tiles read in place (whole rows per rank)" if grid.pc == 1 else "one all-to-all to [VC,*]"
        par = f"2-D block-cyclic [MC,MR] {grid.pr}x{grid.pc} grid, tile {block[0]}x{block[1]}, " \
              f"{how} + {red}"
    else:
        par = f"dp{N} ([VC,*] row blocks, {red})"
    return {
        "m": m, "n": n, "ms": ms, "step_ms": step_ms, "gbs": m * n * 2 / (ms / 1e3) / 1e9, "steps": steps, "warmup": warmup,
        "parallelism": par, "orth_err": orth, "resid_rel": resid, "status": status,
        "top_singular_values": [round(float(x), 3) for x in s[:3].tolist()],
        "grid_pc": grid.pc if grid is not None else 0, "errors": errors,
        "reduction": comm.oneshot_status() if N > 1 else None,
        "native_fused_pass": bool(tallskinny._native_ok(torch.empty(8, 8, dtype=torch.bfloat16, device=dev),
                                                        2 * a.rank)),
    }


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=1_000_000, help="global rows (strong) / rows per GPU (weak)")
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--rank", type=int, default=20)
    ap.add_argument("--iters", type=int, default=2, help="power iterations")
    ap.add_argument("--sketch", default="FJLT")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong")
    ap.add_argument("--layout", default="MC_MR", help="layout of A for strong scaling")
    ap.add_argument("--tile-rows", type=int, default=4096)
    ap.add_argument("--tile-cols", type=int, default=128)
    ap.add_argument("--grid-rows", type=int, default=0, help="process-grid height for [MC,MR] (0: N, i.e. N x 1)")
    ap.add_argument("--no-weak", action="store_true", help="skip the secondary weak-scaling run (N > 1)")
    ap.add_argument("--no-square", action="store_true", help="skip the secondary square-grid run (N > 1)")
    ap.add_argument("--native", type=int, default=1, help="use the fused HIP pass kernel")
    a = ap.parse_args(argv)

    from libskylark_amd.ops import tallskinny
    from libskylark_amd.parallel import init_distributed
    from libskylark_amd.parallel.distmatrix import Grid

    tallskinny.USE_NATIVE = bool(a.native)
    if not torch.cuda.is_available():
        print("bench.py needs a GPU", file=sys.stderr)
        return 2
    comm = init_distributed()
    if comm.size == 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    dev = torch.device("cuda", torch.cuda.current_device())
    N = comm.size
    res = run(a, comm, dev, a.scaling)
    weak = sq = None
    if N > 1 and a.scaling == "strong" and a.layout == "MC_MR" and not a.no_square and \
            Grid.default(comm).pc != res["grid_pc"]:
        sq = run(a, comm, dev, "strong", square=True)
    if N > 1 and a.scaling == "strong" and not a.no_weak:
        weak = run(a, comm, dev, "weak")
    errors = res["errors"] + (sq["errors"] if sq else []) + (weak["errors"] if weak else [])
    ok = res["orth_err"] < 1e-3 and res["resid_rel"] < 5e-2 and not (res["status"] & 16) and not errors
    if comm.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(res["gbs"], 2),
            "unit": "GB/s",
            "n_gpus": N,
            "steps": res["steps"],
            "warmup": res["warmup"],
            "ms_per_step": round(res["ms"], 4),
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic planted rank-20 + Gaussian noise bf16 matrix (Threefry, global indices); "
                    "random-init FJLT sketch",
            "config": {
                "model": f"FJLT + randomized rank-{a.rank} SVD (q={a.iters}) of dense bf16 {res['m']}x{res['n']}",
                "global_batch": res["m"],
                "seq_len": res["n"],
                "parallelism": res["parallelism"],
            },
            "randsvd_ms": round(res["ms"], 4),
            "step_ms": res["step_ms"],
            "check": {"orth_err": res["orth_err"], "resid_rel": res["resid_rel"], "device_status": res["status"],
                      "ok": ok},
            "cold": "every step a new sketch seed; the k x k core is solved from scratch every call",
            "top_singular_values": res["top_singular_values"],
            "native_fused_pass": res["native_fused_pass"],
        }
        if errors:
            out["error"] = errors
        if res["reduction"] is not None:
            # which small all-reduce ran and, when the one-shot path is off,
            # why (its collective self-test outcome on this node)
            out["reduction"] = res["reduction"]
        if sq is not None:
            out["square_grid"] = {"value": round(sq["gbs"], 2), "ms_per_step": round(sq["ms"], 4),
                                  "steps": sq["steps"], "parallelism": sq["parallelism"],
                                  "check": {"orth_err": sq["orth_err"], "resid_rel": sq["resid_rel"]}}
        if weak is not None:
            out["weak"] = {"value": round(weak["gbs"], 2), "ms_per_step": round(weak["ms"], 4),
                           "global_rows": weak["m"], "steps": weak["steps"], "parallelism": weak["parallelism"],
                           "check": {"orth_err": weak["orth_err"], "resid_rel": weak["resid_rel"]}}
        print(json.dumps(out))
        from libskylark_amd.utils.timer import PROFILER
        if PROFILER.enabled:
            for name, r in PROFILER.report().items():
                print(f"[profile] {name}: {r['avg_s'] * 1e3 / max(1, a.steps + a.warmup):.3f} ms/step "
                      f"({r['calls']} calls)", file=sys.stderr)
    if N > 1:
        import torch.distributed as dist
        try:
            comm.check_collectives(agree=True)
        except Exception as e:  # noqa: BLE001
            print(f"collective failure after the bench: {e}", file=sys.stderr)
            ok = False
        comm.close()
        dist.destroy_process_group()
    if errors:
        return 4
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
