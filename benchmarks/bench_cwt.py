"""BASELINE config 2: CWT (CountSketch) of a 1e7 x 1e4 CSR sparse matrix on one
MI355X.  Metric: sketch+apply GB/s = (CSR bytes read: values + column indices
+ row pointers) / apply time.  The sketch (hash buckets + signs, bucket
permutation) is built once; every timed step is one full ``S * A``.

usage: python benchmarks/bench_cwt.py [--rows 1e7] [--cols 1e4] [--nnz-per-row 10] [--S 4096]
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
    ap.add_argument("--rows", type=float, default=1e7)
    ap.add_argument("--cols", type=float, default=1e4)
    ap.add_argument("--nnz-per-row", type=int, default=10)
    ap.add_argument("--S", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rowwise", action="store_true", help="sketch the columns (A S^T) instead")
    ap.add_argument("--sparse-out", action="store_true", help="sparse (CSR) result instead of dense")
    a = ap.parse_args(argv)
    import libskylark_amd as sk
    dev = torch.device("cuda")
    m, n, z = int(a.rows), int(a.cols), a.nnz_per_row
    g = torch.Generator(device=dev).manual_seed(7)
    nnz = m * z
    rowptr = torch.arange(0, nnz + 1, z, dtype=torch.int64, device=dev)
    col = torch.randint(0, n, (nnz,), generator=g, device=dev, dtype=torch.int64)
    col = col.view(m, z).sort(dim=1).values.reshape(-1).to(torch.int32)
    val = torch.randn(nnz, generator=g, device=dev, dtype=torch.float32)
    A = torch.sparse_csr_tensor(rowptr, col, val, (m, n))
    dim = sk.sketch.ROWWISE if a.rowwise else sk.sketch.COLUMNWISE
    S = sk.sketch.CWT(n if a.rowwise else m, a.S, context=sk.Context(11))
    for _ in range(a.warmup):
        out = S.apply(A, dim=dim, sparse_output=a.sparse_out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = S.apply(A, dim=dim, sparse_output=a.sparse_out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    nbytes = nnz * (4 + 4) + (m + 1) * 8
    print(json.dumps({"metric": "CWT sketch+apply GB/s (CSR bytes / apply time)", "value": round(nbytes / dt / 1e9, 2),
                      "unit": "GB/s", "ms_per_step": round(dt * 1e3, 4), "n_gpus": 1,
                      "config": {"rows": m, "cols": n, "nnz": nnz, "S": a.S,
                                 "dim": "rowwise" if a.rowwise else "columnwise",
                                 "out_shape": list(out.shape), "sparse_out": a.sparse_out},
                      "checksum": float((out.values() if out.layout != torch.strided else out).float().norm())}))


if __name__ == "__main__":
    sys.exit(main())
