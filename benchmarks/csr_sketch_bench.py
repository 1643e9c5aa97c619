"""Dense (JLT) sketch of a large CSR matrix on one GPU (csr_sketch.hip).

A: 1e7 x 1e4 CSR, 10 nonzeros per row (1e8 nnz, f32 values, int32 column
indices), sketch size S = 256.
  rowwise     A S^T  (1e7 x 256): the panel kernel on A, one realised panel
  columnwise  S A    (256 x 1e4): CSR of A^T (timed separately), 39 panels
Prints one JSON line per direction: ms, GB/s of CSR bytes (values + column
indices + row pointers), and the phase split.
usage: python benchmarks/csr_sketch_bench.py [--rows R] [--cols C] [--nnz-per-row K] [--S S]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import dense_sketch as DS  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return out, min(ts) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--cols", type=int, default=10_000)
    ap.add_argument("--nnz-per-row", type=int, default=10)
    ap.add_argument("--S", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m, n, k, S = a.rows, a.cols, a.nnz_per_row, a.S
    g = torch.Generator(device=dev).manual_seed(0)
    cols = torch.randint(0, n, (m, k), device=dev, generator=g, dtype=torch.int32).sort(dim=1).values.reshape(-1)
    vals = torch.randn(m * k, device=dev, generator=g)
    rowptr = torch.arange(0, m * k + 1, k, device=dev, dtype=torch.int64)
    A = torch.sparse_csr_tensor(rowptr, cols, vals, (m, n))
    csr_bytes = vals.numel() * 4 + cols.numel() * 4 + rowptr.numel() * 8
    kw = dict(dist=D.Normal(), seed=5, base=0, scale=S ** -0.5)
    # rowwise: A S^T, S is S x n
    Y, ms = timed(lambda: DS.csr_sketch_native(A, S=S, N=n, **kw))
    print(json.dumps({"direction": "rowwise", "shape": [m, n], "nnz": m * k, "S": S, "ms": round(ms, 3),
                      "csr_GBps": round(csr_bytes / ms / 1e6, 1),
                      "out_GBps": round(Y.numel() * 4 / ms / 1e6, 1)}), flush=True)
    del Y
    # columnwise: S A with S S x m: CSR of A^T, then the panel kernel
    At, ms_t = timed(lambda: DS._csr_transpose(A), reps=1)
    Z, ms_k = timed(lambda: DS.csr_sketch_native(At, S=S, N=m, **kw))
    print(json.dumps({"direction": "columnwise", "shape": [m, n], "nnz": m * k, "S": S,
                      "ms": round(ms_t + ms_k, 3), "transpose_ms": round(ms_t, 3), "kernel_ms": round(ms_k, 3),
                      "panels": -(-m // (DS.SPARSE_PANEL_ELEMS // S)),
                      "csr_GBps_kernel": round(csr_bytes / ms_k / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
