"""FETCH_SIZE calibration workloads (run each under `rocprofv3 --pmc FETCH_SIZE`,
one process per workload, see scripts/pmc_calibrate.sh): operations whose
HBM read volume is known exactly, in the access shapes our kernels use.

  stream     torch.sum over a 2 GiB f32 tensor: 16-B coalesced loads, 2^31 B
  ldsdma     the randSVD pass kernel (global_load_lds_dwordx4 ring) over a
             1e6 x 1000 bf16 matrix: 2.0e9 B of A (+ Z, L2-resident)
  gather128  index_select of 2^21 random 128-B rows of a 4 GiB table
  gather64   index_select of 2^21 random 64-B rows of a 4 GiB table
  rgather128 / rgather64  the same shapes (2^24 rows) through a gather kernel
             that keeps 8 random 16-B pieces per lane in flight
             (benchmarks/calib/gather.hip): the random-access bound
  cwt        the CSR CountSketch of config 2 (1e7 x 1e4, 1e8 nnz, S = 4096):
             0.88e9 B of CSR that must be read; the rows are visited in
             random (bucket) order

Each op runs --reps times after one warm-up; prints one JSON line with the
bytes a perfect kernel reads per dispatch and a kernel-name hint for the
parser (scripts/pmc_calib_summary.py)."""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", required=True, choices=["stream", "ldsdma", "gather128", "gather64", "rgather128", "rgather64", "cwt"])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    if a.op == "stream":
        x = torch.ones(1 << 29, dtype=torch.float32, device=dev)
        fn = lambda: x.sum()  # noqa: E731
        exp, hint = x.numel() * 4, "reduce"
    elif a.op == "ldsdma":
        from libskylark_amd.ops import _lib
        vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
        _lib.require()
        _lib.register("sl_rsvd_pass", [vp, i64, i64, i64, vp, i32, vp, vp, i64, i32, i32, vp])
        _lib.register("sl_rsvd_pass_workspace", [i64, i64, i32], C.c_int64)
        m, n, k = 1_000_000, 1000, 40
        A = torch.empty(m, n, dtype=torch.bfloat16, device=dev).normal_(generator=g)
        Zt = torch.randn(k, n, device=dev, generator=g).to(torch.bfloat16)
        ws = torch.zeros(int(_lib.require().sl_rsvd_pass_workspace(m, n, k)), dtype=torch.uint8, device=dev)
        st = vp(torch.cuda.current_stream().cuda_stream)
        fn = lambda: _lib.call("sl_rsvd_pass", vp(A.data_ptr()), m, n, n, vp(Zt.data_ptr()), k,  # noqa: E731
                               vp(ws.data_ptr()), None, k, 0, 0, st)
        exp, hint = m * n * 2, "k_rsvd_pass"
    elif a.op in ("gather128", "gather64"):
        w = 32 if a.op == "gather128" else 16
        table = torch.empty(1 << 30, dtype=torch.float32, device=dev).view(-1, w)
        table.fill_(1.0)
        idx = torch.randint(0, table.shape[0], (1 << 21,), generator=g, device=dev)
        out = torch.empty(idx.numel(), w, dtype=torch.float32, device=dev)
        fn = lambda: torch.index_select(table, 0, idx, out=out)  # noqa: E731
        exp, hint = idx.numel() * w * 4, "gather_kernel"
    elif a.op in ("rgather128", "rgather64"):
        rb = 128 if a.op == "rgather128" else 64
        lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "calib", "libcalib.so"))
        lib.calib_rgather.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_void_p]
        table = torch.ones(1 << 30, dtype=torch.float32, device=dev)
        nrow = table.numel() * 4 // rb
        idx = torch.randint(0, nrow, (1 << 24,), generator=g, device=dev)
        out = torch.empty(idx.numel() * rb // 4, dtype=torch.float32, device=dev)
        st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        fn = lambda: lib.calib_rgather(C.c_void_p(table.data_ptr()), C.c_void_p(idx.data_ptr()),  # noqa: E731
                                       idx.numel(), rb, C.c_void_p(out.data_ptr()), st)
        exp, hint = idx.numel() * rb, "k_rgather"
    else:
        import libskylark_amd as sk
        m, n, z = 10_000_000, 10_000, 10
        nnz = m * z
        rowptr = torch.arange(0, nnz + 1, z, dtype=torch.int64, device=dev)
        col = torch.randint(0, n, (nnz,), generator=g, device=dev, dtype=torch.int64)
        col = col.view(m, z).sort(dim=1).values.reshape(-1).to(torch.int32)
        val = torch.randn(nnz, generator=g, device=dev, dtype=torch.float32)
        A = torch.sparse_csr_tensor(rowptr, col, val, (m, n))
        S = sk.sketch.CWT(m, 4096, context=sk.Context(11))
        fn = lambda: S.apply(A, dim=sk.sketch.COLUMNWISE)  # noqa: E731
        exp, hint = nnz * 8 + (m + 1) * 8, "k_hash_csr"
    fn()
    torch.cuda.synchronize()
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    print(json.dumps({"op": a.op, "expected_read_bytes": exp, "kernel_hint": hint, "reps": a.reps}))


if __name__ == "__main__":
    main()
