"""Breakdown of the random-feature GEMM (1e6 x 512 -> 4096) on gemm_nt.hip's
map epilogues: with/without the cos map, f32 vs bf16 output, bf16 vs bf16x3
operands, rowwise vs columnwise (features along the output rows), the
Gaussian-kernel Gram map, against hipBLASLt's bf16 GEMM alone.  One JSON line
per variant."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.ops import fused as F  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    M, K, N = int(os.environ.get("M", 1_000_000)), 512, 4096
    dev = torch.device("cuda")
    A = torch.randn(M, K, device=dev)
    Ab = A.to(torch.bfloat16)
    W = torch.randn(N, K, device=dev) / 20
    Ws = F.SplitW(W)
    sc = torch.ones(N, device=dev)
    sh = torch.rand(N, device=dev) * 6.28
    fl = 2 * M * K * N
    res = []
    variants = [
        ("fused_bf16_none_f32out", lambda: F.feature_gemm(Ab, Ws, 1, epi=F.EPI_NONE, use_lo=False)),
        ("fused_bf16_cos_f32out", lambda: F.feature_gemm(Ab, Ws, 1, scales=sc, shifts=sh, epi=F.EPI_COS, use_lo=False)),
        ("fused_bf16_cos_bf16out", lambda: F.feature_gemm(Ab, Ws, 1, scales=sc, shifts=sh, epi=F.EPI_COS,
                                                          use_lo=False, out_dtype=torch.bfloat16)),
        ("fused_f32x3_cos_f32out", lambda: F.feature_gemm(A, Ws, 1, scales=sc, shifts=sh, epi=F.EPI_COS)),
        ("fused_f32x3_cos_f32out_columnwise", lambda: F.feature_gemm(A.t(), Ws, 0, scales=sc, shifts=sh,
                                                                    epi=F.EPI_COS)),
        ("fused_bf16_cos_bf16out_columnwise", lambda: F.feature_gemm(Ab.t(), Ws, 0, scales=sc, shifts=sh,
                                                                     epi=F.EPI_COS, use_lo=False,
                                                                     out_dtype=torch.bfloat16)),
        ("fused_f32x3_gauss_gram_f32out", lambda: F.feature_gemm(A, Ws, 1, scales=2 * sc, shifts=-sc,
                                                                 rowterm=-torch.ones(M, device=dev),
                                                                 epi=F.EPI_GAUSS)),
        ("hipblaslt_bf16_gemm_f32out", lambda: torch.mm(Ab, Ws.hi[:N, :K].t(), out_dtype=torch.float32)),
        ("hipblaslt_bf16_gemm_bf16out", lambda: torch.mm(Ab, Ws.hi[:N, :K].t())),
    ]
    for name, fn in variants:
        try:
            t = timeit(fn)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"variant": name, "error": str(e)[:200]}), flush=True)
            continue
        r = {"bench": "feature_gemm_breakdown", "variant": name, "M": M, "K": K, "N": N, "ms": round(t * 1e3, 3),
             "tflops_1term": round(fl / t / 1e12, 1)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
