"""bf16 -> f32 GEMM throughput by operand orientation for the KRR split Gram
(C = P^T Q, 4096 x 4096, K = 16384 / 32768): torch.mm TN (row-major K x s
operands, the current form), NT (transposed s x K operands) and the hand-
written gemm_nt.  usage: python benchmarks/probe/gemm_orient_ab.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from libskylark_amd.ops import gemm  # noqa: E402


def tm(f, it=10):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3


dev = torch.device("cuda")
s = 4096
res = {}
for K in (16384, 32768):
    P = torch.randn(K, s, device=dev).to(torch.bfloat16)
    Q = torch.randn(K, s, device=dev).to(torch.bfloat16)
    Pt, Qt = P.t().contiguous(), Q.t().contiguous()
    fl = 2 * s * s * K
    t1 = tm(lambda: torch.mm(P.t(), Q, out_dtype=torch.float32))
    t2 = tm(lambda: torch.mm(Pt, Qt.t(), out_dtype=torch.float32))
    C = torch.empty(s, s, device=dev)
    t3 = tm(lambda: gemm.gemm_nt(Pt, Qt, out=C))
    t4 = tm(lambda: torch.mm(P.t(), Q))
    res[f"K{K}"] = {"tn_f32out_TF": round(fl / t1 / 1e9, 1), "nt_f32out_TF": round(fl / t2 / 1e9, 1),
                    "gemm_nt_TF": round(fl / t3 / 1e9, 1), "tn_bf16out_TF": round(fl / t4 / 1e9, 1)}
print(json.dumps(res))
