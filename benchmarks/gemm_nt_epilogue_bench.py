"""NT GEMM (gemm_nt.hip) on the random-feature shape, 1e6 x 4096 with the
cosine map, f32 and bf16 out, K = 64 (epilogue-dominated) and K = 512 (the
K1 target), and torch.mm (hipBLASLt, no map) on the same operands.  One
JSON line per case."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libskylark_amd.ops import _lib, gemm  # noqa: E402


def main():
    reps = int(os.environ.get("AB_REPS", 5))
    import ctypes as C
    _lib.require()
    _lib.register("sl_gemm_nt_set_nt_store", [C.c_int], None)
    nts = [int(x) for x in os.environ.get("GEMM_NT_STORE", "-1").split(",")]
    M, N = 1_000_000, 4096
    for K in (64, 512):
        A = torch.randn(M, K, device="cuda").bfloat16()
        B = torch.randn(N, K, device="cuda").bfloat16()
        sc = torch.rand(N, device="cuda") * 0.2
        sh = torch.rand(N, device="cuda") * 6.28
        for odt in (torch.bfloat16, torch.float32):
            out = torch.empty(M, N, device="cuda", dtype=odt)
            f = lambda: gemm.gemm_nt(A, B, out=out, alpha=0.3, cos_scales=sc, cos_shifts=sh)
            for nt in nts:
                _lib.require().sl_gemm_nt_set_nt_store(nt)
                f()
                torch.cuda.synchronize()
                best = 1e9
                for _ in range(3):
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        f()
                    torch.cuda.synchronize()
                    best = min(best, (time.perf_counter() - t0) / reps * 1e3)
                print(json.dumps({"bench": "gemm_nt_epilogue", "M": M, "N": N, "K": K, "map": "cos", "nt_store": nt,
                                  "out": str(odt).split(".")[-1], "ms": round(best, 3),
                                  "TF": round(2.0 * M * N * K / best / 1e9, 1),
                                  "out_TBps": round(out.numel() * out.element_size() / best / 1e9, 2)}), flush=True)
            _lib.require().sl_gemm_nt_set_nt_store(-1)
            # the library's plain GEMM (no map) on the same operands, same box
            if odt == torch.bfloat16:
                g = lambda: torch.mm(A, B.t(), out=out)
            else:
                g = lambda: torch.mm(A, B.t(), out_dtype=torch.float32, out=out)
            g()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(3):
                t0 = time.perf_counter()
                for _ in range(reps):
                    g()
                torch.cuda.synchronize()
                best = min(best, (time.perf_counter() - t0) / reps * 1e3)
            print(json.dumps({"bench": "hipblaslt_plain_gemm", "M": M, "N": N, "K": K, "map": "none",
                              "out": str(odt).split(".")[-1], "ms": round(best, 3),
                              "TF": round(2.0 * M * N * K / best / 1e9, 1)}), flush=True)
            del out
        del A, B


if __name__ == "__main__":
    main()
