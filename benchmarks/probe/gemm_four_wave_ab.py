"""Same-box A/B of the NT GEMM's two main-loop forms for plain products
(gemm_nt.hip: eight waves on LDS-DMA vs four waves staged through
registers, gemm.set_four_wave) against hipBLASLt NT, on the square 8192^3,
the LSRN panel (2e4 x 1e4 x 26816, accumulate as in the sketch loop) and a
short-K product; three interleaved rounds.  (The four-wave kernel and its
gemm.set_four_wave knob were removed after this A/B:
profiles/r6/gemm_four_wave_regstage_ab.jsonl.)"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from libskylark_amd.ops import gemm  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for name, M, N, K, acc, reps in (("square", 8192, 8192, 8192, False, 20), ("lsrn_panel_acc", 20000, 10000, 26816, True, 5),
                                 ("k2048", 16384, 8192, 2048, False, 20)):
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    C = torch.zeros(M, N, device="cuda")
    fl = 2.0 * M * N * K
    ref = None
    for rnd in range(3):
        rec = {"case": name, "round": rnd}
        for fw in (0, 1):
            gemm.set_four_wave(fw)
            ms = timeit(lambda: gemm.gemm_nt(A, B, out=C, accumulate=acc), reps)
            rec[f"four_wave{fw}_TF"] = round(fl / ms / 1e9, 1)
            if rnd == 0 and not acc:
                if ref is None:
                    ref = C.clone()
                else:
                    rec["max_abs_diff_forms"] = float((C - ref).abs().max())
        ms = timeit(lambda: torch.addmm(C, A, B.t(), out_dtype=torch.float32, out=C) if acc
                    else torch.mm(A, B.t(), out_dtype=torch.float32), reps)
        rec["hipblaslt_TF"] = round(fl / ms / 1e9, 1)
        print(json.dumps(rec), flush=True)
    gemm.set_four_wave(-1)
    del A, B, C
    torch.cuda.empty_cache()
