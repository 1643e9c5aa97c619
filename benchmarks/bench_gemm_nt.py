"""Hand-written bf16 NT GEMM (gemm_nt.hip) against hipBLASLt (torch.matmul)
on the framework's shapes: square 8192^3, LSRN's sketch panel product
(t = 2e4 sketch rows x 26.8k panel x 1e4 [A_hi | A_lo] columns) and the
random-feature map (1e6 x 512 -> 4096, cos epilogue, bf16 / f32 out).
Prints one JSON line per case: ms and TFLOP/s of both."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libskylark_amd.ops import _lib, gemm  # noqa: E402
import ctypes  # noqa: E402

# A/B builds of gemm_nt.hip: GEMM_AB_LIBS="tag:path,tag:path"
AB = [(t, ctypes.CDLL(p)) for t, p in (e.split(":", 1) for e in os.environ.get("GEMM_AB_LIBS", "").split(",") if e)]


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def case(name, M, N, K, out_dtype=torch.float32, cos=False):
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=out_dtype)
    sc = torch.rand(N, device="cuda") if cos else None
    sh = torch.rand(N, device="cuda") if cos else None
    ours = {0: timeit(lambda: gemm.gemm_nt(A, B, out=C, cos_scales=sc, cos_shifts=sh))}
    outs = {0: C.float().clone()} if M * N <= 1 << 27 else {}
    tags = {0: "ours"}
    for vi, (tag, L) in enumerate(AB, start=1):   # A/B against other builds of gemm_nt.hip
        vp = ctypes.c_void_p
        f = lambda L=L: L.sl_gemm_nt_bf16(vp(A.data_ptr()), ctypes.c_int64(K), vp(B.data_ptr()), ctypes.c_int64(K),
                                          M, N, K, vp(C.data_ptr()), ctypes.c_int64(N),
                                          _lib.dtype_code(out_dtype), 0, int(cos), ctypes.c_float(1.0),
                                          vp(sc.data_ptr() if cos else None), vp(sh.data_ptr() if cos else None),
                                          vp(_lib.stream_of(A)))
        ours[vi] = timeit(f)
        tags[vi] = tag
        if outs:
            outs[vi] = C.float().clone()
    Bt = B.t()
    if out_dtype == torch.float32:
        lib = timeit(lambda: torch.mm(A, Bt, out_dtype=torch.float32))
    else:
        lib = timeit(lambda: torch.mm(A, Bt))
    errs = {}
    if outs:
        if out_dtype == torch.float32 and not cos:
            ref = torch.mm(A, Bt, out_dtype=torch.float32)
        else:
            ref = A.float() @ B.float().t() if M * N <= 1 << 26 else None
            if ref is not None and cos:
                ref = torch.cos(ref * sc + sh)
        if ref is not None:
            for v, o in outs.items():
                errs[v] = float((o - ref).abs().max() / ref.abs().max())
    fl = 2.0 * M * N * K
    rec = {"case": name, "M": M, "N": N, "K": K, "out": str(out_dtype).split(".")[-1], "cos": cos,
           "hipblaslt_ms": round(lib, 3), "hipblaslt_TF": round(fl / lib / 1e9, 1)}
    for v, ms in ours.items():
        tag = tags[v]
        rec[f"{tag}_ms"] = round(ms, 3)
        rec[f"{tag}_TF"] = round(fl / ms / 1e9, 1)
        rec[f"{tag}_rel_err"] = errs.get(v)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    case("square", 8192, 8192, 8192)
    case("lsrn_panel", 20000, 10000, 26816)
    case("rft_bf16", 1_000_000, 4096, 512, torch.bfloat16, cos=True)
    case("rft_f32", 1_000_000, 4096, 512, torch.float32, cos=True)
