"""A/B of the v4 fused randSVD pass (rsvd_pass.hip) against the v3 pass
(tsk_kernels.hip) on the headline shape (1e6 x 1e3 bf16, k = 40): numerics
of W (and of Y / the fp64 Gram in the final form) against an fp64 reference
on a row subset, then interleaved timing rounds in one process.

usage: python benchmarks/pass4_probe.py [m] [n] [k]"""
from __future__ import annotations

import ctypes as C
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from libskylark_amd.base import distributions as D  # noqa: E402
from libskylark_amd.ops import _lib, rng, tallskinny  # noqa: E402,F401

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_rsvd_pass", [vp, i64, i64, i64, vp, i32, vp, vp, i64, i32, i32, vp])
_lib.register("sl_rsvd_pass_workspace", [i64, i64, i32], C.c_int64)
_lib.register("sl_rsvd_reduce", [vp, i64, i64, i32, vp, i32, i32, vp, i32, vp])


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    dev = torch.device("cuda")
    lib = _lib.require()
    A = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    rng.fill_random(A, D.Normal(), 1, 0, ir=n, ic=1)
    Q, _ = torch.linalg.qr(torch.randn(n, k, device=dev, dtype=torch.float64))
    Zt = Q.t().contiguous().to(torch.bfloat16)
    st = vp(torch.cuda.current_stream().cuda_stream)
    KP = ((k + 15) // 16) * 16
    ws4 = torch.empty(int(lib.sl_rsvd_pass_workspace(m, n, k)), dtype=torch.uint8, device=dev)
    W4 = torch.empty(n, k, device=dev, dtype=torch.float64)
    G4 = torch.empty(k, k, device=dev, dtype=torch.float64)
    Y4 = torch.empty(m, KP, device=dev)
    ws3 = torch.empty(tallskinny.fused_workspace_bytes(m, n, k), dtype=torch.uint8, device=dev)
    WG3 = torch.empty(n + k, k, device=dev, dtype=torch.float64)

    def new(final, variant=0):
        _lib.call("sl_rsvd_pass", _lib.ptr(A), m, n, A.stride(0), _lib.ptr(Zt), k, _lib.ptr(ws4),
                  _lib.ptr(Y4) if final else None, KP, final, variant, st)
        _lib.call("sl_rsvd_reduce", _lib.ptr(ws4), m, n, k, _lib.ptr(W4), 1, k, _lib.ptr(G4) if final else None,
                  k, st)

    def old(final):
        if final:
            tallskinny.fused_pass(A, None, keep_y=True, gram=True, exact=True, ws=ws3, gram64=True, zt=Zt,
                                  wg_out=WG3)
        else:
            tallskinny.fused_pass(A, None, keep_y=False, gram=False, exact=False, ws=ws3, zt=Zt)

    # ---- numerics (fp64 reference over all rows, chunked)
    Zd = Zt.t().double()
    Wr = torch.zeros(n, k, dtype=torch.float64, device=dev)
    Gr = torch.zeros(k, k, dtype=torch.float64, device=dev)
    for r0 in range(0, m, 1 << 17):
        Ab = A[r0:r0 + (1 << 17)].double()
        y = Ab @ Zd
        Wr += Ab.t() @ y
        Gr += y.t() @ y
    out = {"m": m, "n": n, "k": k}
    for final, var in ((0, 0), (1, 0)):
        new(final, var)
        torch.cuda.synchronize()
        out[f"w_relerr_final{final}_v{var}"] = float((W4 - Wr).abs().max() / Wr.abs().max())
        if final:
            out["g_relerr"] = float((G4 - Gr).abs().max() / Gr.abs().max())
            yref = A[:4096].double() @ Zd
            out["y_relerr"] = float((Y4[:4096, :k].double() - yref).abs().max() / yref.abs().max())
            yl = A[-777:].double() @ Zd
            out["y_tail_relerr"] = float((Y4[-777:, :k].double() - yl).abs().max() / yl.abs().max())
    print(json.dumps(out), flush=True)

    # ---- timing: interleaved rounds
    cases = {"v3_inter": lambda: old(False), "v3_final": lambda: old(True),
             "v4_inter": lambda: new(0), "v4_final": lambda: new(1),
             "v4_inter_nb3": lambda: new(0, 3), "v4_final_nb3": lambda: new(1, 3)}
    times = {c: [] for c in cases}
    for f in cases.values():
        f()
    torch.cuda.synchronize()
    for _ in range(7):
        for c, f in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f()
            e1.record()
            e1.synchronize()
            times[c].append(e0.elapsed_time(e1) / 3 * 1e3)
    for c, ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"case": c, "us_median": round(med, 1), "us_min": round(min(ts), 1),
                          "TBps": round(m * n * 2 / med / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
