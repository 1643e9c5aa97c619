"""Phase times of the randSVD small-LA kernel k_gram_la (diagnostic build
benchmarks/native/libcore_stamps.so = rsvd_core.hip with -DSL_CORE_STAMPS):
partial Gram + ticket, partial sum, Cholesky/inverse, core GEMMs, Jacobi, the
factor epilogue, in microseconds of the 100 MHz s_memrealtime clock, plus the
make_zt / make_v kernels' wall time."""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    n, k, r = 1000, 40, 20
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libcore_stamps.so"))
    vp, i32 = C.c_void_p, C.c_int
    lib.sl_rsvd_gram_workspace.argtypes = [i32]
    lib.sl_rsvd_gram_workspace.restype = C.c_int64
    lib.sl_rsvd_inter_la.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp]
    lib.sl_rsvd_final_la.argtypes = [vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp, i32, vp, vp, vp]
    lib.sl_rsvd_make_zt.argtypes = [vp, i32, i32, i32, vp, vp, vp]
    lib.sl_rsvd_make_v.argtypes = [vp, i32, i32, i32, vp, i32, vp, vp, vp, vp]
    dev = torch.device("cuda")
    p = lambda t: vp(t.data_ptr()) if t is not None else None  # noqa: E731
    g = torch.Generator(device="cpu").manual_seed(0)
    # W with a graded spectrum (like A^T A Z after power steps)
    Q1, _ = torch.linalg.qr(torch.randn(n, k, dtype=torch.float64, generator=g))
    Q2, _ = torch.linalg.qr(torch.randn(k, k, dtype=torch.float64, generator=g))
    sv = torch.logspace(6, 1, k, dtype=torch.float64)
    W = ((Q1 * sv) @ Q2.t()).to(dev)
    Yg = torch.randn(3 * k, k, dtype=torch.float64, generator=g)
    Gy = (Yg.t() @ Yg).to(dev)
    ws = torch.zeros(int(lib.sl_rsvd_gram_workspace(k)), dtype=torch.uint8, device=dev)
    Rinv = torch.empty(k, k, dtype=torch.float64, device=dev)
    st = torch.zeros(4, dtype=torch.int32, device=dev)
    M = torch.empty(k, r, device=dev)
    N = torch.empty(k, r, dtype=torch.float64, device=dev)
    s = torch.empty(r, dtype=torch.float64, device=dev)
    s32 = torch.empty(r, device=dev)
    V0 = torch.empty(k + 1, k + 1, dtype=torch.float64, device=dev)
    v0v = torch.zeros(1, dtype=torch.int32, device=dev)
    Zt = torch.empty(k, n, dtype=torch.bfloat16, device=dev)
    V = torch.empty(n, r, device=dev)
    stream = vp(torch.cuda.current_stream().cuda_stream)
    buf = (C.c_ulonglong * 32)()

    def stamps(off, names):
        torch.cuda.synchronize()
        assert lib.sl_core_stamps(buf) == 0
        v = [buf[off + i] for i in range(len(names) + 1)]
        return {names[i]: round((v[i + 1] - v[i]) / 100.0, 2) for i in range(len(names))}

    def timed(f, reps=20):
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        e1.synchronize()
        return round(e0.elapsed_time(e1) / reps * 1e3, 1)

    inter = lambda: lib.sl_rsvd_inter_la(p(W), n, k, k, p(ws), p(Rinv), p(st), stream)  # noqa: E731
    t = timed(inter)
    inter()
    ph = stamps(0, ["partial+ticket", "sum", "chol_inv", "store"])
    print(json.dumps({"kernel": "inter_la", "us": t, "phases_us": ph, "status": int(st[0])}), flush=True)
    for warm in (0, 1):
        def fin():
            if not warm:
                v0v.zero_()
            lib.sl_rsvd_final_la(p(W), n, k, k, p(Gy), r, p(ws), p(M), p(N), p(s), p(st), 40, p(V0), p(v0v), stream)
        t = timed(fin)
        fin()
        ph = stamps(16, ["partial+ticket", "sum", "chol_inv", "gemms+warm", "jacobi", "epilogue"])
        torch.cuda.synchronize()
        rounds = max(1, int(buf[27]))
        jac = {"rounds": int(buf[27]), "cyc_rotations_per_round": round(buf[25] / rounds, 1),
               "cyc_apply_per_round": round(buf[26] / rounds, 1),
               "clock_MHz": round(buf[28] / max(1, buf[29]) * 100.0, 1)}
        print(json.dumps({"kernel": "final_la", "warm": warm, "us": t, "phases_us": ph, "sweeps": int(buf[24]),
                          "jacobi": jac, "status": int(st[0])}), flush=True)
    t = timed(lambda: lib.sl_rsvd_make_zt(p(W), n, k, k, p(Rinv), p(Zt), stream))
    Zr = (W @ Rinv).t()
    err = float((Zt.double() - Zr).abs().max() / Zr.abs().max())
    print(json.dumps({"kernel": "make_zt", "us": t, "relerr": err}), flush=True)
    t = timed(lambda: lib.sl_rsvd_make_v(p(W), n, k, k, p(N), r, p(V), p(s), p(s32), stream))
    Vr = W @ N
    err = float((V.double() - Vr).abs().max() / Vr.abs().max())
    print(json.dumps({"kernel": "make_v", "us": t, "relerr": err}), flush=True)


if __name__ == "__main__":
    main()
