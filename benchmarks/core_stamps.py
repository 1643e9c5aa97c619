"""Phase times of the randSVD pass-boundary kernel k_boundary (diagnostic
build benchmarks/native/libcore_stamps.so = rsvd_core.hip with
-DSL_CORE_STAMPS, see scripts/build_core_stamps.sh), on the bench shape
(n = 1000, k = 40, r = 20), in microseconds of the 100 MHz s_memrealtime
clock:

  rows        block 0: its 16 rows of W loaded into LDS
  gram        block 0: packed partial Gram of its rows
  ticket      block 0: release + ticket
  last_start  the last arriving workgroup's start, relative to block 0's
  sum         last: the nb partials summed into H
  la          last: Cholesky inverse (INTER) / the fp64 core (FINAL)
  release     last: status + generation release
  wait        block 0: from its ticket to seeing the generation (spin)
  rows_out    block 0: its rows of Z^T / V
plus each kernel's wall time from events (20 launches)."""
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
    vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
    lib.sl_rsvd_bnd_workspace.argtypes = [i32]
    lib.sl_rsvd_bnd_workspace.restype = C.c_int64
    lib.sl_rsvd_boundary.argtypes = [i32, i32, i32, i32, vp, vp, vp, i32, vp, vp, vp, vp, vp, i32,
                                     vp, vp, vp, vp, vp, vp, vp]
    dev = torch.device("cuda")
    p = lambda t: vp(t.data_ptr()) if t is not None else None  # noqa: E731
    g = torch.Generator(device="cpu").manual_seed(0)
    # [W; Gy] as the reduce leaves it: W graded (like A^T A Z), Gy = Y^T Y
    Q1, _ = torch.linalg.qr(torch.randn(n, k, dtype=torch.float64, generator=g))
    Q2, _ = torch.linalg.qr(torch.randn(k, k, dtype=torch.float64, generator=g))
    W = (Q1 * torch.logspace(6, 1, k, dtype=torch.float64)) @ Q2.t()
    Yg = torch.randn(3 * k, k, dtype=torch.float64, generator=g)
    Gy = Yg.t() @ Yg
    WG = torch.cat([W.ravel(), Gy.ravel()]).to(dev)
    bws = torch.zeros(int(lib.sl_rsvd_bnd_workspace(k)), dtype=torch.uint8, device=dev)
    st = torch.zeros(4, dtype=torch.int32, device=dev)
    Rinv = torch.empty(k, k, dtype=torch.float64, device=dev)
    Zt = torch.empty(k, n, dtype=torch.bfloat16, device=dev)
    M = torch.empty(k, r, device=dev)
    N = torch.empty(k, r, dtype=torch.float64, device=dev)
    s64 = torch.empty(r, dtype=torch.float64, device=dev)
    s32 = torch.empty(r, device=dev)
    V = torch.empty(n, r, device=dev)
    V0 = torch.empty(k + 1, k + 1, dtype=torch.float64, device=dev)
    v0v = torch.zeros(1, dtype=torch.int32, device=dev)
    stream = vp(torch.cuda.current_stream().cuda_stream)
    buf = (C.c_ulonglong * 32)()

    def launch(final, warm=True):
        if final:
            lib.sl_rsvd_boundary(1, n, k, r, p(WG), p(bws), p(st), 1, None, None, p(M), p(N), p(s64), 0,
                                 p(V0) if warm else None, p(v0v) if warm else None, None, p(V), p(s32), None, stream)
        else:
            lib.sl_rsvd_boundary(0, n, k, 0, p(WG), p(bws), p(st), 0, p(Rinv), p(Zt), None, None, None, 0,
                                 None, None, None, None, None, None, stream)

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

    def phases():
        torch.cuda.synchronize()
        assert lib.sl_core_stamps(buf) == 0
        b = [int(buf[i]) for i in range(11)]
        d = lambda a, c: round((b[c] - b[a]) / 100.0, 2)  # noqa: E731
        return {"rows": d(0, 1), "gram": d(1, 2), "last_start": round((b[10] - b[0]) / 100.0, 2),
                "ticket_to_last": d(2, 3), "sum": d(3, 4), "la": d(4, 5), "release": d(5, 6),
                "wait_block0": d(2, 7), "rows_out": d(7, 8), "total_block0": d(0, 8)}

    for final in (0, 1):
        t = timed(lambda: launch(final))
        launch(final)
        print(json.dumps({"kernel": "k_boundary<%s>" % ("FINAL" if final else "INTER"), "us": t,
                          "phases_us": phases(), "status": int(st[0])}), flush=True)


if __name__ == "__main__":
    main()
