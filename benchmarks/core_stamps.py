"""Phase times of the randSVD pass-boundary kernel k_boundary (diagnostic
build benchmarks/native/libcore_stamps.so = rsvd_core.hip with
-DSL_CORE_STAMPS, see scripts/build_core_stamps.sh) on the bench shape
(n = 1000, k = 40, r = 20), in microseconds of the 100 MHz s_memrealtime
clock.  Every FINAL launch solves its core from scratch.

  gram        block 0: rows of W loaded + packed partial Gram + ticket
  last_start  the last arriving workgroup's start, relative to block 0's
  sum         last: the nb partials summed into H
  worker      FINAL: the Y^T Y worker's Cholesky inverse (its own workgroup)
  worker_wait FINAL last: from the sum to holding the worker's Rt^-1
  la          last: Cholesky inverse (INTER) / the fp64 core (FINAL)
  core_*      FINAL core: C = Rt^-T H Rt^-1, tridiagonalisation, eigenpairs,
              M / N
  release     last: status + generation release
  wait_block0 block 0: from its ticket to seeing the generation (spin)
  rows_out    block 0: its rows of Z^T / V
plus each kernel's wall time from events (20 launches)."""
from __future__ import annotations

import ctypes as C
import json
import os

import torch


def main():
    n, k, r = 1000, 40, 20
    lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libcore_stamps.so"))
    vp, i32 = C.c_void_p, C.c_int
    lib.sl_rsvd_bnd_workspace.argtypes = [i32]
    lib.sl_rsvd_bnd_workspace.restype = C.c_int64
    lib.sl_rsvd_boundary.argtypes = [i32, i32, i32, i32, vp, vp, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    dev = torch.device("cuda")
    p = lambda t: vp(t.data_ptr()) if t is not None else None  # noqa: E731
    g = torch.Generator(device="cpu").manual_seed(0)
    # [W; Gy] as the reduce leaves it after the last pass of the bench: the
    # core C = Rt^-T W^T W Rt^-1 has 20 planted eigenvalues (ratio 0.85^2
    # apart) over a noise floor
    Q1, _ = torch.linalg.qr(torch.randn(n, k, dtype=torch.float64, generator=g))
    Q2, _ = torch.linalg.qr(torch.randn(k, k, dtype=torch.float64, generator=g))
    sv = torch.cat([1e3 * 0.85 ** torch.arange(20, dtype=torch.float64), 20 + torch.rand(k - 20, generator=g, dtype=torch.float64)])
    W = (Q1 * sv) @ Q2.t()
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
    stream = vp(torch.cuda.current_stream().cuda_stream)
    buf = (C.c_ulonglong * 32)()

    def launch(final):
        if final:
            lib.sl_rsvd_boundary(1, n, k, r, p(WG), p(bws), p(st), 1, None, None, p(M), p(N), p(s64), None,
                                 p(V), p(s32), None, stream)
        else:
            lib.sl_rsvd_boundary(0, n, k, 0, p(WG), p(bws), p(st), 0, p(Rinv), p(Zt), None, None, None, None,
                                 None, None, None, stream)

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

    def phases(final):
        torch.cuda.synchronize()
        assert lib.sl_core_stamps(buf) == 0
        b = [int(buf[i]) for i in range(32)]
        d = lambda a, c: round((b[c] - b[a]) / 100.0, 2)  # noqa: E731
        out = {"gram": d(0, 2), "last_start": round((b[10] - b[0]) / 100.0, 2), "ticket_to_last": d(2, 3),
               "sum": d(3, 4), "la": d(4, 5), "release": d(5, 6), "wait_block0": d(2, 7), "rows_out": d(7, 8),
               "total_block0": d(0, 8)}
        if final:
            out.update({"worker": d(11, 12), "worker_end_after_sum": d(4, 12), "worker_wait": d(4, 13),
                        "core_C": d(19, 20), "core_tridiag": d(20, 21), "core_eig": d(21, 22), "core_MN": d(22, 23),
                        "core_total": d(19, 23)})
        return out

    for final in (0, 1):
        t = timed(lambda: launch(final))
        launch(final)
        print(json.dumps({"kernel": "k_boundary<%s>" % ("FINAL" if final else "INTER"), "us": t,
                          "phases_us": phases(final), "status": int(st[0])}), flush=True)


if __name__ == "__main__":
    main()
