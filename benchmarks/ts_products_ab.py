"""Same-box A/B of the general engine's tall-skinny products (rsvd_stream.hip):
Y = A Z work split (split 0 = whole row blocks round-robin, 1 = whole-block
rounds + stream-K tail) and W = A^T Q vectors per wave (av 2 = one
workgroup per CU, 1 = two).  Shapes of the general-engine bench (1e6 x 1000
f32, 2e5 x 5000 f64, k = 40).  One JSON line per (op, dtype, variant, repeat)."""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libskylark_amd.ops import _lib  # noqa: E402

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64


def main():
    _lib.require()
    _lib.register("sl_ts_az", [vp, i64, i64, i64, vp, i32, vp, i64, i32, vp])
    _lib.register("sl_ts_set_az_split", [i32], None)
    _lib.register("sl_ts_set_atq_av", [i32], None)
    _lib.register("sl_ts_atq_workspace", [i64, i64, i32, i32], C.c_int64)
    _lib.register("sl_ts_atq", [vp, i64, i64, i64, vp, i32, vp, i32, vp, i32, vp])
    reps = int(os.environ.get("AB_REPS", 10))
    for dt, code, m, n in ((torch.float32, 0, 1_000_000, 1000), (torch.float64, 1, 200_000, 5000)):
        k = 40
        A = torch.randn(m, n, device="cuda", dtype=dt)
        Z = torch.randn(n, k, device="cuda", dtype=dt)
        Y = torch.empty(m, k, device="cuda", dtype=dt)
        st = vp(torch.cuda.current_stream().cuda_stream)
        f = lambda: _lib.call("sl_ts_az", vp(A.data_ptr()), m, n, n, vp(Z.data_ptr()), k, vp(Y.data_ptr()), k, code, st)
        for rep in range(2):
            for split in (0, 1):
                _lib.require().sl_ts_set_az_split(split)
                f()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    f()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / reps * 1e3
                gb = A.numel() * A.element_size() / 1e9
                print(json.dumps({"bench": "ts_az_split", "dtype": str(dt).split(".")[-1], "m": m, "n": n, "k": k,
                                  "split": split, "rep": rep, "ms": round(ms, 4), "TBps": round(gb / ms, 3)}),
                      flush=True)
        _lib.require().sl_ts_set_az_split(1)
        W = torch.empty(n, k, device="cuda", dtype=torch.float64)
        for rep in range(2):
            for av in (2, 1):
                _lib.require().sl_ts_set_atq_av(av)
                ws = torch.empty(int(_lib.require().sl_ts_atq_workspace(m, n, k, code)), dtype=torch.uint8,
                                 device="cuda")
                h = lambda: _lib.call("sl_ts_atq", vp(A.data_ptr()), m, n, n, vp(Y.data_ptr()), k, vp(W.data_ptr()),
                                      k, vp(ws.data_ptr()), code, st)
                h()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    h()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / reps * 1e3
                print(json.dumps({"bench": "ts_atq_av", "dtype": str(dt).split(".")[-1], "m": m, "n": n, "k": k,
                                  "av": av, "rep": rep, "ms": round(ms, 4), "TBps": round(gb / ms, 3)}), flush=True)
        _lib.require().sl_ts_set_atq_av(2)
        del A, Z, Y, W


if __name__ == "__main__":
    main()
