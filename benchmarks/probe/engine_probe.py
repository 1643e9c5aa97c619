"""The C++ randSVD engine (rsvd_engine.cpp) on the headline problem against the
current Python device path: singular values, subspace agreement, U
orthogonality, residual, per-call time (graph replay + finish) and the device
Jacobi eigensolver against numpy on random symmetric matrices.

usage: python benchmarks/probe/engine_probe.py [m]"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import libskylark_amd as sk  # noqa: E402
from libskylark_amd.ops import _lib  # noqa: E402
from libskylark_amd.parallel import init_distributed  # noqa: E402

vp, i32, i64, u64, f64 = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_double
_lib.register("sl_rsvd_plan_create", [i64, i64, i64, i32, i32, i32, C.POINTER(vp)])
_lib.register("sl_rsvd_plan_destroy", [vp])
_lib.register("sl_rsvd_set_fjlt", [vp, u64, u64, u64, f64, vp])
_lib.register("sl_rsvd_run", [vp, vp, i32, vp, i64, vp, vp, vp])
_lib.register("sl_rsvd_status", [vp, C.POINTER(i32), vp])
_lib.register("sl_sym_eig_jacobi2", [vp, i32, vp, vp, vp, i32, vp])


def jacobi_check(dev):
    st = vp(torch.cuda.current_stream().cuda_stream)
    out = []
    rs = np.random.RandomState(0)
    for k in (8, 17, 40, 48, 64):
        for kind in ("spd", "clustered", "indef"):
            if kind == "spd":
                X = rs.randn(k, 3 * k)
                Cm = X @ X.T
            elif kind == "clustered":
                Q, _ = np.linalg.qr(rs.randn(k, k))
                w = np.concatenate([np.full(k // 2, 1.0), 1e-3 * (1 + rs.rand(k - k // 2))])
                Cm = (Q * w) @ Q.T
            else:
                X = rs.randn(k, k)
                Cm = X + X.T
            Ct = torch.from_numpy(Cm).to(dev)
            w = torch.empty(k, dtype=torch.float64, device=dev)
            V = torch.empty(k, k, dtype=torch.float64, device=dev)
            status = torch.zeros(2, dtype=torch.int32, device=dev)
            _lib.call("sl_sym_eig_jacobi2", _lib.ptr(Ct), k, _lib.ptr(w), _lib.ptr(V), _lib.ptr(status), 0, st)
            torch.cuda.synchronize()
            wr = np.sort(np.linalg.eigvalsh(Cm))[::-1]
            wn, Vn = w.cpu().numpy(), V.cpu().numpy()
            res = np.abs(Cm @ Vn - Vn * wn).max() / np.abs(wr).max()
            orth = np.abs(Vn.T @ Vn - np.eye(k)).max()
            out.append({"k": k, "kind": kind, "w_err": float(np.abs(wn - wr).max() / np.abs(wr).max()),
                        "resid": float(res), "orth": float(orth), "status": int(status[0]),
                        "sweeps": int(status[1])})
    # timing at k = 40
    k = 40
    X = rs.randn(k, 3 * k)
    Ct = torch.from_numpy(X @ X.T).to(dev)
    w = torch.empty(k, dtype=torch.float64, device=dev)
    V = torch.empty(k, k, dtype=torch.float64, device=dev)
    status = torch.zeros(2, dtype=torch.int32, device=dev)
    for _ in range(3):
        _lib.call("sl_sym_eig_jacobi2", _lib.ptr(Ct), k, _lib.ptr(w), _lib.ptr(V), _lib.ptr(status), 0, st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        _lib.call("sl_sym_eig_jacobi2", _lib.ptr(Ct), k, _lib.ptr(w), _lib.ptr(V), _lib.ptr(status), 0, st)
    e1.record()
    e1.synchronize()
    out.append({"jacobi_k40_us": e0.elapsed_time(e1) / 20 * 1e3, "sweeps": int(status[1])})
    return out


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    n, r, q = 1000, 20, 2
    k = 2 * r
    comm = init_distributed()
    dev = torch.device("cuda", 0)
    for row in jacobi_check(dev):
        print(json.dumps(row), flush=True)
    Ad = bench.planted_matrix((m, n), "VC_STAR", comm, dev)
    A = Ad.local
    params = sk.nla.ApproximateSVDParams(num_iterations=q, sketch="FJLT")
    # exact reference: eigh of the f64 Gram A^T A
    Gm = torch.zeros(n, n, dtype=torch.float64, device=dev)
    for r0 in range(0, m, 1 << 17):
        Ab = A[r0:r0 + (1 << 17)].double()
        Gm += Ab.t() @ Ab
    ev, evec = torch.linalg.eigh(Gm)
    s0 = ev.flip(0)[:r].clamp_min(0).sqrt().float()
    V0 = evec.flip(1)[:, :r].float()
    U0 = (A.float() @ V0) / s0
    del Gm
    Us, ss, Vs = sk.nla.approximate_svd(A, r, context=sk.Context(seed=38734), params=params)
    torch.cuda.synchronize()
    print(json.dumps({"svd_py_engine_s_relerr": float(((ss - s0).abs() / s0).max()),
                      "svd_py_status": sk.nla.svd.last_device_status()}), flush=True)

    plan = vp()
    _lib.call("sl_rsvd_plan_create", m, n, A.stride(0), k, r, q, C.byref(plan))
    st = vp(torch.cuda.current_stream().cuda_stream)
    ctx = sk.Context(seed=38734)
    base_d = ctx.counter
    base_s = base_d + n

    def call(use_graph=1, pl=None):
        pl = plan if pl is None else pl
        U = torch.empty(m, r, device=dev)
        s = torch.empty(r, device=dev)
        V = torch.empty(n, r, device=dev)
        _lib.call("sl_rsvd_set_fjlt", pl, ctx.seed, base_d, base_s, math.sqrt(n / k), st)
        _lib.call("sl_rsvd_run", pl, _lib.ptr(A), use_graph, _lib.ptr(U), r, _lib.ptr(s), _lib.ptr(V), st)
        return U, s, V

    for use_graph in (0, 1):
        U, s, V = call(use_graph)
        torch.cuda.synchronize()
        stv = C.c_int(0)
        _lib.call("sl_rsvd_status", plan, C.byref(stv), st)
        Ud = U.double()
        orth = float((Ud.t() @ Ud - torch.eye(r, device=dev, dtype=torch.float64)).abs().max())
        Rr = A.float() @ V - U * s
        resid = float(Rr.double().norm() / s.double().norm())
        # subspace agreement with the Python path
        sv = torch.linalg.svdvals(U0.double().t() @ Ud)
        print(json.dumps({"graph": use_graph, "status": stv.value, "s_relerr_vs_py": float(((s - s0).abs() / s0).max()),
                          "U_subspace_min_cos": float(sv.min()), "orth_err": orth, "resid_rel": resid,
                          "s_top3": [round(float(x), 3) for x in s[:3]], "s_py_top3": [round(float(x), 3) for x in s0[:3]]}),
              flush=True)
    ts = {"engine_graph": [], "python_path": []}
    for _ in range(5):
        for name in ts:
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                if name == "engine_graph":
                    call(1)
                else:
                    sk.nla.approximate_svd(A, r, context=sk.Context(seed=38734), params=params)
            e1.record()
            e1.synchronize()
            ts[name].append(e0.elapsed_time(e1) / 10)
    for name, v in ts.items():
        print(json.dumps({"case": name, "ms_median": round(statistics.median(v), 4), "ms_min": round(min(v), 4)}), flush=True)
    _lib.call("sl_rsvd_plan_destroy", plan)
    _lib.call("sl_rsvd_plan_destroy", plan_cold)


if __name__ == "__main__":
    main()
