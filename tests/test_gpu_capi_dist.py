"""DistMatrix-typed operands through the C ABI with no interpreter in the
call (skylark_capi.cpp dist_layout / native_device.hpp apply_sketch_dist):
two ranks on the box's one GPU, each passing its device shard under the
reference's type names (capi/matrix_types.cpp: DistMatrix_VC_STAR,
DistMatrix_STAR_VC, SharedMatrix, RootMatrix), the sums going through a
callback communicator (sl_device_comm_from_allreduce) that all-reduces over
this test's gloo group -- the same code an RCCL communicator drives across
GPUs.  Covers sketch application (8 layout cases x 7 sketch types),
randSVD (bf16 fused engine; f32 / f64 general engine) and symmetric randSVD
([VC,*] A), kernel Grams, FasterLeastSquares
([VC,*] A and B) and the LIBSVM reader ([VC,*] / [*,VC] examples).
Oracle: the single-rank call of the same C ABI on the whole operand
(DeviceMatrix; host "Matrix" for least squares, plus numpy lstsq) -- the
reference's distributed == local invariant
(tests/unit/DenseSketchApplyElementalTest.cpp:52-101)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

TYPES = [("JLT", []), ("CWT", []), ("FJLT", []), ("UST", []), ("GaussianRFT", [1.5]), ("FastGaussianRFT", [1.3]),
         ("PPT", [2, 0.5, 0.7])]
# (input type, output type, dim): the sketched dimension split (partial sums),
# the other one split (local), replicated / root inputs and outputs
CASES = [("DistMatrix_VC_STAR", "SharedMatrix", 0), ("DistMatrix_VC_STAR", "DistMatrix_VC_STAR", 0),
         ("DistMatrix_VC_STAR", "DistMatrix_VC_STAR", 1), ("DistMatrix_VR_STAR", "RootMatrix", 1),
         ("DistMatrix_STAR_VC", "SharedMatrix", 1), ("DistMatrix_STAR_VR", "DistMatrix_STAR_VC", 0),
         ("SharedMatrix", "DistMatrix_STAR_VC", 0), ("RootMatrix", "SharedMatrix", 1)]


def _worker(rank, world):
    import ctypes as C
    import numpy as np
    import torch
    import torch.distributed as dist
    from libskylark_amd._native import build as B
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    lib = C.CDLL(B.CAPI_LIB)
    vp, i64 = C.c_void_p, C.c_int64
    lib.sl_device_memcpy.argtypes = [vp, vp, i64, C.c_int]
    lib.sl_wrap_raw_dist_device_matrix.argtypes = [vp, C.c_int, i64, i64, i64, vp, C.POINTER(vp)]
    lib.sl_wrap_raw_device_matrix.argtypes = [vp, C.c_int, C.c_int, C.c_int, i64, C.POINTER(vp)]
    lib.sl_dist_local_shape.argtypes = [C.c_char_p, i64, i64, vp] + [C.POINTER(i64)] * 4
    lib.sl_apply_sketch_transform.argtypes = [vp, C.c_char_p, vp, C.c_char_p, vp, C.c_int]
    lib.sl_get_exception_info.argtypes = [C.POINTER(C.c_char_p)]

    def err():
        e = C.c_char_p()
        lib.sl_get_exception_info(C.byref(e))
        return e.value

    @C.CFUNCTYPE(C.c_int, vp, vp, i64, C.c_int, C.c_int, vp, vp)
    def allreduce(send, recv, count, dtype, op, stream, user):
        assert op == 0
        h = np.empty(count, dtype={0: np.float32, 1: np.float64}[dtype])
        lib.sl_device_memcpy(h.ctypes.data, send, h.nbytes, 1)
        t = torch.from_numpy(h)
        dist.all_reduce(t)
        lib.sl_device_memcpy(recv, h.ctypes.data, h.nbytes, 0)
        return 0

    comm = vp()
    assert lib.sl_device_comm_from_allreduce(rank, world, allreduce, None, C.byref(comm)) == 0, err()

    def shard(typ, m, n):
        v = [i64() for _ in range(4)]
        assert lib.sl_dist_local_shape(typ.encode(), m, n, comm, *[C.byref(x) for x in v]) == 0, err()
        return [x.value for x in v]

    def dwrap(typ, G, m, n):
        """this rank's shard of the global m x n matrix G (None: allocate) -> (tensor, wrap)"""
        r0, c0, lm, ln = shard(typ, m, n)
        loc = (G[r0:r0 + lm, c0:c0 + ln].contiguous() if G is not None
               else torch.full((lm, ln), float("nan"), dtype=torch.float64, device=dev))
        if loc.numel() == 0:
            loc = torch.empty(max(lm, 1), max(ln, 1), dtype=torch.float64, device=dev)
        h = vp()
        assert lib.sl_wrap_raw_dist_device_matrix(loc.data_ptr(), 1, m, n, loc.stride(0), comm, C.byref(h)) == 0
        return loc, h, (r0, c0, lm, ln)

    def local_call(sk_h, A, out_shape, dim):
        out = torch.zeros(*out_shape, dtype=torch.float64, device=dev)
        ha, ho = vp(), vp()
        lib.sl_wrap_raw_device_matrix(A.data_ptr(), 1, A.shape[0], A.shape[1], A.stride(0), C.byref(ha))
        lib.sl_wrap_raw_device_matrix(out.data_ptr(), 1, out.shape[0], out.shape[1], out.stride(0), C.byref(ho))
        assert lib.sl_apply_sketch_transform(sk_h, b"DeviceMatrix", ha, b"DeviceMatrix", ho, dim) == 0, err()
        return out

    ctx = vp()
    assert lib.sl_create_default_context(31, C.byref(ctx)) == 0
    g = torch.Generator(device=dev).manual_seed(4)
    N, S = 301, 64
    A0 = torch.randn(N, 23, dtype=torch.float64, device=dev, generator=g)   # dim 0: N x n
    A1 = torch.randn(19, N, dtype=torch.float64, device=dev, generator=g)   # dim 1: m x N
    worst = {}
    for typ, params in TYPES:
        spec = {"PPT": "idd"}.get(typ, "d" * len(params))
        args = [C.c_int(int(p)) if c == "i" else C.c_double(float(p)) for c, p in zip(spec, params)]
        h = vp()
        assert lib.sl_create_sketch_transform(ctx, typ.encode(), N, S, C.byref(h), *args) == 0, err()
        ref = {0: local_call(h, A0, (S, A0.shape[1]), 0), 1: local_call(h, A1, (A1.shape[0], S), 1)}
        for tin, tout, dim in CASES:
            A = A0 if dim == 0 else A1
            om, on = (S, A.shape[1]) if dim == 0 else (A.shape[0], S)
            _, ha, _ = dwrap(tin, A, *A.shape)
            out, ho, (r0, c0, lm, ln) = dwrap(tout, None, om, on)
            rc = lib.sl_apply_sketch_transform(h, tin.encode(), ha, tout.encode(), ho, dim)
            assert rc == 0, (typ, tin, tout, dim, rc, err())
            torch.cuda.synchronize()
            if lm * ln:
                d = (out[:lm, :ln] - ref[dim][r0:r0 + lm, c0:c0 + ln]).abs().max().item()
                worst[(typ, tin, tout, dim)] = d / max(1.0, ref[dim].abs().max().item())
        lib.sl_free_sketch_transform(h)

    # 2-D [MC,MR] operands are refused with a clear code
    h = vp()
    assert lib.sl_create_sketch_transform(ctx, b"JLT", N, S, C.byref(h)) == 0
    _, ha, _ = dwrap("SharedMatrix", A0, *A0.shape)
    out, ho, _ = dwrap("SharedMatrix", None, S, A0.shape[1])
    mcmr = lib.sl_apply_sketch_transform(h, b"DistMatrix", ha, b"SharedMatrix", ho, 0)

    # randSVD of a row-distributed bf16 matrix (U in its rows, S / V replicated)
    # against the one-rank DeviceMatrix call on the whole matrix
    m, n, r = 12_000, 256, 6
    U0 = torch.linalg.qr(torch.randn(m, r, dtype=torch.float64, device=dev, generator=g))[0]
    V0 = torch.linalg.qr(torch.randn(n, r, dtype=torch.float64, device=dev, generator=g))[0]
    Af = ((U0 * (10.0 * 0.6 ** torch.arange(r, device=dev))) @ V0.t()
          + 1e-4 * torch.randn(m, n, dtype=torch.float64, device=dev, generator=g)).to(torch.bfloat16)
    r0, c0, lm, ln = shard("DistMatrix_VC_STAR", m, n)
    Al = Af[r0:r0 + lm].contiguous()
    Ul = torch.empty(lm, r, dtype=torch.float32, device=dev)
    sv = torch.empty(r, 1, dtype=torch.float32, device=dev)
    Vd = torch.empty(n, r, dtype=torch.float32, device=dev)
    hs = []
    for t, dt, gm, gn, ld in ((Al, 2, m, n, n), (Ul, 0, m, r, r), (sv, 0, r, 1, 1), (Vd, 0, n, r, r)):
        w = vp()
        assert lib.sl_wrap_raw_dist_device_matrix(t.data_ptr(), dt, gm, gn, ld, comm, C.byref(w)) == 0
        hs.append(w)
    prm = b'{"num_iterations": 1, "sketch": "FJLT"}'
    lib.sl_approximate_svd.argtypes = [C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp, C.c_uint16,
                                       C.c_char_p, vp]
    c1 = vp()
    assert lib.sl_create_default_context(77, C.byref(c1)) == 0
    rc = lib.sl_approximate_svd(b"DistMatrix_VC_STAR", hs[0], b"DistMatrix_VC_STAR", hs[1], b"SharedMatrix", hs[2],
                                b"SharedMatrix", hs[3], r, prm, c1)
    assert rc == 0, err()
    Uw = torch.empty(m, r, dtype=torch.float32, device=dev)
    s1 = torch.empty(r, 1, dtype=torch.float32, device=dev)
    Vw = torch.empty(n, r, dtype=torch.float32, device=dev)
    ws = []
    for t, dt in ((Af, 2), (Uw, 0), (s1, 0), (Vw, 0)):
        w = vp()
        lib.sl_wrap_raw_device_matrix(t.data_ptr(), dt, t.shape[0], t.shape[1], t.stride(0), C.byref(w))
        ws.append(w)
    c2 = vp()
    assert lib.sl_create_default_context(77, C.byref(c2)) == 0
    assert lib.sl_approximate_svd(b"DeviceMatrix", ws[0], b"DeviceMatrix", ws[1], b"DeviceMatrix", ws[2],
                                  b"DeviceMatrix", ws[3], r, prm, c2) == 0, err()
    torch.cuda.synchronize()
    sg = torch.sign((Vd * Vw).sum(0))
    svd = ((sv - s1).abs().max().item() / s1.abs().max().item(), (Vd * sg - Vw).abs().max().item(),
           (Ul * sg - Uw[r0:r0 + lm]).abs().max().item())

    # f32 / f64 A on the general engine through the same entry point: the
    # row-distributed f32 call vs the one-rank f32 call, and f64 vs numpy
    gm_, gn_, gr_ = 9000, 300, 8
    U1_ = torch.linalg.qr(torch.randn(gm_, 16, dtype=torch.float64, device=dev, generator=g))[0]
    V1_ = torch.linalg.qr(torch.randn(gn_, 16, dtype=torch.float64, device=dev, generator=g))[0]
    A64_ = (U1_ * (20.0 * 0.75 ** torch.arange(16, device=dev))) @ V1_.t() + 1e-6 * torch.randn(
        gm_, gn_, dtype=torch.float64, device=dev, generator=g)
    gen = {}
    for dtn, tdt, dcode in (("f32", torch.float32, 0), ("f64", torch.float64, 1)):
        Ag = A64_.to(tdt)
        r0g, _, lmg, _ = shard("DistMatrix_VC_STAR", gm_, gn_)
        tens = (Ag[r0g:r0g + lmg].contiguous(), torch.empty(lmg, gr_, dtype=tdt, device=dev),
                torch.empty(gr_, 1, dtype=tdt, device=dev), torch.empty(gn_, gr_, dtype=tdt, device=dev))
        hw = []
        for t_, (gm2, gn2) in zip(tens, ((gm_, gn_), (gm_, gr_), (gr_, 1), (gn_, gr_))):
            w = vp()
            assert lib.sl_wrap_raw_dist_device_matrix(t_.data_ptr(), dcode, gm2, gn2, t_.stride(0), comm, C.byref(w)) == 0
            hw.append(w)
        cg = vp()
        assert lib.sl_create_default_context(88, C.byref(cg)) == 0
        pj = b'{"num_iterations": 2, "sketch": "JLT"}'
        assert lib.sl_approximate_svd(b"DistMatrix_VC_STAR", hw[0], b"DistMatrix_VC_STAR", hw[1], b"SharedMatrix", hw[2],
                                      b"SharedMatrix", hw[3], gr_, pj, cg) == 0, err()
        one = (torch.empty(gm_, gr_, dtype=tdt, device=dev), torch.empty(gr_, 1, dtype=tdt, device=dev),
               torch.empty(gn_, gr_, dtype=tdt, device=dev))
        ww = []
        for t_ in (Ag,) + one:
            w = vp()
            lib.sl_wrap_raw_device_matrix(t_.data_ptr(), dcode, t_.shape[0], t_.shape[1], t_.stride(0), C.byref(w))
            ww.append(w)
        cg2 = vp()
        assert lib.sl_create_default_context(88, C.byref(cg2)) == 0
        assert lib.sl_approximate_svd(b"DeviceMatrix", ww[0], b"DeviceMatrix", ww[1], b"DeviceMatrix", ww[2],
                                      b"DeviceMatrix", ww[3], gr_, pj, cg2) == 0, err()
        torch.cuda.synchronize()
        s_true = torch.linalg.svdvals(A64_)[:gr_]
        sgn_ = torch.sign((tens[3] * one[2]).sum(0))
        gen[dtn] = ((tens[2].ravel() - one[1].ravel()).abs().max().item() / one[1].abs().max().item(),
                    (tens[3] * sgn_ - one[2]).abs().max().item(),
                    ((one[1].ravel().double() - s_true).abs() / s_true).max().item())

    # kernel Gram with X's points (rows) split [VC,*], Y replicated -> K rows [VC,*]
    lib.sl_create_kernel.restype = C.c_int
    kh = vp()
    assert lib.sl_create_kernel(b"gaussian", 8, C.byref(kh), C.c_double(0.9)) == 0
    X = torch.randn(41, 8, dtype=torch.float64, device=dev, generator=g)
    Y = torch.randn(8, 17, dtype=torch.float64, device=dev, generator=g)
    Xl, hx, _ = dwrap("DistMatrix_VC_STAR", X, 41, 8)
    Yl, hy, _ = dwrap("SharedMatrix", Y, 8, 17)
    Kl, hk, (kr0, _, klm, _) = dwrap("DistMatrix_VC_STAR", None, 41, 17)
    lib.sl_kernel_gram.argtypes = [C.c_int, C.c_int, vp, C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp]
    assert lib.sl_kernel_gram(2, 1, kh, b"DistMatrix_VC_STAR", hx, b"SharedMatrix", hy, b"DistMatrix_VC_STAR", hk) == 0, err()
    Kref = torch.zeros(41, 17, dtype=torch.float64, device=dev)
    wx, wy, wk = vp(), vp(), vp()
    lib.sl_wrap_raw_device_matrix(X.data_ptr(), 1, 41, 8, 8, C.byref(wx))
    lib.sl_wrap_raw_device_matrix(Y.data_ptr(), 1, 8, 17, 17, C.byref(wy))
    lib.sl_wrap_raw_device_matrix(Kref.data_ptr(), 1, 41, 17, 17, C.byref(wk))
    assert lib.sl_kernel_gram(2, 1, kh, b"DeviceMatrix", wx, b"DeviceMatrix", wy, b"DeviceMatrix", wk) == 0, err()
    torch.cuda.synchronize()
    kdiff = (Kl[:klm] - Kref[kr0:kr0 + klm]).abs().max().item()
    # least squares with A and B row-distributed, X replicated, against the
    # one-rank host-operand call on the same context stream and numpy
    mL, nL, nr = 3000, 40, 2
    gA = np.random.RandomState(8)
    Ah = gA.randn(mL, nL) @ np.diag(np.logspace(0, 3, nL))
    Bh = Ah @ gA.randn(nL, nr) + 1e-3 * gA.randn(mL, nr)
    Ad = torch.from_numpy(Ah).to(dev)
    Bd = torch.from_numpy(Bh).to(dev)
    _, hA, _ = dwrap("DistMatrix_VC_STAR", Ad, mL, nL)
    _, hB, _ = dwrap("DistMatrix_VC_STAR", Bd, mL, nr)
    Xd, hX, _ = dwrap("SharedMatrix", None, nL, nr)
    lib.sl_faster_least_squares.argtypes = [C.c_int, C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp]
    c4 = vp()
    assert lib.sl_create_default_context(55, C.byref(c4)) == 0
    lsp = b'{"tolerance": 1e-14, "iter_lim": 200}'
    assert lib.sl_faster_least_squares(0, b"DistMatrix_VC_STAR", hA, b"DistMatrix_VC_STAR", hB, b"SharedMatrix", hX,
                                       lsp, c4) == 0, err()
    torch.cuda.synchronize()
    Af, Bf, Xf = np.asfortranarray(Ah), np.asfortranarray(Bh), np.zeros((nL, nr), order="F")
    wA, wB, wX = vp(), vp(), vp()
    lib.sl_wrap_raw_matrix.argtypes = [vp, C.c_int, C.c_int, C.POINTER(vp)]
    lib.sl_wrap_raw_matrix(Af.ctypes.data, mL, nL, C.byref(wA))
    lib.sl_wrap_raw_matrix(Bf.ctypes.data, mL, nr, C.byref(wB))
    lib.sl_wrap_raw_matrix(Xf.ctypes.data, nL, nr, C.byref(wX))
    c5 = vp()
    assert lib.sl_create_default_context(55, C.byref(c5)) == 0
    assert lib.sl_faster_least_squares(0, b"Matrix", wA, b"Matrix", wB, b"Matrix", wX, lsp, c5) == 0, err()
    Xls = np.linalg.lstsq(Ah, Bh, rcond=None)[0]
    xd = Xd.cpu().numpy()
    ls = (np.abs(xd - Xf).max() / np.abs(Xf).max(), np.abs(xd - Xls).max() / np.abs(Xls).max())
    # symmetric randSVD of a row-distributed symmetric A (lower triangle read;
    # garbage above it) vs the one-rank host-operand call on the same stream
    ns, rs = 400, 6
    gS = np.random.RandomState(9)
    Qs = np.linalg.qr(gS.randn(ns, ns))[0]
    Sym = (Qs * np.concatenate([50.0 * 0.7 ** np.arange(20), 1e-3 * gS.rand(ns - 20)])) @ Qs.T
    Sym = (Sym + Sym.T) / 2
    Sg = np.tril(Sym) + np.triu(gS.randn(ns, ns), 1)   # only the lower triangle is valid
    Sd = torch.from_numpy(Sg).to(dev)
    _, hS, _ = dwrap("DistMatrix_VC_STAR", Sd, ns, ns)
    sd, hs_, _ = dwrap("SharedMatrix", None, rs, 1)
    Vsd, hv, (vr0, _, vlm, _) = dwrap("DistMatrix_VC_STAR", None, ns, rs)
    lib.sl_approximate_symmetric_svd.argtypes = [C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp, C.c_uint16,
                                                 C.c_char_p, vp]
    c6 = vp()
    assert lib.sl_create_default_context(66, C.byref(c6)) == 0
    sprm = b'{"num_iterations": 2}'
    assert lib.sl_approximate_symmetric_svd(b"DistMatrix_VC_STAR", hS, b"SharedMatrix", hs_, b"DistMatrix_VC_STAR", hv,
                                            rs, sprm, c6) == 0, err()
    torch.cuda.synchronize()
    Sf = np.asfortranarray(Sg)
    sh, Vh = np.zeros((rs, 1), order="F"), np.zeros((ns, rs), order="F")
    w1, w2, w3 = vp(), vp(), vp()
    lib.sl_wrap_raw_matrix(Sf.ctypes.data, ns, ns, C.byref(w1))
    lib.sl_wrap_raw_matrix(sh.ctypes.data, rs, 1, C.byref(w2))
    lib.sl_wrap_raw_matrix(Vh.ctypes.data, ns, rs, C.byref(w3))
    c7 = vp()
    assert lib.sl_create_default_context(66, C.byref(c7)) == 0
    assert lib.sl_approximate_symmetric_svd(b"Matrix", w1, b"Matrix", w2, b"Matrix", w3, rs, sprm, c7) == 0, err()
    s_d = sd.cpu().numpy().ravel()
    Vl = Vsd[:vlm].cpu().numpy()
    Vref = Vh[vr0:vr0 + vlm]
    sgn = np.sign(np.sum(Vl * Vref, axis=0))
    sym = (np.abs(s_d - sh.ravel()).max() / np.abs(sh).max(), np.abs(Vl * sgn - Vref).max(),
           np.abs(s_d - np.linalg.eigvalsh(Sym)[::-1][:rs]).max() / 50.0)
    # LIBSVM into [VC,*] shards (examples as rows) and [*,VC] (SL_COLUMNS)
    # against the host-operand read of the same file
    import os
    import tempfile
    gL = np.random.RandomState(10)
    path = os.path.join(tempfile.gettempdir(), f"sl_dist_{os.getpid()}.libsvm")
    with open(path, "w") as f:
        for i in range(37):
            feats = sorted(gL.choice(12, size=gL.randint(1, 6), replace=False))
            f.write(f"{i % 3} " + " ".join(f"{j + 1}:{gL.rand():.6f}" for j in feats) + "\n")
    Xh = np.zeros((37, 12), order="F")
    Yh = np.zeros((37, 1), order="F")
    wx1, wy1 = vp(), vp()
    lib.sl_wrap_raw_matrix(Xh.ctypes.data, 37, 12, C.byref(wx1))
    lib.sl_wrap_raw_matrix(Yh.ctypes.data, 37, 1, C.byref(wy1))
    lib.sl_readlibsvm.argtypes = [C.c_char_p, C.c_char_p, vp, C.c_char_p, vp, C.c_int, C.c_int, C.c_int]
    assert lib.sl_readlibsvm(path.encode(), b"Matrix", wx1, b"Matrix", wy1, 2, 0, -1) == 0, err()
    io = 0.0
    for direction, xt, xshape, yt, yshape in ((2, "DistMatrix_VC_STAR", (37, 12), "DistMatrix_VC_STAR", (37, 1)),
                                              (1, "DistMatrix_STAR_VC", (12, 37), "SharedMatrix", (1, 37))):
        Xl, hx2, (xr0, xc0, xlm, xln) = dwrap(xt, None, *xshape)
        Yl, hy2, (yr0, yc0, ylm, yln) = dwrap(yt, None, *yshape)
        assert lib.sl_readlibsvm(path.encode(), xt.encode(), hx2, yt.encode(), hy2, direction, 0, -1) == 0, err()
        torch.cuda.synchronize()
        Xr = Xh if direction == 2 else Xh.T
        Yr = Yh if direction == 2 else Yh.T
        io = max(io, np.abs(Xl[:xlm, :xln].cpu().numpy() - Xr[xr0:xr0 + xlm, xc0:xc0 + xln]).max(),
                 np.abs(Yl[:ylm, :yln].cpu().numpy() - Yr[yr0:yr0 + ylm, yc0:yc0 + yln]).max())
    os.remove(path)
    lib.sl_runtime_started.restype = C.c_int
    return worst, mcmr, svd, kdiff, ls, sym, io, gen, lib.sl_runtime_started()


def test_capi_dist_matrix_world2():
    from mp_utils import run_distributed
    res = run_distributed(_worker, 2, timeout=300)
    for worst, mcmr, svd, kdiff, ls, sym, io, gen, started in res:
        assert len(worst) >= len(TYPES) * 4
        bad = {k: v for k, v in worst.items() if v > 1e-12}
        assert not bad, bad
        assert mcmr == 103
        s_rel, v_diff, u_diff = svd
        assert s_rel < 2e-5 and v_diff < 2e-4 and u_diff < 2e-4, svd
        assert kdiff < 1e-13
        assert ls[0] < 1e-9 and ls[1] < 1e-8, ls   # vs the one-rank call, vs numpy lstsq
        assert sym[0] < 1e-10 and sym[1] < 1e-8 and sym[2] < 1e-6, sym
        assert io == 0.0
        # the general engine: distributed vs one rank (f32 / f64 roundoff), s vs the true values
        assert gen["f32"][0] < 1e-5 and gen["f32"][1] < 1e-3 and gen["f32"][2] < 1e-4, gen
        assert gen["f64"][0] < 1e-12 and gen["f64"][1] < 1e-9 and gen["f64"][2] < 1e-9, gen
        assert started == 0   # no call above started the interpreter-side runtime
