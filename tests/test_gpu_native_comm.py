"""Native RCCL communicator (native_comm.cpp) on the box's one GPU: a
single-rank communicator through every entry point (RCCL needs a GPU per
rank, so multi-rank runs are the 8-GPU driver's), against the identity each
collective reduces to at p = 1."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_native_comm_single_rank(dev):
    from libskylark_amd.parallel import native_comm as NC
    if not NC.available():
        pytest.skip("RCCL not loadable")
    c = NC.NativeComm()
    assert (c.rank, c.size) == (0, 1)
    x = torch.randn(1000, dtype=torch.float64, device=dev)
    y = x.clone()
    c.all_reduce(y)
    torch.testing.assert_close(y, x, rtol=0, atol=0)
    c.all_reduce(y, "max")
    torch.testing.assert_close(y, x, rtol=0, atol=0)
    z = torch.randn(64, dtype=torch.float32, device=dev)
    torch.testing.assert_close(c.reduce_scatter(z), z, rtol=0, atol=0)
    torch.testing.assert_close(c.all_gather(z)[0], z, rtol=0, atol=0)
    b = torch.arange(10, dtype=torch.int64, device=dev)
    torch.testing.assert_close(c.broadcast(b.clone()), b)
    w = torch.randn(33, dtype=torch.bfloat16, device=dev)
    torch.testing.assert_close(c.all_to_all_v(w, [33], [33]), w, rtol=0, atol=0)
    torch.cuda.synchronize()
    c.close()


def _capi_comm_worker(rank, world, dtype_name):
    """sl_rsvd_run_comm (fused bf16 engine) / sl_rsvd_gen_run_comm (f32
    general engine) driven by ONE C call per rank at world size 2, the [W; G]
    sums going through a callback communicator (sl_comm_from_allreduce) that
    all-reduces over this test's gloo group -- the same segment / reduce loop
    the C ABI runs on an RCCL communicator across GPUs.  Each rank holds half
    the rows of one global matrix; returns (s, V, this rank's U rows)."""
    import ctypes as C
    import math
    import torch
    import torch.distributed as dist
    import libskylark_amd as sk
    from libskylark_amd.ops import _lib
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    vp, i32, i64, u64, f64 = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_double
    L = _lib.require()
    m, n, r, k, q = 24_000, 512, 8, 16, 1
    g = torch.Generator(device=dev).manual_seed(7)
    U0 = torch.linalg.qr(torch.randn(m, r, device=dev, dtype=torch.float64, generator=g))[0]
    V0 = torch.linalg.qr(torch.randn(n, r, device=dev, dtype=torch.float64, generator=g))[0]
    Afull = (U0 * (10.0 * 0.7 ** torch.arange(r, device=dev))) @ V0.t() + 1e-4 * torch.randn(m, n, device=dev, dtype=torch.float64, generator=g)
    dt = torch.bfloat16 if dtype_name == "bf16" else torch.float32
    Afull = Afull.to(dt)
    rows = slice(rank * (m // world), (rank + 1) * (m // world))
    A = Afull[rows].contiguous()
    ml = A.shape[0]
    ctx = sk.Context(seed=99)
    base_d = ctx.counter
    base_s = base_d + n
    scale = math.sqrt(n / k)
    st = vp(torch.cuda.current_stream().cuda_stream)
    # the callback: sync the stream, sum the device span over gloo (host staging)
    bufs = {}

    @C.CFUNCTYPE(C.c_int, vp, vp, i64, C.c_int, C.c_int, vp, vp)
    def allreduce(send, recv, count, dtype, op, stream, user):
        assert send == recv and dtype == 1 and op == 0
        base, t = bufs["WG"]
        off = (send - base) // 8
        torch.cuda.synchronize()
        h = t[off:off + count].cpu()
        dist.all_reduce(h)
        t[off:off + count].copy_(h)
        return 0

    comm = vp()
    assert L.sl_comm_from_allreduce(rank, world, allreduce, None, C.byref(comm)) == 0
    U = torch.empty(ml, r, dtype=torch.float32, device=dev)
    s = torch.empty(r, dtype=torch.float32, device=dev)
    V = torch.empty(n, r, dtype=torch.float32, device=dev)
    h = vp()
    if dtype_name == "bf16":
        L.sl_rsvd_plan_create.argtypes = [i64, i64, i64, i32, i32, i32, C.POINTER(vp)]
        assert L.sl_rsvd_plan_create(ml, n, n, k, r, q, C.byref(h)) == 0
        WG = torch.zeros((n + k) * k, dtype=torch.float64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        L.sl_rsvd_plan_bind.argtypes = [vp, vp, vp]
        assert L.sl_rsvd_plan_bind(h, vp(WG.data_ptr()), vp(status.data_ptr())) == 0
        L.sl_rsvd_set_fjlt.argtypes = [vp, u64, u64, u64, f64, vp]
        assert L.sl_rsvd_set_fjlt(h, ctx.seed, base_d, base_s, scale, st) == 0
        bufs["WG"] = (WG.data_ptr(), WG)
        L.sl_rsvd_run_comm.argtypes = [vp, vp, vp, vp, i64, vp, vp, vp]
        rc = L.sl_rsvd_run_comm(h, vp(A.data_ptr()), comm, vp(U.data_ptr()), r, vp(s.data_ptr()), vp(V.data_ptr()), st)
    else:
        L.sl_rsvd_gen_create.argtypes = [i64, i64, i64, i32, i32, i32, i32, C.POINTER(vp)]
        assert L.sl_rsvd_gen_create(ml, n, n, k, r, q, 0, C.byref(h)) == 0
        WG = torch.zeros((n + k) * k, dtype=torch.float64, device=dev)
        L.sl_rsvd_gen_bind.argtypes = [vp, vp, vp]
        assert L.sl_rsvd_gen_bind(h, vp(WG.data_ptr()), None) == 0
        L.sl_rsvd_gen_set_fjlt.argtypes = [vp, u64, u64, u64, f64]
        assert L.sl_rsvd_gen_set_fjlt(h, ctx.seed, base_d, base_s, scale) == 0
        bufs["WG"] = (WG.data_ptr(), WG)
        L.sl_rsvd_gen_run_comm.argtypes = [vp, vp, vp, vp, i64, vp, vp, vp]
        rc = L.sl_rsvd_gen_run_comm(h, vp(A.data_ptr()), comm, vp(U.data_ptr()), r, vp(s.data_ptr()), vp(V.data_ptr()), st)
    assert rc == 0, L.sl_last_error() if hasattr(L, "sl_last_error") else rc
    torch.cuda.synchronize()
    # the same call on one rank (the whole matrix, same sketch stream)
    prm = sk.nla.ApproximateSVDParams(num_iterations=q, sketch="FJLT", oversampling_ratio=2)
    U1, s1, V1 = sk.nla.approximate_svd(Afull, r, sk.Context(seed=99), prm)
    torch.cuda.synchronize()
    L.sl_comm_destroy.argtypes = [vp]
    L.sl_comm_destroy(comm)
    return s.cpu(), s1.float().cpu(), V.cpu(), V1.float().cpu(), U.cpu(), U1[rows].float().cpu()


@pytest.mark.parametrize("dtype_name", ["bf16", "f32"])
def test_capi_run_comm_world2(dtype_name):
    from mp_utils import run_distributed
    res = run_distributed(_capi_comm_worker, 2, dtype_name, timeout=240)
    for s, s1, V, V1, U, U1 in res:
        # the two ranks sum in another order than one rank: roundoff only
        torch.testing.assert_close(s, s1, rtol=2e-5, atol=1e-6)
        sg = torch.sign((V * V1).sum(0))
        torch.testing.assert_close(V * sg, V1, rtol=0, atol=2e-4)
        torch.testing.assert_close(U * sg, U1, rtol=0, atol=2e-4)
    torch.testing.assert_close(res[0][0], res[1][0], rtol=0, atol=0)   # every rank the same s
