"""One-shot all-reduce over IPC-mapped receive buffers (oneshot_kernels.hip):
two processes on the box's one GPU (the kernel path is the same as across
GPUs: remote stores into a peer's buffer, flags, rank-ordered sums), handle
exchange over gloo.  Against the sum of the ranks' inputs computed on the
host; repeated calls exercise both buffer sets and the device generation
counter; one call is replayed from a captured hipGraph."""
import pytest
import torch

from mp_utils import run_distributed

pytestmark = pytest.mark.gpu


def _worker(rank, world):
    import torch
    from libskylark_amd.parallel import oneshot
    from libskylark_amd.parallel.comm import world as W
    torch.cuda.set_device(0)
    comm = W()
    os_ = oneshot.OneShotAllReduce(comm, cap=1 << 16)
    if not os_.ok:
        return "unavailable"
    assert os_.reason == "ok", os_.reason
    dev = torch.device("cuda", 0)
    for it, (n, dt) in enumerate([(1, torch.float64), (37, torch.float32), (4096, torch.float64),
                                  (8192, torch.float32), (300, torch.float64)] * 6):
        xs = [torch.arange(n, dtype=torch.float64) * (q + 1) + it for q in range(world)]
        ref = sum(xs)
        x = xs[rank].to(dev, dt)
        os_.all_reduce(x)
        torch.cuda.synchronize()
        assert torch.allclose(x.double().cpu(), ref, rtol=1e-6 if dt == torch.float32 else 1e-14), (it, n)
    # rank-ordered sums: bitwise identical on every rank
    y = (torch.randn(1000, dtype=torch.float64, generator=torch.Generator().manual_seed(rank)) * 1e3).to(dev)
    os_.all_reduce(y)
    got = comm.all_gather_object(y.cpu().numpy().tobytes())
    assert all(g == got[0] for g in got)
    # graph capture and replay
    z = torch.zeros(64, dtype=torch.float64, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        z.fill_(rank + 1.0)
        os_.all_reduce(z)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        z.fill_(rank + 1.0)
        os_.all_reduce(z)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.all(z.cpu() == sum(q + 1.0 for q in range(world)))
    os_.check()
    comm.barrier()
    os_.close()
    return "ok"


@pytest.mark.parametrize("world", [2, 3])
def test_oneshot_allreduce_two_processes_one_gpu(world):
    res = run_distributed(_worker, world, timeout=180)
    if all(r == "unavailable" for r in res):
        pytest.skip("IPC export of uncached device memory unavailable here")
    assert res == ["ok"] * world


def _late_worker(rank, world):
    import time
    import torch
    from libskylark_amd.parallel import oneshot
    from libskylark_amd.parallel.comm import world as W
    torch.cuda.set_device(0)
    comm = W()
    os_ = oneshot.OneShotAllReduce(comm, cap=1 << 12)
    if not os_.ok:
        return "unavailable"
    dev = torch.device("cuda", 0)
    x = torch.full((100,), float(rank + 1), dtype=torch.float64, device=dev)
    if rank == 1:
        time.sleep(2.0)          # far past rank 0's 0.3 s timeout
    os_.all_reduce(x, timeout_s=0.3)
    torch.cuda.synchronize()
    out = {"nan": bool(torch.isnan(x).all()), "sum_ok": bool(torch.all(x == 3.0))}
    try:
        os_.check()
        out["raised"] = False
    except oneshot.OneShotError:
        out["raised"] = True
    os_.close(comm)
    return out


def test_oneshot_late_peer_is_an_error_not_a_partial_sum():
    """a peer later than the timeout must not leave a
    silent partial sum -- the waiting rank's operand is NaN and the
    communicator raises; the late rank itself still gets the true sum."""
    res = run_distributed(_late_worker, 2, timeout=120)
    if all(r == "unavailable" for r in res):
        pytest.skip("IPC export of uncached device memory unavailable here")
    assert res[0] == {"nan": True, "sum_ok": False, "raised": True}, res
    assert res[1] == {"nan": False, "sum_ok": True, "raised": False}, res


def _status_worker(rank, world):
    """Comm.oneshot_status(): set up lazily by the first eligible all-reduce,
    with the self-test outcome as the reason (what bench.py records)."""
    import os
    import torch
    os.environ["SL_ONESHOT"] = "1"
    from libskylark_amd.parallel import oneshot
    oneshot.enable(True)
    from libskylark_amd.parallel.comm import world as W
    torch.cuda.set_device(0)
    comm = W()
    before = comm.oneshot_status()
    x = torch.ones(10, dtype=torch.float64, device="cuda")
    comm.all_reduce(x)
    torch.cuda.synchronize()
    after = comm.oneshot_status()
    comm.check_collectives()
    comm.close()
    return before, after, float(x[0])


def test_oneshot_status_reported():
    res = run_distributed(_status_worker, 2, timeout=120)
    for before, after, v in res:
        assert before == {"enabled": False, "reason": "never set up (no eligible all-reduce yet)"}
        assert v == 2.0
        if after["enabled"]:
            assert after["reason"] == "ok"
        else:
            assert after["reason"] and after["reason"] != "ok"   # the failing stage is named


def _late4_worker(rank, world):
    """4 ranks on the one GPU (gloo coordinates), the one-shot path forced
    on every Comm all-reduce, the bounded wait shortened to 0.3 s; rank 2
    arrives 2 s late.  The waiting ranks' operands are NaN; the collective
    check raises OneShotError on EVERY rank (the late rank summed valid data
    and would not know on its own); the communicator's next all-reduce runs
    on the backend (gloo here, RCCL in production) and is exact."""
    import os
    import time
    import torch
    os.environ["SL_ONESHOT"] = "1"
    os.environ["SL_ONESHOT_TIMEOUT_S"] = "0.3"
    from libskylark_amd.parallel import oneshot
    oneshot.enable(True)
    from libskylark_amd.parallel.comm import world as W
    torch.cuda.set_device(0)
    comm = W()
    dev = torch.device("cuda", 0)
    warm = torch.ones(8, dtype=torch.float64, device=dev)
    comm.all_reduce(warm)                       # sets the path up (collective self-test)
    torch.cuda.synchronize()
    if not comm.oneshot_status()["enabled"]:
        return "unavailable"
    x = torch.full((100,), float(rank + 1), dtype=torch.float64, device=dev)
    if rank == 2:
        time.sleep(2.0)
    comm.all_reduce(x)
    torch.cuda.synchronize()
    out = {"nan": bool(torch.isnan(x).all()), "sum_ok": bool(torch.all(x == 10.0))}
    try:
        comm.check_collectives(agree=True)
        out["raised"] = ""
    except oneshot.OneShotError as e:
        out["raised"] = str(e)
    st = comm.oneshot_status()
    out["enabled_after"] = st["enabled"]
    y = torch.full((100,), float(rank + 1), dtype=torch.float64, device=dev)
    comm.all_reduce(y)                          # the backend now
    torch.cuda.synchronize()
    out["fallback_ok"] = bool(torch.all(y == 10.0))
    comm.close()
    return out


def test_oneshot_delayed_rank_fails_on_every_rank_then_falls_back():
    """a rank delayed past the bounded wait poisons the
    waiters' operands and raises OneShotError on all four ranks; then a clean
    fallback to the backend's all-reduce on the same communicator."""
    res = run_distributed(_late4_worker, 4, timeout=180)
    if all(r == "unavailable" for r in res):
        pytest.skip("IPC export of uncached device memory unavailable here")
    for q, r in enumerate(res):
        assert r["nan"] == (q != 2) and r["sum_ok"] == (q == 2), (q, r)
        assert "timed out on rank(s)" in r["raised"], (q, r)
        assert r["enabled_after"] is False and r["fallback_ok"], (q, r)
    assert len({r["raised"] for r in res}) == 1      # the same reason on every rank
