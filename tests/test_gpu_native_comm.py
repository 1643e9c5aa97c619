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
