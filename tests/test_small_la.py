"""GPU-resident small linear algebra (k <= 64) vs fp64 torch references."""
import pytest
import torch

from libskylark_amd.ops import small_la as SL

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 1, 2, 3, 4, 5], ids=["auto", "lds", "rolled", "wave", "lds1b", "aug"])
def impl(request):
    import ctypes
    from libskylark_amd.ops import _lib
    lib = _lib.require()
    lib.sl_small_chol_impl.argtypes = [ctypes.c_int]
    lib.sl_small_chol_impl(request.param)
    yield request.param
    lib.sl_small_chol_impl(0)


@pytest.mark.parametrize("k", [1, 7, 16, 17, 33, 40, 48, 64])
def test_chol_inv(dev, k, impl):
    X = torch.randn(3 * k + 5, k, dtype=torch.float64)
    G = X.t() @ X
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    R, Ri, Ri32 = SL.chol_inv(G.to(dev), st)
    assert int(st) == 0
    Rr = torch.linalg.cholesky(G).t()
    torch.testing.assert_close(R.cpu(), Rr, rtol=1e-10, atol=1e-10)
    torch.testing.assert_close(Ri.cpu() @ Rr, torch.eye(k, dtype=torch.float64), rtol=1e-9, atol=1e-9)
    torch.testing.assert_close(Ri32.cpu().double(), Ri.cpu(), rtol=1e-6, atol=1e-6)


def test_chol_inv_flags_breakdown(dev, impl):
    G = torch.zeros(5, 5, dtype=torch.float64, device=dev)
    G[0, 0] = 1
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    SL.chol_inv(G, st)
    assert int(st) == 1


@pytest.mark.parametrize("n,k", [(1000, 40), (64, 64), (300, 3)])
def test_cholqr2_device(dev, n, k):
    W = torch.randn(n, k, device=dev) @ torch.diag(torch.logspace(0, 2, k, device=dev))
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    Q, R = SL.cholqr2(W, st, want_r=True)
    assert int(st) == 0
    torch.testing.assert_close(Q.double().t() @ Q.double(), torch.eye(k, dtype=torch.float64, device=dev),
                               atol=2e-6, rtol=0)
    torch.testing.assert_close(Q.double() @ R, W.double(), rtol=1e-5, atol=1e-4 * float(W.abs().max()))


def test_small_matmul(dev):
    A = torch.randn(33, 17, dtype=torch.float64, device=dev)
    B = torch.randn(17, 9, dtype=torch.float64, device=dev)
    C, C32 = SL.small_matmul(A, B, want32=True)
    torch.testing.assert_close(C, A @ B)
    torch.testing.assert_close(C32, (A @ B).float())
