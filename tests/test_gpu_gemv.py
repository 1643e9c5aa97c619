"""Wide-row streaming GEMV (gemv_kernels.hip) against fp64 torch of the
same operands: row counts not a multiple of the 4-row workgroup, column
counts not a multiple of the 1024-float iteration, strided rows, k = 1, 2, 4;
and DenseOp routing a wide (n > 6144) f32 operator through it."""
import pytest
import torch

from libskylark_amd.algorithms.operators import DenseOp
from libskylark_amd.ops import normal_eq

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,n,k", [(1001, 8196, 1), (37, 20000, 2), (5000, 7000, 4), (4, 4, 1), (9, 1028, 4)])
def test_gemv_matches_fp64(m, n, k):
    g = torch.Generator(device="cuda").manual_seed(m + n + k)
    A = torch.randn(m, n, device="cuda", generator=g)
    X = torch.randn(n, k, device="cuda", generator=g)
    assert normal_eq.gemv_ok(A, k)
    Y = normal_eq.gemv(A, X)
    ref = A.double() @ X.double()
    mag = A.double().abs() @ X.double().abs()
    assert ((Y.double() - ref).abs() <= 1e-6 * mag + 1e-30).all()


def test_gemv_strided_rows_and_vector():
    g = torch.Generator(device="cuda").manual_seed(5)
    big = torch.randn(300, 9000, device="cuda", generator=g)
    A = big[:, :8192]                      # lda 9000
    x = torch.randn(8192, device="cuda", generator=g)
    y = normal_eq.gemv(A, x)
    ref = A.double() @ x.double()
    assert y.shape == (300,)
    assert ((y.double() - ref).abs() <= 1e-6 * (A.double().abs() @ x.double().abs())).all()


def test_denseop_wide_uses_gemv():
    g = torch.Generator(device="cuda").manual_seed(9)
    K = torch.randn(2000, 8000, device="cuda", generator=g)
    X = torch.randn(8000, 1, device="cuda", generator=g)
    op = DenseOp(K)
    torch.testing.assert_close(op.matmul(X).double(), K.double() @ X.double(), rtol=1e-5, atol=1e-4)
