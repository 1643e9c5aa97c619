"""Native dense sketch of CSR operands (csr_sketch.hip) against the explicit
operator realised on the host in fp64 (reference dense_transform_Mixed.hpp):
rowwise A S^T and columnwise S A, f32 / f64 values, one and several panels
(sorted-column binary search), a shard at a nonzero input offset, S past one
512-wide column chunk, empty rows."""
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.base import distributions as D
from libskylark_amd.ops import dense_sketch as DS
from libskylark_amd.ops import rng

pytestmark = pytest.mark.gpu


def _csr(m, n, density, dtype, seed, empty_rows=()):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(m, n, generator=g, dtype=torch.float64)
    A = A * (torch.rand(m, n, generator=g) < density)
    for r in empty_rows:
        A[r] = 0
    return A, A.to(dtype).to_sparse_csr().cuda()


def _explicit(S, N, seed, base, scale, dtype=torch.float64):
    # S x N, entry (i, j) = scale * Normal(base + j S + i), realised like the
    # library's dense sketches (f32 operands: the f32 sampler), held in fp64
    return rng.random_matrix(S, N, D.Normal(), seed, base, scale=scale, dtype=dtype,
                             precise=dtype == torch.float64).double()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("S,panel", [(256, 1 << 24), (96, 96 * 37), (20, 20 * 5), (700, 1 << 20)])
def test_csr_sketch_rowwise_matches_explicit(dtype, S, panel):
    m, N = 3000, 400
    A, Ad = _csr(m, N, 0.03, dtype, S, empty_rows=(0, 17, m - 1))
    seed, base, scale = 77, 1234, 0.5
    Y = DS.csr_sketch_native(Ad, dist=D.Normal(), seed=seed, base=base, S=S, N=N, scale=scale, panel_elems=panel)
    ref = A.to(dtype).double() @ _explicit(S, N, seed, base, scale, dtype).t()
    tol = 1e-12 if dtype == torch.float64 else 2e-5
    torch.testing.assert_close(Y.double().cpu(), ref, rtol=0, atol=tol * float(ref.abs().max()))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_jlt_sparse_both_directions_match_dense_input(dtype):
    N, m, S = 5000, 300, 64
    A, Ad = _csr(N, m, 0.01, dtype, 5)
    ctx = sk.Context(11)
    T = sk.sketch.JLT(N, S, context=ctx)
    got = T.apply(Ad, dim="columnwise")
    want = T.apply(A.to(dtype).cuda(), dim="columnwise")
    torch.testing.assert_close(got.double(), want.double(), rtol=0,
                               atol=(1e-12 if dtype == torch.float64 else 3e-5) * float(want.abs().max()))
    T2 = sk.sketch.JLT(m, S, context=ctx)
    got = T2.apply(Ad, dim="rowwise")
    want = T2.apply(A.to(dtype).cuda(), dim="rowwise")
    torch.testing.assert_close(got.double(), want.double(), rtol=0,
                               atol=(1e-12 if dtype == torch.float64 else 3e-5) * float(want.abs().max()))


def test_csr_sketch_shard_offset():
    """A shard holding input columns [in_offset, in_offset + k) of an N-wide
    operand uses exactly those sketch columns."""
    m, N, k0, k, S = 500, 1000, 300, 250, 48
    A, Ad = _csr(m, k, 0.05, torch.float64, 9)
    Y = DS.csr_sketch_native(Ad, dist=D.Normal(), seed=3, base=10, S=S, N=N, scale=1.0, in_offset=k0,
                             panel_elems=S * 64)
    ref = A @ _explicit(S, N, 3, 10, 1.0)[:, k0:k0 + k].t()
    torch.testing.assert_close(Y.cpu(), ref, rtol=0, atol=1e-12 * float(ref.abs().max()))


@pytest.mark.parametrize("dtype,idx", [(torch.float32, torch.int32), (torch.float64, torch.int64)])
def test_csr_transpose_native_exact(dtype, idx):
    """csr_transpose.hip: A^T as CSR with ascending row indices per column,
    bit-identical to the dense transpose (empty rows and columns, a long row)."""
    A, _ = _csr(700, 450, 0.02, dtype, 12, empty_rows=(3, 699))
    A[:, 17] = 0
    A[5, :] = torch.randn(450, dtype=torch.float64).to(dtype).double()
    Ad = A.to(dtype).to_sparse_csr()
    Ad = torch.sparse_csr_tensor(Ad.crow_indices().to(idx), Ad.col_indices().to(idx), Ad.values(), Ad.shape).cuda()
    T = DS._csr_transpose(Ad)
    assert T.shape == (450, 700)
    ref = A.to(dtype).t().contiguous().to_sparse_csr()
    assert torch.equal(T.crow_indices().long().cpu(), ref.crow_indices().long())
    assert torch.equal(T.col_indices().long().cpu(), ref.col_indices().long())
    assert torch.equal(T.values().cpu(), ref.values())
