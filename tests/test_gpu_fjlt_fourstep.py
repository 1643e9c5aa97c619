"""Four-step sampled DCT (fjlt_fourstep.hip) against an fp64 host DCT-II
(scipy, orthonormal) of D A at the sampled rows: radix plans 8/4/5/3/7/2,
partial column chunks, bf16 input, repeated samples, k = 0, k = M and
k > M (the packed real-to-complex partner frequencies), and the FJLT sketch
class end to end (S > the direct-GEMM limit)."""
import numpy as np
import pytest
import torch
from scipy.fft import dct

import libskylark_amd as sk
from libskylark_amd.ops import fut

pytestmark = pytest.mark.gpu


def _ref(A64, d, samples, scale):
    return scale * dct(A64 * d[:, None], type=2, norm="ortho", axis=0)[samples]


@pytest.mark.parametrize("N,m", [(8192, 37), (13440, 64), (100000, 100), (7392, 5)])
def test_fourstep_matches_fp64_dct(N, m):
    split = fut.fourstep_split(N)
    assert split is not None
    g = np.random.default_rng(N)
    A = g.standard_normal((N, m))
    d = g.choice([-1.0, 1.0], N)
    M = N // 2
    samples = np.concatenate([[0, M, M - 1, M + 1, N - 1, 5, 5], g.integers(0, N, 300)])
    Ad = torch.from_numpy(A).float().cuda()
    out = fut.fjlt_fourstep(Ad, torch.from_numpy(d), torch.from_numpy(samples), 1.7)
    ref = _ref(A.astype(np.float32).astype(np.float64), d, samples, 1.7)
    got = out.double().cpu().numpy()
    assert np.abs(got - ref).max() <= 2e-5 * np.abs(ref).max(), (np.abs(got - ref).max(), np.abs(ref).max())


def test_fourstep_bf16_input():
    N, m = 20000, 48
    g = np.random.default_rng(1)
    A = torch.from_numpy(g.standard_normal((N, m))).to(torch.bfloat16)
    d = g.choice([-1.0, 1.0], N)
    samples = g.integers(0, N, 500)
    out = fut.fjlt_fourstep(A.cuda(), torch.from_numpy(d), torch.from_numpy(samples), 1.0)
    ref = _ref(A.double().numpy(), d, samples, 1.0)
    assert np.abs(out.double().cpu().numpy() - ref).max() <= 2e-5 * np.abs(ref).max()


def test_fjlt_sketch_uses_fourstep_and_matches_operator():
    N, m, S = 65536, 40, 1000
    A = torch.randn(N, m, dtype=torch.float64)
    T = sk.sketch.FJLT(N, S, context=sk.Context(21))
    assert fut.fourstep_ok(A.float().cuda(), 0, S)
    got = T.apply(A.float().cuda(), dim="columnwise").double().cpu()
    ref = T.realize(torch.float64, "cpu") @ A
    torch.testing.assert_close(got, ref, rtol=0, atol=3e-5 * float(ref.abs().max()))


def test_fourstep_dense_groups_and_wide_batch():
    """Many sampled frequencies per k2 group (several stage-2 passes of 24) and a
    batch wider than one stage-2 workgroup (300 columns: 256 + a partial 44)."""
    N, m = 8192, 300
    g = np.random.default_rng(7)
    A = g.standard_normal((N, m))
    d = g.choice([-1.0, 1.0], N)
    samples = g.integers(0, N, 3000)
    out = fut.fjlt_fourstep(torch.from_numpy(A).float().cuda(), torch.from_numpy(d), torch.from_numpy(samples), 1.0)
    ref = _ref(A.astype(np.float32).astype(np.float64), d, samples, 1.0)
    assert np.abs(out.double().cpu().numpy() - ref).max() <= 2e-5 * np.abs(ref).max()



@pytest.mark.parametrize("dtype,N,m", [(torch.bfloat16, 100000, 100), (torch.float32, 13440, 1000),
                                       (torch.float32, 8192, 36)])
def test_fourstep_shapes_and_dtypes(dtype, N, m):
    """Partial last column chunk (m = 100, 36), bf16 input on the long
    length, a wide batch (1000 columns: 63 chunks per row of Y)."""
    g = np.random.default_rng(N + m)
    A = torch.from_numpy(g.standard_normal((N, m))).to(dtype)
    d = g.choice([-1.0, 1.0], N)
    samples = g.integers(0, N, 400)
    out = fut.fjlt_fourstep(A.cuda(), torch.from_numpy(d), torch.from_numpy(samples), 1.0).double().cpu()
    ref = _ref(A.double().numpy(), d, samples, 1.0)
    assert np.abs(out.numpy() - ref).max() <= 2e-5 * np.abs(ref).max()


@pytest.mark.parametrize("N,m,S", [(100000, 100, 400), (13440, 70, 3000), (8192, 300, 3000), (65536, 16, 50)])
def test_fourstep_stage2_mfma_matches_valu_and_dct(N, m, S):
    """Stage 2 on the matrix cores (k_fs_stage2m) against the VALU kernel and
    the fp64 DCT: N1 not a multiple of 4 (13440: N1 = 14, masked tail rows),
    groups of more than 32 frequencies (several passes), partial 64-column
    waves, a sparse sample set (groups of 0-2 frequencies)."""
    g = np.random.default_rng(N + m)
    A = torch.from_numpy(g.standard_normal((N, m))).float()
    d = g.choice([-1.0, 1.0], N)
    samples = g.integers(0, N, S)
    outs = []
    try:
        for v in (1, 0):
            fut.set_fourstep_stage2(v)
            outs.append(fut.fjlt_fourstep(A.cuda(), torch.from_numpy(d), torch.from_numpy(samples), 1.0).double().cpu())
    finally:
        fut.set_fourstep_stage2(1)
    ref = _ref(A.double().numpy(), d, samples, 1.0)
    scale = np.abs(ref).max()
    for o in outs:
        assert np.abs(o.numpy() - ref).max() <= 2e-5 * scale
    assert (outs[0] - outs[1]).abs().max().item() <= 2e-6 * scale
