"""GPU FJLT with many samples (fused D-scale/reorder -> rocFFT rfft -> sampled
post-twiddle gather) against the fp64 explicit operator sqrt(N/S) P F D."""
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.ops import fut


@pytest.mark.gpu
@pytest.mark.parametrize("N,m,S,dim,dt", [(4096, 64, 600, 0, torch.float32), (3001, 40, 700, 0, torch.float32),
                                          (2048, 33, 512, 1, torch.float32), (1999, 20, 300, 1, torch.bfloat16),
                                          (1000, 16, 999, 0, torch.bfloat16)])
def test_fjlt_sampled_gpu_vs_operator(dev, N, m, S, dim, dt):
    g = torch.Generator().manual_seed(N)
    A = torch.randn(N, m, generator=g, dtype=torch.float64) if dim == 0 else \
        torch.randn(m, N, generator=g, dtype=torch.float64)
    d = torch.where(torch.rand(N, generator=g) < 0.5, -1.0, 1.0).double()
    samples = torch.randint(0, N, (S,), generator=g)
    scale = (N / S) ** 0.5
    W = fut.dct2_rows_matrix(N, samples, dtype=torch.float64, d=d, scale=scale)   # S x N, fp64, host
    Ad = A.to(dt).double()
    ref = W @ Ad if dim == 0 else Ad @ W.t()
    got = fut.fjlt_sampled(A.to(dev, dt), dim, d, samples, scale).double().cpu()
    err = float((got - ref).norm() / ref.norm())
    assert err < 2e-6, err


@pytest.mark.gpu
def test_fjlt_sketch_large_s_gpu(dev):
    """The FJLT sketch class routes S > 256 through the sampled pipeline."""
    A = torch.randn(5000, 12, dtype=torch.float64)
    S = sk.sketch.FJLT(5000, 800, context=sk.Context(7))
    ref = S.realize(torch.float64) @ A
    got = S.apply(A.float().to(dev), dim=sk.sketch.COLUMNWISE).double().cpu()
    assert float((got - ref).norm() / ref.norm()) < 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize("q,S", [(3, 256), (2, 1000)])
def test_ppt_gpu_fused_product(dev, q, S):
    g = torch.Generator().manual_seed(S)
    A = torch.randn(300, 40, generator=g, dtype=torch.float64)
    P = sk.sketch.PPT(300, S, q=q, c=1.0, gamma=0.5, context=sk.Context(3))
    ref = P.apply(A, dim=sk.sketch.COLUMNWISE)                 # fp64 CPU (folded-spectrum torch path)
    got = P.apply(A.float().to(dev), dim=sk.sketch.COLUMNWISE).double().cpu()
    assert float((got - ref).norm() / ref.norm()) < 1e-4
    As = A.clone()
    As[As.abs() < 1.0] = 0
    got_s = P.apply(As.float().to(dev).to_sparse_csr(), dim=sk.sketch.COLUMNWISE).double().cpu()
    ref_s = P.apply(As, dim=sk.sketch.COLUMNWISE)
    assert float((got_s - ref_s).norm() / ref_s.norm()) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("N,m,dim", [(1024, 40, 0), (4096, 7, 0), (16384, 3, 0), (512, 100, 1), (8, 5, 1), (2048, 33, 1)])
def test_wht_native_vs_hadamard(dev, N, m, dim):
    g = torch.Generator().manual_seed(N + m)
    X = torch.randn(N, m, generator=g, dtype=torch.float64) if dim == 0 else \
        torch.randn(m, N, generator=g, dtype=torch.float64)
    if N <= 2048:
        from scipy.linalg import hadamard
        H = torch.from_numpy(hadamard(N).astype("float64")) / N ** 0.5
        ref = H @ X if dim == 0 else X @ H.t()
    else:
        ref = fut.wht(X, dim)          # host butterfly in f64
    got = fut.wht(X.float().to(dev), dim).double().cpu()
    assert float((got - ref).norm() / ref.norm()) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("N,S,dim", [(8192, 10000, 0), (5000, 6000, 1), (6000, 3000, 0)])
def test_fastfood_large_n_native_pipeline(dev, N, S, dim):
    """Fastfood beyond the dense-W limit runs two native FJLT pipelines per
    block; compare with the host f64 DCT chain of the same sketch."""
    T = sk.sketch.FastGaussianRFT(N, S, sigma=40.0, context=sk.Context(9))
    assert N > T.DENSE_MAX_N
    g = torch.Generator().manual_seed(N)
    A = torch.randn(N, 24, generator=g, dtype=torch.float64) if dim == 0 else \
        torch.randn(24, N, generator=g, dtype=torch.float64)
    ref = T.apply(A, dim=dim)
    got = T.apply(A.float().to(dev), dim=dim).double().cpu()
    err = float((got - ref).norm() / ref.norm())
    assert err < 2e-4, err


@pytest.mark.gpu
@pytest.mark.parametrize("fut_name", ["DCT", "DHT"])
@pytest.mark.parametrize("N,m,dim", [(1000, 24, 0), (777, 10, 1), (4096, 8, 0)])
def test_rfut_gpu_vs_f64(dev, fut_name, N, m, dim):
    """RFUT F D A on the GPU (DCT: native pre-pass + rocFFT R2C + full post
    pass; DHT: half-spectrum R2C) against the fp64 host transform."""
    from libskylark_amd.sketch.fjlt import RFUT
    g = torch.Generator().manual_seed(N + m)
    A = torch.randn(N, m, generator=g, dtype=torch.float64) if dim == 0 else \
        torch.randn(m, N, generator=g, dtype=torch.float64)
    R = RFUT(N, sk.Context(3), fut_name)
    ref = R.apply(A, dim)
    got = R.apply(A.float().to(dev), dim).double().cpu()
    err = float((got - ref).norm() / ref.norm())
    assert err < 2e-6, err
