"""Hand-written bf16 NT GEMM (gemm_nt.hip) against fp32 torch products of
the same bf16 operands: edge tiles (M, N not multiples of 256), several K
slices, accumulate, bf16 output, the cosine feature epilogue, strided views."""
import pytest
import torch

from libskylark_amd.ops import gemm

pytestmark = pytest.mark.gpu


def _ops(M, N, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    B = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    return A, B, A.float() @ B.float().t()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (1000, 700, 320), (513, 1300, 1024), (37, 5, 128),
                                   (2100, 600, 2048), (300, 260, 64 * 3)])
def test_gemm_nt_f32_matches(M, N, K):
    A, B, ref = _ops(M, N, K, M + N)
    C = gemm.gemm_nt(A, B, alpha=0.5)
    torch.testing.assert_close(C, 0.5 * ref, rtol=0, atol=1e-4 * float(ref.abs().max()))


def test_gemm_nt_accumulate_and_views():
    M, N, K = 700, 520, 192
    A, B, ref = _ops(M, N, K, 3)
    big = torch.zeros(M, N + 40, device="cuda")
    base = torch.randn(M, N, device="cuda")
    big[:, 7:7 + N] = base
    Bv = torch.zeros(N, K + 64, device="cuda", dtype=torch.bfloat16)
    Bv[:, :K] = B
    gemm.gemm_nt(A, Bv[:, :K], out=big[:, 7:7 + N], accumulate=True)
    torch.testing.assert_close(big[:, 7:7 + N], base + ref, rtol=0, atol=1e-4 * float(ref.abs().max()))
    assert float(big[:, :7].abs().max()) == 0.0 and float(big[:, 7 + N:].abs().max()) == 0.0


def test_gemm_nt_bf16_out_and_cos_epilogue():
    M, N, K = 900, 640, 256
    A, B, ref = _ops(M, N, K, 4)
    Cb = gemm.gemm_nt(A, B, out_dtype=torch.bfloat16)
    torch.testing.assert_close(Cb.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    sc = torch.rand(N, device="cuda") * 0.2
    sh = torch.rand(N, device="cuda") * 6.28
    Z = gemm.gemm_nt(A, B, alpha=0.3, cos_scales=sc, cos_shifts=sh)
    torch.testing.assert_close(Z, 0.3 * torch.cos(ref * sc + sh), rtol=0, atol=2e-4)


@pytest.mark.parametrize("cos", [False, True])
def test_gemm_nt_bf16_out_is_rne_of_f32_out(cos):
    """bf16 output = round-to-nearest-even of the f32 output, bit for bit (the
    epilogue converts with the hardware v_cvt_pk_bf16_f32)."""
    M, N, K = 1000, 777, 192
    A, B, _ = _ops(M, N, K, 11)
    kw = {}
    if cos:
        kw = dict(alpha=0.3, cos_scales=torch.rand(N, device="cuda") * 0.2,
                  cos_shifts=torch.rand(N, device="cuda") * 6.28)
    C32 = gemm.gemm_nt(A, B, **kw)
    C16 = gemm.gemm_nt(A, B, out_dtype=torch.bfloat16, **kw)
    assert torch.equal(C16, C32.bfloat16())


@pytest.fixture
def nt_store_on():
    gemm.set_nt_store(1)
    try:
        yield
    finally:
        gemm.set_nt_store(-1)


@pytest.mark.parametrize("M,N,K", [(1000, 700, 320), (513, 1300, 1024), (2100, 600, 2048)])
def test_gemm_nt_forced_nt_store_matches(nt_store_on, M, N, K):
    """Non-temporal C stores forced on (the default only turns them on for C
    >= 64 MiB at K <= 2048): f32 out, bf16 out, the cos map and the
    accumulate path against fp32 torch, edge tiles included."""
    A, B, ref = _ops(M, N, K, 7 * M + N)
    tol = 1e-4 * float(ref.abs().max())
    torch.testing.assert_close(gemm.gemm_nt(A, B, alpha=0.5), 0.5 * ref, rtol=0, atol=tol)
    Cb = gemm.gemm_nt(A, B, out_dtype=torch.bfloat16)
    torch.testing.assert_close(Cb.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    sc = torch.rand(N, device="cuda") * 0.2
    sh = torch.rand(N, device="cuda") * 6.28
    Z = gemm.gemm_nt(A, B, alpha=0.3, cos_scales=sc, cos_shifts=sh)
    torch.testing.assert_close(Z, 0.3 * torch.cos(ref * sc + sh), rtol=0, atol=2e-4)
    base = torch.randn(M, N, device="cuda")
    out = base.clone()
    gemm.gemm_nt(A, B, out=out, accumulate=True)
    torch.testing.assert_close(out, base + ref, rtol=0, atol=tol)
    # bit-identical to the default store policy (only the cache policy differs)
    gemm.set_nt_store(0)
    assert torch.equal(gemm.gemm_nt(A, B, alpha=0.3, cos_scales=sc, cos_shifts=sh), Z)


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_gemm_nt_auto_nt_store_large_output(out_dtype):
    """A cos-map output over the auto rule's 64 MiB threshold (f32: 16640 x
    1040 x 4 B = 69 MB, bf16 at 2 x the rows) at K = 512: the production
    feature-map path with non-temporal stores, against fp32 torch."""
    M = 16640 if out_dtype == torch.float32 else 33280
    N, K = 1040, 512
    A, B, ref = _ops(M, N, K, 99)
    assert M * N * (4 if out_dtype == torch.float32 else 2) >= 64 << 20
    sc = torch.rand(N, device="cuda") * 0.2
    sh = torch.rand(N, device="cuda") * 6.28
    Z = gemm.gemm_nt(A, B, alpha=0.3, cos_scales=sc, cos_shifts=sh, out_dtype=out_dtype)
    want = 0.3 * torch.cos(ref * sc + sh)
    atol = 2e-4 if out_dtype == torch.float32 else 2e-3
    torch.testing.assert_close(Z.float(), want, rtol=0, atol=atol)
