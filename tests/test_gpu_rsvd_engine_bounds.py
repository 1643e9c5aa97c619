"""bf16 randSVD on both sides of the engine boundaries:
the fused one-read engine covers n <= 1024 (n % 8 == 0) and k <= 48
(k = 2 r by default), the general engine everything else up to k = 128.
Each case checks the engine the call was routed to and the answer against
an fp64 SVD of the same bf16 operand (reference nla/svd.hpp:222-318; the
distributed-equals-local oracle of tests/unit/DenseSketchApplyElementalTest
is covered by tests/test_gpu_multirank.py)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _planted(m, n, r, seed):
    g = np.random.RandomState(seed)
    U0, _ = np.linalg.qr(g.randn(m, r))
    V0, _ = np.linalg.qr(g.randn(n, r))
    sig = 100.0 * 0.93 ** np.arange(r)
    return (U0 * sig) @ V0.T + 1e-3 * g.randn(m, n)


@pytest.mark.parametrize("n,rank,fused", [
    (1024, 24, True),     # k = 48: the fused engine's largest k
    (1024, 25, False),    # k = 50
    (1032, 24, False),    # n = 1032 > 1024
    (1024, 32, False),    # k = 64
    (1024, 33, False),    # k = 66
    (1032, 33, False),
])
def test_bf16_rsvd_engine_boundaries(n, rank, fused):
    import libskylark_amd as sk
    from libskylark_amd.nla import svd as S
    m = 12000
    A64 = _planted(m, n, rank + 8, seed=n + rank)
    A = torch.from_numpy(A64).to("cuda", torch.bfloat16)
    A64 = A.double().cpu().numpy()          # the operand the engines see
    prm = sk.nla.ApproximateSVDParams(num_iterations=2, sketch="FJLT", check=True)
    U, s, V = sk.nla.approximate_svd(A, rank, sk.Context(seed=7), prm)
    plan = [p for p in S._PLANS.values() if p.Aref() is A][0]
    assert (type(plan) is S._EnginePlan) == fused, type(plan).__name__   # (_GenPlan derives from it)
    sv = np.linalg.svd(A64, compute_uv=False)[:rank]
    s = s.double().cpu().numpy()
    np.testing.assert_allclose(s, sv, rtol=5e-3, atol=5e-3 * sv[0])
    Ud, Vd = U.double().cpu().numpy(), V.double().cpu().numpy()
    assert np.abs(Ud.T @ Ud - np.eye(rank)).max() < 2e-3
    assert np.abs(Vd.T @ Vd - np.eye(rank)).max() < 2e-3
    res = np.linalg.norm(A64 @ Vd - Ud * s) / np.linalg.norm(s)
    assert res < 5e-2, res
