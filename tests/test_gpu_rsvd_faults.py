"""Failure reporting of the device randSVD engine (rsvd_engine.cpp /
rsvd_core.hip k_boundary): a pass-boundary wait that times out must surface
as an error -- on the call itself with ``check=True``, else on the next call
of the plan -- never as silently returned garbage.  The timeout is forced
with the engine's test-only fault knob (``sl_rsvd_plan_set_fault``: the
boundary kernels expect one arrival more than their grid, so no workgroup is
ever last, and every spin is bounded at 1 ms)."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu


def _A(m=20000, n=256, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randn(m, n, device="cuda", generator=g).to(torch.bfloat16)


def _plan_for(A):
    from libskylark_amd.nla import svd as S
    for p in S._PLANS.values():
        if p.Aref() is A:
            return p
    raise AssertionError("no engine plan for this operand")


def _fault(plan, missing, bound_ticks):
    from libskylark_amd.nla.svd import _engine_lib
    _engine_lib().call("sl_rsvd_plan_set_fault", plan.h, missing, C.c_uint64(bound_ticks))


@pytest.mark.parametrize("q", [0, 2])
def test_timeout_raises_on_that_call_with_check(q):
    import libskylark_amd as sk
    A = _A()
    prm = sk.nla.ApproximateSVDParams(num_iterations=q, sketch="FJLT", check=True)
    U, s, V = sk.nla.approximate_svd(A, 10, sk.Context(seed=1), prm)   # clean call builds the plan
    assert torch.isfinite(s).all()
    plan = _plan_for(A)
    _fault(plan, 1, 100_000)    # 1 ms of the 100 MHz clock
    with pytest.raises(RuntimeError, match="timed out"):
        sk.nla.approximate_svd(A, 10, sk.Context(seed=1), prm)
    torch.cuda.synchronize()
    # the timed-out plan is dropped; the next call builds a fresh one and is clean
    from libskylark_amd.nla import svd as S
    assert all(p is not plan for p in S._PLANS.values())
    U2, s2, V2 = sk.nla.approximate_svd(A, 10, sk.Context(seed=1), prm)
    torch.testing.assert_close(s2, s, rtol=1e-5, atol=0)


def test_timeout_reported_by_next_call_without_check():
    import libskylark_amd as sk
    A = _A(seed=1)
    prm = sk.nla.ApproximateSVDParams(num_iterations=1, sketch="FJLT")
    sk.nla.approximate_svd(A, 8, sk.Context(seed=2), prm)
    plan = _plan_for(A)
    _fault(plan, 1, 100_000)
    sk.nla.approximate_svd(A, 8, sk.Context(seed=2), prm)   # returns (asynchronous), flagged on the device
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="timed out"):
        sk.nla.approximate_svd(A, 8, sk.Context(seed=2), prm)


def test_status_word_keeps_timeout_bit():
    """The host-side mask keeps bit 16 (the round-3 mask `& 15` dropped it)."""
    import libskylark_amd as sk
    from libskylark_amd.nla import svd as S
    A = _A(seed=2)
    prm = sk.nla.ApproximateSVDParams(num_iterations=0, sketch="FJLT")
    sk.nla.approximate_svd(A, 8, sk.Context(seed=3), prm)
    plan = _plan_for(A)
    torch.cuda.synchronize()
    plan.status_dev.fill_(S.ST_TIMEOUT)
    if plan.mirror is not None:
        plan.mirror.value = S.ST_TIMEOUT
    plan.status_ev = torch.cuda.Event()
    plan.status_ev.record()
    assert plan.wait_status() & S.ST_TIMEOUT
