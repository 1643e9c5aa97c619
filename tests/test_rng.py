"""RNG core: Threefry known answers, determinism, sampler moments, host == device."""
import math

import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.base import distributions as D
from libskylark_amd.ops import rng

# Random123 known-answer vectors for threefry2x64_13 (also cross-checked
# against rocrand's threefry engine instantiated with 13 rounds).
KAT = [
    ((0, 0, 0, 0), (0xF167B032C3B480BD, 0xE91F9FEE4B7A6FB5)),
    ((2**64 - 1,) * 4, (0xCCDEC5C917A874B1, 0x4DF53ABCA26CEB01)),
    ((0x243F6A8885A308D3, 0x13198A2E03707344, 0xA4093822299F31D0, 0x082EFA98EC4E6C89),
     (0xC3AAC71561042993, 0x3FE7AE8801AFF316)),
]


@pytest.mark.parametrize("inp,out", KAT)
def test_threefry_kat(inp, out):
    assert rng.threefry(*inp) == out


def test_context_counter_accounting():
    ctx = sk.Context(seed=5)
    a = ctx.allocate_random_samples_array(100, D.Normal())
    b = ctx.allocate_random_samples_array(7, D.Normal())
    assert (a.base, b.base, ctx.counter) == (0, 100, 107)
    d = ctx.to_dict()
    assert d["skylark_object_type"] == "context" and d["seed"] == 5 and d["counter"] == 107
    assert sk.Context.from_json(ctx.to_json()) == ctx


def test_random_access_consistency():
    arr = sk.Context(3).allocate_random_samples_array(1000, D.Normal())
    full = arr.realize()
    part = arr.realize(400, 100)
    assert torch.equal(full[400:500], part)
    assert arr[417] == pytest.approx(float(full[417]))


@pytest.mark.parametrize("dist,mean,var", [
    (D.Normal(), 0.0, 1.0),
    (D.Uniform(2.0, 4.0), 3.0, 4.0 / 12),
    (D.Exponential(), 1.0, 1.0),
    (D.Rademacher(), 0.0, 1.0),
    (D.ChiSquared(3.0), 3.0, 6.0),
])
def test_sampler_moments(dist, mean, var):
    x = sk.Context(11).generate_random_samples_array(200000, dist)
    assert float(x.mean()) == pytest.approx(mean, abs=5 * math.sqrt(var / 200000) + 1e-3)
    assert float(x.var()) == pytest.approx(var, rel=0.05)


def test_uniform_int_range():
    x = sk.Context(2).generate_random_samples_array(50000, D.UniformInt(3, 9), dtype=torch.int64)
    assert int(x.min()) == 3 and int(x.max()) == 9
    counts = torch.bincount(x - 3)
    assert counts.min() > 50000 / 7 * 0.9


def test_cauchy_median():
    x = sk.Context(4).generate_random_samples_array(100001, D.Cauchy())
    assert abs(float(x.median())) < 0.02
    q = torch.quantile(x[:50000].float(), torch.tensor([0.25, 0.75]))
    assert q[0].item() == pytest.approx(-1.0, abs=0.05) and q[1].item() == pytest.approx(1.0, abs=0.05)


def test_fill_global_indexing_is_layout_independent():
    """A shard realised with global offsets equals the slice of the whole matrix."""
    full = rng.random_matrix(50, 30, D.Normal(), seed=9, base=123, dtype=torch.float64)
    shard = torch.empty(10, 30, dtype=torch.float64)
    rng.fill_random(shard, D.Normal(), 9, 123, r0=20, c0=0, ir=1, ic=50)
    assert torch.equal(shard, full[20:30])
    tshard = torch.empty(30, 10, dtype=torch.float64).t()  # column-major view
    rng.fill_random(tshard, D.Normal(), 9, 123, r0=20, c0=0, ir=1, ic=50)
    assert torch.equal(tshard, full[20:30])


@pytest.mark.gpu
def test_threefry_host_equals_device(dev):
    blocks = rng.threefry_stream(77, 1000, 512, dev).cpu().view(-1, 2)
    for i in (0, 1, 255, 511):
        a, b = rng.threefry(1000 + i, 0, 77, 0)
        assert (int(blocks[i, 0]) & (2**64 - 1), int(blocks[i, 1]) & (2**64 - 1)) == (a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("dist", [D.Normal(), D.Cauchy(), D.Uniform(-1, 2), D.Rademacher(),
                                  D.Exponential(), D.Levy(), D.ChiSquared(4.0), D.WZTValue(1.5)])
def test_fill_device_matches_host_f64(dev, dist):
    h = rng.random_matrix(64, 33, dist, seed=5, base=17, dtype=torch.float64)
    d = rng.random_matrix(64, 33, dist, seed=5, base=17, dtype=torch.float64, device=dev).cpu()
    torch.testing.assert_close(d, h, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_fill_device_f32_fast_sampler(dev):
    h = rng.random_matrix(256, 64, D.Normal(), seed=5, base=0, dtype=torch.float64)
    d = rng.random_matrix(256, 64, D.Normal(), seed=5, base=0, dtype=torch.float32, device=dev).cpu().double()
    torch.testing.assert_close(d, h, rtol=1e-4, atol=1e-4)
