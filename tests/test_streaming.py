"""Out-of-core (host-streamed) sketch application vs the in-memory apply."""
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.sketch import COLUMNWISE, ROWWISE


def _cases():
    return [
        ("JLT", lambda N, S: sk.sketch.JLT(N, S, context=sk.Context(1))),
        ("CWT", lambda N, S: sk.sketch.CWT(N, S, context=sk.Context(2))),
        ("FJLT", lambda N, S: sk.sketch.FJLT(N, S, context=sk.Context(3))),
        ("GaussianRFT", lambda N, S: sk.sketch.GaussianRFT(N, S, sigma=3.0, context=sk.Context(4))),
    ]


def _check(device, dtype, pin):
    N, S, M = 512, 64, 301
    for name, mk in _cases():
        T = mk(N, S)
        for dim in (COLUMNWISE, ROWWISE):
            A = torch.randn(N, M, dtype=dtype) if dim == COLUMNWISE else torch.randn(M, N, dtype=dtype)
            if pin:
                A = A.pin_memory()
            ref = T.apply(A.to(device), dim=dim).double().cpu()
            # ~7 panels of rows (or columns) per call
            pb = max(1, A.numel() * A.element_size() // 7)
            out = T.apply_streamed(A, dim, device=device, panel_bytes=pb).double().cpu()
            tol = 1e-10 if dtype == torch.float64 else 2e-4
            torch.testing.assert_close(out, ref, rtol=tol, atol=tol * float(ref.abs().max()), msg=f"{name} dim={dim}")


def test_streamed_apply_cpu():
    _check(torch.device("cpu"), torch.float64, pin=False)


@pytest.mark.gpu
@pytest.mark.parametrize("pin", [False, True])
def test_streamed_apply_gpu(dev, pin):
    _check(dev, torch.float32, pin)
