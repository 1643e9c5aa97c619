"""libskylark_amd — MI355X-native randomized numerical linear algebra.

A from-scratch, GPU-first framework with the capabilities of libSkylark
(sketching transforms, sketched NLA, kernel ML), built on PyTorch-ROCm
tensors, hand-written HIP/CDNA4 kernels (``_native/``) and RCCL collectives.

Quick start::

    import torch, libskylark_amd as sk
    sk.initialize(seed=38734)
    S = sk.sketch.JLT(1000, 100)
    SA = S * torch.randn(1000, 50, device="cuda")     # columnwise
    U, s, V = sk.nla.approximate_svd(A, rank=20)
"""
__version__ = "0.1.0"

from .base.context import Context  # noqa: E402

_default_context = Context(seed=38734)


def initialize(seed: int = 38734, counter: int = 0) -> Context:
    """(Re)initialise the library-wide default context (python-skylark ``lib.initialize``)."""
    global _default_context
    _default_context = Context(seed, counter)
    return _default_context


def finalize():
    pass


def default_context() -> Context:
    return _default_context


def set_default_context(ctx: Context):
    global _default_context
    _default_context = ctx


import warnings as _w  # noqa: E402

_w.filterwarnings("ignore", message="Sparse CSR tensor support is in beta state")
_w.filterwarnings("ignore", message="Sparse CSC tensor support is in beta state")

from . import algorithms, base, io, metrics, ml, nla, parallel, sketch  # noqa: E402,F401
