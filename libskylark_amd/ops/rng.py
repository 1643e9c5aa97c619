"""Random realisation ops (native Threefry kernels; host or gfx950 device)."""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib


def fill_random(out: torch.Tensor, dist, seed: int, base: int, r0: int = 0, c0: int = 0,
                ir: int = 1, ic: int | None = None, scale: float = 1.0, precise: bool = False):
    """Fill a 2-D (possibly strided) tensor view with stream samples.

    ``out[r, c] = scale * dist(seed, base + (r0 + r) * ir + (c0 + c) * ic)``.
    The default ``ir=1, ic=<global rows>`` is the reference's column-major
    realisation ``entries[j*S + i]`` (``sketch/dense_transform_data.hpp:79-101``)
    when ``ic`` is the height of the *global* matrix.
    """
    if out.dim() == 1:
        out = out.view(-1, 1)
    if out.dim() != 2:
        raise ValueError("fill_random expects a 1-D or 2-D tensor")
    rows, cols = out.shape
    if ic is None:
        ic = rows
    sr, sc = out.stride()
    p0, p1 = dist.params()
    args = [_lib.ptr(out), _lib.dtype_code(out.dtype), int(dist.code), C.c_uint64(seed & (2**64 - 1)),
            C.c_uint64(base), rows, cols, sr, sc, r0, c0, ir, ic, p0, p1, float(scale), int(bool(precise))]
    if out.is_cuda:
        _lib.call("sl_fill_random", *args, C.c_void_p(_lib.stream_of(out)))
    else:
        _lib.call("sl_fill_random_host", *args)
    return out


def random_matrix(rows: int, cols: int, dist, seed: int, base: int, *, scale: float = 1.0,
                  dtype=torch.float32, device=None, layout: str = "colmajor", precise: bool = False):
    """Realise a whole ``rows x cols`` random matrix (column-major stream order)."""
    out = torch.empty(rows, cols, dtype=dtype, device=device)
    if layout == "colmajor":
        fill_random(out, dist, seed, base, ir=1, ic=rows, scale=scale, precise=precise)
    else:
        fill_random(out, dist, seed, base, ir=cols, ic=1, scale=scale, precise=precise)
    return out


def random_int(seed: int, base: int, n: int, lo: int, hi: int, device=None) -> torch.Tensor:
    out = torch.empty(n, dtype=torch.int64, device=device)
    if n == 0:
        return out
    if out.is_cuda:
        _lib.call("sl_random_int", _lib.ptr(out), C.c_uint64(seed), C.c_uint64(base), n, lo, hi,
                  C.c_void_p(_lib.stream_of(out)))
    else:
        _lib.call("sl_random_int_host", _lib.ptr(out), C.c_uint64(seed), C.c_uint64(base), n, lo, hi)
    return out


def threefry(c0: int, c1: int, k0: int, k1: int):
    out = (C.c_uint64 * 2)()
    _lib.call("sl_threefry_host", C.cast(out, C.c_void_p), C.c_uint64(c0), C.c_uint64(c1),
              C.c_uint64(k0), C.c_uint64(k1))
    return int(out[0]), int(out[1])


def threefry_stream(seed: int, base: int, n: int, device) -> torch.Tensor:
    """Raw Threefry blocks for slots base..base+n-1 on a device (uint64 viewed as int64)."""
    out = torch.empty(2 * n, dtype=torch.int64, device=device)
    _lib.call("sl_threefry", _lib.ptr(out), C.c_uint64(seed), C.c_uint64(base), n,
              C.c_void_p(_lib.stream_of(out)))
    return out
