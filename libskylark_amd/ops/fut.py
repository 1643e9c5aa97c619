"""Fast unitary transforms: DCT-II/III, DHT, WHT along a matrix dimension.

Reference: ``utility/fft/fftw_futs.h:3-126`` (FFTW ``REDFT10``/``REDFT01``
with scale ``1/sqrt(2N)``; ``DHT`` with ``1/sqrt(N)``), SpiralWHT ``WHT_t``.

We implement the *orthonormal* DCT-II (``norm='ortho'``, the semantics of the
reference's pure-Python fallback ``scipy.fftpack.dct(..., norm='ortho')``,
``python-skylark/skylark/sketch.py:FJLT._ppyapply``); the C++ reference's
REDFT10 scaling leaves its k = 0 row sqrt(2) too large, i.e. not unitary.

The transforms run through rocFFT (``torch.fft``, hipFFT) with the
Makhoul even/odd reordering and the post-twiddle; on GPU the twiddle +
scaling is done in the same pass that extracts the real part.
"""
from __future__ import annotations

import math

import weakref

import torch
from ..utils.devcache import version_of


def _move(x, dim):
    return x if dim == 0 else x.transpose(0, 1)


def _cplx(dt):
    return torch.complex128 if dt == torch.float64 else torch.complex64


def _work_dtype(dt):
    return torch.float64 if dt == torch.float64 else torch.float32


def dct2(x: torch.Tensor, dim: int = 0) -> torch.Tensor:
    """Orthonormal DCT-II along ``dim`` of a 2-D tensor (returns a new tensor)."""
    xt = _move(x, dim).to(_work_dtype(x.dtype))
    N = xt.shape[0]
    v = torch.cat([xt[0::2], xt[1::2].flip(0)], dim=0)
    V = torch.fft.fft(v, dim=0)
    k = torch.arange(N, device=x.device, dtype=xt.dtype)
    w = torch.exp(torch.complex(torch.zeros_like(k), -math.pi * k / (2 * N)))
    X = (V * w[:, None]).real
    scale = torch.full((N,), math.sqrt(2.0 / N), dtype=xt.dtype, device=x.device)
    scale[0] = math.sqrt(1.0 / N)
    X = X * scale[:, None]
    return _move(X, dim).contiguous()


def dct3(X: torch.Tensor, dim: int = 0) -> torch.Tensor:
    """Orthonormal DCT-III along ``dim`` (inverse of :func:`dct2`)."""
    Xt = _move(X, dim).to(_work_dtype(X.dtype))
    N = Xt.shape[0]
    scale = torch.full((N,), math.sqrt(2.0 / N), dtype=Xt.dtype, device=X.device)
    scale[0] = math.sqrt(1.0 / N)
    Y = Xt / scale[:, None]  # undo ortho scaling -> un-normalised DCT-II coefficients Z_k
    k = torch.arange(N, device=X.device, dtype=Xt.dtype)
    # Makhoul inverse: V_k = (Z_k - i Z_{N-k}) e^{i pi k / 2N}, Z_N = 0; v = IDFT(V)
    Yr = torch.zeros_like(Y)
    Yr[1:] = Y.flip(0)[:-1]
    w = torch.exp(torch.complex(torch.zeros_like(k), math.pi * k / (2 * N)))
    V = torch.complex(Y, -Yr) * w[:, None]
    v = torch.fft.ifft(V, dim=0).real
    x = torch.empty_like(v)
    h = (N + 1) // 2
    x[0::2] = v[:h]
    x[1::2] = v[h:].flip(0)
    return _move(x, dim).contiguous()


def dht(x: torch.Tensor, dim: int = 0) -> torch.Tensor:
    """Unitary discrete Hartley transform (self-inverse), scale 1/sqrt(N)."""
    xt = _move(x, dim).to(_work_dtype(x.dtype))
    N = xt.shape[0]
    if x.is_cuda and N >= 2:
        # real input: half-spectrum R2C (F_{N-k} = conj F_k), H_k = Re F_k - Im F_k
        # for k <= N/2 and Re F_{N-k} + Im F_{N-k} above
        F = torch.fft.rfft(xt, dim=0)
        lo = F.real - F.imag
        h = N - F.shape[0]                      # rows N/2+1 .. N-1 (count N - (N//2+1))
        hi = (F.real[1:1 + h] + F.imag[1:1 + h]).flip(0)
        H = torch.cat([lo, hi], 0) / math.sqrt(N)
        return _move(H, dim).contiguous()
    F = torch.fft.fft(xt, dim=0)
    H = (F.real - F.imag) / math.sqrt(N)
    return _move(H, dim).contiguous()


def wht(x: torch.Tensor, dim: int = 0) -> torch.Tensor:
    """Orthonormal Walsh-Hadamard transform (N must be a power of two).  On the
    GPU (f32 / bf16, N <= 16384) one LDS kernel per call (``sl_wht``: tile
    load, log2 N in-LDS butterfly stages, scaled store); else the butterfly
    over torch ops."""
    N = x.shape[dim]
    if (x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.dim() == 2 and N >= 1
            and not (N & (N - 1)) and N <= 16384):
        import ctypes as C
        from . import _lib
        _lib.require()
        xc = x if x.stride(1) == 1 else x.contiguous()
        y = torch.empty_like(xc, dtype=torch.float32)
        es, vs = (xc.stride(0), 1) if dim == 0 else (1, xc.stride(0))
        yes, yvs = (y.stride(0), 1) if dim == 0 else (1, y.stride(0))
        nvec = x.shape[1 - dim]
        if (es, vs) != (yes, yvs) or xc.dtype != torch.float32:
            xf = xc.to(torch.float32).contiguous()
            y = xf
            es, vs = (xf.stride(0), 1) if dim == 0 else (1, xf.stride(0))
            xc = xf
        _lib.call("sl_wht", _lib.ptr(xc), _lib.ptr(y), _lib.dtype_code(torch.float32), nvec, N, es, vs,
                  C.c_void_p(_lib.stream_of(x)))
        return y
    xt = _move(x, dim).to(_work_dtype(x.dtype)).contiguous()
    N = xt.shape[0]
    if N & (N - 1):
        raise ValueError("WHT length must be a power of two")
    m = xt.shape[1]
    y = xt.clone()
    h = 1
    while h < N:
        y = y.view(N // (2 * h), 2, h, m)
        a, b = y[:, 0], y[:, 1]
        y = torch.stack([a + b, a - b], dim=1).reshape(N, m)
        h *= 2
    y = y / math.sqrt(N)
    return _move(y, dim).contiguous()


FUTS = {"DCT": (dct2, dct3), "DHT": (dht, dht), "WHT": (wht, wht)}


def dct2_rows_matrix(N: int, rows: torch.Tensor, dtype=torch.float64, device=None, d: torch.Tensor | None = None,
                     scale: float = 1.0, transpose: bool = False) -> torch.Tensor:
    """Explicit rows ``rows`` of the orthonormal DCT-II matrix (len(rows) x N),
    optionally times ``scale * diag(d)`` on the right; ``transpose`` returns the
    N x len(rows) layout.  On the GPU one native launch (``sl_dct2_rows``)."""
    dev = torch.device(device) if device is not None else rows.device
    S = rows.numel()
    if dev.type == "cuda" and dtype in (torch.float32, torch.float64, torch.bfloat16):
        from . import _lib
        _lib.require()
        r = rows.to(device=dev, dtype=torch.int64).contiguous()
        dd = d.to(device=dev, dtype=torch.float64).contiguous() if d is not None else None
        out = torch.empty((N, S) if transpose else (S, N), dtype=dtype, device=dev)
        _lib.call("sl_dct2_rows", _lib.ptr(r), S, N, _lib.ptr(dd) if dd is not None else None, float(scale),
                  _lib.ptr(out), _lib.dtype_code(dtype), out.stride(0), int(transpose), _lib.stream_of(out))
        return out
    k = rows.to(device=dev, dtype=torch.float64)[:, None]
    n = torch.arange(N, device=dev, dtype=torch.float64)[None, :]
    ang = torch.remainder(k * (2 * n + 1), 4 * N) * (math.pi / (2 * N))
    c0 = torch.tensor(math.sqrt(1.0 / N), dtype=torch.float64, device=dev)
    c1 = torch.tensor(math.sqrt(2.0 / N), dtype=torch.float64, device=dev)
    F = torch.cos(ang) * torch.where(k == 0, c0, c1)
    if d is not None:
        F = F * d.to(device=dev, dtype=torch.float64)[None, :]
    F = F * scale
    F = F.t() if transpose else F
    return F.to(dtype).contiguous()


def _register_fjlt():
    import ctypes as C
    from . import _lib
    _lib.register("sl_fjlt_operator", [C.c_void_p, C.c_int64, C.c_int64, C.c_double, C.c_void_p, C.c_int,
                                       C.c_int64, C.c_int, C.c_void_p])
    vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int
    _lib.register("sl_fjlt_pre", [vp, i32, i64, i64, i64, i32, vp, vp, i64, vp])
    _lib.register("sl_fjlt_post", [vp, i64, i64, i64, i32, vp, i64, C.c_double, vp, i64, vp])
    _lib.register("sl_ppt_product", [vp, i32, i64, i64, i64, vp, vp, C.c_double, C.c_double, vp, vp])
    _lib.register("sl_wht", [vp, vp, i32, i64, i32, i64, i64, vp])


_register_fjlt()


def fjlt_operator(prm: torch.Tensor, S: int, N: int, scale: float, out: torch.Tensor,
                  transpose: bool = True) -> torch.Tensor:
    """FJLT operator ``scale * P F D`` realised from stream coordinates held on
    the device (``prm`` = int64 {seed, base_D, base_samples}); graph-capturable
    (``sl_fjlt_operator``).  ``out``: N x S (transpose) or S x N, row-major."""
    import ctypes as C
    from . import _lib
    _lib.require()
    exp = (N, S) if transpose else (S, N)
    if tuple(out.shape) != exp or out.stride(1) != 1 or prm.dtype != torch.int64 or not prm.is_cuda:
        raise ValueError("fjlt_operator: bad operand layout")
    _lib.call("sl_fjlt_operator", _lib.ptr(prm), S, N, float(scale), _lib.ptr(out), _lib.dtype_code(out.dtype),
              out.stride(0), int(transpose), C.c_void_p(_lib.stream_of(out)))
    return out


# ------------------------------------------------------------ four-step path
_FS_REG = [False]


def _fs_lib():
    import ctypes as C
    from . import _lib
    if not _FS_REG[0]:
        _FS_REG[0] = True
        vp, i32, i64, u64 = C.c_void_p, C.c_int, C.c_int64, C.c_uint64
        _lib.register("sl_fs_stage1", [vp, i32, i64, i64, i32, vp, i32, i32, u64, i32, vp, vp])
        _lib.register("sl_fs_stage2", [vp, i32, i32, i32, vp, vp, vp, vp, vp, vp])
        _lib.register("sl_fs_post", [vp, i32, i64, vp, i32, vp, vp, C.c_double, vp, i64, vp])
        _lib.register("sl_fs_set_stage2_variant", [i32], None)
    return _lib


_STAGE2 = [1]


def set_fourstep_stage2(variant: int) -> None:
    """Stage-2 kernel of the four-step DCT: 1 (default) the MFMA kernel,
    0 the VALU kernel (A/B, tests)."""
    _STAGE2[0] = int(variant)
    _fs_lib().require().sl_fs_set_stage2_variant(int(variant))


FS_N2_MAX = 512
FS_N1_MAX = 8192


def _radix_plan(n2: int):
    """Radices (8, 4, 5, 3, 7, 2 greedily) multiplying to n2, or None."""
    rs = []
    for r in (8, 4, 5, 3, 7, 2):
        while n2 % r == 0:
            rs.append(r)
            n2 //= r
    return rs if n2 == 1 else None


def fourstep_split(N: int):
    """(N1, N2, radices) of the four-step sampled DCT for length N, or None:
    N even, M = N / 2 = N1 N2 with N2 <= 512 a 7-smooth divisor (largest
    such: fewest stage-2 terms) and N1 <= 8192."""
    if N % 2 or N < 4096:
        return None
    M = N // 2
    for n2 in range(min(FS_N2_MAX, M), 63, -1):
        if M % n2 == 0 and M // n2 <= FS_N1_MAX:
            rs = _radix_plan(n2)
            if rs is not None:
                return M // n2, n2, rs
    return None


class _FourStepPlan:
    """Host-side grouping of the needed spectrum points of one sample set:
    the frequencies k and M - k (mod M) of every sample, their slots, and
    the CSR of slots by k2 = f mod N2 for stage 2."""

    def __init__(self, N: int, samples: torch.Tensor, dev):
        self.N = N
        self.N1, self.N2, rs = fourstep_split(N)
        self.rplan = sum(r << (4 * i) for i, r in enumerate(rs))
        self.npass = len(rs)

        M = N // 2
        k = samples.detach().to("cpu", torch.int64)
        fa, fb = k % M, (M - k) % M
        F = torch.unique(torch.cat([fa, fb]))             # sorted
        k2, k1 = F % self.N2, F // self.N2
        order = torch.argsort(k2, stable=True)
        cnt = torch.bincount(k2, minlength=self.N2)
        gptr = torch.zeros(self.N2 + 1, dtype=torch.int64)
        gptr[1:] = torch.cumsum(cnt, 0)
        i32 = torch.int32
        self.nslots = F.numel()
        self.gptr = gptr.to(dev, i32)
        self.gk1 = k1[order].to(dev, i32)
        self.gslot = order.to(dev, i32)
        # the same groups largest first, for the MFMA stage-2 kernel (gord:
        # group -> k2): big groups start first and the grid's tail is short
        gord = torch.argsort(cnt, descending=True, stable=True)
        perm = torch.cat([torch.arange(int(gptr[g]), int(gptr[g + 1])) for g in gord.tolist()]) \
            if self.nslots else torch.zeros(0, dtype=torch.int64)
        gptr_s = torch.zeros(self.N2 + 1, dtype=torch.int64)
        gptr_s[1:] = torch.cumsum(cnt[gord], 0)
        self.gord = gord.to(dev, i32)
        self.gptr_s = gptr_s.to(dev, i32)
        self.gk1_s = k1[order][perm].to(dev, i32)
        self.gslot_s = order[perm].to(dev, i32)
        self.sa = torch.searchsorted(F, fa).to(dev, i32)
        self.sb = torch.searchsorted(F, fb).to(dev, i32)
        self.samples = k.to(dev)
        self.S = k.numel()


_FS_PLANS: dict = {}
def _device_copy(d: torch.Tensor, dev, dtype) -> torch.Tensor:
    from ..utils.devcache import device_copy
    return device_copy(d, dev, dtype)


def fourstep_ok(A: torch.Tensor, dim: int, S: int) -> bool:
    """The four-step path covers dim-0 transforms of row-major f32 / bf16
    GPU operands whose length splits (``fourstep_split``) and whose sample
    count keeps stage 2 (2 S N1 terms per column) below a few passes' work."""
    if dim != 0 or not A.is_cuda or A.dtype not in (torch.float32, torch.bfloat16) or A.stride(1) != 1:
        return False
    sp = fourstep_split(A.shape[0])
    return sp is not None and 2 * S * sp[0] <= 64 * (A.shape[0] // 2)


def fjlt_fourstep(A: torch.Tensor, d: torch.Tensor, samples: torch.Tensor, scale: float) -> torch.Tensor:
    """``scale * P F D A`` along dim 0 (F the orthonormal DCT-II) by the
    four-step kernels of ``fjlt_fourstep.hip``; returns S x m f32."""
    import ctypes as C
    L = _fs_lib()
    N, m = A.shape
    # cached per samples tensor OBJECT (weak reference + version counter): a
    # key on the data pointer alone hit stale plans once a dead tensor's
    # memory was reused for different samples
    key = (samples.data_ptr(), samples.numel(), N, str(A.device))
    plan = _FS_PLANS.get(key)
    if plan is not None and (plan.src() is not samples or plan.version != version_of(samples)):
        plan = None
    if plan is None:
        if len(_FS_PLANS) >= 8:
            _FS_PLANS.pop(next(iter(_FS_PLANS)))
        plan = _FourStepPlan(N, samples, A.device)
        plan.src, plan.version = weakref.ref(samples), version_of(samples)
        _FS_PLANS[key] = plan
    st = C.c_void_p(L.stream_of(A))
    dd = _device_copy(d, A.device, torch.float32)
    Y = torch.empty(plan.N2 * plan.N1 * m * 2, dtype=torch.float32, device=A.device)
    L.call("sl_fs_stage1", L.ptr(A), L.dtype_code(A.dtype), A.stride(0), N, m, L.ptr(dd), plan.N1, plan.N2,
           C.c_uint64(plan.rplan), plan.npass, L.ptr(Y), st)
    Zs = torch.empty(plan.nslots * m * 2, dtype=torch.float32, device=A.device)
    if m % 2 == 0 and Y.data_ptr() % 16 == 0 and _STAGE2[0]:
        # the MFMA kernel, groups largest first
        L.call("sl_fs_stage2", L.ptr(Y), plan.N1, plan.N2, m, L.ptr(plan.gptr_s), L.ptr(plan.gk1_s),
               L.ptr(plan.gslot_s), L.ptr(Zs), L.ptr(plan.gord), st)
    else:
        L.call("sl_fs_stage2", L.ptr(Y), plan.N1, plan.N2, m, L.ptr(plan.gptr), L.ptr(plan.gk1),
               L.ptr(plan.gslot), L.ptr(Zs), None, st)
    del Y
    out = torch.empty(plan.S, m, dtype=torch.float32, device=A.device)
    L.call("sl_fs_post", L.ptr(Zs), m, N, L.ptr(plan.samples), plan.S, L.ptr(plan.sa), L.ptr(plan.sb),
           float(scale), L.ptr(out), out.stride(0), st)
    return out


def fjlt_sampled(A: torch.Tensor, dim: int, d: torch.Tensor, samples: torch.Tensor, scale: float) -> torch.Tensor:
    """``scale * P F D A`` along ``dim`` with F the orthonormal DCT-II and P the
    rows ``samples`` (FJLT with many samples, Blendenpik's t = 4n sketch).

    GPU (f32 / bf16 A): one fused pass for D-scaling + Makhoul reordering
    (``sl_fjlt_pre``), rocFFT real-to-complex along ``dim`` (``torch.fft.rfft``),
    and one gather of the S sampled frequencies with the post-twiddle and
    scales (``sl_fjlt_post``) -- the full DCT is never formed.  Elsewhere the
    torch DCT + index_select composition (same numbers up to rounding)."""
    N = A.shape[dim]
    m = A.shape[1 - dim]
    if fourstep_ok(A, dim, samples.numel()):
        return fjlt_fourstep(A, d, samples, scale)
    if A.is_cuda and A.dtype in (torch.float32, torch.bfloat16) and A.stride(1) == 1 and N >= 2:
        import ctypes as C
        from . import _lib
        _lib.require()
        st = C.c_void_p(_lib.stream_of(A))
        dd = _device_copy(d, A.device, torch.float64)   # sl_fjlt_pre takes f64 D
        # always transform along contiguous rows of an m x N buffer (dim 0 input
        # is transposed by the pre-pass itself)
        v = torch.empty(m, N, dtype=torch.float32, device=A.device)
        _lib.call("sl_fjlt_pre", _lib.ptr(A), _lib.dtype_code(A.dtype), N, m, A.stride(0), 2 if dim == 0 else 1,
                  _lib.ptr(dd), _lib.ptr(v), v.stride(0), st)
        V = torch.fft.rfft(v, dim=1)
        del v
        if V.stride(1) != 1:
            V = V.contiguous()
        smp = samples.to(device=A.device, dtype=torch.int64).contiguous()
        S = smp.numel()
        out = torch.empty((S, m) if dim == 0 else (m, S), dtype=torch.float32, device=A.device)
        _lib.call("sl_fjlt_post", _lib.ptr(V), N, m, V.stride(0), 1 + 2 * (1 if dim == 1 else 0), _lib.ptr(smp), S,
                  float(scale), _lib.ptr(out), out.stride(0), st)
        return out
    wd = _work_dtype(A.dtype)
    dv = d.to(device=A.device, dtype=wd)
    X = A.to(wd) * (dv[:, None] if dim == 0 else dv[None, :])
    FA = dct2(X, dim)
    return FA.index_select(dim, samples.to(A.device)) * scale
