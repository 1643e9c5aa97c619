"""Fastfood random features (FastGaussianRFT, FastMaternRFT) and the
Pham-Pagh TensorSketch (PPT).

Fastfood (reference ``sketch/FRFT_data.hpp:26-291``,
``sketch/FRFT_Elemental.hpp:72-250``): block size NB = N, ``numblks =
ceil(S/NB)``; draws in order: S shifts U(0, 2pi), numblks*NB Rademacher (B),
numblks*NB normals (G), numblks*(NB-1) Fisher-Yates swap indices (P); per
block ``x = Sm * F G Pi F (B * a)`` with unitary DCT F, features
``sqrt(2/S) cos(x + shift)``.  ``Sm = sqrt(N)/sigma`` (Gaussian: the
reference's ``1/(sigma sqrt N)`` times the N of its two un-normalised
transforms) or ``sqrt(2 nu / chi2_{2 nu}) sqrt(N) / l`` (Matérn, S chi-squared
draws).

PPT (``sketch/PPT_data.hpp:24-122``, ``sketch/PPT_Elemental.hpp:140-185``):
q CountSketches, then q hash indices and q ±1 values for the homogeneous
term; per column ``P = prod_i FFT(sqrt(gamma) CWT_i(a) + sqrt(c) h_i e_idx_i)``,
``SA = IFFT(P)`` (scaled by 1/S).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..base import distributions as D
from ..ops import fut as _fut
from ..ops import hash_sketch as _hs
from .base import COLUMNWISE, ROWWISE, SketchTransform, register
from .rft import EPI_COS, _FeatureMap
from ..ops import _lib as _L
import ctypes as _C

_vp, _i32, _i64, _f32 = _C.c_void_p, _C.c_int, _C.c_int64, _C.c_float
_L.register("sl_fastfood_tables", [_i32, _vp, _vp])
_L.register("sl_fastfood_apply", [_vp, _i32, _i64, _i32, _i64, _vp, _vp, _vp, _vp, _vp, _f32, _i32, _i32, _i32, _i32,
                                  _i32, _i32, _vp, _vp, _i64, _vp])


class _Fastfood(_FeatureMap):
    mode = EPI_COS

    def _build(self, ctx):
        N, S = self._N, self._S
        self.NB = N
        self.numblks = (S + N - 1) // N
        nb, NB = self.numblks, self.NB
        self.outscale = math.sqrt(2.0 / S)
        self.shifts = ctx.generate_random_samples_array(S, D.Uniform(0.0, 2 * math.pi))
        self.B = ctx.generate_random_samples_array(nb * NB, D.Rademacher()).view(nb, NB)
        self.G = ctx.generate_random_samples_array(nb * NB, D.Normal()).view(nb, NB)
        # nb Fisher-Yates permutations of length NB (reference FRFT_data.hpp:91-116:
        # nb (NB - 1) draws); native, unbiased bounded integers
        import ctypes as C
        from ..ops import _lib
        perms = torch.empty(nb, NB, dtype=torch.int64)
        _lib.call("sl_fastfood_perms_host", _lib.ptr(perms), C.c_uint64(ctx.seed), C.c_uint64(ctx.counter), nb, NB)
        ctx.counter += nb * (NB - 1)
        self.perms = perms
        self.scales = None
        self._Sm = self._make_Sm(ctx)

    def _make_Sm(self, ctx) -> torch.Tensor:
        raise NotImplementedError

    # Largest input dimension realised as a dense W for the fused MFMA path.
    DENSE_MAX_N = 4096

    def realize_W(self, dtype=torch.float64, device=None) -> torch.Tensor:
        """The Fastfood operator as an explicit S x N matrix: every block
        ``Sm * F G Pi F B`` applied to the identity (same draws, exact same
        linear map).  On the MI355X the fused feature GEMM with this W (one
        MFMA launch with the cos epilogue) beats the FFT chain (two DCTs, a
        gather and three scalings per block, each a pass over HBM) for
        N <= DENSE_MAX_N; larger N keep the O(S log N) transform."""
        if self._N > self.DENSE_MAX_N:
            raise ValueError("Fastfood dense realisation is limited to N <= DENSE_MAX_N")
        eye = torch.eye(self._N, dtype=torch.float64, device=device)
        return self._features_pre(eye, COLUMNWISE).to(dtype)

    # ---- fused native path (fastfood.hip): one workgroup per (row, block)
    FUSED_MIN_N, FUSED_MAX_N = 1024, 16384

    def _fused_ok(self, A, dim) -> bool:
        N = self._N
        return (A.is_cuda and dim == ROWWISE and A.dtype in (torch.float32, torch.bfloat16)
                and A.layout == torch.strided and A.dim() == 2 and A.stride(1) == 1
                and self.FUSED_MIN_N <= N <= self.FUSED_MAX_N and (N & (N - 1)) == 0
                and A.shape[0] < 2 ** 31 and self.numblks <= 65535)

    def _fused_operands(self, dev):
        """Device copies of the block draws and the per-N twiddle tables (cached)."""
        key = str(dev)
        cache = self.__dict__.setdefault("_ffdev", {})
        if key not in cache:
            import ctypes as C
            from ..ops import _lib
            M = self._N // 2
            tabn = 2 * (M + (M + 1) + self._N)   # W_M, W_N (k <= M), W_4N complex (sl_fastfood_tables_size)
            tab = torch.empty(tabn, dtype=torch.float32, device=dev)
            _lib.call("sl_fastfood_tables", self._N, _lib.ptr(tab), C.c_void_p(_lib.stream_of(tab)))
            cache[key] = {
                "B": self.B.to(dev, torch.float32).contiguous(),
                "P": self.perms.to(dev, torch.int32).contiguous(),
                "G": self.G.to(dev, torch.float32).contiguous(),
                "Sm": self._Sm.to(dev, torch.float32).contiguous(),
                "sh": self.shifts.to(dev, torch.float32).contiguous(),
                "tab": tab,
            }
        return cache[key]

    def _fused_apply(self, A, out_rows, epi: bool):
        """Rowwise features (m x (i1 - i0)) of A (m x N) in one launch; epi:
        the cosine epilogue fused (outscale cos(. + shift))."""
        import ctypes as C
        from ..ops import _lib
        i0, i1 = out_rows if out_rows is not None else (0, self._S)
        m, N = A.shape
        ops = self._fused_operands(A.device)
        out = torch.empty(m, i1 - i0, dtype=torch.float32, device=A.device)
        if m == 0 or i1 <= i0:
            return out
        b0, b1 = i0 // N, (i1 + N - 1) // N
        _lib.call("sl_fastfood_apply", _lib.ptr(A), _lib.dtype_code(A.dtype), m, N, A.stride(0),
                  _lib.ptr(ops["B"]), _lib.ptr(ops["P"]), _lib.ptr(ops["G"]), _lib.ptr(ops["Sm"]),
                  _lib.ptr(ops["sh"]), float(self.outscale), 1 if epi else 0, self._S, b0, b1, i0, i1,
                  _lib.ptr(ops["tab"]), _lib.ptr(out), out.stride(0), C.c_void_p(_lib.stream_of(A)))
        return out

    # the fused kernel replaces the dense-W GEMM from this N up (measured,
    # profiles/r5/fastfood_v1.jsonl: N = 4096, S = 8192: 5.0 vs 11.7 ms;
    # N = 2048: 5.96 vs 6.29 ms; at N = 1024 the GEMM wins, 3.4 vs 8.3 ms)
    FUSED_PREFER_N = 2048

    def _apply_dense(self, A, dim, in_offset=0, out_rows=None):
        if (in_offset == 0 and A.shape[dim] == self._N and self._N >= self.FUSED_PREFER_N
                and self._fused_ok(A, dim)):
            return self._fused_apply(A, out_rows, epi=True)   # transform + cosine in one launch
        return super()._apply_dense(A, dim, in_offset, out_rows)

    def _features_pre(self, A, dim, in_offset=0, out_rows=None):
        if in_offset != 0 or A.shape[dim] != self._N:
            raise ValueError("Fastfood needs the whole input dimension on one device")
        if self._fused_ok(A, dim):
            return self._fused_apply(A, out_rows, epi=False)
        if A.is_cuda and A.dtype in (torch.float32, torch.bfloat16) and A.layout == torch.strided and self._N >= 2:
            return self._features_pre_gpu(A, dim, out_rows)
        X = A if dim == COLUMNWISE else A.t()
        wdt = torch.float64 if A.dtype == torch.float64 else torch.float32
        X = X.to(wdt)
        outs = []
        dev = A.device
        for i in range(self.numblks):
            s, e = i * self.NB, min((i + 1) * self.NB, self._S)
            W = X * self.B[i].to(dev, wdt)[:, None]
            W = _fut.dct2(W, 0)
            W = W.index_select(0, self.perms[i].to(dev))
            W = W * self.G[i].to(dev, wdt)[:, None]
            W = _fut.dct2(W, 0)
            W = W[: e - s] * self._Sm[s:e].to(dev, wdt)[:, None]
            outs.append(W)
        Z = torch.cat(outs, 0)
        if out_rows is not None:
            Z = Z[out_rows[0]:out_rows[1]]
        return Z if dim == COLUMNWISE else Z.t().contiguous()

    def _features_pre_gpu(self, A, dim, out_rows=None):
        """Per block ``Sm F G Pi F B`` as two native FJLT pipelines
        (``ops.fut.fjlt_sampled``: fused diagonal scale + Makhoul reorder,
        rocFFT R2C, fused post-twiddle gather): the permutation Pi is the
        first pipeline's sample set, G the second's diagonal, the first
        e - s frequencies its samples; no DCT is ever materialised beyond the
        two spectra and no torch elementwise pass runs in between (reference
        ``sketch/FRFT_Elemental.hpp:72-250``)."""
        dev = A.device
        X = A if A.stride(-1) == 1 else A.contiguous()
        outs = []
        r0, r1 = out_rows if out_rows is not None else (0, self._S)
        for i in range(self.numblks):
            s, e = i * self.NB, min((i + 1) * self.NB, self._S)
            if e <= r0 or s >= r1:
                continue
            lo, hi = max(s, r0), min(e, r1)
            Wb = _fut.fjlt_sampled(X, dim, self.B[i], self.perms[i], 1.0)
            Wb = _fut.fjlt_sampled(Wb, dim, self.G[i], torch.arange(lo - s, hi - s), 1.0)
            sm = self._Sm[lo:hi].to(dev, torch.float32)
            outs.append(Wb * (sm[:, None] if dim == COLUMNWISE else sm[None, :]))
        if not outs:
            shape = (0, A.shape[1]) if dim == COLUMNWISE else (A.shape[0], 0)
            return torch.zeros(shape, dtype=torch.float32, device=dev)
        return torch.cat(outs, 0 if dim == COLUMNWISE else 1).contiguous()


@register
class FastGaussianRFT(_Fastfood):
    sketch_type = "FastGaussianRFT"

    def __init__(self, n, s, sigma=1.0, context=None):
        self._sigma = float(sigma)
        super().__init__(n, s, context)

    def _make_Sm(self, ctx):
        return torch.full((self._S,), math.sqrt(self._N) / self._sigma, dtype=torch.float64)

    def _extra_params(self):
        return {"sigma": self._sigma}

    @classmethod
    def _params_from_dict(cls, d):
        return {"sigma": float(d["sigma"])}


@register
class FastMaternRFT(_Fastfood):
    sketch_type = "FastMaternRFT"

    def __init__(self, n, s, nu=1.5, l=1.0, context=None):  # noqa: E741
        self._nu, self._l = float(nu), float(l)
        super().__init__(n, s, context)

    def _make_Sm(self, ctx):
        chi = ctx.generate_random_samples_array(self._S, D.ChiSquared(2 * self._nu))
        return torch.sqrt(2.0 * self._nu / chi) * math.sqrt(self._N) / self._l

    def _extra_params(self):
        return {"nu": self._nu, "l": self._l}

    @classmethod
    def _params_from_dict(cls, d):
        return {"nu": float(d["nu"]), "l": float(d["l"])}


Fastfood = FastGaussianRFT


@register
class PPT(SketchTransform):
    """TensorSketch for the polynomial kernel (gamma <x,y> + c)^q."""

    sketch_type = "PPT"

    def __init__(self, n, s, q=3, c=1.0, gamma=1.0, context=None):
        self._q, self._c, self._gamma = int(q), float(c), float(gamma)
        super().__init__(n, s, context)

    def _build(self, ctx):
        from .hash import CWT
        self.cwts = []
        for _ in range(self._q):
            cw = CWT.__new__(CWT)
            cw._N, cw._S = self._N, self._S
            cw._creation_context = ctx.copy()
            cw._params = {}
            cw._build(ctx)
            self.cwts.append(cw)
        self.hash_idx = ctx.generate_random_samples_array(self._q, D.UniformInt(0, self._S - 1), dtype=torch.int64)
        self.hash_val = ctx.generate_random_samples_array(self._q, D.Rademacher())

    def _apply_dense(self, A, dim, in_offset=0, out_rows=None):
        """Reference loop (PPT_Elemental.hpp:140-185): per column,
        ``P = prod_i FFT(sqrt(gamma) C_i a + sqrt(c) h_i e_{idx_i})``,
        ``SA = IFFT(P)`` (1/S normalised).  Here: the q CountSketches of the
        whole block (dense or CSR input -- sparse input is never densified),
        ONE batched real FFT over the q x S x m stack, ONE fused q-way
        complex product with the scale and the constant term folded into the
        spectrum (``sl_ppt_product`` on GPU), one inverse real FFT."""
        sparse = A.layout == torch.sparse_csr
        if dim == COLUMNWISE:
            X = A
        else:
            X = A.to_sparse_coo().t().coalesce().to_sparse_csr() if sparse else A.t()
        vdt = X.values().dtype if sparse else X.dtype
        wdt = torch.float64 if vdt == torch.float64 else torch.float32
        if not sparse:
            X = X.to(wdt).contiguous()
        m = X.shape[1]
        S, q = self._S, self._q
        sg, sc = math.sqrt(self._gamma), math.sqrt(self._c)
        if q == 0:
            out = torch.zeros(S, m, dtype=wdt, device=A.device)
            return out if dim == COLUMNWISE else out.t().contiguous()
        W = torch.empty(q, S, m, dtype=wdt, device=A.device)
        for i, cw in enumerate(self.cwts):
            W[i] = (_hs.apply_csr_dense_out(cw._hd, X, 0) if sparse else _hs.apply_dense(cw._hd, X, 0)).to(wdt)
        F = torch.fft.rfft(W, dim=1)                      # q x (S/2+1) x m
        del W
        K = F.shape[1]
        if F.is_cuda and F.dtype == torch.complex64:
            import ctypes as C
            from ..ops import _lib
            _lib.require()
            F = F.contiguous()
            P = torch.empty(K, m, dtype=torch.complex64, device=A.device)
            from ..utils.devcache import device_copy
            idx = device_copy(self.hash_idx, A.device, torch.int64)
            hv = device_copy(self.hash_val, A.device, torch.float64)
            _lib.call("sl_ppt_product", _lib.ptr(F), q, K, m, S, _lib.ptr(idx), _lib.ptr(hv), sg, sc, _lib.ptr(P),
                      C.c_void_p(_lib.stream_of(F)))
        else:
            kk = torch.arange(K, dtype=torch.float64, device=A.device)
            P = None
            for i in range(q):
                e = torch.remainder(kk * int(self.hash_idx[i]), S)
                delta = sc * float(self.hash_val[i]) * torch.exp(torch.complex(torch.zeros_like(e), -2 * math.pi * e / S))
                Fi = sg * F[i] + delta.to(F.dtype)[:, None]
                P = Fi if P is None else P * Fi
        out = torch.fft.irfft(P, n=S, dim=0).to(wdt)
        return out if dim == COLUMNWISE else out.t().contiguous()

    def _apply_sparse(self, A, dim, sparse_out):
        return self._apply_dense(A, dim)

    def apply_local_shard(self, A_local, dim, in_offset, out_rows=None):
        return self._apply_dense(A_local, dim, in_offset)

    def _extra_params(self):
        return {"q": self._q, "c": self._c, "gamma": self._gamma}

    @classmethod
    def _params_from_dict(cls, d):
        return {"q": int(d["q"]), "c": float(d["c"]), "gamma": float(d["gamma"])}
