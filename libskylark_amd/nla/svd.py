"""Randomized SVD (Halko-Martinsson-Tropp) and power iteration.

Reference: ``nla/svd.hpp`` — ``approximate_svd_params_t`` (ratio 2, additive 0,
iterations 0, skip_qr false, ``:22-48``), ``PowerIteration`` (``:71-149``),
``ApproximateSVD`` (``:222-318``: ``k = max(r, min(n, ratio*r + add))``, JLT
rowwise sketch, power iteration, ``El::SVD`` of the n x k iterate,
``U = Q B_1``), ``ApproximateSymmetricSVD`` (``:321-392``).

MI355X formulation (tall case m >= n, A row-distributed one shard per GPU):
a subspace iteration pass needs ``Q = orth(A Z)`` and ``A^T Q``.  With
``Y = A Z``, ``R = chol(Y^T Y)``: ``Q = Y R^{-1}`` and ``A^T Q = (A^T Y)
R^{-1}`` — so ONE streaming read of A (``ops.tallskinny.fused_pass``)
yields both, where the textbook loop reads A twice.  The reference itself
uses this identity in its ``skip_qr, num_iterations == 0`` branch
(``nla/svd.hpp:263-269``).  Per pass the only collective is one all-reduce of
``[A^T Y | Y^T Y]`` ((n + k) x k floats).  Robustness: the n x k iterate is
re-orthonormalised exactly (Householder, fp64) between passes; the final
basis is CholeskyQR2-refined from the stored ``Y`` (m x k, a fraction of A's
bytes); if a Gram factorisation fails the code falls back to TSQR.  The
GPU-resident plan (``_DevicePlan``) instead takes an fp64 Gram of the stored
f32 ``Y`` on the f64 matrix cores (``ops.tallskinny.gram64``) and needs one
fp64 CholeskyQR only.
"""
from __future__ import annotations

import ctypes
import math
import os
import sys
import time
import weakref

from dataclasses import dataclass

import numpy as np
import torch
from scipy.linalg import solve_triangular

from ..base import linalg as L
from ..base.context import Context
from ..base.exceptions import InvalidParametersError, SkylarkError
from ..parallel.comm import Comm
from ..parallel.distmatrix import DistMatrix
from ..utils.timer import PROFILER


@dataclass
class ApproximateSVDParams:
    oversampling_ratio: int = 2
    oversampling_additive: int = 0
    num_iterations: int = 0
    skip_qr: bool = False
    sketch: str = "JLT"          # "JLT" (reference) | "FJLT" | "CWT"
    graph: bool = True           # replay the device path as hipGraphs once warm
    # device path: wait for this call's status word and raise / warn for THIS
    # call.  None = True on the general-precision engine (f32 / f64 operands,
    # the host path's synchronous failure semantics) and False on the fused
    # bf16 engine (flags surface on the next call or last_device_status())
    check: bool | None = None
    am_i_printing: bool = False
    log_level: int = 0
    prefix: str = ""
    debug_level: int = 0

    @classmethod
    def from_dict(cls, d: dict):
        keys = cls.__dataclass_fields__.keys()
        return cls(**{k: v for k, v in d.items() if k in keys})

    def to_dict(self):
        return dict(self.__dict__)


approximate_svd_params_t = ApproximateSVDParams


def _sketch_operator(kind: str, n: int, k: int, ctx: Context, device, dtype) -> torch.Tensor:
    """Z0 = Omega^T (n x k) for the rowwise sketch A Omega^T."""
    from .. import sketch as S
    cls = {"JLT": S.JLT, "FJLT": S.FJLT, "CWT": S.CWT, "CT": S.CT}.get(kind.upper())
    if cls is None:
        raise InvalidParametersError(f"unsupported sketch {kind} for approximate_svd")
    sk = cls(n, k, context=ctx)
    if kind.upper() == "FJLT":
        return sk.realize(dtype=dtype, device=device, transpose=True)
    if kind.upper() == "CWT":
        return sk.realize(dtype=torch.float64).t().to(device=device, dtype=dtype).contiguous()
    return sk.realize(dtype=torch.float64, device=device).t().to(dtype).contiguous()


_ROWBUF: dict = {}


def _whole_rows(A) -> bool:
    """[MC,MR] whose grid has one column: each rank stores complete rows."""
    return A.layout == "MC_MR" and A.grid is not None and A.grid.pc == 1


def _as_rowdist(A):
    """(local row shard tensor, comm, m_global, DistMatrix or None).

    A non-row-distributed DistMatrix (e.g. ``[MC,MR]``) is redistributed to
    ``[VC,*]`` by one all-to-all into a persistent per-geometry buffer, so
    repeated calls on the same operand keep a stable shard address (the
    device plan and its graphs stay valid) and allocate nothing."""
    if isinstance(A, DistMatrix):
        if _whole_rows(A):
            # [MC,MR] on a p x 1 grid: every rank already holds whole rows (its
            # cyclic row tiles).  randSVD only ever reduces over rows, so the
            # local tile IS a row shard -- no data moves; U comes back in the
            # same local row order (_u_like)
            return A.local, A.comm, A.shape[0], A
        if A.layout not in ("VC_STAR", "VR_STAR"):
            key = (A.layout, A.shape, A.block, None if A.grid is None else (A.grid.pr, A.grid.pc),
                   A.comm.rank, A.comm.size, id(A.comm.group), A.local.dtype, str(A.local.device))
            buf = _ROWBUF.get(key)
            with PROFILER.phase("svd.redistribute"):
                R = A.redistribute("VC_STAR", out=buf)
            if buf is None:
                if len(_ROWBUF) >= 2:
                    _ROWBUF.pop(next(iter(_ROWBUF)))
                _ROWBUF[key] = R.local
            A = R
        return A.local, A.comm, A.shape[0], A
    return A, _LocalComm(), A.shape[0], None


def _u_like(U_loc, m, rank, comm, Ad, A):
    """U as a DistMatrix in A's layout (the reference's UType follows A's
    type, nla/svd.hpp:222); computed row-distributed, moved by one
    all-to-all of the m x rank factor when A is 2-D."""
    if isinstance(A, DistMatrix) and _whole_rows(A):
        # local rows of U are A's local rows (its cyclic row tiles), all r columns
        return DistMatrix(U_loc.contiguous(), (m, rank), "MC_MR", comm, A.grid, (A.block[0], max(1, rank)))
    U = DistMatrix(U_loc.contiguous(), (m, rank), "VC_STAR", comm)
    if isinstance(A, DistMatrix) and A.layout not in ("VC_STAR", "VR_STAR"):
        with PROFILER.phase("svd.redistribute"):
            U = U.redistribute(A.layout, A.grid, A.block if A.layout == "MC_MR" else None)
    return U


class _LocalComm(Comm):
    def __init__(self):
        self.group, self.rank, self.size, self.backend, self._active = None, 0, 1, None, False


def _small_chol_inv(G: torch.Tensor):
    """R^{-1} for R = chol(G)^T (upper), fp64; None when G is not numerically SPD."""
    L_, info = torch.linalg.cholesky_ex(G)
    if int(info) != 0:
        return None, None
    R = L_.t()
    I = torch.eye(R.shape[0], dtype=R.dtype, device=R.device)
    Rinv = torch.linalg.solve_triangular(R, I, upper=True)
    return R, Rinv


def approximate_svd(A, rank: int, context: Context | None = None,
                    params: ApproximateSVDParams | None = None):
    """Rank-``rank`` approximate SVD ``A ~ U diag(s) V^T``.

    ``A``: dense ``torch.Tensor`` (any device/dtype) or a DistMatrix.  Returns
    ``(U, s, V)``; U is row-distributed like A (a DistMatrix ``[VC,*]`` when A
    is distributed), s and V replicated.
    """
    if _TRACE:
        _T0[0] = time.perf_counter()
    from .. import default_context
    ctx = context if context is not None else default_context()
    params = params or ApproximateSVDParams()
    m, n = (A.shape if not isinstance(A, DistMatrix) else A.shape)
    if rank > min(m, n):
        raise InvalidParametersError(f"Incompatible matrix dimensions ({min(m, n)}) and target rank ({rank})")
    if m < n:
        # wide (reference's m < n branch, nla/svd.hpp:287-317): work on the
        # tall A^T and swap the factors.  For a DistMatrix, U (m x rank, from
        # the replicated right factor of A^T) is sliced into A's layout with no
        # communication and V (n x rank) is gathered to every rank like the
        # tall case's V.
        At = _transpose(A)
        Ut, s, Vt = approximate_svd(At, rank, ctx, params)
        if isinstance(A, DistMatrix):
            U = DistMatrix.from_global(Vt, A.layout, A.comm, A.grid, A.block if A.layout == "MC_MR" else None)
            return U, s, Ut.to_global()
        return Vt, s, Ut
    k = max(rank, min(n, params.oversampling_ratio * rank + params.oversampling_additive))
    A_in = A
    A_loc, comm, _, Ad = _as_rowdist(A)
    dev = A_loc.device
    work = torch.float64 if A_loc.dtype == torch.float64 else torch.float32
    from ..ops import tallskinny as T

    _LAST_ENGINE[0] = "host"
    if A_loc.is_cuda:
        res = _approximate_svd_device(A_loc, comm, m, n, rank, k, ctx, params)
        if res is not None:
            U_loc, s, V = res
            if Ad is not None:
                return _u_like(U_loc, m, rank, comm, Ad, A_in), s, V
            return U_loc, s, V
    prof = PROFILER
    with prof.phase("svd.sketch"):
        Zh = _sketch_operator(params.sketch, n, k, ctx, "cpu", torch.float64).numpy()
    q = max(0, int(params.num_iterations))
    Y = W = G = None
    for it in range(q + 1):
        last = it == q
        with prof.phase("svd.fused_pass"):
            # intermediate passes only need orth(A^T A Z): no Gram, bf16 y for W
            Wd, Gd, Y = T.fused_pass(A_loc, torch.from_numpy(Zh).to(dev, work), keep_y=last,
                                     gram=last, exact=last)
        with prof.phase("svd.allreduce_small"):
            WG = torch.cat([Wd.double(), Gd.double()], 0) if last else Wd.double().contiguous()
            comm.all_reduce(WG)
            WGh = WG.cpu().numpy()
        W, G = WGh[:n], (WGh[n:] if last else None)
        if last:
            break
        with prof.phase("svd.host_orth"):
            # orth(A^T Q) = orth(W R^{-1}) = orth(W): R^{-1} only re-mixes columns
            Zh = _normalize_cols(W) if params.skip_qr else _cholqr2_host(W)[0]
    # ---- final basis Q = Y Rt^{-1}: CholeskyQR2 on the stored Y, first factor
    #      from the pass's own Gram (no extra read), refinement Gram(s) exact f32.
    with prof.phase("svd.final_qr"):
        R1 = _chol_upper(G)
        if R1 is None:
            _, G1 = T.f32_xm(Y, None, store=False, gram=True) if work == torch.float32 else (None, L.gram(Y, None))
            comm.all_reduce(G1)
            R1 = _chol_upper(G1.cpu().numpy())
    if R1 is None:
        # rank-deficient / ill-conditioned sample (e.g. repeated FJLT samples):
        # Householder TSQR gives an orthonormal Q regardless; one extra pass
        # over A forms A^T Q explicitly.
        Qx, _ = L.tsqr(Y, comm)
        Qx = Qx.to(work)
        Vt = L.gemm_tn(A_loc.to(work) if A_loc.dtype != work else A_loc, Qx, comm).double().cpu().numpy()
        Qv, Rv = _cholqr2_host(Vt)
        Ur, s, Vrt = np.linalg.svd(Rv)
        Ub = torch.from_numpy(np.ascontiguousarray(Vrt.T[:, :rank])).to(dev, work)
        U_loc = Qx @ Ub
        s = torch.from_numpy(s[:rank].copy()).to(dev, work)
        V = torch.from_numpy(np.ascontiguousarray((Qv @ Ur)[:, :rank])).to(dev, work)
        if Ad is not None:
            return _u_like(U_loc, m, rank, comm, Ad, A_in), s, V
        return U_loc, s, V
    Rt = R1
    with prof.phase("svd.final_qr"):
        for _ in range(2):  # CholeskyQR2, a third step only if still far from orthonormal
            Rinv = _rsolve(np.eye(k), Rt)
            if work == torch.float32:
                _, G2 = T.f32_xm(Y, torch.from_numpy(Rinv).float().to(dev), store=False, gram=True)
            else:
                G2 = L.gram(Y @ torch.from_numpy(Rinv).to(dev, work), None)
            comm.all_reduce(G2)
            R2 = _chol_upper(G2.cpu().numpy())
            if R2 is None:
                break
            Rt = R2 @ Rt
            if np.abs(R2 - np.eye(k)).max() < 1e-3:
                break
    with prof.phase("svd.small_svd"):
        Vt = _rsolve(W, Rt)  # = A^T Q  (n x k), Q = Y Rt^{-1} orthonormal
        # SVD of A^T Q = V S Ub^T  =>  B = Q^T A = Ub S V^T   (QR first: n x k -> k x k)
        Qv, Rv = _cholqr2_host(Vt)
        Ur, s, Vrt = np.linalg.svd(Rv)
        Vv = Qv @ Ur
        Ub = Vrt.T
        M = _rsolve(np.eye(k), Rt) @ Ub[:, :rank]  # U = Y Rt^{-1} Ub_r
        Mt = torch.from_numpy(np.ascontiguousarray(M)).to(dev, work)
    with prof.phase("svd.form_U"):
        U_loc = T.f32_xm(Y, Mt, store=True)[0] if work == torch.float32 else Y @ Mt
    s = torch.from_numpy(s[:rank].copy()).to(dev, work)
    V = torch.from_numpy(np.ascontiguousarray(Vv[:, :rank])).to(dev, work)
    if Ad is not None:
        return _u_like(U_loc, m, rank, comm, Ad, A_in), s, V
    return U_loc, s, V


vp_, i32_, i64_, u64_, f64_ = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double



_ENGINE_REG = [False]


def _engine_lib():
    from ..ops import _lib
    if not _ENGINE_REG[0]:
        _ENGINE_REG[0] = True
        _lib.register("sl_rsvd_plan_create", [i64_, i64_, i64_, i32_, i32_, i32_, ctypes.POINTER(vp_)])
        _lib.register("sl_rsvd_plan_destroy", [vp_])
        _lib.register("sl_rsvd_set_fjlt", [vp_, u64_, u64_, u64_, f64_, vp_])
        _lib.register("sl_rsvd_set_zt", [vp_, vp_, vp_])
        _lib.register("sl_rsvd_set_dense", [vp_, i32_, u64_, u64_, f64_, f64_, f64_, vp_])
        _lib.register("sl_rsvd_segment", [vp_, vp_, i32_, vp_])
        _lib.register("sl_rsvd_reduce_buffer", [vp_], vp_)
        _lib.register("sl_rsvd_finish", [vp_, vp_, i64_, vp_, vp_, vp_])
        _lib.register("sl_rsvd_run", [vp_, vp_, i32_, vp_, i64_, vp_, vp_, vp_])
        _lib.register("sl_rsvd_plan_bind", [vp_, vp_, vp_])
        _lib.register("sl_rsvd_status_mirror", [vp_], vp_)
        _lib.register("sl_rsvd_flush", [vp_, vp_])
        _lib.register("sl_rsvd_plan_set_fault", [vp_, i32_, u64_])
        _lib.register("sl_rsvd_gen_create", [i64_, i64_, i64_, i32_, i32_, i32_, i32_, ctypes.POINTER(vp_)])
        _lib.register("sl_rsvd_gen_destroy", [vp_])
        _lib.register("sl_rsvd_gen_bind", [vp_, vp_, vp_])
        _lib.register("sl_rsvd_gen_native", [vp_], ctypes.c_int)
        _lib.register("sl_rsvd_gen_set_fjlt", [vp_, u64_, u64_, u64_, f64_])
        _lib.register("sl_rsvd_gen_set_dense", [vp_, i32_, u64_, u64_, f64_, f64_, f64_])
        _lib.register("sl_rsvd_gen_set_z", [vp_, vp_, vp_])
        _lib.register("sl_rsvd_gen_segment", [vp_, vp_, i32_, vp_])
        _lib.register("sl_rsvd_gen_reduce_span", [vp_, i32_, ctypes.POINTER(i64_), ctypes.POINTER(i64_)])
        _lib.register("sl_rsvd_gen_finish", [vp_, vp_, i64_, vp_, vp_, vp_])
        _lib.register("sl_rsvd_gen_run", [vp_, vp_, vp_, i64_, vp_, vp_, vp_])
    return _lib


# status bits of a device call (rsvd_core.hip)
ST_PIVOT, ST_NONFINITE, ST_NOCONV, ST_RANK, ST_TIMEOUT = 1, 2, 4, 8, 16


class _EnginePlan:
    """Device randSVD for one (A, k, rank, q) configuration on the C++ engine
    (``_native/src/rsvd_engine.cpp``): every stage of the call -- sketch
    operator, q + 1 fused passes, the CholeskyQRs between them, the fp64
    core (Cholesky, C = Rt^-T W^T W Rt^-1, tridiagonal eigensolve) and the
    U = Y M / V = W N finish -- runs on the GPU; nothing returns to the host
    inside a call.

    One rank: one ctypes call replays the engine's own hipGraph of the
    segments and launches the finish into fresh U / s / V tensors.  Several
    ranks: the engine's segments with ``comm.all_reduce`` of the [W; G]
    buffer between them; when every all-reduce is the one-shot IPC kernel
    the segments and collectives are captured as one torch CUDA graph.

    The device status word (pivot dropped, non-finite data, no eigensolver
    convergence, rank < r, a boundary wait timed out) is copied back
    asynchronously: by default a flag of a call is reported by the next call
    on the plan (``last_status``), never by a host sync.  With
    ``ApproximateSVDParams(check=True)`` the call itself synchronises on its
    own status word and raises (timeout, non-finite data) before returning."""

    def __init__(self, A_loc, comm, n, rank, k, q, use_graph):
        L = _engine_lib()
        m = A_loc.shape[0]
        self.dev = A_loc.device
        self.Aref = weakref.ref(A_loc)
        self.comm, self.n, self.rank, self.k, self.q = comm, n, rank, k, q
        self.m = m
        self.use_graph = use_graph
        h = ctypes.c_void_p()
        L.call("sl_rsvd_plan_create", m, n, A_loc.stride(0), k, rank, q, ctypes.byref(h))
        self.h = h
        self._fin = weakref.finalize(self, _destroy_plan, h.value)
        # [W (n x k); G (k x k)] f64 reduce buffer (all-reduced across ranks
        # between the segments) and the device status word, torch-owned
        self.WG = torch.empty((n + k) * k, dtype=torch.float64, device=self.dev)
        self.status_dev = torch.zeros(1, dtype=torch.int32, device=self.dev)
        L.call("sl_rsvd_plan_bind", h, ctypes.c_void_p(self.WG.data_ptr()), ctypes.c_void_p(self.status_dev.data_ptr()))
        # the final kernel writes the call's status word into host-mapped
        # memory (no D2H copy node); fallback: a pinned copy after the call
        fn = L.require().sl_rsvd_status_mirror
        fn.argtypes, fn.restype = [vp_], vp_
        mp = fn(h)
        self.mirror = ctypes.c_int.from_address(mp) if mp else None
        self.status_host = torch.zeros(1, dtype=torch.int32).pin_memory() if self.mirror is None else None
        self.status_ev = None
        self.last_status = 0
        self.poisoned = False
        self.calls = 0
        self.g = None          # multi-rank: torch graph of segments + one-shot all-reduces
        self.g_failed = False

    def graph_built(self):
        return self.calls >= 2 and self.use_graph

    def _segments(self, A):
        L = _engine_lib()
        st = ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        for i in range(self.q + 2):
            with PROFILER.phase("svd.segment"):
                L.call("sl_rsvd_segment", self.h, ctypes.c_void_p(A.data_ptr()), i, st)
            if i <= self.q:
                cnt = (self.n + self.k if i == self.q else self.n) * self.k
                with PROFILER.phase("svd.allreduce_small"):
                    self.comm.all_reduce(self.WG[:cnt])

    def _collectives_capturable(self):
        os_ = getattr(self.comm, "_oneshot", None)
        return bool(os_) and self.calls >= 1 and os_.fits(self.WG)

    def __call__(self, A, Z=None, fjlt=None, dense=None):
        L = _engine_lib()
        dev = self.dev
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        self._poll_status()
        if fjlt is not None:
            L.call("sl_rsvd_set_fjlt", self.h, int(fjlt[0]), int(fjlt[1]), int(fjlt[2]), float(fjlt[3]), st)
        elif dense is not None:
            code, seed, base, p0, p1, scale = dense
            L.call("sl_rsvd_set_dense", self.h, int(code), int(seed), int(base), float(p0), float(p1), float(scale), st)
        else:
            Zt = Z.t().to(torch.bfloat16).contiguous()
            L.call("sl_rsvd_set_zt", self.h, ctypes.c_void_p(Zt.data_ptr()), st)
        r = self.rank
        U = torch.empty(self.m, r, dtype=torch.float32, device=dev)
        s = torch.empty(r, dtype=torch.float32, device=dev)
        V = torch.empty(self.n, r, dtype=torch.float32, device=dev)
        warm = self.use_graph and self.calls >= 1 and not PROFILER.enabled
        if self.comm.size == 1:
            L.call("sl_rsvd_run", self.h, ctypes.c_void_p(A.data_ptr()), 1 if warm else 0,
                   ctypes.c_void_p(U.data_ptr()), r, ctypes.c_void_p(s.data_ptr()), ctypes.c_void_p(V.data_ptr()), st)
        else:
            # the deferred FJLT operator launches here, never inside a capture
            L.call("sl_rsvd_flush", self.h, st)
            if warm and self.g is None and not self.g_failed and self._collectives_capturable():
                try:
                    g = torch.cuda.CUDAGraph()
                    side = torch.cuda.Stream(device=dev)
                    side.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                        self._segments(A)
                    torch.cuda.current_stream(dev).wait_stream(side)
                    self.g = g
                except Exception:  # noqa: BLE001 - capture unsupported here: stay eager
                    self.g, self.g_failed = None, True
            if self.g is not None:
                self.g.replay()
            else:
                self._segments(A)
            with PROFILER.phase("svd.form_U"):
                L.call("sl_rsvd_finish", self.h, ctypes.c_void_p(U.data_ptr()), r, ctypes.c_void_p(s.data_ptr()),
                       ctypes.c_void_p(V.data_ptr()), st)
        # status word of this call back to the host, no wait
        if self.status_ev is None:
            self.status_ev = torch.cuda.Event()
        if self.mirror is None or self.comm.size > 1:
            # several ranks: the finish runs outside the engine's graph and the
            # mirror is written by the final kernel too; one path for both
            if self.status_host is None:
                self.status_host = torch.zeros(1, dtype=torch.int32).pin_memory()
            self.status_host.copy_(self.status_dev, non_blocking=True)
        self.status_ev.record()
        self.calls += 1
        return U, s, V

    def _poll_status(self):
        if self.status_ev is not None and self.status_ev.query():
            self.status_ev = None   # consumed: a flag is reported once
            self.last_status = self._status_word()
            self._report(self.last_status, "previous call")

    def _report(self, st, which):
        if st & ST_TIMEOUT:
            self.poisoned = True   # sync words left mid-protocol: never reused
            _drop_plan(self)
            raise RuntimeError(f"approximate_svd (device): a pass-boundary wait timed out (status {st}); "
                               f"the {which}'s results are invalid")
        if st & (ST_NONFINITE | ST_RANK | ST_NOCONV):
            import warnings
            warnings.warn(f"approximate_svd (device): {which} flagged status {st} "
                          "(2: non-finite data, 4: eigensolver not converged, 8: numerical rank < r)",
                          RuntimeWarning, stacklevel=4)

    def _status_word(self) -> int:
        mask = ST_PIVOT | ST_NONFINITE | ST_NOCONV | ST_RANK | ST_TIMEOUT
        if self.mirror is not None and self.comm.size == 1:
            return int(self.mirror.value) & mask
        return int(self.status_host[0]) & mask

    def wait_status(self) -> int:
        """Synchronise with the last call and return its status bits (read
        from the device status word itself)."""
        if self.status_ev is not None:
            self.status_ev.synchronize()
            self.status_ev = None
            mask = ST_PIVOT | ST_NONFINITE | ST_NOCONV | ST_RANK | ST_TIMEOUT
            self.last_status = (int(self.status_dev.cpu()[0]) | self._status_word()) & mask
        return self.last_status

    def check(self):
        """Raise / warn on this plan's most recent call (synchronises)."""
        st = self.wait_status()
        self._report(st, "call")


def _drop_plan(plan):
    for key, p in list(_PLANS.items()):
        if p is plan:
            _PLANS.pop(key, None)


class _GenPlan(_EnginePlan):
    """Device randSVD of f32 / f64 / bf16 A of any width (k <= 128) on the
    general-precision engine (``_native/src/rsvd_general.hip``): the two
    products over A per pass are rocBLAS GEMMs, the CholeskyQR factors and the
    core eigensolver the one-wave kernels (k <= 64) or rocSOLVER (k <= 128),
    W / H / G and the core in f64 -- no host round trip inside a call.  U, s,
    V come back in A's precision (f32 for bf16 A).  Same segment contract,
    status handling and multi-rank all-reduces as :class:`_EnginePlan`."""

    def __init__(self, A_loc, comm, n, rank, k, q):
        L = _engine_lib()
        from ..ops import _lib as OL
        m = A_loc.shape[0]
        self.dev = A_loc.device
        self.Aref = weakref.ref(A_loc)
        self.comm, self.n, self.rank, self.k, self.q, self.m = comm, n, rank, k, q, m
        self.use_graph = False
        self.out_dtype = torch.float64 if A_loc.dtype == torch.float64 else torch.float32
        dt = {torch.float32: 0, torch.float64: 1, torch.bfloat16: 2}[A_loc.dtype]
        self.A_dtype = A_loc.dtype
        h = ctypes.c_void_p()
        L.call("sl_rsvd_gen_create", m, n, A_loc.stride(0), k, rank, q, dt, ctypes.byref(h))
        self.h = h
        self._fin = weakref.finalize(self, _destroy_gen_plan, h.value)
        # hand-written products only (f32 / f64 A, k <= 64): no rocBLAS call
        self.native = bool(L.require().sl_rsvd_gen_native(h))
        self.WG = torch.empty((n + k) * k, dtype=torch.float64, device=self.dev)
        self.status_words = torch.zeros(16, dtype=torch.int32, device=self.dev)
        self.status_dev = self.status_words[:1]
        L.call("sl_rsvd_gen_bind", h, ctypes.c_void_p(self.WG.data_ptr()),
               ctypes.c_void_p(self.status_words.data_ptr()))
        self.mirror = None
        self.status_host = torch.zeros(1, dtype=torch.int32).pin_memory()
        self.status_ev = None
        self.last_status = 0
        self.poisoned = False
        self.calls = 0
        self.g, self.g_failed = None, True
        del OL

    def _segments(self, A):
        L = _engine_lib()
        st = ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        off, cnt = ctypes.c_int64(), ctypes.c_int64()
        fn = L.require().sl_rsvd_gen_num_segments   # returns the count (not a status code)
        fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
        for i in range(fn(self.h)):
            with PROFILER.phase("svd.segment"):
                L.call("sl_rsvd_gen_segment", self.h, ctypes.c_void_p(A.data_ptr()), i, st)
            L.call("sl_rsvd_gen_reduce_span", self.h, i, ctypes.byref(off), ctypes.byref(cnt))
            if cnt.value:
                with PROFILER.phase("svd.allreduce_small"):
                    self.comm.all_reduce(self.WG[off.value:off.value + cnt.value])

    def __call__(self, A, Z=None, fjlt=None, dense=None):
        L = _engine_lib()
        dev = self.dev
        st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        self._poll_status()
        if fjlt is not None:
            L.call("sl_rsvd_gen_set_fjlt", self.h, int(fjlt[0]), int(fjlt[1]), int(fjlt[2]), float(fjlt[3]))
        elif dense is not None:
            code, seed, base, p0, p1, scale = dense
            L.call("sl_rsvd_gen_set_dense", self.h, int(code), int(seed), int(base), float(p0), float(p1), float(scale))
        else:
            Zc = Z.to(self.A_dtype).contiguous()
            L.call("sl_rsvd_gen_set_z", self.h, ctypes.c_void_p(Zc.data_ptr()), st)
        r = self.rank
        U = torch.empty(self.m, r, dtype=self.out_dtype, device=dev)
        s = torch.empty(r, dtype=self.out_dtype, device=dev)
        V = torch.empty(self.n, r, dtype=self.out_dtype, device=dev)
        if self.comm.size == 1:
            L.call("sl_rsvd_gen_run", self.h, ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(U.data_ptr()), r,
                   ctypes.c_void_p(s.data_ptr()), ctypes.c_void_p(V.data_ptr()), st)
        else:
            self._segments(A)
            with PROFILER.phase("svd.form_U"):
                L.call("sl_rsvd_gen_finish", self.h, ctypes.c_void_p(U.data_ptr()), r, ctypes.c_void_p(s.data_ptr()),
                       ctypes.c_void_p(V.data_ptr()), st)
        if self.status_ev is None:
            self.status_ev = torch.cuda.Event()
        self.status_host.copy_(self.status_dev, non_blocking=True)
        self.status_ev.record()
        self.calls += 1
        return U, s, V


def _destroy_gen_plan(ptr):
    try:
        from ..ops import _lib
        lib = _lib.load(build_if_missing=False)
        if lib is not None and ptr:
            torch.cuda.synchronize()
            lib.sl_rsvd_gen_destroy(ctypes.c_void_p(ptr))
    except Exception:  # noqa: BLE001 - interpreter shutdown
        pass


def _destroy_plan(ptr):
    try:
        from ..ops import _lib
        lib = _lib.load(build_if_missing=False)
        if lib is not None and ptr:
            torch.cuda.synchronize()
            lib.sl_rsvd_plan_destroy(ctypes.c_void_p(ptr))
    except Exception:  # noqa: BLE001 - interpreter shutdown
        pass


_PLANS: dict = {}
_TRACE = os.environ.get("SKH_TRACE_SVD", "0") == "1"   # host-side phase timestamps
_T0 = [0.0]


def _engine_ok(A_loc, n, k) -> bool:
    return (A_loc.is_cuda and A_loc.dtype == torch.bfloat16 and A_loc.stride(1) == 1 and A_loc.stride(0) % 8 == 0
            and n % 8 == 0 and 16 <= n <= 1024 and 1 <= k <= 48 and A_loc.shape[0] >= 1)


def _gen_ok(A_loc, n, k) -> bool:
    return (A_loc.is_cuda and A_loc.dtype in (torch.float32, torch.float64, torch.bfloat16)
            and A_loc.stride(1) == 1 and A_loc.stride(0) >= n and 1 <= k <= min(n, 128) and A_loc.shape[0] >= 1)


_DUMMY: dict = {}


def _uniform_shard(A_loc, n):
    """(shard, rows) with the engine choice a function of rank-uniform values
    only (n, k, dtype, device type), so every rank of a multi-rank call picks
    the same engine and joins the same collectives with no agreement round:
    a rank that owns no rows runs on one zero row (it adds nothing to any
    sum; its U slice is cut back to 0 rows), and a shard whose strides the
    engines cannot take is made contiguous (rows % 8 == 0 then depends on n
    alone).  (A rank-local cache of an agreement collective could let one
    rank skip the collective another one enters.)"""
    rows = A_loc.shape[0]
    if rows == 0:
        key = (n, A_loc.dtype, str(A_loc.device))
        z = _DUMMY.get(key)
        if z is None:
            z = _DUMMY[key] = torch.zeros(1, n, dtype=A_loc.dtype, device=A_loc.device)
        return z, 0
    if A_loc.stride(1) != 1 or A_loc.stride(0) < n or (n % 8 == 0 and A_loc.stride(0) % 8 != 0):
        A_loc = A_loc.contiguous()
    return A_loc, rows


def _approximate_svd_device(A_loc, comm, m, n, rank, k, ctx, params):
    """GPU-resident path: the C++ engines run the whole call; no host
    synchronisation inside it.  bf16 A with n <= 1024, k <= 48: the fused
    engine (one read of A per pass); any other f32 / f64 / bf16 A with k <= 128:
    the general-precision engine.  Returns None when neither covers the call
    (the caller then runs the host-driven path)."""
    rows = A_loc.shape[0]
    if comm.size > 1:
        A_loc, rows = _uniform_shard(A_loc, n)
    fused, gen = _engine_ok(A_loc, n, k), _gen_ok(A_loc, n, k)
    if not fused and not gen:
        return None
    if _TRACE:
        print(f"[svd.trace] python_prep={(time.perf_counter() - _T0[0]) * 1e6:.0f}us", file=sys.stderr)
    dev = A_loc.device
    fjlt = None
    Z = None
    dense = None
    kind = params.sketch.upper()
    if kind in ("JLT", "CT"):
        # dense operator: the engine realises it on the device from the
        # sketch's stream (same f64 -> f32 -> bf16 values as realize())
        from .. import sketch as S
        sk = (S.JLT if kind == "JLT" else S.CT)(n, k, context=ctx)
        p0, p1 = sk.dist.params()
        dense = (sk.dist.code, sk.entries.seed, sk.entries.base, p0, p1, sk.scale)
    elif kind == "FJLT":
        # FJLT_data draw layout: N Rademacher signs, then S sample rows; the
        # operator itself is realised on the device by the engine
        base_d = ctx.counter
        base_s = base_d + n
        ctx.counter = base_s + k
        fjlt = (ctx.seed, base_d, base_s, math.sqrt(n / k))
    else:
        with PROFILER.phase("svd.sketch"):
            Z = _sketch_operator(params.sketch, n, k, ctx, dev, torch.float32)
    q = max(0, int(params.num_iterations))
    key = (A_loc.data_ptr(), tuple(A_loc.shape), tuple(A_loc.stride()), str(dev), rank, k, q, comm.size,
           id(getattr(comm, "group", None)), A_loc.dtype, fused)
    plan = _PLANS.get(key)
    if plan is not None and (plan.Aref() is None or plan.poisoned):
        plan = None  # the operand this plan was built for is gone / a timed-out plan
    if plan is None:
        if len(_PLANS) >= 4:
            _PLANS.pop(next(iter(_PLANS)))
        plan = None
        if fused:
            try:
                plan = _EnginePlan(A_loc, comm, n, rank, k, q, bool(params.graph) and dev.type == "cuda")
            except (RuntimeError, SkylarkError):
                # e.g. the boundary grid cannot be co-resident on this device
                # (a device property: the same on every rank of a node)
                if not gen:
                    raise
        if plan is None:
            plan = _GenPlan(A_loc, comm, n, rank, k, q)
        _PLANS[key] = plan
    out = plan(A_loc, Z=Z, fjlt=fjlt, dense=dense)
    _LAST_ENGINE[0] = "fused" if type(plan) is _EnginePlan else "general"
    if rows != A_loc.shape[0]:
        out = (out[0][:rows],) + tuple(out[1:])   # a rank without rows ran on one zero row
    check = params.check if params.check is not None else isinstance(plan, _GenPlan)
    if check:
        plan.check()
    return out


_LAST_ENGINE = ["none"]


def last_engine() -> str:
    """Which path ran this process's most recent approximate_svd call:
    "fused" (one-read bf16 engine), "general" (general-precision engine) or
    "host" (host-driven small algebra).  Multi-rank callers compare it
    across ranks (bench.py): every rank must have run the same one."""
    return _LAST_ENGINE[0]


def last_device_status(wait: bool = True) -> int:
    """Status bits of the most recent device randSVD call (0 = clean; see
    ``ST_*``)."""
    if not _PLANS:
        return 0
    plan = list(_PLANS.values())[-1]
    return plan.wait_status() if wait else plan.last_status


# ------------------------------------------------------- host small LA (fp64)
def _chol_upper(G: np.ndarray):
    """Upper Cholesky factor R (G = R^T R) or None if G is not numerically SPD."""
    try:
        R = np.linalg.cholesky(0.5 * (G + G.T)).T
    except np.linalg.LinAlgError:
        return None
    d = np.abs(np.diag(R))
    if d.min() <= 1e-13 * d.max():
        return None
    return R


def _rsolve(X: np.ndarray, R: np.ndarray) -> np.ndarray:
    """X R^{-1} for upper-triangular R."""
    return solve_triangular(R, X.T, trans="T", lower=False).T


def _cholqr2_host(W: np.ndarray):
    """CholeskyQR2 of a small n x k fp64 matrix; Householder QR if it breaks down."""
    R1 = _chol_upper(W.T @ W)
    if R1 is not None:
        Q1 = _rsolve(W, R1)
        R2 = _chol_upper(Q1.T @ Q1)
        if R2 is not None:
            return _rsolve(Q1, R2), R2 @ R1
    Q, R = np.linalg.qr(W)
    return Q, R


def _normalize_cols(W: np.ndarray) -> np.ndarray:
    return W / np.maximum(np.linalg.norm(W, axis=0, keepdims=True), 1e-300)


def _transpose(A):
    if isinstance(A, DistMatrix):
        g = A.redistribute("STAR_VC")
        return DistMatrix(g.local.t().contiguous(), (A.shape[1], A.shape[0]), "VC_STAR", A.comm)
    if isinstance(A, torch.Tensor) and A.is_cuda and A.layout == torch.strided:
        # one transposing copy: the device engines need unit column stride
        return A.t().contiguous()
    return A.t()


# ------------------------------------------------------------ power iteration
def power_iteration(A, V: torch.Tensor, iternum: int, ortho: bool = True, comm: Comm | None = None):
    """``V <- (A^T A)^iternum V`` with optional re-orthonormalisation
    (reference ``PowerIteration(ADJOINT, NORMAL, NORMAL, ...)``).  Returns (U = A V, V)."""
    A_loc, c, _, _ = _as_rowdist(A)
    c = comm or c
    work = torch.float64 if A_loc.dtype == torch.float64 else torch.float32
    from ..ops import tallskinny as T
    U = T.matmul(A_loc, V, out_dtype=work)
    for _ in range(iternum):
        if ortho:
            U = L.orthonormalize(U, c)
        V = L.gemm_tn(A_loc.to(work), U, c)
        if ortho:
            V, _ = torch.linalg.qr(V, mode="reduced")
        U = T.matmul(A_loc, V, out_dtype=work)
    return U, V


def _symm_operator(A, uplo: str, work, comm):
    """``X -> A X`` for a symmetric A of which only the ``uplo`` triangle is
    read (reference ``base::Symm(El::LEFT, uplo, ...)``, base/Symm.hpp; the
    other triangle may hold anything).

    * dense local: the full symmetric matrix is formed once from the triangle;
    * sparse CSR local: entries outside the triangle are dropped, the rest
      mirrored (diagonal once);
    * row-distributed DistMatrix (any layout, redistributed to ``[VC,*]``):
      ``A X = T X + T^T X - D X`` with T the local rows of the triangle; the
      ``T^T X`` part is a partial n x k product on every rank combined by ONE
      reduce-scatter onto the row distribution.  X and the result are
      row-distributed (local rows)."""
    lower = str(uplo).upper().startswith("L")
    if isinstance(A, DistMatrix):
        D = A if A.layout in ("VC_STAR", "VR_STAR") else A.redistribute("VC_STAR")
        r0, r1 = D.row_range()
        n = D.shape[1]
        loc = D.local.to(work)
        rows = torch.arange(r0, r1, device=loc.device)[:, None]
        cols = torch.arange(n, device=loc.device)[None, :]
        T = torch.where((cols <= rows) if lower else (cols >= rows), loc, torch.zeros((), dtype=work, device=loc.device))
        diag = loc[torch.arange(r1 - r0, device=loc.device), torch.arange(r0, r1, device=loc.device)] if r1 > r0 else \
            torch.zeros(0, dtype=work, device=loc.device)
        counts = D.row_counts()

        def mv(Xloc):
            Xfull = D.comm.all_gather_v(Xloc.contiguous(), counts, 0)     # n x k replicated
            part = T.t() @ Xloc                                             # n x k partial
            Tt = D.comm.reduce_scatter_v(part, counts, 0)                   # my rows of T^T X
            return T @ Xfull + Tt - diag[:, None] * Xloc
        return mv, (r0, r1), D
    if A.layout != torch.strided:
        Acoo = A.to_sparse_coo().coalesce() if A.layout != torch.sparse_coo else A.coalesce()
        i, j = Acoo.indices()
        v = Acoo.values().to(work)
        keep = (i >= j) if lower else (i <= j)
        i, j, v = i[keep], j[keep], v[keep]
        off = i != j
        I = torch.cat([i, j[off]])
        J = torch.cat([j, i[off]])
        V = torch.cat([v, v[off]])
        S = torch.sparse_coo_tensor(torch.stack([I, J]), V, A.shape).coalesce().to_sparse_csr()
        return (lambda X: torch.sparse.mm(S, X)), None, None
    Aw = A.to(work)
    T = torch.tril(Aw) if lower else torch.triu(Aw)
    S = T + T.t() - torch.diag(torch.diagonal(Aw))
    return (lambda X: S @ X), None, None


def approximate_symmetric_svd(A, rank: int, context: Context | None = None,
                              params: ApproximateSVDParams | None = None, uplo: str = "L"):
    """Approximate eigendecomposition of a symmetric matrix (reference
    ``ApproximateSymmetricSVD``, ``nla/svd.hpp:321-392``): Gaussian Omega
    (``base::GaussianMatrix``), ``Symm`` power iterations, Rayleigh-Ritz with a
    symmetric eigensolver sorted by SIGNED value, descending (El::DESCENDING).
    Only the ``uplo`` ("L"/"U") triangle of A is read.

    ``A``: dense tensor, sparse CSR/COO tensor, or a DistMatrix (row-sharded
    work, replicated k x k Rayleigh-Ritz).  Returns ``(V, s)``; V is a
    ``[VC,*]`` DistMatrix when A is distributed."""
    from .. import default_context
    from ..base import distributions as D
    from ..ops import rng
    ctx = context if context is not None else default_context()
    params = params or ApproximateSVDParams()
    if A.shape[0] != A.shape[1]:
        raise InvalidParametersError(f"Matrix is not square ({A.shape[0]} x {A.shape[1]}) -- symmetric matrix required")
    n = A.shape[0]
    if rank > n:
        raise InvalidParametersError(f"Incompatible matrix dimensions ({n}) and target rank ({rank}).")
    k = max(rank, min(n, params.oversampling_ratio * rank + params.oversampling_additive))
    if isinstance(A, DistMatrix):
        dtype, dev = A.local.dtype, A.local.device
    else:
        dtype = A.values().dtype if A.layout != torch.strided else A.dtype
        dev = A.device
    work = torch.float64 if dtype == torch.float64 else torch.float32
    comm = A.comm if isinstance(A, DistMatrix) else _LocalComm()
    mv, rr, Dm = _symm_operator(A, uplo, work, comm)
    r0, r1 = rr if rr is not None else (0, n)
    # Omega: global-index Gaussian (identical for every layout / rank count)
    arr = ctx.allocate_random_samples_array(n * k, D.Normal())
    Om = torch.empty(r1 - r0, k, dtype=work, device=dev)
    rng.fill_random(Om, D.Normal(), arr.seed, arr.base, r0=r0, c0=0, ir=1, ic=n)

    def orth(X):
        if Dm is None:
            return torch.linalg.qr(X, mode="reduced")[0]
        return L.orthonormalize(X, comm, method="tsqr")

    V = mv(Om)
    for _ in range(params.num_iterations):
        if not params.skip_qr:
            V = orth(V)
        V = mv(V)
    Q = orth(V)
    U = mv(Q)
    B = Q.t() @ U
    if Dm is not None:
        comm.all_reduce(B)
    B = 0.5 * (B + B.t())
    w, E = torch.linalg.eigh(B.double())
    order = torch.argsort(w, descending=True)[:rank]
    Vr = (Q.double() @ E[:, order].to(Q.device)).to(work)
    s = w[order].to(device=dev, dtype=work)
    if Dm is not None:
        return DistMatrix(Vr.contiguous(), (n, rank), "VC_STAR", comm), s
    return Vr, s


ApproximateSVD = approximate_svd
ApproximateSymmetricSVD = approximate_symmetric_svd
PowerIteration = power_iteration
