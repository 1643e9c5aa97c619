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
from ..base.exceptions import InvalidParametersError
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

    if A_loc.is_cuda and work == torch.float32 and T._native_ok(A_loc, k):
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


class _DevicePlan:
    """Device randSVD for one (A, k, rank, q) configuration, replayed as two
    hipGraphs once warm (``ApproximateSVDParams.graph``).

    Segment 1 (sketch Z -> power passes -> final pass -> fp64 Gram and
    CholeskyQR of Y -> k x k Gram of A^T Q) and segment 2 (V and the k x r
    map of U from the host eigensolve) are each one graph: the ~30 launches
    per call collapse into two replays, so the short kernels between the
    streaming passes no longer wait on host launch latency.  Graph inputs are
    static buffers (the sketch Z and the eigenpairs); A is read in place, so
    replays always see A's current contents.  The small outputs (s, V) are
    cloned out of graph memory; U = Y M is one eager launch into a fresh
    tensor (no m x r copy).  With more than
    one rank segment 1 is split at its all-reduces: each piece is its own
    graph and the collectives run eagerly between the replays (no RCCL
    capture); if a capture fails the plan stays eager.
    """

    def __init__(self, A_loc, comm, n, rank, k, q, skip_qr, use_graph):
        from ..ops import tallskinny as T
        dev = A_loc.device
        m = A_loc.shape[0]
        # weak: a cached plan must not keep a multi-GB operand alive
        self.Aref = weakref.ref(A_loc)
        self.dev = dev
        self.comm, self.n, self.rank, self.k, self.q, self.skip_qr = comm, n, rank, k, q, skip_qr
        self.Zs = torch.empty(n, k, dtype=torch.float32, device=dev)
        # the fused pass's operand in its bf16 k x n layout, written in place by
        # the FJLT realisation and by each CholeskyQR step (no cast/transpose
        # launches between the passes)
        self.Zt = torch.empty(k, n, dtype=torch.bfloat16, device=dev)
        # [W; G] of the final pass, reduced straight into one f64 buffer
        self.WG = torch.empty(n + k, k, dtype=torch.float64, device=dev)
        # FJLT sketches are realised inside segment 1 from device-held stream
        # coordinates {seed, base_D, base_samples} (ops.fut.fjlt_operator)
        self.prm = torch.zeros(3, dtype=torch.int64, device=dev)
        self.prm_host = torch.zeros(3, dtype=torch.int64).pin_memory()
        self.fjlt_scale = None
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.small = torch.zeros(k * rank + rank, dtype=torch.float64, device=dev)
        self.small_host = torch.zeros(k * rank + rank, dtype=torch.float64).pin_memory()
        self.small_np = self.small_host.numpy()
        self.host_pin = self.host_ev = None
        self.ws = torch.empty(T.fused_workspace_bytes(m, n, k), dtype=torch.uint8, device=dev)
        self.ws32 = torch.empty(max(T.f32_workspace_bytes(m), T.f32_workspace_bytes(n)), dtype=torch.uint8,
                                device=dev)
        # k x k eigensolve on the device (sym_eig.hip tridiagonal path): the
        # whole call is then one graph with no host round trip; status bit 1
        # sends that call's eigensolve back to host LAPACK.  Opt-in: measured
        # 178 us for k = 40 (serial f64 division chains on one CU) against
        # ~70 us host LAPACK + ~60 us of round trip (profiles/eig_device_r2.jsonl)
        self.dev_eig = (k <= 64 and rank <= 32 and os.environ.get("SL_SVD_DEVICE_EIG", "0") == "1"
                        and dev.type == "cuda")
        self.eig_status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.use_graph = use_graph
        # alternate row directions across passes (Infinity-Cache reuse; measured
        # no gain: 1.77 vs 1.78 ms)
        self.snake = os.environ.get("SL_SVD_SNAKE", "0") == "1"
        # final pass: fp64 Gram of Y inside the pass (default) or by a separate
        # streaming kernel after a Gram-free pass (SL_SVD_SPLIT_GRAM=1; measured
        # equal under rocprof: 551 + 73 + 10 vs 624 + 5 us)
        self.split_gram = os.environ.get("SL_SVD_SPLIT_GRAM", "0") == "1"
        self.ws32g = torch.empty(T.gram64_workspace_bytes(m, k), dtype=torch.uint8, device=dev) \
            if self.split_gram else None
        self._xm_fn = None
        self._fu_fn = None
        self.g1 = self.g2 = None
        self.piece_graphs = None   # multi-rank: per-piece graphs (False: capture failed)
        self._Wout = [None] * (q + 1)
        self.calls = 0

    # ---- segment 1 as pieces separated by the collectives: with one rank the
    # pieces are captured into one graph; with several, each piece is its own
    # graph and the all-reduces run eagerly between replays, so multi-GPU
    # steps replay ~5 graphs instead of launching ~35 kernels from Python.
    def _piece_pass(self, i):
        from ..ops import small_la as SL
        from ..ops import tallskinny as T
        prof = PROFILER
        A = self.Aref()
        if i == 0:
            self.status.zero_()
            if self.dev_eig:
                self.eig_status.zero_()
            if self.fjlt_scale is not None:
                from ..ops import fut as F
                with prof.phase("svd.sketch"):
                    F.fjlt_operator(self.prm, self.k, self.n, self.fjlt_scale, self.Zt, transpose=False)
            else:
                self.Zt.copy_(self.Zs.t())
            Z = None
        else:
            with prof.phase("svd.orth"):
                # only the subspace matters between passes: one CholeskyQR step
                W = self._Wout[i - 1]
                if self.skip_qr:
                    self.Zt.copy_((W / W.norm(dim=0, keepdim=True).clamp_min(1e-30)).t())
                else:
                    SL.cholqr(W, self.status, ws=self.ws32, zt_out=self.Zt)
                Z = None
        if i < self.q:
            with prof.phase("svd.fused_pass"):
                # every piece writes its own output slot: a piece's capture then
                # reads its predecessor's graph-owned result, never its own warm-up's
                # odd passes walk the rows backwards: each pass starts on the
                # rows the previous one read last (Infinity-Cache resident)
                self._Wout[i], _, _ = T.fused_pass(A, Z, keep_y=False, gram=False, exact=False, ws=self.ws,
                                                   zt=self.Zt, reverse=self.snake and i % 2 == 1)
            return self._Wout[i]
        with prof.phase("svd.fused_pass"):
            # fp64 Gram of the f32 Y on the f64 matrix cores, formed inside the
            # same pass (no second read of Y): one fp64 CholeskyQR then leaves
            # Q = Y R^{-1} orthogonal to ~kappa(Y)^2 eps64 (CholeskyQR2 with an
            # f32 second Gram only reached ~eps32, at three times the work);
            # W (f64) and G land in the [W; G] buffer the all-reduce takes
            if self.split_gram:
                # the pass without its Gram specialisation (~160 us faster at
                # 1e6 x 1e3), then the fp64 Gram of the stored f32 Y by its own
                # streaming kernel (~80 us) straight into [W; G]
                _, _, Y = T.fused_pass(A, Z, keep_y=True, gram=False, exact=True, ws=self.ws, zt=self.Zt,
                                       wg_out=self.WG, reverse=self.snake and i % 2 == 1)
                T.gram64(Y, ws=self.ws32g, out=self.WG[self.n:])
            else:
                _, _, Y = T.fused_pass(A, Z, keep_y=True, gram=True, exact=True, ws=self.ws, gram64=True,
                                       zt=self.Zt, wg_out=self.WG, reverse=self.snake and i % 2 == 1)
        self._WG = self.WG
        self.Y = Y
        return self._WG

    def _piece_core(self):
        from ..ops import small_la as SL
        n = self.n
        W, G = self._WG[:n], self._WG[n:]
        with PROFILER.phase("svd.final_qr"):
            _, Rti, _ = SL.chol_inv(G, self.status)
            # B^T = A^T Q = W Rt^{-1} (n x k); its right singular pairs come from the
            # k x k f64 Gram C = Rt^{-T} (W^T W) Rt^{-1} = Ub S^2 Ub^T (host eigensolve).
            # sigma_i keeps relative accuracy ~eps64 (sigma_1/sigma_i)^2, far below
            # the bf16 data error for every rank the sketch resolves.
            # svd_core.hip: Vt = W Rt^{-1} and the symmetric C, staged with the
            # breakdown status as [C | status] (2 launches)
            Vt, self.host_src = SL.svd_core(W, Rti, self.status)
        self.Rti, self.Vt = Rti, Vt
        if self.dev_eig:
            with PROFILER.phase("svd.eig"):
                SL.sym_eig_tridiag(self.host_src, self.rank, out=self.small, sqrt=True, status=self.eig_status,
                                   ldc=self.k)
            self.seg2()

    def pieces(self):
        """[(graph-able piece, tensor to all-reduce after it or None)]"""
        out = [(lambda i=i: self._piece_pass(i), True) for i in range(self.q + 1)]
        out.append((self._piece_core, False))
        return out

    def seg1(self):
        with PROFILER.phase("svd.allreduce_small"):
            pass
        for fn, reduce_after in self.pieces():
            t = fn()
            if reduce_after:
                with PROFILER.phase("svd.allreduce_small"):
                    self.comm.all_reduce(t)

    def seg2(self):
        from ..ops import small_la as SL
        r = self.rank
        with PROFILER.phase("svd.form_U"):
            # V = A^T Q Ub S^{-1} = Vt Ub S^{-1};  U = Y M with M = Rt^{-1} Ub (one launch)
            self.V, self.M, self.s = SL.svd_finish(self.Vt, self.Rti, self.small, r)

    def _collectives_capturable(self):
        """True once this communicator's one-shot path holds every operand the
        segment all-reduces (set up by the first, eager call)."""
        os_ = getattr(self.comm, "_oneshot", None)
        if not os_ or self.calls < 1:
            return False
        outs = [w for w in self._Wout if w is not None] + [self.WG]
        return all(os_.fits(t) for t in outs)

    def graph_built(self):
        return self.g1 is not None or bool(self.piece_graphs)

    def reset_graphs(self):
        self.g1 = self.g2 = None
        self.piece_graphs = None
        self.calls = 0

    def _finish_u_ok(self):
        Y = self.Y
        return (not PROFILER.enabled and Y is not None and Y.is_cuda and Y.dtype == torch.float32
                and Y.is_contiguous() and self.Vt.is_contiguous() and self.Rti.is_contiguous())

    def _finish_u(self):
        if self._fu_fn is None:
            from ..ops import _lib
            fn = getattr(_lib.require(), "sl_svd_finish_u")
            P, I, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
            fn.argtypes = [P, I, I, P, P, I, P, P, P, P, L, P, P]
            fn.restype = ctypes.c_int
            self._fu_fn = fn
        n, k = self.Vt.shape
        r = self.rank
        m = self.Y.shape[0]
        dev = self.dev
        V = torch.empty(n, r, dtype=torch.float32, device=dev)
        M = torch.empty(k, r, dtype=torch.float32, device=dev)
        s = torch.empty(r, dtype=torch.float32, device=dev)
        U = torch.empty(m, r, dtype=torch.float32, device=dev)
        rc = self._fu_fn(self.Vt.data_ptr(), n, k, self.Rti.data_ptr(), self.small.data_ptr(), r, V.data_ptr(),
                         M.data_ptr(), s.data_ptr(), self.Y.data_ptr(), m, U.data_ptr(),
                         torch.cuda.current_stream(dev).cuda_stream)
        if rc != 0:
            from ..ops import _lib
            _lib.call("sl_svd_finish", _lib.ptr(self.Vt), n, k, _lib.ptr(self.Rti), _lib.ptr(self.small), r,
                      _lib.ptr(V), _lib.ptr(M), _lib.ptr(s), ctypes.c_void_p(_lib.stream_of(V)))
            from ..ops import tallskinny as T
            U = T.f32_xm(self.Y, M, store=True)[0]
        return U, s, V

    def _form_u(self):
        """U = Y M (m x r f32) with the launch arguments bound once: this launch
        sits between the second replay and the end of the call, so its
        Python overhead is on the critical path (~25 -> ~8 us)."""
        from ..ops import tallskinny as T
        Y, M = self.Y, self.M
        if not (Y.is_cuda and Y.is_contiguous() and M.is_contiguous() and M.dtype == torch.float32):
            return T.f32_xm(Y, M, store=True)[0]
        if self._xm_fn is None:
            from ..ops import _lib
            T.f32_xm  # noqa: B018 - registers the signature
            fn = getattr(_lib.require(), "sl_tsk_f32_xm")
            if fn.argtypes is None:
                fn.argtypes = _lib.SIGNATURES["sl_tsk_f32_xm"]
                fn.restype = ctypes.c_int
            self._xm_fn = fn
        m, k = Y.shape
        r = M.shape[1]
        U = torch.empty(m, r, dtype=torch.float32, device=self.dev)
        rc = self._xm_fn(Y.data_ptr(), m, k, k, M.data_ptr(), r, U.data_ptr(), r, None, None,
                         torch.cuda.current_stream(self.dev).cuda_stream)
        if rc != 0:
            return T.f32_xm(Y, M, store=True)[0]
        return U

    def _capture(self, fn, want_out=False):
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # thread-local capture: with RCCL the process group's watchdog thread
        # polls events concurrently, which a global-mode capture would reject
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            out = fn()
        return (g, out) if want_out else g

    def _run(self, which):
        fn = self.seg1 if which == 1 else self.seg2
        g = self.g1 if which == 1 else self.g2
        warm = self.use_graph and self.calls >= 1 and not PROFILER.enabled
        if which == 1 and self.comm.size > 1 and self._collectives_capturable():
            # every all-reduce of segment 1 is the one-shot kernel
            # (parallel/oneshot.py): the whole segment, collectives included,
            # is one graph, as with a single rank
            pass
        elif which == 1 and self.comm.size > 1 and self.piece_graphs is not False:
            # multi-rank: one graph per piece, eager collectives in between
            if self.piece_graphs is None and warm:
                try:
                    self.piece_graphs = [(*self._capture(f, want_out=True), r) for f, r in self.pieces()]
                except Exception:  # noqa: BLE001 - capture unsupported here: stay eager
                    self.piece_graphs = False
            if self.piece_graphs:
                for gp, out, reduce_after in self.piece_graphs:
                    gp.replay()
                    if reduce_after:
                        with PROFILER.phase("svd.allreduce_small"):
                            self.comm.all_reduce(out)
                return
            fn()
            return
        if g is None and warm:
            try:
                g = self._capture(fn)
            except Exception:  # noqa: BLE001 - capture unsupported here: stay eager
                self.use_graph, g = False, None
            if which == 1:
                self.g1 = g
            else:
                self.g2 = g
        if g is not None:
            g.replay()
        else:
            fn()

    def __call__(self, Z=None, fjlt=None):
        """``Z``: realised sketch operator (n x k), or ``fjlt`` = (seed, base_D,
        base_samples, scale) to realise an FJLT inside the graph."""
        if fjlt is not None:
            if self.fjlt_scale is None and self.graph_built():
                self.reset_graphs()
            self.fjlt_scale = float(fjlt[3])
            # pinned + non_blocking (no host wait): the previous call's copy of
            # this buffer finished before that call's synchronising D2H
            self.prm_host[0], self.prm_host[1], self.prm_host[2] = int(fjlt[0]), int(fjlt[1]), int(fjlt[2])
            self.prm.copy_(self.prm_host, non_blocking=True)
        else:
            if self.fjlt_scale is not None:
                self.fjlt_scale = None
                self.reset_graphs()
            self.Zs.copy_(Z)
        tr = _TRACE and [time.perf_counter()]
        self._run(1)
        if self.dev_eig:
            from ..ops import tallskinny as T
            with PROFILER.phase("svd.form_U"):
                U, _ = T.f32_xm(self.Y, self.M, store=True)
            if not int(self.eig_status.item()):
                self.calls += 1
                if tr:
                    tr.append(time.perf_counter())
                    print(f"[svd.trace] device_eig call={(tr[1] - tr[0]) * 1e6:.0f}us", file=sys.stderr)
                return U, self.s.clone(), self.V.clone()
            # flagged (near-repeated eigenvalues, non-finite data or a vanishing
            # r-th eigenvalue): this call's k x k eigensolve goes to host LAPACK
        tr and tr.append(time.perf_counter())
        # [C | status] into a pinned buffer; wait for that copy only
        if self.host_pin is None:
            self.host_pin = torch.empty(self.host_src.numel(), dtype=torch.float64).pin_memory()
            self.host_np = self.host_pin.numpy()
            self.host_ev = torch.cuda.Event()
        self.host_pin.copy_(self.host_src, non_blocking=True)
        self.host_ev.record()
        self.host_ev.synchronize()
        host = self.host_pin
        tr and tr.append(time.perf_counter())
        k, r = self.k, self.rank
        # host[-1] != 0: a CholeskyQR pivot was dropped (rank-deficient block --
        # e.g. an FJLT that sampled the same row twice, or a low-rank A); the
        # dropped direction is an exactly-zero column from then on, harmless
        # while at least r directions survive.  Non-finite data or fewer than
        # r surviving directions send the call to the robust host path.
        # numpy views of the pinned buffers: no torch dispatch on this path
        Cm = self.host_np[:k * k].reshape(k, k)
        if not np.isfinite(Cm).all():
            return None
        # C is exactly symmetric (svd_core.hip); eigh returns ascending eigenpairs
        got = _host_eigh_np(Cm)
        if got is None:
            return None
        evals, evecs = got
        if not evals[k - r] > 1e-30 * max(evals[-1], 1e-300):
            return None
        pin = self.small_np
        pin[:k * r].reshape(k, r)[:] = evecs[:, ::-1][:, :r]
        np.sqrt(np.maximum(evals[::-1][:r], 0.0), out=pin[k * r:])
        tr and tr.append(time.perf_counter())
        # pinned + non_blocking: the copy is ordered on the stream, the host
        # does not wait (the buffer is rewritten only after the next call's
        # synchronising D2H, which follows this copy in stream order)
        self.small.copy_(self.small_host, non_blocking=True)
        tr and tr.append(time.perf_counter())
        from ..ops import small_la as SL
        from ..ops import tallskinny as T
        if self.dev_eig:
            # eager, into fresh tensors: the graph's own V / M / s buffers stay
            # bound to the device-eigensolver variant captured in segment 1
            V, M, s = SL.svd_finish(self.Vt, self.Rti, self.small, r)
            U, _ = T.f32_xm(self.Y, M, store=True)
            self.calls += 1
            return U, s, V
        if self._finish_u_ok():
            # V, M, s and U = Y M into fresh tensors from ONE host call (two
            # launches): no second graph replay, no clones out of graph memory
            out = self._finish_u()
            tr and tr.append(time.perf_counter())
            self.calls += 1
        else:
            self._run(2)
            tr and tr.append(time.perf_counter())
            self.calls += 1
            with PROFILER.phase("svd.form_U"):
                # outside the graph: U lands in a fresh allocation, so the m x r
                # result needs no copy out of the graph's static memory
                U = self._form_u()
            out = U, self.s.clone(), self.V.clone()
        if tr:
            tr.append(time.perf_counter())
            names = ["replay1", "d2h_sync", "eigh", "h2d", "replay2", "form_U"]
            print("[svd.trace] " + " ".join(f"{n}={(b - a) * 1e6:.0f}us" for n, a, b in zip(names, tr, tr[1:])),
                  file=sys.stderr)
        return out


_EIG_BACKEND = os.environ.get("SL_HOST_EIG", "torch")


def _host_eigh_np(C: np.ndarray):
    """(w ascending, V) of a small symmetric f64 matrix (numpy in / out), or
    None on a LAPACK failure.  ``SL_HOST_EIG`` picks the LAPACK route:
    "torch" (single-threaded torch.linalg.eigh on a zero-copy view, the
    measured fastest), "scipy" (dsyevd through scipy.linalg.lapack) or
    "numpy"."""
    if _EIG_BACKEND == "scipy":
        from scipy.linalg import lapack
        w, v, info = lapack.dsyevd(C, compute_v=1, lower=0)
        return (w, v) if info == 0 else None
    if _EIG_BACKEND == "numpy":
        return np.linalg.eigh(C)
    w, v = _host_eigh(torch.from_numpy(C))
    return w.numpy(), v.numpy()


def _host_eigh(C: torch.Tensor):
    """LAPACK eigh of the k x k core on ONE host thread: for k ~ 40 the
    threaded BLAS costs 2-4x more than it saves (measured 177 us single
    threaded vs 290-700 us threaded on the build host).  A device Jacobi
    (ops.small_la.sym_eig_topr) was measured at ~500 us for k = 40, so the
    host solve stays on the randSVD critical path."""
    n = torch.get_num_threads()
    if n == 1:
        return torch.linalg.eigh(C)
    torch.set_num_threads(1)
    try:
        return torch.linalg.eigh(C)
    finally:
        torch.set_num_threads(n)


_PLANS: dict = {}
_TRACE = os.environ.get("SKH_TRACE_SVD", "0") == "1"   # host-side phase timestamps
_T0 = [0.0]


def _approximate_svd_device(A_loc, comm, m, n, rank, k, ctx, params):
    """GPU-resident path (bf16 A on gfx950): every iteration stays on the device;
    one host synchronisation per call (the k x k eigensolve + status check).

    Returns None when a Cholesky breakdown was flagged (the caller then reruns
    the robust host path with the same, rewound, context)."""
    if _TRACE:
        print(f"[svd.trace] python_prep={(time.perf_counter() - _T0[0]) * 1e6:.0f}us", file=sys.stderr)
    ctx0 = ctx.copy()
    dev = A_loc.device
    fjlt = None
    if params.sketch.upper() == "FJLT":
        # FJLT_data draw layout: N Rademacher signs, then S sample rows; the
        # operator itself is realised on the device inside the plan's graph
        base_d = ctx.counter
        base_s = base_d + n
        ctx.counter = base_s + k
        fjlt = (ctx.seed, base_d, base_s, math.sqrt(n / k))
        Z = None
    else:
        with PROFILER.phase("svd.sketch"):
            Z = _sketch_operator(params.sketch, n, k, ctx, dev, torch.float32)
    q = max(0, int(params.num_iterations))
    key = (A_loc.data_ptr(), tuple(A_loc.shape), tuple(A_loc.stride()), A_loc.dtype, str(dev), rank, k, q,
           bool(params.skip_qr), comm.size, id(getattr(comm, "group", None)))
    plan = _PLANS.get(key)
    if plan is not None and plan.Aref() is None:
        plan = None  # the operand this plan was built for is gone
    if plan is None:
        if len(_PLANS) >= 4:
            _PLANS.pop(next(iter(_PLANS)))
        # multi-rank: capture collectives only on request — a capture that fails on
        # one rank but not another would desynchronise the collectives
        use_graph = bool(params.graph) and dev.type == "cuda"
        plan = _DevicePlan(A_loc, comm, n, rank, k, q, params.skip_qr, use_graph)
        _PLANS[key] = plan
    res = plan(Z, fjlt=fjlt)
    if res is None:
        ctx.seed, ctx.counter = ctx0.seed, ctx0.counter
    return res


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
