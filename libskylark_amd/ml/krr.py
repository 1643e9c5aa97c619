"""Kernel ridge regression family (reference ``ml/krr.hpp:8-732``).

All solvers take data points as ROWS (``X`` n x d, ``Y`` n x t targets);
``direction="columns"`` accepts the reference's d x n layout.  ``X``/``Y`` may
be local tensors or row-distributed ([VC,*]) DistMatrices: every rank then
holds a block of examples and the only collectives are all-reduces of
feature-space quantities (s x s, s x t) or all-gathers of n x t direction
blocks, sized for xGMI (few, large messages).

* :func:`kernel_ridge` — exact: ``(K + lambda I) A = Y`` via Cholesky (``:49-90``).
* :func:`approximate_kernel_ridge` — random features ``Z = S(X)``, optional
  CWT/FJLT sketch of the regression, ridge solve (``:94-196``).
* :func:`sketched_approximate_kernel_ridge` — features generated piecemeal
  (<= max_split/2 at a time) and each sketched immediately (``:199-309``).
* :class:`FeatureMapPrecond` + :func:`faster_kernel_ridge` — CG on
  ``K + lambda I`` with the Woodbury random-feature preconditioner
  ``P = (U^T U + lambda I)^{-1}`` (``:312-540``).
* :func:`large_scale_kernel_ridge` — block coordinate descent over feature
  blocks with per-block Cholesky factors (``:546-730``).  The reference trains
  on UNSCALED blocks yet marks the model ``scale_maps=true``; here the blocks
  are scaled by ``sqrt(s_j / s)`` in training too, so training and the
  model's prediction agree.
"""
from __future__ import annotations

import ctypes as C
import os

import math
from dataclasses import dataclass

import torch

from ..algorithms.krylov import CallablePrecond, IdPrecond, KrylovIterParams, cg
from ..algorithms.operators import DenseOp, DistSymOp
from ..base.context import Context
from ..parallel.comm import Comm
from ..parallel.distmatrix import DistMatrix
from .. import sketch as SK
from .kernels import Kernel, _dir, _points


@dataclass
class KrrParams:
    am_i_printing: bool = False
    log_level: int = 0
    prefix: str = ""
    debug_level: int = 0
    use_fast: bool = False
    sketched_rr: bool = False
    sketch_size: int = -1
    fast_sketch: bool = False
    iter_lim: int = 1000
    res_print: int = 10
    tolerance: float = 1e-3
    max_split: int = 0
    precond_f32: bool = True   # GPU: apply the feature-map preconditioner in f32 single-read passes
    # FasterKernelRidge preconditioner: "features" (the reference's random-
    # feature Woodbury form, feature_map_precond_t) or "nystrom" (s landmark
    # columns of the Gram the solver holds; converges at small lambda where
    # the random-feature approximation error ||K - U U^T|| / lambda does not)
    precond: str = "features"


krr_params_t = KrrParams


def _log(p, lvl, msg):
    if p.am_i_printing and p.log_level >= lvl:
        print(f"{p.prefix}{msg}", flush=True)


class _Data:
    """Row-major local example block + communicator for X/Y inputs."""

    def __init__(self, X, direction):
        if isinstance(X, DistMatrix):
            D = X if X.layout in ("VC_STAR", "VR_STAR") else X.redistribute("VC_STAR")
            if _dir(direction) != "rows":
                D = DistMatrix(D.to_global().t().contiguous(), (D.shape[1], D.shape[0]), "STAR_STAR",
                               D.comm).redistribute("VC_STAR")
            self.local, self.comm, self.n, self.D = D.local, D.comm, D.shape[0], D
        else:
            self.local, self.comm, self.D = _points(X, direction), Comm.single(), None
            self.n = self.local.shape[0]
        self.distributed = self.comm.size > 1

    def rows_of(self, Y, direction="rows"):
        """Local row block of targets ``Y`` (given globally, locally or distributed)."""
        if isinstance(Y, DistMatrix):
            return Y.redistribute("VC_STAR").local if Y.layout != "VC_STAR" else Y.local
        Y = Y if isinstance(Y, torch.Tensor) else torch.as_tensor(Y)
        if Y.dim() == 1:
            Y = Y[:, None]
        if self.D is not None and Y.shape[0] == self.n and self.local.shape[0] != self.n:
            s, e = self.D.row_range()
            Y = Y[s:e]
        return Y.to(self.local.device)

    def allreduce(self, t):
        if self.distributed:
            self.comm.all_reduce(t)
        return t


SPLIT_GRAM_ROWS = 8192   # rows per f32-accumulated chunk of the split Gram
# row blocks of the split Gram's block-upper-triangle form (1: the full s x s
# products, the default); env SKH_KRR_GRAM_BLOCKS for A/Bs -- 2 / 4 / 8 blocks
# cut the flops to 75 / 62 / 56% but ran 0.193 / 0.243 / 0.336 s against 0.190
# (profiles/r6/krr_gram_blocks_ab.jsonl: the narrower products run far slower)
SPLIT_GRAM_BLOCKS = int(os.environ.get("SKH_KRR_GRAM_BLOCKS", "1"))


def _split3(Zc: torch.Tensor):
    """f32 -> three bf16 planes with H + M + L == Zc exactly (8 + 8 + 8
    mantissa bits; values whose low parts underflow bf16's range lose them)."""
    H = Zc.to(torch.bfloat16)
    r = Zc - H.float()
    Mp = r.to(torch.bfloat16)
    L = (r - Mp.float()).to(torch.bfloat16)
    return H, Mp, L


def _gram_split(Z: torch.Tensor, G: torch.Tensor) -> None:
    """G += Z^T Z for f32 Z on the GPU from exact bf16 products on the matrix
    cores: Z = H + M + L (bf16 planes), Z^T Z = H^T H + M^T M + (H^T M + M^T H)
    + (H^T L + L^T H) up to the M L / L L terms (< 2^-32 of |z|^2).  Per row
    chunk one kernel (gemm_nt.hip k_split3_t) writes the planes transposed
    and stacked, S = [L | H | M | H | L] (s x 5 R), and two NT GEMMs on
    windows of S give [H M][H M]^T + [H M H L][L H M H]^T (hipBLASLt NT: 1.16-
    1.44 PF on these shapes against 0.91-1.10 for the TN form of row-major
    planes, profiles/r6/gemm_orient_ab.json).  Every product is exact in f32;
    the sums are f32 within a chunk of SPLIT_GRAM_ROWS rows (relative error
    ~2^-24 sqrt(4 x rows) of sum |z_i z_j|, ~1e-5 -- the level of the f32
    feature map's own rounding) and f64 across chunks."""
    from ..ops import _lib
    n, s = Z.shape
    R = SPLIT_GRAM_ROWS
    if not _lib.available() or Z.stride(1) != 1:
        for r0 in range(0, n, R):
            H, Mp, L = _split3(Z[r0:r0 + R])
            A1 = torch.cat([H, Mp])
            Cm = torch.mm(A1.t(), A1, out_dtype=torch.float32)
            Cm += torch.mm(torch.cat([H, Mp, H, L]).t(), torch.cat([L, H, Mp, H]), out_dtype=torch.float32)
            G += Cm.double()
        return
    _lib.register("sl_split3_bf16_t", [C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_void_p, C.c_int, C.c_int64,
                                       C.c_void_p])
    seg = -(-min(R, n) // 64) * 64
    S = torch.empty(s, 5 * seg, dtype=torch.bfloat16, device=Z.device)
    st = C.c_void_p(_lib.stream_of(Z))
    # both window products are symmetric: with nb > 1 only the block upper
    # triangle (row block b against columns b.. of the s x s result) is
    # formed, (nb + 1) / 2nb of the flops, and mirrored once at the end
    nb = SPLIT_GRAM_BLOCKS if s % SPLIT_GRAM_BLOCKS == 0 and (s // SPLIT_GRAM_BLOCKS) % 64 == 0 else 1
    bs = s // nb
    Gu = torch.zeros_like(G) if nb > 1 else G
    for r0 in range(0, n, R):
        w = min(R, n - r0)
        _lib.call("sl_split3_bf16_t", _lib.ptr(Z[r0:]), w, s, Z.stride(0), _lib.ptr(S), seg, 5 * seg, st)
        A = S[:, seg:3 * seg]
        B1, B2 = S[:, seg:5 * seg], S[:, :4 * seg]
        if nb == 1:
            Cm = torch.mm(A, A.t(), out_dtype=torch.float32)
            Cm += torch.mm(B1, B2.t(), out_dtype=torch.float32)
            G += Cm.double()
            continue
        for b in range(nb):
            rb, cb = slice(b * bs, (b + 1) * bs), slice(b * bs, s)
            Cm = torch.mm(A[rb], A[cb].t(), out_dtype=torch.float32)
            Cm += torch.mm(B1[rb], B2[cb].t(), out_dtype=torch.float32)
            Gu[rb, cb] += Cm.double()
    if nb > 1:
        G += torch.triu(Gu) + torch.triu(Gu, 1).t()


def _ridge(Z: torch.Tensor, Y: torch.Tensor, lam: float, data: _Data | None = None) -> torch.Tensor:
    """W = argmin |Z W - Y|^2 + lam |W|^2 via the s x s normal equations in
    fp64 (reference ``El::Ridge``); distributed Z: all-reduce [Z^T Z | Z^T Y].
    f32 Z on the GPU: Z^T Z from exact split products (:func:`_gram_split`)
    and Z^T Y from one streaming pass (f32); otherwise fp64 products and sums."""
    s = Z.shape[1]
    t = Y.shape[1] if Y.dim() > 1 else 1
    Y2 = Y if Y.dim() > 1 else Y[:, None]
    # [Z^T Z | Z^T Y] accumulated in fp64 over row chunks: no n x s fp64 copy
    # of Z (32 GB for 1e6 x 4096 features), same fp64 products and sums
    G = torch.zeros(s, s + t, dtype=torch.float64, device=Z.device)
    split = Z.is_cuda and Z.dtype == torch.float32 and os.environ.get("SKH_KRR_F64_GRAM", "0") != "1"
    from ..ops import normal_eq
    if split:
        Gzz = torch.zeros(s, s, dtype=torch.float64, device=Z.device)
        _gram_split(Z, Gzz)
        G[:, :s] = Gzz
    if split and normal_eq.native_ok(Z, t) and Y2.shape[0] == Z.shape[0]:
        # Z^T Y from one streaming read of Z (ata_kernels.hip dual pass: f32
        # products and block sums) -- the fp64 chunk copies of Z took ~40 ms
        G[:, s:] = normal_eq.dual(Z, Y2.to(torch.float32).contiguous())[0].double()
    else:
        chunk = max(1, (1 << 27) // max(1, s + t))
        for r0 in range(0, Z.shape[0], chunk):
            Zc = Z[r0:r0 + chunk].to(torch.float64)
            if not split:
                G[:, :s].addmm_(Zc.t(), Zc)
            G[:, s:].addmm_(Zc.t(), Y2[r0:r0 + chunk].to(torch.float64))
    if data is not None:
        data.allreduce(G)
    C = G[:, :s]
    C.diagonal().add_(lam)
    Lc = torch.linalg.cholesky(C)
    return torch.cholesky_solve(G[:, s:], Lc)


def _features(S, Xl: torch.Tensor) -> torch.Tensor:
    """Rowwise feature map of the local example block (n_loc x s)."""
    return S.apply(Xl, dim=SK.ROWWISE)


def kernel_ridge(k: Kernel, X, Y, lam: float, direction="rows", params: KrrParams | None = None) -> torch.Tensor:
    """Exact KRR: returns A (n x t) with ``(K + lam I) A = Y``.  Distributed X:
    each rank builds its [VC,*] row block of K; the n x n system is gathered
    and factored (Cholesky on one GPU per rank; exact KRR is O(n^3) anyway —
    use :func:`faster_kernel_ridge` for large n)."""
    p = params or KrrParams()
    data = _Data(X, direction)
    _log(p, 1, "Computing kernel matrix...")
    if data.distributed:
        Kd = k.gram(data.D)
        K = Kd.to_global()
        Yg = data.comm.all_gather_v(data.rows_of(Y).contiguous(), data.D.row_counts())
    else:
        K = k.symmetric_gram(data.local)
        Yg = data.rows_of(Y)
    dt = torch.float64
    K = K.to(dt)
    K.diagonal().add_(lam)
    _log(p, 1, "Solving the equation...")
    Lc = torch.linalg.cholesky(K)
    A = torch.cholesky_solve(Yg.to(dt), Lc)
    return A


def approximate_kernel_ridge(k: Kernel, X, Y, lam: float, s: int, context: Context | None = None,
                             direction="rows", params: KrrParams | None = None):
    """Random-feature ridge: returns ``(S, W)`` with the feature transform and
    the s x t weights.  ``params.sketched_rr`` sketches the n x s problem with
    FJLT (or CWT if ``fast_sketch``) of size ``sketch_size`` (default 4s)."""
    from .. import default_context
    ctx = context or default_context()
    p = params or KrrParams()
    data = _Data(X, direction)
    _log(p, 1, "Create and apply the feature transform...")
    S = k.create_rft(s, fast=p.use_fast, context=ctx)
    Z = _features(S, data.local)
    Yl = data.rows_of(Y).to(Z.dtype)
    if p.sketched_rr:
        _log(p, 1, "Sketching the regression problem...")
        t = 4 * s if p.sketch_size == -1 else p.sketch_size
        R = (SK.CWT if p.fast_sketch else SK.FJLT)(data.n, t, context=ctx)
        Z, Yl = _sketch_rows(R, Z, Yl, data)
        data = None
    _log(p, 1, "Solving the regression problem...")
    W = _ridge(Z, Yl, lam, data)
    return S, W


def _sketch_rows(R, Z, Yl, data: _Data):
    """Columnwise sketch of [Z Y] (n x (s+t)) -> t x (s+t), replicated on every rank."""
    ZY = torch.cat([Z, Yl.to(Z.dtype)], dim=1)
    if data.distributed:
        D = DistMatrix(ZY.contiguous(), (data.n, ZY.shape[1]), "VC_STAR", data.comm)
        SZY = R.apply(D, dim=SK.COLUMNWISE)
        SZY = SZY.to_global() if isinstance(SZY, DistMatrix) else SZY
    else:
        SZY = R.apply(ZY, dim=SK.COLUMNWISE)
    return SZY[:, :Z.shape[1]], SZY[:, Z.shape[1]:]


def _feature_blocks(k: Kernel, s: int, d: int, p: KrrParams, ctx: Context):
    sinc = d if p.max_split == 0 else max(1, p.max_split // 2)
    maps, remains = [], s
    while remains > 0:
        thiss = remains if remains <= 2 * sinc else sinc
        maps.append(k.create_rft(thiss, fast=p.use_fast, context=ctx))
        remains -= thiss
    return maps


def sketched_approximate_kernel_ridge(k: Kernel, X, Y, lam: float, s: int, t: int = -1,
                                      context: Context | None = None, direction="rows",
                                      params: KrrParams | None = None):
    """Memory-limited approximate KRR: features are produced in blocks of at
    most ``max_split/2`` and each block is sketched (FJLT or CWT, size t)
    immediately, so the n x s feature matrix is never materialised.
    Returns ``(scale_maps=True, transforms, W)``."""
    from .. import default_context
    ctx = context or default_context()
    p = params or KrrParams()
    data = _Data(X, direction)
    t = 4 * s if t == -1 else t
    R = (SK.CWT if p.fast_sketch else SK.FJLT)(data.n, t, context=ctx)
    Yl = data.rows_of(Y)
    maps = _feature_blocks(k, s, k.get_dim(), p, ctx)
    SZ_blocks = []
    SY = None
    for j, S in enumerate(maps):
        Z = _features(S, data.local) * math.sqrt(S.get_S() / s)
        SZj, SYj = _sketch_rows(R, Z, Yl if j == 0 else Yl[:, :0], data)
        if j == 0:
            SY = SYj
        SZ_blocks.append(SZj)
    SZ = torch.cat(SZ_blocks, dim=1)
    W = _ridge(SZ, SY, lam, None)
    return True, maps, W


class FeatureMapPrecond:
    """Woodbury preconditioner for ``K + lam I`` from ``s`` random features
    (reference ``feature_map_precond_t`` ``krr.hpp:312-449``):
    ``U = S(X)`` (n x s),  ``C = I + U^T U / lam = L L^T``,
    ``V = U L^{-T} / lam``;  ``apply(B) = B / lam - V (V^T B)`` — two GEMMs
    (plus one s x t all-reduce when the examples are distributed)."""

    is_id = False

    def __init__(self, k: Kernel, lam: float, X, s: int, context: Context | None = None,
                 direction="rows", params: KrrParams | None = None, data: _Data | None = None):
        from .. import default_context
        ctx = context or default_context()
        p = params or KrrParams()
        self.data = data or _Data(X, direction)
        self.lam = float(lam)
        S = k.create_rft(s, fast=p.use_fast, context=ctx)
        U = _features(S, self.data.local).to(torch.float64)
        C = U.t() @ U
        self.data.allreduce(C)
        C = C / self.lam
        C.diagonal().add_(1.0)
        Lc = torch.linalg.cholesky(C)
        # V = U L^{-T} / lam   (n_loc x s)
        self.V = torch.linalg.solve_triangular(Lc, U.t(), upper=False).t() / self.lam
        # on the GPU the application runs in f32 on two single-read passes
        # (V^T B by the one-pass dual kernel, V (V^T B) by the streaming
        # GEMV): it is a preconditioner, so f32 only changes the iterates'
        # path, not the solution CG converges to; the f64 V^T B the library
        # ran as a Tensile GEMM of one column took 2.9 ms at n = 1e5, s = 512
        self._v32 = None
        if self.V.is_cuda and getattr(p, "precond_f32", True):
            from ..ops import normal_eq
            V32 = self.V.to(torch.float32).contiguous()
            if normal_eq.native_ok(V32, 1) and normal_eq.gemv_ok(V32, 1):
                self._v32 = V32

    def apply(self, B):
        if (self._v32 is not None and B.is_cuda and B.dtype == torch.float32 and B.dim() == 2
                and B.shape[1] in (1, 2, 4)):
            from ..ops import normal_eq
            Bf = B.to(torch.float32).contiguous()
            VB = normal_eq.dual(self._v32, Bf)[0]      # s x t
            if self.data is not None:
                self.data.allreduce(VB)
            return (Bf / self.lam - normal_eq.gemv(self._v32, VB)).to(B.dtype)
        VB = self.V.t() @ B.to(self.V.dtype)
        if self.data is not None:
            self.data.allreduce(VB)
        # (lam I + U U^T)^{-1} B = B / lam - U C^{-1} U^T B / lam^2 = B / lam - V V^T B
        return (B.to(self.V.dtype) / self.lam - self.V @ VB).to(B.dtype)

    apply_adjoint = apply


feature_map_precond_t = FeatureMapPrecond


class NystromPrecond(FeatureMapPrecond):
    """Woodbury preconditioner for ``K + lam I`` from ``s`` landmark columns
    of the Gram itself (Nystrom): ``U = K[:, L]`` (L: s examples sampled
    without replacement from the context's stream), ``W = K[L, L]``,
    ``(lam I + U W^{-1} U^T)^{-1} B = B / lam - V V^T B`` with ``lam W + U^T U
    = L L^T`` and ``V = U L^{-T} / sqrt(lam)``.  The random-feature form
    approximates K to O(n / sqrt(s)) in norm, so at small lam its
    preconditioned condition number ``1 + ||K - U U^T|| / lam`` stays large
    (lam = 1e-2 stalls at 1000 iterations); the Nystrom
    error is the Gram's own spectral tail.  ``Kl``: the solver's local rows
    of ``K + lam I`` (n_loc x n), ``row0``: their first global row."""

    def __init__(self, Kl: torch.Tensor, lam: float, s: int, n: int, row0: int = 0,
                 context: Context | None = None, params: KrrParams | None = None, data: _Data | None = None):
        from .. import default_context
        from ..sketch.fjlt import _fisher_yates_prefix
        ctx = context or default_context()
        p = params or KrrParams()
        self.data = data
        self.lam = float(lam)
        s = min(int(s), n)
        idx = torch.as_tensor(_fisher_yates_prefix(ctx, n, s), dtype=torch.long)
        idx_d = idx.to(Kl.device)
        U = Kl.index_select(1, idx_d).to(torch.float64)        # n_loc x s, lam on the landmark rows
        nl = Kl.shape[0]
        loc = (idx >= row0) & (idx < row0 + nl)
        li = torch.nonzero(loc).flatten()
        if li.numel():
            rows = (idx[li] - row0).to(Kl.device)
            U[rows, li.to(Kl.device)] -= self.lam                # K itself, not K + lam I
        Wb = torch.zeros(s, s, dtype=torch.float64, device=Kl.device)
        if li.numel():
            Wb[li.to(Kl.device)] = U[(idx[li] - row0).to(Kl.device)]
        M = U.t() @ U
        if data is not None:
            data.allreduce(Wb)
            data.allreduce(M)
        M += self.lam * 0.5 * (Wb + Wb.t())
        # a landmark pair at (numerically) the same point leaves W singular;
        # lam W + U^T U stays SPD up to rounding -- a relative jitter covers it
        M.diagonal().add_(1e-12 * float(M.diagonal().abs().max()))
        Lc = torch.linalg.cholesky(M)
        self.V = torch.linalg.solve_triangular(Lc, U.t(), upper=False).t() / math.sqrt(self.lam)
        self._v32 = None
        if self.V.is_cuda and getattr(p, "precond_f32", True):
            from ..ops import normal_eq
            V32 = self.V.to(torch.float32).contiguous()
            if normal_eq.native_ok(V32, 1) and normal_eq.gemv_ok(V32, 1):
                self._v32 = V32


def faster_kernel_ridge(k: Kernel, X, Y, lam: float, s: int, context: Context | None = None,
                        direction="rows", params: KrrParams | None = None) -> torch.Tensor:
    """CG on ``(K + lam I) A = Y`` preconditioned by :class:`FeatureMapPrecond`
    (``s == 0``: no preconditioner).  Returns the local row block of A."""
    p = params or KrrParams()
    data = _Data(X, direction)
    _log(p, 1, "Computing kernel matrix...")
    if data.distributed:
        Kd = k.gram(data.D)
        Kd.local.diagonal(offset=data.D.row_range()[0]).add_(lam)
        op = DistSymOp(Kd)
    else:
        K = k.symmetric_gram(data.local)
        K.diagonal().add_(lam)
        op = DenseOp(K)
    _log(p, 1, "Creating preconditioner...")
    if s == 0:
        P = IdPrecond()
    elif p.precond == "nystrom":
        Kl = Kd.local if data.distributed else K
        r0 = data.D.row_range()[0] if data.distributed else 0
        P = NystromPrecond(Kl, lam, s, data.n, r0, context, params=p, data=data if data.distributed else None)
    else:
        P = FeatureMapPrecond(k, lam, None, s, context, params=p, data=data)
    Yl = data.rows_of(Y).to(op.dtype)
    kp = KrylovIterParams(tolerance=p.tolerance, iter_lim=p.iter_lim, res_print=p.res_print,
                          am_i_printing=p.am_i_printing, log_level=p.log_level - 1, prefix=p.prefix + "\t")
    A, _ = cg(op, Yl, params=kp, M=P)
    return A


def large_scale_kernel_ridge(k: Kernel, X, Y, lam: float, s: int, context: Context | None = None,
                             direction="rows", params: KrrParams | None = None):
    """Block coordinate descent over feature blocks.  Returns
    ``(scale_maps=True, transforms, W)`` with W s x t."""
    from .. import default_context
    ctx = context or default_context()
    p = params or KrrParams()
    data = _Data(X, direction)
    maps = _feature_blocks(k, s, k.get_dim(), p, ctx)
    Yl = data.rows_of(Y).to(torch.float64)
    t = Yl.shape[1]
    W = torch.zeros(s, t, dtype=torch.float64, device=Yl.device)
    Rr = Yl.clone()
    offs, o = [], 0
    for S in maps:
        offs.append(o)
        o += S.get_S()
    # features are regenerated each sweep (memory-limited design of the
    # reference); cache them when they fit
    cache = {}
    budget = 1 << 31
    factors = []

    def Zof(j):
        if j in cache:
            return cache[j]
        Z = (_features(maps[j], data.local) * math.sqrt(maps[j].get_S() / s)).to(torch.float64)
        if Z.numel() * 8 * (len(cache) + 1) < budget:
            cache[j] = Z
        return Z

    for it in range(max(1, p.iter_lim)):
        delsize = 0.0
        for j, S in enumerate(maps):
            Z = Zof(j)
            if it == 0:
                C = Z.t() @ Z
                data.allreduce(C)
                C.diagonal().add_(lam)
                factors.append(torch.linalg.cholesky(C))
            W0 = W[offs[j]:offs[j] + S.get_S()]
            ZR = Z.t() @ Rr
            data.allreduce(ZR)
            ZR = ZR - lam * W0
            dW = torch.cholesky_solve(ZR, factors[j])
            W0 += dW
            Rr -= Z @ dW
            delsize += float((dW * dW).sum())
        if it > 0:
            reldel = math.sqrt(delsize) / max(float(W.norm()), 1e-300)
            _log(p, 2, f"Iteration {it}, relupdate = {reldel:.2e}")
            if reldel < p.tolerance:
                _log(p, 2, "Convergence!")
                break
    return True, maps, W


KernelRidge = kernel_ridge
ApproximateKernelRidge = approximate_kernel_ridge
SketchedApproximateKernelRidge = sketched_approximate_kernel_ridge
FasterKernelRidge = faster_kernel_ridge
LargeScaleKernelRidge = large_scale_kernel_ridge
