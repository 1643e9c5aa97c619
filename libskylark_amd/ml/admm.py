"""Block-splitting ADMM for regularised loss minimisation over random features.

Reference ``ml/BlockADMM.hpp:16-611`` (Sindhwani & Avron; Parikh & Boyd
block splitting).  Data-parallel over ranks (each GPU holds ``n_i`` examples),
model-split over ``NumFeaturePartitions`` feature blocks ``Z_j = s_j``-dim
random features of X.  Per iteration, on every rank:

    mu_ij -= Wbar ; Obar -= nu ; O = prox_loss(Obar, 1/rho)
    for each feature block j:
        Z_j = map_j(X) (cached if requested),  first iteration caches
        (Z_j^T Z_j + I)^{-1};  Wi_j = Cache_j (Wbar_j - mu_ij_j + ZtObar_j
        + Z_j^T (del_o / (P_f + 1) + nu));  o_j = Z_j Wi_j ...
    consensus:  Wbar = (sum_ranks Wi + W) / (P + 1);  mu += W - Wbar

MI355X redesign of the communication: the reference broadcasts Wbar from
rank 0 and reduces Wi to rank 0 (two collectives + root-only regulariser
prox).  Here ONE all-reduce of the D x k block ``Wi`` per iteration gives
every rank the sum; the (cheap, deterministic) regulariser prox and
consensus update are computed redundantly on every GPU, so Wbar is already
replicated — no broadcast, no root bottleneck.  The loss is reduced with the
same all-reduce (appended scalar).  Validation accuracy likewise.

Per feature block and iteration Z_j is read TWICE, not four times: the pairs
{Z Wbar_j, Z^T dsum} and {o = Z Wi_j, Z^T o} each come from one streaming
pass (``ops/normal_eq.py``: ``dual`` and ``ata``; f32 on the GPU, k <= 4
targets), and the loss / regulariser / validation statistics stay on the
device until they are logged (one host transfer per logged iteration).

Layout: examples as ROWS (X n_i x d); outputs O are k x n_i as in the
reference's losses.  Feature blocks run back-to-back on the GPU (each is a
fused RNG-GEMM + cos feature map and three GEMMs; the reference's OpenMP
block parallelism is replaced by GPU-wide parallelism inside each block).
"""
from __future__ import annotations

import math
import time

import torch

from ..algorithms.loss import Loss, _targets_matrix, make_loss
from ..algorithms.regularizers import Regularizer, make_regularizer
from ..base import quasirand as Q
from ..base.context import Context
from ..ops import normal_eq
from ..parallel.comm import Comm
from ..parallel.distmatrix import DistMatrix
from ..sketch import ROWWISE
from .model import HilbertModel

_LOSS_CODE = {"squared": 0, "lad": 1, "hinge": 2, "logistic": 3}
_ADMM_REG = [False]


def _admm_lib():
    """admm_kernels.hip: the fused per-iteration pre / post passes."""
    import ctypes as C
    from ..ops import _lib
    if not _ADMM_REG[0]:
        _ADMM_REG[0] = True
        vp, i32, i64, f64 = C.c_void_p, C.c_int, C.c_int64, C.c_double
        _lib.register("sl_admm_partials", [i64], C.c_int64)
        _lib.register("sl_admm_pre", [i32, i32, i64, vp, vp, vp, vp, f64, f64, vp, vp, vp])
        _lib.register("sl_admm_post", [i32, i32, i32, i64, vp, vp, vp, vp, f64, vp, vp, vp, vp, vp])
    return _lib


def _partition(D: int, P: int):
    """Block sizes floor(nf/np) recursively (reference constructor ``:143-152``)."""
    starts, sizes, cstart, nf, np_ = [], [], 0, D, P
    for _ in range(P):
        sj = nf // np_
        starts.append(cstart)
        sizes.append(sj)
        cstart += sj
        nf -= sj
        np_ -= 1
    return starts, sizes


def num_targets(Y: torch.Tensor, comm: Comm) -> int:
    """Reference ``GetNumTargets``: 1 if labels are ±1, else max label + 1."""
    mn = torch.tensor([float(Y.min()) if Y.numel() else 1e300], dtype=torch.float64)
    mx = torch.tensor([float(Y.max()) if Y.numel() else -1e300], dtype=torch.float64)
    if comm.size > 1:
        comm.all_reduce_min(mn)
        comm.all_reduce_max(mx)
    return 1 if int(mn.item()) == -1 else int(mx.item()) + 1


def _gram(Z: torch.Tensor, dt) -> torch.Tensor:
    """Z^T Z in f64 for the block's normal-equation inverse.  A bf16 feature
    cache on the GPU takes a bf16 GEMM with f32 output (exact products, f32
    sums: what the f32 GEMM of the widened values computes, ~9x faster);
    otherwise the GEMM in the compute dtype."""
    if Z.dtype == torch.bfloat16 and Z.is_cuda:
        try:
            # split-K as a batch: Z^T Z over 1e6 rows is a 1024 x 1024 output,
            # 16 output tiles for one GEMM on 256 CUs; 16 row slices fill the
            # chip (1e6 x 1024: 3.9 -> 2.0 ms, profiles/r6/admm_gram_ab.json)
            ni = Z.shape[0]
            b = next((b for b in (16, 8, 4, 2) if ni % b == 0 and ni // b >= 4096), 1)
            if b > 1 and Z.is_contiguous():
                Zb = Z.view(b, ni // b, Z.shape[1])
                return torch.bmm(Zb.transpose(1, 2), Zb, out_dtype=torch.float32).sum(0).to(torch.float64)
            return torch.mm(Z.t(), Z, out_dtype=torch.float32).to(torch.float64)
        except (RuntimeError, TypeError):
            pass
    Zc = Z.to(dt) if Z.dtype != dt else Z
    return (Zc.t() @ Zc).to(torch.float64)


class BlockADMMSolver:
    """``BlockADMMSolver(loss, regularizer, lam, NumFeatures, kernel=None,
    tag="regular"|"fast"|"quasi", NumFeaturePartitions=1, context=None)`` or
    ``BlockADMMSolver(loss, regularizer, lam, feature_maps=[...], scale_maps=True)``."""

    def __init__(self, loss, regularizer, lam: float, NumFeatures: int = 0, kernel=None, tag: str = "regular",
                 NumFeaturePartitions: int = 1, context: Context | None = None, feature_maps=None,
                 scale_maps: bool = True):
        from .. import default_context
        self.loss: Loss = make_loss(loss) if not isinstance(loss, Loss) else loss
        self.regularizer: Regularizer = (make_regularizer(regularizer) if not isinstance(regularizer, Regularizer)
                                         else regularizer)
        self.lam = float(lam)
        self.rho, self.maxiter, self.tol = 1.0, 1000, 0.1
        self.cache_transforms = False
        # storage type of the cached feature blocks: None = the compute dtype;
        # torch.bfloat16 halves the bytes every iteration streams (the one-pass
        # kernels widen to f32; the block's (Z^T Z + I)^-1 is formed from the
        # same rounded Z, so the solver is exact for the features it holds)
        self.cache_dtype = None
        self.num_threads = 1
        self.one_pass = True      # fused Z-pair passes where the kernel applies
        self.native_prox = True   # fused native prox / consensus passes (admm_kernels.hip) on that path
        self.mfma_pass = True     # bf16 feature cache: the two Z passes on the matrix cores (normal_eq.pass_mfma)
        if feature_maps is not None:
            self.maps = list(feature_maps)
            self.sizes = [S.get_S() for S in self.maps]
            self.starts = [sum(self.sizes[:i]) for i in range(len(self.sizes))]
            self.D = sum(self.sizes)
            self.scale = bool(scale_maps)
        else:
            self.D = int(NumFeatures)
            self.starts, self.sizes = _partition(self.D, NumFeaturePartitions)
            if kernel is None:
                self.maps, self.scale = [], False
            else:
                ctx = context or default_context()
                if tag == "quasi":
                    seq = Q.LeapedHaltonSequence(kernel.qrft_sequence_dim())
                    self.maps = [kernel.create_qrft(sj, sequence=seq, skip=st, context=ctx)
                                 for st, sj in zip(self.starts, self.sizes)]
                else:
                    self.maps = [kernel.create_rft(sj, fast=(tag == "fast"), context=ctx) for sj in self.sizes]
                self.scale = True
        self.P = len(self.sizes)

    # reference setters
    def set_rho(self, rho):
        self.rho = float(rho)

    def set_maxiter(self, it):
        self.maxiter = int(it)

    def set_tol(self, tol):
        self.tol = float(tol)

    def set_cache_transform(self, flag: bool):
        self.cache_transforms = bool(flag)

    def set_cache_dtype(self, dtype):
        """Storage type of the cached feature blocks (``torch.bfloat16``: half
        the HBM traffic per iteration on the GPU one-pass path; ``None``: the
        compute dtype).  An extension knob, not in the reference."""
        if dtype not in (None, torch.float32, torch.float64, torch.bfloat16):
            raise ValueError("cache dtype: None, float32, float64 or bfloat16")
        self.cache_dtype = dtype

    def set_nthreads(self, n):
        self.num_threads = int(n)

    def get_numfeatures(self):
        return self.D

    def get_feature_maps(self):
        return self.maps

    def _Z(self, j: int, X: torch.Tensor, dt) -> torch.Tensor:
        if not self.maps:
            return X[:, self.starts[j]:self.starts[j] + self.sizes[j]].to(dt)
        Z = self.maps[j].apply(X, dim=ROWWISE).to(dt)
        if self.scale:
            Z = Z * math.sqrt(self.sizes[j] / X.shape[1])
        return Z

    def train(self, X, Y, Xv=None, Yv=None, regression: bool = False, comm: Comm | None = None,
              dtype=None, log=print) -> HilbertModel:
        """Returns a :class:`HilbertModel`.  ``X`` (n_i x d) / ``Y`` (n_i labels
        or n_i x k targets) are this rank's examples (DistMatrix [VC,*] accepted)."""
        if isinstance(X, DistMatrix):
            comm = comm or X.comm
            X = X.local
        if isinstance(Y, DistMatrix):
            Y = Y.local
        comm = comm or Comm(None)
        X = X.to_dense() if X.layout != torch.strided else X
        dev = X.device
        dt = dtype or (X.dtype if X.dtype in (torch.float32, torch.float64) else torch.float32)
        Y = Y.to(dev)
        if Y.dim() == 2 and Y.shape[1] == 1:
            Y = Y[:, 0]
        ni = X.shape[0]
        k = (Y.shape[1] if Y.dim() == 2 else 1) if regression else num_targets(Y, comm)
        D, P, rank_count = self.D, self.P, comm.size
        model = HilbertModel(self.maps, self.scale, D, k, regression, input_size=X.shape[1])
        Wbar = torch.zeros(D, k, dtype=dt, device=dev)
        O = torch.zeros(k, ni, dtype=dt, device=dev)
        Obar = torch.zeros_like(O)
        nu = torch.zeros_like(O)
        W = torch.zeros(D, k, dtype=dt, device=dev)
        mu = torch.zeros_like(W)
        Wi = torch.zeros_like(W)
        mu_ij = torch.zeros_like(W)
        ZtObar = torch.zeros_like(W)
        del_o = torch.zeros(k, ni, dtype=dt, device=dev)
        cache, zcache = [None] * P, [None] * P
        # class labels -> the k x n_i +-1 target matrix, built once (every loss
        # prox / evaluation takes it as given targets)
        Yt = Y if regression or Y.dim() != 1 or k == 1 else _targets_matrix(Y, k, Wbar)
        # one-pass kernels for the two Z pairs per block (f32 on the GPU, k <= 4)
        kp = 1 if k == 1 else (2 if k == 2 else 4)
        fused = self.one_pass and dev.type == "cuda" and dt == torch.float32 and k <= 4
        Dp = torch.zeros(kp, ni, dtype=dt, device=dev) if fused else None
        # padded (s_j x kp) operands of the one-pass kernels, allocated once
        pads = {}
        # the per-iteration element-wise work on the k x n_i block as two
        # native passes (admm_kernels.hip) on the fused path: the block sums
        # arrive in zw_sum / zo_sum (n_i x kp), which the post pass zeroes
        lcode = _LOSS_CODE.get(getattr(self.loss, "name", ""))
        native = (fused and self.native_prox and lcode is not None
                  and ((Yt.dim() == 2 and Yt.shape[0] == k) or (Yt.dim() == 1 and k == 1))
                  and (lcode != 3 or k >= 2))
        if native:
            L = _admm_lib()
            L.require()
            Yt = (Yt[None, :] if Yt.dim() == 1 else Yt).to(dt).contiguous()
            zw_sum = torch.zeros(ni, kp, dtype=dt, device=dev)
            zo_sum = torch.zeros(ni, kp, dtype=dt, device=dev)
            partial = torch.zeros(int(L.require().sl_admm_partials(ni)), dtype=torch.float64, device=dev)
            st_ = L.stream_of(O)

        def padded(tag, j, Wj):
            if Wj.shape[1] == kp:
                return Wj.contiguous()
            if (tag, j) not in pads:
                pads[tag, j] = torch.zeros(Wj.shape[0], kp, dtype=dt, device=dev)
            pads[tag, j][:, :Wj.shape[1]] = Wj
            return pads[tag, j]
        t0 = time.time()
        self.history = []
        pending = []
        for it in range(1, self.maxiter + 1):
            mu_ij -= Wbar
            if native:
                # Obar -= nu; O = prox(Obar); Dp[:k] = del_o + (P + 1) nu
                L.call("sl_admm_pre", lcode, k, ni, L.ptr(Obar), L.ptr(nu), L.ptr(del_o), L.ptr(Yt),
                       1.0 / self.rho, P + 1.0, L.ptr(O), L.ptr(Dp), st_)
                dsum = Dp[:k]
            else:
                Obar -= nu
                O = self.loss.proxoperator(Obar, 1.0 / self.rho, Yt).to(dt)
                sum_o = torch.zeros(k, ni, dtype=dt, device=dev)
                wbar_out = torch.zeros(k, ni, dtype=dt, device=dev)
                dsum = del_o + (P + 1.0) * nu  # k x ni
                if fused:
                    Dp[:k] = dsum
                    # the one-pass kernels' n_i x kp outputs summed as they come
                    # (contiguous adds); folded into the k x n_i sums once
                    zw_sum = torch.zeros(ni, kp, dtype=dt, device=dev)
                    zo_sum = torch.zeros(ni, kp, dtype=dt, device=dev)
            W = self.regularizer.proxoperator(Wbar - mu, self.lam / self.rho).to(dt)
            for j in range(P):
                st, sj = self.starts[j], self.sizes[j]
                if self.cache_transforms and zcache[j] is not None:
                    Z = zcache[j]
                else:
                    Z = self._Z(j, X, dt)  # ni x sj
                    if (self.cache_transforms and self.cache_dtype is not None and fused
                            and self.cache_dtype != Z.dtype):
                        Z = Z.to(self.cache_dtype)   # the one-pass kernels read it as stored
                    if self.cache_transforms:
                        zcache[j] = Z
                if Z.dtype != dt and not (fused and normal_eq.native_ok(Z, kp)):
                    Z = Z.to(dt)   # stored narrower than the compute dtype, no native pass: widen
                if cache[j] is None:
                    C = _gram(Z, dt)
                    C.diagonal().add_(1.0)
                    cache[j] = torch.cholesky_inverse(torch.linalg.cholesky(C)).to(dt)
                Wb = Wbar[st:st + sj]
                one_pass = fused and normal_eq.native_ok(Z, kp)
                # bf16 feature cache: both passes on the matrix cores (the
                # randSVD fused pass's EXT form) instead of the VALU widening
                # kernel
                mfma = (one_pass and self.mfma_pass and Z.dtype == torch.bfloat16
                        and normal_eq.mfma_ok(Z, kp, Dp.t()))
                if mfma:
                    ztd, yz = normal_eq.pass_mfma(Z, padded("wb", j, Wb), D=Dp.t())
                    zw_sum += yz
                    ztd = ztd[:, :k]
                elif one_pass:
                    # pass 1: {Z Wbar_j, Z^T dsum^T} from one read of Z
                    ztd, _ = normal_eq.dual(Z, Dp.t(), padded("wb", j, Wb), y_out=zw_sum)   # zw_sum += Z Wb
                    ztd = ztd[:, :k]
                elif native:
                    zw_sum[:, :k] += Z @ Wb
                    ztd = Z.t() @ dsum.t()
                else:
                    wbar_out += (Z @ Wb).t()
                    ztd = Z.t() @ dsum.t()
                rhs = Wb - mu_ij[st:st + sj] + ZtObar[st:st + sj] + ztd / (P + 1.0)
                Wi_j = cache[j] @ rhs
                Wi[st:st + sj] = Wi_j
                if mfma:
                    zto, yo = normal_eq.pass_mfma(Z, padded("wi", j, Wi_j))
                    zo_sum += yo
                    ZtObar[st:st + sj] = zto[:, :k]
                elif one_pass:
                    # pass 2: {o = Z Wi_j, Z^T o} from one read of Z
                    zto, _ = normal_eq.ata(Z, padded("wi", j, Wi_j), want_y=True, y_out=zo_sum)   # zo_sum += o
                    ZtObar[st:st + sj] = zto[:, :k]
                else:
                    o = (Z @ Wi_j).t()  # k x ni
                    ZtObar[st:st + sj] = Z.t() @ o.t()
                    if native:
                        zo_sum[:, :k] += o.t()
                    else:
                        sum_o += o
                mu_ij[st:st + sj] += Wi_j
            if native:
                # del_o = O - sum o; Obar = O - del_o / (P + 1); nu += O - Obar; the loss partials
                L.call("sl_admm_post", lcode, k, kp, ni, L.ptr(O), L.ptr(zo_sum), L.ptr(zw_sum), L.ptr(Yt),
                       P + 1.0, L.ptr(Obar), L.ptr(nu), L.ptr(del_o), L.ptr(partial), st_)
                stats = [partial.sum()]
            else:
                if fused:
                    wbar_out += zw_sum[:, :k].t()
                    sum_o += zo_sum[:, :k].t()
                sum_o = O - sum_o
                del_o = sum_o.clone()
                stats = [self.loss.evaluate_t(wbar_out, Yt).to(torch.float64)]
            # ---- one all-reduce: [Wi | loss | validation stats]; all on the device
            if Xv is not None:
                stats += list(self._validate_t(model, Wbar, Xv, Yv, regression))
            else:
                stats += [torch.zeros((), dtype=torch.float64, device=dev)] * 2
            buf = torch.cat([Wi.reshape(-1).to(torch.float64), torch.stack(stats)])
            if rank_count > 1:
                comm.all_reduce(buf)
            Wsum = buf[:D * k].reshape(D, k).to(dt)
            tail = torch.cat([buf[D * k:], (self.lam * self.regularizer.evaluate_t(Wbar)).to(torch.float64)[None]])
            pending.append((it, *self._stage(tail), time.time() - t0))
            if log is not None:
                # iteration it - 1 is logged once iteration it is queued: the host
                # waits on that iteration's event while the GPU runs this one
                while len(pending) > 1:
                    self._log(self._record(*pending.pop(0), Xv is not None, regression), comm, log)
            if not native:
                Obar = O - sum_o / (P + 1.0)
                nu = nu + O - Obar
            Wbar = (Wsum + W) / (rank_count + 1.0)
            mu = mu + W - Wbar
            model.coef = Wbar
        for p_ in pending:   # iterations not logged yet: host transfers at the end
            rec = self._record(*p_, Xv is not None, regression)
            if log is not None:
                self._log(rec, comm, log)
        self.history.sort(key=lambda r: r["iteration"])
        model.coef = Wbar.to(torch.float64).cpu() if not Wbar.is_cuda else Wbar.to(torch.float64)
        return model

    @staticmethod
    def _stage(tail):
        """Starts the device -> host copy of an iteration's statistics (pinned
        buffer, non-blocking) and returns it with the event that completes it."""
        if not tail.is_cuda:
            return tail, None
        host = torch.empty(tail.shape, dtype=tail.dtype, pin_memory=True)
        host.copy_(tail, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return host, ev

    @staticmethod
    def _log(rec, comm, log):
        if comm.rank == 0:
            msg = f"iteration {rec['iteration']} objective {rec['objective']:g}"
            if "accuracy" in rec:
                msg += f" accuracy {rec['accuracy']:.2f}"
            log(msg + f" time {rec['time']:.3f} seconds")

    def _record(self, it, tail, ev, elapsed, has_val, regression):
        if ev is not None:
            ev.synchronize()
        totalloss, s0, s1, reg = (float(v) for v in tail)
        rec = {"iteration": it, "objective": totalloss + reg, "time": elapsed}
        if has_val:
            rec["accuracy"] = math.sqrt(s0 / s1) if regression else 100.0 * s0 / max(s1, 1)
        self.history.append(rec)
        return rec

    @staticmethod
    def _validate_t(model, Wbar, Xv, Yv, regression):
        """(s0, s1) validation statistics as device scalars."""
        model.coef = Wbar
        labels, DV = model.predict(Xv.to(Wbar.device))
        Yv = Yv.to(DV.device)
        if regression:
            Yr = Yv if Yv.dim() == 2 else Yv[:, None]
            return ((DV - Yr) ** 2).sum().double(), (Yr ** 2).sum().double()
        correct = (labels.to(torch.float64) == Yv.reshape(-1).to(torch.float64)).sum().double()
        return correct, torch.tensor(float(Yv.numel()), dtype=torch.float64, device=DV.device)


BlockADMM = BlockADMMSolver
