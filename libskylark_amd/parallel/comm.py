"""Process-group handle + collectives (one process per GPU, RCCL over xGMI).

Replaces the reference's Boost.MPI communicator use
(``utility/get_communicator.hpp:25-63``; every call site in SURVEY.md 2.5).
``torch.distributed`` backend ``"nccl"`` is RCCL on ROCm; ``"gloo"`` is used
for CPU tensors (plumbing tests, host metadata).  Rendezvous always uses
127.0.0.1 unless MASTER_ADDR says otherwise.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def init_distributed(backend: str | None = None, device: str | None = None, timeout_s: int = 600):
    """Initialise the default process group from torchrun-style env vars.

    Returns the world :class:`Comm`.  With WORLD_SIZE unset this is a
    single-rank communicator that performs no communication.
    """
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend is None:
            backend = os.environ.get("SKH_DIST_BACKEND") or (
                "nccl" if (device != "cpu" and torch.cuda.is_available()) else "gloo")
        if torch.cuda.is_available() and device != "cpu":
            # one process per GPU; modulo only matters for rehearsals with more
            # ranks than GPUs (gloo backend)
            lr = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(lr % max(1, torch.cuda.device_count()))
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
    return Comm()


class Comm:
    """Thin wrapper around a process group (None = WORLD)."""

    def __init__(self, group=None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.size = dist.get_world_size(group)
            self.backend = dist.get_backend(group)
            self._active = self.size > 1
        else:
            self.rank, self.size, self.backend, self._active = 0, 1, None, False
        self.bytes_sent = 0   # payload bytes this rank put on the wire (diagnostics, tests)

    @classmethod
    def single(cls) -> "Comm":
        """A one-rank communicator that never communicates (process-local data)."""
        c = cls.__new__(cls)
        c.group, c.rank, c.size, c.backend, c._active = None, 0, 1, None, False
        c.bytes_sent = 0
        return c

    @property
    def is_root(self):
        return self.rank == 0

    def collective_device(self) -> torch.device:
        """Where tensors must live for this backend's collectives (RCCL: the
        current GPU; gloo / single rank: host)."""
        if self.backend == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    # Every collective stages its operands onto collective_device() and hands
    # results back on the caller's device, so host tensors may be passed on
    # an RCCL communicator (IO paths build their buffers on the host) and GPU
    # tensors on a gloo one (multi-rank rehearsals on one GPU).
    def _stage(self, t: torch.Tensor) -> torch.Tensor:
        dev = self.collective_device()
        return t if t.device == dev else t.to(dev)

    def _count(self, nbytes: int):
        self.bytes_sent = getattr(self, "bytes_sent", 0) + int(nbytes)

    def _oneshot_for(self, t: torch.Tensor):
        """The one-shot path for a small device SUM operand, or None (opt-in,
        parallel/oneshot.py; set up collectively on first use)."""
        from . import oneshot
        if not oneshot.enabled(self) or not t.is_cuda:
            return None
        os_ = getattr(self, "_oneshot", None)
        if os_ is None:
            try:
                os_ = oneshot.OneShotAllReduce(self, device=t.device)
                self.oneshot_reason = os_.reason
            except Exception as e:  # noqa: BLE001 - no IPC / no native library: stay on RCCL
                os_ = False
                self.oneshot_reason = f"setup raised {type(e).__name__}: {e}"
            if os_ is not False and not os_.ok:
                os_ = False
            self._oneshot = os_
        return os_ if (os_ and os_.fits(t)) else None

    def oneshot_status(self) -> dict:
        """Whether small device all-reduces go through the one-shot path, and
        why not when they do not (set up lazily on the first eligible call)."""
        from . import oneshot
        os_ = getattr(self, "_oneshot", None)
        if not self._active or self.size < 2:
            return {"enabled": False, "reason": "single rank"}
        if not oneshot.enabled(self):
            return {"enabled": False, "reason": f"disabled (SL_ONESHOT={oneshot._MODE}, backend {self.backend})"}
        if os_ is None:
            return {"enabled": False, "reason": "never set up (no eligible all-reduce yet)"}
        return {"enabled": bool(os_), "reason": getattr(self, "oneshot_reason", "unknown")}

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM if dist.is_available() else None):
        if self._active and op == dist.ReduceOp.SUM:
            os_ = self._oneshot_for(t)
            if os_ is not None:
                os_.all_reduce(t)
                self._count(t.numel() * t.element_size() * (self.size - 1))
                return t
        if self._active:
            st = self._stage(t)
            dist.all_reduce(st, op=op, group=self.group)
            if st is not t:
                t.copy_(st)
            self._count(2 * t.numel() * t.element_size() * (self.size - 1) // self.size)
        return t

    def check_collectives(self, agree: bool = False):
        """Raise if an asynchronous collective of this communicator failed
        (a one-shot all-reduce whose peer missed the timeout).

        ``agree=True`` (collective): every rank learns every rank's state
        through the backend's own collective, so a timeout seen by ANY rank
        raises :class:`~.oneshot.OneShotError` on EVERY rank -- the late rank
        itself summed valid data and would not know -- and the one-shot path
        of this communicator is dropped: its later all-reduces go to RCCL
        (or gloo), and ``oneshot_status()`` names the ranks that timed out."""
        os_ = getattr(self, "_oneshot", None)
        if not agree:
            if os_:
                os_.check()
            return
        mine = False
        if os_:
            try:
                os_.check()
            except Exception:  # noqa: BLE001 - reported collectively below
                mine = True
        if not self._active or self.size < 2:
            if mine:
                os_.check()
            return
        flags = self.all_gather_object(bool(mine))
        bad = [q for q, f in enumerate(flags) if f]
        if bad:
            from .oneshot import OneShotError
            reason = (f"one-shot all-reduce timed out on rank(s) {bad} (their operands were poisoned with NaN); "
                      "the path is dropped for this communicator, later all-reduces use the backend")
            if os_:
                os_.close(self)
            self._oneshot = False
            self.oneshot_reason = reason
            raise OneShotError(reason)

    def close(self):
        """Release this communicator's one-shot IPC buffers collectively
        (barrier before any rank frees a buffer its peers map)."""
        os_ = getattr(self, "_oneshot", None)
        if os_:
            os_.close(self)
        self._oneshot = None

    def all_reduce_max(self, t):
        return self.all_reduce(t, op=dist.ReduceOp.MAX)

    def all_reduce_min(self, t):
        return self.all_reduce(t, op=dist.ReduceOp.MIN)

    def reduce(self, t: torch.Tensor, root: int = 0):
        if self._active:
            st = self._stage(t)
            dist.reduce(st, dst=self.global_rank(root), group=self.group)
            if st is not t and self.rank == root:
                t.copy_(st)
        return t

    def broadcast(self, t: torch.Tensor, root: int = 0):
        if self._active:
            st = self._stage(t)
            dist.broadcast(st, src=self.global_rank(root), group=self.group)
            if st is not t:
                t.copy_(st)
            if self.rank == root:
                self._count(t.numel() * t.element_size())
        return t

    def all_gather(self, t: torch.Tensor, dim: int = 0) -> torch.Tensor:
        """Concatenate equal-shaped shards along ``dim``."""
        if not self._active:
            return t
        src_dev = t.device
        t = self._stage(t).contiguous()
        if dim != 0:
            t = t.movedim(dim, 0).contiguous()
        out = torch.empty((self.size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        self._count(t.numel() * t.element_size() * (self.size - 1))
        if dim != 0:
            out = out.view((self.size, t.shape[0]) + tuple(t.shape[1:]))
            out = torch.cat(list(out.unbind(0)), 0).movedim(0, dim)
        return out.to(src_dev)

    def all_gather_v(self, t: torch.Tensor, counts, dim: int = 0) -> torch.Tensor:
        """All-gather shards of unequal size along ``dim`` (counts per rank)."""
        if not self._active:
            return t
        mx = max(counts)
        tt = t.movedim(dim, 0)
        if all(c == mx for c in counts):
            return self.all_gather(tt.contiguous(), 0).movedim(0, dim)
        buf = torch.zeros((mx,) + tuple(tt.shape[1:]), dtype=t.dtype, device=t.device)
        buf[: tt.shape[0]].copy_(tt)
        g = self.all_gather(buf, 0)
        g = g.view((self.size, mx) + tuple(g.shape[1:]))
        parts = [g[r, :counts[r]] for r in range(self.size)]
        return torch.cat(parts, 0).movedim(0, dim)

    def reduce_scatter_v(self, t: torch.Tensor, counts, dim: int = 0) -> torch.Tensor:
        """Sum ``t`` over ranks and keep this rank's slice (counts along dim).

        Unequal counts are padded to the largest one and reduced with ONE
        reduce-scatter (never an all-reduce of the whole operand)."""
        if not self._active:
            return t
        if dim != 0:
            return self.reduce_scatter_v(t.movedim(dim, 0).contiguous(), counts, 0).movedim(0, dim)
        src_dev = t.device
        t = self._stage(t)
        mx = max(counts)
        tail = tuple(t.shape[1:])
        if all(c == mx for c in counts):
            buf = t.contiguous()
        else:
            buf = torch.zeros((self.size * mx,) + tail, dtype=t.dtype, device=t.device)
            off = 0
            for r, c in enumerate(counts):
                buf[r * mx: r * mx + c].copy_(t[off: off + c])
                off += c
        out = torch.empty((mx,) + tail, dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(out, buf, group=self.group)
        self._count(buf.numel() * buf.element_size() * (self.size - 1) // self.size)
        return out[: counts[self.rank]].to(src_dev)

    def all_to_all_v(self, sends: list[torch.Tensor], recv_counts=None) -> list[torch.Tensor]:
        """Exchange per-destination tensors (equal trailing dims): ``sends[d]``
        goes to rank d; returns the list of pieces received from each rank.

        One ``all_to_all_single`` with split sizes (RCCL and gloo alike);
        ``recv_counts`` (rows from every source) skips the size exchange when
        the caller already knows the geometry."""
        if not self._active:
            return list(sends)
        src_dev = sends[0].device
        dt = sends[0].dtype
        tail = tuple(sends[0].shape[1:])
        row = 1
        for x in tail:
            row *= int(x)
        dev = self.collective_device()
        send_counts = [int(s.shape[0]) for s in sends]
        if recv_counts is None:
            sz = torch.tensor(send_counts, dtype=torch.int64, device=dev)
            rsz = torch.empty_like(sz)
            dist.all_to_all_single(rsz, sz, group=self.group)
            recv_counts = [int(x) for x in rsz.tolist()]
        flat = torch.cat([s.reshape(-1).to(dev) for s in sends]) if sends else torch.empty(0, dtype=dt, device=dev)
        out = torch.empty(sum(recv_counts) * row, dtype=dt, device=dev)
        dist.all_to_all_single(out, flat, [c * row for c in recv_counts], [c * row for c in send_counts],
                               group=self.group)
        self._count((flat.numel() - send_counts[self.rank] * row) * flat.element_size())
        pieces = torch.split(out, [c * row for c in recv_counts])
        return [p.view((c,) + tail).to(src_dev) for p, c in zip(pieces, recv_counts)]

    def barrier(self):
        if self._active:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)

    def global_rank(self, r: int) -> int:
        if self.group is None or not self._active:
            return r
        return dist.get_global_rank(self.group, r)

    def split(self, color: int, key: int | None = None) -> "Comm":
        """MPI_Comm_split analogue; must be called collectively by all ranks."""
        if not self._active:
            return Comm(None)
        colors = self.all_gather_object((color, self.rank if key is None else key))
        groups = {}
        for r, (c, k) in enumerate(colors):
            groups.setdefault(c, []).append((k, self.global_rank(r)))
        mine = None
        for c in sorted(groups):
            ranks = [g for _, g in sorted(groups[c])]
            pg = dist.new_group(ranks=ranks)
            if c == color:
                mine = pg
        return Comm(mine)

    def all_gather_object(self, obj):
        if not self._active:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj, group=self.group)
        return out


_WORLD = None


def world() -> Comm:
    global _WORLD
    if _WORLD is None or (dist.is_initialized() and _WORLD.size != dist.get_world_size()):
        _WORLD = Comm()
    return _WORLD


def balanced_counts(n: int, p: int):
    """Contiguous 1-D block distribution of n items over p ranks."""
    q, r = divmod(n, p)
    return [q + (1 if i < r else 0) for i in range(p)]


def balanced_offsets(n: int, p: int):
    c = balanced_counts(n, p)
    off = [0]
    for x in c:
        off.append(off[-1] + x)
    return off
