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

    @classmethod
    def single(cls) -> "Comm":
        """A one-rank communicator that never communicates (process-local data)."""
        c = cls.__new__(cls)
        c.group, c.rank, c.size, c.backend, c._active = None, 0, 1, None, False
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

    def _ready(self, t):
        return t

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM if dist.is_available() else None):
        if self._active:
            dist.all_reduce(t, op=op, group=self.group)
        return t

    def all_reduce_max(self, t):
        return self.all_reduce(t, op=dist.ReduceOp.MAX)

    def all_reduce_min(self, t):
        return self.all_reduce(t, op=dist.ReduceOp.MIN)

    def reduce(self, t: torch.Tensor, root: int = 0):
        if self._active:
            dist.reduce(t, dst=self.global_rank(root), group=self.group)
        return t

    def broadcast(self, t: torch.Tensor, root: int = 0):
        if self._active:
            dist.broadcast(t, src=self.global_rank(root), group=self.group)
        return t

    def all_gather(self, t: torch.Tensor, dim: int = 0) -> torch.Tensor:
        """Concatenate equal-shaped shards along ``dim``."""
        if not self._active:
            return t
        t = t.contiguous()
        if dim == 0:
            out = torch.empty((self.size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t, group=self.group)
            return out
        parts = [torch.empty_like(t) for _ in range(self.size)]
        dist.all_gather(parts, t, group=self.group)
        return torch.cat(parts, dim)

    def all_gather_v(self, t: torch.Tensor, counts, dim: int = 0) -> torch.Tensor:
        """All-gather shards of unequal size along ``dim`` (counts per rank)."""
        if not self._active:
            return t
        mx = max(counts)
        pad = list(t.shape)
        pad[dim] = mx
        buf = torch.zeros(pad, dtype=t.dtype, device=t.device)
        buf.narrow(dim, 0, t.shape[dim]).copy_(t)
        g = self.all_gather(buf.movedim(dim, 0).contiguous(), 0)
        g = g.view((self.size, mx) + tuple(g.shape[1:]))
        parts = [g[r, :counts[r]] for r in range(self.size)]
        return torch.cat(parts, 0).movedim(0, dim)

    def reduce_scatter_v(self, t: torch.Tensor, counts, dim: int = 0) -> torch.Tensor:
        """Sum ``t`` over ranks and keep this rank's slice (counts along dim)."""
        if not self._active:
            return t
        if dim != 0:
            return self.reduce_scatter_v(t.movedim(dim, 0).contiguous(), counts, 0).movedim(0, dim)
        mx = max(counts)
        if all(c == mx for c in counts) and self.backend == "nccl":
            out = torch.empty((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            dist.reduce_scatter_tensor(out, t.contiguous(), group=self.group)
            return out
        # general path: all-reduce and slice (gloo has no reduce_scatter)
        tt = t.contiguous().clone()
        self.all_reduce(tt)
        off = sum(counts[: self.rank])
        return tt[off: off + counts[self.rank]].contiguous()

    def all_to_all_v(self, sends: list[torch.Tensor]) -> list[torch.Tensor]:
        """Exchange a list of per-destination tensors (any shapes with equal trailing dims)."""
        if not self._active:
            return sends
        # exchange sizes first
        dev = sends[0].device
        sz = torch.tensor([s.shape[0] for s in sends], dtype=torch.int64, device=dev)
        rsz = torch.empty_like(sz)
        allsz = None
        if self.backend == "gloo":
            allsz = self.all_gather(sz.view(1, -1), 0)
            rsz = allsz[:, self.rank].contiguous()
        else:
            dist.all_to_all_single(rsz, sz, group=self.group)
        rs = [int(x) for x in rsz.tolist()]
        tail = tuple(sends[0].shape[1:])
        recvs = [torch.empty((n,) + tail, dtype=sends[0].dtype, device=dev) for n in rs]
        if self.backend == "gloo":
            # gloo lacks all_to_all: emulate with an all-gather of padded buffers
            mx = max(int(allsz.max()), 1)  # same padded size on every rank
            buf = torch.zeros((self.size, mx) + tail, dtype=sends[0].dtype, device=dev)
            for i, s in enumerate(sends):
                buf[i, : s.shape[0]] = s
            allb = self.all_gather(buf.view((1,) + tuple(buf.shape)), 0)
            for src in range(self.size):
                recvs[src].copy_(allb[src, self.rank, : rs[src]])
            return recvs
        dist.all_to_all([r.contiguous() for r in recvs], [s.contiguous() for s in sends], group=self.group)
        return recvs

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
