"""Native RCCL communicator driven from C++ (``_native/src/native_comm.cpp``).

SURVEY.md 2.5 asks for a C++ ``Comm`` (RCCL communicator + HIP stream) with
all-reduce / reduce-scatter / all-gather / all-to-all(v) / broadcast /
send / recv on device pointers, so native code never bounces through
Python for a collective.  This module creates such a communicator over the
ranks of a :class:`~.comm.Comm` (the unique id travels over that process
group) and exposes the same operations on torch tensors; ``handle`` is the
``void*`` the C-level entry points take.

One GPU per rank (RCCL rejects two ranks on one device); a single-rank
communicator is valid and is what the one-GPU tests use.
"""
from __future__ import annotations

import ctypes as C

import torch

from ..ops import _lib

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_comm_available", [])
_lib.register("sl_comm_unique_id_bytes", [])
_lib.register("sl_comm_unique_id", [vp])
_lib.register("sl_comm_init", [vp, i32, i32, C.POINTER(C.c_void_p)])
_lib.register("sl_comm_destroy", [vp])
_lib.register("sl_comm_all_reduce", [vp, vp, vp, i64, i32, i32, vp])
_lib.register("sl_comm_reduce_scatter", [vp, vp, vp, i64, i32, i32, vp])
_lib.register("sl_comm_all_gather", [vp, vp, vp, i64, i32, vp])
_lib.register("sl_comm_broadcast", [vp, vp, vp, i64, i32, i32, vp])
_lib.register("sl_comm_all_to_all_v", [vp, vp, vp, vp, vp, vp, vp, i32, vp])
_lib.register("sl_comm_send", [vp, vp, i64, i32, i32, vp])
_lib.register("sl_comm_recv", [vp, vp, i64, i32, i32, vp])

_DT = {torch.float32: 0, torch.float64: 1, torch.bfloat16: 2, torch.float16: 3, torch.int32: 10, torch.int64: 11}
_OP = {"sum": 0, "prod": 1, "max": 2, "min": 3}


def available() -> bool:
    lib = _lib.load()
    if lib is None or not hasattr(lib, "sl_comm_available"):
        return False
    lib.sl_comm_available.restype = C.c_int
    return bool(lib.sl_comm_available())


def _dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"native comm: dtype {t.dtype} not supported") from None


def _stream(t):
    return vp(_lib.stream_of(t))


class NativeComm:
    """RCCL communicator over the ranks of ``comm`` (collective constructor)."""

    def __init__(self, comm=None):
        from .comm import world
        comm = comm or world()
        self.rank, self.size = comm.rank, comm.size
        lib = _lib.require()
        lib.sl_comm_unique_id_bytes.restype = C.c_int
        nb = int(lib.sl_comm_unique_id_bytes())
        uid = (C.c_char * nb)()
        if self.rank == 0:
            _lib.call("sl_comm_unique_id", uid)
        ids = comm.all_gather_object(bytes(uid) if self.rank == 0 else None)
        uid = (C.c_char * nb).from_buffer_copy(ids[0])
        h = C.c_void_p()
        _lib.call("sl_comm_init", uid, self.size, self.rank, C.byref(h))
        self.handle = h

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        _lib.call("sl_comm_all_reduce", self.handle, _lib.ptr(t), _lib.ptr(t), t.numel(), _dt(t), _OP[op], _stream(t))
        return t

    def reduce_scatter(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """Sum of ``t`` (size * c elements, contiguous) over ranks; returns this rank's block of c."""
        c = t.numel() // self.size
        out = torch.empty(c, dtype=t.dtype, device=t.device)
        _lib.call("sl_comm_reduce_scatter", self.handle, _lib.ptr(t), _lib.ptr(out), c, _dt(t), _OP[op], _stream(t))
        return out

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty(self.size * t.numel(), dtype=t.dtype, device=t.device)
        _lib.call("sl_comm_all_gather", self.handle, _lib.ptr(t), _lib.ptr(out), t.numel(), _dt(t), _stream(t))
        return out.view((self.size,) + tuple(t.shape))

    def broadcast(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        _lib.call("sl_comm_broadcast", self.handle, _lib.ptr(t), _lib.ptr(t), t.numel(), _dt(t), root, _stream(t))
        return t

    def all_to_all_v(self, send: torch.Tensor, send_counts, recv_counts) -> torch.Tensor:
        """Flat all-to-all(v) in elements: ``send_counts[q]`` consecutive
        elements of ``send`` go to rank q; returns the concatenation of what
        every rank sent here (``recv_counts[q]`` from rank q)."""
        sc = (C.c_int64 * self.size)(*[int(x) for x in send_counts])
        rcn = (C.c_int64 * self.size)(*[int(x) for x in recv_counts])
        so = (C.c_int64 * self.size)()
        ro = (C.c_int64 * self.size)()
        a = b = 0
        for q in range(self.size):
            so[q], ro[q] = a, b
            a += sc[q]
            b += rcn[q]
        out = torch.empty(b, dtype=send.dtype, device=send.device)
        _lib.call("sl_comm_all_to_all_v", self.handle, _lib.ptr(send), sc, so, _lib.ptr(out), rcn, ro, _dt(send),
                  _stream(send))
        return out

    def send(self, t: torch.Tensor, peer: int):
        _lib.call("sl_comm_send", self.handle, _lib.ptr(t), t.numel(), _dt(t), peer, _stream(t))

    def recv(self, t: torch.Tensor, peer: int) -> torch.Tensor:
        _lib.call("sl_comm_recv", self.handle, _lib.ptr(t), t.numel(), _dt(t), peer, _stream(t))
        return t

    def close(self):
        if self.handle:
            _lib.call("sl_comm_destroy", self.handle)
            self.handle = None
