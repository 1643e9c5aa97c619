"""One-shot all-reduce for small device operands.

The Krylov scalars, the CondEst norms and the (n + k) x k partial results of
the randSVD passes are tens to hundreds of KB: a ring all-reduce over the
point-to-point xGMI mesh pays 2(p-1) latency-bound steps for them.  Here each
rank pushes its operand once into every peer's receive buffer (mapped into
this process by IPC), waits for the peers' flags in its own buffer and sums
the p slots in rank order -- one kernel, one xGMI hop, the same bits on
every rank, capturable in a hipGraph (``_native/src/oneshot_kernels.hip``).

Reference reduction sites: ``base/inner.hpp:22,84,170`` (MPI_Allreduce of
column norms / dots), ``nla/svd.hpp`` (El::AllReduce of the small factors).

On by default for RCCL communicators (``SL_ONESHOT=auto``; ``1`` forces it,
``0`` disables it): :class:`~.comm.Comm` then routes f32 / f64 device
all-reduces of at most ``cap`` bytes here and everything else to RCCL.
Setup is collective and ends with a self-test (exact sums over both
generation buffers); if any rank cannot export or map the buffers, or the
test fails or times out anywhere, every rank stays on RCCL.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from ..ops import _lib

vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
_lib.register("sl_oneshot_alloc", [i64, i32, C.POINTER(C.c_void_p), vp])
_lib.register("sl_oneshot_open", [vp, C.POINTER(C.c_void_p)])
_lib.register("sl_oneshot_close", [vp])
_lib.register("sl_oneshot_free", [vp])
_lib.register("sl_oneshot_handle_bytes", [])
_lib.register("sl_oneshot_buffer_bytes", [i64, i32], C.c_int64)
_lib.register("sl_oneshot_allreduce", [vp, i64, i32, i32, i32, vp, i64, vp, vp, C.c_double, vp])

DEFAULT_CAP = 1 << 20      # bytes per slot: covers (n + k) x k f64 for n <= 3000, k = 40
TIMEOUT_S = 30.0


def _timeout() -> float:
    """Bounded wait of each call (SL_ONESHOT_TIMEOUT_S overrides TIMEOUT_S:
    the fault rehearsals shorten it)."""
    v = os.environ.get("SL_ONESHOT_TIMEOUT_S")
    return float(v) if v else TIMEOUT_S


class OneShotError(RuntimeError):
    pass


class OneShotAllReduce:
    """Peer-mapped receive buffers of one communicator (collective constructor)."""

    def __init__(self, comm, cap: int = DEFAULT_CAP, device=None):
        self.comm = comm
        self.p, self.rank = comm.size, comm.rank
        self.cap = int(cap)
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.ok = False
        self._local = None
        self._peers = []
        # why the path is (not) in use, the same string on every rank
        # (bench.py records it): "ok" or the first failing stage and ranks
        self.reason = "not set up"
        lib = _lib.load()
        hb = int(lib.sl_oneshot_handle_bytes()) if lib is not None and hasattr(lib, "sl_oneshot_alloc") else 0
        mine = None
        why = None
        if not hb:
            why = "no native one-shot kernels"
        elif not 2 <= self.p <= 16:
            why = f"world size {self.p} outside 2..16"
        else:
            with torch.cuda.device(self.dev):
                buf = C.c_void_p()
                h = (C.c_char * hb)()
                if _lib.require().sl_oneshot_alloc(self.cap, self.p, C.byref(buf), h) == 0:
                    self._local = buf
                    mine = bytes(h)
                else:
                    why = "IPC export of the receive buffer failed"
        handles = comm.all_gather_object(mine)
        ok = all(x is not None for x in handles)
        bases = []
        if ok:
            with torch.cuda.device(self.dev):
                for q, h in enumerate(handles):
                    if q == self.rank:
                        bases.append(self._local.value)
                        continue
                    ptr = C.c_void_p()
                    hbuf = (C.c_char * len(h)).from_buffer_copy(h)
                    if _lib.require().sl_oneshot_open(hbuf, C.byref(ptr)) != 0:
                        ok = False
                        why = f"IPC open of rank {q}'s buffer failed"
                        break
                    self._peers.append(ptr)
                    bases.append(ptr.value)
        # every rank must agree before anyone uses the path
        flags = comm.all_gather_object((bool(ok), why))
        self.ok = all(f for f, _ in flags)
        if not self.ok:
            bad = [(q, w) for q, (f, w) in enumerate(flags) if not f]
            self.reason = "; ".join(f"rank {q}: {w or 'a peer could not export its buffer'}" for q, w in bad[:4])
            self.close()
            return
        self.bases = torch.tensor(bases, dtype=torch.int64, device=self.dev)
        self.state = torch.zeros(2, dtype=torch.int64, device=self.dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.dev)
        # the collective must not start before every peer has mapped this buffer
        comm.barrier()
        # self-test on this hardware before any caller relies on the path: both
        # generation buffers, f32 and f64, rank-dependent operands, exact
        # expected sums; any mismatch or timed-out wait on any rank -> every
        # rank falls back to RCCL
        good, why = self._self_test()
        res = comm.all_gather_object((bool(good), why))
        self.ok = all(g for g, _ in res)
        if self.ok:
            self.reason = "ok"
        else:
            self.reason = "; ".join(f"rank {q}: self-test {w}" for q, (g, w) in enumerate(res) if not g)
            self.close()

    def _self_test(self, timeout_s: float = 5.0):
        """(passed, failure description)"""
        try:
            p = self.p
            for it, dt in enumerate((torch.float64, torch.float32, torch.float64, torch.float32)):
                n = 257 + 64 * it
                base = torch.arange(1, n + 1, dtype=dt, device=self.dev)
                x = base * float(self.rank + 1)
                _lib.call("sl_oneshot_allreduce", _lib.ptr(x), x.numel(), _lib.dtype_code(x.dtype), self.rank, p,
                          _lib.ptr(self.bases), self.cap, _lib.ptr(self.state), _lib.ptr(self.err), float(timeout_s),
                          vp(_lib.stream_of(x)))
                want = base * float(p * (p + 1) // 2)
                if int(self.err.item()):
                    return False, f"timed out waiting for a peer (round {it})"
                if not torch.equal(x, want):
                    return False, f"wrong sum (round {it}, {str(dt).split('.')[-1]})"
            return True, None
        except Exception as e:  # noqa: BLE001 - any failure: stay on RCCL
            return False, f"raised {type(e).__name__}: {e}"

    def fits(self, t: torch.Tensor) -> bool:
        return (self.ok and t.is_cuda and t.device == self.dev and t.dtype in (torch.float32, torch.float64)
                and t.is_contiguous() and t.numel() * t.element_size() <= self.cap)

    def all_reduce(self, t: torch.Tensor, timeout_s: float | None = None) -> torch.Tensor:
        """In-place sum of ``t`` over the ranks (stream-ordered, no host sync).

        A peer later than the timeout leaves NaN in ``t`` on the waiting rank
        (never a silent partial sum) and sets the error word; the error word
        is copied back asynchronously after every eager call and a flagged
        earlier call raises :class:`OneShotError` at the next one
        (:meth:`check` raises synchronously)."""
        if not self.fits(t):
            raise OneShotError("one-shot all-reduce: operand does not fit this buffer")
        self._poll()
        _lib.call("sl_oneshot_allreduce", _lib.ptr(t), t.numel(), _lib.dtype_code(t.dtype), self.rank, self.p,
                  _lib.ptr(self.bases), self.cap, _lib.ptr(self.state), _lib.ptr(self.err),
                  float(_timeout() if timeout_s is None else timeout_s), vp(_lib.stream_of(t)))
        if not torch.cuda.is_current_stream_capturing():
            if getattr(self, "_err_host", None) is None:
                self._err_host = torch.zeros(1, dtype=torch.int32).pin_memory()
                self._err_ev = torch.cuda.Event()
            self._err_host.copy_(self.err, non_blocking=True)
            self._err_ev.record()
        return t

    def _poll(self):
        ev = getattr(self, "_err_ev", None)
        if ev is None or torch.cuda.is_current_stream_capturing():
            return   # event queries are not permitted while a stream captures
        if ev.query() and int(self._err_host[0]):
            raise OneShotError("one-shot all-reduce: a peer did not arrive within the timeout "
                               "(the operand of that call was poisoned with NaN)")

    def check(self):
        """Raise if any earlier call timed out waiting for a peer (host sync)."""
        if int(self.err.item()):
            raise OneShotError("one-shot all-reduce: a peer did not arrive within the timeout "
                               "(the operand of that call was poisoned with NaN)")

    def close(self, comm=None):
        """Unmap the peers' buffers and free this rank's (collectively when a
        communicator is given: nobody frees a buffer a peer still maps)."""
        lib = _lib.load()
        if lib is None:
            return
        if comm is not None and self.ok:
            torch.cuda.synchronize(self.dev)
            comm.barrier()
        for ptr in self._peers:
            lib.sl_oneshot_close(ptr)
        self._peers = []
        if comm is not None and self.ok:
            comm.barrier()
        if self._local is not None:
            lib.sl_oneshot_free(self._local)
            self._local = None
        self.ok = False


# "1": always (also for gloo process groups over CUDA tensors, e.g. several
# ranks sharing one GPU in tests); "auto" (default): RCCL process groups, i.e.
# one rank per GPU -- each communicator still self-tests its buffers first;
# "0": never
_MODE = os.environ.get("SL_ONESHOT", "auto")
_ENABLED = _MODE == "1"


def enabled(comm=None) -> bool:
    if _ENABLED:
        return True
    return _MODE == "auto" and comm is not None and getattr(comm, "backend", None) == "nccl"


def enable(flag: bool = True):
    """Route small device all-reduces of every :class:`Comm` through the
    one-shot path (buffers are set up lazily, collectively, per communicator
    on its first eligible all-reduce)."""
    global _ENABLED, _MODE
    _ENABLED = bool(flag)
    _MODE = "1" if flag else "0"
