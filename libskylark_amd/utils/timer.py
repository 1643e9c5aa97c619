"""Phase timers / profiler (reference ``utility/timer.hpp:6-72``: SKYLARK_TIMER_*
macros; per-rank accumulation, min/max/avg reduced over ranks and printed on
rank 0).

MI355X version: timers are enabled by ``SKH_PROFILE=1`` (or
``Profiler.enable()``); when enabled each phase boundary synchronises the
current HIP stream so the host clock measures device work, and an optional
roctx range is pushed so phases show up in rocprofv3 traces.  Disabled timers
cost one attribute lookup.
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict

import torch


class Profiler:
    enabled = os.environ.get("SKH_PROFILE", "0") == "1"

    def __init__(self):
        self.acc = defaultdict(float)
        self.calls = defaultdict(int)

    @classmethod
    def enable(cls, on: bool = True):
        cls.enabled = on

    def reset(self):
        self.acc.clear()
        self.calls.clear()

    @contextlib.contextmanager
    def phase(self, name: str, device=None):
        if not self.enabled:
            yield
            return
        if torch.cuda.is_available():
            torch.cuda.synchronize(device)
        rng = None
        try:
            rng = torch.cuda.nvtx.range_push(name) if torch.cuda.is_available() else None
        except Exception:  # noqa: BLE001
            rng = None
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if torch.cuda.is_available():
                torch.cuda.synchronize(device)
            self.acc[name] += time.perf_counter() - t0
            self.calls[name] += 1
            if rng is not None:
                try:
                    torch.cuda.nvtx.range_pop()
                except Exception:  # noqa: BLE001
                    pass

    def report(self, comm=None, prefix: str = "") -> dict:
        """min/max/avg over ranks (reference SKYLARK_TIMER_PRINT)."""
        out = {}
        for name, v in sorted(self.acc.items()):
            t = torch.tensor([v, v, v], dtype=torch.float64)
            if comm is not None and comm.size > 1:
                dev = torch.device("cuda", torch.cuda.current_device()) if comm.backend == "nccl" else "cpu"
                a = t.to(dev)
                mn, mx, sm = a[0:1].clone(), a[1:2].clone(), a[2:3].clone()
                comm.all_reduce_min(mn)
                comm.all_reduce_max(mx)
                comm.all_reduce(sm)
                t = torch.cat([mn, mx, sm / comm.size]).cpu()
            out[name] = {"min_s": float(t[0]), "max_s": float(t[1]), "avg_s": float(t[2]), "calls": self.calls[name]}
        return out

    def print(self, comm=None, prefix: str = ""):
        rep = self.report(comm)
        if comm is None or comm.rank == 0:
            for name, r in rep.items():
                print(f"{prefix}{name}: min {r['min_s']:.6f}s max {r['max_s']:.6f}s avg {r['avg_s']:.6f}s ({r['calls']} calls)")
        return rep


PROFILER = Profiler()


def phase(name: str):
    return PROFILER.phase(name)
