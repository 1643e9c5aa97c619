"""Common algorithm parameters, logging and matrix debug printing.

Reference: ``base/params.hpp:12-40`` (``params_t{am_i_printing, log_level,
log_stream, prefix, debug_level}`` with a JSON constructor, threaded through
every algorithm) and ``utility/external/print.hpp:13-60`` (``print_t``:
dump a matrix when ``debug_level > 1``, used e.g. in ``LSQR.hpp:64,76``).
The per-algorithm parameter classes (``ApproximateSVDParams``,
``KrylovIterParams``, ...) carry the same fields; this base supplies the
shared behaviour: ``log(level, msg)`` writes ``prefix + msg`` to
``log_stream`` on the printing rank when ``level <= log_level``.
"""
from __future__ import annotations

import json
import sys
from dataclasses import asdict, dataclass, field
from typing import Any

import torch


@dataclass
class Params:
    am_i_printing: bool = False
    log_level: int = 0
    prefix: str = ""
    debug_level: int = 0
    log_stream: Any = field(default=None, repr=False, compare=False)

    @classmethod
    def from_json(cls, s):
        d = json.loads(s) if isinstance(s, str) else dict(s)
        keys = {f for f in cls.__dataclass_fields__ if f != "log_stream"}
        return cls(**{k: v for k, v in d.items() if k in keys})

    def to_json(self) -> str:
        d = asdict(self)
        d.pop("log_stream", None)
        return json.dumps(d)

    def log(self, level: int, msg: str):
        if self.am_i_printing and level <= self.log_level:
            print(f"{self.prefix}{msg}", file=self.log_stream or sys.stdout, flush=True)

    def print_matrix(self, X, name: str):
        print_matrix(X, name, self.am_i_printing, self.debug_level, stream=self.log_stream)


def print_matrix(X, name: str, am_i_printing: bool = True, debug_level: int = 2, stream=None,
                 max_rows: int = 20, max_cols: int = 10):
    """Debug dump of a (possibly distributed / sparse) matrix when
    ``debug_level > 1`` (reference ``print_t::apply``).  Distributed matrices
    are gathered collectively first, so every rank must call it."""
    if debug_level <= 1:
        return
    from ..parallel.distmatrix import DistMatrix
    from .sparse import SparseMatrix
    if isinstance(X, DistMatrix):
        X = X.to_global()
    if isinstance(X, SparseMatrix):
        X = X.to_dense()
    if isinstance(X, torch.Tensor) and X.layout != torch.strided:
        X = X.to_dense()
    if not am_i_printing:
        return
    out = stream or sys.stdout
    T = torch.as_tensor(X).detach().cpu()
    if T.dim() == 1:
        T = T.view(-1, 1)
    print(f"{name} ({T.shape[0]} x {T.shape[1]}, {T.dtype}):", file=out)
    for i in range(min(T.shape[0], max_rows)):
        row = " ".join(f"{float(v): .6e}" for v in T[i, :max_cols])
        print(f"  {row}{' ...' if T.shape[1] > max_cols else ''}", file=out)
    if T.shape[0] > max_rows:
        print("  ...", file=out)
    out.flush()


__all__ = ["Params", "print_matrix"]
