"""Global sketch-application knobs (reference ``sketch/sketch_params.hpp:13-34``:
``sketch::params::blocksize`` = panel width of the lazily realised S,
``factor`` = threshold of the ``[MC,MR]`` panel-algorithm selection).

* ``blocksize``: columns of S realised per panel by the dense transforms;
  0 (default) sizes panels by memory instead (``ops.dense_sketch.PANEL_ELEMS``
  entries, ~128-512 MB on the MI355X's 288 GB HBM, which keeps each GEMM long).
* ``deterministic``: bit-reproducible GPU results where a kernel would
  otherwise accumulate with atomics (CountSketch of CSR input).
* ``factor``: selects the ``[MC,MR]`` columnwise dense-sketch algorithm.
  *Outer panel* (all-gather A's sketched dimension inside each grid column,
  every rank realises only its own output rows, no reduction) is used when
  ``S * 20 > N * factor``; otherwise *panel matrix* (local partial product +
  one reduction in the grid-column communicator).  At the default factor 20
  the rule compares the two collective volumes (N vs S rows per grid column)
  directly; a larger factor favours reductions, as in the reference.
"""
from __future__ import annotations

_BLOCKSIZE = 0
_FACTOR = 20
_DETERMINISTIC = False
_MC_MR_ALGO = "auto"


def get_mc_mr_algorithm() -> str:
    return _MC_MR_ALGO


def set_mc_mr_algorithm(name: str):
    """Force the [MC,MR] sketch algorithm: "inner", "outer", "panel" or "auto"."""
    global _MC_MR_ALGO
    if name not in ("auto", "inner", "outer", "panel"):
        raise ValueError("mc_mr algorithm: auto | inner | outer | panel")
    _MC_MR_ALGO = name


def get_deterministic() -> bool:
    return _DETERMINISTIC


def set_deterministic(flag: bool):
    """Bit-reproducible sketch application on the GPU: CountSketch of CSR
    input accumulates in int64 fixed point instead of LDS float atomics (about
    the same speed; see ``hash_kernels.hip``).  Everything else is already
    deterministic."""
    global _DETERMINISTIC
    _DETERMINISTIC = bool(flag)


def get_blocksize() -> int:
    return _BLOCKSIZE


def set_blocksize(b: int):
    global _BLOCKSIZE
    if b < 0:
        raise ValueError("blocksize must be >= 0")
    _BLOCKSIZE = int(b)


def get_factor() -> int:
    return _FACTOR


def set_factor(f: int):
    global _FACTOR
    if f <= 0:
        raise ValueError("factor must be positive")
    _FACTOR = int(f)
