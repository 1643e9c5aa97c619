"""Sketch transform base class, registry and (de)serialisation.

Parity targets:
  * ``sketch_transform_t<I,O>::apply(A, SA, columnwise_tag|rowwise_tag)``
    (reference ``sketch/sketch_transform.hpp:16-88``): columnwise maps
    ``A (N x m) -> S A (S x m)``, rowwise maps ``A (m x N) -> A S^T (m x S)``
    (``sketch/transforms.hpp:13-17``);
  * Python operators ``S * A`` (columnwise) and ``S / A`` (rowwise) and
    ``serialize`` / ``deserialize_sketch`` / pickle
    (``python-skylark/skylark/sketch.py:47-221``);
  * JSON schema of ``sketch_transform_data_t::add_common``
    (``sketch/sketch_transform_data.hpp:64-71``): ``skylark_object_type``,
    ``sketch_type``, ``skylark_version``, ``N``, ``S``, ``creation_context``
    plus type-specific keys;
  * factory ``from_ptree`` keyed by ``sketch_type`` (``sketch/sketch_add.hpp``),
    accepting the reference's ``FastMaternnRFT`` misspelling as an alias.

Operands: ``torch.Tensor`` (dense, any device; sparse CSR/COO), ``numpy``
arrays, ``scipy.sparse`` matrices, and :class:`~libskylark_amd.parallel.DistMatrix`.
Results come back in the input's container type.
"""
from __future__ import annotations

import json

import numpy as np
import torch

from .. import __version__
from ..base.context import Context
from ..base.exceptions import DimensionMismatchError, InvalidParametersError, UnsupportedError

COLUMNWISE, ROWWISE = 0, 1

_REGISTRY: dict[str, type] = {}
_ALIASES = {"FastMaternnRFT": "FastMaternRFT", "CountSketch": "CWT", "FastJLT": "FJLT",
            "Fastfood": "FastGaussianRFT", "URST": "UST", "TensorSketch": "PPT"}


def register(cls):
    _REGISTRY[cls.sketch_type] = cls
    return cls


def sketch_class(name: str):
    name = _ALIASES.get(name, name)
    try:
        return _REGISTRY[name]
    except KeyError:
        raise UnsupportedError(f"unknown sketch type {name!r}") from None


def parse_dim(dim) -> int:
    if dim in (0, "columnwise", "left", "col", "columns"):
        return COLUMNWISE
    if dim in (1, "rowwise", "right", "row", "rows"):
        return ROWWISE
    raise ValueError("Dimension must be either columnwise/rowwise or left/right or 0/1")


# ---------------------------------------------------------------- operands
class Operand:
    """Normalised view of an input/output matrix."""

    def __init__(self, obj):
        self.orig = obj
        self.kind = None
        self.to_back = lambda t: t
        if isinstance(obj, torch.Tensor):
            if obj.layout == torch.sparse_csr:
                self.kind, self.t = "csr", obj
            elif obj.layout == torch.sparse_coo:
                self.kind, self.t = "csr", obj.coalesce().to_sparse_csr()
            elif obj.layout == torch.sparse_csc:
                self.kind, self.t = "csr", obj.to_sparse_coo().coalesce().to_sparse_csr()
            else:
                self.kind, self.t = "dense", obj
        elif isinstance(obj, np.ndarray):
            self.kind = "dense"
            self.t = torch.from_numpy(np.asarray(obj) if obj.ndim == 2 else obj.reshape(-1, 1))
            self.to_back = lambda t: t.detach().cpu().numpy() if isinstance(t, torch.Tensor) and not t.is_sparse and t.layout == torch.strided else t
        elif _is_scipy_sparse(obj):
            import scipy.sparse as sp
            csr = sp.csr_matrix(obj)
            self.kind = "csr"
            self.t = torch.sparse_csr_tensor(torch.from_numpy(csr.indptr.astype(np.int64)),
                                             torch.from_numpy(csr.indices.astype(np.int64)),
                                             torch.from_numpy(csr.data), size=csr.shape)
            self.to_back = _torch_to_scipy_or_numpy
        else:
            from ..parallel.distmatrix import DistMatrix
            if isinstance(obj, DistMatrix):
                self.kind, self.t = "dist", obj
            else:
                raise UnsupportedError(f"unsupported operand type {type(obj)}")

    @property
    def shape(self):
        return tuple(self.t.shape)


def _is_scipy_sparse(obj):
    try:
        import scipy.sparse as sp
        return sp.issparse(obj)
    except Exception:  # noqa: BLE001
        return False


def _torch_to_scipy_or_numpy(t):
    if isinstance(t, torch.Tensor) and t.layout == torch.sparse_csr:
        import scipy.sparse as sp
        t = t.cpu()
        return sp.csr_matrix((t.values().numpy(), t.col_indices().numpy(), t.crow_indices().numpy()),
                             shape=tuple(t.shape))
    if isinstance(t, torch.Tensor):
        return t.detach().cpu().numpy()
    return t


# ---------------------------------------------------------------- base class
class SketchTransform:
    """Base class of every sketch: ``N`` -> ``S`` dimensional map.

    Sub-classes draw all their random data in ``_build(ctx)`` from a *copy*
    of the creation context, and advance the caller's context by the same
    amount, exactly as the reference's ``*_data_t::build()`` chain does.
    """

    sketch_type = "abstract"
    supports_sparse_output = False

    def __init__(self, n: int, s: int, context: Context | None = None, **params):
        from .. import default_context
        if n <= 0 or s <= 0:
            raise InvalidParametersError("sketch dimensions must be positive")
        self._N, self._S = int(n), int(s)
        ctx = context if context is not None else default_context()
        self._creation_context = ctx.copy()
        self._params = params
        work = ctx.copy()
        self._build(work)
        ctx.counter = work.counter  # advance the caller's stream

    # -- to implement
    def _build(self, ctx: Context):
        raise NotImplementedError

    def _apply_dense(self, A: torch.Tensor, dim: int) -> torch.Tensor:
        raise NotImplementedError

    def _apply_sparse(self, A: torch.Tensor, dim: int, sparse_out: bool):
        # default: densify (transforms with native sparse kernels override this)
        return self._apply_dense(A.to_dense(), dim)

    def _extra_params(self) -> dict:
        return {}

    # -- API
    def getindim(self):
        return self._N

    def getsketchdim(self):
        return self._S

    get_N = getindim
    get_S = getsketchdim

    def apply(self, A, SA=None, dim=COLUMNWISE, out_dtype=None, sparse_output: bool | None = None):
        """Apply the transform along ``dim``; returns SA (also written into SA if given)."""
        dim = parse_dim(dim)
        if type(A).__name__ == "DistSparse2D":
            # 2-D block-sparse distribution (CombBLAS analogue): local tile + one reduction
            if A.shape[dim] != self._N:
                raise DimensionMismatchError(
                    f"Sketched dimension is incorrect (input): got {A.shape[dim]}, expected {self._N}")
            return A.sketch(self, dim)
        op = Operand(A)
        if op.kind == "dist":
            from ..parallel.dist_sketch import dist_apply
            return dist_apply(self, op.t, SA, dim)
        if len(op.shape) != 2:
            raise DimensionMismatchError("sketch input must be a matrix")
        if op.shape[dim] != self._N:
            raise DimensionMismatchError(
                f"Sketched dimension is incorrect (input): got {op.shape[dim]}, expected {self._N}")
        if op.kind == "csr":
            want_sparse = self.supports_sparse_output if sparse_output is None else sparse_output
            if SA is not None:
                want_sparse = isinstance(SA, torch.Tensor) and SA.is_sparse or _is_scipy_sparse(SA)
            if want_sparse and not self.supports_sparse_output:
                raise UnsupportedError(f"{self.sketch_type} cannot produce sparse output")
            res = self._apply_sparse(op.t, dim, want_sparse)
        else:
            res = self._apply_dense(op.t, dim)
        if out_dtype is not None and res.layout == torch.strided:
            res = res.to(out_dtype)
        if SA is not None:
            sop = Operand(SA)
            exp = (self._S, op.shape[1]) if dim == COLUMNWISE else (op.shape[0], self._S)
            if sop.shape != exp:
                raise DimensionMismatchError(f"Sketched dimension is incorrect (output): {sop.shape} != {exp}")
            if sop.kind == "dense":
                sop.t.copy_(res.to(sop.t.dtype).to(sop.t.device) if res.layout == torch.strided else res.to_dense())
                return SA
        return op.to_back(res)

    def apply_streamed(self, A, dim=COLUMNWISE, **kw):
        """Sketch a host-resident dense matrix through the GPU panel by panel
        (pinned double-buffered H2D on a copy stream; see ``sketch.streaming``)."""
        from .streaming import apply_streamed
        return apply_streamed(self, A, dim, **kw)

    def __mul__(self, A):
        return self.apply(A, None, COLUMNWISE)

    def __truediv__(self, A):
        return self.apply(A, None, ROWWISE)

    __div__ = __truediv__

    def columnwise(self, A, SA=None):
        return self.apply(A, SA, COLUMNWISE)

    def rowwise(self, A, SA=None):
        return self.apply(A, SA, ROWWISE)

    # -- serialization
    def to_dict(self) -> dict:
        d = {"skylark_object_type": "sketch", "sketch_type": self.sketch_type,
             "skylark_version": __version__, "N": self._N, "S": self._S,
             "creation_context": self._creation_context.to_dict()}
        d.update(self._extra_params())
        return d

    to_ptree = to_dict

    def serialize(self) -> dict:
        return self.to_dict()

    def to_json(self) -> str:
        return json.dumps(self.to_dict())

    @classmethod
    def _from_dict(cls, d: dict):
        ctx = Context.from_dict(d["creation_context"])
        kw = cls._params_from_dict(d)
        return cls(int(d["N"]), int(d["S"]), context=ctx, **kw)

    @classmethod
    def _params_from_dict(cls, d: dict) -> dict:
        return {}

    def __getstate__(self):
        return {"_obj": self.to_dict()}

    def __setstate__(self, state):
        other = deserialize_sketch(state["_obj"])
        self.__dict__.update(other.__dict__)

    def __repr__(self):
        return f"{self.sketch_type}(N={self._N}, S={self._S}, ctx={self._creation_context})"


def deserialize_sketch(d) -> SketchTransform:
    """Rebuild a sketch from its serialised dict/JSON (reference ``from_ptree``)."""
    if isinstance(d, str):
        d = json.loads(d)
    if d.get("skylark_object_type", "sketch") != "sketch":
        raise InvalidParametersError("not a serialized sketch")
    return sketch_class(str(d["sketch_type"]))._from_dict(d)


from_ptree = deserialize_sketch
from_json = deserialize_sketch


def supported_sketch_transforms():
    """(type, input, output) combos, reference ``sl_supported_sketch_transforms``."""
    ins = ["Matrix", "SparseMatrix", "DistMatrix", "DistMatrix_VC_STAR", "DistMatrix_VR_STAR",
           "DistMatrix_STAR_VC", "DistMatrix_STAR_VR", "SharedMatrix", "RootMatrix"]
    out = []
    for name, cls in sorted(_REGISTRY.items()):
        for i in ins:
            outs = ["Matrix"] if i in ("Matrix", "SparseMatrix") else ["SharedMatrix", "RootMatrix", i]
            if i == "SparseMatrix" and cls.supports_sparse_output:
                outs = outs + ["SparseMatrix"]
            for o in outs:
                out.append((name, i, o))
    return out
