"""Python side of the C API (``libskylark_capi.so``, ``_native/capi/skylark_capi.cpp``).

The C library keeps the reference's ``sl_*`` ABI (``capi/*.hpp``): opaque
context / sketch / kernel handles, raw host matrix wraps, string-typed
dispatch ("Matrix", "SparseMatrix"), JSON parameter strings, error codes +
``sl_strerror`` / ``sl_get_exception_info``.  Each entry point marshals its
arguments to these functions (embedding CPython if the caller is a plain C
program), so C callers run the same MI355X compute path as Python users:
host buffers are staged to the GPU when one is present, processed by the
HIP kernels, and copied back.

Matrix conventions (as Elemental's ``El::Matrix<double>``): "Matrix" is a
column-major double buffer ``(data, m, n)``; "SparseMatrix" is CSC
``(indptr[n+1], indices[nnz], values[nnz], m, n)`` — the reference's
``base::sparse_matrix_t``.  Sparse outputs are produced by the library and
read back with ``sl_raw_sp_matrix_*``.
"""
from __future__ import annotations

import ctypes as C
import json

import numpy as np
import torch

from . import ml, nla, sketch
from .base.context import Context
from .base.exceptions import InvalidParametersError, SkylarkError

_DEV = None


def _device():
    global _DEV
    if _DEV is None:
        _DEV = torch.device("cuda:0") if torch.cuda.is_available() else torch.device("cpu")
    return _DEV


# ----------------------------------------------------------------- matrices
class SparseOut:
    """Library-owned CSC result (``sl_raw_sp_matrix_*`` accessors)."""

    def __init__(self):
        self.indptr = np.zeros(1, dtype=np.int32)
        self.indices = np.zeros(0, dtype=np.int32)
        self.values = np.zeros(0, dtype=np.float64)
        self.shape = (0, 0)
        self.updated = False

    def set_from_torch(self, T: torch.Tensor):
        T = T.detach().cpu().to(torch.float64)
        T = T.to_sparse_csc() if T.layout != torch.sparse_csc else T
        self.indptr = T.ccol_indices().numpy().astype(np.int32)
        self.indices = T.row_indices().numpy().astype(np.int32)
        self.values = T.values().numpy().astype(np.float64)
        self.shape = tuple(T.shape)
        self.updated = True


def _dense_view(addr: int, m: int, n: int) -> np.ndarray:
    if m * n == 0:
        return np.zeros((m, n), order="F")
    buf = (C.c_double * (m * n)).from_address(addr)
    return np.ndarray((m, n), dtype=np.float64, buffer=buf, order="F")


def _int_view(addr: int, count: int) -> np.ndarray:
    if count == 0:
        return np.zeros(0, dtype=np.int32)
    return np.ctypeslib.as_array((C.c_int32 * count).from_address(addr))


def _input(kind: str, desc):
    """desc: ("Matrix", addr, m, n) or ("SparseMatrix", indptr, ind, vals, nnz, m, n)."""
    if kind == "Matrix":
        addr, m, n = desc
        return torch.from_numpy(np.ascontiguousarray(_dense_view(addr, m, n))).to(_device())
    if kind == "SparseMatrix":
        ip, ind, vals, nnz, m, n = desc
        indptr = torch.from_numpy(_int_view(ip, n + 1).astype(np.int64))
        indices = torch.from_numpy(_int_view(ind, nnz).astype(np.int64))
        v = torch.from_numpy(np.ctypeslib.as_array((C.c_double * nnz).from_address(vals)).copy()) if nnz else \
            torch.zeros(0, dtype=torch.float64)
        T = torch.sparse_csc_tensor(indptr, indices, v, (m, n)).to_sparse_csr()
        return T.to(_device())
    raise InvalidParametersError(f"unsupported matrix type {kind}")


def _write_dense(desc, T: torch.Tensor):
    addr, m, n = desc
    T = T.detach().to_dense() if T.layout != torch.strided else T.detach()
    if tuple(T.shape) != (m, n):
        raise InvalidParametersError(f"output is {tuple(T.shape)}, wrap is {(m, n)}")
    _dense_view(addr, m, n)[...] = T.cpu().to(torch.float64).numpy()


def _output(kind, desc, T):
    if kind == "Matrix":
        _write_dense(desc, T)
    elif kind == "SparseMatrix":
        desc.set_from_torch(T if T.layout != torch.strided else T.to_sparse_csr())
    else:
        raise InvalidParametersError(f"unsupported output type {kind}")


# ------------------------------------------------------------------ context
def create_context(seed: int) -> Context:
    return Context(int(seed))


# ------------------------------------------------------------------ sketches
_PARAMS = {  # C varargs per transform (reference csketch.cpp:379-560)
    "CT": ("C",), "WZT": ("p",), "GaussianRFT": ("sigma",), "LaplacianRFT": ("sigma",),
    "MaternRFT": ("nu", "l"), "GaussianQRFT": ("sigma", "skip"), "LaplacianQRFT": ("sigma", "skip"),
    "ExpSemigroupRLT": ("beta",), "ExpSemigroupQRLT": ("beta", "skip"), "FastGaussianRFT": ("sigma",),
    "FastMaternRFT": ("nu", "l"), "PPT": ("q", "c", "gamma"),
}


def sketch_param_spec(type_name: str) -> str:
    """Varargs layout for the C side: 'd' double, 'i' int."""
    spec = {"skip": "i", "q": "i"}
    return "".join(spec.get(p, "d") for p in _PARAMS.get(type_name, ()))


def create_sketch(ctx: Context, type_name: str, n: int, s: int, params: tuple):
    try:
        cls = sketch.base.sketch_class(type_name)
    except SkylarkError as e:  # reference: unknown transform type -> 111
        err = SkylarkError(f"unknown sketch transform type {type_name!r}")
        err.code = 111
        raise err from e
    names = _PARAMS.get(type_name, ())
    kw = dict(zip(names, params))
    pos = [kw[k] for k in names if k != "skip"]
    if "skip" in kw:
        return cls(n, s, *pos, skip=int(kw["skip"]), context=ctx)
    return cls(n, s, *pos, context=ctx)


def serialize_sketch(S) -> str:
    return S.to_json()


def deserialize_sketch(data: str):
    return sketch.deserialize_sketch(json.loads(data))


def apply_sketch(S, in_kind: str, A_desc, out_kind: str, SA_out, dim: int):
    A = _input(in_kind, A_desc)
    SA = S.apply(A, dim=dim, sparse_output=(out_kind == "SparseMatrix") or None)
    _output(out_kind, SA_out, SA)


def supported_sketch_transforms() -> str:
    return " ".join(f'("{t}","{i}","{o}")' for t, i, o in sketch.supported_sketch_transforms())


# ----------------------------------------------------------------------- NLA
def _svd_params(js: str):
    d = json.loads(js) if js else {}
    p = nla.ApproximateSVDParams()
    for k in ("oversampling_ratio", "oversampling_additive", "num_iterations"):
        if k in d:
            setattr(p, k, int(d[k]))
    if "skip_qr" in d:
        v = d["skip_qr"]
        p.skip_qr = v if isinstance(v, bool) else str(v).lower() in ("1", "true")
    return p


def approximate_svd(A_kind, A_desc, U_desc, S_desc, V_desc, k, params_json, ctx):
    A = _input(A_kind, A_desc)
    U, s, V = nla.approximate_svd(A, int(k), ctx, _svd_params(params_json))
    _write_dense(U_desc, U)
    _write_dense(S_desc, s.reshape(-1, 1))
    _write_dense(V_desc, V)


def approximate_symmetric_svd(A_kind, A_desc, S_desc, V_desc, k, params_json, ctx):
    A = _input(A_kind, A_desc)
    V, s = nla.approximate_symmetric_svd(A, int(k), ctx, _svd_params(params_json))
    _write_dense(S_desc, s.reshape(-1, 1))
    _write_dense(V_desc, V)


def faster_least_squares(orientation, A_kind, A_desc, B_desc, X_desc, params_json, ctx):
    A = _input(A_kind, A_desc)
    B = _input("Matrix", B_desc)
    d = json.loads(params_json) if params_json else {}
    p = nla.FasterLSParams.from_dict(d)
    X = nla.faster_least_squares(A.to(torch.float64), B.to(torch.float64), ctx,
                                 "normal" if int(orientation) == 0 else "adjoint", p)
    _write_dense(X_desc, X)


# ------------------------------------------------------------------ kernels
_KPARAMS = {"linear": "", "gaussian": "d", "laplacian": "d", "expsemigroup": "d", "polynomial": "idd",
            "matern": "dd"}


def kernel_param_spec(type_name: str) -> str:
    return _KPARAMS.get(type_name.lower(), "")


def create_kernel(type_name: str, N: int, params: tuple):
    return ml.kernel(type_name.lower(), int(N), *params)


def kernel_gram(dirX: int, dirY: int, k, X_kind, X_desc, Y_kind, Y_desc, K_desc):
    """dir codes as the reference python binding: 1 = columns, 2 = rows."""
    X = _input(X_kind, X_desc)
    Y = _input(Y_kind, Y_desc)
    # reference ckernel.cpp:112-115: SL_COLUMNS (1) is columns, anything else rows
    d = lambda v: "columns" if int(v) == 1 else "rows"  # noqa: E731
    K = k.gram(X, dirX=d(dirX), dirY=d(dirY), Y=Y)
    _write_dense(K_desc, K)


# ----------------------------------------------------------------------- IO
def readlibsvm(fname: str, X_kind, X_out, Y_desc, direction: int, min_d: int, max_n: int):
    from .io import read_libsvm
    X, Y = read_libsvm(fname, min_d=int(min_d), max_n=int(max_n), sparse=(X_kind == "SparseMatrix"))
    if int(direction) == 1:  # SL_COLUMNS: examples are columns (d x n); anything else rows (reference cio.cpp:17-18)
        X = X.t()
        Yd = Y.reshape(1, -1)
    else:
        Yd = Y.reshape(-1, 1)
    _output(X_kind, X_out, X)
    if Y_desc is not None:
        _write_dense(Y_desc, Yd)


def error_code(exc: BaseException) -> int:
    if isinstance(exc, SkylarkError):
        return int(getattr(exc, "code", 100))
    if isinstance(exc, (ValueError, KeyError)):
        return 109
    return 100
