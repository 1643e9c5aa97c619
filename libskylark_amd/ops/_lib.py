"""ctypes binding of the native HIP library ``libskylark_hip.so``.

The library exposes a plain C ABI (``sl_*`` functions taking raw host/device
pointers and a ``hipStream_t``), so Python passes ``tensor.data_ptr()`` and
``torch.cuda.current_stream().cuda_stream``.  It is loaded AFTER ``import
torch`` so that its ``libamdhip64.so.7`` dependency resolves to the HIP
runtime torch already mapped (same soname): one runtime, one set of streams.

On a machine with a GPU the native library is mandatory: if it is missing
every GPU op raises instead of silently falling back (``require()``).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

from ..base.exceptions import NativeLibraryError, raise_for_code

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_native", "libskylark_hip.so")

_lock = threading.Lock()
_lib = None
_load_error = None

i32, i64, u64, f64, vp, cp = C.c_int, C.c_int64, C.c_uint64, C.c_double, C.c_void_p, C.c_char_p

# name -> argtypes (restype is always c_int error code unless listed in _RESTYPE)
SIGNATURES = {
    "sl_version": [],
    "sl_ust_noreplace_host": [vp, u64, u64, i64, i64],
    "sl_fastfood_perms_host": [vp, u64, u64, i64, i64],
    "sl_last_error": [],
    "sl_fill_random": [vp, i32, i32, u64, u64, i64, i64, i64, i64, i64, i64, i64, i64, f64, f64, f64, i32, vp],
    "sl_fill_random_host": [vp, i32, i32, u64, u64, i64, i64, i64, i64, i64, i64, i64, i64, f64, f64, f64, i32],
    "sl_random_int": [vp, u64, u64, i64, i64, i64, vp],
    "sl_random_int_host": [vp, u64, u64, i64, i64, i64],
    "sl_threefry": [vp, u64, u64, i64, vp],
    "sl_threefry_host": [vp, u64, u64, u64, u64],
    "sl_halton": [vp, vp, i64, i64, i64, i64, vp],
    "sl_halton_host": [vp, vp, i64, i64, i64, i64],
    "sl_uniform_prefix_host": [vp, u64, u64, i64],
    "sl_dct2_rows": [vp, i64, i64, vp, f64, vp, i32, i64, i32, vp],
}
_RESTYPE = {"sl_last_error": cp}


def _try_build():
    """Build in-tree if the .so is absent (CPU container: hipcc cross-compiles)."""
    from .._native import build as _b
    return _b.build()


def load(build_if_missing: bool = True):
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        try:
            if not os.path.exists(LIB_PATH) and build_if_missing and os.environ.get("SKH_NO_BUILD") != "1":
                _try_build()
            lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
            for name, args in list(SIGNATURES.items()):
                fn = getattr(lib, name, None)
                if fn is None:
                    continue
                fn.argtypes = args
                fn.restype = _RESTYPE.get(name, C.c_int)
            _lib = lib
        except Exception as e:  # noqa: BLE001
            _load_error = e
            _lib = None
    return _lib


def register(name: str, argtypes, restype=C.c_int):
    """Declare a native symbol (used by op modules for their own kernels)."""
    SIGNATURES[name] = argtypes
    if restype is not C.c_int:
        _RESTYPE[name] = restype
    if _lib is not None:
        fn = getattr(_lib, name, None)
        if fn is not None:
            fn.argtypes = argtypes
            fn.restype = restype


def available() -> bool:
    return load() is not None


def require():
    lib = load()
    if lib is None:
        raise NativeLibraryError(
            f"native library {LIB_PATH} could not be loaded ({_load_error}); "
            "run `python -m libskylark_amd._native.build`")
    return lib


def call(name: str, *args):
    """Call an ``sl_*`` function and translate its error code."""
    lib = require()
    fn = getattr(lib, name, None)
    if fn is None:
        raise NativeLibraryError(f"native symbol {name} missing from {LIB_PATH} (stale build?)")
    if fn.argtypes is None:
        if name not in SIGNATURES:
            # never call with ctypes' default int conversion: a 64-bit size or
            # stride would be passed as a 32-bit int with undefined upper bits
            raise NativeLibraryError(f"{name}: no registered signature (import the ops module that declares it)")
        fn.argtypes = SIGNATURES[name]
        fn.restype = _RESTYPE.get(name, C.c_int)
    rc = fn(*args)
    if rc != 0:
        msg = lib.sl_last_error()
        raise_for_code(rc, f"{name}: {msg.decode() if msg else ''}")
    return rc


def stream_of(t: torch.Tensor):
    """hipStream_t (as int) of the current stream on t's device."""
    if t.is_cuda:
        return torch.cuda.current_stream(t.device).cuda_stream
    return None


def ptr(t: torch.Tensor):
    return C.c_void_p(t.data_ptr())


DTYPE_CODE = {torch.float32: 0, torch.float64: 1, torch.bfloat16: 2, torch.float16: 3}


def dtype_code(dt: torch.dtype) -> int:
    try:
        return DTYPE_CODE[dt]
    except KeyError:
        raise NativeLibraryError(f"dtype {dt} not supported by native kernels") from None
