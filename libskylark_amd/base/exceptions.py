"""Exception hierarchy and error codes.

Mirrors the reference's Boost.Exception hierarchy and its integer codes
(``base/exception.hpp:33-245``) and the Python binding's error classes
(``python-skylark/skylark/errors.py``): C ABI functions return an ``int``
code, Python raises the matching class.
"""
from __future__ import annotations


class SkylarkError(Exception):
    code = 100


class AllocationError(SkylarkError):
    code = 101


class UnsupportedMatrixDistributionError(SkylarkError):
    code = 102


class UnsupportedError(SkylarkError):
    """Unsupported transform / input / output combination."""
    code = 103


class DimensionMismatchError(SkylarkError, ValueError):
    code = 104


# reference python binding spelling (errors.py)
DimensionMistmatchError = DimensionMismatchError


class CombBLASError(SkylarkError):
    code = 105


class NativeLibraryError(SkylarkError, RuntimeError):
    """HIP/native layer failure (the reference's 'lower layer' error)."""
    code = 106


LowerLayerError = NativeLibraryError


class IOError_(SkylarkError):
    code = 107


class NLAError(SkylarkError):
    code = 108


class InvalidParametersError(SkylarkError, ValueError):
    code = 109


InvalidObjectError = InvalidParametersError
# python-skylark errors.py spellings
InvalidParamterError = InvalidParametersError
ParameterMistmatchError = DimensionMismatchError


class UnsupportedBaseOperation(SkylarkError):
    code = 110


class MLError(SkylarkError):
    code = 111


_BY_CODE = {c.code: c for c in (SkylarkError, AllocationError, UnsupportedMatrixDistributionError,
                                UnsupportedError, DimensionMismatchError, CombBLASError,
                                NativeLibraryError, IOError_, NLAError, InvalidParametersError,
                                UnsupportedBaseOperation, MLError)}


def error_class(code: int):
    return _BY_CODE.get(code, SkylarkError)


def raise_for_code(code: int, msg: str = ""):
    cls = error_class(code)
    raise cls(f"[{code}] {msg}")


def strerror(code: int) -> str:
    return {0: "success"}.get(code, error_class(code).__name__)
