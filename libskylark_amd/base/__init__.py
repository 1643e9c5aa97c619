"""Base layer: context, random streams, distributions, QMC, exceptions,
random matrices, sparse matrices, cross-type BLAS, parameters."""
from . import distributions, exceptions, quasirand  # noqa: F401
from .blas import (QR, Axpy, ColumnView, ComputedMatrix, DenseCopy, ExplicitUnitary, Gemm, Gemv,  # noqa: F401
                   Height, RowDot, RowView, Scale, Symm, Trsm, Width)
from .context import Context, RandomSamplesArray  # noqa: F401
from .exceptions import *  # noqa: F401,F403
from .params import Params, print_matrix  # noqa: F401
from .random_matrices import GaussianMatrix, RandomMatrix, UniformMatrix  # noqa: F401
from .sparse import DistSparseMatrix, GraphAdapter, SparseMatrix  # noqa: F401
