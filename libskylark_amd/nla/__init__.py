"""Sketch-accelerated numerical linear algebra (reference ``nla/``)."""
from .condest import CondEst, CondEstParams, CondEstResult, condest, condest_params_t  # noqa: F401
from .least_squares import (ApproximateLeastSquares, FasterLeastSquares, FasterLSParams,  # noqa: F401
                            approximate_least_squares, faster_least_squares, faster_ls_params_t,
                            lsrn_least_squares)
from .spectral import ChebyshevDiffMatrix, ChebyshevPoints, chebyshev_diff_matrix, chebyshev_points  # noqa: F401
from .svd import (ApproximateSVD, ApproximateSVDParams, ApproximateSymmetricSVD, PowerIteration,  # noqa: F401
                  approximate_svd, approximate_svd_params_t, approximate_symmetric_svd, power_iteration)

# python-skylark names (python-skylark/skylark/nla/nla.py); its SVDParams
# defaults to two power iterations where the C++ parameter struct has none
from dataclasses import dataclass as _dataclass  # noqa: E402


@_dataclass
class SVDParams(ApproximateSVDParams):
    num_iterations: int = 2


FasterLeastSquaresParams = FasterLSParams
