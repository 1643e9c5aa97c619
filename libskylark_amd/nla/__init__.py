"""Sketch-accelerated numerical linear algebra (reference ``nla/``)."""
from .condest import CondEst, CondEstParams, CondEstResult, condest, condest_params_t  # noqa: F401
from .least_squares import (ApproximateLeastSquares, FasterLeastSquares, FasterLSParams,  # noqa: F401
                            approximate_least_squares, faster_least_squares, faster_ls_params_t,
                            lsrn_least_squares)
from .spectral import ChebyshevDiffMatrix, ChebyshevPoints, chebyshev_diff_matrix, chebyshev_points  # noqa: F401
from .svd import (ApproximateSVD, ApproximateSVDParams, ApproximateSymmetricSVD, PowerIteration,  # noqa: F401
                  approximate_svd, approximate_svd_params_t, approximate_symmetric_svd, power_iteration)
