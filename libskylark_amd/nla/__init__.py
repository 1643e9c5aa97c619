"""Sketch-accelerated numerical linear algebra (reference ``nla/``)."""
from .svd import (ApproximateSVD, ApproximateSVDParams, ApproximateSymmetricSVD, PowerIteration,  # noqa: F401
                  approximate_svd, approximate_svd_params_t, approximate_symmetric_svd, power_iteration)
