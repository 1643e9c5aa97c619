"""Iterative algorithms (reference ``algorithms/``): Krylov, asynchronous, regression."""
from . import asynch, krylov, loss, operators, regression, regularizers  # noqa: F401
from .asynch import AsyFCG, AsyIterParams, AsyRGS, asy_fcg, asy_rgs  # noqa: F401
from .krylov import (CG, LSQR, ChebyshevLS, FlexibleCG, IdPrecond, KrylovIterParams, MatPrecond,  # noqa: F401
                     TriInversePrecond, cg, chebyshev_ls, flexible_cg, lsqr)
from .loss import HingeLoss, LADLoss, LogisticLoss, SquaredLoss, make_loss  # noqa: F401
from .regression import (AcceleratedRegressionSolver, RegressionProblem, RegressionSolver,  # noqa: F401
                         SketchedRegressionSolver)
from .regularizers import L1Regularizer, L2Regularizer, NoRegularizer, make_regularizer  # noqa: F401
