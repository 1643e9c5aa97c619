"""Machine learning on sketches (reference ``ml/``): kernels, KRR/RLSC,
BlockADMM, models, graph analytics."""
from . import admm, coding, graph, hilbert, kernels, krr, model, nonlinear, rlsc  # noqa: F401
from .admm import BlockADMM, BlockADMMSolver  # noqa: F401
from .coding import DummyCoding, DummyDecode, dummy_coding, dummy_decode  # noqa: F401
from .graph import (ApproximateASE, FindLocalCluster, SimpleGraph, TimeDependentPPR, approximate_ase,  # noqa: F401
                    find_local_cluster, time_dependent_ppr)
from .hilbert import HilbertOptions, get_solver, large_scale_kernel_learning, parse_options  # noqa: F401
from .kernels import (ExpSemiGroup, ExpSemigroup, Gaussian, Gram, Kernel, Laplacian, Linear, Matern,  # noqa: F401
                      Polynomial, SymmetricGram, gram_dist, kernel, kernel_from_dict)
from .krr import (ApproximateKernelRidge, FasterKernelRidge, FeatureMapPrecond, KernelRidge, KrrParams,  # noqa: F401
                  LargeScaleKernelRidge, SketchedApproximateKernelRidge, approximate_kernel_ridge,
                  faster_kernel_ridge, kernel_ridge, krr_params_t, large_scale_kernel_ridge,
                  sketched_approximate_kernel_ridge)
from .model import FeatureExpansionModel, HilbertModel, KernelModel, load_model, model_from_dict  # noqa: F401
from .rlsc import (ApproximateKernelRLSC, FasterKernelRLSC, KernelRLSC, LargeScaleKernelRLSC,  # noqa: F401
                   SketchedApproximateKernelRLSC, approximate_kernel_rlsc, faster_kernel_rlsc, kernel_rlsc,
                   large_scale_kernel_rlsc, sketched_approximate_kernel_rlsc)
from .nonlinear import (RLS, NystromRLS, SketchPCR, SketchRLS, approximate_domsubspace_basis,  # noqa: F401
                        euclidean, nystromrls, rls, sketchpcr, sketchrls)
from . import nonlinear as distances  # noqa: F401  (python-skylark ml.distances.euclidean)
