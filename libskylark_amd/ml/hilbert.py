"""Large-scale kernel learning driver: options, solver factory, training entry.

Reference ``ml/hilbert.hpp:11-276`` (``GetSolver``, ``ShiftForLogistic``,
``LargeScaleKernelLearning``) and ``ml/options.hpp:26-381``
(``hilbert_options_t``: enums, defaults, command-line, ``print()`` header
written at the top of model files).  The same flags and integer codes are
accepted by the ``skylark_ml`` CLI (:mod:`libskylark_amd.cli.ml`).
"""
from __future__ import annotations

import argparse
import shlex
from dataclasses import dataclass, field

import torch

from ..base.context import Context
from ..parallel.comm import Comm
from .. import sketch as SK
from . import kernels as K
from .admm import BlockADMMSolver, num_targets

LOSSES = ["Squared Loss", "Least Absolute Deviations", "Hinge Loss (SVMs)", "Logistic Loss"]
REGULARIZERS = ["No Regularizer", "L2", "L1"]
SEQUENCES = ["Monte Carlo", "Leaped Halton"]
KERNELS = ["Linear", "Gaussian", "Polynomial", "Laplacian", "ExpSemigroup", "Matern"]
FILEFORMATS = ["libsvm-dense", "libsvm-sparse", "hdf5_dense", "hdf5_sparse"]
SQUARED, LAD, HINGE, LOGISTIC = range(4)
NOREG, L2, L1 = range(3)
MONTECARLO, LEAPED_HALTON = range(2)
K_LINEAR, K_GAUSSIAN, K_POLYNOMIAL, K_LAPLACIAN, K_EXPSEMIGROUP, K_MATERN = range(6)


@dataclass
class HilbertOptions:
    regression: bool = False
    decisionvals: bool = False
    lossfunction: int = SQUARED
    regularizer: int = NOREG
    kernel: int = K_LINEAR
    kernelparam: float = 1.0
    kernelparam2: float = 0.0
    kernelparam3: float = 1.0
    lam: float = 0.0
    tolerance: float = 0.001
    rho: float = 1.0
    seed: int = 12345
    randomfeatures: int = 0
    numfeaturepartitions: int = 1
    numthreads: int = 1
    usefast: bool = False
    seqtype: int = MONTECARLO
    cachetransforms: bool = False
    fileformat: int = 0
    MAXITER: int = 20
    trainfile: str = ""
    modelfile: str = ""
    valfile: str = ""
    testfile: str = ""
    outputfile: str = ""
    cmdline: str = ""
    exit_on_return: bool = False

    @property
    def lambda_(self):
        return self.lam

    def print(self) -> str:
        """Model-file header (reference ``hilbert_options_t::print``)."""
        o = ["# Generated using skylark_ml using the following command-line: ", f"#\t{self.cmdline}", "#",
             f"# Regression? = {self.regression}", f"# Training File = {self.trainfile}",
             f"# Model File = {self.modelfile}", f"# Validation File = {self.valfile}",
             f"# Test File = {self.testfile}", f"# File Format = {self.fileformat}",
             f"# Loss function = {self.lossfunction} ({LOSSES[self.lossfunction]})",
             f"# Regularizer = {self.regularizer} ({REGULARIZERS[self.regularizer]})",
             f"# Kernel = {self.kernel} ({KERNELS[self.kernel]})", f"# Kernel Parameter = {self.kernelparam}",
             f"# Second Kernel Parameter = {self.kernelparam2}", f"# Third Kernel Parameter = {self.kernelparam3}",
             f"# Regularization Parameter = {self.lam}", f"# Maximum Iterations = {self.MAXITER}",
             f"# Tolerance = {self.tolerance}", f"# rho = {self.rho}", f"# Seed = {self.seed}",
             f"# Random Features = {self.randomfeatures}", f"# Cache transforms? = {self.cachetransforms}",
             f"# Use fast, if availble? = {self.usefast}",
             f"# Sequence = {self.seqtype} ({SEQUENCES[self.seqtype]})",
             f"# Number of feature partitions = {self.numfeaturepartitions}",
             f"# Threads = {self.numthreads}", "#"]
        return "\n".join(o) + "\n"


hilbert_options_t = HilbertOptions


def build_parser(prog="skylark_ml") -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog=prog, description="Usage: skylark_ml [options] --trainfile trainfile "
                                "--modelfile modelfile\nUsage: skylark_ml --modelfile modelfile --testfile testfile")
    a = p.add_argument
    a("-l", "--lossfunction", type=int, default=SQUARED, help="Loss function (0:SQUARED, 1:LAD, 2:HINGE, 3:LOGISTIC)")
    a("-r", "--regularizer", type=int, default=NOREG, help="Regularizer (0:None, 1:L2, 2:L1)")
    a("-k", "--kernel", type=int, default=K_LINEAR,
      help="Kernel (0:LINEAR, 1:GAUSSIAN, 2:POLYNOMIAL, 3:LAPLACIAN, 4:EXPSEMIGROUP, 5:MATERN)")
    a("-g", "--kernelparam", type=float, default=1.0, help="Kernel Parameter")
    a("-x", "--kernelparam2", type=float, default=0.0, help="Second Kernel Parameter (Polynomial: c)")
    a("-y", "--kernelparam3", type=float, default=1.0, help="Third Kernel Parameter (Polynomial: gamma)")
    a("-c", "--lambda", dest="lam", type=float, default=0.0, help="Regularization Parameter")
    a("-e", "--tolerance", type=float, default=0.001)
    a("--rho", type=float, default=1.0, help="ADMM rho parameter")
    a("-s", "--seed", type=int, default=12345)
    a("-f", "--randomfeatures", type=int, default=0)
    a("-n", "--numfeaturepartitions", type=int, default=1)
    a("-t", "--numthreads", type=int, default=1)
    a("--regression", action="store_true")
    a("--usefast", action="store_true")
    a("-q", "--usequasi", dest="seqtype", type=int, default=MONTECARLO)
    a("--cachetransforms", action="store_true")
    a("--decisionvals", action="store_true")
    a("--fileformat", type=int, default=0)
    a("-i", "--MAXITER", type=int, default=20)
    a("--trainfile", default="")
    a("--modelfile", default="")
    a("--valfile", default="")
    a("--testfile", default="")
    a("--outputfile", default="")
    a("positional", nargs="*")
    return p


def parse_options(argv) -> HilbertOptions:
    ns = build_parser().parse_args(argv)
    d = {k: v for k, v in vars(ns).items() if k != "positional"}
    pos = list(ns.positional)
    if pos and not d["trainfile"]:
        d["trainfile"] = pos.pop(0)
    if pos and not d["modelfile"]:
        d["modelfile"] = pos.pop(0)
    o = HilbertOptions(**d)
    o.cmdline = " ".join(shlex.quote(a) for a in ["skylark_ml", *argv])
    return o


def make_kernel(options: HilbertOptions, d: int):
    kp = options.kernelparam
    if options.kernel == K_LINEAR:
        return K.Linear(d)
    if options.kernel == K_GAUSSIAN:
        return K.Gaussian(d, kp)
    if options.kernel == K_POLYNOMIAL:
        return K.Polynomial(d, int(kp), options.kernelparam2, options.kernelparam3)
    if options.kernel == K_LAPLACIAN:
        return K.Laplacian(d, kp)
    if options.kernel == K_EXPSEMIGROUP:
        return K.ExpSemigroup(d, kp)
    if options.kernel == K_MATERN:
        return K.Matern(d, kp, options.kernelparam2)
    raise ValueError(f"unknown kernel code {options.kernel}")


def get_solver(context: Context, options: HilbertOptions, dimensions: int) -> BlockADMMSolver:
    """Reference ``GetSolver``: loss/regulariser/kernel/map-type from options."""
    reg = NOREG if options.lam == 0 else options.regularizer
    common = dict(loss=options.lossfunction, regularizer=reg, lam=options.lam)
    P = options.numfeaturepartitions
    k = make_kernel(options, dimensions)
    if options.kernel == K_LINEAR:
        if options.randomfeatures == 0:
            solver = BlockADMMSolver(NumFeatures=dimensions, NumFeaturePartitions=P, **common)
        else:
            from .admm import _partition
            _, sizes = _partition(options.randomfeatures, P)
            maps = [SK.CWT(dimensions, sj, context=context) for sj in sizes]
            solver = BlockADMMSolver(feature_maps=maps, scale_maps=True, **common)
    else:
        quasi_ok = options.kernel in (K_GAUSSIAN, K_LAPLACIAN, K_EXPSEMIGROUP)
        fast_ok = options.kernel in (K_GAUSSIAN, K_MATERN)
        if options.seqtype == LEAPED_HALTON and quasi_ok and not options.usefast:
            tag = "quasi"
        elif options.usefast and fast_ok:
            tag = "fast"
        else:
            tag = "regular"
        solver = BlockADMMSolver(NumFeatures=options.randomfeatures, kernel=k, tag=tag, NumFeaturePartitions=P,
                                 context=context, **common)
    solver.set_rho(options.rho)
    solver.set_maxiter(options.MAXITER)
    solver.set_tol(options.tolerance)
    solver.set_nthreads(options.numthreads)
    solver.set_cache_transform(options.cachetransforms)
    return solver


GetSolver = get_solver


def shift_for_logistic(Y: torch.Tensor) -> torch.Tensor:
    """±1 labels -> {0, 1} (reference ``ShiftForLogistic``)."""
    return 0.5 * (Y + 1.0)


def large_scale_kernel_learning(comm: Comm, X, Y, context: Context, options: HilbertOptions, Xv=None, Yv=None,
                                log=print):
    """Train with BlockADMM and save the model from rank 0.  Returns the model."""
    d = X.shape[1]
    targets = 1 if options.regression else num_targets(Y, comm)
    if not options.regression and options.lossfunction == LOGISTIC and targets == 1:
        Y = shift_for_logistic(Y)
        if Yv is not None:
            Yv = shift_for_logistic(Yv)
    solver = get_solver(context, options, d)
    model = solver.train(X, Y, Xv, Yv, options.regression, comm, log=log)
    if comm.rank == 0 and options.modelfile:
        model.save(options.modelfile, options.print())
    return model


LargeScaleKernelLearning = large_scale_kernel_learning
