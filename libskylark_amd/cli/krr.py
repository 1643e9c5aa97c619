"""``skylark_krr``: kernel ridge regression / RLSC trainer and predictor
(reference ``ml/skylark_krr.cpp:20-1167``: algorithms 0-5 + experimental
100/101, kernels Gaussian(0)/Laplacian(1)/Polynomial(2)/Linear(100),
``--predict`` mode with a saved model).

    python -m libskylark_amd.cli.krr -a 1 -k 0 -g 10 -l 0.01 -f 2000 --model m.json train.libsvm test.libsvm
    python -m libskylark_amd.cli.krr --predict --model m.json test.libsvm
"""
from __future__ import annotations

import argparse
import shlex
import sys

import torch

from .. import io as IO
from .. import ml
from ..base.context import Context
from ._common import Timer, setup, write_ascii

CLASSIC, FASTER, APPROXIMATE, SKETCHED, FAST_SKETCHED, LARGE_SCALE, EXP1, EXP2 = 0, 1, 2, 3, 4, 5, 100, 101


def build_parser():
    p = argparse.ArgumentParser(prog="skylark_krr")
    p.add_argument("trainfile", nargs="?", default="")
    p.add_argument("testfile", nargs="?", default="")
    p.add_argument("--trainfile", dest="trainfile_opt", default="")
    p.add_argument("--testfile", dest="testfile_opt", default="")
    p.add_argument("--outputfile", default="")
    p.add_argument("--predict", action="store_true")
    p.add_argument("--model", default="model.dat")
    p.add_argument("--logfile", default="")
    p.add_argument("-k", "--kernel", type=int, default=0)
    p.add_argument("-a", "--algorithm", type=int, default=FASTER)
    p.add_argument("-s", "--seed", type=int, default=38734)
    p.add_argument("-g", "--kernelparam", type=float, default=10.0)
    p.add_argument("-x", "--kernelparam2", type=float, default=0.0)
    p.add_argument("-y", "--kernelparam3", type=float, default=1.0)
    p.add_argument("-l", "--lambda", dest="lam", type=float, default=0.01)
    p.add_argument("-t", "--tolerance", type=float, default=0.0)
    p.add_argument("-c", "--maxsplit", type=int, default=0)
    p.add_argument("-i", "--maxit", type=int, default=0)
    p.add_argument("-p", "--partial", type=int, default=-1)
    p.add_argument("-z", "--sample", type=int, default=-1)
    p.add_argument("--decisionvals", action="store_true")
    p.add_argument("--single", action="store_true")
    p.add_argument("--fast", action="store_true")
    p.add_argument("--regression", action="store_true")
    p.add_argument("-f", "--numfeatures", type=int, default=2000)
    p.add_argument("-r", "--sketchsize", type=int, default=-1)
    p.add_argument("--fileformat", type=int, default=0)
    p.add_argument("--cpu", action="store_true")
    return p


def make_kernel(a, d):
    if a.kernel == 0:
        return ml.Gaussian(d, a.kernelparam)
    if a.kernel == 1:
        return ml.Laplacian(d, a.kernelparam)
    if a.kernel == 2:
        return ml.Polynomial(d, int(a.kernelparam), a.kernelparam2, a.kernelparam3)
    if a.kernel == 100:
        return ml.Linear(d)
    raise SystemExit(f"unknown kernel {a.kernel}")


def train(a, comm, dev, ctx, log):
    dt = torch.float32 if a.single else torch.float64
    T = Timer(comm)
    T.start("Reading the matrix... ")
    X, L = IO.read_libsvm(a.trainfile, max_n=a.partial, dtype=dt)
    if a.sample > 0 and a.sample < X.shape[0]:
        from ..base import distributions as D
        arr = ctx.allocate_random_samples_array(X.shape[0], D.Uniform())
        from ..ops import rng
        u = torch.empty(X.shape[0], 1, dtype=torch.float64)
        rng.fill_random(u, D.Uniform(), arr.seed, arr.base, ir=1, ic=X.shape[0])
        keep = torch.argsort(u[:, 0])[:a.sample].sort().values
        X, L = X[keep], L[keep]
    X, L = X.to(dev), L.to(dev)
    T.done()
    k = make_kernel(a, X.shape[1])
    p = ml.KrrParams(use_fast=a.fast, max_split=a.maxsplit, am_i_printing=comm.rank == 0, log_level=1)
    T.start("Training...\n")
    Yreg = L[:, None].to(dt)
    alg = a.algorithm
    if alg == CLASSIC:
        if a.regression:
            A, rc = ml.kernel_ridge(k, X, Yreg, a.lam, params=p), None
        else:
            A, rc = ml.kernel_rlsc(k, X, L, a.lam, params=p)
        model = ml.KernelModel(k, X, A, a.trainfile, a.partial, a.fileformat, rc)
    elif alg == FASTER:
        p.iter_lim = a.maxit or 1000
        p.tolerance = a.tolerance or 1e-3
        if a.regression:
            A, rc = ml.faster_kernel_ridge(k, X, Yreg, a.lam, a.numfeatures, ctx, params=p), None
        else:
            A, rc = ml.faster_kernel_rlsc(k, X, L, a.lam, a.numfeatures, ctx, params=p)
        model = ml.KernelModel(k, X, A, a.trainfile, a.partial, a.fileformat, rc)
    elif alg in (APPROXIMATE, EXP1, EXP2):
        p.sketched_rr = alg != APPROXIMATE
        p.fast_sketch = alg == EXP2
        if a.regression:
            (S, W), rc = ml.approximate_kernel_ridge(k, X, Yreg, a.lam, a.numfeatures, ctx, params=p), None
        else:
            S, W, rc = ml.approximate_kernel_rlsc(k, X, L, a.lam, a.numfeatures, ctx, params=p)
        model = ml.FeatureExpansionModel([S], W, False, rc)
    elif alg in (SKETCHED, FAST_SKETCHED):
        p.sketched_rr, p.sketch_size, p.fast_sketch = True, a.sketchsize, alg == FAST_SKETCHED
        if a.regression:
            sc, maps, W = ml.sketched_approximate_kernel_ridge(k, X, Yreg, a.lam, a.numfeatures, a.sketchsize, ctx,
                                                               params=p)
            rc = None
        else:
            sc, maps, W, rc = ml.sketched_approximate_kernel_rlsc(k, X, L, a.lam, a.numfeatures, a.sketchsize, ctx,
                                                                  params=p)
        model = ml.FeatureExpansionModel(maps, W, sc, rc)
    elif alg == LARGE_SCALE:
        p.iter_lim = a.maxit or 20
        p.tolerance = a.tolerance or 1e-1
        if a.regression:
            sc, maps, W = ml.large_scale_kernel_ridge(k, X, Yreg, a.lam, a.numfeatures, ctx, params=p)
            rc = None
        else:
            sc, maps, W, rc = ml.large_scale_kernel_rlsc(k, X, L, a.lam, a.numfeatures, ctx, params=p)
        model = ml.FeatureExpansionModel(maps, W, sc, rc)
    else:
        raise SystemExit(f"unknown algorithm {alg}")
    T.done()
    if a.model != "NOSAVE" and comm.rank == 0:
        header = ("# Generated using kernel_regression using the following command-line: \n"
                  f"#\t{log}\n# Number of ranks is {comm.size}\n")
        model.save(a.model, header)
    return model


def evaluate(a, model, comm, dev):
    X, L = IO.read_libsvm(a.testfile, min_d=model.get_input_size(), dtype=torch.float64)
    X = X[:, :model.get_input_size()].to(dev)
    labels, DV = model.predict(X)
    if model.regression:
        err = float((DV[:, 0].cpu() - L).norm() / L.norm())
        if comm.rank == 0:
            print(f"Test error: {err:.4e}")
    else:
        wrong = float((labels.cpu() != L).double().mean()) * 100
        if comm.rank == 0:
            print(f"Test error: {wrong:.2f}%")
    if a.outputfile and comm.rank == 0:
        write_ascii(DV if (model.regression or a.decisionvals) else labels, a.outputfile + ".txt")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    a = build_parser().parse_args(argv)
    a.trainfile = a.trainfile_opt or a.trainfile
    a.testfile = a.testfile_opt or a.testfile
    comm, dev = setup(a.cpu)
    ctx = Context(a.seed)
    if a.predict:
        model = ml.load_model(a.model)
        if not a.testfile:
            a.testfile = a.trainfile
        evaluate(a, model, comm, dev)
        return 0
    if not a.trainfile:
        print("Input training file is required.")
        return -1
    model = train(a, comm, dev, ctx, " ".join(shlex.quote(x) for x in ["skylark_krr", *argv]))
    if a.testfile:
        evaluate(a, model, comm, dev)
    return 0


if __name__ == "__main__":
    sys.exit(main())
