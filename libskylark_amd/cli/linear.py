"""``skylark_linear``: least squares on a LIBSVM file (reference
``nla/skylark_linear.cpp:18-201``): ``--highprecision`` runs Blendenpik-LSQR
(FasterLeastSquares), otherwise FJLT sketch-and-solve (ApproximateLeastSquares).
The solution is written to ``<outputfile>.txt``."""
from __future__ import annotations

import argparse
import sys

import torch

from .. import io as IO
from .. import nla
from ..base.context import Context
from ..parallel.distmatrix import DistMatrix
from ._common import Timer, host_if_small, setup, write_ascii


def build_parser():
    p = argparse.ArgumentParser(prog="skylark_linear")
    p.add_argument("inputfile", nargs="?")
    p.add_argument("outputfile", nargs="?", default="out")
    p.add_argument("-d", "--directory", action="store_true")
    p.add_argument("-s", "--seed", type=int, default=38734)
    p.add_argument("--hdfs", default="")
    p.add_argument("--port", type=int, default=0)
    p.add_argument("-p", "--highprecision", action="store_true", help="Solve to high precision.")
    p.add_argument("-f", "--single", action="store_true", help="Single precision instead of double.")
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--gpu", action="store_true", help="use the GPU even for small problems")
    return p


def main(argv=None):
    a = build_parser().parse_args(argv)
    if not a.inputfile:
        print("Input file is required.")
        return -1
    comm, dev = setup(a.cpu)
    ctx = Context(a.seed)
    dt = torch.float32 if a.single else torch.float64
    T = Timer(comm)
    T.start("Reading the matrix... ")
    if a.hdfs:
        # file or directory on HDFS (or any fsspec URL), streamed block by block
        url = IO.hdfs_url(a.hdfs if not a.port else f"{a.hdfs}:{a.port}", a.inputfile)
        A, b = IO.read_libsvm_stream(url, dtype=dt, device=dev, comm=comm if comm.size > 1 else None)
        if comm.size == 1:
            b = b[:, None]
    elif a.directory:
        A, b = IO.read_dir_libsvm(a.inputfile, dtype=dt, device=dev, comm=comm if comm.size > 1 else None)
        if comm.size == 1:
            b = b[:, None]
    elif comm.size > 1:
        A, b = IO.read_libsvm_dist(a.inputfile, comm, dtype=dt, device=dev)
    else:
        A, b = IO.read_libsvm(a.inputfile, dtype=dt, device=dev)
        b = b[:, None]
        sdev = host_if_small(dev, A.shape[0] * A.shape[1], comm, a.gpu)
        A, b = A.to(sdev), b.to(sdev)
    T.done()
    T.start("Solving the least squares problem... ")
    if a.highprecision:
        x = nla.faster_least_squares(A, b, ctx)
    else:
        x = nla.approximate_least_squares(A, b, ctx)
    T.done()
    T.start("Writing results... ")
    if comm.rank == 0:
        write_ascii(x.to_global() if isinstance(x, DistMatrix) else x, a.outputfile + ".txt")
    T.done()
    return 0


if __name__ == "__main__":
    sys.exit(main())
