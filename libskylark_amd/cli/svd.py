"""``skylark_svd``: randomized SVD of a LIBSVM / arc-list matrix or a random
profile matrix (reference ``nla/skylark_svd.cpp:21-476``, same flags).

    python -m libskylark_amd.cli.svd -k 10 --prefix usps usps.train
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m libskylark_amd.cli.svd --profile 1000000 1000 -k 20

Writes ``<prefix>.U.txt``, ``<prefix>.S.txt``, ``<prefix>.V.txt`` (rank 0).
The ``--profile m n`` mode generates a uniform random matrix (the reference's
built-in benchmark) distributed as [VC,*] row blocks, one block per GPU.
"""
from __future__ import annotations

import argparse
import sys

import torch

from .. import nla
from ..base import distributions as D
from ..base.context import Context
from ..parallel.distmatrix import DistMatrix
from ._common import Timer, setup, write_ascii


def build_parser():
    p = argparse.ArgumentParser(prog="skylark_svd", description="Usage: skylark_svd [options] input-file-name")
    p.add_argument("inputfile", nargs="?", help="Input file (libsvm format by default).")
    p.add_argument("--filetype", default="LIBSVM", help="Input file type (LIBSVM or ARC_LIST).")
    p.add_argument("-d", "--directory", action="store_true", help="inputfile is a directory of files.")
    p.add_argument("-s", "--seed", type=int, default=38734)
    p.add_argument("--hdfs", default="", help="HDFS namenode (or any fsspec URL prefix); input is streamed.")
    p.add_argument("--port", type=int, default=0)
    p.add_argument("-k", "--rank", type=int, default=6, help="Target rank.")
    p.add_argument("-i", "--powerits", type=int, default=2, help="Number of power iterations.")
    p.add_argument("--skipqr", action="store_true")
    p.add_argument("-r", "--ratio", type=int, default=2)
    p.add_argument("-a", "--additive", type=int, default=0)
    p.add_argument("--symmetric", action="store_true")
    p.add_argument("--lower", action="store_true")
    p.add_argument("--sparse", action="store_true")
    p.add_argument("--single", action="store_true", help="Single precision instead of double.")
    p.add_argument("--bf16", action="store_true", help="bf16 storage of A (MI355X fused path).")
    p.add_argument("--profile", type=int, nargs="+", help="Generate a random m x n matrix (profile mode).")
    p.add_argument("--prefix", default="out")
    p.add_argument("--cpu", action="store_true")
    return p


def _read_inputs(a, comm, dev, dtype):
    import os
    from .. import io as IO
    if a.hdfs:
        url = IO.hdfs_url(a.hdfs if not getattr(a, "port", 0) else f"{a.hdfs}:{a.port}", a.inputfile)
        if a.filetype.upper() == "ARC_LIST":
            raise SystemExit("ARC_LIST input from HDFS is not supported; use LIBSVM")
        A = IO.read_libsvm_stream(url, sparse=a.sparse, dtype=dtype, device=dev,
                                  comm=comm if comm.size > 1 else None)[0]
        return A
    files = [a.inputfile]
    if a.directory:
        files = sorted(os.path.join(a.inputfile, f) for f in os.listdir(a.inputfile))
    if a.filetype.upper() == "ARC_LIST":
        A = IO.read_arc_list(files[0], symmetrize=True, comm=comm if comm.size > 1 else None, dtype=dtype)
        return A if isinstance(A, DistMatrix) else A.to(dev)
    if len(files) == 1:
        if comm.size > 1:
            return IO.read_libsvm_dist(files[0], comm, sparse=a.sparse, dtype=dtype, device=dev)[0]
        return IO.read_libsvm(files[0], sparse=a.sparse, dtype=dtype, device=dev)[0]
    # directory: the concatenation of all files (ReadDirLIBSVM; [VC,*] rows with several ranks)
    if comm.size > 1:
        return IO.read_dir_libsvm(a.inputfile, sparse=a.sparse, dtype=dtype, device=dev, comm=comm)[0]
    return IO.read_dir_libsvm(a.inputfile, sparse=a.sparse, dtype=dtype, device=dev)[0]


def main(argv=None):
    a = build_parser().parse_args(argv)
    if not a.profile and not a.inputfile:
        print("Input file is required.")
        return -1
    if a.profile and len(a.profile) < 2:
        print("Please specify height and width for --profile.")
        return -1
    comm, dev = setup(a.cpu)
    ctx = Context(a.seed)
    dtype = torch.bfloat16 if a.bf16 else (torch.float32 if a.single else torch.float64)
    params = nla.ApproximateSVDParams(oversampling_ratio=a.ratio, oversampling_additive=a.additive,
                                      num_iterations=a.powerits, skip_qr=a.skipqr)
    T = Timer(comm)
    if a.profile:
        T.start("Generating random matrix... ")
        m, n = a.profile[0], a.profile[1]
        arr = ctx.allocate_random_samples_array(m * n, D.Uniform(0.0, 1.0))
        A = DistMatrix.random((m, n), "VC_STAR", comm, dist=D.Uniform(0.0, 1.0), seed=arr.seed, base=arr.base,
                              dtype=dtype, device=dev)
        if comm.size == 1:
            A = A.local
        T.done()
    else:
        T.start("Reading the matrix... ")
        A = _read_inputs(a, comm, dev, dtype if dtype != torch.bfloat16 else torch.float32)
        T.done()
    T.start("Computing approximate SVD... ")
    if a.symmetric:
        if a.profile:
            raise SystemExit("Uniform symmetric matrix generating not supported yet.")
        Ag = A.to_global() if isinstance(A, DistMatrix) else A
        V, S = nla.approximate_symmetric_svd(Ag, a.rank, ctx, params, uplo="L" if a.lower else "U")
        U = None
    else:
        U, S, V = nla.approximate_svd(A, a.rank, ctx, params)
    T.done()
    T.start("Writing results... ")
    if U is not None and isinstance(U, DistMatrix):
        U = U.to_global()
    if comm.rank == 0:
        if U is not None:
            write_ascii(U, a.prefix + ".U.txt")
        write_ascii(S, a.prefix + ".S.txt")
        write_ascii(V.to_global() if isinstance(V, DistMatrix) else V, a.prefix + ".V.txt")
    T.done()
    return 0


if __name__ == "__main__":
    sys.exit(main())
