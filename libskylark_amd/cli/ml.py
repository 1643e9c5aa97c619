"""``skylark_ml``: BlockADMM training / testing / interactive prediction
(reference ``ml/skylark_ml.cpp:15-174``; flags from ``ml/options.hpp``).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m libskylark_amd.cli.ml \\
        -k 1 -g 10 -f 10000 -l 2 -r 1 -c 0.01 --trainfile train.libsvm --modelfile model.json
    python -m libskylark_amd.cli.ml --modelfile model.json --testfile test.libsvm
    python -m libskylark_amd.cli.ml --modelfile model.json < examples.libsvm

Training is data-parallel: every rank reads its byte range of the training
file (one GPU per rank) and BlockADMM reaches consensus with one all-reduce
per iteration.
"""
from __future__ import annotations

import sys

import torch

from .. import io as IO
from ..base.context import Context
from ..ml.hilbert import large_scale_kernel_learning, parse_options
from ..ml.model import HilbertModel
from ._common import setup, write_ascii


def _read(o, fname, comm, dev, min_d=0):
    if comm.size > 1:
        X, Y = IO.read_libsvm_dist(fname, comm, min_d=min_d, dtype=torch.float64, device=dev)
        return X.local, Y.local[:, 0]
    X, Y = IO.read(o.fileformat if o.fileformat in (0, 1) else o.fileformat, fname, min_d=min_d)
    return X.to(dev), Y.to(dev)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if "-h" in argv or "--help" in argv:
        from ..ml.hilbert import build_parser
        build_parser().print_help()
        return 0
    o = parse_options(argv)
    comm, dev = setup()
    ctx = Context(o.seed)
    if o.trainfile:
        if comm.rank == 0:
            print("Reading training data...", flush=True)
        X, Y = _read(o, o.trainfile, comm, dev)
        Xv = Yv = None
        if o.valfile:
            Xv, Yv = _read(o, o.valfile, comm, dev, X.shape[1])
        large_scale_kernel_learning(comm, X.to(torch.float32) if dev.type == "cuda" else X, Y, ctx, o, Xv, Yv)
        return 0
    model = HilbertModel.load(o.modelfile)
    if o.testfile:
        X, Y = _read(o, o.testfile, comm, dev, model.get_input_size())
        X = X[:, :model.get_input_size()]
        labels, DV = model.predict(X.to(torch.float64))
        Y = Y.to(DV.device)
        if model.is_regression():
            st = torch.stack([((DV[:, 0] - Y) ** 2).sum(), (Y ** 2).sum()]).to(torch.float64)
            comm.all_reduce(st)
            if o.outputfile and comm.rank == 0:
                write_ascii(DV, o.outputfile + ".txt")
            if comm.rank == 0:
                print(f"Test error: {float((st[0] / st[1]).sqrt()):.4e}")
        else:
            st = torch.tensor([float((labels.to(Y.device) == Y).sum()), float(Y.numel())], dtype=torch.float64)
            comm.all_reduce(st)
            if o.outputfile and comm.rank == 0:
                write_ascii(DV if o.decisionvals else labels, o.outputfile + ".txt")
            if comm.rank == 0:
                print(f"Test error: {(st[1] - st[0]) * 100.0 / st[1]:.2f}%")
        return 0
    # interactive: one LIBSVM-style example per stdin line (no label)
    d = model.get_input_size()
    for line in sys.stdin:
        if not line.strip():
            break
        x = torch.zeros(1, d, dtype=torch.float64)
        for tok in line.split():
            if ":" in tok:
                i, v = tok.split(":", 1)
                x[0, int(i) - 1] = float(v)
        labels, DV = model.predict(x)
        print(float(DV[0, 0]) if model.is_regression() else int(labels[0]), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
