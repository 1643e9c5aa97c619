"""``skylark_graph_se``: approximate adjacency spectral embedding of a graph
(reference ``ml/skylark_graph_se.cpp``).  Writes ``<prefix>.vec.txt`` (n x k)
and ``<prefix>.index.txt`` (row -> vertex) unless ``--numeric``."""
from __future__ import annotations

import argparse
import sys

from .. import nla
from ..base.context import Context
from ..ml.graph import SimpleGraph, approximate_ase
from ._common import Timer, host_if_small, setup, write_ascii


def build_parser():
    p = argparse.ArgumentParser(prog="skylark_graph_se")
    p.add_argument("graphfile_pos", nargs="?", default="", metavar="graphfile")
    p.add_argument("-g", "--graphfile", default="")
    p.add_argument("-s", "--seed", type=int, default=38734)
    p.add_argument("--hdfs", default="")
    p.add_argument("--port", type=int, default=0)
    p.add_argument("-k", "--rank", type=int, default=10)
    p.add_argument("-i", "--powerits", type=int, default=2)
    p.add_argument("--skipqr", action="store_true")
    p.add_argument("-r", "--ratio", type=int, default=2)
    p.add_argument("-a", "--additive", type=int, default=0)
    p.add_argument("-n", "--numeric", action="store_true")
    p.add_argument("--prefix", default="out")
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--gpu", action="store_true", help="use the GPU even for small graphs")
    return p


def main(argv=None):
    a = build_parser().parse_args(argv)
    a.graphfile = a.graphfile or a.graphfile_pos
    if not a.graphfile:
        raise SystemExit("skylark_graph_se: a graph file is required (positional or -g)")
    if a.hdfs:
        from ..io.remote import hdfs_url
        a.graphfile = hdfs_url(a.hdfs if not a.port else f"{a.hdfs}:{a.port}", a.graphfile)
    comm, dev = setup(a.cpu)
    T = Timer(comm)
    T.start("Reading the graph... ")
    G = SimpleGraph.from_file(a.graphfile)
    T.done()
    T.start("Computing embeddings... ")
    p = nla.ApproximateSVDParams(oversampling_ratio=a.ratio, oversampling_additive=a.additive,
                                 num_iterations=a.powerits, skip_qr=a.skipqr)
    n = G.num_vertices()
    X, indexmap = approximate_ase(G, a.rank, Context(a.seed), p, device=host_if_small(dev, n * n, comm, a.gpu))
    T.done()
    T.start("Writing results... ")
    if comm.rank == 0:
        write_ascii(X, a.prefix + ".vec.txt")
        if not a.numeric:
            with open(a.prefix + ".index.txt", "w") as f:
                for i, v in enumerate(indexmap):
                    f.write(f"{i}\t{v}\n")
    T.done()
    return 0


if __name__ == "__main__":
    sys.exit(main())
