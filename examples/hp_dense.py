"""JLT sketch of a 2-D block-cyclic distributed dense matrix, columnwise and
rowwise (reference examples/hp_dense.cpp: JLT on an [MC,MR] Elemental matrix).

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 examples/hp_dense.py --m 20000 --n 1000 --s 500
    python examples/hp_dense.py            # single process
"""
import argparse

import torch

from _common import Timer, device

import libskylark_amd as sk
from libskylark_amd.parallel import DistMatrix, init_distributed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=4000)
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--s", type=int, default=100)
    ap.add_argument("--seed", type=int, default=38734)
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    comm = init_distributed()
    dev = device(a.device)
    ctx = sk.Context(a.seed)
    A = sk.base.GaussianMatrix(a.m, a.n, ctx, dtype=torch.float32, device=dev, layout="MC_MR", comm=comm)
    S = sk.sketch.JLT(a.m, a.s, context=ctx)
    with Timer("columnwise S*A ([MC,MR] -> [MC,MR])"):
        SA = S.apply(A, dim="columnwise")
    R = sk.sketch.JLT(a.n, a.s, context=ctx)
    with Timer("rowwise A*R^T ([MC,MR] -> [MC,MR])"):
        AR = R.apply(A, dim="rowwise")
    sa = SA.to_global() if isinstance(SA, DistMatrix) else SA
    ar = AR.to_global() if isinstance(AR, DistMatrix) else AR
    if comm.rank == 0:
        print(f"SA: {tuple(sa.shape)}  |SA|_F / |A|_F = {float(sa.norm()) / float(A.to_global().norm()):.3f}")
        print(f"AR^T: {tuple(ar.shape)}")


if __name__ == "__main__":
    main()
