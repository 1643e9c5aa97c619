"""Shared plumbing for the command-line tools.

Launch one process per GPU with ``torchrun`` (``--master-addr 127.0.0.1``);
each rank binds ``cuda:LOCAL_RANK`` and joins the RCCL process group.  A plain
``python -m libskylark_amd.cli.<tool>`` runs single-process (GPU 0 if present).
"""
from __future__ import annotations

import os
import time

import torch

from ..parallel.comm import init_distributed


def setup(cpu: bool = False):
    """Returns ``(comm, device)``."""
    use_gpu = torch.cuda.is_available() and not cpu
    comm = init_distributed(device="cuda" if use_gpu else "cpu")
    if use_gpu:
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(lr)
        dev = torch.device("cuda", lr)
    else:
        dev = torch.device("cpu")
    _warm_up(dev)
    return comm, dev


def _warm_up(dev):
    """Runtime initialisation outside the timed phases (the reference's
    ``El::Initialize`` / MPI start-up is not timed either): load the native
    library and, on a GPU, create the BLAS / solver handles with tiny calls."""
    from ..ops import _lib
    _lib.load()
    if dev.type == "cuda":
        # BLAS kernels are loaded per (dtype, transpose) variant on first use:
        # touch the f32 / f64 NN, TN and NT GEMMs and the solver paths once
        for dt in (torch.float32, torch.float64):
            a = torch.ones(64, 64, dtype=dt, device=dev)
            ((a @ a) + (a.t() @ a) + (a @ a.t())).sum().item()
        torch.linalg.qr(a)[0].sum().item()
        torch.linalg.cholesky_ex(a + 64 * torch.eye(64, dtype=a.dtype, device=dev))[0].sum().item()
    # Small problems stay on the host (host_if_small) even when a GPU is
    # present, so the host LAPACK / sparse paths are initialised as well.
    a = torch.eye(8, dtype=torch.float64) + 0.5
    torch.linalg.qr(a)
    torch.linalg.eigh(a)
    torch.linalg.svd(a)
    torch.sparse.mm(a.to_sparse_csr(), a)
    from ..ops.rng import fill_random
    from ..base.distributions import Normal
    fill_random(torch.empty(8, dtype=torch.float64), Normal(), 0, 0)


# Below this many matrix entries a single-process solve is latency bound:
# library initialisation and kernel launch latency on the GPU exceed the whole
# host computation (measured: skylark_linear on 8192 x 12 took 0.115 s on the
# MI355X vs 0.006 s on the host), so the tools keep such problems on the host
# unless --gpu is given.
SMALL_PROBLEM = 1 << 20


def host_if_small(dev, n_entries: int, comm, force_gpu: bool = False):
    if comm.size == 1 and not force_gpu and n_entries < SMALL_PROBLEM:
        # A problem this small runs in well under a millisecond on one core;
        # waking the intra-op thread pool costs more than it saves (and its
        # spin-up jitter was 10-25 ms in measurements of skylark_graph_se).
        torch.set_num_threads(1)
        return torch.device("cpu")
    return dev


class Timer:
    def __init__(self, comm, verbose=True):
        self.comm, self.verbose, self.t = comm, verbose, time.time()

    def start(self, msg: str):
        if self.verbose and self.comm.rank == 0:
            print(msg, end="", flush=True)
        self.t = time.time()

    def done(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if self.verbose and self.comm.rank == 0:
            print(f"took {time.time() - self.t:.2e} sec", flush=True)


def write_ascii(M: torch.Tensor, path: str):
    """Elemental ``El::Write(..., ASCII)`` style: one matrix row per line."""
    M = M.detach().to(torch.float64).cpu()
    if M.dim() == 1:
        M = M[:, None]
    with open(path, "w") as f:
        for row in M.tolist():
            f.write(" ".join(f"{v:.17g}" for v in row) + "\n")


def read_ascii(path: str) -> torch.Tensor:
    rows = []
    with open(path) as f:
        for line in f:
            if line.strip():
                rows.append([float(x) for x in line.split()])
    return torch.tensor(rows, dtype=torch.float64)
