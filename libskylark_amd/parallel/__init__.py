"""Distributed layer: process groups (RCCL/gloo), DistMatrix layouts, distributed ops."""
from .comm import Comm, balanced_counts, balanced_offsets, init_distributed, world  # noqa: F401
from .distmatrix import LAYOUTS, DistMatrix, Grid, canon  # noqa: F401
from .dist_sparse2d import DistSparse2D  # noqa: F401,E402
