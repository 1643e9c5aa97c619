"""LIBSVM text IO (reference ``utility/io/libsvm_io.hpp:33-2006``, ``ml/io.hpp:529-865``).

Reading is native (``sl_libsvm_scan`` / ``sl_libsvm_fill``: memory-mapped
text, multi-threaded two-pass parse straight into CSR).  Distributed reading
is byte-range parallel: each rank parses only its line-aligned slice of the
file (no root bottleneck, no point-to-point shipping of blocks as in the
reference), the feature dimension is agreed with one all-reduce(max), and
the rows are rebalanced to the [VC,*] block layout with one all-to-all.

Examples are ROWS: ``X`` is n x d (dense or sparse CSR), ``Y`` n labels.
"""
from __future__ import annotations

import ctypes as C
import mmap
import os

import numpy as np
import torch

from ..ops import _lib as L
from ..parallel.comm import Comm, balanced_counts
from ..parallel.distmatrix import DistMatrix

L.register("sl_libsvm_range", [L.vp, L.i64, L.i32, L.i32, L.vp, L.vp])
L.register("sl_libsvm_scan", [L.vp, L.i64, L.i32, L.vp, L.vp, L.vp, L.vp])
L.register("sl_libsvm_fill", [L.vp, L.vp, L.vp, L.i32, L.i64, L.vp, L.vp, L.vp, L.vp])

_NTHREADS = max(1, min(16, (os.cpu_count() or 1)))


def _p(a):
    return C.c_void_p(a.ctypes.data)


class _Mapped:
    def __init__(self, fname):
        self.f = open(fname, "rb")
        self.size = os.fstat(self.f.fileno()).st_size
        if self.size:
            self.mm = mmap.mmap(self.f.fileno(), 0, access=mmap.ACCESS_READ)
            self.arr = np.frombuffer(self.mm, dtype=np.uint8)
            self.addr = self.arr.ctypes.data
        else:
            self.mm, self.arr, self.addr = None, None, 0

    def close(self):
        self.arr = None
        if self.mm is not None:
            self.mm.close()
        self.f.close()


def _parse(addr: int, start: int, end: int, max_n: int = -1):
    """Parse bytes [start, end) -> (labels, rowptr, cols, vals, maxidx)."""
    if end <= start:
        z = np.zeros(0, dtype=np.int64)
        return np.zeros(0), np.zeros(1, dtype=np.int64), z, np.zeros(0), 0
    stats = np.zeros(4, dtype=np.int64)
    ranges = np.zeros(2 * _NTHREADS, dtype=np.int64)
    counts = np.zeros(2 * _NTHREADS, dtype=np.int64)
    nch = np.zeros(1, dtype=np.int32)
    base = C.c_void_p(addr + start)
    L.call("sl_libsvm_scan", base, end - start, _NTHREADS, _p(stats), _p(ranges), _p(counts), _p(nch))
    rows = int(stats[0]) if max_n < 0 else min(int(stats[0]), max_n)
    nnz = int(stats[1])
    labels = np.zeros(rows, dtype=np.float64)
    rowptr = np.zeros(rows + 1, dtype=np.int64)
    cols = np.zeros(nnz, dtype=np.int64)
    vals = np.zeros(nnz, dtype=np.float64)
    L.call("sl_libsvm_fill", base, _p(ranges), _p(counts), int(nch[0]), max_n, _p(labels), _p(rowptr), _p(cols),
           _p(vals))
    nnz = int(rowptr[-1])
    return labels, rowptr, cols[:nnz], vals[:nnz], int(stats[2])


def _rows_sorted(rowptr, cols) -> bool:
    """Column indices strictly increasing inside every row."""
    inc = np.diff(cols) > 0
    if len(inc) == 0:
        return True
    starts = rowptr[1:-1] - 1            # positions where a new row begins (diff across rows is free)
    starts = starts[(starts >= 0) & (starts < len(inc))]
    inc[starts] = True
    return bool(inc.all())


def _to_tensor(labels, rowptr, cols, vals, d, sparse, dtype, device):
    n = len(labels)
    rp = np.asarray(rowptr, dtype=np.int64)
    cl = np.asarray(cols, dtype=np.int64)
    if len(cl) and not (np.all(np.diff(cl) > 0) or _rows_sorted(rp, cl)):
        # entries out of order / repeated within a row (legal LIBSVM): sort, sum duplicates
        rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
        coo = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, cl])), torch.from_numpy(vals).to(dtype), (n, d))
        X = coo.coalesce().to_sparse_csr()
    else:
        X = torch.sparse_csr_tensor(torch.from_numpy(rp), torch.from_numpy(cl), torch.from_numpy(vals).to(dtype),
                                    (n, d), check_invariants=True)
    if not sparse:
        X = X.to_dense()
    if device is not None:
        X = X.to(device)
    return X, torch.from_numpy(labels).to(device) if device is not None else torch.from_numpy(labels)


def read_libsvm(fname: str, min_d: int = 0, max_n: int = -1, sparse: bool = False, dtype=torch.float64,
                device=None):
    """Local read: returns ``(X, Y)`` with ``X`` n x d (``d = max(max index, min_d)``)."""
    L.require()
    m = _Mapped(fname)
    try:
        labels, rowptr, cols, vals, maxidx = _parse(m.addr, 0, m.size, max_n)
    finally:
        m.close()
    return _to_tensor(labels, rowptr, cols, vals, max(maxidx, min_d), sparse, dtype, device)


def read_dir_libsvm(dirname: str, min_d: int = 0, max_n: int = -1, sparse: bool = False, dtype=torch.float64,
                    device=None, comm: Comm | None = None):
    """Read every file of a directory (sorted by name) as one LIBSVM dataset
    (reference ``ReadDirLIBSVM``, ``utility/io/libsvm_io.hpp:926-1483``): the
    rows are concatenated in file order and ``d`` is the largest index over
    all files.  With ``comm`` (several ranks) the files are split over the
    ranks in contiguous runs and the result is a ``[VC,*]`` DistMatrix pair."""
    import os
    files = sorted(os.path.join(dirname, f) for f in os.listdir(dirname)
                   if os.path.isfile(os.path.join(dirname, f)) and not f.startswith("."))
    if not files:
        raise FileNotFoundError(f"no files in {dirname}")
    dist = comm is not None and comm.size > 1
    mine = files
    if dist:
        from ..parallel.comm import balanced_offsets
        off = balanced_offsets(len(files), comm.size)
        mine = files[off[comm.rank]:off[comm.rank + 1]]
    parts, labels, d = [], [], min_d
    for f in mine:
        m = _Mapped(f)
        try:
            lab, rowptr, cols, vals, maxidx = _parse(m.addr, 0, m.size, -1)
        finally:
            m.close()
        parts.append((lab, rowptr, cols, vals))
        d = max(d, maxidx)
    if dist:
        dt = torch.tensor([d], dtype=torch.int64, device=comm.collective_device())
        comm.all_reduce_max(dt)
        d = int(dt.item())
    Xs, Ys = [], []
    for lab, rowptr, cols, vals in parts:
        X, Y = _to_tensor(lab, rowptr, cols, vals, d, True, dtype, None)
        Xs.append(X)
        Ys.append(Y)
    if Xs:
        X = torch.cat([x.to_sparse_coo() for x in Xs], 0).coalesce().to_sparse_csr()
        Y = torch.cat(Ys)
    else:
        X = torch.sparse_csr_tensor(torch.zeros(1, dtype=torch.int64), torch.zeros(0, dtype=torch.int64),
                                    torch.zeros(0, dtype=dtype), (0, d))
        Y = torch.zeros(0, dtype=torch.float64)
    if max_n >= 0 and not dist:
        X, Y = X.to_dense()[:max_n].to_sparse_csr(), Y[:max_n]
    if not sparse:
        X = X.to_dense()
    X, Y = X.to(device) if device is not None else X, Y.to(device) if device is not None else Y
    if not dist:
        return X, Y
    from ..parallel.comm import balanced_counts
    cnt = torch.tensor([X.shape[0]], dtype=torch.int64, device=comm.collective_device())
    have = [int(c) for c in comm.all_gather(cnt, 0).tolist()]
    n = sum(have)
    # the file split need not match the balanced row blocks: rebalance
    Xl, Yl = _rebalance(comm, X.to_dense() if X.layout != torch.strided else X, Y, have, balanced_counts(n, comm.size))
    if sparse:
        Xl = Xl.to_sparse_csr()
    return (DistMatrix(Xl, (n, d), "VC_STAR", comm), DistMatrix(Yl[:, None].contiguous(), (n, 1), "VC_STAR", comm))


ReadDirLIBSVM = read_dir_libsvm


def read_libsvm_dist(fname: str, comm: Comm | None = None, min_d: int = 0, sparse: bool = False,
                     dtype=torch.float64, device=None):
    """Distributed read: returns ``(X, Y)`` as [VC,*] DistMatrices (rows balanced)."""
    L.require()
    comm = comm or Comm(None)
    m = _Mapped(fname)
    try:
        s, e = np.zeros(1, dtype=np.int64), np.zeros(1, dtype=np.int64)
        if m.size:
            L.call("sl_libsvm_range", C.c_void_p(m.addr), m.size, comm.rank, comm.size, _p(s), _p(e))
        labels, rowptr, cols, vals, maxidx = _parse(m.addr, int(s[0]), int(e[0]))
    finally:
        m.close()
    st = torch.tensor([len(labels), max(maxidx, min_d)], dtype=torch.int64)
    if comm.size > 1:
        allst = comm.all_gather_object((len(labels), max(maxidx, min_d)))
    else:
        allst = [(int(st[0]), int(st[1]))]
    d = max(x[1] for x in allst)
    have = [x[0] for x in allst]
    n = sum(have)
    want = balanced_counts(n, comm.size)
    X, Y = _to_tensor(labels, rowptr, cols, vals, d, False, dtype, None)
    if comm.size > 1:
        X, Y = _rebalance(comm, X, Y, have, want)
    if sparse:
        X = X.to_sparse_csr()
    if device is not None:
        X, Y = X.to(device), Y.to(device)
    return (DistMatrix(X, (n, d), "VC_STAR", comm), DistMatrix(Y[:, None].contiguous(), (n, 1), "VC_STAR", comm))


def _rebalance(comm: Comm, X, Y, have, want):
    """Move rows from the byte-range partition ``have`` to the block layout ``want``."""
    me = comm.rank
    hs = int(np.sum(have[:me]))
    XY = torch.cat([X, Y[:, None].to(X.dtype)], dim=1)
    sends = []
    ws = np.concatenate([[0], np.cumsum(want)])
    for r in range(comm.size):
        lo, hi = max(hs, int(ws[r])), min(hs + have[me], int(ws[r + 1]))
        sends.append(XY[lo - hs:hi - hs].contiguous() if hi > lo else XY[:0].contiguous())
    recv = comm.all_to_all_v(sends)
    out = torch.cat(recv, dim=0)
    return out[:, :-1].contiguous(), out[:, -1].contiguous()


def write_libsvm(fname: str, X, Y, precision: int = 17):
    """Write rows of X (dense or sparse) with labels Y; zero entries are skipped."""
    if isinstance(X, DistMatrix):
        X = X.to_global()
    if isinstance(Y, DistMatrix):
        Y = Y.to_global()
    Xc = X.detach().cpu()
    Y = torch.as_tensor(Y).reshape(-1).cpu().tolist()
    if Xc.layout == torch.strided:
        Xc = Xc.to_sparse_csr()
    Xc = Xc.to_sparse_csr()
    rp, ci, va = Xc.crow_indices().tolist(), Xc.col_indices().tolist(), Xc.values().tolist()
    with open(fname, "w") as f:
        for i, lab in enumerate(Y):
            lab_s = str(int(lab)) if float(lab).is_integer() else repr(float(lab))
            parts = [lab_s] + [f"{ci[k] + 1}:{va[k]:.{precision}g}" for k in range(rp[i], rp[i + 1]) if va[k] != 0]
            f.write(" ".join(parts) + "\n")


ReadLIBSVM = read_libsvm
WriteLIBSVM = write_libsvm
