"""Data IO (reference ``utility/io/*``, ``ml/io.hpp``).

* LIBSVM: native multi-threaded parser, byte-range distributed reader,
  writer (:mod:`.libsvm`).
* Arc lists (edge lists): byte-range parallel read into a sparse adjacency
  (:func:`read_arc_list`), reference ``utility/io/arc_list.hpp``.
* HDF5: ``ReadHDF5``/``write_hdf5`` use h5py when present, otherwise the
  built-in reader/writer of ``io/h5.py`` (no libhdf5 needed).
* Remote / HDFS: :class:`LineStreamer`, :class:`LineStreamerIterator`,
  :func:`read_libsvm_stream` over fsspec URLs (:mod:`.remote`).
* :func:`read` — ``ml/io.hpp:869`` dispatch on fileformat code
  (0 libsvm-dense, 1 libsvm-sparse, 2 hdf5-dense, 3 hdf5-sparse).
"""
from __future__ import annotations

import numpy as np
import torch

from ..base.exceptions import IOError_
from .libsvm import (ReadDirLIBSVM, ReadLIBSVM, WriteLIBSVM, read_dir_libsvm, read_libsvm,  # noqa: F401
                     read_libsvm_dist, write_libsvm)
from .remote import (LineStreamer, LineStreamerIterator, ReadLIBSVMStream, hdfs_url,  # noqa: F401
                     read_libsvm_stream)

LIBSVM_DENSE, LIBSVM_SPARSE, HDF5_DENSE, HDF5_SPARSE = range(4)


def _h5py():
    try:
        import h5py  # noqa: F401
        return h5py
    except ImportError:
        return None


class _H5Native:
    """Adapter giving the built-in reader/writer (io/h5.py) h5py's File shape."""

    @staticmethod
    def File(fname, mode="r"):
        from .h5 import H5File
        if mode != "r":
            raise ValueError("the built-in HDF5 module reads via H5File and writes via write_h5")
        return H5File(fname)


def _h5_slice(f, name, axis, s0, s1):
    if hasattr(f, "read_slice"):                 # built-in reader (mmap hyperslab)
        return f.read_slice(name, axis, s0, s1)
    ds = f[name]                                 # h5py: hyperslab selection
    return np.asarray(ds[:, s0:s1] if axis == 1 else ds[s0:s1])


def read_hdf5(fname: str, max_n: int = -1, sparse: bool = False, dtype=torch.float64, comm=None):
    """Reference layout: datasets ``X`` (d x n, examples as columns) and ``Y``
    (also the python-skylark dataset names ``Features`` / ``Labels``); sparse
    files hold ``dimensions``, ``indptr``, ``indices``, ``values``.  Returns
    ``(X, Y)`` with examples as ROWS.  Uses h5py when importable, else the
    built-in reader (``io/h5.py``).

    With a multi-rank ``comm`` every rank reads only ITS balanced block of
    examples (a column hyperslab of ``X``, the matching ``indptr`` range and
    ``indices``/``values`` slices) and the result is a pair of ``[VC,*]``
    DistMatrices -- where the reference reads on rank 0 and ships chunks by
    send/recv (``ml/io.hpp:256-526``, ``utility/io/hdf5_io.hpp:148-262``)."""
    h5 = _h5py() or _H5Native
    dist = comm is not None and comm.size > 1
    with h5.File(fname, "r") as f:
        if "indptr" in f:
            dims = np.asarray(f["dimensions"])
            d, n = int(dims[0]), int(dims[1])
            n = n if max_n < 0 else min(n, max_n)
            r0, r1 = _my_rows(n, comm) if dist else (0, n)
            ip = np.asarray(_h5_slice(f, "indptr", 0, r0, r1 + 1), dtype=np.int64)
            a, b = int(ip[0]), int(ip[-1])
            X = torch.sparse_csr_tensor(torch.from_numpy(ip - a),
                                        torch.from_numpy(np.asarray(_h5_slice(f, "indices", 0, a, b), dtype=np.int64)),
                                        torch.from_numpy(np.asarray(_h5_slice(f, "values", 0, a, b),
                                                                    dtype=np.float64)).to(dtype),
                                        (r1 - r0, d))
            if not sparse:
                X = X.to_dense()
            yname = "Y"
        else:
            xname, yname = ("X", "Y") if "X" in f else ("Features", "Labels")
            d, n = _h5_shape(f, xname)
            n = n if max_n < 0 else min(n, max_n)
            r0, r1 = _my_rows(n, comm) if dist else (0, n)
            Xd = _h5_slice(f, xname, 1, r0, r1)
            X = torch.from_numpy(np.ascontiguousarray(Xd.T)).to(dtype)
            if sparse:
                X = X.to_sparse_csr()
        yshape = _h5_shape(f, yname)
        if len(yshape) == 1:
            Yall = _h5_slice(f, yname, 0, r0, r1)
        else:   # 1 x n or n x 1 label arrays
            Yall = np.asarray(f[yname]).reshape(-1)[r0:r1]
        Y = torch.from_numpy(np.asarray(Yall).reshape(-1)[: r1 - r0].astype(np.float64))
    if dist:
        from ..parallel.distmatrix import DistMatrix
        return (DistMatrix(X, (n, d), "VC_STAR", comm), DistMatrix(Y[:, None].contiguous(), (n, 1), "VC_STAR", comm))
    return X, Y


def _h5_shape(f, name):
    if hasattr(f, "read_slice"):
        return tuple(int(x) for x in f.shape(name))
    return tuple(int(x) for x in f[name].shape)


def _my_rows(n, comm):
    from ..parallel.comm import balanced_offsets
    off = balanced_offsets(n, comm.size)
    return off[comm.rank], off[comm.rank + 1]


def write_hdf5(fname: str, X, Y):
    """Write the reference layout (dense: ``X`` d x n + ``Y``; sparse:
    ``dimensions``/``indptr``/``indices``/``values`` + ``Y``)."""
    if X.layout != torch.strided:
        Xc = X.to_sparse_csr().cpu()
        data = {"dimensions": np.array([X.shape[1], X.shape[0], Xc.values().numel()], dtype=np.int64),
                "indptr": Xc.crow_indices().numpy(), "indices": Xc.col_indices().numpy(),
                "values": Xc.values().double().numpy()}
    else:
        data = {"X": X.detach().cpu().t().contiguous().double().numpy()}
    data["Y"] = torch.as_tensor(Y).reshape(-1).cpu().double().numpy()
    h5py = _h5py()
    if h5py is None:
        from .h5 import write_h5
        write_h5(fname, data)
        return
    with h5py.File(fname, "w") as f:
        for k, v in data.items():
            f[k] = v


def read(fileformat: int, fname: str, min_d: int = 0, comm=None, dtype=torch.float64, device=None):
    """Dispatch on the reference's fileformat codes; distributed when ``comm`` has >1 rank."""
    if fileformat in (LIBSVM_DENSE, LIBSVM_SPARSE):
        if comm is not None and comm.size > 1:
            return read_libsvm_dist(fname, comm, min_d, fileformat == LIBSVM_SPARSE, dtype, device)
        return read_libsvm(fname, min_d, sparse=(fileformat == LIBSVM_SPARSE), dtype=dtype, device=device)
    if fileformat in (HDF5_DENSE, HDF5_SPARSE):
        return read_hdf5(fname, sparse=(fileformat == HDF5_SPARSE), dtype=dtype,
                         comm=comm if (comm is not None and comm.size > 1) else None)
    raise IOError_(f"unknown file format code {fileformat}")


def read_arc_list(fname: str, symmetrize: bool = False, comm=None, dtype=torch.float64):
    """Edge list ``u v [w]`` (0-based vertex ids, ``#`` comments) -> sparse CSR
    adjacency n x n (n = max id + 1).  With a multi-rank ``comm`` each rank
    parses its byte range (line-aligned) and the result is a [VC,*]
    DistMatrix of adjacency rows (reference MPI-IO reader,
    ``utility/io/arc_list.hpp:151-325``)."""
    import os
    size = os.path.getsize(fname)
    rank, P = (comm.rank, comm.size) if comm is not None else (0, 1)
    with open(fname, "rb") as f:
        lo, hi = size * rank // P, size * (rank + 1) // P

        def align(pos):
            if pos <= 0 or pos >= size:
                return min(max(pos, 0), size)
            f.seek(pos - 1)
            if f.read(1) == b"\n":
                return pos
            f.seek(pos)
            f.readline()
            return f.tell()
        lo, hi = align(lo), align(hi)
        f.seek(lo)
        data = f.read(hi - lo).decode()
    rows = []
    for line in data.splitlines():
        if not line.strip() or line.lstrip().startswith("#"):
            continue
        t = line.split()
        rows.append((int(t[0]), int(t[1]), float(t[2]) if len(t) > 2 else 1.0))
    e = np.array(rows, dtype=np.float64).reshape(-1, 3)
    if symmetrize:
        e = np.concatenate([e, e[:, [1, 0, 2]]], axis=0)
    n_loc = int(e[:, :2].max()) + 1 if len(e) else 0
    if comm is None or P == 1:
        return _csr(e, 0, n_loc, n_loc, dtype)
    # route every edge to the rank owning its source row ([VC,*] blocks): one all-to-all
    from ..parallel.comm import balanced_offsets
    from ..parallel.distmatrix import DistMatrix
    n = max(comm.all_gather_object(n_loc))
    offs = np.asarray(balanced_offsets(n, P))
    owner = np.searchsorted(offs, e[:, 0], side="right") - 1
    sends = [torch.from_numpy(np.ascontiguousarray(e[owner == r])) for r in range(P)]
    mine = torch.cat(comm.all_to_all_v(sends), dim=0).numpy()
    return DistMatrix(_csr(mine, int(offs[rank]), int(offs[rank + 1] - offs[rank]), n, dtype), (n, n), "VC_STAR",
                      comm)


def _csr(e, row0, nrows, ncols, dtype):
    src, dst, w = e[:, 0].astype(np.int64) - row0, e[:, 1].astype(np.int64), e[:, 2]
    return torch.sparse_coo_tensor(torch.from_numpy(np.stack([src, dst])), torch.from_numpy(w).to(dtype),
                                   (nrows, ncols)).coalesce().to_sparse_csr()


ReadArcList = read_arc_list
ReadHDF5 = read_hdf5


def readlibsvm(fname: str, X=None, Y=None, direction="rows", min_d: int = 0, max_n: int = -1, comm=None,
               sparse: bool = False, dtype=torch.float64):
    """python-skylark ``skylark.io.readlibsvm`` (``python-skylark/skylark/io.py``):
    ``(X, Y)`` with examples as rows (``direction`` "rows" / 1) or columns
    ("columns" / 0).  ``X`` / ``Y`` given as DistMatrix templates select a
    distributed read over their communicator; otherwise a local read."""
    if direction in (0, "columns"):
        cols = True
    elif direction in (1, "rows"):
        cols = False
    else:
        raise ValueError("Direction must be either columns/rows or 0/1")
    from ..parallel.distmatrix import DistMatrix
    tmpl = X if isinstance(X, DistMatrix) else (Y if isinstance(Y, DistMatrix) else None)
    if tmpl is not None or comm is not None:
        c = comm or tmpl.comm
        Xd, Yd = read_libsvm_dist(fname, c, min_d=min_d, sparse=sparse, dtype=dtype)
        if cols:
            Xd = Xd.redistribute("STAR_VC") if hasattr(Xd, "redistribute") and not sparse else Xd
        return Xd, Yd
    Xl, Yl = read_libsvm(fname, min_d=min_d, max_n=max_n, sparse=sparse, dtype=dtype)
    if cols:
        Xl = Xl.t().to_sparse_csr() if sparse else Xl.t().contiguous()
    return Xl, Yl

