"""Streaming line input from remote / non-local filesystems (reference
``utility/hdfs.hpp:11-199`` ``hdfs_line_streamer_t`` /
``hdfs_line_streamer_iterator_t`` and the HDFS LIBSVM readers of
``utility/io/libsvm_io.hpp:1509-2000``).

The reference links libhdfs directly.  Here every filesystem goes through
``fsspec`` (``hdfs://`` -> pyarrow's HadoopFileSystem when libhdfs is present
on the machine, plus ``file://``, ``memory://``, ``s3://`` ... whatever
fsspec has a driver for), so the same streamer serves HDFS and any other
remote store.  Bytes are pulled in ``bufsize`` blocks; LIBSVM parsing is the
native multi-threaded parser applied to line-aligned blocks of the stream, so
a remote file is never held whole in host memory and parsing overlaps nothing
but the next read (IO-bound by construction).
"""
from __future__ import annotations

import numpy as np
import torch

from ..base.exceptions import IOError_

DEFAULT_BUFSIZE = 1 << 20


def _fs_and_path(path: str, fs=None):
    import fsspec
    if fs is not None:
        return fs, path
    try:
        fs, p = fsspec.core.url_to_fs(path)
    except Exception as e:  # missing driver (e.g. no libhdfs), bad URL
        raise IOError_(f"cannot open filesystem for {path!r}: {e}") from e
    return fs, p


def hdfs_url(namenode: str, path: str) -> str:
    """CLI helper: ``--hdfs <namenode>`` + input path -> an fsspec URL.
    A namenode that already carries a scheme is used as given."""
    if "://" in namenode:
        return namenode.rstrip("/") + "/" + path.lstrip("/")
    return f"hdfs://{namenode}/{path.lstrip('/')}"


class LineStreamer:
    """``getline`` / ``eof`` / ``rewind`` / ``close`` over one remote file,
    reading ``bufsize`` bytes at a time (``hdfs_line_streamer_t``).  Also
    iterable (yields lines without the trailing newline) and a context
    manager."""

    def __init__(self, path: str, bufsize: int = DEFAULT_BUFSIZE, fs=None):
        self.bufsize = int(bufsize)
        self.fs, self.path = _fs_and_path(path, fs)
        try:
            self._f = self.fs.open(self.path, "rb")
        except Exception as e:
            raise IOError_(f"Failed to open file {path}: {e}") from e
        self._buf = b""
        self._eof = False
        self._closed = False

    def _fill(self) -> bool:
        blk = self._f.read(self.bufsize)
        if not blk:
            return False
        self._buf += blk
        return True

    def getline(self) -> str:
        while True:
            i = self._buf.find(b"\n")
            if i >= 0:
                line, self._buf = self._buf[:i], self._buf[i + 1:]
                return line.decode()
            if not self._fill():
                self._eof = True
                line, self._buf = self._buf, b""
                return line.decode()

    def eof(self) -> bool:
        return self._eof and not self._buf

    def read_block(self, target: int) -> bytes:
        """Up to ~``target`` bytes ending at a line boundary (b"" at EOF)."""
        while len(self._buf) < target and self._fill():
            pass
        if not self._buf:
            self._eof = True
            return b""
        if len(self._buf) <= target:
            cut = len(self._buf)
            if self._buf[-1:] != b"\n":
                # keep reading until the current line ends (or the file does):
                # search each newly read piece for the first newline and cut
                # there, so block_bytes keeps bounding memory
                i = -1
                while i < 0:
                    old = len(self._buf)
                    if not self._fill():
                        break
                    i = self._buf.find(b"\n", old)
                cut = len(self._buf) if i < 0 else i + 1
        else:
            cut = self._buf.rfind(b"\n", 0, target) + 1
            if cut == 0:
                i = self._buf.find(b"\n", target)
                while i < 0 and self._fill():
                    i = self._buf.find(b"\n", target)
                cut = len(self._buf) if i < 0 else i + 1
        blk, self._buf = self._buf[:cut], self._buf[cut:]
        return blk

    def rewind(self):
        self._f.seek(0)
        self._buf, self._eof = b"", False

    def close(self):
        if not self._closed:
            self._f.close()
            self._closed = True

    def __iter__(self):
        while True:
            line = self.getline()
            if self.eof() and not line:
                return
            yield line

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LineStreamerIterator:
    """One :class:`LineStreamer` per file of ``path`` (a file or a directory,
    files in name order) — ``hdfs_line_streamer_iterator_t``."""

    def __init__(self, path: str, bufsize: int = DEFAULT_BUFSIZE, fs=None):
        self.fs, self.path = _fs_and_path(path, fs)
        self.bufsize = bufsize
        if self.fs.isdir(self.path):
            self.files = sorted(e["name"] for e in self.fs.ls(self.path, detail=True) if e["type"] == "file")
        elif self.fs.exists(self.path):
            self.files = [self.path]
        else:
            raise IOError_(f"no such file or directory: {path}")
        self._idx = 0

    def reset(self):
        self._idx = 0

    def next(self):
        if self._idx == len(self.files):
            return None
        s = LineStreamer(self.files[self._idx], self.bufsize, fs=self.fs)
        self._idx += 1
        return s

    def __iter__(self):
        self.reset()
        while (s := self.next()) is not None:
            yield s


def read_libsvm_stream(path: str, min_d: int = 0, max_n: int = -1, sparse: bool = False, dtype=torch.float64,
                       device=None, block_bytes: int = 64 << 20, fs=None, comm=None):
    """LIBSVM from a remote file or directory (all files concatenated), parsed
    block-by-block with the native parser.  With a multi-rank ``comm`` the
    files are dealt round-robin to ranks, the dimension is agreed with one
    all-gather, and rows are rebalanced to [VC,*] (as :func:`read_libsvm_dist`)."""
    from ..ops import _lib as L
    from .libsvm import _parse, _to_tensor
    L.require()
    it = LineStreamerIterator(path, fs=fs)
    rank, P = (comm.rank, comm.size) if comm is not None else (0, 1)
    mine = it.files[rank::P] if P > 1 else it.files
    labels, rowptrs, cols, vals, d = [], [], [], [], 0
    nrows, nnz = 0, 0
    for fname in mine:
        with LineStreamer(fname, fs=it.fs) as s:
            while True:
                left = -1 if max_n < 0 else max_n - nrows
                if left == 0:
                    break
                blk = s.read_block(block_bytes)
                if not blk:
                    break
                arr = np.frombuffer(blk, dtype=np.uint8)
                lab, rp, c, v, mx = _parse(arr.ctypes.data, 0, arr.size, left)
                labels.append(lab), cols.append(c), vals.append(v)
                rowptrs.append(rp[1:] + nnz)
                nrows, nnz, d = nrows + len(lab), nnz + len(c), max(d, mx)
        if max_n >= 0 and nrows >= max_n:
            break
    cat = (lambda xs, dt: np.concatenate(xs) if xs else np.zeros(0, dtype=dt))
    lab = cat(labels, np.float64)
    rp = np.concatenate([np.zeros(1, dtype=np.int64)] + rowptrs)
    c, v = cat(cols, np.int64), cat(vals, np.float64)
    d = max(d, min_d)
    if P == 1:
        return _to_tensor(lab, rp, c, v, d, sparse, dtype, device)
    from ..parallel.comm import balanced_counts
    from ..parallel.distmatrix import DistMatrix
    from .libsvm import _rebalance
    allst = comm.all_gather_object((len(lab), d))
    d = max(x[1] for x in allst)
    have = [x[0] for x in allst]
    n = sum(have)
    X, Y = _to_tensor(lab, rp, c, v, d, False, dtype, None)
    X, Y = _rebalance(comm, X, Y, have, balanced_counts(n, P))
    if sparse:
        X = X.to_sparse_csr()
    if device is not None:
        X, Y = X.to(device), Y.to(device)
    return (DistMatrix(X, (n, d), "VC_STAR", comm), DistMatrix(Y[:, None].contiguous(), (n, 1), "VC_STAR", comm))


ReadLIBSVMStream = read_libsvm_stream
