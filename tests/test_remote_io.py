"""Remote / HDFS-style streamed input (reference ``utility/hdfs.hpp``,
``libsvm_io.hpp:1509-2000``).  No HDFS cluster exists here: the same code
paths run over fsspec's ``memory://`` and ``file://`` filesystems, which is
what an ``hdfs://`` URL resolves to through fsspec once libhdfs is present."""
import numpy as np
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.io import remote
from mp_utils import run_distributed

fsspec = pytest.importorskip("fsspec")


def _libsvm_bytes(X, Y):
    lines = []
    for i in range(X.shape[0]):
        nz = [f"{j + 1}:{X[i, j]:.17g}" for j in range(X.shape[1]) if X[i, j] != 0]
        lines.append(" ".join([f"{Y[i]:.17g}"] + nz))
    return ("\n".join(lines) + "\n").encode()


def _data(n=257, d=9, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d)) * (rng.random((n, d)) < 0.6)
    X[:, -1] = 1.0  # pin the dimension
    return X, rng.integers(0, 3, n).astype(np.float64)


def _put(url, data):
    fs, p = fsspec.core.url_to_fs(url)
    with fs.open(p, "wb") as f:
        f.write(data)


def test_line_streamer_small_buffer():
    url = "memory://sk_remote/lines.txt"
    text = "alpha\nbeta gamma\n\nlast-without-newline"
    _put(url, text.encode())
    with remote.LineStreamer(url, bufsize=3) as s:
        got = []
        while True:
            line = s.getline()
            if s.eof() and not line:
                break
            got.append(line)
            if s.eof():
                break
        assert got == ["alpha", "beta gamma", "", "last-without-newline"]
        s.rewind()
        assert list(s) == got


def test_line_streamer_iterator_directory():
    for i in range(3):
        _put(f"memory://sk_remote/dir/part-{i}", f"file{i}\n".encode())
    it = remote.LineStreamerIterator("memory://sk_remote/dir", bufsize=4)
    assert [next(iter(s)) for s in it] == ["file0", "file1", "file2"]
    it.reset()
    assert it.next() is not None
    with pytest.raises(sk.base.exceptions.IOError_):
        remote.LineStreamerIterator("memory://sk_remote/missing")


@pytest.mark.parametrize("block", [64, 1 << 20])
def test_read_libsvm_stream_matches_local(tmp_path, block):
    X, Y = _data()
    data = _libsvm_bytes(X, Y)
    _put("memory://sk_remote/a.libsvm", data)
    Xs, Ys = remote.read_libsvm_stream("memory://sk_remote/a.libsvm", block_bytes=block)
    np.testing.assert_array_equal(Xs.numpy(), X)
    np.testing.assert_array_equal(Ys.numpy(), Y)
    # file:// URL and max_n / sparse / min_d
    f = tmp_path / "a.libsvm"
    f.write_bytes(data)
    Xf, Yf = remote.read_libsvm_stream(f"file://{f}", max_n=100, sparse=True, min_d=12, block_bytes=block)
    assert Xf.layout == torch.sparse_csr and Xf.shape == (100, 12)
    np.testing.assert_array_equal(Xf.to_dense()[:, :9].numpy(), X[:100])
    Xl, _ = sk.io.read_libsvm(str(f))
    np.testing.assert_array_equal(Xl.numpy(), X)


def test_read_libsvm_stream_directory():
    X, Y = _data(n=100)
    for i, (lo, hi) in enumerate([(0, 30), (30, 31), (31, 100)]):
        _put(f"memory://sk_remote/ddir/part-{i:03d}", _libsvm_bytes(X[lo:hi], Y[lo:hi]))
    Xs, Ys = remote.read_libsvm_stream("memory://sk_remote/ddir", block_bytes=128)
    np.testing.assert_array_equal(Xs.numpy(), X)
    np.testing.assert_array_equal(Ys.numpy(), Y)


def test_hdfs_url():
    assert remote.hdfs_url("namenode:9000", "/data/x") == "hdfs://namenode:9000/data/x"
    assert remote.hdfs_url("memory://root", "x") == "memory://root/x"


def test_linear_cli_hdfs_flag(tmp_path):
    from libskylark_amd.cli import linear
    from libskylark_amd.cli._common import read_ascii
    g = np.random.default_rng(3)
    A = g.standard_normal((300, 6))
    x = g.standard_normal(6)
    f = tmp_path / "ls.libsvm"
    f.write_bytes(_libsvm_bytes(A, A @ x))
    out = str(tmp_path / "x")
    # --hdfs with a scheme-carrying prefix routes the read through the streamer
    assert linear.main([str(f).lstrip("/"), out, "--hdfs", "file:///", "-p", "--cpu"]) == 0
    np.testing.assert_allclose(read_ascii(out + ".txt").numpy().reshape(-1), x, rtol=1e-8, atol=1e-8)


def _dist_stream(rank, world, root):
    from libskylark_amd.parallel.comm import Comm
    X, Y = remote.read_libsvm_stream(f"file://{root}", comm=Comm(), block_bytes=100)
    return X.local.numpy(), Y.local.numpy().reshape(-1), X.shape


def test_read_libsvm_stream_distributed(tmp_path):
    X, Y = _data(n=90, seed=5)
    d = tmp_path / "parts"
    d.mkdir()
    for i, (lo, hi) in enumerate([(0, 10), (10, 50), (50, 90)]):
        (d / f"p{i}").write_bytes(_libsvm_bytes(X[lo:hi], Y[lo:hi]))
    res = run_distributed(_dist_stream, 2, str(d))
    assert all(r[2] == (90, 9) for r in res)
    # files dealt round-robin (p0, p2 -> rank 0; p1 -> rank 1), then rebalanced to [VC,*] blocks
    rows = np.concatenate([r[0] for r in res])
    labs = np.concatenate([r[1] for r in res])
    assert [len(r[0]) for r in res] == [45, 45]
    order = np.r_[0:10, 50:90, 10:50]
    np.testing.assert_array_equal(rows, X[order])
    np.testing.assert_array_equal(labs, Y[order])
