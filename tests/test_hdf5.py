"""Built-in HDF5 reader/writer (io/h5.py): the reference's own dataset file,
round trips in the reference layouts, chunked + deflate datasets."""
import os
import struct
import zlib

import numpy as np
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.io.h5 import H5File, write_h5

USPS = "/root/reference/python-skylark/skylark/datasets/usps.hdf5"


@pytest.mark.skipif(not os.path.exists(USPS), reason="reference dataset not mounted")
def test_reads_reference_usps_dataset():
    f = H5File(USPS)
    assert sorted(f.keys()) == ["Features", "Labels"]
    F, L = f["Features"], f["Labels"]
    assert F.shape == (256, 2007) and L.shape == (2007,)
    assert F.min() >= -1.0 and F.max() <= 1.0
    assert set(np.unique(L).tolist()) == set(float(i) for i in range(1, 11))
    X, Y = sk.io.read_hdf5(USPS)
    assert X.shape == (2007, 256) and torch.equal(Y, torch.from_numpy(L))


def test_roundtrip_dense_and_sparse(tmp_path):
    g = torch.Generator().manual_seed(0)
    X = torch.randn(40, 9, generator=g, dtype=torch.float64)
    Y = torch.arange(40, dtype=torch.float64)
    p = str(tmp_path / "d.h5")
    sk.io.write_hdf5(p, X, Y)
    X2, Y2 = sk.io.read_hdf5(p)
    assert torch.equal(X, X2) and torch.equal(Y, Y2)
    X[torch.rand(40, 9, generator=g) > 0.3] = 0
    ps = str(tmp_path / "s.h5")
    sk.io.write_hdf5(ps, X.to_sparse_csr(), Y)
    X3, _ = sk.io.read_hdf5(ps, sparse=True)
    assert X3.layout == torch.sparse_csr and torch.equal(X3.to_dense(), X)
    X4, _ = sk.io.read_hdf5(ps, max_n=10)
    assert torch.equal(X4, X[:10])


def test_integer_and_float32_datasets(tmp_path):
    p = str(tmp_path / "m.h5")
    data = {"a": np.arange(12, dtype=np.int32).reshape(3, 4), "b": np.float32([1.5, -2.0]),
            "c": np.arange(5, dtype=np.uint64)}
    write_h5(p, data)
    f = H5File(p)
    for k, v in data.items():
        assert f[k].dtype == v.dtype and np.array_equal(f[k], v)


def test_chunked_deflate_dataset_reader():
    """Hand-built chunked + deflate dataset (v1 B-tree chunk index) parsed by
    the reader's chunk path (the layout libhdf5 writes for compressed data)."""
    from libskylark_amd.io.h5 import _Reader
    A = np.arange(6 * 5, dtype="<f8").reshape(6, 5)
    chunks = [((0, 0), A[0:4, 0:5]), ((4, 0), A[4:6, 0:5])]
    blob = bytearray(b"\x89HDF\r\n\x1a\n" + bytes(200))
    recs = []
    for (r0, c0), blk in chunks:
        full = np.zeros((4, 5), dtype="<f8")
        full[:blk.shape[0], :blk.shape[1]] = blk
        comp = zlib.compress(full.tobytes())
        recs.append((len(blob), len(comp), (r0, c0)))
        blob += comp
    btree = len(blob)
    node = bytearray(b"TREE" + bytes([1, 0]) + struct.pack("<H", len(recs)) + struct.pack("<QQ", 2**64 - 1, 2**64 - 1))
    for addr, size, (r0, c0) in recs:
        node += struct.pack("<II", size, 0) + struct.pack("<QQQ", r0, c0, 0) + struct.pack("<Q", addr)
    node += struct.pack("<II", 0, 0) + struct.pack("<QQQ", 6, 5, 0)
    blob += node
    r = _Reader(bytes(blob[:8]) + bytes([0, 0, 0, 0, 0, 8, 8]) + bytes(blob[15:]))
    out = r._read_chunked(btree, (6, 5), (4, 5), np.dtype("<f8"), [(1, (6,))])
    assert np.array_equal(out, A)


def _dist_h5_worker(rank, world, dense_path, sparse_path):
    from libskylark_amd.parallel.comm import world as W
    comm = W()
    Xl, Yl = sk.io.read_hdf5(dense_path)
    Xd, Yd = sk.io.read_hdf5(dense_path, comm=comm)
    assert Xd.layout == "VC_STAR" and Xd.shape == tuple(Xl.shape)
    torch.testing.assert_close(Xd.to_global(), Xl)
    torch.testing.assert_close(Yd.to_global()[:, 0], Yl)
    Xs, Ys = sk.io.read_hdf5(sparse_path, sparse=True, comm=comm)
    Xsl, _ = sk.io.read_hdf5(sparse_path, sparse=True)
    r0, r1 = Xs.row_range()
    torch.testing.assert_close(Xs.local.to_dense(), Xsl.to_dense()[r0:r1])
    return True


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_hdf5_hyperslabs(tmp_path, world):
    """Each rank reads only its example block (reference rank-0 read +
    send/recv, ml/io.hpp:256-526)."""
    from mp_utils import run_distributed
    g = torch.Generator().manual_seed(0)
    X = torch.randn(37, 6, generator=g, dtype=torch.float64)
    X[X.abs() < 0.7] = 0
    Y = torch.arange(37, dtype=torch.float64)
    p, ps = tmp_path / "d.h5", tmp_path / "s.h5"
    sk.io.write_hdf5(str(p), X, Y)
    sk.io.write_hdf5(str(ps), X.to_sparse_csr(), Y)
    run_distributed(_dist_h5_worker, world, str(p), str(ps))
