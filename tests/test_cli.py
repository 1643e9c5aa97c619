"""Command-line tools, driven in-process (CPU) with small files."""
import numpy as np
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd.cli import community, graph_se, krr, linear, ml as mlcli, svd
from libskylark_amd.cli._common import read_ascii


def _blobs_file(path, n=240, seed=0, regression=False):
    g = torch.Generator().manual_seed(seed)
    lab = torch.randint(0, 3, (n,), generator=g)
    c = torch.tensor([[2.0, 0, 0, 0], [0, 2.0, 0, 0], [0, 0, 2.0, 0]], dtype=torch.float64)
    X = c[lab] + 0.4 * torch.randn(n, 4, generator=g, dtype=torch.float64)
    Y = X[:, 0] * 0.5 if regression else lab.to(torch.float64)
    sk.io.write_libsvm(str(path), X, Y)
    return X, Y


def test_svd_cli_profile_and_file(tmp_path, capsys):
    pre = str(tmp_path / "p")
    assert svd.main(["--profile", "300", "40", "-k", "4", "--prefix", pre, "--cpu"]) == 0
    S = read_ascii(pre + ".S.txt")[:, 0]
    assert S.shape == (4,) and float(S[0]) > float(S[-1])
    U0, _ = np.linalg.qr(np.random.default_rng(0).standard_normal((100, 3)))
    A = U0 @ np.diag([5.0, 3.0, 1.0]) @ np.linalg.qr(np.random.default_rng(1).standard_normal((12, 3)))[0].T
    f = tmp_path / "a.libsvm"
    sk.io.write_libsvm(str(f), torch.from_numpy(A), torch.zeros(100))
    pre = str(tmp_path / "q")
    assert svd.main([str(f), "-k", "3", "--prefix", pre, "--cpu"]) == 0
    np.testing.assert_allclose(read_ascii(pre + ".S.txt")[:, 0].numpy(), [5, 3, 1], rtol=1e-8)
    U = read_ascii(pre + ".U.txt").numpy()
    assert U.shape == (100, 3)


def test_linear_cli(tmp_path):
    g = torch.Generator().manual_seed(2)
    A = torch.randn(500, 8, generator=g, dtype=torch.float64)
    x = torch.randn(8, generator=g, dtype=torch.float64)
    b = A @ x
    f = tmp_path / "ls.libsvm"
    sk.io.write_libsvm(str(f), A, b)
    out = str(tmp_path / "x")
    assert linear.main([str(f), out, "-p", "--cpu"]) == 0
    np.testing.assert_allclose(read_ascii(out + ".txt")[:, 0].numpy(), x.numpy(), rtol=1e-8, atol=1e-8)


def test_ml_cli_train_test(tmp_path, capsys):
    tr, te = tmp_path / "tr.libsvm", tmp_path / "te.libsvm"
    _blobs_file(tr, 300, 0)
    _blobs_file(te, 100, 1)
    model = str(tmp_path / "model.json")
    assert mlcli.main(["-k", "1", "-g", "1.0", "-f", "128", "-l", "2", "-r", "1", "-c", "0.01", "-i", "15",
                       "--trainfile", str(tr), "--modelfile", model]) == 0
    assert open(model).readline().startswith("# Generated using skylark_ml")
    capsys.readouterr()
    assert mlcli.main(["--modelfile", model, "--testfile", str(te)]) == 0
    out = capsys.readouterr().out
    err = float(out.strip().split()[-1].rstrip("%"))
    assert err < 10.0


@pytest.mark.parametrize("alg", ["0", "1", "2", "3", "5"])
def test_krr_cli(tmp_path, capsys, alg):
    tr, te = tmp_path / "tr.libsvm", tmp_path / "te.libsvm"
    _blobs_file(tr, 200, 0)
    _blobs_file(te, 80, 1)
    model = str(tmp_path / "m.json")
    args = ["-a", alg, "-k", "0", "-g", "1.0", "-l", "0.1", "-f", "256", "--model", model, str(tr), str(te),
            "--cpu"]
    assert krr.main(args) == 0
    out = capsys.readouterr().out
    err = float([ln for ln in out.splitlines() if ln.startswith("Test error")][-1].split()[-1].rstrip("%"))
    assert err < 10.0
    # predict mode reloads the saved model
    assert krr.main(["--predict", "--model", model, str(te), "--cpu"]) == 0


def test_community_and_graph_se(tmp_path, capsys):
    edges = [(b + i, b + j) for b in (0, 10) for i in range(8) for j in range(i + 1, 8)] + [(7, 10)]
    f = tmp_path / "g.txt"
    f.write_text("# two cliques\n" + "".join(f"{u} {v}\n" for u, v in edges))
    assert community.main(["-g", str(f), "-s", "2", "-r", "-q"]) == 0
    out = capsys.readouterr().out.split()
    assert sorted(int(v) for v in out) == list(range(8))
    pre = str(tmp_path / "emb")
    assert graph_se.main(["-g", str(f), "-k", "2", "--prefix", pre, "--cpu"]) == 0
    X = read_ascii(pre + ".vec.txt")
    assert X.shape == (16, 2)


def test_convert2hdf5_cli_roundtrip(tmp_path):
    import libskylark_amd as sk
    from libskylark_amd.cli import convert2hdf5
    src = tmp_path / "a.libsvm"
    src.write_text("1 1:0.5 3:2.0\n-1 2:1.5\n1 1:-1.0 2:0.25 3:1.0\n")
    out = tmp_path / "a.h5"
    convert2hdf5.main([str(src), str(out)])
    X, Y = sk.io.read_hdf5(str(out))
    assert X.shape == (3, 3) and Y.tolist() == [1.0, -1.0, 1.0]
    assert float(X[0, 2]) == 2.0 and float(X[1, 1]) == 1.5
