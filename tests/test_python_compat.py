"""python-skylark API surface (``python-skylark/skylark/{ml/utils,ml/modeling,
elemhelper,io}.py``): dummycoding / dummydecode, LinearizedKernelModel on a
model file, create_elemental_matrix / local2distributed (world 1 and gloo
world 4), readlibsvm rows / columns."""
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd import elemhelper
from libskylark_amd.ml import modeling, utils

from mp_utils import run_distributed


def test_dummycoding_roundtrip():
    Y = [1, 3, 2, 3]
    D = utils.dummycoding(Y)
    assert D.shape == (4, 3)
    torch.testing.assert_close(D, torch.tensor([[1, 0, 0], [0, 0, 1], [0, 1, 0], [0, 0, 1]], dtype=torch.float64))
    assert utils.dummydecode(D).tolist() == Y
    Z = utils.dummycoding([0, 2], K=4, zerobased=True)
    assert Z.shape == (2, 4) and utils.dummydecode(Z, zerobased=True).tolist() == [0, 2]


def test_linearized_kernel_model(tmp_path):
    from libskylark_amd import ml
    g = torch.Generator().manual_seed(0)
    X = torch.randn(200, 5, generator=g, dtype=torch.float64)
    lab = (X[:, 0] > 0).double() * 2 - 1
    solver = ml.BlockADMMSolver("squared", "l2", 0.01, 64, kernel=ml.Gaussian(5, 1.0), NumFeaturePartitions=1,
                                context=sk.Context(3))
    solver.set_maxiter(10)
    model = solver.train(X, lab, regression=True, log=None)
    f = tmp_path / "model.json"
    model.save(str(f), "# header\n")
    lk = modeling.LinearizedKernelModel(str(f))
    assert lk.get_input_dimension() == 5
    torch.testing.assert_close(lk.predict(X), model.decision_function(X))


def test_elemhelper_local():
    A = torch.arange(30, dtype=torch.float64).reshape(5, 6)
    D = elemhelper.create_elemental_matrix(5, 6, lambda i, j: 6 * i + j, layout="VC_STAR")
    torch.testing.assert_close(D.to_global(), A)
    D2 = elemhelper.local2distributed(A, layout="MC_MR")
    torch.testing.assert_close(D2.to_global(), A)
    D3 = elemhelper.create_elemental_matrix(3, 2, lambda i, j: float(i == j), layout="STAR_STAR")
    torch.testing.assert_close(D3.to_global(), torch.eye(3, 2, dtype=torch.float64))


def _eh_worker(rank, world):
    A = torch.arange(77, dtype=torch.float64).reshape(11, 7)
    for layout in ("MC_MR", "VC_STAR", "STAR_VR", "CIRC_CIRC", "STAR_STAR"):
        D = elemhelper.create_elemental_matrix(11, 7, lambda i, j: 7 * i + j, layout=layout)
        torch.testing.assert_close(D.to_global(), A)
        torch.testing.assert_close(elemhelper.local2distributed(A, layout=layout).local, D.local)
    return True


def test_elemhelper_distributed():
    assert all(run_distributed(_eh_worker, 4))


def test_readlibsvm_rows_and_columns(tmp_path):
    from libskylark_amd import io
    f = tmp_path / "d.libsvm"
    f.write_text("1 1:0.5 3:2\n-1 2:1.5\n1 1:1 2:2 3:3\n")
    X, Y = io.readlibsvm(str(f), direction="rows")
    torch.testing.assert_close(X, torch.tensor([[0.5, 0, 2], [0, 1.5, 0], [1, 2, 3]], dtype=torch.float64))
    assert Y.tolist() == [1, -1, 1]
    Xc, _ = io.readlibsvm(str(f), direction=0, min_d=4)
    assert Xc.shape == (4, 3)
    torch.testing.assert_close(Xc[:3], X.t())
    with pytest.raises(ValueError):
        io.readlibsvm(str(f), direction="diagonal")


def test_nla_param_aliases():
    from libskylark_amd import nla
    p = nla.SVDParams()
    assert (p.oversampling_ratio, p.oversampling_additive, p.num_iterations, p.skip_qr) == (2, 0, 2, False)
    assert nla.FasterLeastSquaresParams is nla.FasterLSParams
