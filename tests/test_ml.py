"""ML layer: kernels, KRR family, RLSC, BlockADMM, models, graph, IO.

Oracles: closed-form kernel definitions (reference ``ml/kernels.hpp`` maps),
exact KRR solves (torch.linalg), reference JSON schemas, hand-built graphs
with known community structure.  The reference has no unit tests for these
(SURVEY.md 4); parity of random-feature paths is statistical.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd import ml

torch.manual_seed(0)


def _comm():
    from libskylark_amd.parallel.comm import world
    return world()


def _data(n=80, d=6, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, d, generator=g, dtype=torch.float64)


@pytest.mark.parametrize("name", ["linear", "gaussian", "polynomial", "laplacian", "expsemigroup", "matern"])
def test_kernel_gram_matches_definition(name):
    X, Y = _data(40, 5, 1), _data(30, 5, 2)
    if name == "expsemigroup":
        X, Y = X.abs(), Y.abs()
    k = {"linear": ml.Linear(5), "gaussian": ml.Gaussian(5, 1.7), "polynomial": ml.Polynomial(5, 3, 0.5, 0.7),
         "laplacian": ml.Laplacian(5, 2.5), "expsemigroup": ml.ExpSemigroup(5, 0.4),
         "matern": ml.Matern(5, 2.5, 1.3)}[name]
    K = k.gram(X, Y=Y)
    diff = X[:, None, :] - Y[None, :, :]
    ref = {"linear": lambda: X @ Y.t(),
           "gaussian": lambda: torch.exp(-(diff ** 2).sum(-1) / (2 * 1.7 ** 2)),
           "polynomial": lambda: (0.7 * X @ Y.t() + 0.5) ** 3,
           "laplacian": lambda: torch.exp(-diff.abs().sum(-1) / 2.5),
           "expsemigroup": lambda: torch.exp(-0.4 * torch.sqrt(X[:, None, :] + Y[None, :, :]).sum(-1)),
           "matern": lambda: (lambda r: (1 + math.sqrt(5) * r + 5 * r * r / 3) * torch.exp(-math.sqrt(5) * r))(
               diff.pow(2).sum(-1).sqrt() / 1.3)}[name]()
    torch.testing.assert_close(K, ref, rtol=1e-9, atol=1e-9)
    # columns direction == rows on the transpose; symmetric default Y = X
    torch.testing.assert_close(k.gram(X.t(), dirX="columns", Y=Y.t(), dirY="columns"), K)
    torch.testing.assert_close(k.gram(X), k.symmetric_gram(X))
    # serialization round trip
    k2 = ml.kernel_from_dict(json.loads(k.to_json()))
    assert k2 == k


def test_kernel_factory_and_boost_strings():
    k = ml.kernel("gaussian", 4, 2.0)
    assert isinstance(k, ml.Gaussian) and k.get_dim() == 4
    d = {"skylark_object_type": "kernel", "kernel_type": "polynomial", "q": "2", "c": "1", "gamma": "0.5", "N": "4"}
    assert ml.kernel_from_dict(d) == ml.Polynomial(4, 2, 1.0, 0.5)
    with pytest.raises(ValueError):
        ml.kernel("nope", 3)


@pytest.mark.parametrize("kern", [ml.Gaussian(6, 2.0), ml.Laplacian(6, 3.0), ml.Matern(6, 1.5, 2.0)])
def test_random_features_approximate_kernel(kern):
    X = _data(60, 6, 3) * 0.5
    S = kern.create_rft(6000, context=sk.Context(11))
    Z = S.apply(X, dim=sk.sketch.ROWWISE)
    K = kern.gram(X) if not isinstance(kern, ml.Matern) else kern.gram(X)
    err = float((Z @ Z.t() - K).abs().max())
    assert err < 0.08


def test_gram_distributed_rows_match_local():
    from mp_utils import run_distributed
    run_distributed(_dist_gram_worker, 2)


def _dist_gram_worker(rank, world):
    comm = _comm()
    from libskylark_amd.parallel.distmatrix import DistMatrix
    X = _data(37, 4, 5)
    k = ml.Gaussian(4, 1.1)
    Kd = k.gram(DistMatrix.from_global(X, "VC_STAR", comm))
    torch.testing.assert_close(Kd.to_global(), k.gram(X))


def test_exact_krr():
    X = _data(70, 4, 1)
    Y = torch.sin(X.sum(1, keepdim=True))
    k = ml.Gaussian(4, 1.5)
    A = ml.kernel_ridge(k, X, Y, 0.1)
    K = k.gram(X)
    torch.testing.assert_close((K + 0.1 * torch.eye(70, dtype=torch.float64)) @ A, Y, rtol=1e-8, atol=1e-8)


def test_approximate_and_faster_krr_close_to_exact():
    X = _data(300, 4, 2) * 0.7
    Y = torch.sin(X.sum(1, keepdim=True))
    k = ml.Gaussian(4, 1.5)
    lam = 0.05
    A = ml.kernel_ridge(k, X, Y, lam)
    pred_exact = k.gram(X) @ A
    S, W = ml.approximate_kernel_ridge(k, X, Y, lam, 2000, sk.Context(3))
    pred = S.apply(X, dim=sk.sketch.ROWWISE) @ W
    assert float((pred - pred_exact).norm() / pred_exact.norm()) < 0.05
    p = ml.KrrParams(tolerance=1e-10, iter_lim=500)
    A2 = ml.faster_kernel_ridge(k, X, Y, lam, 200, sk.Context(4), params=p)
    torch.testing.assert_close(A2, A, rtol=1e-6, atol=1e-6)
    # preconditioner is exact Woodbury inverse of (lam I + U U^T)
    P = ml.FeatureMapPrecond(k, lam, X, 50, sk.Context(5))
    U = k.create_rft(50, context=sk.Context(5)).apply(X, dim=sk.sketch.ROWWISE)
    Mx = lam * torch.eye(300, dtype=torch.float64) + U @ U.t()
    B = torch.randn(300, 2, dtype=torch.float64)
    torch.testing.assert_close(P.apply(Mx @ B), B, rtol=1e-7, atol=1e-7)


def test_sketched_and_largescale_krr():
    X = _data(400, 3, 4) * 0.6
    Y = torch.cos(X[:, :1])
    k = ml.Gaussian(3, 1.2)
    lam = 1.0  # block Gauss-Seidel converges slowly for tiny lambda; check the fixed point
    scale, maps, W = ml.large_scale_kernel_ridge(k, X, Y, lam, 300, sk.Context(1),
                                                 params=ml.KrrParams(max_split=100, iter_lim=500, tolerance=1e-12))
    assert scale and len(maps) > 1
    Z = torch.cat([S.apply(X, dim=sk.sketch.ROWWISE) * math.sqrt(S.get_S() / 300) for S in maps], 1)
    Wr = torch.linalg.solve(Z.t() @ Z + lam * torch.eye(300, dtype=torch.float64), Z.t() @ Y)
    assert float((W - Wr).norm() / Wr.norm()) < 1e-3
    lam = 0.01
    scale, maps, W2 = ml.sketched_approximate_kernel_ridge(k, X, Y, lam, 300, 1200, sk.Context(1),
                                                           params=ml.KrrParams(max_split=200))
    Z2 = torch.cat([S.apply(X, dim=sk.sketch.ROWWISE) * math.sqrt(S.get_S() / 300) for S in maps], 1)
    assert float((Z2 @ W2 - Y).norm() / Y.norm()) < 0.2


def test_rlsc_and_coding():
    Y, coding, rc = ml.dummy_coding(torch.tensor([3, 1, 3, 2, 1]))
    assert rc == [3, 1, 2] and coding == {3: 0, 1: 1, 2: 2}
    assert Y.tolist()[0] == [1, -1, -1] and Y.tolist()[1] == [-1, 1, -1]
    assert ml.dummy_decode(Y, rc) == [3, 1, 3, 2, 1]
    g = torch.Generator().manual_seed(0)
    c = torch.tensor([[2.0, 0, 0], [0, 2.0, 0], [0, 0, 2.0]], dtype=torch.float64)
    lab = torch.randint(0, 3, (150,), generator=g)
    X = c[lab] + 0.3 * torch.randn(150, 3, generator=g, dtype=torch.float64)
    k = ml.Gaussian(3, 1.0)
    A, rc = ml.kernel_rlsc(k, X, lab, 0.1)
    pred = ml.dummy_decode(k.gram(X) @ A, rc)
    assert np.mean(np.array(pred) == lab.numpy()) > 0.95
    S, W, rc2 = ml.approximate_kernel_rlsc(k, X, lab, 0.1, 500, sk.Context(2))
    pred2 = ml.dummy_decode(S.apply(X, dim=sk.sketch.ROWWISE) @ W, rc2)
    assert np.mean(np.array(pred2) == lab.numpy()) > 0.9


def _blobs(n, seed):
    g = torch.Generator().manual_seed(seed)
    lab = torch.randint(0, 3, (n,), generator=g)
    c = torch.tensor([[2.0, 0, 0, 0], [0, 2.0, 0, 0], [0, 0, 2.0, 0]], dtype=torch.float64)
    X = c[lab] + 0.4 * torch.randn(n, 4, generator=g, dtype=torch.float64)
    return X, lab.to(torch.float64)


@pytest.mark.parametrize("loss", ["hinge", "logistic", "squared"])
def test_block_admm_classification(loss, tmp_path):
    X, lab = _blobs(300, 0)
    Xv, labv = _blobs(100, 1)
    solver = ml.BlockADMMSolver(loss, "l2", 0.01, 200, kernel=ml.Gaussian(4, 1.0), NumFeaturePartitions=2,
                                context=sk.Context(7))
    solver.set_maxiter(30)
    model = solver.train(X, lab, Xv, labv, regression=False, log=None)
    pred, _ = model.predict(Xv)
    acc = float((pred == labv).double().mean())
    assert acc > 0.9, acc
    assert solver.history[-1]["accuracy"] > 90
    # model JSON round trip (reference schema)
    f = tmp_path / "m.json"
    model.save(str(f), "# header line\n")
    d = json.loads("".join(ln for ln in open(f) if not ln.startswith("#")))
    assert d["skylark_object_type"] == "model:linear-on-features"
    assert d["feature_mapping"]["number_maps"] == 2
    m2 = ml.load_model(str(f))
    torch.testing.assert_close(m2.predict(Xv)[1], model.predict(Xv)[1])


def test_block_admm_regression_linear_features():
    g = torch.Generator().manual_seed(3)
    X = torch.randn(400, 5, generator=g, dtype=torch.float64)
    w = torch.randn(5, 1, generator=g, dtype=torch.float64)
    Y = (X @ w)[:, 0]
    solver = ml.BlockADMMSolver("squared", "l2", 1e-4, 5, NumFeaturePartitions=1)
    solver.set_maxiter(60)
    model = solver.train(X, Y, regression=True, log=None)
    torch.testing.assert_close(model.coef, w, rtol=5e-2, atol=5e-2)


def test_block_admm_distributed_matches_serial():
    from mp_utils import run_distributed
    run_distributed(_admm_worker, 2)


def _admm_worker(rank, world):
    comm = _comm()
    X, lab = _blobs(200, 0)
    mk = lambda: ml.BlockADMMSolver("hinge", "l2", 0.01, 64, kernel=ml.Gaussian(4, 1.0), context=sk.Context(7))
    s = mk()
    s.set_maxiter(5)
    lo, hi = (0, 100) if comm.rank == 0 else (100, 200)
    m = s.train(X[lo:hi], lab[lo:hi], regression=False, comm=comm, log=None)
    # every rank holds the same consensus model
    allc = comm.all_gather_object(m.coef.numpy())
    np.testing.assert_allclose(allc[0], allc[1])


def test_hilbert_options_and_solver_factory(tmp_path):
    o = ml.parse_options(["-k", "1", "-g", "1.5", "-f", "64", "-l", "2", "-r", "1", "-c", "0.1", "-i", "3",
                          "--regression", "train.txt", "model.json"])
    assert o.kernel == 1 and o.randomfeatures == 64 and o.trainfile == "train.txt" and o.modelfile == "model.json"
    s = ml.get_solver(sk.Context(1), o, 10)
    assert s.get_numfeatures() == 64 and s.maxiter == 3 and len(s.get_feature_maps()) == 1
    assert "Generated using skylark_ml" in o.print()
    o2 = ml.parse_options(["-k", "1", "-f", "64", "-q", "1", "-n", "2"])
    s2 = ml.get_solver(sk.Context(1), o2, 10)
    assert type(s2.get_feature_maps()[0]).__name__ == "GaussianQRFT"


def test_feature_expansion_and_kernel_models(tmp_path):
    X = _data(50, 3, 9)
    Y = X[:, :1] ** 2
    k = ml.Gaussian(3, 1.0)
    S, W = ml.approximate_kernel_ridge(k, X, Y, 0.1, 128, sk.Context(1))
    fm = ml.FeatureExpansionModel(S, W)
    f = tmp_path / "fe.json"
    fm.save(str(f))
    fm2 = ml.load_model(str(f))
    torch.testing.assert_close(fm2.predict(X)[0], fm.predict(X)[0])
    # kernel model: data location reread from a LIBSVM file
    data = tmp_path / "train.libsvm"
    sk.io.write_libsvm(str(data), X, Y[:, 0])
    A = ml.kernel_ridge(k, X, Y, 0.1)
    km = ml.KernelModel(k, X, A, data_location=str(data))
    f2 = tmp_path / "k.json"
    km.save(str(f2))
    km2 = ml.load_model(str(f2))
    torch.testing.assert_close(km2.predict(X)[0], km.predict(X)[0], rtol=1e-10, atol=1e-10)


# ------------------------------------------------------------------ IO
def test_libsvm_roundtrip(tmp_path):
    g = torch.Generator().manual_seed(0)
    X = torch.randn(257, 9, generator=g, dtype=torch.float64)
    X[X.abs() < 0.8] = 0
    Y = torch.randint(-1, 3, (257,), generator=g).to(torch.float64)
    f = tmp_path / "d.libsvm"
    sk.io.write_libsvm(str(f), X, Y)
    with open(f, "a") as fh:
        fh.write("# trailing comment\n\n")
    Xr, Yr = sk.io.read_libsvm(str(f), min_d=9)
    torch.testing.assert_close(Xr, X)
    torch.testing.assert_close(Yr, Y)
    Xs, _ = sk.io.read_libsvm(str(f), min_d=12, sparse=True, max_n=10)
    assert Xs.shape == (10, 12) and Xs.layout == torch.sparse_csr
    torch.testing.assert_close(Xs.to_dense()[:, :9], X[:10])


def test_libsvm_distributed(tmp_path):
    from mp_utils import run_distributed
    g = torch.Generator().manual_seed(1)
    X = torch.randn(101, 7, generator=g, dtype=torch.float64)
    Y = torch.arange(101, dtype=torch.float64)
    f = tmp_path / "d.libsvm"
    sk.io.write_libsvm(str(f), X, Y)
    run_distributed(_libsvm_worker, 3, str(f))


def _libsvm_worker(rank, world, fname):
    comm = _comm()
    Xd, Yd = sk.io.read_libsvm_dist(fname, comm)
    X, Y = sk.io.read_libsvm(fname)
    torch.testing.assert_close(Xd.to_global(), X)
    torch.testing.assert_close(Yd.to_global()[:, 0], Y)


def test_arc_list(tmp_path):
    f = tmp_path / "g.txt"
    f.write_text("# edges\n0 1\n1 2 2.5\n3 0\n")
    A = sk.io.read_arc_list(str(f), symmetrize=True).to_dense()
    assert A.shape == (4, 4) and A[1, 2] == 2.5 and A[2, 1] == 2.5 and A[0, 3] == 1


# --------------------------------------------------------------- graph
def _two_cliques():
    edges = []
    for base in (0, 10):
        for i in range(8):
            for j in range(i + 1, 8):
                edges.append((base + i, base + j))
    edges.append((7, 10))
    return ml.SimpleGraph(np.array(edges))


def test_local_cluster_finds_clique():
    G = _two_cliques()
    assert G.num_vertices() == 16 and G.num_edges() == 2 * (2 * 28 + 1)
    cluster, cond = ml.find_local_cluster(G, [2], recursive=True)
    assert cluster == set(range(8))
    assert cond == pytest.approx(1 / 57)
    y, x = ml.time_dependent_ppr(G, {2: 1.0})
    assert len(x) == 4 and x[0] == pytest.approx(5.0)
    assert y[2][-1] > y[12][-1] if 12 in y else True


def test_approximate_ase():
    G = _two_cliques()
    p = sk.nla.ApproximateSVDParams(num_iterations=3)
    X, idx = ml.approximate_ase(G, 2, sk.Context(1), p)
    assert X.shape == (16, 2)
    # the leading two eigenvectors separate the cliques
    col = X[:, 1]
    a = col[[idx.index(i) for i in range(8)]]
    b = col[[idx.index(i) for i in range(10, 18)]]
    assert (a.sign() == a[0].sign()).all() and (b.sign() == b[0].sign()).all() and a[0].sign() != b[0].sign()


def test_read_dir_libsvm(tmp_path):
    import libskylark_amd as sk
    (tmp_path / "a").write_text("1 1:1.0 2:2.0\n2 3:3.0\n")
    (tmp_path / "b").write_text("3 5:5.0\n")
    X, Y = sk.io.read_dir_libsvm(str(tmp_path))
    assert X.shape == (3, 5) and Y.tolist() == [1.0, 2.0, 3.0]
    assert float(X[2, 4]) == 5.0 and float(X[1, 2]) == 3.0
    Xs, _ = sk.io.ReadDirLIBSVM(str(tmp_path), sparse=True, min_d=7)
    assert Xs.layout == torch.sparse_csr and Xs.shape == (3, 7)


def _dir_worker(rank, world, d):
    import libskylark_amd as sk
    from libskylark_amd.parallel.comm import world as W
    X, Y = sk.io.read_dir_libsvm(d, comm=W())
    Xg, Yg = X.to_global(), Y.to_global()
    ref, refy = sk.io.read_dir_libsvm(d)
    assert torch.equal(Xg, ref.to(Xg.dtype)) and torch.equal(Yg[:, 0], refy)


def test_read_dir_libsvm_distributed(tmp_path):
    from mp_utils import run_distributed
    for i in range(3):
        (tmp_path / f"f{i}").write_text("".join(f"{i + j} {j + 1}:{float(i * 10 + j)}\n" for j in range(1 + i)))
    run_distributed(_dir_worker, 2, str(tmp_path))


def test_libsvm_parser_bounds(tmp_path):
    """The parser stays inside each line and the mapping: no trailing newline
    at EOF, an empty value must not swallow the next line's label, and a
    0 (or negative) feature index is rejected instead of becoming column -1."""
    from libskylark_amd.io import read_libsvm
    from libskylark_amd.ops._lib import NativeLibraryError
    p = tmp_path / "noeol.svm"
    p.write_bytes(b"1 1:0.5 3:2\n-1 2:1.25")   # last line has no newline
    X, Y = read_libsvm(str(p))
    assert Y.tolist() == [1.0, -1.0]
    assert X.tolist() == [[0.5, 0.0, 2.0], [0.0, 1.25, 0.0]]
    for bad in (b"1 0:1.0\n", b"1 2:\n-1 1:1\n", b"1 -3:1\n", b"1 x:1\n"):
        q = tmp_path / "bad.svm"
        q.write_bytes(bad)
        with pytest.raises((NativeLibraryError, RuntimeError, ValueError)):
            read_libsvm(str(q))


def test_nystrom_precond_converges_at_small_lambda():
    """at lambda = 1e-2 the reference's random-feature
    Woodbury preconditioner leaves CG slow (its approximation error of K
    divided by lambda bounds the preconditioned condition number); the
    Nystrom option (KrrParams.precond = "nystrom", landmark columns of the
    Gram the solver already holds) converges in a fraction of the iterations.
    CPU, fp64."""
    import libskylark_amd as sk
    from libskylark_amd.algorithms import krylov as K
    from libskylark_amd.algorithms.operators import DenseOp
    from libskylark_amd.ml import krr
    g = torch.Generator().manual_seed(0)
    n, d, lam = 3000, 16, 1e-2
    X = torch.randn(n, d, generator=g, dtype=torch.float64)
    Y = torch.randn(n, 1, generator=g, dtype=torch.float64)
    ker = sk.ml.kernel("gaussian", d, 4.0)
    Kg = ker.symmetric_gram(X)
    Kg.diagonal().add_(lam)
    op = DenseOp(Kg)

    def iters(P):
        p = K.KrylovIterParams(tolerance=1e-6, iter_lim=2000)
        A, code = K.cg(op, Y, params=p, M=P)
        assert code == -1
        assert float((Kg @ A - Y).norm() / Y.norm()) < 1e-5
        return p.iterations

    it_f = iters(krr.FeatureMapPrecond(ker, lam, X, 512, sk.Context(seed=3)))
    it_n = iters(krr.NystromPrecond(Kg, lam, 512, n, 0, sk.Context(seed=3)))
    assert it_n * 3 < it_f, (it_n, it_f)
    # the public entry point with the option
    A = sk.ml.faster_kernel_ridge(ker, X, Y, lam, 512, sk.Context(seed=3),
                                  params=krr.KrrParams(precond="nystrom", tolerance=1e-6))
    assert float((Kg @ A - Y).norm() / Y.norm()) < 1e-4
