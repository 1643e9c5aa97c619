"""C API (``libskylark_capi.so``): the reference's sl_* ABI.

Checked two ways: in-process through ctypes (joins the running interpreter)
and from a stand-alone C program compiled here (embeds CPython) — the way a
C/C++ user of the reference links ``libcskylark``.
"""
import ctypes as C
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest
import torch

import libskylark_amd as sk
from libskylark_amd._native import build as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def capi():
    B.build_capi()
    lib = C.CDLL(B.CAPI_LIB)
    lib.sl_strerror.restype = C.c_char_p
    lib.sl_supported_sketch_transforms.restype = C.c_char_p
    return lib


def _wrap(lib, A):
    A = np.asfortranarray(A, dtype=np.float64)
    h = C.c_void_p()
    assert lib.sl_wrap_raw_matrix(A.ctypes.data_as(C.c_void_p), A.shape[0], A.shape[1], C.byref(h)) == 0
    return A, h


def test_context_sketch_apply_serialize(capi):
    ctx = C.c_void_p()
    assert capi.sl_create_default_context(7, C.byref(ctx)) == 0
    S = C.c_void_p()
    assert capi.sl_create_sketch_transform(ctx, b"JLT", 50, 10, C.byref(S)) == 0
    A, hA = _wrap(capi, np.random.default_rng(0).standard_normal((50, 6)))
    SA, hSA = _wrap(capi, np.zeros((10, 6)))
    assert capi.sl_apply_sketch_transform(S, b"Matrix", hA, b"Matrix", hSA, 0) == 0
    ref = sk.sketch.JLT(50, 10, context=sk.Context(7)).apply(torch.from_numpy(A.copy()))
    np.testing.assert_allclose(SA, ref.numpy(), rtol=1e-10, atol=1e-10)
    # serialize -> deserialize -> same operator
    data = C.c_char_p()
    assert capi.sl_serialize_sketch_transform(S, C.byref(data)) == 0
    d = json.loads(data.value.decode())
    assert d["sketch_type"] == "JLT" and d["N"] == 50
    S2 = C.c_void_p()
    assert capi.sl_deserialize_sketch_transform(data.value, C.byref(S2)) == 0
    SA2, hSA2 = _wrap(capi, np.zeros((10, 6)))
    assert capi.sl_apply_sketch_transform(S2, b"Matrix", hA, b"Matrix", hSA2, 0) == 0
    np.testing.assert_allclose(SA2, SA)
    # rowwise with a parameterised transform (varargs double)
    R = C.c_void_p()
    assert capi.sl_create_sketch_transform(ctx, b"GaussianRFT", 6, 20, C.byref(R), C.c_double(1.5)) == 0
    Z, hZ = _wrap(capi, np.zeros((50, 20)))
    assert capi.sl_apply_sketch_transform(R, b"Matrix", hA, b"Matrix", hZ, 1) == 0
    assert np.abs(Z).max() <= np.sqrt(2 / 20) + 1e-12
    for h in (S, S2, R):
        assert capi.sl_free_sketch_transform(h) == 0
    assert capi.sl_free_context(ctx) == 0


def test_errors_and_info(capi):
    ctx = C.c_void_p()
    capi.sl_create_default_context(1, C.byref(ctx))
    S = C.c_void_p()
    assert capi.sl_create_sketch_transform(ctx, b"NoSuchSketch", 5, 3, C.byref(S)) == 111
    assert capi.sl_strerror(104) == b"Dimension mismatch"
    info = C.c_char_p()
    capi.sl_get_exception_info(C.byref(info))
    assert b"NoSuchSketch" in info.value
    assert b'("JLT","Matrix","Matrix")' in capi.sl_supported_sketch_transforms()


def test_sparse_output_cwt(capi):
    ctx = C.c_void_p()
    capi.sl_create_default_context(3, C.byref(ctx))
    S = C.c_void_p()
    assert capi.sl_create_sketch_transform(ctx, b"CWT", 40, 8, C.byref(S)) == 0
    rng = np.random.default_rng(1)
    Ad = rng.standard_normal((40, 5)) * (rng.random((40, 5)) < 0.3)
    import scipy.sparse as sp
    Acsc = sp.csc_matrix(Ad)
    ip = Acsc.indptr.astype(np.int32)
    ind = Acsc.indices.astype(np.int32)
    val = Acsc.data.astype(np.float64)
    hA, hO = C.c_void_p(), C.c_void_p()
    capi.sl_wrap_raw_sp_matrix(ip.ctypes.data_as(C.c_void_p), ind.ctypes.data_as(C.c_void_p),
                               val.ctypes.data_as(C.c_void_p), len(val), 40, 5, C.byref(hA))
    capi.sl_wrap_raw_sp_matrix(None, None, None, 0, 0, 0, C.byref(hO))
    assert capi.sl_apply_sketch_transform(S, b"SparseMatrix", hA, b"SparseMatrix", hO, 0) == 0
    nnz, h, w = C.c_int(), C.c_int(), C.c_int()
    capi.sl_raw_sp_matrix_nnz(hO, C.byref(nnz))
    capi.sl_raw_sp_matrix_height(hO, C.byref(h))
    capi.sl_raw_sp_matrix_width(hO, C.byref(w))
    oip = np.zeros(w.value + 1, dtype=np.int32)
    oind = np.zeros(nnz.value, dtype=np.int32)
    oval = np.zeros(nnz.value)
    capi.sl_raw_sp_matrix_data(hO, oip.ctypes.data_as(C.c_void_p), oind.ctypes.data_as(C.c_void_p),
                               oval.ctypes.data_as(C.c_void_p))
    got = sp.csc_matrix((oval, oind, oip), shape=(h.value, w.value)).toarray()
    ref = sk.sketch.CWT(40, 8, context=sk.Context(3)).apply(torch.from_numpy(Ad)).numpy()
    np.testing.assert_allclose(got, ref, atol=1e-12)
    capi.sl_free_raw_sp_matrix_wrap(hA)
    capi.sl_free_raw_sp_matrix_wrap(hO)


def test_svd_kernel_libsvm(capi, tmp_path):
    ctx = C.c_void_p()
    capi.sl_create_default_context(5, C.byref(ctx))
    rng = np.random.default_rng(2)
    U0, _ = np.linalg.qr(rng.standard_normal((200, 5)))
    V0, _ = np.linalg.qr(rng.standard_normal((30, 5)))
    A = U0 @ np.diag([10, 8, 6, 4, 2.0]) @ V0.T
    A, hA = _wrap(capi, A)
    U, hU = _wrap(capi, np.zeros((200, 5)))
    s, hS = _wrap(capi, np.zeros((5, 1)))
    V, hV = _wrap(capi, np.zeros((30, 5)))
    params = json.dumps({"oversampling_ratio": 2, "oversampling_additive": 0, "num_iterations": 2,
                         "skip_qr": False}).encode()
    assert capi.sl_approximate_svd(b"Matrix", hA, b"Matrix", hU, b"Matrix", hS, b"Matrix", hV, 5, params, ctx) == 0
    np.testing.assert_allclose(s[:, 0], [10, 8, 6, 4, 2], rtol=1e-8)
    K = C.c_void_p()
    assert capi.sl_create_kernel(b"gaussian", 30, C.byref(K), C.c_double(2.0)) == 0
    X, hX = _wrap(capi, rng.standard_normal((30, 12)))
    Km, hK = _wrap(capi, np.zeros((12, 12)))
    assert capi.sl_kernel_gram(1, 1, K, b"Matrix", hX, b"Matrix", hX, b"Matrix", hK) == 0
    d2 = ((X[:, :, None] - X[:, None, :]) ** 2).sum(0)
    np.testing.assert_allclose(Km, np.exp(-d2 / 8.0), rtol=1e-10)
    f = tmp_path / "d.libsvm"
    f.write_text("1 1:0.5 3:2\n-1 2:1.5\n")
    Xl, hXl = _wrap(capi, np.zeros((3, 2)))
    Yl, hYl = _wrap(capi, np.zeros((1, 2)))
    assert capi.sl_readlibsvm(str(f).encode(), b"Matrix", hXl, b"Matrix", hYl, 1, 0, -1) == 0
    np.testing.assert_allclose(Xl, [[0.5, 0], [0, 1.5], [2, 0]])
    np.testing.assert_allclose(Yl, [[1, -1]])


C_PROGRAM = textwrap.dedent(r"""
    #include <stdio.h>
    #include <stdlib.h>
    #include <stdint.h>
    typedef struct sl_context_t sl_context_t;
    typedef struct sl_sketch_transform_t sl_sketch_transform_t;
    int sl_create_default_context(int, sl_context_t**);
    int sl_create_sketch_transform(sl_context_t*, char*, int, int, sl_sketch_transform_t**, ...);
    int sl_apply_sketch_transform(sl_sketch_transform_t*, char*, void*, char*, void*, int);
    int sl_serialize_sketch_transform(const sl_sketch_transform_t*, char**);
    int sl_wrap_raw_matrix(double*, int, int, void**);
    int sl_free_sketch_transform(sl_sketch_transform_t*);
    int sl_free_context(sl_context_t*);
    int main(void) {
        sl_context_t* ctx; sl_sketch_transform_t* S; void *A, *SA;
        double a[20 * 3], sa[4 * 3];
        for (int i = 0; i < 60; ++i) a[i] = (double)(i % 7) - 3.0;
        if (sl_create_default_context(11, &ctx)) return 1;
        if (sl_create_sketch_transform(ctx, "FJLT", 20, 4, &S)) return 2;
        sl_wrap_raw_matrix(a, 20, 3, &A);
        sl_wrap_raw_matrix(sa, 4, 3, &SA);
        if (sl_apply_sketch_transform(S, "Matrix", A, "Matrix", SA, 0)) return 3;
        for (int i = 0; i < 12; ++i) printf("%.17g\n", sa[i]);
        sl_free_sketch_transform(S); sl_free_context(ctx);
        return 0;
    }
""")


def test_standalone_c_program(capi, tmp_path):
    import sysconfig
    src = tmp_path / "prog.c"
    src.write_text(C_PROGRAM)
    exe = tmp_path / "prog"
    libdir = os.path.dirname(B.CAPI_LIB)
    r = subprocess.run(["gcc", str(src), "-o", str(exe), f"-L{libdir}", "-lskylark_capi", f"-Wl,-rpath,{libdir}",
                        f"-Wl,-rpath,{sysconfig.get_config_var('LIBDIR')}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, PYTHONPATH=ROOT, SKH_NO_BUILD="1", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.array([float(x) for x in r.stdout.split()]).reshape(3, 4).T
    a = np.array([(i % 7) - 3.0 for i in range(60)]).reshape(3, 20).T
    ref = sk.sketch.FJLT(20, 4, context=sk.Context(11)).apply(torch.from_numpy(a)).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)
