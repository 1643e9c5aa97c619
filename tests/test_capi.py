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


@pytest.mark.parametrize("typ,param", [("JLT", None), ("CT", 2.5), ("CWT", None), ("MMT", None), ("WZT", 1.5)])
def test_native_sketch_parity(capi, typ, param):
    """The interpreter-free C path (native_sketch.hpp) builds the same operator
    as the runtime from the same context stream: apply both ways, JSON both
    ways, and a second sketch from the same context (counter advanced alike)."""
    N, S, n = 37, 9, 5
    ctx = C.c_void_p()
    assert capi.sl_create_default_context(13, C.byref(ctx)) == 0
    pctx = sk.Context(13)
    cls = getattr(sk.sketch, typ)
    hs, pys = [], []
    for _ in range(2):     # the second draw checks the counter bookkeeping
        h = C.c_void_p()
        args = [C.c_double(param)] if param is not None else []
        assert capi.sl_create_sketch_transform(ctx, typ.encode(), N, S, C.byref(h), *args) == 0
        hs.append(h)
        pys.append(cls(N, S, param, context=pctx) if param is not None else cls(N, S, context=pctx))
    rng = np.random.default_rng(1)
    A = rng.standard_normal((N, n))
    B = rng.standard_normal((n, N))
    for h, T in zip(hs, pys):
        Aw, hA = _wrap(capi, A)
        SA, hSA = _wrap(capi, np.zeros((S, n)))
        assert capi.sl_apply_sketch_transform(h, b"Matrix", hA, b"Matrix", hSA, 0) == 0
        np.testing.assert_allclose(SA, T.apply(torch.from_numpy(A.copy()), dim=0).numpy(), rtol=1e-11, atol=1e-11)
        Bw, hB = _wrap(capi, B)
        SB, hSB = _wrap(capi, np.zeros((n, S)))
        assert capi.sl_apply_sketch_transform(h, b"Matrix", hB, b"Matrix", hSB, 1) == 0
        np.testing.assert_allclose(SB, T.apply(torch.from_numpy(B.copy()), dim=1).numpy(), rtol=1e-11, atol=1e-11)
        # C JSON -> runtime, runtime JSON -> C
        data = C.c_char_p()
        assert capi.sl_serialize_sketch_transform(h, C.byref(data)) == 0
        T2 = sk.sketch.deserialize_sketch(json.loads(data.value.decode()))
        np.testing.assert_allclose(T2.apply(torch.from_numpy(A.copy()), dim=0).numpy(), SA, rtol=1e-11, atol=1e-11)
        h2 = C.c_void_p()
        assert capi.sl_deserialize_sketch_transform(T.to_json().encode(), C.byref(h2)) == 0
        SA2, hSA2 = _wrap(capi, np.zeros((S, n)))
        assert capi.sl_apply_sketch_transform(h2, b"Matrix", hA, b"Matrix", hSA2, 0) == 0
        np.testing.assert_allclose(SA2, SA, rtol=0, atol=0)
        # dimension mismatch is the reference's code 104
        bad, hbad = _wrap(capi, np.zeros((S + 1, n)))
        assert capi.sl_apply_sketch_transform(h, b"Matrix", hA, b"Matrix", hbad, 0) == 104
        capi.sl_free_sketch_transform(h2)
    for h in hs:
        capi.sl_free_sketch_transform(h)
    capi.sl_free_context(ctx)


C_NATIVE_PROGRAM = textwrap.dedent(r"""
    #include <stdio.h>
    #include <stdlib.h>
    typedef struct sl_context_t sl_context_t;
    typedef struct sl_sketch_transform_t sl_sketch_transform_t;
    int sl_create_default_context(int, sl_context_t**);
    int sl_create_sketch_transform(sl_context_t*, char*, int, int, sl_sketch_transform_t**, ...);
    int sl_apply_sketch_transform(sl_sketch_transform_t*, char*, void*, char*, void*, int);
    int sl_serialize_sketch_transform(const sl_sketch_transform_t*, char**);
    int sl_wrap_raw_matrix(double*, int, int, void**);
    int sl_free_sketch_transform(sl_sketch_transform_t*);
    int sl_free_context(sl_context_t*);
    int sl_runtime_started(void);
    int main(void) {
        sl_context_t* ctx; sl_sketch_transform_t *J, *W;
        if (sl_create_default_context(21, &ctx)) return 1;
        if (sl_create_sketch_transform(ctx, "JLT", 30, 6, &J)) return 2;
        if (sl_create_sketch_transform(ctx, "WZT", 30, 6, &W, 1.5)) return 3;
        double a[30 * 2], sa[6 * 2], sw[6 * 2];
        for (int i = 0; i < 60; ++i) a[i] = (i % 5) - 2.0;
        void *hA, *hS, *hW;
        sl_wrap_raw_matrix(a, 30, 2, &hA); sl_wrap_raw_matrix(sa, 6, 2, &hS); sl_wrap_raw_matrix(sw, 6, 2, &hW);
        if (sl_apply_sketch_transform(J, "Matrix", hA, "Matrix", hS, 0)) return 4;
        if (sl_apply_sketch_transform(W, "Matrix", hA, "Matrix", hW, 0)) return 5;
        char* js; if (sl_serialize_sketch_transform(W, &js)) return 6;
        for (int i = 0; i < 12; ++i) printf("%.17g ", sa[i]);
        for (int i = 0; i < 12; ++i) printf("%.17g ", sw[i]);
        printf("\n%s\n%d\n", js, sl_runtime_started());
        free(js); sl_free_sketch_transform(J); sl_free_sketch_transform(W); sl_free_context(ctx);
        return 0;
    }
""")


def test_native_c_program_is_interpreter_free(capi, tmp_path):
    """A C program using only contexts and the native sketches never starts
    the embedded runtime, and computes the runtime's operator."""
    import sysconfig
    src = tmp_path / "nat.c"
    src.write_text(C_NATIVE_PROGRAM)
    exe = tmp_path / "nat"
    libdir = os.path.dirname(B.CAPI_LIB)
    r = subprocess.run(["gcc", str(src), "-o", str(exe), f"-L{libdir}", "-lskylark_capi", f"-Wl,-rpath,{libdir}",
                        f"-Wl,-rpath,{sysconfig.get_config_var('LIBDIR')}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().split("\n")
    vals = np.array([float(x) for x in lines[0].split()])
    assert lines[2].strip() == "0"                      # runtime never started
    a = np.array([(i % 5) - 2.0 for i in range(60)]).reshape(2, 30).T
    ctx = sk.Context(21)
    J = sk.sketch.JLT(30, 6, context=ctx)
    W = sk.sketch.WZT(30, 6, 1.5, context=ctx)
    np.testing.assert_allclose(vals[:12].reshape(2, 6).T, J.apply(torch.from_numpy(a)).numpy(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(vals[12:].reshape(2, 6).T, W.apply(torch.from_numpy(a)).numpy(), rtol=1e-12, atol=1e-12)
    assert json.loads(lines[1])["sketch_type"] == "WZT"
