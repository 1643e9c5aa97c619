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


C_DEVICE_PROGRAM = textwrap.dedent(r"""
    #include <math.h>
    #include <stdint.h>
    #include <stdio.h>
    #include <stdlib.h>
    #include <string.h>
    typedef struct sl_context_t sl_context_t;
    typedef struct sl_sketch_transform_t sl_sketch_transform_t;
    typedef struct sl_kernel_t sl_kernel_t;
    int sl_create_default_context(int, sl_context_t**);
    int sl_create_sketch_transform(sl_context_t*, char*, int, int, sl_sketch_transform_t**, ...);
    int sl_apply_sketch_transform(sl_sketch_transform_t*, char*, void*, char*, void*, int);
    int sl_free_sketch_transform(sl_sketch_transform_t*);
    int sl_approximate_svd(char*, void*, char*, void*, char*, void*, char*, void*, uint16_t, char*, sl_context_t*);
    int sl_create_kernel(char*, int, sl_kernel_t**, ...);
    int sl_kernel_gram(int, int, sl_kernel_t*, char*, void*, char*, void*, char*, void*);
    int sl_free_kernel(sl_kernel_t*);
    int sl_free_context(sl_context_t*);
    int sl_runtime_started(void);
    int sl_wrap_raw_device_matrix(void*, int, int, int, int64_t, void**);
    int sl_free_raw_device_matrix_wrap(void*);
    int sl_device_malloc(int64_t, void**);
    int sl_device_free(void*);
    int sl_device_memcpy(void*, const void*, int64_t, int);
    void sl_get_exception_info(char**);
    int sl_create_context(int, void*, sl_context_t**);
    int sl_device_comm_id_bytes(void);
    int sl_device_comm_unique_id(void*);
    int sl_device_comm_create(const void*, int, int, void**);
    int sl_device_comm_free(void*);

    static uint64_t st = 88172645463325252ull;
    static double urand(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (st >> 11) * (1.0 / 9007199254740992.0) - 0.5; }
    static int fail(int code, int rc) { char* e; sl_get_exception_info(&e); fprintf(stderr, "step %d rc %d: %s\n", code, rc, e); return code; }
    static void* up(const void* h, int64_t bytes) { void* d; if (sl_device_malloc(bytes, &d)) return NULL; sl_device_memcpy(d, h, bytes, 0); return d; }
    static void* dev(int64_t bytes) { void* d; return sl_device_malloc(bytes, &d) ? NULL : d; }
    static void dump(const char* dir, const char* name, const void* d, int64_t bytes) {
        void* h = malloc(bytes); sl_device_memcpy(h, d, bytes, 1);
        char p[1024]; snprintf(p, sizeof p, "%s/%s.bin", dir, name);
        FILE* f = fopen(p, "wb"); fwrite(h, 1, bytes, f); fclose(f); free(h);
    }
    static void* wrap(void* d, int dt, int m, int n) { void* w; sl_wrap_raw_device_matrix(d, dt, m, n, n, &w); return w; }
    static uint16_t bf16(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7fffu + ((u >> 16) & 1u); return (uint16_t)(u >> 16); }

    int main(int argc, char** argv) {
        const char* out = argv[1];
        int rc;
        sl_context_t* ctx; if (sl_create_default_context(17, &ctx)) return 1;
        sl_sketch_transform_t *J, *F, *W;
        if ((rc = sl_create_sketch_transform(ctx, "JLT", 300, 20, &J))) return fail(2, rc);
        if ((rc = sl_create_sketch_transform(ctx, "FJLT", 300, 16, &F))) return fail(3, rc);
        if ((rc = sl_create_sketch_transform(ctx, "CWT", 300, 10, &W))) return fail(4, rc);
        /* JLT columnwise, f64: A 300 x 7 -> 20 x 7 */
        double* a = malloc(300 * 7 * 8); for (int i = 0; i < 300 * 7; ++i) a[i] = urand();
        void* dA = up(a, 300 * 7 * 8); void* dSA = dev(20 * 7 * 8);
        if ((rc = sl_apply_sketch_transform(J, "DeviceMatrix", wrap(dA, 1, 300, 7), "DeviceMatrix", wrap(dSA, 1, 20, 7), 0))) return fail(5, rc);
        dump(out, "jlt_A", dA, 300 * 7 * 8); dump(out, "jlt_SA", dSA, 20 * 7 * 8);
        /* FJLT rowwise, f32: A 9 x 300 -> 9 x 16 */
        float* b = malloc(9 * 300 * 4); for (int i = 0; i < 9 * 300; ++i) b[i] = (float)urand();
        void* dB = up(b, 9 * 300 * 4); void* dSB = dev(9 * 16 * 4);
        if ((rc = sl_apply_sketch_transform(F, "DeviceMatrix", wrap(dB, 0, 9, 300), "DeviceMatrix", wrap(dSB, 0, 9, 16), 1))) return fail(6, rc);
        dump(out, "fjlt_A", dB, 9 * 300 * 4); dump(out, "fjlt_SA", dSB, 9 * 16 * 4);
        /* CWT columnwise, f32: A 300 x 5 -> 10 x 5 */
        float* c = malloc(300 * 5 * 4); for (int i = 0; i < 300 * 5; ++i) c[i] = (float)urand();
        void* dC = up(c, 300 * 5 * 4); void* dSC = dev(10 * 5 * 4);
        if ((rc = sl_apply_sketch_transform(W, "DeviceMatrix", wrap(dC, 0, 300, 5), "DeviceMatrix", wrap(dSC, 0, 10, 5), 0))) return fail(7, rc);
        dump(out, "cwt_A", dC, 300 * 5 * 4); dump(out, "cwt_SA", dSC, 10 * 5 * 4);
        /* randSVD of a bf16 4096 x 64 matrix with a decaying spectrum, rank 5, q = 2 */
        const int m = 4096, n = 64, r = 5;
        float* u = malloc(m * 8 * 4); float* v = malloc(n * 8 * 4);
        for (int i = 0; i < m * 8; ++i) u[i] = (float)urand();
        for (int i = 0; i < n * 8; ++i) v[i] = (float)urand();
        uint16_t* ab = malloc((size_t)m * n * 2);
        for (int i = 0; i < m; ++i) for (int j = 0; j < n; ++j) {
            double x = 0.01 * urand();
            for (int t = 0; t < 8; ++t) x += pow(0.5, t) * u[i * 8 + t] * v[j * 8 + t];
            ab[(size_t)i * n + j] = bf16((float)x);
        }
        void* dX = up(ab, (int64_t)m * n * 2); void* dU = dev(m * r * 4); void* dS = dev(r * 4); void* dV = dev(n * r * 4);
        void *wX = wrap(dX, 2, m, n), *wU = wrap(dU, 0, m, r), *wS = wrap(dS, 0, r, 1), *wV = wrap(dV, 0, n, r);
        char prm[] = "{\"num_iterations\": 2, \"sketch\": \"JLT\"}";
        if ((rc = sl_approximate_svd("DeviceMatrix", wX, "DeviceMatrix", wU, "DeviceMatrix", wS, "DeviceMatrix", wV, r, prm, ctx))) return fail(8, rc);
        dump(out, "svd_A", dX, (int64_t)m * n * 2); dump(out, "svd_U", dU, m * r * 4); dump(out, "svd_S", dS, r * 4); dump(out, "svd_V", dV, n * r * 4);
        /* second call replays the engine's graph: same operator counter advances */
        if ((rc = sl_approximate_svd("DeviceMatrix", wX, "DeviceMatrix", wU, "DeviceMatrix", wS, "DeviceMatrix", wV, r, prm, ctx))) return fail(9, rc);
        dump(out, "svd_S2", dS, r * 4);
        /* Gaussian Gram: X 50 points as rows (f64, 50 x 8), Y 30 points as columns (8 x 30) */
        double* x = malloc(50 * 8 * 8); double* y = malloc(8 * 30 * 8);
        for (int i = 0; i < 400; ++i) x[i] = urand();
        for (int i = 0; i < 240; ++i) y[i] = urand();
        void* dXk = up(x, 50 * 8 * 8); void* dYk = up(y, 8 * 30 * 8); void* dK = dev(50 * 30 * 8); void* dK2 = dev(50 * 30 * 8);
        sl_kernel_t *G, *Lk;
        if ((rc = sl_create_kernel("gaussian", 8, &G, 0.7))) return fail(10, rc);
        if ((rc = sl_create_kernel("laplacian", 8, &Lk, 1.3))) return fail(11, rc);
        if ((rc = sl_kernel_gram(2, 1, G, "DeviceMatrix", wrap(dXk, 1, 50, 8), "DeviceMatrix", wrap(dYk, 1, 8, 30), "DeviceMatrix", wrap(dK, 1, 50, 30)))) return fail(12, rc);
        if ((rc = sl_kernel_gram(2, 1, Lk, "DeviceMatrix", wrap(dXk, 1, 50, 8), "DeviceMatrix", wrap(dYk, 1, 8, 30), "DeviceMatrix", wrap(dK2, 1, 50, 30)))) return fail(13, rc);
        dump(out, "k_X", dXk, 400 * 8); dump(out, "k_Y", dYk, 240 * 8); dump(out, "k_G", dK, 1500 * 8); dump(out, "k_L", dK2, 1500 * 8);
        /* the distributed call over a (1-rank) RCCL device communicator equals the local call */
        char id[512]; int nb = sl_device_comm_id_bytes(); if (nb <= 0 || nb > 512) return fail(14, nb);
        if ((rc = sl_device_comm_unique_id(id))) return fail(15, rc);
        void* comm; if ((rc = sl_device_comm_create(id, 1, 0, &comm))) return fail(16, rc);
        sl_context_t *c2, *c3; sl_create_context(5, comm, &c2); sl_create_default_context(5, &c3);
        char prm2[] = "{\"num_iterations\": 1, \"sketch\": \"FJLT\"}";
        if ((rc = sl_approximate_svd("DeviceMatrix", wX, "DeviceMatrix", wU, "DeviceMatrix", wS, "DeviceMatrix", wV, r, prm2, c2))) return fail(17, rc);
        dump(out, "svd_S_comm", dS, r * 4);
        if ((rc = sl_approximate_svd("DeviceMatrix", wX, "DeviceMatrix", wU, "DeviceMatrix", wS, "DeviceMatrix", wV, r, prm2, c3))) return fail(18, rc);
        dump(out, "svd_S_local", dS, r * 4);
        sl_device_comm_free(comm); sl_free_context(c2); sl_free_context(c3);
        printf("%d\n", sl_runtime_started());
        sl_free_kernel(G); sl_free_kernel(Lk);
        sl_free_sketch_transform(J); sl_free_sketch_transform(F); sl_free_sketch_transform(W); sl_free_context(ctx);
        return 0;
    }
""")


@pytest.mark.gpu
def test_device_c_program_is_interpreter_free(capi, tmp_path):
    """A C program runs device sketches (JLT / FJLT / CWT), the randSVD engine
    and a kernel Gram on GPU buffers through the C ABI without ever starting
    the interpreter, and matches the Python runtime's results on the same
    contexts (reference capi/csketch.cpp:614-680,
    capi/cnla.cpp:15-84, capi/ckernel.cpp:34-128)."""
    import sysconfig
    src = tmp_path / "dev.c"
    src.write_text(C_DEVICE_PROGRAM)
    exe = tmp_path / "dev"
    libdir = os.path.dirname(B.CAPI_LIB)
    r = subprocess.run(["gcc", str(src), "-o", str(exe), f"-L{libdir}", "-lskylark_capi", f"-Wl,-rpath,{libdir}",
                        f"-Wl,-rpath,{sysconfig.get_config_var('LIBDIR')}", "-lm"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().split("\n")[-1] == "0"      # the runtime never started

    def ld(name, dt, shape):
        return torch.from_numpy(np.fromfile(tmp_path / f"{name}.bin", dtype=dt).reshape(shape))

    dev = torch.device("cuda")
    ctx = sk.Context(17)
    J = sk.sketch.JLT(300, 20, context=ctx)
    F = sk.sketch.FJLT(300, 16, context=ctx)
    W = sk.sketch.CWT(300, 10, context=ctx)
    A = ld("jlt_A", np.float64, (300, 7))
    torch.testing.assert_close(ld("jlt_SA", np.float64, (20, 7)), J.apply(A, dim=0), rtol=1e-10, atol=1e-10)
    B_ = ld("fjlt_A", np.float32, (9, 300))
    ref = F.apply(B_.double(), dim=1).float()
    torch.testing.assert_close(ld("fjlt_SA", np.float32, (9, 16)), ref, rtol=1e-4, atol=1e-4)
    Cm = ld("cwt_A", np.float32, (300, 5))
    torch.testing.assert_close(ld("cwt_SA", np.float32, (10, 5)), W.apply(Cm.double(), dim=0).float(),
                               rtol=1e-5, atol=1e-5)
    # randSVD: same engine, same sketch stream -> same factors
    Ab = ld("svd_A", np.int16, (4096, 64)).view(torch.bfloat16).to(dev)
    p = sk.nla.ApproximateSVDParams(num_iterations=2, sketch="JLT")
    U, s, V = sk.nla.approximate_svd(Ab, 5, ctx, p)
    sc = ld("svd_S", np.float32, (5,))
    torch.testing.assert_close(sc, s.cpu(), rtol=1e-5, atol=1e-5)
    Uc = ld("svd_U", np.float32, (4096, 5)).double()
    cos = torch.linalg.svdvals(Uc.t() @ U.cpu().double())
    assert float(cos.min()) > 0.9999, cos
    s_true = torch.linalg.svdvals(Ab.double().cpu())[:5]
    assert float(((sc.double() - s_true).abs() / s_true).max()) < 1e-2
    U2, s2, _ = sk.nla.approximate_svd(Ab, 5, ctx, p)
    torch.testing.assert_close(ld("svd_S2", np.float32, (5,)), s2.cpu(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ld("svd_S_comm", np.float32, (5,)), ld("svd_S_local", np.float32, (5,)),
                               rtol=1e-6, atol=1e-6)
    # kernel Grams (points: X rows, Y columns)
    X = ld("k_X", np.float64, (50, 8))
    Y = ld("k_Y", np.float64, (8, 30))
    G = sk.ml.kernel("gaussian", 8, 0.7)
    Lk = sk.ml.kernel("laplacian", 8, 1.3)
    torch.testing.assert_close(ld("k_G", np.float64, (50, 30)), G.gram(X, dirX="rows", dirY="columns", Y=Y),
                               rtol=1e-10, atol=1e-12)
    torch.testing.assert_close(ld("k_L", np.float64, (50, 30)), Lk.gram(X, dirX="rows", dirY="columns", Y=Y),
                               rtol=1e-10, atol=1e-12)


# every sketch type of the runtime, created natively by the C ABI (varargs as
# the reference's csketch.cpp) -- parity with the runtime's operator on the
# same context stream, JSON both ways, dense and sparse host operands
ALL_TYPES = [
    ("SJLT", []), ("UST", []), ("FJLT", []),
    ("GaussianRFT", [1.5]), ("LaplacianRFT", [0.8]), ("MaternRFT", [1.5, 2.0]),
    ("GaussianQRFT", [1.2, 3]), ("LaplacianQRFT", [0.9, 0]), ("ExpSemigroupRLT", [0.7]),
    ("ExpSemigroupQRLT", [0.6, 2]), ("FastGaussianRFT", [1.3]), ("FastMaternRFT", [2.5, 1.1]),
    ("PPT", [3, 0.5, 0.7]),
]


def _cargs(typ, params):
    spec = {"GaussianQRFT": "di", "LaplacianQRFT": "di", "ExpSemigroupQRLT": "di", "PPT": "idd"}.get(typ, "d" * len(params))
    return [C.c_int(int(p)) if c == "i" else C.c_double(float(p)) for c, p in zip(spec, params)]


def _pysketch(typ, N, S, params, ctx):
    cls = getattr(sk.sketch, typ)
    if typ in ("GaussianQRFT", "LaplacianQRFT", "ExpSemigroupQRLT"):
        return cls(N, S, params[0], skip=int(params[1]), context=ctx)
    if typ == "PPT":
        return cls(N, S, int(params[0]), params[1], params[2], context=ctx)
    return cls(N, S, *params, context=ctx)


def _apply_both(capi, h, T, A, dim, S):
    Aw, hA = _wrap(capi, A)
    shape = (S, A.shape[1]) if dim == 0 else (A.shape[0], S)
    SA, hSA = _wrap(capi, np.zeros(shape))
    assert capi.sl_apply_sketch_transform(h, b"Matrix", hA, b"Matrix", hSA, dim) == 0
    ref = T.apply(torch.from_numpy(A.copy()), dim=dim)
    ref = ref.to_dense() if ref.layout != torch.strided else ref
    return SA, ref.double().numpy()


@pytest.mark.parametrize("typ,params", ALL_TYPES, ids=[t for t, _ in ALL_TYPES])
def test_native_all_sketch_types(capi, typ, params):
    N, S, n = 37, 80 if typ.startswith("Fast") else 16, 5
    ctx = C.c_void_p()
    assert capi.sl_create_default_context(29, C.byref(ctx)) == 0
    pctx = sk.Context(29)
    rng = np.random.default_rng(3)
    pos = typ.startswith("ExpSemigroup")
    for rep in range(2):   # the second sketch checks the counter bookkeeping
        h = C.c_void_p()
        assert capi.sl_create_sketch_transform(ctx, typ.encode(), N, S, C.byref(h), *_cargs(typ, params)) == 0
        T = _pysketch(typ, N, S, params, pctx)
        A = rng.standard_normal((N, n))
        B = rng.standard_normal((n, N))
        if pos:
            A, B = np.abs(A) * 0.1, np.abs(B) * 0.1
        got, ref = _apply_both(capi, h, T, A, 0, S)
        np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-10, err_msg=f"{typ} columnwise rep {rep}")
        got, ref = _apply_both(capi, h, T, B, 1, S)
        np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-10, err_msg=f"{typ} rowwise rep {rep}")
        # C JSON -> runtime, runtime JSON -> C
        data = C.c_char_p()
        assert capi.sl_serialize_sketch_transform(h, C.byref(data)) == 0
        T2 = sk.sketch.deserialize_sketch(json.loads(data.value.decode()))
        got, _ = _apply_both(capi, h, T2, A, 0, S)
        np.testing.assert_allclose(T2.apply(torch.from_numpy(A.copy()), dim=0).double().numpy(), got, rtol=1e-9,
                                   atol=1e-10)
        h2 = C.c_void_p()
        assert capi.sl_deserialize_sketch_transform(T.to_json().encode(), C.byref(h2)) == 0
        got2, ref = _apply_both(capi, h2, T, A, 0, S)
        np.testing.assert_allclose(got2, ref, rtol=1e-9, atol=1e-10)
        capi.sl_free_sketch_transform(h2)
        capi.sl_free_sketch_transform(h)
    capi.sl_free_context(ctx)


def _wrap_csc(capi, Ad):
    import scipy.sparse as sp
    Acsc = sp.csc_matrix(Ad)
    arrs = (Acsc.indptr.astype(np.int32), Acsc.indices.astype(np.int32), Acsc.data.astype(np.float64))
    h = C.c_void_p()
    capi.sl_wrap_raw_sp_matrix(arrs[0].ctypes.data_as(C.c_void_p), arrs[1].ctypes.data_as(C.c_void_p),
                               arrs[2].ctypes.data_as(C.c_void_p), len(arrs[2]), Ad.shape[0], Ad.shape[1], C.byref(h))
    return arrs, h


def _read_sparse(capi, hO):
    import scipy.sparse as sp
    nnz, h, w = C.c_int(), C.c_int(), C.c_int()
    capi.sl_raw_sp_matrix_nnz(hO, C.byref(nnz))
    capi.sl_raw_sp_matrix_height(hO, C.byref(h))
    capi.sl_raw_sp_matrix_width(hO, C.byref(w))
    oip = np.zeros(w.value + 1, dtype=np.int32)
    oind = np.zeros(nnz.value, dtype=np.int32)
    oval = np.zeros(nnz.value)
    capi.sl_raw_sp_matrix_data(hO, oip.ctypes.data_as(C.c_void_p), oind.ctypes.data_as(C.c_void_p),
                               oval.ctypes.data_as(C.c_void_p))
    return sp.csc_matrix((oval, oind, oip), shape=(h.value, w.value)).toarray()


@pytest.mark.parametrize("typ,params,sparse_out", [("JLT", [], False), ("CWT", [], True), ("WZT", [1.3], True),
                                                   ("GaussianRFT", [1.1], False), ("UST", [], True),
                                                   ("PPT", [2, 1.0, 0.5], False)])
def test_native_sparse_input(capi, typ, params, sparse_out):
    """SparseMatrix (CSC) inputs on the native path, dense or sparse outputs,
    both directions, against the runtime on the dense equivalent."""
    N, S, n = 40, 12, 6
    ctx = C.c_void_p()
    capi.sl_create_default_context(31, C.byref(ctx))
    h = C.c_void_p()
    assert capi.sl_create_sketch_transform(ctx, typ.encode(), N, S, C.byref(h), *_cargs(typ, params)) == 0
    T = _pysketch(typ, N, S, params, sk.Context(31))
    rng = np.random.default_rng(4)
    for dim in (0, 1):
        Ad = rng.standard_normal((N, n) if dim == 0 else (n, N)) * (rng.random((N, n) if dim == 0 else (n, N)) < 0.3)
        arrs, hA = _wrap_csc(capi, Ad)
        shape = (S, n) if dim == 0 else (n, S)
        if sparse_out:
            hO = C.c_void_p()
            capi.sl_wrap_raw_sp_matrix(None, None, None, 0, 0, 0, C.byref(hO))
            assert capi.sl_apply_sketch_transform(h, b"SparseMatrix", hA, b"SparseMatrix", hO, dim) == 0
            got = _read_sparse(capi, hO)
            upd = C.c_bool()
            capi.sl_raw_sp_matrix_struct_updated(hO, C.byref(upd))
            assert upd.value
            capi.sl_free_raw_sp_matrix_wrap(hO)
        else:
            got, hO = _wrap(capi, np.zeros(shape))
            assert capi.sl_apply_sketch_transform(h, b"SparseMatrix", hA, b"Matrix", hO, dim) == 0
        ref = T.apply(torch.from_numpy(Ad.copy()), dim=dim).double().numpy()
        np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-10, err_msg=f"{typ} dim {dim}")
        capi.sl_free_raw_sp_matrix_wrap(hA)
    capi.sl_free_sketch_transform(h)


@pytest.mark.parametrize("js", [
    {"sketch_type": "UST", "replace": False},
    {"sketch_type": "NURST", "p": list(np.linspace(0.1, 2.0, 30))},
    {"sketch_type": "GaussianQRFT", "sigma": 2.0, "skip": 5,
     "sequence": {"skylark_object_type": "qmc_sequence", "sequence_type": "leaped halton", "d": 31, "leap": 7}},
])
def test_native_deserialized_types(capi, js):
    """Types / parameters reachable only through JSON (UST without
    replacement, NURST's probability vector, a custom QMC leap)."""
    d = {"skylark_object_type": "sketch", "skylark_version": "0.1.0", "N": 30, "S": 9,
         "creation_context": {"skylark_object_type": "context", "seed": 77, "counter": 1234}}
    d.update(js)
    T = sk.sketch.deserialize_sketch(d)
    h = C.c_void_p()
    assert capi.sl_deserialize_sketch_transform(json.dumps(d).encode(), C.byref(h)) == 0
    A = np.random.default_rng(5).standard_normal((30, 4))
    got, ref = _apply_both(capi, h, T, A, 0, 9)
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-10)
    data = C.c_char_p()
    capi.sl_serialize_sketch_transform(h, C.byref(data))
    T2 = sk.sketch.deserialize_sketch(json.loads(data.value.decode()))
    np.testing.assert_allclose(T2.apply(torch.from_numpy(A.copy()), dim=0).numpy(), ref, rtol=1e-12, atol=1e-12)
    capi.sl_free_sketch_transform(h)


C_HOST_DEVICE_PROGRAM = textwrap.dedent(r"""
    #include <math.h>
    #include <stdint.h>
    #include <stdio.h>
    #include <stdlib.h>
    #include <string.h>
    typedef struct sl_context_t sl_context_t;
    typedef struct sl_sketch_transform_t sl_sketch_transform_t;
    int sl_create_default_context(int, sl_context_t**);
    int sl_create_sketch_transform(sl_context_t*, char*, int, int, sl_sketch_transform_t**, ...);
    int sl_apply_sketch_transform(sl_sketch_transform_t*, char*, void*, char*, void*, int);
    int sl_free_sketch_transform(sl_sketch_transform_t*);
    int sl_approximate_svd(char*, void*, char*, void*, char*, void*, char*, void*, uint16_t, char*, sl_context_t*);
    int sl_approximate_symmetric_svd(char*, void*, char*, void*, char*, void*, uint16_t, char*, sl_context_t*);
    int sl_faster_least_squares(int, char*, void*, char*, void*, char*, void*, char*, sl_context_t*);
    int sl_readlibsvm(char*, char*, void*, char*, void*, int, int, int);
    typedef struct sl_kernel_t sl_kernel_t;
    int sl_create_kernel(char*, int, sl_kernel_t**, ...);
    int sl_kernel_gram(int, int, sl_kernel_t*, char*, void*, char*, void*, char*, void*);
    int sl_free_kernel(sl_kernel_t*);
    int sl_free_context(sl_context_t*);
    int sl_runtime_started(void);
    int sl_wrap_raw_matrix(double*, int, int, void**);
    int sl_wrap_raw_sp_matrix(int*, int*, double*, int, int, int, void**);
    int sl_raw_sp_matrix_nnz(void*, int*);
    int sl_raw_sp_matrix_data(void*, int32_t*, int32_t*, double*);
    void sl_get_exception_info(char**);

    static uint64_t st = 88172645463325252ull;
    static double urand(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (st >> 11) * (1.0 / 9007199254740992.0); }
    static const char* OUT;
    static int fail(int code, int rc) { char* e; sl_get_exception_info(&e); fprintf(stderr, "step %d rc %d: %s\n", code, rc, e); return code; }
    static void dump(const char* name, const void* p, size_t bytes) {
        char path[1024]; snprintf(path, sizeof path, "%s/%s.bin", OUT, name);
        FILE* f = fopen(path, "wb"); fwrite(p, 1, bytes, f); fclose(f);
    }
    static void* W(double* d, int m, int n) { void* w; sl_wrap_raw_matrix(d, m, n, &w); return w; }

    #define N 300
    static double A[N * 7], B[9 * N];
    static int apply_pair(sl_sketch_transform_t* T, const char* name, int S, int step) {
        double* sa = calloc((size_t)S * 7, 8); double* sb = calloc((size_t)9 * S, 8);
        int rc;
        if ((rc = sl_apply_sketch_transform(T, "Matrix", W(A, N, 7), "Matrix", W(sa, S, 7), 0))) return fail(step, rc);
        if ((rc = sl_apply_sketch_transform(T, "Matrix", W(B, 9, N), "Matrix", W(sb, 9, S), 1))) return fail(step + 1, rc);
        char nm[128];
        snprintf(nm, sizeof nm, "%s_c", name); dump(nm, sa, (size_t)S * 7 * 8);
        snprintf(nm, sizeof nm, "%s_r", name); dump(nm, sb, (size_t)9 * S * 8);
        free(sa); free(sb);
        return 0;
    }

    int main(int argc, char** argv) {
        OUT = argv[1];
        int rc;
        for (int i = 0; i < N * 7; ++i) A[i] = urand();
        for (int i = 0; i < 9 * N; ++i) B[i] = urand();
        dump("A", A, sizeof A); dump("B", B, sizeof B);
        sl_context_t* ctx; if (sl_create_default_context(41, &ctx)) return 1;
        sl_sketch_transform_t* T[18];
        if ((rc = sl_create_sketch_transform(ctx, "JLT", N, 64, &T[0]))) return fail(2, rc);
        if ((rc = sl_create_sketch_transform(ctx, "CT", N, 64, &T[1], 2.0))) return fail(3, rc);
        if ((rc = sl_create_sketch_transform(ctx, "SJLT", N, 64, &T[2]))) return fail(4, rc);
        if ((rc = sl_create_sketch_transform(ctx, "CWT", N, 64, &T[3]))) return fail(5, rc);
        if ((rc = sl_create_sketch_transform(ctx, "MMT", N, 64, &T[4]))) return fail(6, rc);
        if ((rc = sl_create_sketch_transform(ctx, "WZT", N, 64, &T[5], 1.5))) return fail(7, rc);
        if ((rc = sl_create_sketch_transform(ctx, "FJLT", N, 64, &T[6]))) return fail(8, rc);
        if ((rc = sl_create_sketch_transform(ctx, "UST", N, 64, &T[7]))) return fail(9, rc);
        if ((rc = sl_create_sketch_transform(ctx, "GaussianRFT", N, 64, &T[8], 1.5))) return fail(10, rc);
        if ((rc = sl_create_sketch_transform(ctx, "LaplacianRFT", N, 64, &T[9], 0.8))) return fail(11, rc);
        if ((rc = sl_create_sketch_transform(ctx, "MaternRFT", N, 64, &T[10], 1.5, 2.0))) return fail(12, rc);
        if ((rc = sl_create_sketch_transform(ctx, "GaussianQRFT", N, 64, &T[11], 1.2, 3))) return fail(13, rc);
        if ((rc = sl_create_sketch_transform(ctx, "LaplacianQRFT", N, 64, &T[12], 0.9, 0))) return fail(14, rc);
        if ((rc = sl_create_sketch_transform(ctx, "ExpSemigroupRLT", N, 64, &T[13], 0.7))) return fail(15, rc);
        if ((rc = sl_create_sketch_transform(ctx, "ExpSemigroupQRLT", N, 64, &T[14], 0.6, 2))) return fail(16, rc);
        if ((rc = sl_create_sketch_transform(ctx, "FastGaussianRFT", N, 700, &T[15], 1.3))) return fail(17, rc);
        if ((rc = sl_create_sketch_transform(ctx, "FastMaternRFT", N, 700, &T[16], 2.5, 1.1))) return fail(18, rc);
        if ((rc = sl_create_sketch_transform(ctx, "PPT", N, 64, &T[17], 3, 0.5, 0.7))) return fail(19, rc);
        const char* names[18] = {"JLT", "CT", "SJLT", "CWT", "MMT", "WZT", "FJLT", "UST", "GaussianRFT", "LaplacianRFT",
                                 "MaternRFT", "GaussianQRFT", "LaplacianQRFT", "ExpSemigroupRLT", "ExpSemigroupQRLT",
                                 "FastGaussianRFT", "FastMaternRFT", "PPT"};
        for (int t = 0; t < 18; ++t)
            if ((rc = apply_pair(T[t], names[t], t == 15 || t == 16 ? 700 : 64, 100 + 2 * t))) return rc;
        /* sparse input (CSC of A with ~30% of the entries kept), dense and sparse outputs */
        int ip[8], ind[N * 7]; double val[N * 7]; int nnz = 0;
        for (int j = 0; j < 7; ++j) { ip[j] = nnz; for (int i = 0; i < N; ++i) if (A[i + j * N] < 0.3) { ind[nnz] = i; val[nnz++] = A[i + j * N]; } }
        ip[7] = nnz;
        void* sA; sl_wrap_raw_sp_matrix(ip, ind, val, nnz, N, 7, &sA);
        double sj[64 * 7], sc[64 * 7];
        if ((rc = sl_apply_sketch_transform(T[0], "SparseMatrix", sA, "Matrix", W(sj, 64, 7), 0))) return fail(40, rc);
        if ((rc = sl_apply_sketch_transform(T[3], "SparseMatrix", sA, "Matrix", W(sc, 64, 7), 0))) return fail(41, rc);
        void* so; sl_wrap_raw_sp_matrix(NULL, NULL, NULL, 0, 0, 0, &so);
        if ((rc = sl_apply_sketch_transform(T[3], "SparseMatrix", sA, "SparseMatrix", so, 0))) return fail(42, rc);
        int onnz; sl_raw_sp_matrix_nnz(so, &onnz);
        int32_t oip[8]; int32_t* oind = malloc(4 * (onnz + 1)); double* oval = malloc(8 * (onnz + 1));
        sl_raw_sp_matrix_data(so, oip, oind, oval);
        dump("sp_JLT", sj, sizeof sj); dump("sp_CWT", sc, sizeof sc);
        dump("spo_ip", oip, sizeof oip); dump("spo_ind", oind, 4 * onnz); dump("spo_val", oval, 8 * onnz);
        /* a sketched dimension too long for the LDS row path (transposing fallback) */
        const int NL = 30000;
        sl_sketch_transform_t* TL;
        if ((rc = sl_create_sketch_transform(ctx, "CWT", NL, 50, &TL))) return fail(43, rc);
        double* AL = malloc(8 * (size_t)NL * 3); double sl[50 * 3];
        for (int i = 0; i < NL * 3; ++i) AL[i] = urand() - 0.5;
        if ((rc = sl_apply_sketch_transform(TL, "Matrix", W(AL, NL, 3), "Matrix", W(sl, 50, 3), 0))) return fail(44, rc);
        dump("L_A", AL, 8 * (size_t)NL * 3); dump("L_SA", sl, sizeof sl);
        /* ApproximateSVD: tall and wide host matrices with a decaying spectrum */
        const int m = 2000, n = 300, r = 10;
        double* M = malloc(8 * (size_t)m * n); double* Mt = malloc(8 * (size_t)m * n);
        double *u = malloc(8 * m * 12), *v = malloc(8 * n * 12);
        for (int i = 0; i < m * 12; ++i) u[i] = urand() - 0.5;
        for (int i = 0; i < n * 12; ++i) v[i] = urand() - 0.5;
        for (int j = 0; j < n; ++j) for (int i = 0; i < m; ++i) {
            double x = 1e-6 * (urand() - 0.5);
            for (int t = 0; t < 12; ++t) x += pow(0.6, t) * u[i + t * m] * v[j + t * n];
            M[i + (size_t)j * m] = x; Mt[j + (size_t)i * n] = x;
        }
        dump("svd_A", M, 8 * (size_t)m * n);
        double *U = malloc(8 * m * r), *Sv = malloc(8 * r), *V = malloc(8 * n * r);
        char prm[] = "{\"num_iterations\": 2, \"oversampling_ratio\": 2, \"sketch\": \"FJLT\"}";
        if ((rc = sl_approximate_svd("Matrix", W(M, m, n), "Matrix", W(U, m, r), "Matrix", W(Sv, r, 1), "Matrix", W(V, n, r), r, prm, ctx))) return fail(50, rc);
        dump("svd_U", U, 8 * m * r); dump("svd_S", Sv, 8 * r); dump("svd_V", V, 8 * n * r);
        char prm2[] = "{\"num_iterations\": 1, \"sketch\": \"JLT\"}";
        if ((rc = sl_approximate_svd("Matrix", W(Mt, n, m), "Matrix", W(V, n, r), "Matrix", W(Sv, r, 1), "Matrix", W(U, m, r), r, prm2, ctx))) return fail(51, rc);
        dump("svdw_U", V, 8 * n * r); dump("svdw_S", Sv, 8 * r); dump("svdw_V", U, 8 * m * r);
        /* ApproximateSymmetricSVD (lower triangle read) */
        const int ns = 400, rs = 8;
        double* Sy = calloc((size_t)ns * ns, 8);
        for (int j = 0; j < ns; ++j) for (int i = j; i < ns; ++i) {
            double x = 0;
            for (int t = 0; t < 12; ++t) x += (t % 2 ? -1.0 : 1.0) * pow(0.6, t) * u[i + t * m] * u[j + t * m];
            Sy[i + (size_t)j * ns] = x;   /* upper triangle left zero: only the lower one is read */
        }
        dump("sym_A", Sy, 8 * (size_t)ns * ns);
        double *Vs = malloc(8 * ns * rs), *Ss = malloc(8 * rs);
        char prm3[] = "{\"num_iterations\": 2}";
        if ((rc = sl_approximate_symmetric_svd("Matrix", W(Sy, ns, ns), "Matrix", W(Ss, rs, 1), "Matrix", W(Vs, ns, rs), rs, prm3, ctx))) return fail(52, rc);
        dump("sym_S", Ss, 8 * rs); dump("sym_V", Vs, 8 * ns * rs);
        /* FasterLeastSquares (Blendenpik) */
        const int lm = 3000, ln = 60;
        double *LA = malloc(8 * lm * ln), *Lb = malloc(8 * lm * 2), *Lx = malloc(8 * ln * 2);
        for (int i = 0; i < lm * ln; ++i) LA[i] = urand() - 0.5 + (i % (lm + 1) == 0 ? 3.0 : 0.0);
        for (int i = 0; i < lm * 2; ++i) Lb[i] = urand() - 0.5;
        dump("ls_A", LA, 8 * lm * ln); dump("ls_b", Lb, 8 * lm * 2);
        if ((rc = sl_faster_least_squares(0, "Matrix", W(LA, lm, ln), "Matrix", W(Lb, lm, 2), "Matrix", W(Lx, ln, 2), "", ctx))) return fail(53, rc);
        dump("ls_x", Lx, 8 * ln * 2);
        /* LIBSVM reader: dense and sparse, both directions */
        char fn[1024]; snprintf(fn, sizeof fn, "%s/d.libsvm", OUT);
        FILE* f = fopen(fn, "w"); fprintf(f, "1 1:0.5 3:2\n-1 2:1.5\n# comment\n2 4:-1 1:0.25\n"); fclose(f);
        double X1[4 * 3], Y1[3], X2[3 * 5], X0[3 * 4], Y0[3];
        if ((rc = sl_readlibsvm(fn, "Matrix", W(X1, 4, 3), "Matrix", W(Y1, 1, 3), 1, 0, -1))) return fail(60, rc);
        if ((rc = sl_readlibsvm(fn, "Matrix", W(X2, 3, 5), NULL, NULL, 2, 5, -1))) return fail(61, rc);
        /* direction 0 is not SL_COLUMNS: rows, as the reference's cio.cpp maps it */
        if ((rc = sl_readlibsvm(fn, "Matrix", W(X0, 3, 4), "Matrix", W(Y0, 3, 1), 0, 0, -1))) return fail(63, rc);
        dump("lib_X0", X0, sizeof X0); dump("lib_Y0", Y0, sizeof Y0);
        void* xs; sl_wrap_raw_sp_matrix(NULL, NULL, NULL, 0, 0, 0, &xs);
        if ((rc = sl_readlibsvm(fn, "SparseMatrix", xs, "Matrix", W(Y1, 1, 3), 1, 0, -1))) return fail(62, rc);
        int xnnz; sl_raw_sp_matrix_nnz(xs, &xnnz);
        int32_t xip[4], xind[16]; double xval[16];
        sl_raw_sp_matrix_data(xs, xip, xind, xval);
        dump("lib_X1", X1, sizeof X1); dump("lib_Y1", Y1, sizeof Y1); dump("lib_X2", X2, sizeof X2);
        dump("lib_sip", xip, sizeof xip); dump("lib_sind", xind, 4 * xnnz); dump("lib_sval", xval, 8 * xnnz);
        /* kernel Grams on host Matrix operands (reference capi/ckernel.cpp):
           A (300 x 7): 7 points as columns; B (9 x 300): 9 points as rows */
        sl_kernel_t *kg, *kl, *kp;
        if ((rc = sl_create_kernel("gaussian", N, &kg, 0.9))) return fail(70, rc);
        if ((rc = sl_create_kernel("laplacian", N, &kl, 1.7))) return fail(71, rc);
        if ((rc = sl_create_kernel("polynomial", N, &kp, 2, 1.0, 0.01))) return fail(72, rc);
        double *Kg = malloc(8 * 9 * 7), *Kl = malloc(8 * 7 * 9), *Kp = malloc(8 * 9 * 9);
        if ((rc = sl_kernel_gram(2, 1, kg, "Matrix", W(B, 9, N), "Matrix", W(A, N, 7), "Matrix", W(Kg, 9, 7)))) return fail(73, rc);
        if ((rc = sl_kernel_gram(1, 2, kl, "Matrix", W(A, N, 7), "Matrix", W(B, 9, N), "Matrix", W(Kl, 7, 9)))) return fail(74, rc);
        if ((rc = sl_kernel_gram(2, 2, kp, "Matrix", W(B, 9, N), "Matrix", W(B, 9, N), "Matrix", W(Kp, 9, 9)))) return fail(75, rc);
        /* direction 0 is not SL_COLUMNS: rows (reference ckernel.cpp maps only 1 to columns) */
        double* Kg0 = malloc(8 * 9 * 7);
        if ((rc = sl_kernel_gram(0, 1, kg, "Matrix", W(B, 9, N), "Matrix", W(A, N, 7), "Matrix", W(Kg0, 9, 7)))) return fail(76, rc);
        dump("kg", Kg, 8 * 9 * 7); dump("kl", Kl, 8 * 7 * 9); dump("kp", Kp, 8 * 9 * 9); dump("kg0", Kg0, 8 * 9 * 7);
        sl_free_kernel(kg); sl_free_kernel(kl); sl_free_kernel(kp);
        printf("%d\n", sl_runtime_started());
        for (int t = 0; t < 18; ++t) sl_free_sketch_transform(T[t]);
        sl_free_sketch_transform(TL); sl_free_context(ctx);
        return 0;
    }
""")


@pytest.mark.gpu
def test_host_operands_on_device_interpreter_free(capi, tmp_path):
    """A C program drives every sketch type, sparse inputs / outputs, the
    three NLA entry points and the LIBSVM reader on host "Matrix" /
    "SparseMatrix" operands: staged to the GPU, never starting the embedded
    runtime, and equal to the runtime's results on the same context (VERDICT
    r3 item 5; reference capi/csketch.cpp, capi/cnla.cpp, capi/cio.cpp)."""
    import sysconfig
    src = tmp_path / "hd.c"
    src.write_text(C_HOST_DEVICE_PROGRAM)
    exe = tmp_path / "hd"
    libdir = os.path.dirname(B.CAPI_LIB)
    r = subprocess.run(["gcc", str(src), "-o", str(exe), f"-L{libdir}", "-lskylark_capi", f"-Wl,-rpath,{libdir}",
                        f"-Wl,-rpath,{sysconfig.get_config_var('LIBDIR')}", "-lm"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().split("\n")[-1] == "0"      # the runtime never started

    def ld(name, shape, dt=np.float64):
        return np.fromfile(tmp_path / f"{name}.bin", dtype=dt).reshape(shape, order="F")

    A = ld("A", (300, 7))
    Bm = ld("B", (9, 300))
    ctx = sk.Context(41)
    specs = [("JLT", []), ("CT", [2.0]), ("SJLT", []), ("CWT", []), ("MMT", []), ("WZT", [1.5]), ("FJLT", []),
             ("UST", []), ("GaussianRFT", [1.5]), ("LaplacianRFT", [0.8]), ("MaternRFT", [1.5, 2.0]),
             ("GaussianQRFT", [1.2, 3]), ("LaplacianQRFT", [0.9, 0]), ("ExpSemigroupRLT", [0.7]),
             ("ExpSemigroupQRLT", [0.6, 2]), ("FastGaussianRFT", [1.3]), ("FastMaternRFT", [2.5, 1.1]),
             ("PPT", [3, 0.5, 0.7])]
    Ts = {}
    for typ, prm in specs:
        S = 700 if typ.startswith("Fast") else 64
        T = _pysketch(typ, 300, S, prm, ctx)
        Ts[typ] = T
        for tag, X, dim, shape in (("c", A, 0, (S, 7)), ("r", Bm, 1, (9, S))):
            ref = T.apply(torch.from_numpy(X.copy()), dim=dim)
            ref = (ref.to_dense() if ref.layout != torch.strided else ref).double().numpy()
            np.testing.assert_allclose(ld(f"{typ}_{tag}", shape), ref, rtol=1e-8, atol=1e-9, err_msg=f"{typ} {tag}")
    As = np.where(A < 0.3, A, 0.0)
    np.testing.assert_allclose(ld("sp_JLT", (64, 7)), Ts["JLT"].apply(torch.from_numpy(As)).numpy(), rtol=1e-9, atol=1e-10)
    refc = Ts["CWT"].apply(torch.from_numpy(As)).numpy()
    np.testing.assert_allclose(ld("sp_CWT", (64, 7)), refc, rtol=1e-9, atol=1e-10)
    import scipy.sparse as sp
    oip = np.fromfile(tmp_path / "spo_ip.bin", dtype=np.int32)
    got = sp.csc_matrix((np.fromfile(tmp_path / "spo_val.bin"), np.fromfile(tmp_path / "spo_ind.bin", dtype=np.int32),
                         oip), shape=(64, 7)).toarray()
    np.testing.assert_allclose(got, refc, rtol=1e-9, atol=1e-10)
    TL = sk.sketch.CWT(30000, 50, context=ctx)
    np.testing.assert_allclose(ld("L_SA", (50, 3)), TL.apply(torch.from_numpy(ld("L_A", (30000, 3)))).numpy(),
                               rtol=1e-9, atol=1e-9)
    # NLA: the same device engine from the runtime (f64 operand on the GPU)
    M = ld("svd_A", (2000, 300))
    p = sk.nla.ApproximateSVDParams(num_iterations=2, sketch="FJLT")
    U, s, V = sk.nla.approximate_svd(torch.from_numpy(M).cuda(), 10, ctx, p)
    np.testing.assert_allclose(ld("svd_S", (10,)), s.cpu().numpy(), rtol=1e-10)

    def same_pairs(Uc, Vc, Ur, Vr):
        # singular pairs up to one sign per pair (the C program may solve the
        # transposed problem, whose eigenvector signs are its own)
        sg = np.sign(np.sum(Uc * Ur, axis=0))
        np.testing.assert_allclose(Uc * sg, Ur, atol=1e-8)
        np.testing.assert_allclose(Vc * sg, Vr, atol=1e-8)

    same_pairs(ld("svd_U", (2000, 10)), ld("svd_V", (300, 10)), U.cpu().numpy(), V.cpu().numpy())
    p2 = sk.nla.ApproximateSVDParams(num_iterations=1, sketch="JLT")
    U2, s2, V2 = sk.nla.approximate_svd(torch.from_numpy(M.T.copy()).cuda(), 10, ctx, p2)
    np.testing.assert_allclose(ld("svdw_S", (10,)), s2.cpu().numpy(), rtol=1e-10)
    same_pairs(ld("svdw_U", (300, 10)), ld("svdw_V", (2000, 10)), U2.cpu().numpy(), V2.cpu().numpy())
    Sy = ld("sym_A", (400, 400))
    Vr, sr = sk.nla.approximate_symmetric_svd(torch.from_numpy(Sy), 8, ctx, sk.nla.ApproximateSVDParams(num_iterations=2))
    np.testing.assert_allclose(ld("sym_S", (8,)), sr.numpy(), rtol=1e-9, atol=1e-12)
    Vc = ld("sym_V", (400, 8))
    # the rank-12 indefinite matrix has 6 positive eigenvalues: the top 8 by
    # signed value end in its null space, where any orthonormal pair is right;
    # the well-determined columns span the same subspace
    good = int((np.abs(sr.numpy()) > 1e-8 * abs(float(sr[0]))).sum())
    Vg, Vrg = Vc[:, :good], Vr.numpy()[:, :good]
    np.testing.assert_allclose(Vg @ Vg.T, Vrg @ Vrg.T, atol=1e-8)
    LA, Lb = ld("ls_A", (3000, 60)), ld("ls_b", (3000, 2))
    X = np.linalg.lstsq(LA, Lb, rcond=None)[0]
    np.testing.assert_allclose(ld("ls_x", (60, 2)), X, rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(ld("lib_X1", (4, 3)), [[0.5, 0, 0.25], [0, 1.5, 0], [2, 0, 0], [0, 0, -1]])
    np.testing.assert_allclose(ld("lib_Y1", (1, 3)), [[1, -1, 2]])
    np.testing.assert_allclose(ld("lib_X2", (3, 5)), [[0.5, 0, 2, 0, 0], [0, 1.5, 0, 0, 0], [0.25, 0, 0, -1, 0]])
    np.testing.assert_allclose(ld("lib_X0", (3, 4)), ld("lib_X1", (4, 3)).T)   # direction 0 = rows
    np.testing.assert_allclose(ld("lib_Y0", (3, 1)), [[1], [-1], [2]])
    sip = np.fromfile(tmp_path / "lib_sip.bin", dtype=np.int32)
    Xs = sp.csc_matrix((np.fromfile(tmp_path / "lib_sval.bin"), np.fromfile(tmp_path / "lib_sind.bin", dtype=np.int32),
                        sip), shape=(4, 3)).toarray()
    np.testing.assert_allclose(Xs, ld("lib_X1", (4, 3)))
    # kernel Grams on host matrices (native): against the runtime's kernels
    Xp = torch.from_numpy(A.copy())            # 300 x 7: the 7 points as columns of A^T
    Bp = torch.from_numpy(Bm.copy())           # 9 x 300: 9 points as rows
    kg = sk.ml.Gaussian(300, sigma=0.9)
    kl = sk.ml.Laplacian(300, sigma=1.7)
    kp = sk.ml.Polynomial(300, q=2, c=1.0, gamma=0.01)
    np.testing.assert_array_equal(ld("kg0", (9, 7)), ld("kg", (9, 7)))
    np.testing.assert_allclose(ld("kg", (9, 7)), kg.gram(Bp, dirX="rows", dirY="columns", Y=Xp).numpy(),
                               rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(ld("kl", (7, 9)), kl.gram(Xp, dirX="columns", dirY="rows", Y=Bp).numpy(),
                               rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(ld("kp", (9, 9)), kp.gram(Bp, dirX="rows", dirY="rows", Y=Bp).numpy(),
                               rtol=1e-9, atol=1e-12)


def test_dist_matrix_types_shapes_and_errors(capi):
    """DistMatrix-typed operands in the C ABI (host-side checks, no device
    work): the shard geometry of every native layout matches the runtime's
    DistMatrix (parallel/distmatrix.py balanced blocks) on a 3-rank callback
    communicator; the 2-D [MC,MR] type is refused (103) and a mix of
    distributed and local types is an error (109) before any device call."""
    from libskylark_amd.parallel.distmatrix import DistMatrix
    from libskylark_amd.parallel.comm import Comm
    i64, vp = C.c_int64, C.c_void_p
    capi.sl_dist_local_shape.argtypes = [C.c_char_p, i64, i64, vp] + [C.POINTER(i64)] * 4

    def shape(typ, m, n, comm):
        v = [i64() for _ in range(4)]
        rc = capi.sl_dist_local_shape(typ, m, n, comm, *[C.byref(x) for x in v])
        return rc, [x.value for x in v]

    assert shape(b"DistMatrix_VC_STAR", 10, 4, None) == (0, [0, 0, 10, 4])
    assert shape(b"DistMatrix", 10, 4, None)[0] == 103
    assert shape(b"Matrix", 10, 4, None)[0] == 109

    @C.CFUNCTYPE(C.c_int, vp, vp, i64, C.c_int, C.c_int, vp, vp)
    def never(send, recv, count, dtype, op, stream, user):
        return 1

    class _FakeComm:   # the runtime's geometry for rank r of 3
        def __init__(self, r):
            self.rank, self.size = r, 3

    capi.sl_device_comm_from_allreduce.argtypes = [C.c_int, C.c_int, vp, vp, C.POINTER(vp)]
    for r in range(3):
        comm = vp()
        rc = capi.sl_device_comm_from_allreduce(r, 3, C.cast(never, vp), None, C.byref(comm))
        if rc == 106:
            pytest.skip("native HIP library not loadable here")
        assert rc == 0
        for typ, layout in ((b"DistMatrix_VC_STAR", "VC_STAR"), (b"DistMatrix_VR_STAR", "VR_STAR"),
                            (b"DistMatrix_STAR_VC", "STAR_VC"), (b"DistMatrix_STAR_VR", "STAR_VR"),
                            (b"SharedMatrix", "STAR_STAR"), (b"RootMatrix", "CIRC_CIRC")):
            d = DistMatrix(torch.empty(0), (10, 7), layout, comm=_FakeComm(r))
            rb, cb = d.row_blocks(), d.col_blocks()
            want = [rb[0][0] if rb else 0, cb[0][0] if cb else 0, *d.local_shape()]
            rc, got = shape(typ, 10, 7, comm)
            assert rc == 0 and got == want, (typ, r, got, want)
    # type checks come before any device work
    ctx, h, a = vp(), vp(), vp()
    assert capi.sl_create_default_context(3, C.byref(ctx)) == 0
    assert capi.sl_create_sketch_transform(ctx, b"JLT", 10, 4, C.byref(h)) == 0
    capi.sl_wrap_raw_dist_device_matrix.argtypes = [vp, C.c_int, i64, i64, i64, vp, C.POINTER(vp)]
    assert capi.sl_wrap_raw_dist_device_matrix(None, 1, 10, 3, 3, None, C.byref(a)) == 0
    assert capi.sl_apply_sketch_transform(h, b"DistMatrix", a, b"SharedMatrix", a, 0) == 103
    assert capi.sl_apply_sketch_transform(h, b"DistMatrix_VC_STAR", a, b"Matrix", a, 0) == 109
    capi.sl_free_raw_dist_device_matrix_wrap(a)
    capi.sl_free_sketch_transform(h)
    capi.sl_free_context(ctx)


def test_dist_matrix_entry_points_refuse_before_device_work(capi):
    """Every DistMatrix-aware entry point checks its type strings first: the
    2-D [MC,MR] "DistMatrix" is refused with 103 and a mix of distributed and
    local operands with 109, before any device call (so these hold on a host
    without a GPU)."""
    vp, i64 = C.c_void_p, C.c_int64
    capi.sl_wrap_raw_dist_device_matrix.argtypes = [vp, C.c_int, i64, i64, i64, vp, C.POINTER(vp)]
    d = vp()
    assert capi.sl_wrap_raw_dist_device_matrix(None, 1, 10, 3, 3, None, C.byref(d)) == 0
    ctx = vp()
    assert capi.sl_create_default_context(5, C.byref(ctx)) == 0
    prm = b'{"num_iterations": 1}'
    capi.sl_approximate_svd.argtypes = [C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp, C.c_uint16,
                                        C.c_char_p, vp]
    capi.sl_approximate_symmetric_svd.argtypes = [C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp, C.c_uint16,
                                                  C.c_char_p, vp]
    capi.sl_faster_least_squares.argtypes = [C.c_int, C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp]
    capi.sl_readlibsvm.argtypes = [C.c_char_p, C.c_char_p, vp, C.c_char_p, vp, C.c_int, C.c_int, C.c_int]
    capi.sl_kernel_gram.argtypes = [C.c_int, C.c_int, vp, C.c_char_p, vp, C.c_char_p, vp, C.c_char_p, vp]
    for a_t, b_t, want in ((b"DistMatrix", b"DistMatrix", 103), (b"DistMatrix_VC_STAR", b"Matrix", 109)):
        assert capi.sl_approximate_svd(a_t, d, b_t, d, b"SharedMatrix", d, b"SharedMatrix", d, 2, prm, ctx) == want
        assert capi.sl_approximate_symmetric_svd(a_t, d, b"SharedMatrix", d, b_t, d, 2, prm, ctx) == want
        assert capi.sl_faster_least_squares(0, a_t, d, b_t, d, b"SharedMatrix", d, b"{}", ctx) == want
        assert capi.sl_readlibsvm(b"/nonexistent", a_t, d, b_t, d, 2, 0, -1) == want
        k = vp()
        assert capi.sl_create_kernel(b"gaussian", 3, C.byref(k), C.c_double(1.0)) == 0
        assert capi.sl_kernel_gram(2, 1, k, a_t, d, b_t, d, b"SharedMatrix", d) == want
        capi.sl_free_kernel(k)
    # layouts the paths do not take: a column-distributed A for randSVD / least squares
    assert capi.sl_approximate_svd(b"DistMatrix_STAR_VC", d, b"DistMatrix_STAR_VC", d, b"SharedMatrix", d,
                                   b"SharedMatrix", d, 2, prm, ctx) == 103
    assert capi.sl_faster_least_squares(1, b"DistMatrix_VC_STAR", d, b"DistMatrix_VC_STAR", d, b"SharedMatrix", d,
                                        b"{}", ctx) == 103
    capi.sl_free_raw_dist_device_matrix_wrap(d)
    capi.sl_free_context(ctx)
