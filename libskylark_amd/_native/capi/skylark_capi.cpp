// C API of the framework: the reference's sl_* ABI (capi/basec.hpp,
// sketchc.hpp, nlac.hpp, kernelc.hpp, ioc.hpp) over the MI355X runtime.
//
// Native paths (no interpreter):
//  - contexts, kernel objects and EVERY sketch type of the reference (all
//    19): creation and JSON (de)serialisation in C++ (native_sketch.hpp, the
//    same counter-based streams as the runtime), application on host
//    "Matrix" / "SparseMatrix" operands (staged to the GPU, or on host
//    threads when there is none) and on "DeviceMatrix" operands;
//  - sl_approximate_svd / sl_approximate_symmetric_svd /
//    sl_faster_least_squares on "Matrix" and "DeviceMatrix" operands (the C++
//    randSVD engines of libskylark_hip.so);
//  - sl_kernel_gram on "Matrix" and "DeviceMatrix" operands (the Gram
//    kernels of libskylark_hip.so, host matrices staged to the GPU);
//  - sl_readlibsvm into "Matrix" / "SparseMatrix" (libsvm_io.cpp).
//  - DistMatrix-typed operands (device shards over a device communicator:
//    DistMatrix_VC_STAR / _VR_STAR, DistMatrix_STAR_VC / _STAR_VR,
//    SharedMatrix, RootMatrix; sl_wrap_raw_dist_device_matrix) in
//    sl_apply_sketch_transform (every sketch type: the ranks' column ranges
//    of the operator summed by all-reduce), sl_approximate_svd ([VC,*] A),
//    sl_approximate_symmetric_svd ([VC,*] A), sl_faster_least_squares
//    ([VC,*] A and B), sl_kernel_gram (points split over the ranks) and
//    sl_readlibsvm (each rank's examples) -- no interpreter.  The
//    2-D [MC,MR] "DistMatrix" has no native path.
// Everything else (runtime-only kernels, the remaining entry points) goes
// through the Python/HIP runtime
// (libskylark_amd + libskylark_hip.so); a natively created sketch or context
// is handed to it lazily (via its JSON / seed + counter), so the two paths
// see the same objects and the same random streams (sl_runtime_started()
// reports whether it ever started).  This library embeds CPython when such a
// call comes from a plain C/C++ program (first call initialises the
// interpreter, adds this library's package root to sys.path, and imports
// libskylark_amd.capi), or joins the running interpreter when loaded from
// Python.  Every runtime entry point:
//   - takes the GIL (PyGILState_Ensure),
//   - converts handles / raw matrix wraps / varargs to Python objects,
//   - calls libskylark_amd.capi.<fn>,
//   - maps a Python exception to the reference's integer error code and
//     keeps the formatted traceback for sl_get_exception_info().
#include <Python.h>
#include <dlfcn.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include <algorithm>

#include "native_sketch.hpp"
#include "native_device.hpp"

#define SL_CAPI extern "C" __attribute__((visibility("default")))

// seed + counter are the context's state; obj (the runtime's Context) is
// created on first use by a Python-path call and kept in sync around it
struct sl_context_t {
  PyObject* obj;
  uint64_t seed;
  uint64_t counter;
  void* dcomm;   // NativeComm (RCCL) of the DeviceMatrix paths, or null
};
struct sl_sketch_transform_t {
  PyObject* obj;          // runtime object (created lazily for native sketches)
  slnat::Sketch* nat;     // native operator, or null
};
struct sl_kernel_t {
  PyObject* obj;          // runtime object (created lazily for natively known kernels)
  sldev::Kern nat;        // native parameters (type K_NONE: runtime-only kernel)
  std::string type;
};
struct sl_raw_device_matrix_t {
  sldev::DevMat d;
};
// a DistMatrix-typed operand: this rank's device shard of a global matrix
// (the layout comes with the type string at each call, as in the reference)
struct sl_raw_dist_device_matrix_t {
  sldev::DistMat d;
};
struct sl_raw_matrix_t {
  double* data;
  int m, n;
};
struct sl_raw_sp_matrix_t {
  int* indptr;
  int* ind;
  double* data;
  int nnz, m, n;
  PyObject* out;  // library-owned result (capi.SparseOut) when a runtime call produced it
  // library-owned result of a native call (CSC), read back by sl_raw_sp_matrix_*
  bool nat = false, nat_updated = false;
  int nat_m = 0, nat_n = 0;
  std::vector<int> nat_indptr, nat_ind;
  std::vector<double> nat_val;
};

namespace {

std::once_flag g_init;
PyObject* g_mod = nullptr;
std::string g_last_error;
std::string g_supported;

void init_python() {
  if (!Py_IsInitialized()) {
    Py_InitializeEx(0);
    // hand the GIL back; every entry point re-acquires it
    PyEval_SaveThread();
  }
  PyGILState_STATE st = PyGILState_Ensure();
  Dl_info info;
  if (dladdr((void*)&init_python, &info) && info.dli_fname) {
    // <root>/libskylark_amd/_native/libskylark_capi.so -> <root>
    std::string p(info.dli_fname);
    for (int i = 0; i < 3; ++i) {
      auto k = p.find_last_of('/');
      if (k == std::string::npos) break;
      p = p.substr(0, k);
    }
    PyObject* sys_path = PySys_GetObject("path");
    PyObject* s = PyUnicode_FromString(p.c_str());
    if (sys_path && s && !PySequence_Contains(sys_path, s)) PyList_Append(sys_path, s);
    Py_XDECREF(s);
  }
  g_mod = PyImport_ImportModule("libskylark_amd.capi");
  if (!g_mod) {
    PyErr_Print();
  }
  PyGILState_Release(st);
}

struct Gil {
  PyGILState_STATE st;
  Gil() {
    std::call_once(g_init, init_python);
    st = PyGILState_Ensure();
  }
  ~Gil() { PyGILState_Release(st); }
};

// Convert the pending Python exception to an error code (and keep the text).
int fail() {
  PyObject *t, *v, *tb;
  PyErr_Fetch(&t, &v, &tb);
  PyErr_NormalizeException(&t, &v, &tb);
  int code = 100;
  g_last_error = "unknown error";
  if (v) {
    PyObject* tbm = PyImport_ImportModule("traceback");
    if (tbm) {
      PyObject* lines = PyObject_CallMethod(tbm, "format_exception", "OOO", t ? t : Py_None, v, tb ? tb : Py_None);
      if (lines) {
        PyObject* sep = PyUnicode_FromString("");
        PyObject* joined = PyUnicode_Join(sep, lines);
        if (joined) g_last_error = PyUnicode_AsUTF8(joined);
        Py_XDECREF(joined);
        Py_XDECREF(sep);
        Py_DECREF(lines);
      }
      Py_DECREF(tbm);
    }
    if (g_mod) {
      PyObject* c = PyObject_CallMethod(g_mod, "error_code", "O", v);
      if (c) {
        code = (int)PyLong_AsLong(c);
        Py_DECREF(c);
      }
    }
  }
  PyErr_Clear();
  Py_XDECREF(t);
  Py_XDECREF(v);
  Py_XDECREF(tb);
  return code;
}

PyObject* call(const char* fn, PyObject* args) {
  if (!g_mod) {
    PyErr_SetString(PyExc_RuntimeError, "libskylark_amd.capi could not be imported");
    Py_XDECREF(args);
    return nullptr;
  }
  PyObject* f = PyObject_GetAttrString(g_mod, fn);
  if (!f) {
    Py_XDECREF(args);
    return nullptr;
  }
  PyObject* r = PyObject_CallObject(f, args);
  Py_DECREF(f);
  Py_XDECREF(args);
  return r;
}

// runtime Context for a C context, its counter set from the native state
PyObject* py_ctx(sl_context_t* c) {
  if (!c->obj) {
    c->obj = call("create_context", Py_BuildValue("(K)", (unsigned long long)c->seed));
    if (!c->obj) return nullptr;
  }
  PyObject* v = PyLong_FromUnsignedLongLong(c->counter);
  PyObject_SetAttrString(c->obj, "counter", v);
  Py_XDECREF(v);
  return c->obj;
}

// after a runtime call: the runtime may have advanced the counter
void ctx_sync_back(sl_context_t* c) {
  if (!c->obj) return;
  PyObject *t, *v0, *tb;
  PyErr_Fetch(&t, &v0, &tb);      // keep a pending error for fail()
  PyObject* v = PyObject_GetAttrString(c->obj, "counter");
  if (v) {
    c->counter = PyLong_AsUnsignedLongLong(v);
    Py_DECREF(v);
  }
  PyErr_Clear();
  PyErr_Restore(t, v0, tb);
}

// runtime object of a sketch (a native one is rebuilt from its JSON)
PyObject* py_sketch(sl_sketch_transform_t* S) {
  if (!S->obj && S->nat) S->obj = call("deserialize_sketch", Py_BuildValue("(s)", slnat::to_json(*S->nat).c_str()));
  return S->obj;
}

bool is_device(const char* type) { return !strcmp(type, "DeviceMatrix"); }

// layout of a DistMatrix type name (reference capi/matrix_types.cpp); -1: not
// a distributed type; -2: the 2-D [MC,MR] "DistMatrix", which has no native
// path (redistribute to [VC,*] / [*,VC] first)
int dist_layout(const char* type) {
  if (!strcmp(type, "DistMatrix_VC_STAR") || !strcmp(type, "DistMatrix_VR_STAR")) return sldev::LY_ROWS;
  if (!strcmp(type, "DistMatrix_STAR_VC") || !strcmp(type, "DistMatrix_STAR_VR")) return sldev::LY_COLS;
  if (!strcmp(type, "SharedMatrix")) return sldev::LY_STAR;
  if (!strcmp(type, "RootMatrix")) return sldev::LY_ROOT;
  if (!strcmp(type, "DistMatrix")) return -2;
  return -1;
}

const sldev::DistMat& distmat(void* A) { return ((sl_raw_dist_device_matrix_t*)A)->d; }

// shard of a distributed operand as a local DeviceMatrix view
sldev::DevMat dist_local(int ly, const sldev::DistMat& d, int rank, int size) {
  int64_t r0, c0, lm, ln;
  sldev::shard_of(ly, d.m, d.n, rank, size, &r0, &c0, &lm, &ln);
  return sldev::DevMat{d.data, d.dtype, lm, ln, d.ld};
}

// both types distributed (or both not); sets the layouts; error text on a mix
int dist_pair(const char* fn, const char* a, const char* b, int* la, int* lb) {
  *la = dist_layout(a);
  *lb = dist_layout(b);
  if (*la == -1 && *lb == -1) return 0;
  if (*la == -2 || *lb == -2) {
    g_last_error = std::string(fn) + ": 2-D [MC,MR] DistMatrix operands have no native path; use DistMatrix_VC_STAR / "
                   "DistMatrix_STAR_VC (or the Python runtime's redistribute)";
    return 103;
  }
  if (*la < 0 || *lb < 0) {
    g_last_error = std::string(fn) + ": mix of distributed and local operand types";
    return 109;
  }
  return 0;
}

sldev::DevMat& devmat(void* A) { return ((sl_raw_device_matrix_t*)A)->d; }

int native_fail(int code) {
  g_last_error = sldev::error();
  return code;
}

PyObject* dense_desc(void* A) {
  auto* M = (sl_raw_matrix_t*)A;
  return Py_BuildValue("(Kii)", (unsigned long long)(uintptr_t)M->data, M->m, M->n);
}

PyObject* sparse_in_desc(void* A) {
  auto* M = (sl_raw_sp_matrix_t*)A;
  return Py_BuildValue("(KKKiii)", (unsigned long long)(uintptr_t)M->indptr,
                       (unsigned long long)(uintptr_t)M->ind, (unsigned long long)(uintptr_t)M->data, M->nnz, M->m,
                       M->n);
}

PyObject* in_desc(const char* type, void* A) {
  if (!strcmp(type, "Matrix")) return dense_desc(A);
  if (!strcmp(type, "SparseMatrix")) return sparse_in_desc(A);
  PyErr_Format(PyExc_ValueError, "unsupported matrix type %s (host C API takes Matrix / SparseMatrix)", type);
  return nullptr;
}

PyObject* out_desc(const char* type, void* A) {
  if (!strcmp(type, "Matrix")) return dense_desc(A);
  if (!strcmp(type, "SparseMatrix")) {
    auto* M = (sl_raw_sp_matrix_t*)A;
    if (!M->out) {
      M->out = call("SparseOut", PyTuple_New(0));
      if (!M->out) return nullptr;
    }
    Py_INCREF(M->out);
    return M->out;
  }
  PyErr_Format(PyExc_ValueError, "unsupported output matrix type %s", type);
  return nullptr;
}

// Build a tuple of varargs from a spec string ('d' double, 'i' int).
PyObject* varargs_tuple(const std::string& spec, va_list ap) {
  PyObject* t = PyTuple_New((Py_ssize_t)spec.size());
  for (size_t i = 0; i < spec.size(); ++i) {
    PyObject* o = spec[i] == 'i' ? PyLong_FromLong(va_arg(ap, int)) : PyFloat_FromDouble(va_arg(ap, double));
    PyTuple_SET_ITEM(t, (Py_ssize_t)i, o);
  }
  return t;
}

std::string spec_of(const char* fn, const char* type) {
  PyObject* r = call(fn, Py_BuildValue("(s)", type));
  std::string s;
  if (r) {
    s = PyUnicode_AsUTF8(r);
    Py_DECREF(r);
  } else {
    PyErr_Clear();
  }
  return s;
}

}  // namespace

// ------------------------------------------------------------------- base
SL_CAPI const char* sl_strerror(const int code) {
  switch (code) {
    case 0: return "No error";
    case 100: return "Skylark failure";
    case 101: return "Failed to allocate memory";
    case 102: return "Unsupported matrix distribution";
    case 103: return "Unsupported operation";
    case 104: return "Dimension mismatch";
    case 105: return "CombBLAS failure";
    case 106: return "Native (HIP) library failure";
    case 107: return "IO failure";
    case 108: return "NLA failure";
    case 109: return "Invalid parameters";
    case 110: return "Unsupported base operation";
    case 111: return "Unknown transform type";
    default: return "Unknown error code";
  }
}

SL_CAPI bool sl_has_elemental() { return false; }
SL_CAPI bool sl_has_combblas() { return false; }

SL_CAPI char* sl_supported_sketch_transforms() {
  Gil g;
  PyObject* r = call("supported_sketch_transforms", PyTuple_New(0));
  if (!r) {
    fail();
    return nullptr;
  }
  g_supported = PyUnicode_AsUTF8(r);
  Py_DECREF(r);
  return (char*)g_supported.c_str();
}

SL_CAPI void sl_get_exception_info(char** info) { *info = strdup(g_last_error.c_str()); }
SL_CAPI void sl_print_exception_trace() { fprintf(stderr, "%s\n", g_last_error.c_str()); }

SL_CAPI int sl_create_default_context(int seed, sl_context_t** ctxt) {
  *ctxt = new sl_context_t{nullptr, (uint64_t)(int64_t)seed, 0, nullptr};
  return 0;
}

// comm: null, or a device communicator from sl_device_comm_create (RCCL over
// xGMI); the DeviceMatrix randSVD of a context with a communicator is the
// distributed call over the ranks' row shards.  (The runtime paths use
// torch.distributed's world, set up by the launcher.)
SL_CAPI int sl_create_context(int seed, void* comm, sl_context_t** ctxt) {
  const int rc = sl_create_default_context(seed, ctxt);
  if (rc == 0) (*ctxt)->dcomm = comm;
  return rc;
}

// ----------------------------------------------------- device communicator
// RCCL communicator of the C ABI's distributed device paths (NativeComm):
// rank 0 gets an id, the caller ships it to every rank (MPI, a file, ...),
// every rank creates its communicator with it (collective).
SL_CAPI int sl_device_comm_id_bytes() {
  auto& L = sldev::lib();
  return L.loaded ? L.comm_id_bytes() : -1;
}

SL_CAPI int sl_device_comm_unique_id(void* out) {
  auto& L = sldev::lib();
  if (!L.loaded) { g_last_error = L.err; return 106; }
  if (L.comm_unique_id(out)) { g_last_error = L.last_error(); return 106; }
  return 0;
}

SL_CAPI int sl_device_comm_create(const void* id, int nranks, int rank, void** comm) {
  auto& L = sldev::lib();
  if (!L.loaded) { g_last_error = L.err; return 106; }
  if (L.comm_init(id, nranks, rank, comm)) { g_last_error = L.last_error(); return 106; }
  return 0;
}

SL_CAPI int sl_device_comm_free(void* comm) {
  auto& L = sldev::lib();
  if (!L.loaded || !comm) return 0;
  return L.comm_destroy(comm) ? 106 : 0;
}

// HIP device of the calling thread (one process per GPU)
SL_CAPI int sl_device_set(int dev) {
  auto& L = sldev::lib();
  if (!L.loaded) { g_last_error = L.err; return 106; }
  if (L.set_device(dev)) { g_last_error = L.last_error(); return 106; }
  return 0;
}

SL_CAPI int sl_free_context(sl_context_t* ctxt) {
  if (!ctxt) return 0;
  if (ctxt->obj) {
    Gil g;
    Py_XDECREF(ctxt->obj);
  }
  delete ctxt;
  return 0;
}

// 1 once a call has needed the embedded runtime (tests: the native path stays interpreter-free)
SL_CAPI int sl_runtime_started() { return Py_IsInitialized() && g_mod ? 1 : 0; }

SL_CAPI int sl_wrap_raw_matrix(double* data, int m, int n, void** A) {
  *A = new sl_raw_matrix_t{data, m, n};
  return 0;
}

SL_CAPI int sl_free_raw_matrix_wrap(void* A) {
  delete (sl_raw_matrix_t*)A;
  return 0;
}

// A GPU buffer as a "DeviceMatrix": row-major m x n, leading dimension ld
// (elements), dtype 0 f32 / 1 f64 / 2 bf16.  The caller owns the memory.
SL_CAPI int sl_wrap_raw_device_matrix(void* data, int dtype, int m, int n, int64_t ld, void** A) {
  if (dtype < 0 || dtype > 2 || m < 0 || n < 0 || ld < n) return 109;
  *A = new sl_raw_device_matrix_t{sldev::DevMat{data, dtype, m, n, ld}};
  return 0;
}

SL_CAPI int sl_free_raw_device_matrix_wrap(void* A) {
  delete (sl_raw_device_matrix_t*)A;
  return 0;
}

// DistMatrix-typed operand: local = this rank's shard (device, row-major, ld)
// of the global m x n matrix; comm = the device communicator the matrix lives
// on (sl_device_comm_create, a caller's all-reduce through
// sl_device_comm_from_allreduce, or null for one rank).  Pass the wrap with
// the reference's type names: DistMatrix_VC_STAR / _VR_STAR (row blocks),
// DistMatrix_STAR_VC / _STAR_VR (column blocks), SharedMatrix (replicated),
// RootMatrix (rank 0); sl_dist_local_shape gives the shard's shape.
SL_CAPI int sl_wrap_raw_dist_device_matrix(void* local, int dtype, int64_t m, int64_t n, int64_t ld, void* comm,
                                           void** A) {
  if (dtype < 0 || dtype > 2 || m < 0 || n < 0 || ld < 0) return 109;
  *A = new sl_raw_dist_device_matrix_t{sldev::DistMat{local, dtype, m, n, ld, comm}};
  return 0;
}

SL_CAPI int sl_free_raw_dist_device_matrix_wrap(void* A) {
  delete (sl_raw_dist_device_matrix_t*)A;
  return 0;
}

// this rank's shard (row / column offset and shape) of a global m x n matrix of the given type
SL_CAPI int sl_dist_local_shape(char* type, int64_t m, int64_t n, void* comm, int64_t* r0, int64_t* c0, int64_t* lm,
                                int64_t* ln) {
  const int ly = dist_layout(type);
  if (ly < 0) {
    g_last_error = std::string("sl_dist_local_shape: not a native distributed type: ") + type;
    return ly == -2 ? 103 : 109;
  }
  int rank = 0, size = 1;
  if (comm) {
    const int rc = sldev::comm_rank_size(comm, &rank, &size);
    if (rc) return native_fail(rc);
  }
  sldev::shard_of(ly, m, n, rank, size, r0, c0, lm, ln);
  return 0;
}

// a callback communicator (the caller's all-reduce, e.g. over MPI): the
// distributed paths only all-reduce.  fn(send, recv, count, dtype, op, stream, user) -> 0
SL_CAPI int sl_device_comm_from_allreduce(int rank, int size, void* fn, void* user, void** comm) {
  sldev::Lib& L = sldev::lib();
  if (!L.loaded) {
    g_last_error = "device C API: " + L.err;
    return 106;
  }
  using F = int (*)(int, int, void*, void*, void**);
  static F f = (F)dlsym(L.h, "sl_comm_from_allreduce");
  if (!f) {
    g_last_error = "sl_comm_from_allreduce missing";
    return 106;
  }
  return f(rank, size, fn, user, comm) ? (g_last_error = L.last_error(), 106) : 0;
}

// device memory helpers for C callers of the DeviceMatrix paths (kind: 0
// host->device, 1 device->host, 2 device->device)
SL_CAPI int sl_device_malloc(int64_t bytes, void** p) {
  auto& L = sldev::lib();
  if (!L.loaded) { g_last_error = L.err; return 106; }
  return L.dev_malloc(bytes, p) ? 101 : 0;
}

SL_CAPI int sl_device_free(void* p) {
  auto& L = sldev::lib();
  return L.loaded ? (L.dev_free(p) ? 106 : 0) : 106;
}

SL_CAPI int sl_device_memcpy(void* dst, const void* src, int64_t bytes, int kind) {
  auto& L = sldev::lib();
  if (!L.loaded) { g_last_error = L.err; return 106; }
  if (L.dev_memcpy(dst, src, bytes, kind, nullptr) || L.dev_sync(nullptr)) {
    g_last_error = L.last_error();
    return 106;
  }
  return 0;
}

SL_CAPI int sl_wrap_raw_sp_matrix(int* indptr, int* ind, double* data, int nnz, int n_rows, int n_cols, void** A) {
  auto* M = new sl_raw_sp_matrix_t();
  *M = sl_raw_sp_matrix_t{indptr, ind, data, nnz, n_rows, n_cols, nullptr};
  *A = M;
  return 0;
}

SL_CAPI int sl_free_raw_sp_matrix_wrap(void* A) {
  auto* M = (sl_raw_sp_matrix_t*)A;
  if (M->out) {
    Gil g;
    Py_DECREF(M->out);
  }
  delete M;
  return 0;
}

namespace {
template <typename F>
int sp_query(void* A, F&& f) {
  auto* M = (sl_raw_sp_matrix_t*)A;
  if (!M->out) return 109;
  Gil g;
  return f(M->out);
}
long attr_long(PyObject* o, const char* name, int idx = -1) {
  PyObject* a = PyObject_GetAttrString(o, name);
  if (!a) return -1;
  long v;
  if (idx >= 0) {
    PyObject* it = PySequence_GetItem(a, idx);
    v = PyLong_AsLong(it);
    Py_XDECREF(it);
  } else {
    v = PyObject_IsTrue(a);
  }
  Py_DECREF(a);
  return v;
}
long array_len(PyObject* o, const char* name) {
  PyObject* a = PyObject_GetAttrString(o, name);
  if (!a) return -1;
  long v = (long)PyObject_Length(a);
  Py_DECREF(a);
  return v;
}
void copy_array(PyObject* o, const char* name, void* dst, size_t elem) {
  PyObject* a = PyObject_GetAttrString(o, name);
  if (!a) return;
  PyObject* b = PyObject_CallMethod(a, "tobytes", nullptr);
  if (b) {
    char* p;
    Py_ssize_t n;
    PyBytes_AsStringAndSize(b, &p, &n);
    memcpy(dst, p, (size_t)n);
    Py_DECREF(b);
  }
  (void)elem;
  Py_DECREF(a);
}
sl_raw_sp_matrix_t* sp_nat(void* A) {
  auto* M = (sl_raw_sp_matrix_t*)A;
  return M->nat && !M->out ? M : nullptr;
}
// store a column-major dense m x n result as the native CSC output (exact zeros dropped)
void set_sparse_out(void* A, const double* X, int64_t m, int64_t n) {
  auto* M = (sl_raw_sp_matrix_t*)A;
  if (M->out) {
    Gil g;
    Py_DECREF(M->out);
    M->out = nullptr;
  }
  M->nat = true;
  M->nat_updated = true;
  M->nat_m = (int)m;
  M->nat_n = (int)n;
  M->nat_indptr.assign((size_t)n + 1, 0);
  M->nat_ind.clear();
  M->nat_val.clear();
  for (int64_t j = 0; j < n; ++j) {
    for (int64_t i = 0; i < m; ++i) {
      const double v = X[i + j * m];
      if (v != 0.0) {
        M->nat_ind.push_back((int)i);
        M->nat_val.push_back(v);
      }
    }
    M->nat_indptr[(size_t)j + 1] = (int)M->nat_ind.size();
  }
}
// dense column-major copy of a CSC input
std::vector<double> csc_dense(const sl_raw_sp_matrix_t* M) {
  std::vector<double> D((size_t)M->m * (size_t)M->n, 0.0);
  for (int j = 0; j < M->n; ++j)
    for (int q = M->indptr[j]; q < M->indptr[j + 1]; ++q) D[(size_t)M->ind[q] + (size_t)j * (size_t)M->m] += M->data[q];
  return D;
}
}  // namespace

SL_CAPI int sl_raw_sp_matrix_struct_updated(void* A, bool* updated) {
  if (auto* M = sp_nat(A)) {
    *updated = M->nat_updated;
    return 0;
  }
  return sp_query(A, [&](PyObject* o) {
    *updated = attr_long(o, "updated") != 0;
    return 0;
  });
}

SL_CAPI int sl_raw_sp_matrix_reset_update_flag(void* A) {
  if (auto* M = sp_nat(A)) {
    M->nat_updated = false;
    return 0;
  }
  return sp_query(A, [&](PyObject* o) {
    PyObject_SetAttrString(o, "updated", Py_False);
    return 0;
  });
}

SL_CAPI int sl_raw_sp_matrix_nnz(void* A, int* nnz) {
  if (auto* M = sp_nat(A)) {
    *nnz = (int)M->nat_val.size();
    return 0;
  }
  return sp_query(A, [&](PyObject* o) {
    *nnz = (int)array_len(o, "values");
    return 0;
  });
}

SL_CAPI int sl_raw_sp_matrix_height(void* A, int* h) {
  if (auto* M = sp_nat(A)) {
    *h = M->nat_m;
    return 0;
  }
  return sp_query(A, [&](PyObject* o) {
    *h = (int)attr_long(o, "shape", 0);
    return 0;
  });
}

SL_CAPI int sl_raw_sp_matrix_width(void* A, int* w) {
  if (auto* M = sp_nat(A)) {
    *w = M->nat_n;
    return 0;
  }
  return sp_query(A, [&](PyObject* o) {
    *w = (int)attr_long(o, "shape", 1);
    return 0;
  });
}

SL_CAPI int sl_raw_sp_matrix_data(void* A, int32_t* indptr, int32_t* indices, double* values) {
  if (auto* M = sp_nat(A)) {
    memcpy(indptr, M->nat_indptr.data(), sizeof(int) * M->nat_indptr.size());
    if (!M->nat_ind.empty()) {
      memcpy(indices, M->nat_ind.data(), sizeof(int) * M->nat_ind.size());
      memcpy(values, M->nat_val.data(), sizeof(double) * M->nat_val.size());
    }
    return 0;
  }
  return sp_query(A, [&](PyObject* o) {
    copy_array(o, "indptr", indptr, 4);
    copy_array(o, "indices", indices, 4);
    copy_array(o, "values", values, 8);
    return 0;
  });
}

// ---------------------------------------------------------------- sketches
SL_CAPI int sl_create_sketch_transform(sl_context_t* ctxt, char* type, int n, int s, sl_sketch_transform_t** sketch,
                                       ...) {
  if (slnat::supported(type) && n > 0 && s > 0 && strcmp(type, "NURST") != 0) {
    auto* ns = new slnat::Sketch();
    ns->type = type;
    ns->N = n;
    ns->S = s;
    ns->seed = ctxt->seed;
    ns->ctr0 = ctxt->counter;
    const std::string spec = slnat::vararg_spec(ns->type);
    double dv[4] = {0, 0, 0, 0};
    int64_t iv[4] = {0, 0, 0, 0};
    va_list ap;
    va_start(ap, sketch);
    for (size_t i = 0; i < spec.size() && i < 4; ++i) {
      if (spec[i] == 'i') iv[i] = va_arg(ap, int);
      else dv[i] = va_arg(ap, double);
    }
    va_end(ap);
    slnat::set_params(*ns, dv, iv);
    std::string err;
    const uint64_t c = slnat::build(*ns, &err);
    if (!err.empty()) {
      g_last_error = "sl_create_sketch_transform: " + err;
      delete ns;
      return 109;
    }
    ctxt->counter = c;
    *sketch = new sl_sketch_transform_t{nullptr, ns};
    return 0;
  }
  Gil g;
  std::string spec = spec_of("sketch_param_spec", type);
  va_list ap;
  va_start(ap, sketch);
  PyObject* params = varargs_tuple(spec, ap);
  va_end(ap);
  PyObject* c = py_ctx(ctxt);
  if (!c) {
    Py_XDECREF(params);
    return fail();
  }
  PyObject* r = call("create_sketch", Py_BuildValue("(OsiiN)", c, type, n, s, params));
  ctx_sync_back(ctxt);
  if (!r) {
    int code = fail();
    return code == 100 || code == 109 ? 111 : code;
  }
  *sketch = new sl_sketch_transform_t{r, nullptr};
  return 0;
}

SL_CAPI int sl_deserialize_sketch_transform(const char* data, sl_sketch_transform_t** sketch) {
  slnat::Sketch tmp;
  if (slnat::from_json(data, tmp)) {
    *sketch = new sl_sketch_transform_t{nullptr, new slnat::Sketch(std::move(tmp))};
    return 0;
  }
  Gil g;
  PyObject* r = call("deserialize_sketch", Py_BuildValue("(s)", data));
  if (!r) return fail();
  *sketch = new sl_sketch_transform_t{r, nullptr};
  return 0;
}

SL_CAPI int sl_serialize_sketch_transform(const sl_sketch_transform_t* sketch, char** data) {
  if (sketch->nat) {
    *data = strdup(slnat::to_json(*sketch->nat).c_str());
    return 0;
  }
  Gil g;
  PyObject* r = call("serialize_sketch", Py_BuildValue("(O)", sketch->obj));
  if (!r) return fail();
  *data = strdup(PyUnicode_AsUTF8(r));
  Py_DECREF(r);
  return 0;
}

SL_CAPI int sl_free_sketch_transform(sl_sketch_transform_t* S) {
  if (!S) return 0;
  if (S->obj) {
    Gil g;
    Py_XDECREF(S->obj);
  }
  delete S->nat;
  delete S;
  return 0;
}

SL_CAPI int sl_apply_sketch_transform(sl_sketch_transform_t* S, char* input_type, void* A, char* output_type,
                                      void* SA, int dim) {
  int lin, lout;
  if (const int e = dist_pair("sl_apply_sketch_transform", input_type, output_type, &lin, &lout)) return e;
  if (lin >= 0) {
    if (!S->nat) {
      g_last_error = "sl_apply_sketch_transform: this sketch type has no device C path";
      return 103;
    }
    if (dim != 0 && dim != 1) {
      g_last_error = "sl_apply_sketch_transform: dim must be 0 (columnwise) or 1 (rowwise)";
      return 109;
    }
    const int rc = sldev::apply_sketch_dist(*S->nat, lin, distmat(A), lout, distmat(SA), dim);
    return rc ? native_fail(rc) : 0;
  }
  if (is_device(input_type) || is_device(output_type)) {
    if (!is_device(input_type) || !is_device(output_type)) {
      g_last_error = "sl_apply_sketch_transform: DeviceMatrix input needs a DeviceMatrix output";
      return 109;
    }
    if (!S->nat) {
      g_last_error = "sl_apply_sketch_transform: this sketch type has no device C path";
      return 103;
    }
    const int rc = sldev::apply_sketch(*S->nat, devmat(A), devmat(SA), dim);
    return rc ? native_fail(rc) : 0;
  }
  const bool in_dense = !strcmp(input_type, "Matrix"), in_sparse = !strcmp(input_type, "SparseMatrix");
  const bool out_dense = !strcmp(output_type, "Matrix"), out_sparse = !strcmp(output_type, "SparseMatrix");
  if (S->nat && (in_dense || in_sparse) && (out_dense || (out_sparse && in_sparse))) {
    // host operands: staged to the GPU when one is present, else the host path
    const slnat::Sketch& sk = *S->nat;
    if (dim != 0 && dim != 1) {
      g_last_error = "sl_apply_sketch_transform: dim must be 0 (columnwise) or 1 (rowwise)";
      return 109;
    }
    int64_t m, n;
    if (in_dense) {
      m = ((sl_raw_matrix_t*)A)->m;
      n = ((sl_raw_matrix_t*)A)->n;
    } else {
      m = ((sl_raw_sp_matrix_t*)A)->m;
      n = ((sl_raw_sp_matrix_t*)A)->n;
    }
    const int64_t sm = dim == 0 ? sk.S : m, sn = dim == 0 ? n : sk.S;
    if (out_dense && (((sl_raw_matrix_t*)SA)->m != sm || ((sl_raw_matrix_t*)SA)->n != sn)) {
      g_last_error = "sl_apply_sketch_transform: dimension mismatch (output)";
      return 104;
    }
    if ((dim == 0 ? m : n) != sk.N) {
      g_last_error = "sl_apply_sketch_transform: dimension mismatch (input)";
      return 104;
    }
    std::vector<double> tmp;
    double* out = out_dense ? ((sl_raw_matrix_t*)SA)->data : nullptr;
    if (!out) {
      tmp.assign((size_t)(sm * sn), 0.0);
      out = tmp.data();
    }
    int rc;
    if (sldev::device_present()) {
      if (in_dense) {
        rc = sldev::apply_host_dense(sk, ((sl_raw_matrix_t*)A)->data, m, n, out, sm, sn, dim);
      } else {
        auto* M = (sl_raw_sp_matrix_t*)A;
        rc = sldev::apply_host_csc(sk, M->indptr, M->ind, M->data, M->nnz, m, n, out, sm, sn, dim);
      }
      if (rc) return native_fail(rc);
    } else {
      std::vector<double> dense;
      const double* a = in_dense ? ((sl_raw_matrix_t*)A)->data : nullptr;
      if (!a) {
        dense = csc_dense((sl_raw_sp_matrix_t*)A);
        a = dense.data();
      }
      rc = slnat::apply(sk, a, m, n, out, sm, sn, dim);
      if (rc) {
        g_last_error = "sl_apply_sketch_transform: dimension mismatch";
        return rc;
      }
    }
    if (out_sparse) set_sparse_out(SA, out, sm, sn);
    return 0;
  }
  Gil g;
  PyObject* so = py_sketch(S);
  if (!so) return fail();
  PyObject* a = in_desc(input_type, A);
  if (!a) return fail();
  PyObject* o = out_desc(output_type, SA);
  if (!o) {
    Py_DECREF(a);
    return fail();
  }
  PyObject* r = call("apply_sketch", Py_BuildValue("(OsNsNi)", so, input_type, a, output_type, o, dim));
  if (!r) return fail();
  Py_DECREF(r);
  return 0;
}

// --------------------------------------------------------------------- NLA
SL_CAPI int sl_approximate_svd(char* A_type, void* A, char* U_type, void* U, char* S_type, void* Sv, char* V_type,
                               void* V, uint16_t k, char* params, sl_context_t* ctxt) {
  int la, lu;
  if (const int e = dist_pair("sl_approximate_svd", A_type, U_type, &la, &lu)) return e;
  if (la >= 0) {
    // row-distributed A ([VC,*] / [VR,*]): U in A's rows, S and V replicated;
    // the engine's pass sums all-reduced over A's communicator
    if (la != sldev::LY_ROWS || lu != sldev::LY_ROWS || dist_layout(S_type) != sldev::LY_STAR ||
        dist_layout(V_type) != sldev::LY_STAR) {
      g_last_error = "sl_approximate_svd: distributed A must be DistMatrix_VC_STAR / _VR_STAR with U in the same "
                     "layout and S, V SharedMatrix";
      return 103;
    }
    const sldev::DistMat &a = distmat(A), &u = distmat(U), &sv = distmat(Sv), &v = distmat(V);
    if (u.comm != a.comm || sv.comm != a.comm || v.comm != a.comm) {
      g_last_error = "sl_approximate_svd: operands on different communicators";
      return 109;
    }
    if (u.m != a.m) {
      g_last_error = "sl_approximate_svd: U must have A's rows";
      return 104;
    }
    int rank = 0, size = 1;
    int rc = sldev::comm_rank_size(a.comm, &rank, &size);
    if (rc) return native_fail(rc);
    rc = sldev::approximate_svd(dist_local(la, a, rank, size), dist_local(lu, u, rank, size),
                                dist_local(sldev::LY_STAR, sv, rank, size), dist_local(sldev::LY_STAR, v, rank, size),
                                (int)k, params, ctxt->seed, ctxt->counter, a.comm);
    return rc ? native_fail(rc) : 0;
  }
  if (is_device(A_type)) {
    if (!is_device(U_type) || !is_device(S_type) || !is_device(V_type)) {
      g_last_error = "sl_approximate_svd: DeviceMatrix A needs DeviceMatrix U, S, V";
      return 109;
    }
    const int rc = sldev::approximate_svd(devmat(A), devmat(U), devmat(Sv), devmat(V), (int)k, params, ctxt->seed,
                                          ctxt->counter, ctxt->dcomm);
    return rc ? native_fail(rc) : 0;
  }
  if (!strcmp(A_type, "Matrix") && !strcmp(U_type, "Matrix") && !strcmp(S_type, "Matrix") && !strcmp(V_type, "Matrix") &&
      sldev::device_present()) {
    auto *a = (sl_raw_matrix_t*)A, *u = (sl_raw_matrix_t*)U, *sv = (sl_raw_matrix_t*)Sv, *v = (sl_raw_matrix_t*)V;
    if (u->m != a->m || u->n != (int)k || v->m != a->n || v->n != (int)k || (int64_t)sv->m * sv->n != (int64_t)k) {
      g_last_error = "sl_approximate_svd: output shapes (U m x k, S k x 1, V n x k)";
      return 104;
    }
    uint64_t ctr = ctxt->counter;
    const int rc = sldev::approximate_svd_host(a->data, a->m, a->n, u->data, sv->data, v->data, (int)k, params,
                                               ctxt->seed, ctr);
    if (rc != sldev::HOST_DECLINED) {
      if (rc) return native_fail(rc);
      ctxt->counter = ctr;
      return 0;
    }
  }
  Gil g;
  (void)U_type;
  (void)S_type;
  (void)V_type;
  PyObject* a = in_desc(A_type, A);
  if (!a) return fail();
  PyObject* r = call("approximate_svd", Py_BuildValue("(sNNNNisO)", A_type, a, dense_desc(U), dense_desc(Sv),
                                                      dense_desc(V), (int)k, params ? params : "", py_ctx(ctxt)));
  ctx_sync_back(ctxt);
  if (!r) return fail();
  Py_DECREF(r);
  return 0;
}

SL_CAPI int sl_approximate_symmetric_svd(char* A_type, void* A, char* S_type, void* Sv, char* V_type, void* V,
                                         uint16_t k, char* params, sl_context_t* ctxt) {
  int la, lv;
  if (const int e = dist_pair("sl_approximate_symmetric_svd", A_type, V_type, &la, &lv)) return e;
  if (la >= 0) {
    if (la != sldev::LY_ROWS || dist_layout(S_type) != sldev::LY_STAR || (lv != sldev::LY_STAR && lv != sldev::LY_ROWS)) {
      g_last_error = "sl_approximate_symmetric_svd: distributed A must be DistMatrix_VC_STAR / _VR_STAR, S "
                     "SharedMatrix, V SharedMatrix or A's layout";
      return 103;
    }
    uint64_t ctr = ctxt->counter;
    const int rc = sldev::approximate_symmetric_svd_dist(distmat(A), distmat(Sv), lv, distmat(V), (int)k, params,
                                                         ctxt->seed, ctr);
    if (rc) return native_fail(rc);
    ctxt->counter = ctr;
    return 0;
  }
  if (!strcmp(A_type, "Matrix") && !strcmp(S_type, "Matrix") && !strcmp(V_type, "Matrix") && sldev::device_present()) {
    auto *a = (sl_raw_matrix_t*)A, *sv = (sl_raw_matrix_t*)Sv, *v = (sl_raw_matrix_t*)V;
    if (a->m != a->n) {
      g_last_error = "sl_approximate_symmetric_svd: matrix is not square -- symmetric matrix required";
      return 109;
    }
    if (v->m != a->n || v->n != (int)k || (int64_t)sv->m * sv->n != (int64_t)k) {
      g_last_error = "sl_approximate_symmetric_svd: output shapes (S k x 1, V n x k)";
      return 104;
    }
    uint64_t ctr = ctxt->counter;
    const int rc = sldev::approximate_symmetric_svd_host(a->data, a->n, sv->data, v->data, (int)k, params, ctxt->seed,
                                                         ctr);
    if (rc) return native_fail(rc);
    ctxt->counter = ctr;
    return 0;
  }
  Gil g;
  (void)S_type;
  (void)V_type;
  PyObject* a = in_desc(A_type, A);
  if (!a) return fail();
  PyObject* r = call("approximate_symmetric_svd", Py_BuildValue("(sNNNisO)", A_type, a, dense_desc(Sv),
                                                                dense_desc(V), (int)k, params ? params : "",
                                                                py_ctx(ctxt)));
  ctx_sync_back(ctxt);
  if (!r) return fail();
  Py_DECREF(r);
  return 0;
}

SL_CAPI int sl_faster_least_squares(int orientation, char* A_type, void* A, char* B_type, void* B, char* X_type,
                                    void* X, char* params, sl_context_t* ctxt) {
  int la, lb;
  if (const int e = dist_pair("sl_faster_least_squares", A_type, B_type, &la, &lb)) return e;
  if (la >= 0) {
    if (orientation != 0 || la != sldev::LY_ROWS || lb != sldev::LY_ROWS || dist_layout(X_type) != sldev::LY_STAR) {
      g_last_error = "sl_faster_least_squares: distributed operands: orientation NORMAL, A and B DistMatrix_VC_STAR / "
                     "_VR_STAR, X SharedMatrix";
      return 103;
    }
    uint64_t ctr = ctxt->counter;
    const int rc = sldev::faster_least_squares_dist(distmat(A), distmat(B), distmat(X), params, ctxt->seed, ctr);
    if (rc) return native_fail(rc);
    ctxt->counter = ctr;
    return 0;
  }
  if (!strcmp(A_type, "Matrix") && !strcmp(B_type, "Matrix") && !strcmp(X_type, "Matrix") && sldev::device_present()) {
    auto *a = (sl_raw_matrix_t*)A, *b = (sl_raw_matrix_t*)B, *x = (sl_raw_matrix_t*)X;
    uint64_t ctr = ctxt->counter;
    const int rc = sldev::faster_least_squares_host(orientation, a->data, a->m, a->n, b->data, b->m, b->n, x->data, x->m,
                                                    x->n, params, ctxt->seed, ctr);
    if (rc != sldev::HOST_DECLINED) {
      if (rc) return native_fail(rc);
      ctxt->counter = ctr;
      return 0;
    }
  }
  Gil g;
  (void)B_type;
  (void)X_type;
  PyObject* a = in_desc(A_type, A);
  if (!a) return fail();
  PyObject* r = call("faster_least_squares", Py_BuildValue("(isNNNsO)", orientation, A_type, a, dense_desc(B),
                                                           dense_desc(X), params ? params : "", py_ctx(ctxt)));
  ctx_sync_back(ctxt);
  if (!r) return fail();
  Py_DECREF(r);
  return 0;
}

// ----------------------------------------------------------------- kernels
namespace {
// runtime object of a kernel (a native one is created on first host use)
PyObject* py_kernel(sl_kernel_t* k) {
  if (k->obj) return k->obj;
  const auto& n = k->nat;
  PyObject* params = nullptr;
  switch (n.type) {
    case sldev::K_LINEAR: params = PyTuple_New(0); break;
    case sldev::K_GAUSSIAN:
    case sldev::K_LAPLACIAN:
    case sldev::K_EXPSEMIGROUP: params = Py_BuildValue("(d)", n.p[0]); break;
    case sldev::K_POLYNOMIAL: params = Py_BuildValue("(idd)", (int)n.p[0], n.p[1], n.p[2]); break;
    case sldev::K_MATERN: params = Py_BuildValue("(dd)", n.p[0], n.p[1]); break;
    default: PyErr_SetString(PyExc_ValueError, "unknown kernel"); return nullptr;
  }
  k->obj = call("create_kernel", Py_BuildValue("(siN)", k->type.c_str(), n.N, params));
  return k->obj;
}
}  // namespace

// Kernels known to the native layer (linear, gaussian(sigma), laplacian(sigma),
// expsemigroup(beta), polynomial(int q, c, gamma), matern(nu, l)) are created
// without the interpreter; others go to the runtime.
SL_CAPI int sl_create_kernel(char* type, int N, sl_kernel_t** kernel, ...) {
  const int kt = sldev::kernel_type_of(type);
  if (kt != sldev::K_NONE) {
    auto* k = new sl_kernel_t{nullptr, sldev::Kern{}, type};
    k->nat.type = kt;
    k->nat.N = N;
    va_list ap;
    va_start(ap, kernel);
    switch (kt) {
      case sldev::K_GAUSSIAN:
      case sldev::K_LAPLACIAN:
      case sldev::K_EXPSEMIGROUP: k->nat.p[0] = va_arg(ap, double); break;
      case sldev::K_POLYNOMIAL:
        k->nat.p[0] = (double)va_arg(ap, int);
        k->nat.p[1] = va_arg(ap, double);
        k->nat.p[2] = va_arg(ap, double);
        break;
      case sldev::K_MATERN:
        k->nat.p[0] = va_arg(ap, double);
        k->nat.p[1] = va_arg(ap, double);
        break;
      default: break;
    }
    va_end(ap);
    *kernel = k;
    return 0;
  }
  Gil g;
  std::string spec = spec_of("kernel_param_spec", type);
  va_list ap;
  va_start(ap, kernel);
  PyObject* params = varargs_tuple(spec, ap);
  va_end(ap);
  PyObject* r = call("create_kernel", Py_BuildValue("(siN)", type, N, params));
  if (!r) return fail();
  *kernel = new sl_kernel_t{r, sldev::Kern{}, type};
  return 0;
}

SL_CAPI int sl_free_kernel(sl_kernel_t* k) {
  if (!k) return 0;
  if (k->obj) {
    Gil g;
    Py_XDECREF(k->obj);
  }
  delete k;
  return 0;
}

SL_CAPI int sl_kernel_gram(int dirX, int dirY, sl_kernel_t* k, char* X_type, void* X, char* Y_type, void* Y,
                           char* K_type, void* K) {
  int lx, ly;
  if (const int e = dist_pair("sl_kernel_gram", X_type, Y_type, &lx, &ly)) return e;
  if (lx >= 0) {
    // K's rows follow X's points and its columns Y's points: X's points (rows,
    // dirX != SL_COLUMNS) split as [VC,*] give K's rows as [VC,*]; Y's points
    // (columns, dirY == SL_COLUMNS) split as [*,VC] give K's columns as [*,VC];
    // the other operand replicated.  Every rank forms its block, no communication.
    const int lk = dist_layout(K_type);
    const bool xr = dirX != 1, yc = dirY == 1;
    int want = -1;
    if (lx == sldev::LY_STAR && ly == sldev::LY_STAR) want = sldev::LY_STAR;
    else if (lx == sldev::LY_ROWS && xr && ly == sldev::LY_STAR) want = sldev::LY_ROWS;
    else if (lx == sldev::LY_STAR && ly == sldev::LY_COLS && yc) want = sldev::LY_COLS;
    if (want < 0 || lk != want) {
      g_last_error = "sl_kernel_gram: distributed operands: X's points as DistMatrix_VC_STAR rows (K the same), or Y's "
                     "points as DistMatrix_STAR_VC columns (K the same), the other SharedMatrix";
      return 103;
    }
    if (k->nat.type == sldev::K_NONE) {
      g_last_error = "sl_kernel_gram: this kernel has no device C path";
      return 103;
    }
    const sldev::DistMat &x = distmat(X), &y = distmat(Y), &kk = distmat(K);
    int rank = 0, size = 1;
    int rc = sldev::comm_rank_size(x.comm, &rank, &size);
    if (rc) return native_fail(rc);
    const sldev::DevMat kl = dist_local(lk, kk, rank, size);
    if (kl.m == 0 || kl.n == 0) return 0;
    rc = sldev::kernel_gram(k->nat, dirX, dirY, dist_local(lx, x, rank, size), dist_local(ly, y, rank, size), kl);
    return rc ? native_fail(rc) : 0;
  }
  if (is_device(X_type) || is_device(Y_type) || is_device(K_type)) {
    if (!is_device(X_type) || !is_device(Y_type) || !is_device(K_type)) {
      g_last_error = "sl_kernel_gram: mix of DeviceMatrix and host operands";
      return 109;
    }
    if (k->nat.type == sldev::K_NONE) {
      g_last_error = "sl_kernel_gram: this kernel has no device C path";
      return 103;
    }
    const int rc = sldev::kernel_gram(k->nat, dirX, dirY, devmat(X), devmat(Y), devmat(K));
    return rc ? native_fail(rc) : 0;
  }
  if (!strcmp(X_type, "Matrix") && !strcmp(Y_type, "Matrix") && !strcmp(K_type, "Matrix") &&
      k->nat.type != sldev::K_NONE && sldev::device_present()) {
    // host operands, natively: staged to the GPU (no interpreter)
    const auto* x = (const sl_raw_matrix_t*)X;
    const auto* y = (const sl_raw_matrix_t*)Y;
    const auto* kk = (const sl_raw_matrix_t*)K;
    const int rc = sldev::kernel_gram_host(k->nat, dirX, dirY, x->data, x->m, x->n, y->data, y->m, y->n, kk->data,
                                           kk->m, kk->n);
    return rc ? native_fail(rc) : 0;
  }
  Gil g;
  (void)K_type;
  PyObject* ko = py_kernel(k);
  if (!ko) return fail();
  PyObject* x = in_desc(X_type, X);
  if (!x) return fail();
  PyObject* y = in_desc(Y_type, Y);
  if (!y) {
    Py_DECREF(x);
    return fail();
  }
  PyObject* r = call("kernel_gram", Py_BuildValue("(iiOsNsNN)", dirX, dirY, ko, X_type, x, Y_type, y,
                                                  dense_desc(K)));
  if (!r) return fail();
  Py_DECREF(r);
  return 0;
}

// ---------------------------------------------------------------------- IO
SL_CAPI int sl_readlibsvm(char* fname, char* X_type, void* X, char* Y_type, void* Y, int direction, int min_d,
                          int max_n) {
  int lx, ly;
  if (const int e = dist_pair("sl_readlibsvm", X_type, Y ? Y_type : X_type, &lx, &ly)) return e;
  if (lx >= 0) {
    // DistMatrix X (f64 device shards): examples as rows split [VC,*] (direction
    // rows: n x d) or as columns split [*,VC] (SL_COLUMNS: d x n); Y (labels,
    // n x 1 / 1 x n) in the matching layout or replicated.  Every rank parses
    // the file and uploads its own examples.
    const bool cols = direction == 1;
    const int want = cols ? sldev::LY_COLS : sldev::LY_ROWS;
    if (lx != want || (Y && ly != want && ly != sldev::LY_STAR)) {
      g_last_error = "sl_readlibsvm: distributed X must be DistMatrix_VC_STAR (examples as rows) or DistMatrix_STAR_VC "
                     "(SL_COLUMNS), Y in the same layout or SharedMatrix";
      return 103;
    }
    sldev::Libsvm L;
    int rc = sldev::read_libsvm(fname, min_d, max_n, L);
    if (rc) return native_fail(rc);
    const sldev::DistMat& x = distmat(X);
    const int64_t n = L.rows, d = L.d;
    if (x.dtype != sldev::F64 || x.m != (cols ? d : n) || x.n != (cols ? n : d)) {
      g_last_error = "sl_readlibsvm: X wrap has the wrong global shape or dtype (f64)";
      return 109;
    }
    int rank = 0, size = 1;
    if ((rc = sldev::comm_rank_size(x.comm, &rank, &size))) return native_fail(rc);
    int64_t r0, c0, lm, ln;
    sldev::shard_of(lx, x.m, x.n, rank, size, &r0, &c0, &lm, &ln);
    const int64_t e0 = cols ? c0 : r0, ne = cols ? ln : lm;   // this rank's examples
    std::vector<double> h((size_t)std::max<int64_t>(1, lm * ln), 0.0);
    for (int64_t i = e0; i < e0 + ne; ++i)
      for (int64_t q = L.rowptr[(size_t)i]; q < L.rowptr[(size_t)i + 1]; ++q) {
        const int64_t j = L.cols[(size_t)q];
        h[(size_t)(cols ? j * ln + (i - e0) : (i - e0) * ln + j)] += L.vals[(size_t)q];
      }
    sldev::Lib& Lb = sldev::lib();
    if (lm * ln > 0 &&
        (rc = sldev::check(Lb.dev_memcpy2d(x.data, x.ld * 8, h.data(), ln * 8, ln * 8, lm, 0, nullptr), "copy")))
      return native_fail(rc);
    if (Y) {
      const sldev::DistMat& y = distmat(Y);
      if (y.dtype != sldev::F64 || y.m != (cols ? 1 : n) || y.n != (cols ? n : 1) || y.comm != x.comm) {
        g_last_error = "sl_readlibsvm: Y wrap has the wrong global shape, dtype (f64) or communicator";
        return 109;
      }
      int64_t yr0, yc0, ylm, yln;
      sldev::shard_of(ly, y.m, y.n, rank, size, &yr0, &yc0, &ylm, &yln);
      const int64_t y0 = cols ? yc0 : yr0, ny = ylm * yln;   // the labels of this shard, in example order
      if (ny > 0) {
        // a column of labels is strided by ld, a row contiguous
        if (cols) rc = sldev::check(Lb.dev_memcpy(y.data, L.labels.data() + y0, ny * 8, 0, nullptr), "copy");
        else rc = sldev::check(Lb.dev_memcpy2d(y.data, y.ld * 8, L.labels.data() + y0, 8, 8, ny, 0, nullptr), "copy");
        if (rc) return native_fail(rc);
      }
    }
    return 0;
  }
  const bool xd = !strcmp(X_type, "Matrix"), xs = !strcmp(X_type, "SparseMatrix");
  if ((xd || xs) && (!Y || !strcmp(Y_type, "Matrix")) && sldev::lib().loaded) {
    // native LIBSVM reader (libsvm_io.cpp): examples are columns (direction
    // SL_COLUMNS = 1: d x n, labels 1 x n) or rows (anything else, as the
    // reference's cio.cpp:17-18 maps it: n x d, labels n x 1)
    sldev::Libsvm L;
    const int rc = sldev::read_libsvm(fname, min_d, max_n, L);
    if (rc) return native_fail(rc);
    const bool cols = direction == 1;
    const int64_t n = L.rows, d = L.d;
    const int64_t xm = cols ? d : n, xn = cols ? n : d;
    if (Y) {
      auto* y = (sl_raw_matrix_t*)Y;
      if (y->m != (cols ? 1 : n) || y->n != (cols ? n : 1)) {
        g_last_error = "sl_readlibsvm: Y wrap has the wrong shape";
        return 109;
      }
      memcpy(y->data, L.labels.data(), sizeof(double) * (size_t)n);
    }
    // (example i, feature j) -> column-major (j, i) or (i, j)
    auto at = [&](int64_t i, int64_t j) -> size_t { return cols ? (size_t)(j + i * xm) : (size_t)(i + j * xm); };
    if (xd) {
      auto* x = (sl_raw_matrix_t*)X;
      if (x->m != xm || x->n != xn) {
        g_last_error = "sl_readlibsvm: X wrap has the wrong shape";
        return 109;
      }
      memset(x->data, 0, sizeof(double) * (size_t)(xm * xn));
      for (int64_t i = 0; i < n; ++i)
        for (int64_t q = L.rowptr[(size_t)i]; q < L.rowptr[(size_t)i + 1]; ++q)
          x->data[at(i, L.cols[(size_t)q])] += L.vals[(size_t)q];
      return 0;
    }
    // CSC built directly (entries sorted, duplicates summed): columns are the
    // examples (direction columns) or the features (rows)
    std::vector<std::vector<std::pair<int, double>>> colv((size_t)xn);
    for (int64_t i = 0; i < n; ++i)
      for (int64_t q = L.rowptr[(size_t)i]; q < L.rowptr[(size_t)i + 1]; ++q) {
        const int64_t j = L.cols[(size_t)q];
        if (cols) colv[(size_t)i].push_back({(int)j, L.vals[(size_t)q]});
        else colv[(size_t)j].push_back({(int)i, L.vals[(size_t)q]});
      }
    auto* M = (sl_raw_sp_matrix_t*)X;
    if (M->out) {
      Gil g;
      Py_DECREF(M->out);
      M->out = nullptr;
    }
    M->nat = M->nat_updated = true;
    M->nat_m = (int)xm;
    M->nat_n = (int)xn;
    M->nat_indptr.assign((size_t)xn + 1, 0);
    M->nat_ind.clear();
    M->nat_val.clear();
    for (int64_t j = 0; j < xn; ++j) {
      auto& v = colv[(size_t)j];
      std::stable_sort(v.begin(), v.end(), [](const std::pair<int, double>& a, const std::pair<int, double>& b) {
        return a.first < b.first;
      });
      for (size_t t = 0; t < v.size(); ++t) {
        if (t && v[t].first == v[t - 1].first) M->nat_val.back() += v[t].second;
        else {
          M->nat_ind.push_back(v[t].first);
          M->nat_val.push_back(v[t].second);
        }
      }
      M->nat_indptr[(size_t)j + 1] = (int)M->nat_ind.size();
    }
    return 0;
  }
  Gil g;
  (void)Y_type;
  PyObject* xo = out_desc(X_type, X);
  if (!xo) return fail();
  PyObject* yo = Y ? dense_desc(Y) : (Py_INCREF(Py_None), Py_None);
  PyObject* r = call("readlibsvm", Py_BuildValue("(ssNNiii)", fname, X_type, xo, yo, direction, min_d, max_n));
  if (!r) return fail();
  Py_DECREF(r);
  return 0;
}
