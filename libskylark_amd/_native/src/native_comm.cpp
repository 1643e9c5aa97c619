// Native collective layer: an RCCL communicator driven from
// C++ on device pointers and HIP streams, so native code (the C API, the
// runtime) can all-reduce / reduce-scatter / all-gather / all-to-all /
// broadcast / send / recv without bouncing through Python.  It replaces the
// reference's Boost.MPI + MPI calls on the same sites (base/inner.hpp,
// base/Gemm.hpp, sketch/*_Elemental*.hpp redistributions, ml/BlockADMM.hpp).
//
// RCCL is resolved at run time (dlsym on the process, then librccl.so.1), so
// a process that already loaded PyTorch's bundled RCCL shares that one
// library and nothing links against a second copy.  Unique-id exchange is
// the caller's job (the Python layer uses its process group for it).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "sl_common.hpp"

namespace {

struct Rccl {
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) err_str = nullptr;
  bool ok = false;
};

Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = RTLD_DEFAULT;
    if (!dlsym(h, "ncclCommInitRank")) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h || !dlsym(h, "ncclCommInitRank")) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return x;
#define SL_SYM(f, n) x.f = (decltype(x.f))dlsym(h, n)
    SL_SYM(get_id, "ncclGetUniqueId");
    SL_SYM(init, "ncclCommInitRank");
    SL_SYM(destroy, "ncclCommDestroy");
    SL_SYM(all_reduce, "ncclAllReduce");
    SL_SYM(reduce_scatter, "ncclReduceScatter");
    SL_SYM(all_gather, "ncclAllGather");
    SL_SYM(broadcast, "ncclBroadcast");
    SL_SYM(send, "ncclSend");
    SL_SYM(recv, "ncclRecv");
    SL_SYM(group_start, "ncclGroupStart");
    SL_SYM(group_end, "ncclGroupEnd");
    SL_SYM(err_str, "ncclGetErrorString");
#undef SL_SYM
    x.ok = x.get_id && x.init && x.destroy && x.all_reduce && x.reduce_scatter && x.all_gather && x.broadcast &&
           x.send && x.recv && x.group_start && x.group_end;
    return x;
  }();
  return r;
}

// all-reduce supplied by the caller (an MPI communicator, a test's process
// group, ...): sum / prod / max / min of count elements of dtype, device
// pointers, stream-ordered on `stream` (the callee synchronises as it needs)
typedef int (*SlAllReduceFn)(const void* send, void* recv, int64_t count, int dtype, int op, void* stream,
                             void* user);

struct SlComm {
  ncclComm_t comm = nullptr;
  int rank = 0, size = 1;
  SlAllReduceFn ar = nullptr;   // callback communicator (no RCCL) when set
  void* user = nullptr;
};

int check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return SL_OK;
  char buf[256];
  snprintf(buf, sizeof buf, "%s: %s", what, rccl().err_str ? rccl().err_str(r) : "rccl error");
  sl_set_last_error(buf);
  return SL_ERR_HIP;
}

// SL dtype codes (sl_common.hpp) -> RCCL
bool to_nccl(int dt, ncclDataType_t* out) {
  switch (dt) {
    case SL_F32: *out = ncclFloat32; return true;
    case SL_F64: *out = ncclFloat64; return true;
    case SL_BF16: *out = ncclBfloat16; return true;
    case 3: *out = ncclFloat16; return true;
    case 10: *out = ncclInt32; return true;
    case 11: *out = ncclInt64; return true;
    default: return false;
  }
}

bool to_op(int op, ncclRedOp_t* out) {
  switch (op) {
    case 0: *out = ncclSum; return true;
    case 1: *out = ncclProd; return true;
    case 2: *out = ncclMax; return true;
    case 3: *out = ncclMin; return true;
    default: return false;
  }
}

size_t elem_size(int dt) {
  switch (dt) {
    case SL_F64: case 11: return 8;
    case SL_BF16: case 3: return 2;
    default: return 4;
  }
}

SlComm* as_comm(void* c) { return (SlComm*)c; }

}  // namespace

SL_API int sl_comm_available() { return rccl().ok ? 1 : 0; }

SL_API int sl_comm_unique_id_bytes() { return (int)sizeof(ncclUniqueId); }

SL_API int sl_comm_unique_id(void* out) {
  if (!rccl().ok) { sl_set_last_error("RCCL not found"); return SL_ERR_UNSUPPORTED; }
  ncclUniqueId id;
  const int rc = check(rccl().get_id(&id), "ncclGetUniqueId");
  if (rc == SL_OK) memcpy(out, &id, sizeof id);
  return rc;
}

// Collective over the ranks that pass the same id; the current HIP device is used.
SL_API int sl_comm_init(const void* id, int nranks, int rank, void** comm_out) {
  if (!rccl().ok) { sl_set_last_error("RCCL not found"); return SL_ERR_UNSUPPORTED; }
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  SlComm* c = new SlComm;
  const int rc = check(rccl().init(&c->comm, nranks, uid, rank), "ncclCommInitRank");
  if (rc != SL_OK) { delete c; return rc; }
  c->rank = rank;
  c->size = nranks;
  *comm_out = c;
  return SL_OK;
}

// A communicator whose all-reduce is the caller's function (e.g. an MPI_Allreduce
// wrapper from a C program, as the reference's C API takes MPI communicators);
// sl_rsvd_run_comm / sl_rsvd_gen_run_comm only need the all-reduce.  The other
// collectives report SL_ERR_UNSUPPORTED on such a communicator.
SL_API int sl_comm_from_allreduce(int rank, int size, SlAllReduceFn fn, void* user, void** comm_out) {
  if (!fn || size < 1 || rank < 0 || rank >= size) { sl_set_last_error("comm: bad callback communicator"); return SL_ERR_INVALID; }
  SlComm* c = new SlComm;
  c->rank = rank;
  c->size = size;
  c->ar = fn;
  c->user = user;
  *comm_out = c;
  return SL_OK;
}

// this rank and the communicator size (null: one rank)
SL_API int sl_comm_rank_size(void* comm, int* rank, int* size) {
  SlComm* c = as_comm(comm);
  *rank = c ? c->rank : 0;
  *size = c ? c->size : 1;
  return SL_OK;
}

SL_API int sl_comm_destroy(void* comm) {
  SlComm* c = as_comm(comm);
  if (!c) return SL_OK;
  const int rc = c->comm ? check(rccl().destroy(c->comm), "ncclCommDestroy") : SL_OK;
  delete c;
  return rc;
}

SL_API int sl_comm_all_reduce(void* comm, const void* send, void* recv, int64_t count, int dtype, int op,
                              void* stream) {
  SlComm* c = as_comm(comm);
  if (c->ar) {
    const int rc = c->ar(send, recv, count, dtype, op, stream, c->user);
    if (rc != 0) sl_set_last_error("comm: the caller's all-reduce failed");
    return rc == 0 ? SL_OK : SL_ERR_GENERIC;
  }
  ncclDataType_t t; ncclRedOp_t o;
  if (!to_nccl(dtype, &t) || !to_op(op, &o)) { sl_set_last_error("comm: dtype/op"); return SL_ERR_UNSUPPORTED; }
  return check(rccl().all_reduce(send, recv, (size_t)count, t, o, as_comm(comm)->comm, (hipStream_t)stream),
               "ncclAllReduce");
}

// recv (count) <- the rank's block of the sum of send (count * size)
SL_API int sl_comm_reduce_scatter(void* comm, const void* send, void* recv, int64_t count, int dtype, int op,
                                  void* stream) {
  if (as_comm(comm)->ar) { sl_set_last_error("comm: a callback communicator only all-reduces"); return SL_ERR_UNSUPPORTED; }
  ncclDataType_t t; ncclRedOp_t o;
  if (!to_nccl(dtype, &t) || !to_op(op, &o)) { sl_set_last_error("comm: dtype/op"); return SL_ERR_UNSUPPORTED; }
  return check(rccl().reduce_scatter(send, recv, (size_t)count, t, o, as_comm(comm)->comm, (hipStream_t)stream),
               "ncclReduceScatter");
}

// recv (count * size) <- concatenation of every rank's send (count)
SL_API int sl_comm_all_gather(void* comm, const void* send, void* recv, int64_t count, int dtype, void* stream) {
  if (as_comm(comm)->ar) { sl_set_last_error("comm: a callback communicator only all-reduces"); return SL_ERR_UNSUPPORTED; }
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) { sl_set_last_error("comm: dtype"); return SL_ERR_UNSUPPORTED; }
  return check(rccl().all_gather(send, recv, (size_t)count, t, as_comm(comm)->comm, (hipStream_t)stream),
               "ncclAllGather");
}

SL_API int sl_comm_broadcast(void* comm, const void* send, void* recv, int64_t count, int dtype, int root,
                             void* stream) {
  if (as_comm(comm)->ar) { sl_set_last_error("comm: a callback communicator only all-reduces"); return SL_ERR_UNSUPPORTED; }
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) { sl_set_last_error("comm: dtype"); return SL_ERR_UNSUPPORTED; }
  return check(rccl().broadcast(send, recv, (size_t)count, t, root, as_comm(comm)->comm, (hipStream_t)stream),
               "ncclBroadcast");
}

// All-to-all(v) as grouped point-to-point: send_counts[q] elements from
// send + send_offs[q] go to rank q, recv_counts[q] from rank q land at
// recv + recv_offs[q] (host arrays of length size).  Every xGMI link carries
// its own pair concurrently.
SL_API int sl_comm_all_to_all_v(void* comm, const void* send, const int64_t* send_counts, const int64_t* send_offs,
                                void* recv, const int64_t* recv_counts, const int64_t* recv_offs, int dtype,
                                void* stream) {
  if (as_comm(comm)->ar) { sl_set_last_error("comm: a callback communicator only all-reduces"); return SL_ERR_UNSUPPORTED; }
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) { sl_set_last_error("comm: dtype"); return SL_ERR_UNSUPPORTED; }
  SlComm* c = as_comm(comm);
  const size_t es = elem_size(dtype);
  hipStream_t s = (hipStream_t)stream;
  int rc = check(rccl().group_start(), "ncclGroupStart");
  if (rc != SL_OK) return rc;
  for (int q = 0; q < c->size && rc == SL_OK; ++q) {
    if (send_counts[q] > 0)
      rc = check(rccl().send((const char*)send + send_offs[q] * es, (size_t)send_counts[q], t, q, c->comm, s),
                 "ncclSend");
    if (rc == SL_OK && recv_counts[q] > 0)
      rc = check(rccl().recv((char*)recv + recv_offs[q] * es, (size_t)recv_counts[q], t, q, c->comm, s),
                 "ncclRecv");
  }
  const int rc2 = check(rccl().group_end(), "ncclGroupEnd");
  return rc != SL_OK ? rc : rc2;
}

SL_API int sl_comm_send(void* comm, const void* buf, int64_t count, int dtype, int peer, void* stream) {
  if (as_comm(comm)->ar) { sl_set_last_error("comm: a callback communicator only all-reduces"); return SL_ERR_UNSUPPORTED; }
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) { sl_set_last_error("comm: dtype"); return SL_ERR_UNSUPPORTED; }
  return check(rccl().send(buf, (size_t)count, t, peer, as_comm(comm)->comm, (hipStream_t)stream), "ncclSend");
}

SL_API int sl_comm_recv(void* comm, void* buf, int64_t count, int dtype, int peer, void* stream) {
  if (as_comm(comm)->ar) { sl_set_last_error("comm: a callback communicator only all-reduces"); return SL_ERR_UNSUPPORTED; }
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) { sl_set_last_error("comm: dtype"); return SL_ERR_UNSUPPORTED; }
  return check(rccl().recv(buf, (size_t)count, t, peer, as_comm(comm)->comm, (hipStream_t)stream), "ncclRecv");
}
