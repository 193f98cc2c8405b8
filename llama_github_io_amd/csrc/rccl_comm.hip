// Native RCCL transport of the row-sharded engine (the MI355X replacement of water/MRTask.java's reduce tree
// and water/RPC.java's fan-out for the tree builders).
//
// One communicator per process (one process per GPU), created from a unique id that rank 0 draws and the
// torch.distributed process group broadcasts (parallel/rccl.py). Collectives are enqueued on the caller's
// HIP stream, so a whole row-sharded tree (h2o_tree_dist: ~45 kernels + ~14 collectives) is ONE host call
// that never waits for the device; the same stream ordering makes the sequence hipGraph-capturable.
//
// RCCL is resolved at run time from the library torch already mapped (torch/lib/librccl.so): the process then
// holds a single RCCL instance, shared with ProcessGroupNCCL, and this library links no RCCL of its own.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "abi.h"

namespace {

struct Rccl {
  void* so = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclGetVersion) get_version = nullptr;
};

Rccl g_rccl;

template <typename F>
bool sym(void* so, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(so, name));
  return out != nullptr;
}

ncclDataType_t nccl_dtype(int dt) {
  switch (dt) {
    case 0: return ncclFloat32;
    case 1: return ncclFloat64;
    case 3: return ncclInt64;
    case 4: return ncclInt32;
    default: return ncclUint8;
  }
}

}  // namespace

extern "C" {

// Load RCCL from `path` (prefer the copy already mapped in the process). 0 = ok, -1 = dlopen failed,
// -2 = a symbol is missing.
int h2o_rccl_load(const char* path) {
  if (g_rccl.so) return 0;
  void* so = dlopen(path, RTLD_NOW | RTLD_NOLOAD);
  if (!so) so = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!so) return -1;
  Rccl r;
  r.so = so;
  bool ok = sym(so, "ncclGetUniqueId", r.get_unique_id) && sym(so, "ncclCommInitRank", r.comm_init_rank) &&
            sym(so, "ncclCommDestroy", r.comm_destroy) && sym(so, "ncclCommAbort", r.comm_abort) &&
            sym(so, "ncclAllReduce", r.all_reduce) && sym(so, "ncclReduceScatter", r.reduce_scatter) &&
            sym(so, "ncclAllGather", r.all_gather) && sym(so, "ncclGetErrorString", r.error_string) &&
            sym(so, "ncclGetVersion", r.get_version);
  if (!ok) return -2;
  g_rccl = r;
  return 0;
}

int h2o_rccl_version() {
  int v = 0;
  if (!g_rccl.so || g_rccl.get_version(&v) != ncclSuccess) return -1;
  return v;
}

const char* h2o_rccl_error(int rc) {
  if (!g_rccl.so) return "RCCL not loaded";
  return g_rccl.error_string((ncclResult_t)rc);
}

int h2o_rccl_unique_id(void* out /*NCCL_UNIQUE_ID_BYTES*/) {
  if (!g_rccl.so) return -1;
  ncclUniqueId id;
  const ncclResult_t rc = g_rccl.get_unique_id(&id);
  if (rc != ncclSuccess) return (int)rc;
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

int h2o_rccl_id_bytes() { return (int)sizeof(ncclUniqueId); }

// communicator of `nranks` on the CURRENT HIP device (the caller set it: torch.cuda.set_device)
int h2o_rccl_init(void** comm, int nranks, const void* uid, int rank) {
  if (!g_rccl.so) return -1;
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  ncclComm_t c = nullptr;
  const ncclResult_t rc = g_rccl.comm_init_rank(&c, nranks, id, rank);
  if (rc != ncclSuccess) return (int)rc;
  *comm = c;
  return 0;
}

int h2o_rccl_destroy(void* comm, int abort_) {
  if (!g_rccl.so || !comm) return 0;
  return (int)(abort_ ? g_rccl.comm_abort((ncclComm_t)comm) : g_rccl.comm_destroy((ncclComm_t)comm));
}

// The h2o_coll_fn of csrc/tree_kernels.hip: ctx = ncclComm_t. op 0 = all-reduce (sum, count elements),
// 1 = reduce-scatter (sum, count = elements received per rank), 2 = all-gather (count = elements sent per rank).
// Returns 0 or an ncclResult_t (+1000 so it cannot be read as a hipError_t).
int h2o_rccl_coll(void* ctx, int op, const void* send, void* recv, long long count, int dtype, hipStream_t s) {
  if (!g_rccl.so || !ctx) return 1999;
  if (count <= 0) return 0;
  const ncclComm_t comm = (ncclComm_t)ctx;
  const ncclDataType_t dt = nccl_dtype(dtype);
  ncclResult_t rc;
  switch (op) {
    case 0: rc = g_rccl.all_reduce(send, recv, (size_t)count, dt, ncclSum, comm, s); break;
    case 1: rc = g_rccl.reduce_scatter(send, recv, (size_t)count, dt, ncclSum, comm, s); break;
    case 2: rc = g_rccl.all_gather(send, recv, (size_t)count, dt, comm, s); break;
    default: return 1998;
  }
  return rc == ncclSuccess ? 0 : 1000 + (int)rc;
}

}  // extern "C"
