// Data-parallel gradient exchange on RCCL, called on the caller's HIP streams
// (dopamine_amd/parallel.py, BASELINE config 4).
//
// The reference has no multi-GPU path: its _train_op (dqn_agent.py:432) applies one
// replica's gradient.  North-star config 4 runs one learner + one 1M buffer per GPU and
// averages the gradients over xGMI each step.  torch.distributed's ProcessGroupNCCL puts
// every collective on an internal stream of its own (fork from the caller's stream, join
// back, plus a watchdog event per work item): inside a captured HIP graph each of those
// is a cross-queue edge.  Here the learner owns the communicators and issues
// ncclAllReduce / ncclReduceScatter / ncclAllGather directly on the stream it chooses --
// the fc bucket on its comm stream, the conv bucket on the main stream -- so a captured
// step has exactly one fork and one join.  torch.distributed stays the launcher and the
// bootstrap (rank 0's ncclUniqueId is broadcast over the process group).
//
// RCCL is opened with dlopen on first use, so the library loads (and its exports can be
// checked) on a host without a GPU or RCCL.
#include <dlfcn.h>
#include <rccl/rccl.h>   // types, enums and prototypes only: the library itself is dlopened

#include <cstring>
#include <mutex>

#include "common.h"

static_assert(DQ_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "ncclUniqueId size changed");
static_assert(sizeof(ncclUniqueId) == DQ_COMM_ID_BYTES, "ncclUniqueId layout changed");

namespace dq {
namespace {

// the entry points used here, typed by rccl.h's own declarations
struct Rccl {
  decltype(&ncclGetUniqueId) GetUniqueId;
  decltype(&ncclCommInitRank) CommInitRank;
  decltype(&ncclCommDestroy) CommDestroy;
  decltype(&ncclAllReduce) AllReduce;
  decltype(&ncclReduceScatter) ReduceScatter;
  decltype(&ncclAllGather) AllGather;
  decltype(&ncclGetErrorString) GetErrorString;
  decltype(&ncclGetVersion) GetVersion;
};

Rccl g_rccl;
std::string g_open_error;

bool open_rccl() {
  static std::once_flag once;
  static bool ok = false;
  std::call_once(once, [] {
    void* h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      g_open_error = std::string("cannot open librccl.so.1: ") + (e ? e : "?");
      return;
    }
    auto sym = [&](const char* n) { return dlsym(h, n); };
#define DQ_SYM(field, name)                                        \
  g_rccl.field = reinterpret_cast<decltype(g_rccl.field)>(sym(name)); \
  if (!g_rccl.field) {                                             \
    g_open_error = std::string("librccl.so.1 lacks ") + name;      \
    return;                                                        \
  }
    DQ_SYM(GetUniqueId, "ncclGetUniqueId")
    DQ_SYM(CommInitRank, "ncclCommInitRank")
    DQ_SYM(CommDestroy, "ncclCommDestroy")
    DQ_SYM(AllReduce, "ncclAllReduce")
    DQ_SYM(ReduceScatter, "ncclReduceScatter")
    DQ_SYM(AllGather, "ncclAllGather")
    DQ_SYM(GetErrorString, "ncclGetErrorString")
    DQ_SYM(GetVersion, "ncclGetVersion")
#undef DQ_SYM
    int v = 0;
    if (g_rccl.GetVersion(&v) != ncclSuccess || v / 100 != NCCL_VERSION_CODE / 100) {
      g_open_error = "librccl.so.1 version " + std::to_string(v) + " differs from rccl.h's " +
                     std::to_string(NCCL_VERSION_CODE) + " (major.minor)";
      return;
    }
    ok = true;
  });
  if (!ok) set_error(g_open_error);
  return ok;
}

int nccl_status(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return DQ_OK;
  set_error(std::string(what) + ": " + g_rccl.GetErrorString(r));
  return DQ_E_HIP;
}

}  // namespace
}  // namespace dq

struct dq_comm {
  ncclComm_t comm;
  int32_t nranks, rank, device;
};

using namespace dq;

extern "C" {

int dq_comm_unique_id(uint8_t* id_out) {
  DQ_CHECK_ARG(id_out, "dq_comm_unique_id: id_out is NULL");
  if (!open_rccl()) return DQ_E_HIP;
  ncclUniqueId id;
  int rc = nccl_status(g_rccl.GetUniqueId(&id), "ncclGetUniqueId");
  if (rc) return rc;
  std::memcpy(id_out, id.internal, DQ_COMM_ID_BYTES);
  return DQ_OK;
}

int dq_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device,
                   dq_comm** out) {
  DQ_CHECK_ARG(id && out, "dq_comm_create: NULL argument");
  DQ_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "dq_comm_create: bad rank / nranks");
  if (!open_rccl()) return DQ_E_HIP;
  DQ_CHECK_HIP(hipSetDevice(device));
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, DQ_COMM_ID_BYTES);
  ncclComm_t c = nullptr;
  int rc = nccl_status(g_rccl.CommInitRank(&c, nranks, uid, rank), "ncclCommInitRank");
  if (rc) return rc;
  *out = new dq_comm{c, nranks, rank, device};
  return DQ_OK;
}

int dq_comm_destroy(dq_comm* c) {
  if (!c) return DQ_OK;
  int rc = nccl_status(g_rccl.CommDestroy(c->comm), "ncclCommDestroy");
  delete c;
  return rc;
}

int dq_comm_allreduce_mean(dq_comm* c, float* buf, int64_t n, void* stream) {
  DQ_CHECK_ARG(c && (buf || n == 0) && n >= 0, "dq_comm_allreduce_mean: bad argument");
  if (n == 0) return DQ_OK;
  return nccl_status(g_rccl.AllReduce(buf, buf, (size_t)n, ncclFloat32, ncclAvg, c->comm,
                                      (hipStream_t)stream), "ncclAllReduce");
}

int dq_comm_reduce_scatter_mean(dq_comm* c, float* buf, int64_t n_per_rank, void* stream) {
  DQ_CHECK_ARG(c && buf && n_per_rank > 0, "dq_comm_reduce_scatter_mean: bad argument");
  float* mine = buf + (int64_t)c->rank * n_per_rank;   // in place: recv = send + rank * count
  return nccl_status(g_rccl.ReduceScatter(buf, mine, (size_t)n_per_rank, ncclFloat32, ncclAvg,
                                          c->comm, (hipStream_t)stream), "ncclReduceScatter");
}

int dq_comm_all_gather(dq_comm* c, float* buf, int64_t n_per_rank, void* stream) {
  DQ_CHECK_ARG(c && buf && n_per_rank > 0, "dq_comm_all_gather: bad argument");
  const float* mine = buf + (int64_t)c->rank * n_per_rank;   // in place
  return nccl_status(g_rccl.AllGather(mine, buf, (size_t)n_per_rank, ncclFloat32, c->comm,
                                      (hipStream_t)stream), "ncclAllGather");
}

int dq_comm_version(void) {
  if (!open_rccl()) return -1;
  int v = 0;
  return g_rccl.GetVersion(&v) == 0 ? v : -1;
}

}  // extern "C"
