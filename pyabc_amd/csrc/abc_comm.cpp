// Multi-GPU collectives behind the C ABI (include/abcgpu.h, "multi-GPU
// collectives"): thin, stream-ordered wrappers over RCCL, which is opened
// with dlopen on first use so that libabcgpu.so loads on hosts without it.
// One process per GPU; the transport is xGMI between the GPUs of a node.
#include <cstring>
#include <dlfcn.h>
#include <mutex>
#include <rccl/rccl.h>
#include "abc_common.h"

namespace {

struct Rccl {
  bool ok = false;
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllGather) allgather = nullptr;
  decltype(&ncclAllReduce) allreduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclGetErrorString) errstr = nullptr;
  char why[256] = "";
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      snprintf(r.why, sizeof r.why, "dlopen librccl.so.1: %s", dlerror());
      return;
    }
#define ABC_SYM(field, name)                                              \
    r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, name));        \
    if (!r.field) { snprintf(r.why, sizeof r.why, "dlsym %s", name); return; }
    ABC_SYM(get_id, "ncclGetUniqueId")
    ABC_SYM(init, "ncclCommInitRank")
    ABC_SYM(destroy, "ncclCommDestroy")
    ABC_SYM(allgather, "ncclAllGather")
    ABC_SYM(allreduce, "ncclAllReduce")
    ABC_SYM(broadcast, "ncclBroadcast")
    ABC_SYM(errstr, "ncclGetErrorString")
#undef ABC_SYM
    r.ok = true;
  });
  return r;
}

#define ABC_RCCL_LOADED()                                                        \
  Rccl& R = rccl();                                                              \
  if (!R.ok) return abc::set_error(ABC_ERR_COMM, "RCCL unavailable: %s", R.why)
#define ABC_RCCL(call, what)                                                     \
  do {                                                                           \
    const ncclResult_t e_ = (call);                                              \
    if (e_ != ncclSuccess)                                                       \
      return abc::set_error(ABC_ERR_COMM, "%s: %s", what, R.errstr(e_));         \
  } while (0)

}  // namespace

extern "C" int abc_comm_unique_id(void* id) {
  ABC_CHECK_ARG(id != nullptr, "comm_unique_id: null id");
  ABC_RCCL_LOADED();
  ncclUniqueId u;
  ABC_RCCL(R.get_id(&u), "ncclGetUniqueId");
  std::memcpy(id, &u, sizeof u);
  return ABC_OK;
}

extern "C" int abc_comm_init(void** comm, int nranks, int rank, const void* id) {
  ABC_CHECK_ARG(comm && id, "comm_init: null pointer");
  ABC_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "comm_init: bad rank %d of %d",
                rank, nranks);
  ABC_RCCL_LOADED();
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  ncclComm_t c = nullptr;
  ABC_RCCL(R.init(&c, nranks, u, rank), "ncclCommInitRank");
  *comm = c;
  return ABC_OK;
}

extern "C" int abc_comm_destroy(void* comm) {
  if (comm == nullptr) return ABC_OK;
  ABC_RCCL_LOADED();
  ABC_RCCL(R.destroy(static_cast<ncclComm_t>(comm)), "ncclCommDestroy");
  return ABC_OK;
}

extern "C" int abc_comm_allgather(void* comm, const void* send, void* recv, size_t bytes,
                                  void* stream) {
  ABC_CHECK_ARG(comm && (bytes == 0 || (send && recv)), "comm_allgather: null pointer");
  ABC_RCCL_LOADED();
  ABC_RCCL(R.allgather(send, recv, bytes, ncclUint8, static_cast<ncclComm_t>(comm),
                       abc::as_stream(stream)),
           "ncclAllGather");
  return ABC_OK;
}

extern "C" int abc_comm_allreduce(void* comm, const void* send, void* recv, size_t count,
                                  int dtype, int op, void* stream) {
  ABC_CHECK_ARG(comm && (count == 0 || (send && recv)), "comm_allreduce: null pointer");
  ABC_CHECK_ARG(dtype == ABC_COMM_F64 || dtype == ABC_COMM_I64, "comm_allreduce: dtype %d",
                dtype);
  ABC_CHECK_ARG(op >= ABC_COMM_SUM && op <= ABC_COMM_MIN, "comm_allreduce: op %d", op);
  ABC_RCCL_LOADED();
  const ncclDataType_t t = dtype == ABC_COMM_F64 ? ncclFloat64 : ncclInt64;
  const ncclRedOp_t o = op == ABC_COMM_SUM ? ncclSum : (op == ABC_COMM_MAX ? ncclMax : ncclMin);
  ABC_RCCL(R.allreduce(send, recv, count, t, o, static_cast<ncclComm_t>(comm),
                       abc::as_stream(stream)),
           "ncclAllReduce");
  return ABC_OK;
}

extern "C" int abc_comm_broadcast(void* comm, void* buf, size_t bytes, int root,
                                  void* stream) {
  ABC_CHECK_ARG(comm && (bytes == 0 || buf), "comm_broadcast: null pointer");
  ABC_RCCL_LOADED();
  ABC_RCCL(R.broadcast(buf, buf, bytes, ncclUint8, root, static_cast<ncclComm_t>(comm),
                       abc::as_stream(stream)),
           "ncclBroadcast");
  return ABC_OK;
}
