// collective.hip -- the C-ABI all-gather of the date-sharded pass: one
// RCCL communicator per context, over xGMI on an 8 x MI355X node.  A host that is not Python
// (cgo / JNI / N-API) runs the sharded run_demo.py:31-67 pass with these calls around the shard
// kernels: csm_comm_unique_id on one rank, the 128 bytes handed to the others out of band,
// csm_allgather_init on every rank, then csm_allgather for the summary exchange (collective 1)
// and the per-date decile rows (collective 2) -- the same two all-gathers DateShardPipeline
// makes through torch.distributed.
//
// RCCL is opened at first use (dlopen of librccl.so.1, the soname torch's bundled RCCL also
// carries): libcsmom.so keeps loading on hosts without it, and a process that already holds an
// RCCL (torch's) shares that one instead of mapping a second.  Host code only: no kernels.
#include <dlfcn.h>
#include <string.h>

#include <rccl/rccl.h>

#include "csm_common.h"

namespace {

struct Rccl {
  bool tried = false, ok = false;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  char why[256] = {0};
};

Rccl& rccl() {
  static Rccl r;
  if (r.tried) return r;
  r.tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    snprintf(r.why, sizeof(r.why), "cannot open librccl: %s", dlerror());
    return r;
  }
  r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
  r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
  r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
  r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
  r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
  r.ok = r.get_unique_id && r.comm_init_rank && r.all_gather && r.comm_destroy && r.error_string;
  if (!r.ok) snprintf(r.why, sizeof(r.why), "librccl lacks an entry point");
  return r;
}

}  // namespace

#define RCCL_CHECK(ctx, call)                                                              \
  do {                                                                                     \
    ncclResult_t e_ = (call);                                                              \
    if (e_ != ncclSuccess)                                                                 \
      return set_err(ctx, CSM_E_RCCL, "%s: %s", #call, rccl().error_string(e_));           \
  } while (0)

extern "C" {

int csm_comm_unique_id(void* unique_id) {
  if (!unique_id) return CSM_E_INVAL;
  Rccl& r = rccl();
  if (!r.ok) return CSM_E_RCCL;
  ncclUniqueId id;
  if (r.get_unique_id(&id) != ncclSuccess) return CSM_E_RCCL;
  static_assert(sizeof(id) == CSM_UNIQUE_ID_BYTES, "ncclUniqueId is 128 bytes");
  memcpy(unique_id, &id, sizeof(id));
  return CSM_OK;
}

int csm_allgather_init(csm_ctx* ctx, const void* unique_id, int32_t rank, int32_t nranks) {
  int st = prep(ctx);
  if (st) return st;
  if (!unique_id || nranks < 1 || rank < 0 || rank >= nranks)
    return set_err(ctx, CSM_E_INVAL, "csm_allgather_init: bad arguments (rank=%d nranks=%d)", rank,
                   nranks);
  Rccl& r = rccl();
  if (!r.ok) return set_err(ctx, CSM_E_RCCL, "csm_allgather_init: %s", r.why);
  if (ctx->comm) {
    RCCL_CHECK(ctx, r.comm_destroy((ncclComm_t)ctx->comm));
    ctx->comm = nullptr;
  }
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  ncclComm_t comm = nullptr;
  RCCL_CHECK(ctx, r.comm_init_rank(&comm, nranks, id, rank));
  ctx->comm = comm;
  ctx->comm_rank = rank;
  ctx->comm_size = nranks;
  return CSM_OK;
}

int csm_allgather(csm_ctx* ctx, const void* send, void* recv, int64_t bytes) {
  int st = prep(ctx);
  if (st) return st;
  if (!ctx->comm) return set_err(ctx, CSM_E_INVAL, "csm_allgather: no communicator (csm_allgather_init)");
  if ((!send || !recv) && bytes > 0)
    return set_err(ctx, CSM_E_INVAL, "csm_allgather: null buffer");
  if (bytes < 0) return set_err(ctx, CSM_E_INVAL, "csm_allgather: bytes=%lld", (long long)bytes);
  if (bytes == 0) return CSM_OK;
  RCCL_CHECK(ctx, rccl().all_gather(send, recv, (size_t)bytes, ncclUint8, (ncclComm_t)ctx->comm,
                                    ctx->stream));
  return CSM_OK;
}

int csm_allgather_free(csm_ctx* ctx) {
  if (!ctx) return CSM_E_INVAL;
  if (ctx->comm) {
    (void)hipSetDevice(ctx->device);
    Rccl& r = rccl();
    ncclComm_t c = (ncclComm_t)ctx->comm;
    ctx->comm = nullptr;
    ctx->comm_size = 0;
    if (r.ok) RCCL_CHECK(ctx, r.comm_destroy(c));
  }
  return CSM_OK;
}

}  // extern "C"
