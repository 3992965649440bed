// spg — native RCCL transport for the SPMD calls (spg_set_comm_rccl): the per-round allgathers of a
// sharded R1CSProof / SPARK proof / multi_evaluate go over RCCL on the context's own stream (xGMI between the GPUs
// of a node) instead of through a caller callback, so no host language runtime sits in the exchange.
//
// librccl.so.1 is opened at first use (dlopen): libspg itself does not link it, so callers that never shard do not
// load it. Every exchange is a few hundred bytes (the status word + 3 scalars of a round, or a W-entry tree level):
// host staging (page-locked) -> device send buffer -> ncclAllGather -> device receive buffer -> host staging, all
// on ctx->stream, then one bounded wait that polls ncclCommGetAsyncError, so a dead peer fails the call (the comm is
// aborted) instead of hanging it. The wait is SPG_RCCL_TIMEOUT_S seconds (default 600: a peer may legitimately
// spend minutes in a first-use table build before its next exchange). A timed-out or failed communicator is aborted
// and stays unusable: every later exchange on it fails at once, and the caller installs a new transport.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <stdlib.h>
#include <string>

#include "ctx.hpp"

namespace spg {

namespace {

struct RcclApi {
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllGather) allgather = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string err;
};

const RcclApi& api() {
  static const RcclApi a = [] {
    RcclApi r;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      r.err = std::string("dlopen(librccl.so.1): ") + dlerror();
      return r;
    }
    r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
    r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
    r.allgather = (decltype(r.allgather))dlsym(h, "ncclAllGather");
    r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
    r.abort = (decltype(r.abort))dlsym(h, "ncclCommAbort");
    r.async_error = (decltype(r.async_error))dlsym(h, "ncclCommGetAsyncError");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    if (!r.get_id || !r.init_rank || !r.allgather || !r.destroy || !r.abort || !r.async_error || !r.error_string)
      r.err = "librccl.so.1 lacks an nccl* entry point";
    return r;
  }();
  return a;
}

struct RcclComm {
  spg_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  int nranks = 1;
  uint8_t* d_buf = nullptr;  // send (cap) | receive (nranks x cap)
  uint8_t* h_buf = nullptr;  // page-locked staging of the same layout
  size_t cap = 0;
  bool dead = false;
};

// true once ctx->stream holds no queued work (bounded: an aborted collective should drain at once)
bool drain(hipStream_t s, int seconds) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipErrorNotReady) return e == hipSuccess;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(seconds)) return false;
  }
}

void rccl_free(void* p) {
  RcclComm* c = (RcclComm*)p;
  if (!c) return;
  if (c->comm) (c->dead ? api().abort : api().destroy)(c->comm);
  // the stream may still hold the aborted exchange's copies: the staging buffers outlive them (a dead communicator
  // whose stream never drains leaks them rather than freeing memory a copy may still touch)
  if (!c->dead || drain(c->ctx->stream, 10)) {
    if (c->d_buf) hipFree(c->d_buf);
    if (c->h_buf) hipHostFree(c->h_buf);
  }
  delete c;
}

int grow(RcclComm* c, size_t bytes) {
  if (bytes <= c->cap) return 0;
  size_t cap = 256;
  while (cap < bytes) cap <<= 1;
  if (c->d_buf) {
    hipStreamSynchronize(c->ctx->stream);
    hipFree(c->d_buf);
    hipHostFree(c->h_buf);
    c->d_buf = c->h_buf = nullptr;
    c->cap = 0;
  }
  const size_t total = cap * (size_t)(c->nranks + 1);
  if (hipMalloc(&c->d_buf, total) != hipSuccess) return -1;
  if (hipHostMalloc(&c->h_buf, total) != hipSuccess) return -1;
  c->cap = cap;
  return 0;
}

// spg_allgather_fn over RCCL (the transport comm.hpp frames each rank's status into)
int rccl_allgather(void* user, const void* send, size_t bytes, void* recv) {
  RcclComm* c = (RcclComm*)user;
  const RcclApi& a = api();
  if (c->dead) return -1;
  if (grow(c, bytes)) return -1;
  hipStream_t s = c->ctx->stream;
  memcpy(c->h_buf, send, bytes);
  uint8_t* d_recv = c->d_buf + c->cap;
  if ((hipMemcpyAsync)(c->d_buf, c->h_buf, bytes, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
  if (a.allgather(c->d_buf, d_recv, bytes, ncclUint8, c->comm, s) != ncclSuccess) return -1;
  if ((hipMemcpyAsync)(c->h_buf + c->cap, d_recv, bytes * (size_t)c->nranks, hipMemcpyDeviceToHost, s) != hipSuccess)
    return -1;
  // bounded wait: a peer that died leaves the collective pending forever
  static const long timeout_s = getenv("SPG_RCCL_TIMEOUT_S") ? std::max(1L, atol(getenv("SPG_RCCL_TIMEOUT_S"))) : 600L;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) return -1;
    ncclResult_t ae = ncclSuccess;
    if (a.async_error(c->comm, &ae) != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress) ||
        std::chrono::steady_clock::now() - t0 > std::chrono::seconds(timeout_s)) {
      c->dead = true;
      a.abort(c->comm);
      c->comm = nullptr;
      drain(s, 10);
      return -1;
    }
  }
  memcpy(recv, c->h_buf + c->cap, bytes * (size_t)c->nranks);
  return 0;
}

}  // namespace

}  // namespace spg

using namespace spg;

extern "C" int spg_rccl_unique_id(uint8_t id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  if (!id) return SPG_E_ARG;
  const RcclApi& a = api();
  if (!a.err.empty()) return SPG_E_ARG;
  ncclUniqueId u;
  if (a.get_id(&u) != ncclSuccess) return SPG_E_HIP;
  memcpy(id, &u, 128);
  return SPG_OK;
}

extern "C" int spg_set_comm_rccl(spg_ctx* ctx, const uint8_t id[128], int rank, int nranks) {
  if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return SPG_E_ARG;
  const RcclApi& a = api();
  if (!a.err.empty()) return set_err(ctx, SPG_E_ARG, "RCCL transport: " + a.err);
  SPG_HIP(ctx, hipSetDevice(ctx->device));
  RcclComm* c = new RcclComm();
  c->ctx = ctx;
  c->nranks = nranks;
  ncclUniqueId u;
  memcpy(&u, id, 128);
  const ncclResult_t r = a.init_rank(&c->comm, nranks, u, rank);  // collective: blocks until every rank joins
  if (r != ncclSuccess) {
    c->comm = nullptr;
    rccl_free(c);
    return set_err(ctx, SPG_E_HIP, std::string("ncclCommInitRank: ") + a.error_string(r));
  }
  if (ctx->comm_owned_free) ctx->comm_owned_free(ctx->comm_owned);
  ctx->comm_owned = c;
  ctx->comm_owned_free = rccl_free;
  ctx->rank = rank;
  ctx->nranks = nranks;
  ctx->allgather = rccl_allgather;
  ctx->comm_user = c;
  return SPG_OK;
}

extern "C" int spg_comm_allgather(spg_ctx* ctx, const void* send, size_t bytes, void* recv) {
  if (!ctx || (bytes && (!send || !recv))) return SPG_E_ARG;
  if (!ctx->allgather) {
    if (ctx->nranks != 1) return set_err(ctx, SPG_E_ARG, "no communicator set");
    if (bytes) memmove(recv, send, bytes);
    return SPG_OK;
  }
  if (ctx->allgather(ctx->comm_user, send, bytes, recv) != 0) return set_err(ctx, SPG_E_HIP, "allgather failed");
  return SPG_OK;
}
