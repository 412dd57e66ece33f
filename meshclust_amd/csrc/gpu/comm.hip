// comm.hip -- the ranks' exchange for one clustering shared by several GPUs:
// an all-gather of equal byte blocks over RCCL (xGMI between the GPUs of a node), called from
// C++ by the host driver (meshclust_amd/csrc/host/cluster.cpp: one 1 KiB block per get_close
// step, the new centres once per mean-shift iteration).
//
// librccl is opened at run time (dlopen, RTLD_LOCAL), so libmcgpu has no link-time dependency
// on it and a process that already holds torch's RCCL keeps its own copy.  The blocks are host
// memory at the ABI (the driver needs them on the host: the bvec mirror and the step decision
// live there); they cross PCIe through pinned staging buffers on a stream of the rank's GPU.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>

#include "mcgpu.hpp"

namespace {

struct Rccl {
  bool ok = false;
  std::string why;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl &rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = nullptr;
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) {
      r.why = std::string("cannot open librccl: ") + dlerror();
      return;
    }
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
    r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
    r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
    r.abort = (decltype(r.abort))dlsym(h, "ncclCommAbort");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    r.ok = r.get_unique_id && r.init_rank && r.all_gather && r.destroy && r.abort && r.error_string;
    if (!r.ok) r.why = "librccl lacks the ncclGetUniqueId/CommInitRank/AllGather/CommDestroy entry points";
  });
  return r;
}

int rccl_fail(ncclResult_t e, const char *what) {
  mcg::set_error(std::string(what) + ": " + rccl().error_string(e));
  return MC_ERR_HIP;
}

}  // namespace

struct mc_comm {
  int device = 0, rank = 0, world = 1;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  void *d_send = nullptr, *d_recv = nullptr, *h_send = nullptr, *h_recv = nullptr;
  size_t cap = 0;  // bytes per block the staging buffers hold
  uint64_t calls = 0, bytes = 0;
};

extern "C" {

int mc_comm_unique_id(uint8_t *id) {
  const Rccl &r = rccl();
  if (!r.ok) {
    mcg::set_error(r.why);
    return MC_ERR_UNSUPPORTED;
  }
  if (!id) return MC_ERR_ARG;
  ncclUniqueId u;
  ncclResult_t e = r.get_unique_id(&u);
  if (e != ncclSuccess) return rccl_fail(e, "ncclGetUniqueId");
  memcpy(id, &u, sizeof u);
  return MC_OK;
}

int mc_comm_create(int device, int rank, int world, const uint8_t *id, mc_comm **out) {
  const Rccl &r = rccl();
  if (!r.ok) {
    mcg::set_error(r.why);
    return MC_ERR_UNSUPPORTED;
  }
  if (!id || !out || world < 1 || rank < 0 || rank >= world) return MC_ERR_ARG;
  MCG_CHECK(hipSetDevice(device));
  auto *c = new mc_comm();
  c->device = device;
  c->rank = rank;
  c->world = world;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  hipError_t he = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (he != hipSuccess) {
    delete c;
    return mcg::hip_fail(he, "hipStreamCreateWithFlags");
  }
  ncclResult_t e = r.init_rank(&c->comm, world, u, rank);  // blocks until every rank joined
  if (e != ncclSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return rccl_fail(e, "ncclCommInitRank");
  }
  *out = c;
  return MC_OK;
}

int mc_comm_allgather(mc_comm *c, const void *in, uint64_t bytes, void *out) {
  if (!c || (bytes && (!in || !out))) return MC_ERR_ARG;
  if (!c->comm) {
    mcg::set_error("RCCL communicator was aborted");
    return MC_ERR_STATE;
  }
  const Rccl &r = rccl();
  c->calls++;
  c->bytes += bytes * (uint64_t)c->world;
  if (bytes == 0) return MC_OK;
  MCG_CHECK(hipSetDevice(c->device));
  if (bytes > c->cap) {
    size_t cap = 4096;
    while (cap < bytes) cap *= 2;
    if (c->d_send) (void)hipFree(c->d_send);
    if (c->d_recv) (void)hipFree(c->d_recv);
    if (c->h_send) (void)hipHostFree(c->h_send);
    if (c->h_recv) (void)hipHostFree(c->h_recv);
    c->d_send = c->d_recv = c->h_send = c->h_recv = nullptr;
    c->cap = 0;
    MCG_CHECK(hipMalloc(&c->d_send, cap));
    MCG_CHECK(hipMalloc(&c->d_recv, cap * c->world));
    MCG_CHECK(hipHostMalloc(&c->h_send, cap, hipHostMallocDefault));
    MCG_CHECK(hipHostMalloc(&c->h_recv, cap * c->world, hipHostMallocDefault));
    c->cap = cap;
  }
  memcpy(c->h_send, in, bytes);
  MCG_CHECK(hipMemcpyAsync(c->d_send, c->h_send, bytes, hipMemcpyHostToDevice, c->stream));
  ncclResult_t e = r.all_gather(c->d_send, c->d_recv, bytes, ncclUint8, c->comm, c->stream);
  if (e != ncclSuccess) return rccl_fail(e, "ncclAllGather");
  MCG_CHECK(hipMemcpyAsync(c->h_recv, c->d_recv, bytes * c->world, hipMemcpyDeviceToHost, c->stream));
  // A rank that failed before this all-gather never joins it: wait with a deadline
  // (MC_COMM_TIMEOUT_S, default 300 s) and abort the communicator, so every waiting rank
  // returns an error instead of blocking forever.
  const double limit = getenv("MC_COMM_TIMEOUT_S") ? atof(getenv("MC_COMM_TIMEOUT_S")) : 300.0;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t it = 0;; it++) {
    const hipError_t q = hipStreamQuery(c->stream);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) return mcg::hip_fail(q, "all-gather stream");
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
      r.abort(c->comm);
      c->comm = nullptr;
      mcg::set_error("RCCL all-gather timed out (a rank did not join: MC_COMM_TIMEOUT_S)");
      return MC_ERR_HIP;
    }
    if (it > 2000) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  memcpy(out, c->h_recv, bytes * c->world);
  return MC_OK;
}

int mc_comm_stats(const mc_comm *c, uint64_t *calls, uint64_t *bytes) {
  if (!c) return MC_ERR_ARG;
  if (calls) *calls = c->calls;
  if (bytes) *bytes = c->bytes;
  return MC_OK;
}

int mc_comm_destroy(mc_comm *c, int abort) {
  if (!c) return MC_OK;
  (void)hipSetDevice(c->device);
  const Rccl &r = rccl();
  if (c->comm) (void)(abort ? r.abort(c->comm) : r.destroy(c->comm));
  if (c->d_send) (void)hipFree(c->d_send);
  if (c->d_recv) (void)hipFree(c->d_recv);
  if (c->h_send) (void)hipHostFree(c->h_send);
  if (c->h_recv) (void)hipHostFree(c->h_recv);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return MC_OK;
}

}  // extern "C"
