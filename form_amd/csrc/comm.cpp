// comm.cpp — the exchange step of the sharded C5 path (SURVEY.md §8(e),
// BASELINE.json north_star "RCCL all-reduce of the 6x6 normal equations over xGMI").
//
// One rank per GPU; every rank holds the same voxel map and a contiguous shard of the
// queries, reduces its shard to the normal equations on the device, and the sums are
// all-reduced over RCCL ON THE CONTEXT STREAM, device buffer to device buffer, right
// behind the linearization kernel: no host hop between the kernel and the
// collective.  The messages are tiny (29 doubles for the single-pose system, 92 per
// pair otherwise): latency-bound, one ncclAllReduce (RCCL picks its low-latency
// protocol), never a bucketed ring.  RCCL is loaded on first use (dlopen: the one
// already in the process — torch's — if present, else ROCm's), so libfmx.so stays
// loadable where RCCL is absent and single-GPU users never touch it.
#include <dlfcn.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>

#include <rccl/rccl.h>

#include "fmx_device.hpp"
#include "fmx_internal.hpp"

namespace fmx {
namespace {

struct Rccl {
  void* so = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  // optional (every RCCL of this image has them): the bounded wait's error poll and abort
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  std::string err;
  bool load() {
    if (so) return true;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names) {  // an RCCL already in the process first (torch's)
      so = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
      if (so) break;
    }
    for (const char* n : names) {
      if (so) break;
      so = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    }
    if (!so) {
      err = std::string("RCCL not found: ") + dlerror();
      return false;
    }
    get_unique_id = reinterpret_cast<decltype(get_unique_id)>(dlsym(so, "ncclGetUniqueId"));
    comm_init_rank = reinterpret_cast<decltype(comm_init_rank)>(dlsym(so, "ncclCommInitRank"));
    all_reduce = reinterpret_cast<decltype(all_reduce)>(dlsym(so, "ncclAllReduce"));
    comm_destroy = reinterpret_cast<decltype(comm_destroy)>(dlsym(so, "ncclCommDestroy"));
    error_string = reinterpret_cast<decltype(error_string)>(dlsym(so, "ncclGetErrorString"));
    async_error = reinterpret_cast<decltype(async_error)>(dlsym(so, "ncclCommGetAsyncError"));
    comm_abort = reinterpret_cast<decltype(comm_abort)>(dlsym(so, "ncclCommAbort"));
    if (!get_unique_id || !comm_init_rank || !all_reduce || !comm_destroy || !error_string) {
      err = "RCCL library lacks the nccl* entry points";
      so = nullptr;
      return false;
    }
    return true;
  }
};
Rccl& rccl() {
  static Rccl r;
  return r;
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw StatusError(FMX_E_RCCL, std::string(what) + ": " + rccl().error_string(r));
}

}  // namespace

void comm_unique_id(uint8_t id[128]) {
  if (!rccl().load()) throw StatusError(FMX_E_RCCL, rccl().err);
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId u;
  check(rccl().get_unique_id(&u), "ncclGetUniqueId");
  std::memcpy(id, &u, sizeof(u));
}

void comm_init(fmx_ctx* c, const uint8_t id[128], int nranks, int rank) {
  if (!rccl().load()) throw StatusError(FMX_E_RCCL, rccl().err);
  if (nranks < 1 || rank < 0 || rank >= nranks) throw StatusError(FMX_E_INVAL, "bad rank / nranks");
  comm_destroy(c);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t comm = nullptr;
  check(rccl().comm_init_rank(&comm, nranks, u, rank), "ncclCommInitRank");
  c->comm = comm;
  c->comm_failed = false;
  c->comm_size = nranks;
  c->comm_rank = rank;
}

void comm_destroy(fmx_ctx* c) {
  if (!c->comm) return;
  (void)rccl().comm_destroy(static_cast<ncclComm_t>(c->comm));
  c->comm = nullptr;
  c->comm_size = 1;
  c->comm_rank = 0;
}

// In-place sum of n doubles in device memory over the communicator, on the context
// stream (ordered after the kernel that produced them).
void comm_allreduce_sum(fmx_ctx* c, double* dev, size_t n) {
  if (!c->comm) return;
  check(rccl().all_reduce(dev, dev, n, ncclFloat64, ncclSum, static_cast<ncclComm_t>(c->comm), c->stream),
        "ncclAllReduce");
}

namespace {

// The all-reduced sums to the caller's pinned host buffer, then the completion word:
// one block behind the collective on the context stream, every element stored
// write-through at system scope (host_store), each wave drained, then one lane
// publishes seq.  The sharded path thus keeps the single-GPU path's flag wait
// (wait_flag, a few us after the data lands) instead of a hipMemcpyAsync D2H plus a
// hipStreamQuery spin (~20-50 us per round trip on this image).
// hold (test switch FMX_TEST_WITHHOLD_FLAG only, else null): the block does not publish
// and instead stays on the stream, like a collective that never completes, until the
// host releases it (*hold != 0, set by the abort path) or 20 s have passed — so even
// the test kernel always exits.
constexpr int kPublishThreads = 256;
__global__ __launch_bounds__(kPublishThreads) void k_publish_sums(const double* __restrict__ src, double* dst,
                                                                  uint32_t n, uint32_t* flag, uint32_t seq,
                                                                  const uint32_t* hold) {
  if (hold) {
    if (threadIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
      while (__hip_atomic_load(hold, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u &&
             __builtin_amdgcn_s_memrealtime() - t0 < 2000000000ull)
        __builtin_amdgcn_s_sleep(127);
    }
    __syncthreads();
    return;  // withheld: no sums, no word
  }
  for (uint32_t i = threadIdx.x; i < n; i += kPublishThreads) host_store(dst + i, src[i]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) publish_flag(flag, seq);
}

// FMX_COMM_TIMEOUT_S (default 60): how long a rank waits for the all-reduced system.
double comm_timeout_s() {
  static const double v = [] {
    const char* e = std::getenv("FMX_COMM_TIMEOUT_S");
    const double t = e && *e ? std::atof(e) : 60.0;
    return t > 0 ? t : 60.0;
  }();
  return v;
}
bool withhold_flag() {  // test switch: see k_publish_sums
  static const bool v = std::getenv("FMX_TEST_WITHHOLD_FLAG") != nullptr;
  return v;
}

// The sharded path's wait for the completion word behind ncclAllReduce.  A rank whose
// peer died or never joined would otherwise spin forever (the stream stays busy inside
// the collective, so wait_flag's stream check never fires): here the wait polls
// ncclCommGetAsyncError and is bounded by FMX_COMM_TIMEOUT_S.  On either, the
// communicator is aborted (ncclCommAbort makes the RCCL kernels exit), the stream is
// drained, and the call fails with FMX_E_RCCL.  The context then refuses every sharded
// call (comm_check) until fmx_comm_init attaches a new communicator: its queries are a
// shard, so a rank-local system would silently stand in for the global one.
void comm_wait_flag(fmx_ctx* c, const volatile uint32_t* f, uint32_t seq, uint32_t* hold) {
  HostScope hs(1);
  ++c->host_waits;
  const auto t0 = std::chrono::steady_clock::now();
  const double limit = comm_timeout_s();
  std::string why;
  for (uint32_t spins = 1;; ++spins) {
    if (flag_reached(*f, seq)) {
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
      return;
    }
    if ((spins & 0x3FFF) != 0) continue;
    const hipError_t e = hipStreamQuery(c->stream);
    if (e == hipSuccess) {
      if (flag_reached(*f, seq)) continue;
      why = "the collective's stream completed without publishing the all-reduced system";
      break;
    }
    if (e != hipErrorNotReady) throw HipError(std::string("hipStreamQuery: ") + hipGetErrorString(e));
    ncclResult_t ae = ncclSuccess;
    if (rccl().async_error && rccl().async_error(static_cast<ncclComm_t>(c->comm), &ae) == ncclSuccess &&
        ae != ncclSuccess && ae != ncclInProgress) {
      why = std::string("RCCL asynchronous error: ") + rccl().error_string(ae);
      break;
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
      why = "no all-reduced system within FMX_COMM_TIMEOUT_S = " + std::to_string(limit) + " s";
      break;
    }
  }
  // fail instead of hang: release a withheld test kernel, abort the communicator (its
  // kernels exit; the abort may itself wait for the device work queued behind the
  // collective, hence the release first), drain the stream
  if (hold) __atomic_store_n(hold, 1u, __ATOMIC_RELEASE);
  ncclComm_t comm = static_cast<ncclComm_t>(c->comm);
  c->comm = nullptr;
  c->comm_size = 1;
  c->comm_rank = 0;
  c->comm_failed = true;
  if (rccl().comm_abort) (void)rccl().comm_abort(comm);
  else (void)rccl().comm_destroy(comm);
  (void)hipStreamSynchronize(c->stream);
  throw StatusError(FMX_E_RCCL, "all-reduce of the normal equations failed (communicator aborted): " + why);
}

}  // namespace

void comm_check(const fmx_ctx* c) {
  if (c->comm_failed)
    throw StatusError(FMX_E_RCCL, "the communicator was aborted by an earlier failure; sharded calls fail until "
                                  "fmx_comm_init attaches a new one");
}

void comm_allreduce_publish(fmx_ctx* c, double* dev, size_t n, HBuf<double>& host) {
  if (n > 0xFFFFFFFFu) throw StatusError(FMX_E_INVAL, "all-reduce too large");
  comm_allreduce_sum(c, dev, n);
  host.ensure(n);
  const uint32_t seq = next_flag(c);
  uint32_t* hold_h = nullptr;
  const uint32_t* hold_d = nullptr;
  if (withhold_flag() && c->comm) {  // test switch: the word is withheld, the stream held
    c->h_hold.ensure(1);
    c->h_hold.p[0] = 0;
    hold_h = c->h_hold.p;
    hold_d = c->h_hold.d;
  }
  hipLaunchKernelGGL(k_publish_sums, dim3(1), dim3(kPublishThreads), 0, c->stream, dev, host.d, (uint32_t)n,
                     c->h_flag.d, seq, hold_d);
  FMX_HIP(hipGetLastError());
  if (c->comm) comm_wait_flag(c, c->h_flag.p, seq, hold_h);
  else wait_flag(c, c->h_flag.p, seq);
}

}  // namespace fmx
