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

// The all-reduced sums to the caller's pinned host buffer, then the completion word:
// one block behind the collective on the context stream, every element stored
// write-through at system scope (host_store), each wave drained, then one lane
// publishes seq.  The sharded path thus keeps the single-GPU path's flag wait
// (wait_flag, a few us after the data lands) instead of a hipMemcpyAsync D2H plus a
// hipStreamQuery spin (~20-50 us per round trip on this image).
constexpr int kPublishThreads = 256;
__global__ __launch_bounds__(kPublishThreads) void k_publish_sums(const double* __restrict__ src, double* dst,
                                                                  uint32_t n, uint32_t* flag, uint32_t seq) {
  for (uint32_t i = threadIdx.x; i < n; i += kPublishThreads) host_store(dst + i, src[i]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) publish_flag(flag, seq);
}

void comm_allreduce_publish(fmx_ctx* c, double* dev, size_t n, HBuf<double>& host) {
  if (n > 0xFFFFFFFFu) throw StatusError(FMX_E_INVAL, "all-reduce too large");
  comm_allreduce_sum(c, dev, n);
  host.ensure(n);
  const uint32_t seq = next_flag(c);
  hipLaunchKernelGGL(k_publish_sums, dim3(1), dim3(kPublishThreads), 0, c->stream, dev, host.d, (uint32_t)n,
                     c->h_flag.d, seq);
  FMX_HIP(hipGetLastError());
  wait_flag(c, c->h_flag.p, seq);
}

}  // namespace fmx
