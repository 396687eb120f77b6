// Round-trip floor of "launch -> kernel publishes a completion word in pinned host
// memory -> host spins on it" (diagnostic for the window linearization's per-call
// overhead): small vs 3.5 KB kernel arguments, 1 block vs 200 blocks with a ticket.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <atomic>

struct Big { double m[36][12]; };
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ void publish(uint32_t* f, uint32_t s) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(f, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_small(uint32_t* f, uint32_t s, uint32_t* t, double* hg) {
  if (threadIdx.x == 0) {
    if (gridDim.x == 1) { publish(f, s); return; }
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(hg + blockIdx.x), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      publish(f, s);
    }
  }
}
__global__ void k_big(uint32_t* f, uint32_t s, uint32_t* t, double* hg, Big b) {
  if (threadIdx.x == 0) {
    if (b.m[blockIdx.x % 36][3] == 12345.0) hg[0] = 1;
    if (gridDim.x == 1) { publish(f, s); return; }
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(hg + blockIdx.x), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      publish(f, s);
    }
  }
}
// Persistent variant: every block polls a command word in pinned host memory
// (relaxed system-scope loads + s_sleep), does the same ticket + publish, loops;
// op word 1 = exit; a 2 s idle timeout always drains the grid.
__global__ void k_server(const uint32_t* cmd, uint32_t* f, uint32_t* t, double* hg, uint32_t last) {
  __shared__ uint32_t s_seq, s_op;
  for (;;) {
    if (threadIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t v, op = 0;
      for (;;) {
        v = __hip_atomic_load(cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v != last) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { op = 2; break; }
        __builtin_amdgcn_s_sleep(4);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      if (op == 0) op = __hip_atomic_load(cmd + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      s_seq = v;
      s_op = op;
    }
    __syncthreads();
    const uint32_t seq = s_seq, op = s_op;
    __syncthreads();
    if (op != 0) return;
    last = seq;
    if (threadIdx.x == 0) {
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(hg + blockIdx.x), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (__hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
        __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        publish(f, seq);
      }
    }
  }
}
int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint32_t *hf, *df, *t;
  double *hg, *dg;
  CK(hipHostMalloc(&hf, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&df, hf, 0));
  CK(hipHostMalloc(&hg, 1 << 16, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&dg, hg, 0));
  CK(hipMalloc(&t, 64));
  CK(hipMemset(t, 0, 64));
  *hf = 0;
  Big b;
  memset(&b, 0, sizeof(b));
  uint32_t seq = 0;
  for (int big = 0; big < 2; ++big)
    for (int grid : {1, 200}) {
      const int N = 2000;
      double tl = 0, t0 = 0;
      for (int i = 0; i < N + 100; ++i) {
        if (i == 100) t0 = now(), tl = 0;
        ++seq;
        double a = now();
        if (big) hipLaunchKernelGGL(k_big, dim3(grid), dim3(64), 0, st, df, seq, t, dg, b);
        else hipLaunchKernelGGL(k_small, dim3(grid), dim3(64), 0, st, df, seq, t, dg);
        tl += now() - a;
        while (*(volatile uint32_t*)hf != seq) {}
      }
      double tt = now() - t0;
      printf("%s args, grid %3d: round trip %.2f us (host launch call %.2f us)\n", big ? "3.5KB" : "small", grid,
             tt / N * 1e6, tl / N * 1e6);
    }
  uint32_t *hc, *dc;
  CK(hipHostMalloc(&hc, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&dc, hc, 0));
  for (int grid : {1, 200, 512}) {
    const uint32_t base = 100000u * (uint32_t)grid;
    hc[0] = base; hc[1] = 0;
    hipLaunchKernelGGL(k_server, dim3(grid), dim3(256), 0, st, dc, df, t, dg, base);
    const int N = 2000;
    double t0 = 0;
    uint32_t cs = base;
    for (int i = 0; i < N + 100; ++i) {
      if (i == 100) t0 = now();
      ++cs;
      std::atomic_thread_fence(std::memory_order_release);
      *(volatile uint32_t*)hc = cs;
      while (*(volatile uint32_t*)hf != cs) {}
    }
    double tt = now() - t0;
    hc[1] = 1;
    std::atomic_thread_fence(std::memory_order_release);
    *(volatile uint32_t*)hc = ++cs;
    CK(hipStreamSynchronize(st));
    printf("persistent server, grid %3d: round trip %.2f us\n", grid, tt / N * 1e6);
  }
  return 0;
}
