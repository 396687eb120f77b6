// Round-trip floor of "launch -> kernel publishes a completion word in pinned host
// memory -> host spins on it" (diagnostic for the window linearization's per-call
// overhead): small vs 3.5 KB kernel arguments, 1 block vs 200 blocks with a ticket.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

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
  return 0;
}
