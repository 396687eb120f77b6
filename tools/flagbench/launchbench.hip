// Host cost of one kernel launch call on this ROCm ("split launch call,
// dispatch and pickup"): the window linearization's launch takes ~4 us of host time per
// LM trial.  Variants, each followed by a spin on the kernel's completion word:
//   ggl      hipLaunchKernelGGL, a 1.6-KB by-value argument block (k_win_linearize<16>'s size)
//   ggl_s    hipLaunchKernelGGL, 64 B of arguments
//   module   hipModuleLaunchKernel on the hipFunction_t (hipGetFuncBySymbol, looked up once),
//            the argument block passed pre-packed (HIP_LAUNCH_PARAM_BUFFER_POINTER)
//   ext      hipExtLaunchKernel (function address + args array)
// 160 blocks x 256 threads, a ticket over the blocks, the last publishes the word.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x)                                                \
  do {                                                       \
    hipError_t e = (x);                                      \
    if (e != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      return 1;                                              \
    }                                                        \
  } while (0)

struct Big {
  double m[16][12];
  uint32_t* f;
  uint32_t* t;
  uint32_t seq;
};
struct Small {
  uint32_t* f;
  uint32_t* t;
  uint32_t seq;
};

template <class A>
__device__ __forceinline__ void body(const A& a, double v) {
  if (threadIdx.x == 0) {
    if (v == 12345.0) a.t[1] = 1;
    if (__hip_atomic_fetch_add(a.t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(a.t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.f, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
__global__ void k_big(Big a) { body(a, a.m[blockIdx.x % 16][threadIdx.x % 12]); }
__global__ void k_small(Small a) { body(a, 0.0); }

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint32_t *hf, *df, *t;
  CK(hipHostMalloc(&hf, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&df, hf, 0));
  CK(hipMalloc(&t, 64));
  CK(hipMemset(t, 0, 64));
  *hf = 0;
  hipFunction_t fb;
  CK(hipGetFuncBySymbol(&fb, reinterpret_cast<const void*>(k_big)));
  Big b;
  std::memset(&b, 0, sizeof(b));
  b.f = df;
  b.t = t;
  Small s{df, t, 0};
  uint32_t seq = 0;
  const int N = 3000;
  const char* names[4] = {"ggl (1.6 KB args)", "ggl_s (24 B args)", "module + packed args", "hipExtLaunchKernel"};
  for (int rep = 0; rep < 2; ++rep)
    for (int v = 0; v < 4; ++v) {
      std::vector<double> call, rt;
      for (int i = 0; i < N + 200; ++i) {
        ++seq;
        b.seq = seq;
        s.seq = seq;
        const double a0 = now();
        if (v == 0) {
          hipLaunchKernelGGL(k_big, dim3(160), dim3(256), 0, st, b);
        } else if (v == 1) {
          hipLaunchKernelGGL(k_small, dim3(160), dim3(256), 0, st, s);
        } else if (v == 2) {
          size_t sz = sizeof(b);
          void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &b, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
          CK(hipModuleLaunchKernel(fb, 160, 1, 1, 256, 1, 1, 0, st, nullptr, cfg));
        } else {
          void* args[] = {&b};
          CK(hipExtLaunchKernel(reinterpret_cast<const void*>(k_big), dim3(160), dim3(256), args, 0, st, nullptr,
                                nullptr, 0));
        }
        const double a1 = now();
        while (*(volatile uint32_t*)hf != seq) {
        }
        const double a2 = now();
        if (i >= 200) {
          call.push_back(a1 - a0);
          rt.push_back(a2 - a0);
        }
      }
      std::sort(call.begin(), call.end());
      std::sort(rt.begin(), rt.end());
      printf("%-24s call p50 %.2f us p90 %.2f | launch->word p50 %.2f us p90 %.2f\n", names[v], call[N / 2] * 1e6,
             call[N * 9 / 10] * 1e6, rt[N / 2] * 1e6, rt[N * 9 / 10] * 1e6);
    }
  return 0;
}
