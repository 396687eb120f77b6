// latbench.hip — latency of the steps a one-workgroup serial chain is made of on gfx950
// (what bounds the device Cholesky of cholbench.hip and the last-block tails of the
// match and window kernels): a dependent LDS load chain, a workgroup barrier, a
// barrier after LDS stores, an fp64 sqrt / reciprocal chain, a cross-lane shuffle chain.
// Each kernel is one 256-thread workgroup looping N times; ns per step from the 100-MHz
// s_memrealtime counter.
//   hipcc -O3 --offload-arch=gfx950 tools/cholbench/latbench.hip -o tools/cholbench/latbench
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 4096;

__global__ __launch_bounds__(256) void k_lat(int which, double* out, unsigned long long* dt) {
  __shared__ int s_idx[256];
  __shared__ double s_v[256];
  const int tid = threadIdx.x;
  s_idx[tid] = (tid + 1) & 255;
  s_v[tid] = tid;
  __syncthreads();
  double x = 1.0 + tid;
  int idx = tid;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (which == 0) {  // dependent LDS loads
    for (int i = 0; i < N; ++i) idx = s_idx[idx];
    x += idx;
  } else if (which == 1) {  // bare barrier
    for (int i = 0; i < N; ++i) __syncthreads();
  } else if (which == 2) {  // LDS store, barrier, neighbour's value
    for (int i = 0; i < N; ++i) {
      s_v[tid] = x;
      __syncthreads();
      x = s_v[(tid + 1) & 255] + 1.0;
      __syncthreads();
    }
  } else if (which == 3) {  // fp64 sqrt chain
    for (int i = 0; i < N; ++i) x = sqrt(x + 1.0);
  } else if (which == 4) {  // fp64 reciprocal chain
    for (int i = 0; i < N; ++i) x = 1.0 / (x + 1.0);
  } else if (which == 5) {  // cross-lane shuffle chain
    for (int i = 0; i < N; ++i) x = __shfl(x, (threadIdx.x + 1) & 63) + 1.0;
  } else if (which == 6) {  // fp64 FMA chain
    for (int i = 0; i < N; ++i) x = fma(x, 0.999, 1e-3);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  out[tid] = x;
  if (tid == 0) *dt = t1 - t0;
}

int main() {
  const char* names[] = {"lds_load_chain", "barrier", "lds_store_barrier_load_barrier", "f64_sqrt_chain",
                         "f64_recip_chain", "shfl_chain", "f64_fma_chain"};
  double* dout;
  unsigned long long* ddt;
  if (hipMalloc(&dout, 256 * 8) != hipSuccess || hipMalloc(&ddt, 8) != hipSuccess) return 1;
  printf("step,ns_per_step\n");
  for (int w = 0; w < 7; ++w) {
    unsigned long long dt = 0;
    for (int rep = 0; rep < 3; ++rep) {  // the last of three back-to-back launches
      hipLaunchKernelGGL(k_lat, dim3(1), dim3(256), 0, 0, w, dout, ddt);
      if (hipDeviceSynchronize() != hipSuccess) return 1;
    }
    if (hipMemcpy(&dt, ddt, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("%s,%.2f\n", names[w], dt * 10.0 / N);
  }
  return 0;
}
