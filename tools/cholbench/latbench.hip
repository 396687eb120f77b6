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

__global__ __launch_bounds__(256) void k_lat(int which, double* out, unsigned long long* dt, int* gidx,
                                             unsigned* host_word) {
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
  } else if (which == 7) {  // dependent global loads (small table: cache-resident)
    for (int i = 0; i < N; ++i) idx = gidx[idx];
    x += idx;
  } else if (which == 8) {  // dependent agent-scope atomic loads (as the last-block tails read)
    for (int i = 0; i < N; ++i) idx = __hip_atomic_load(gidx + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x += idx;
  } else if (which == 9) {  // dependent agent-scope fetch-adds (tickets)
    for (int i = 0; i < N; ++i)
      idx = __hip_atomic_fetch_add(gidx + 256 + (idx & 255), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 255;
    x += idx;
  } else if (which == 10) {  // system-scope store to host memory, waited for (a completion word)
    for (int i = 0; i < N / 16; ++i) {
      __hip_atomic_store(host_word + tid, (unsigned)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  out[tid] = x;
  if (tid == 0) *dt = t1 - t0;
}


// The last-block pattern of k_match / k_win_linearize: every block stores one word per
// thread (agent scope, as the kernels' per-block counts), waits for it, takes a ticket;
// the last block then reads one word of every block with agent-scope loads (one round) —
// words written by blocks on the other XCDs, whose L2s are not this one's.  Reported:
// the last block's read round (us) and the ticket-to-end span of the last block.
__global__ __launch_bounds__(256) void k_tail(unsigned* words, unsigned* ticket, unsigned long long* dt, int rounds) {
  const int tid = threadIdx.x;
  __hip_atomic_store(words + (size_t)blockIdx.x * 256 + tid, blockIdx.x + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int s_last;
  if (tid == 0) s_last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned acc = 0;
  const unsigned R = (gridDim.x + 255) / 256;  // blocks per thread, as the match tail's R-runs
  for (int r = 0; r < rounds; ++r) {  // dependent rounds: thread t reads word 0 of blocks [R t, R t + R)
    unsigned part = 0;
    for (unsigned u = 0; u < R; ++u) {
      const unsigned b = tid * R + u;
      if (b < gridDim.x)
        part += __hip_atomic_load(words + (size_t)b * 256 + (acc & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    acc += part & 1;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {
    dt[0] = t1 - t0;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (acc == 0xFFFFFFFFu) words[0] = acc;
}

int main() {
  const char* names[] = {"lds_load_chain", "barrier", "lds_store_barrier_load_barrier", "f64_sqrt_chain",
                         "f64_recip_chain", "shfl_chain", "f64_fma_chain", "global_load_chain",
                         "agent_atomic_load_chain", "agent_fetch_add_chain", "host_store_acked"};
  double* dout;
  unsigned long long* ddt;
  int* gidx;
  unsigned* hw;
  if (hipMalloc(&dout, 256 * 8) != hipSuccess || hipMalloc(&ddt, 8) != hipSuccess) return 1;
  if (hipMalloc(&gidx, 512 * 4) != hipSuccess || hipHostMalloc(&hw, 256 * 4, hipHostMallocDefault) != hipSuccess) return 1;
  {
    int h[512];
    for (int i = 0; i < 512; ++i) h[i] = i < 256 ? (i + 1) & 255 : 0;
    if (hipMemcpy(gidx, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
  }
  printf("step,ns_per_step\n");
  for (int w = 0; w < 11; ++w) {
    unsigned long long dt = 0;
    for (int rep = 0; rep < 3; ++rep) {  // the last of three back-to-back launches
      hipLaunchKernelGGL(k_lat, dim3(1), dim3(256), 0, 0, w, dout, ddt, gidx, hw);
      if (hipDeviceSynchronize() != hipSuccess) return 1;
    }
    if (hipMemcpy(&dt, ddt, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("%s,%.2f\n", names[w], dt * 10.0 / (w == 10 ? N / 16 : N));
  }
  // last-block read rounds over words written by 1200 blocks (C4 match: ~1215 blocks)
  {
    unsigned *words, *ticket;
    unsigned long long* dt2;
    const int nb = 1200;
    if (hipMalloc(&words, (size_t)nb * 256 * 4) != hipSuccess || hipMalloc(&ticket, 4) != hipSuccess ||
        hipMalloc(&dt2, 8) != hipSuccess)
      return 1;
    if (hipMemset(ticket, 0, 4) != hipSuccess) return 1;
    for (int rounds : {1, 4}) {
      unsigned long long v = 0;
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_tail, dim3(nb), dim3(256), 0, 0, words, ticket, dt2, rounds);
        if (hipDeviceSynchronize() != hipSuccess) return 1;
      }
      if (hipMemcpy(&v, dt2, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      printf("last_block_%d_rounds_over_%d_blocks_us,%.2f\n", rounds, nb, v * 0.01);
    }
  }
  return 0;
}
