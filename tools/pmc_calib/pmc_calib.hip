// pmc_calib — calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE against known byte counts for
// the access patterns of the fmx kernels (MI355X_MICROARCH.md §HBM: only 16-B-per-lane
// streams are calibrated there; "calibrate on a known byte count in your own access
// pattern").  Buffers are 2 GiB (far beyond the 256-MiB Infinity Cache), every line is
// touched once per launch (random permutation), so each kernel's bytes come from HBM:
//   k_stream   : 16 B per lane, coalesced (the guide's reference pattern)
//   k_brick    : one lane per random 64-B line, reading 8 B at +0 and 8 B at +8..+40
//                (a k_match brick probe: key + one cell's [beg, end))
//   k_rec32    : one lane per random 32-B record, two 16-B loads (a k_match candidate)
//   k_rec32g   : 8 lanes per group reading 8 consecutive 32-B records (a group's
//                coalesced share of one cell's records)
//   k_wstream  : 16-B-per-lane coalesced stores (reference for WRITE_SIZE)
//   k_wrec32   : one lane per random 32-B record store (the match's scattered outputs)
// Prints one line per kernel: name, launches, known bytes per launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_stream(const float4* __restrict__ a, size_t n, float* out) {
  float s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;
}
__global__ void k_brick(const unsigned char* __restrict__ base, const uint32_t* __restrict__ perm, size_t m, float* out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= m) return;
  const unsigned char* line = base + (size_t)perm[i] * 64;
  const unsigned long long k = *reinterpret_cast<const unsigned long long*>(line);
  const int c = (int)(i & 7);
  const uint2 be = *reinterpret_cast<const uint2*>(line + 8 + 4 * (c & 6));
  if (k == 7ull && be.x == 3u) out[0] = 1.f;
}
__global__ void k_rec32(const double4* __restrict__ r, const uint32_t* __restrict__ perm, size_t m, float* out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= m) return;
  const double4 v = r[perm[i]];
  if (v.x + v.y + v.z + v.w == 12345.0) out[0] = 1.f;
}
__global__ void k_rec32g(const double4* __restrict__ r, const uint32_t* __restrict__ perm, size_t m, float* out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // group of 8 lanes per 256-B run
  if (i / 8 >= m) return;
  const double4 v = r[(size_t)perm[i / 8] * 8 + (i & 7)];
  if (v.x + v.y + v.z + v.w == 12345.0) out[0] = 1.f;
}
__global__ void k_wstream(float4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}
__global__ void k_wrec32(double4* __restrict__ r, const uint32_t* __restrict__ perm, size_t m) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= m) return;
  r[perm[i]] = make_double4(1.0, 2.0, 3.0, (double)i);
}

int main() {
  const size_t bytes = (size_t)2 << 30;
  void* buf;
  float* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 0, bytes));
  const size_t m = 4u << 20;  // 4M random items per launch
  std::mt19937_64 rng(7);
  auto perm_of = [&](size_t universe) {
    std::vector<uint32_t> p(m);
    std::uniform_int_distribution<uint64_t> d(0, universe - 1);
    // distinct items: stride the universe so no two picks share a 64-B line
    const size_t step = universe / m;
    for (size_t i = 0; i < m; ++i) p[i] = (uint32_t)(i * step + d(rng) % std::max<size_t>(step, 1));
    std::shuffle(p.begin(), p.end(), rng);
    return p;
  };
  uint32_t *d_pl, *d_pr, *d_pg;
  CK(hipMalloc(&d_pl, m * 4));
  CK(hipMalloc(&d_pr, m * 4));
  CK(hipMalloc(&d_pg, m * 4));
  auto pl = perm_of(bytes / 64), pr = perm_of(bytes / 32), pg = perm_of(bytes / 256);
  // records: keep at most one per 64-B line (even slots only), as a random gather would
  for (auto& x : pr) x &= ~1u;
  CK(hipMemcpy(d_pl, pl.data(), m * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pr, pr.data(), m * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pg, pg.data(), m * 4, hipMemcpyHostToDevice));
  const int reps = 3;
  const size_t nstream = (size_t)1 << 26;  // 1 GiB of float4
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const float4*)buf, nstream, out);
    hipLaunchKernelGGL(k_brick, dim3((m + 255) / 256), dim3(256), 0, 0, (const unsigned char*)buf, d_pl, m, out);
    hipLaunchKernelGGL(k_rec32, dim3((m + 255) / 256), dim3(256), 0, 0, (const double4*)buf, d_pr, m, out);
    hipLaunchKernelGGL(k_rec32g, dim3((8 * m + 255) / 256), dim3(256), 0, 0, (const double4*)buf, d_pg, m, out);
    hipLaunchKernelGGL(k_wstream, dim3(8192), dim3(256), 0, 0, (float4*)buf, nstream);
    hipLaunchKernelGGL(k_wrec32, dim3((m + 255) / 256), dim3(256), 0, 0, (double4*)buf, d_pr, m);
  }
  CK(hipDeviceSynchronize());
  printf("k_stream %d %zu\n", reps, nstream * 16);
  printf("k_brick %d %zu\n", reps, m * 64);
  printf("k_rec32 %d %zu\n", reps, m * 32);
  printf("k_rec32g %d %zu\n", reps, m * 256);
  printf("k_wstream %d %zu\n", reps, nstream * 16);
  printf("k_wrec32 %d %zu\n", reps, m * 32);
  return 0;
}
