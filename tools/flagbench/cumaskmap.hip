// The CU-mask bit -> (XCD, SE, SH, CU) map of this MI355X: one stream per single-bit mask,
// a few workgroups each recording XCC_ID / HW_ID.  Prints "bit xcd se sh cu" lines.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void k_where(uint32_t* out) {
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  }
}
int main() {
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int ncu = pr.multiProcessorCount, nw = (ncu + 31) / 32;
  uint32_t* d;
  CK(hipMalloc(&d, 64 * 8));
  std::vector<uint32_t> h(128);
  (void)0;
  for (int i = 0; i < ncu; i += 8) {  // bits i .. i+7 (a lone bit leaves XCDs without a CU: ignored)
    std::vector<uint32_t> m(nw, 0);
    m[i / 32] = 0xFFu << (i % 32);
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
    hipLaunchKernelGGL(k_where, dim3(64), dim3(64), 0, s, d);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h.data(), d, 64 * 8, hipMemcpyDeviceToHost));
    printf("bits %3d-%3d:", i, i + 7);
    for (int x = 0; x < 8; ++x) {  // per XCD: the distinct (se, cu) its blocks ran on
      uint32_t seen[8];
      int ns = 0;
      for (int b = 0; b < 64; ++b)
        if ((h[2 * b + 1] & 0xF) == (uint32_t)x) {
          const uint32_t v = (((h[2 * b] >> 13) & 7) << 4) | ((h[2 * b] >> 8) & 0xF);
          bool dup = false;
          for (int q = 0; q < ns; ++q) dup = dup || seen[q] == v;
          if (!dup && ns < 8) seen[ns++] = v;
        }
      printf(" x%d:", x);
      for (int q = 0; q < ns; ++q) printf("%s%u.%u", q ? "," : "", seen[q] >> 4, seen[q] & 0xF);
    }
    printf("\n");
    CK(hipStreamDestroy(s));
  }
  return 0;
}
