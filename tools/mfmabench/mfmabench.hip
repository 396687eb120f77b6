// Cycle costs of the window kernel's building blocks on one wave (diagnostic):
// dependent / independent v_mfma_f64_16x16x4_f64 chains, an LDS stage + 16 MFMAs.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ long long stamp() {
  long long t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}
#define CKE(x) (void)(x)
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void k_dep(double* out, long long* cyc, double x0) {
  f64x4 acc = {0, 0, 0, 0};
  double x = x0 + threadIdx.x;
  long long t0 = stamp();
  #pragma unroll
  for (int i = 0; i < 64; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, acc, 0, 0, 0);
  double r = acc[0] + acc[1] + acc[2] + acc[3];
  asm volatile("" :: "v"(r) : "memory");
  long long t1 = stamp();
  out[threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_ind(double* out, long long* cyc, double x0) {
  f64x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
  double x = x0 + threadIdx.x;
  long long t0 = stamp();
  #pragma unroll
  for (int i = 0; i < 16; ++i) {
    a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a3, 0, 0, 0);
  }
  double r = a0[0] + a1[1] + a2[2] + a3[3];
  asm volatile("" :: "v"(r) : "memory");
  long long t1 = stamp();
  out[threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_fma(double* out, long long* cyc, double x0) {
  double a[8];
  for (int i = 0; i < 8; ++i) a[i] = x0 + i + threadIdx.x;
  long long t0 = stamp();
  #pragma unroll
  for (int i = 0; i < 64; ++i)
    #pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = __builtin_fma(a[j], 1.0000001, 0.5);
  double s = 0; for (int i = 0; i < 8; ++i) s += a[i];
  asm volatile("" :: "v"(s) : "memory");
  long long t1 = stamp();
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
  double* out; long long* cyc; long long h;
  CKE(hipMalloc(&out, 4096)); CKE(hipMalloc(&cyc, 64));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_dep, dim3(1), dim3(64), 0, 0, out, cyc, 1.0); CKE(hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost));
    printf("64 dependent mfma_f64_16x16x4: %lld cycles (%.1f per MFMA)\n", h, h / 64.0);
    hipLaunchKernelGGL(k_ind, dim3(1), dim3(64), 0, 0, out, cyc, 1.0); CKE(hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost));
    printf("64 mfma_f64 in 4 independent chains: %lld cycles (%.1f per MFMA)\n", h, h / 64.0);
    hipLaunchKernelGGL(k_fma, dim3(1), dim3(64), 0, 0, out, cyc, 1.0); CKE(hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost));
    printf("512 v_fma_f64 (8 chains): %lld cycles (%.2f per instr)\n", h, h / 512.0);
  }
  return 0;
}
