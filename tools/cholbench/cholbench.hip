// cholbench.hip — how fast can ONE workgroup factor and solve the smoother's dense LM
// system on gfx950?  (VERDICT r4 "next round" 3b: a one-workgroup device LM step with an
// fp64-MFMA blocked Cholesky; round 2 measured only a scalar-LDS factor.)
// Standalone microbenchmark, not part of libfmx:
//   hipcc -O3 --offload-arch=gfx950 tools/cholbench/cholbench.hip -o tools/cholbench/cholbench
// One 256-thread workgroup holds the (D+1)-padded matrix in LDS (D <= 128: 132 KB),
// factors it right-looking in 16-column panels — the 16 x 16 diagonal block by one wave
// (column steps, no block barrier), the panel rows by one thread each (16-step forward
// substitution), the trailing lower triangle by v_mfma_f64_16x16x4f64 tiles (4 per
// 16-deep panel) spread over the four waves — then solves L y = g, L^T x = y in one
// wave with the right-hand side in registers (one dependent step per column).
// Reported per D: in-kernel time of the factor and of the two solves (s_memrealtime,
// 100 MHz), launch-to-completion time over back-to-back launches (HIP events), and the
// solution's error against a host Cholesky.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kMax = 128, kLd = kMax + 1, kThreads = 256;

__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(kThreads) void k_chol(const double* __restrict__ A, const double* __restrict__ g,
                                                   double* __restrict__ x, int D, unsigned long long* stamps) {
  extern __shared__ double L[];  // [kMax][kLd]
  __shared__ double s_rd[kMax];  // 1 / L_jj
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int Dp = (D + 15) & ~15;
  for (int e = tid; e < Dp * Dp; e += kThreads) {
    const int i = e / Dp, j = e % Dp;
    L[i * kLd + j] = (i < D && j < D) ? A[(size_t)i * D + j] : (i == j ? 1.0 : 0.0);
  }
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  for (int k0 = 0; k0 < Dp; k0 += 16) {
    if (w == 0) {  // the 16 x 16 diagonal block, column by column (lower part only)
      for (int j = 0; j < 16; ++j) {
        const int c = k0 + j;
        const double d = sqrt(L[c * kLd + c]);
        const double rd = 1.0 / d;
        wave_lds_sync();
        if (lane < 16 && lane > j) L[(k0 + lane) * kLd + c] *= rd;
        if (lane == j) {
          L[c * kLd + c] = d;
          s_rd[c] = rd;
        }
        wave_lds_sync();
        for (int e = lane; e < 256; e += 64) {
          const int i = e >> 4, m = e & 15;
          if (m > j && i >= m) L[(k0 + i) * kLd + k0 + m] -= L[(k0 + i) * kLd + c] * L[(k0 + m) * kLd + c];
        }
        wave_lds_sync();
      }
    }
    __syncthreads();
    for (int r = k0 + 16 + tid; r < Dp; r += kThreads) {  // panel rows: v = a L11^-T
      double v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = L[r * kLd + k0 + c];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        double s = v[j];
#pragma unroll
        for (int c = 0; c < j; ++c) s -= v[c] * L[(k0 + j) * kLd + k0 + c];
        v[j] = s * s_rd[k0 + j];
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) L[r * kLd + k0 + c] = v[c];
    }
    __syncthreads();
    const int T = (Dp - k0 - 16) / 16;  // trailing lower triangle: T (T + 1) / 2 tiles of 16 x 16
    const int ntiles = T * (T + 1) / 2;
    for (int t = w; t < ntiles; t += kThreads / 64) {
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= t) ++I;
      const int J = t - I * (I + 1) / 2;
      const int r0 = k0 + 16 + 16 * I, c0 = k0 + 16 + 16 * J;
      f64x4 acc = {0.0, 0.0, 0.0, 0.0};
      double a[4], b[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {  // A[i][k] = L[r0 + i][k], B[k][j] = L[c0 + j][k]
        const int k = k0 + 4 * kk + (lane >> 4);
        a[kk] = L[(r0 + (lane & 15)) * kLd + k];
        b[kk] = L[(c0 + (lane & 15)) * kLd + k];
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kk], b[kk], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) L[(r0 + (lane >> 4) + 4 * r) * kLd + c0 + (lane & 15)] -= acc[r];
    }
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
  if (w == 0) {  // L y = g, then L^T x = y; lane l holds entries l and l + 64
    double b0 = lane < D ? g[lane] : 0.0, b1 = lane + 64 < D ? g[lane + 64] : 0.0;
    for (int j = 0; j < Dp; ++j) {
      const double yj = __shfl(j < 64 ? b0 : b1, j & 63) * s_rd[j];
      if (lane == (j & 63)) {
        if (j < 64) b0 = yj;
        else b1 = yj;
      }
      if (lane > j) b0 -= L[lane * kLd + j] * yj;
      if (lane + 64 > j && lane + 64 < Dp) b1 -= L[(lane + 64) * kLd + j] * yj;
    }
    for (int j = Dp - 1; j >= 0; --j) {
      const double xj = __shfl(j < 64 ? b0 : b1, j & 63) * s_rd[j];
      if (lane == (j & 63)) {
        if (j < 64) b0 = xj;
        else b1 = xj;
      }
      if (lane < j) b0 -= L[j * kLd + lane] * xj;
      if (lane + 64 < j) b1 -= L[j * kLd + lane + 64] * xj;
    }
    if (lane < D) x[lane] = b0;
    if (lane + 64 < D) x[lane + 64] = b1;
  }
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {
    stamps[0] = t1 - t0;
    stamps[1] = t2 - t1;
    stamps[2] = c1 - c0;
  }
}


// Version 2 of the factor: the diagonal block's column step as ONE wave-synchronous
// pass (the rank-1 update from the unscaled column, scaled by 1 / L_jj, then the column
// scaled: every lane's loads precede its stores), the 16 x 16 inverse of the diagonal
// factor by 16 lanes (one column each), and the panel rows as MFMA tiles L21 = A21 X^T.
__global__ __launch_bounds__(kThreads) void k_chol2(const double* __restrict__ A, const double* __restrict__ g,
                                                    double* __restrict__ x, int D, unsigned long long* stamps) {
  extern __shared__ double L[];  // [kMax][kLd]
  __shared__ double s_rd[kMax];
  __shared__ double s_x[16][17];  // X = L11^-1 (lower)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int Dp = (D + 15) & ~15;
  for (int e = tid; e < Dp * Dp; e += kThreads) {
    const int i = e / Dp, j = e % Dp;
    L[i * kLd + j] = (i < D && j < D) ? A[(size_t)i * D + j] : (i == j ? 1.0 : 0.0);
  }
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  for (int k0 = 0; k0 < Dp; k0 += 16) {
    if (w == 0) {
      for (int j = 0; j < 16; ++j) {
        const int c = k0 + j;
        const double piv = L[c * kLd + c];
        const double rp = 1.0 / piv;
        double upd[4], lij = 0.0;
        int ii[4], mm[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = lane + 64 * q, i = e >> 4, m = e & 15;
          ii[q] = i;
          mm[q] = m;
          upd[q] = (m > j && i >= m) ? L[(k0 + i) * kLd + c] * L[(k0 + m) * kLd + c] : 0.0;
        }
        if (lane < 16 && lane > j) lij = L[(k0 + lane) * kLd + c];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (mm[q] > j && ii[q] >= mm[q]) L[(k0 + ii[q]) * kLd + k0 + mm[q]] -= upd[q] * rp;
        const double d = sqrt(piv), rd = 1.0 / d;
        if (lane < 16 && lane > j) L[(k0 + lane) * kLd + c] = lij * rd;
        if (lane == j) {
          L[c * kLd + c] = d;
          s_rd[c] = rd;
        }
        wave_lds_sync();
      }
      if (lane < 16) {  // column `lane` of X = L11^-1: forward substitution
        double xv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          double s = i == lane ? 1.0 : 0.0;
#pragma unroll
          for (int k = 0; k < i; ++k) s -= L[(k0 + i) * kLd + k0 + k] * xv[k];
          xv[i] = s * s_rd[k0 + i];
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) s_x[i][lane] = xv[i];
      }
    }
    __syncthreads();
    const int T = (Dp - k0 - 16) / 16;
    for (int t = w; t < T; t += kThreads / 64) {  // panel tile t: L21 rows r0.. = A21 X^T
      const int r0 = k0 + 16 + 16 * t;
      f64x4 acc = {0.0, 0.0, 0.0, 0.0};
      double a[4], b[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {  // A[i][k] = A21[r0 + i][k0 + k], B[k][j] = X[j][k]
        const int k = 4 * kk + (lane >> 4);
        a[kk] = L[(r0 + (lane & 15)) * kLd + k0 + k];
        b[kk] = s_x[lane & 15][k];
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kk], b[kk], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) L[(r0 + (lane >> 4) + 4 * r) * kLd + k0 + (lane & 15)] = acc[r];
    }
    __syncthreads();
    const int ntiles = T * (T + 1) / 2;
    for (int t = w; t < ntiles; t += kThreads / 64) {
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= t) ++I;
      const int J = t - I * (I + 1) / 2;
      const int r0 = k0 + 16 + 16 * I, c0 = k0 + 16 + 16 * J;
      f64x4 acc = {0.0, 0.0, 0.0, 0.0};
      double a[4], b[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k = k0 + 4 * kk + (lane >> 4);
        a[kk] = L[(r0 + (lane & 15)) * kLd + k];
        b[kk] = L[(c0 + (lane & 15)) * kLd + k];
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kk], b[kk], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) L[(r0 + (lane >> 4) + 4 * r) * kLd + c0 + (lane & 15)] -= acc[r];
    }
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
  if (w == 0) {
    double b0 = lane < D ? g[lane] : 0.0, b1 = lane + 64 < D ? g[lane + 64] : 0.0;
    for (int j = 0; j < Dp; ++j) {
      const double yj = __shfl(j < 64 ? b0 : b1, j & 63) * s_rd[j];
      if (lane == (j & 63)) {
        if (j < 64) b0 = yj;
        else b1 = yj;
      }
      if (lane > j) b0 -= L[lane * kLd + j] * yj;
      if (lane + 64 > j && lane + 64 < Dp) b1 -= L[(lane + 64) * kLd + j] * yj;
    }
    for (int j = Dp - 1; j >= 0; --j) {
      const double xj = __shfl(j < 64 ? b0 : b1, j & 63) * s_rd[j];
      if (lane == (j & 63)) {
        if (j < 64) b0 = xj;
        else b1 = xj;
      }
      if (lane < j) b0 -= L[j * kLd + lane] * xj;
      if (lane + 64 < j) b1 -= L[j * kLd + lane + 64] * xj;
    }
    if (lane < D) x[lane] = b0;
    if (lane + 64 < D) x[lane + 64] = b1;
  }
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {
    stamps[0] = t1 - t0;
    stamps[1] = t2 - t1;
    stamps[2] = c1 - c0;
  }
}

static void host_solve(const std::vector<double>& A, const std::vector<double>& g, std::vector<double>& x, int D) {
  std::vector<double> L(A);
  for (int j = 0; j < D; ++j) {
    double s = L[j * D + j];
    for (int k = 0; k < j; ++k) s -= L[j * D + k] * L[j * D + k];
    L[j * D + j] = std::sqrt(s);
    for (int i = j + 1; i < D; ++i) {
      double t = L[i * D + j];
      for (int k = 0; k < j; ++k) t -= L[i * D + k] * L[j * D + k];
      L[i * D + j] = t / L[j * D + j];
    }
  }
  std::vector<double> y(D);
  for (int i = 0; i < D; ++i) {
    double s = g[i];
    for (int k = 0; k < i; ++k) s -= L[i * D + k] * y[k];
    y[i] = s / L[i * D + i];
  }
  x.assign(D, 0.0);
  for (int i = D - 1; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < D; ++k) s -= L[k * D + i] * x[k];
    x[i] = s / L[i * D + i];
  }
}

int main() {
  const size_t smem = (size_t)kMax * kLd * sizeof(double);
  CK(hipFuncSetAttribute((const void*)k_chol, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  CK(hipFuncSetAttribute((const void*)k_chol2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd;
  printf("version,D,factor_us,solves_us,launch_to_done_us,max_rel_err,factor_core_clocks,core_MHz\n");
  for (int ver = 1; ver <= 2; ++ver)
  for (int D : {72, 108, 126}) {
    auto kern = ver == 1 ? k_chol : k_chol2;
    std::vector<double> M((size_t)D * D), A((size_t)D * D, 0.0), g(D), xr, xg(D);
    for (auto& v : M) v = nd(rng);
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        double s = i == j ? D : 0.0;
        for (int k = 0; k < D; ++k) s += M[i * D + k] * M[j * D + k];
        A[i * D + j] = s;
      }
    for (auto& v : g) v = nd(rng);
    host_solve(A, g, xr, D);
    double *dA, *dg, *dx;
    unsigned long long* ds;
    CK(hipMalloc(&dA, A.size() * 8));
    CK(hipMalloc(&dg, D * 8));
    CK(hipMalloc(&dx, D * 8));
    CK(hipMalloc(&ds, 24));
    CK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dg, g.data(), D * 8, hipMemcpyHostToDevice));
    for (int it = 0; it < 20; ++it) hipLaunchKernelGGL(kern, dim3(1), dim3(kThreads), smem, 0, dA, dg, dx, D, ds);
    CK(hipDeviceSynchronize());
    // launch-to-completion, one at a time (what an LM step would pay per trial)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int N = 200;
    double tot = 0;
    for (int it = 0; it < N; ++it) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(kern, dim3(1), dim3(kThreads), smem, 0, dA, dg, dx, D, ds);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tot += ms;
    }
    unsigned long long st[3];
    CK(hipMemcpy(st, ds, 24, hipMemcpyDeviceToHost));
    CK(hipMemcpy(xg.data(), dx, D * 8, hipMemcpyDeviceToHost));
    double err = 0;
    for (int i = 0; i < D; ++i) err = std::fmax(err, std::fabs(xg[i] - xr[i]) / (std::fabs(xr[i]) + 1e-300));
    printf("v%d,%d,%.2f,%.2f,%.2f,%.2e,%llu,%.0f\n", ver, D, st[0] * 0.01, st[1] * 0.01, tot / N * 1e3, err, st[2],
           st[2] / (st[0] * 0.01));
    fflush(stdout);
    CK(hipFree(dA));
    CK(hipFree(dg));
    CK(hipFree(dx));
    CK(hipFree(ds));
  }
  return 0;
}
