// Single-workgroup dense Cholesky + triangular solves of an n x n SPD system in LDS
// (diagnostic: is a device-side window LM step cheap enough?).  Times one solve
// inside the kernel (s_memrealtime, 100 MHz) and checks the residual on the host.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int NMAX = 128;
template <int T>
__global__ __launch_bounds__(T) void k_chol(const double* A, const double* g, double* x, int n, unsigned long long* t) {
  __shared__ double a[NMAX * (NMAX + 1)];
  __shared__ double y[NMAX];
  const int ld = n + 1, tid = threadIdx.x;
  for (int i = tid; i < n * n; i += T) a[(i / n) * ld + i % n] = A[i];
  for (int i = tid; i < n; i += T) y[i] = g[i];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  // right-looking, lower factor in the lower triangle: column k final after step k
  for (int k = 0; k < n; ++k) {
    const double dkk = sqrt(a[k * ld + k]);
    // scale column k below the diagonal, then rank-1 update of the trailing lower part
    for (int i = k + 1 + tid; i < n; i += T) a[i * ld + k] /= dkk;
    __syncthreads();
    if (tid == 0) a[k * ld + k] = dkk;
    const int m = n - k - 1;  // trailing size; elements (i, j), k < j <= i < n, linear index over rows
    const int tot = m * (m + 1) / 2;
    for (int e = tid; e < tot; e += T) {
      // row r (0-based in trailing) with r(r+1)/2 <= e
      int r = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
      while ((r + 1) * (r + 2) / 2 <= e) ++r;
      while (r * (r + 1) / 2 > e) --r;
      const int c = e - r * (r + 1) / 2;
      const int i = k + 1 + r, j = k + 1 + c;
      a[i * ld + j] -= a[i * ld + k] * a[j * ld + k];
    }
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  // forward L y = g: column sweep
  for (int k = 0; k < n; ++k) {
    if (tid == 0) y[k] /= a[k * ld + k];
    __syncthreads();
    for (int i = k + 1 + tid; i < n; i += T) y[i] -= a[i * ld + k] * y[k];
    __syncthreads();
  }
  // back L^T x = y
  for (int k = n - 1; k >= 0; --k) {
    if (tid == 0) y[k] /= a[k * ld + k];
    __syncthreads();
    for (int i = tid; i < k; i += T) y[i] -= a[k * ld + i] * y[k];
    __syncthreads();
  }
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
  for (int i = tid; i < n; i += T) x[i] = y[i];
  if (tid == 0) { t[0] = t1 - t0; t[1] = t2 - t1; }
}

// one wave, no barriers: lane l owns rows l, l+64 (wave-synchronous LDS)
__global__ __launch_bounds__(64) void k_chol_wave(const double* A, const double* g, double* x, int n, unsigned long long* t) {
  __shared__ double a[NMAX * (NMAX + 1)];
  __shared__ double y[NMAX];
  const int ld = n + 1, l = threadIdx.x;
  for (int i = l; i < n * n; i += 64) a[(i / n) * ld + i % n] = A[i];
  for (int i = l; i < n; i += 64) y[i] = g[i];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int k = 0; k < n; ++k) {
    const double dkk = sqrt(a[k * ld + k]);
    __builtin_amdgcn_wave_barrier();
    double lik[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = l + 64 * h;
      lik[h] = 0;
      if (i > k && i < n) { lik[h] = a[i * ld + k] / dkk; a[i * ld + k] = lik[h]; }
    }
    if (l == 0) a[k * ld + k] = dkk;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = l + 64 * h;
      if (i > k && i < n)
        for (int j = k + 1; j <= i; ++j) a[i * ld + j] -= lik[h] * a[j * ld + k];
    }
    __builtin_amdgcn_wave_barrier();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  for (int k = 0; k < n; ++k) {
    const double yk = y[k] / a[k * ld + k];
    __builtin_amdgcn_wave_barrier();
    if (l == 0) y[k] = yk;
    for (int i = k + 1 + l; i < n; i += 64) y[i] -= a[i * ld + k] * yk;
    __builtin_amdgcn_wave_barrier();
  }
  for (int k = n - 1; k >= 0; --k) {
    const double yk = y[k] / a[k * ld + k];
    __builtin_amdgcn_wave_barrier();
    if (l == 0) y[k] = yk;
    for (int i = l; i < k; i += 64) y[i] -= a[k * ld + i] * yk;
    __builtin_amdgcn_wave_barrier();
  }
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
  for (int i = l; i < n; i += 64) x[i] = y[i];
  if (l == 0) { t[0] = t1 - t0; t[1] = t2 - t1; }
}

int main() {
  for (int n : {72, 120}) {
    std::mt19937_64 rng(3);
    std::normal_distribution<double> nd;
    std::vector<double> A(n * n, 0.0), g(n), x(n);
    for (int r = 0; r < 2 * n; ++r) {
      std::vector<double> v(n);
      for (auto& q : v) q = nd(rng);
      for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) A[i * n + j] += v[i] * v[j];
    }
    for (auto& q : g) q = nd(rng);
    double *dA, *dg, *dx;
    unsigned long long* dt;
    CK(hipMalloc(&dA, n * n * 8)); CK(hipMalloc(&dg, n * 8)); CK(hipMalloc(&dx, n * 8)); CK(hipMalloc(&dt, 16));
    CK(hipMemcpy(dA, A.data(), n * n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dg, g.data(), n * 8, hipMemcpyHostToDevice));
    for (int variant = 0; variant < 4; ++variant) {
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      unsigned long long ts[2] = {0, 0}, best[2] = {~0ull, ~0ull};
      float ms_best = 1e9;
      for (int rep = 0; rep < 20; ++rep) {
        CK(hipEventRecord(e0));
        if (variant == 0) hipLaunchKernelGGL(k_chol<256>, dim3(1), dim3(256), 0, 0, dA, dg, dx, n, dt);
        else if (variant == 1) hipLaunchKernelGGL(k_chol<512>, dim3(1), dim3(512), 0, 0, dA, dg, dx, n, dt);
        else if (variant == 2) hipLaunchKernelGGL(k_chol<1024>, dim3(1), dim3(1024), 0, 0, dA, dg, dx, n, dt);
        else hipLaunchKernelGGL(k_chol_wave, dim3(1), dim3(64), 0, 0, dA, dg, dx, n, dt);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(ts, dt, 16, hipMemcpyDeviceToHost));
        if (ts[0] + ts[1] < best[0] + best[1]) { best[0] = ts[0]; best[1] = ts[1]; }
        if (ms < ms_best) ms_best = ms;
      }
      CK(hipMemcpy(x.data(), dx, n * 8, hipMemcpyDeviceToHost));
      double res = 0, gn = 0;
      for (int i = 0; i < n; ++i) { double s = 0; for (int j = 0; j < n; ++j) s += A[i * n + j] * x[j]; res = fmax(res, fabs(s - g[i])); gn = fmax(gn, fabs(g[i])); }
      const char* nm[4] = {"256 thr", "512 thr", "1024 thr", "1 wave"};
      printf("n=%d %-8s factor %.2f us, solves %.2f us, kernel (event) %.2f us, residual %.1e\n", n, nm[variant],
             best[0] * 0.01, best[1] * 0.01, ms_best * 1e3, res / gn);
    }
  }
  return 0;
}
