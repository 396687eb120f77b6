#include <chrono>
#include <cstdio>
#include <vector>
#include <random>
#include <cstring>
#include <cmath>
#include <algorithm>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
double T[4];
bool chol(std::vector<double>& A, const double* g, double* x, int n) {
  constexpr int B = 6;
  double* a = A.data();
  double t0 = now();
  double tp = 0;
  for (int kb = 0; kb < n; kb += B) {
    const int ke = std::min(n, kb + B);
    double tq = now();
    for (int k = kb; k < ke; ++k) {
      double* __restrict Uk = a + (size_t)k * n;
      const double s = Uk[k];
      if (!(s > 0)) return false;
      const double ukk = std::sqrt(s);
      Uk[k] = ukk;
      for (int m = k + 1; m < n; ++m) Uk[m] = Uk[m] / ukk;
      for (int i = k + 1; i < ke; ++i) {
        double* __restrict Ai = a + (size_t)i * n;
        const double uki = Uk[i];
        for (int m = i; m < n; ++m) Ai[m] -= uki * Uk[m];
      }
    }
    tp += now() - tq;
    const double* U[B];
    for (int t = 0; t < B; ++t) U[t] = a + (size_t)(kb + t) * n;
    for (int i = ke; i < n; ++i) {
      double* __restrict Ai = a + (size_t)i * n;
      double u[B];
      for (int t = 0; t < B; ++t) u[t] = U[t][i];
      for (int m = i; m < n; ++m) {
        double v = Ai[m];
        for (int t = 0; t < B; ++t) v -= u[t] * U[t][m];
        Ai[m] = v;
      }
    }
  }
  double t1 = now();
  std::vector<double> y(g, g + n);
  for (int k = 0; k < n; ++k) {
    const double* Uk = a + (size_t)k * n;
    y[k] = y[k] / Uk[k];
    const double yk = y[k];
    for (int m = k + 1; m < n; ++m) y[m] -= Uk[m] * yk;
  }
  double t2 = now();
  for (int i = n - 1; i >= 0; --i) {
    const double* Ui = a + (size_t)i * n;
    double s = y[i];
    for (int k = i + 1; k < n; ++k) s -= Ui[k] * x[k];
    x[i] = s / Ui[i];
  }
  double t3 = now();
  T[0] += tp; T[1] += t1 - t0 - tp; T[2] += t2 - t1; T[3] += t3 - t2;
  return true;
}
__attribute__((target("avx2,fma"))) bool chol2(std::vector<double>& A, const double* g, double* x, int n) {
  constexpr int B = 6;
  double* a = A.data();
  double t0 = now();
  double tp = 0;
  for (int kb = 0; kb < n; kb += B) {
    const int ke = std::min(n, kb + B);
    double tq = now();
    for (int k = kb; k < ke; ++k) {
      double* __restrict Uk = a + (size_t)k * n;
      const double s = Uk[k];
      if (!(s > 0)) return false;
      const double ukk = std::sqrt(s);
      Uk[k] = ukk;
      for (int m = k + 1; m < n; ++m) Uk[m] = Uk[m] / ukk;
      for (int i = k + 1; i < ke; ++i) {
        double* __restrict Ai = a + (size_t)i * n;
        const double uki = Uk[i];
        for (int m = i; m < n; ++m) Ai[m] = __builtin_fma(-uki, Uk[m], Ai[m]);
      }
    }
    tp += now() - tq;
    const double* U[B];
    for (int t = 0; t < B; ++t) U[t] = a + (size_t)(kb + t) * n;
    for (int i = ke; i < n; ++i) {
      double* __restrict Ai = a + (size_t)i * n;
      double u[B];
      for (int t = 0; t < B; ++t) u[t] = U[t][i];
      for (int m = i; m < n; ++m) {
        double v = Ai[m];
        for (int t = 0; t < B; ++t) v = __builtin_fma(-u[t], U[t][m], v);
        Ai[m] = v;
      }
    }
  }
  double t1 = now();
  std::vector<double> y(g, g + n);
  for (int k = 0; k < n; ++k) {
    const double* Uk = a + (size_t)k * n;
    y[k] = y[k] / Uk[k];
    const double yk = y[k];
    for (int m = k + 1; m < n; ++m) y[m] = __builtin_fma(-Uk[m], yk, y[m]);
  }
  double t2 = now();
  for (int i = n - 1; i >= 0; --i) {
    const double* Ui = a + (size_t)i * n;
    double s4[4] = {0, 0, 0, 0};
    int k = i + 1;
    for (; k + 4 <= n; k += 4)
      for (int l = 0; l < 4; ++l) s4[l] = __builtin_fma(Ui[k + l], x[k + l], s4[l]);
    double s = y[i] - ((s4[0] + s4[1]) + (s4[2] + s4[3]));
    for (; k < n; ++k) s = __builtin_fma(-Ui[k], x[k], s);
    x[i] = s / Ui[i];
  }
  double t3 = now();
  T[0] += tp; T[1] += t1 - t0 - tp; T[2] += t2 - t1; T[3] += t3 - t2;
  return true;
}
__attribute__((target("avx2,fma"))) bool chol3(std::vector<double>& A, const double* g, double* x, int n) {
  constexpr int B = 6;
  double* a = A.data();
  double t0 = now();
  double tp = 0;
  for (int kb = 0; kb < n; kb += B) {
    const int ke = std::min(n, kb + B);
    double tq = now();
    for (int k = kb; k < ke; ++k) {
      double* __restrict Uk = a + (size_t)k * n;
      const double s = Uk[k];
      if (!(s > 0)) return false;
      const double ukk = std::sqrt(s);
      Uk[k] = ukk;
      for (int m = k + 1; m < n; ++m) Uk[m] = Uk[m] / ukk;
      for (int i = k + 1; i < ke; ++i) {
        double* __restrict Ai = a + (size_t)i * n;
        const double uki = Uk[i];
        for (int m = i; m < n; ++m) Ai[m] = __builtin_fma(-uki, Uk[m], Ai[m]);
      }
    }
    tp += now() - tq;
    const double* U[B];
    for (int t = 0; t < B; ++t) U[t] = a + (size_t)(kb + t) * n;
    int i = ke;
    for (; i + 2 <= n; i += 2) {  // two rows per pass: each U load feeds both
      double* __restrict A0 = a + (size_t)i * n;
      double* __restrict A1 = A0 + n;
      double u0[B], u1[B];
      for (int t = 0; t < B; ++t) { u0[t] = U[t][i]; u1[t] = U[t][i + 1]; }
      // element (i, i) of row 0 alone; then both rows over m >= i + 1
      { double v = A0[i]; for (int t = 0; t < B; ++t) v = __builtin_fma(-u0[t], U[t][i], v); A0[i] = v; }
      typedef double v4 __attribute__((vector_size(32)));
      int m = i + 1;
      for (; m + 4 <= n; m += 4) {
        v4 x0, x1; __builtin_memcpy(&x0, A0 + m, 32); __builtin_memcpy(&x1, A1 + m, 32);
        for (int t = 0; t < B; ++t) {
          v4 uu; __builtin_memcpy(&uu, U[t] + m, 32);
          x0 = x0 - (v4){u0[t], u0[t], u0[t], u0[t]} * uu;
          x1 = x1 - (v4){u1[t], u1[t], u1[t], u1[t]} * uu;
        }
        __builtin_memcpy(A0 + m, &x0, 32); __builtin_memcpy(A1 + m, &x1, 32);
      }
      for (; m < n; ++m) {
        double v0 = A0[m], v1 = A1[m];
        for (int t = 0; t < B; ++t) { v0 = __builtin_fma(-u0[t], U[t][m], v0); v1 = __builtin_fma(-u1[t], U[t][m], v1); }
        A0[m] = v0; A1[m] = v1;
      }
    }
    for (; i < n; ++i) {
      double* __restrict Ai = a + (size_t)i * n;
      double u[B];
      for (int t = 0; t < B; ++t) u[t] = U[t][i];
      for (int m = i; m < n; ++m) {
        double v = Ai[m];
        for (int t = 0; t < B; ++t) v = __builtin_fma(-u[t], U[t][m], v);
        Ai[m] = v;
      }
    }
  }
  double t1 = now();
  std::vector<double> y(g, g + n);
  for (int k = 0; k < n; ++k) {
    const double* Uk = a + (size_t)k * n;
    y[k] = y[k] / Uk[k];
    const double yk = y[k];
    for (int m = k + 1; m < n; ++m) y[m] = __builtin_fma(-Uk[m], yk, y[m]);
  }
  double t2 = now();
  for (int i = n - 1; i >= 0; --i) {
    const double* Ui = a + (size_t)i * n;
    double s4[4] = {0, 0, 0, 0};
    int k = i + 1;
    for (; k + 4 <= n; k += 4)
      for (int l = 0; l < 4; ++l) s4[l] = __builtin_fma(Ui[k + l], x[k + l], s4[l]);
    double s = y[i] - ((s4[0] + s4[1]) + (s4[2] + s4[3]));
    for (; k < n; ++k) s = __builtin_fma(-Ui[k], x[k], s);
    x[i] = s / Ui[i];
  }
  double t3 = now();
  T[0] += tp; T[1] += t1 - t0 - tp; T[2] += t2 - t1; T[3] += t3 - t2;
  return true;
}
__attribute__((target("avx2,fma"))) bool chol4(std::vector<double>& A, const double* g, double* x, int n) {
  constexpr int B = 6;
  double* a = A.data();
  double t0 = now();
  double tp = 0;
  for (int kb = 0; kb < n; kb += B) {
    const int ke = std::min(n, kb + B);
    double tq = now();
    for (int k = kb; k < ke; ++k) {
      double* __restrict Uk = a + (size_t)k * n;
      const double s = Uk[k];
      if (!(s > 0)) return false;
      const double ukk = std::sqrt(s);
      Uk[k] = ukk;
      for (int m = k + 1; m < n; ++m) Uk[m] = Uk[m] / ukk;
      for (int i = k + 1; i < ke; ++i) {
        double* __restrict Ai = a + (size_t)i * n;
        const double uki = Uk[i];
        for (int m = i; m < n; ++m) Ai[m] = __builtin_fma(-uki, Uk[m], Ai[m]);
      }
    }
    tp += now() - tq;
    const double* U[B];
    for (int t = 0; t < B; ++t) U[t] = a + (size_t)(kb + t) * n;
    int i = ke;
    for (; i + 2 <= n; i += 2) {  // two rows per pass: each U load feeds both
      double* __restrict A0 = a + (size_t)i * n;
      double* __restrict A1 = A0 + n;
      double u0[B], u1[B];
      for (int t = 0; t < B; ++t) { u0[t] = U[t][i]; u1[t] = U[t][i + 1]; }
      // element (i, i) of row 0 alone; then both rows over m >= i + 1
      { double v = A0[i]; for (int t = 0; t < B; ++t) v = __builtin_fma(-u0[t], U[t][i], v); A0[i] = v; }
      int m = i + 1;
      for (; m < n; ++m) {
        double v0 = A0[m], v1 = A1[m];
        for (int t = 0; t < B; ++t) { v0 = __builtin_fma(-u0[t], U[t][m], v0); v1 = __builtin_fma(-u1[t], U[t][m], v1); }
        A0[m] = v0; A1[m] = v1;
      }
    }
    for (; i < n; ++i) {
      double* __restrict Ai = a + (size_t)i * n;
      double u[B];
      for (int t = 0; t < B; ++t) u[t] = U[t][i];
      for (int m = i; m < n; ++m) {
        double v = Ai[m];
        for (int t = 0; t < B; ++t) v = __builtin_fma(-u[t], U[t][m], v);
        Ai[m] = v;
      }
    }
  }
  double t1 = now();
  std::vector<double> y(g, g + n);
  for (int k = 0; k < n; ++k) {
    const double* Uk = a + (size_t)k * n;
    y[k] = y[k] / Uk[k];
    const double yk = y[k];
    for (int m = k + 1; m < n; ++m) y[m] = __builtin_fma(-Uk[m], yk, y[m]);
  }
  double t2 = now();
  for (int i = n - 1; i >= 0; --i) {
    const double* Ui = a + (size_t)i * n;
    double s4[4] = {0, 0, 0, 0};
    int k = i + 1;
    for (; k + 4 <= n; k += 4)
      for (int l = 0; l < 4; ++l) s4[l] = __builtin_fma(Ui[k + l], x[k + l], s4[l]);
    double s = y[i] - ((s4[0] + s4[1]) + (s4[2] + s4[3]));
    for (; k < n; ++k) s = __builtin_fma(-Ui[k], x[k], s);
    x[i] = s / Ui[i];
  }
  double t3 = now();
  T[0] += tp; T[1] += t1 - t0 - tp; T[2] += t2 - t1; T[3] += t3 - t2;
  return true;
}
int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 72;
  std::mt19937_64 rng(1); std::normal_distribution<double> nd;
  std::vector<double> A((size_t)n*n, 0.0), g(n), x(n);
  for (int r = 0; r < 2*n; ++r) { std::vector<double> a(n); for (auto& v : a) v = nd(rng); for (int i=0;i<n;++i) for (int j=0;j<n;++j) A[i*n+j]+=a[i]*a[j]; }
  for (auto& v : g) v = nd(rng);
  std::vector<double> B;
  int reps = 20000; double t0 = now();
  std::vector<double> x1 = x;
  for (int r = 0; r < reps; ++r) { B = A; chol(B, g.data(), x1.data(), n); }
  printf("n=%d total %.2f us: panel %.2f trailing %.2f fwd %.2f back %.2f\n", n, (now()-t0)/reps*1e6, T[0]/reps*1e6, T[1]/reps*1e6, T[2]/reps*1e6, T[3]/reps*1e6);
  for (double& t : T) t = 0;
  t0 = now();
  for (int r = 0; r < reps; ++r) { B = A; chol2(B, g.data(), x.data(), n); }
  double md = 0;
  { std::vector<double> x3 = x; double T2[4]; for (int q=0;q<4;++q) T2[q]=T[q]; double t3 = now();
    for (int r = 0; r < reps; ++r) { B = A; chol3(B, g.data(), x3.data(), n); }
    printf("2row: %.2f us\n", (now()-t3)/reps*1e6);
    t3 = now(); std::vector<double> x4 = x;
    for (int r = 0; r < reps; ++r) { B = A; chol4(B, g.data(), x4.data(), n); }
    printf("2row-scalar-fma: %.2f us\n", (now()-t3)/reps*1e6); for (int q=0;q<4;++q) T[q]=T2[q]; } for (int i = 0; i < n; ++i) md = std::max(md, std::abs(x[i] - x1[i]) / (std::abs(x1[i]) + 1e-300));
  printf("fma: n=%d total %.2f us: panel %.2f trailing %.2f fwd %.2f back %.2f  (max rel diff %.2e)\n", n, (now()-t0)/reps*1e6, T[0]/reps*1e6, T[1]/reps*1e6, T[2]/reps*1e6, T[3]/reps*1e6, md);
}
