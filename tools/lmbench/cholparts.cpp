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
int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 72;
  std::mt19937_64 rng(1); std::normal_distribution<double> nd;
  std::vector<double> A((size_t)n*n, 0.0), g(n), x(n);
  for (int r = 0; r < 2*n; ++r) { std::vector<double> a(n); for (auto& v : a) v = nd(rng); for (int i=0;i<n;++i) for (int j=0;j<n;++j) A[i*n+j]+=a[i]*a[j]; }
  for (auto& v : g) v = nd(rng);
  std::vector<double> B;
  int reps = 20000; double t0 = now();
  for (int r = 0; r < reps; ++r) { B = A; chol(B, g.data(), x.data(), n); }
  printf("n=%d total %.2f us: panel %.2f trailing %.2f fwd %.2f back %.2f\n", n, (now()-t0)/reps*1e6, T[0]/reps*1e6, T[1]/reps*1e6, T[2]/reps*1e6, T[3]/reps*1e6);
}
