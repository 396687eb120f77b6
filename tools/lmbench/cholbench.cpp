// Host Cholesky microbenchmark: time and relative residual of fmxh::chol_solve at n
// (FMX_CHOL_AVX2 / FMX_CHOL_PLAIN select the lower SIMD paths).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
namespace fmxh { bool chol_solve(std::vector<double>& A, const double* g, double* x, int n); }
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 72;
  std::mt19937_64 rng(1); std::normal_distribution<double> nd;
  std::vector<double> A((size_t)n*n, 0.0), g(n), x(n);
  for (int r = 0; r < 2*n; ++r) { std::vector<double> a(n); for (auto& v : a) v = nd(rng); for (int i=0;i<n;++i) for (int j=0;j<n;++j) A[i*n+j]+=a[i]*a[j]; }
  for (auto& v : g) v = nd(rng);
  std::vector<double> B;
  int reps = 20000; double t0 = now();
  for (int r = 0; r < reps; ++r) { B = A; fmxh::chol_solve(B, g.data(), x.data(), n); }
  const double t = (now()-t0)/reps*1e6;
  double rn = 0, gn = 0;
  for (int i = 0; i < n; ++i) { double s = 0; for (int j = 0; j < n; ++j) s += A[i*n+j]*x[j]; rn += (s-g[i])*(s-g[i]); gn += g[i]*g[i]; }
  printf("n=%d chol_solve %.2f us, |Ax-g|/|g| %.2e, x0 %.17g\n", n, t, std::sqrt(rn/gn), x[0]);
}
