// Host-only exercise of the window smoother (form_amd/csrc/smoother.cpp) for the
// sanitizer build (tools/asan_check.sh): dense LM over a small window with priors, a
// LinearContainerFactor and pair factors whose linearization comes from a callback
// (the device's role), in both the plain and the split (lin_begin / lin_end) forms, then
// the Schur marginal and the Cholesky solve on random SPD systems.  Checks: the LM
// converges to the priors' poses (the pair factors are consistent with them), the split
// form gives the same result bit for bit, and chol_solve solves.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "smoother.hpp"

using namespace fmxh;

// A pair factor between poses a, b whose residual is the relative pose's tangent
// minus a measured one, linearized numerically (13 columns: H_a, H_b, -r), packed.
static void pair_G(const Pose& a, const Pose& b, const Pose& meas, double* G) {
  auto res = [&](const Pose& x, const Pose& y, double* r) {
    logmap(compose(inverse(meas), compose(inverse(x), y)), r);
  };
  double r0[6];
  res(a, b, r0);
  double J[6][12];
  const double h = 1e-7;
  for (int c = 0; c < 12; ++c) {
    double d[6] = {0, 0, 0, 0, 0, 0};
    d[c % 6] = h;
    const Pose da = c < 6 ? compose(a, expmap(d)) : a, db = c < 6 ? b : compose(b, expmap(d));
    double r1[6];
    res(da, db, r1);
    for (int i = 0; i < 6; ++i) J[i][c] = (r1[i] - r0[i]) / h;
  }
  int q = 0;
  for (int i = 0; i < 13; ++i)
    for (int j = i; j < 13; ++j) {
      double s = 0;
      for (int k = 0; k < 6; ++k) {
        const double ai = i < 12 ? J[k][i] : -r0[k], aj = j < 12 ? J[k][j] : -r0[k];
        s += ai * aj;
      }
      G[q++] = s;
    }
  G[91] = 0.5 * (r0[0] * r0[0] + r0[1] * r0[1] + r0[2] * r0[2] + r0[3] * r0[3] + r0[4] * r0[4] + r0[5] * r0[5]);
}

int main() {
  std::mt19937 rng(7);
  std::normal_distribution<double> nd(0.0, 1.0);
  const int n = 6;
  std::vector<Pose> truth(n), x0(n);
  for (int k = 0; k < n; ++k) {
    double xi[6];
    for (double& v : xi) v = 0.3 * nd(rng);
    truth[k] = expmap(xi);
    for (double& v : xi) v = 0.02 * nd(rng);
    x0[k] = compose(truth[k], expmap(xi));
  }
  WinGraph g;
  for (int k = 0; k < n; ++k) g.keys.push_back(10 + k);
  std::vector<PriorF> pri = {{10, truth[0], 1e-3}};
  for (auto& p : pri) g.priors.push_back(&p);
  LinF lf;  // a weak linear factor on keys 11, 12 at the truth
  lf.keys = {11, 12};
  lf.lin = {truth[1], truth[2]};
  lf.info.assign(13 * 13, 0.0);
  for (int i = 0; i < 12; ++i) lf.info[i * 13 + i] = 1.0;
  g.lins.push_back(&lf);
  std::vector<Pose> meas;
  for (int k = 0; k + 1 < n; ++k) {
    g.pairs.push_back({k, k + 1});
    meas.push_back(compose(inverse(truth[k]), truth[k + 1]));
  }
  g.pairs.push_back({0, n - 1});
  meas.push_back(compose(inverse(truth[0]), truth[n - 1]));
  g.lin_pairs = [&](const std::vector<Pose>& x, double* G) {
    for (size_t p = 0; p < g.pairs.size(); ++p) pair_G(x[g.pairs[p].first], x[g.pairs[p].second], meas[p], G + 92 * p);
  };
  const WinLMResult R1 = window_lm(g, x0);
  // split form: the callback pair of the device path
  std::vector<Pose> pend;
  WinGraph g2 = g;
  g2.lin_pairs = nullptr;
  g2.lin_begin = [&](const std::vector<Pose>& x) { pend = x; };
  g2.lin_end = [&](double* G) { g.lin_pairs(pend, G); };
  const WinLMResult R2 = window_lm(g2, x0);
  double err = 0, diff = 0;
  for (int k = 0; k < n; ++k)
    for (int e = 0; e < 12; ++e) {
      err = std::fmax(err, std::fabs(R1.x[k].m[e] - truth[k].m[e]));
      diff = std::fmax(diff, std::fabs(R1.x[k].m[e] - R2.x[k].m[e]));
    }
  printf("lm iters %d lins %d, max |x - truth| %.3e, split vs plain %.3e\n", R1.iters, R1.lins, err, diff);
  if (!(err < 1e-6) || diff != 0.0) return 1;
  // Cholesky factor bit for bit against the scalar FMA recurrence (right-looking, k
  // ascending per element, rows scaled by the reciprocal of the pivot): every FMA host
  // path (AVX2, AVX-512, any blocking) must round exactly like it
  if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) {
    for (int D : {6, 7, 13, 18, 61, 96, 108, 150, 157}) {
      std::vector<double> M((size_t)D * D), H((size_t)D * D), g0(D), xs(D);
      for (double& v : M) v = nd(rng);
      for (int i = 0; i < D; ++i)
        for (int j = 0; j < D; ++j) {
          double s = i == j ? D : 0.0;
          for (int k = 0; k < D; ++k) s += M[(size_t)i * D + k] * M[(size_t)j * D + k];
          H[(size_t)i * D + j] = s;
        }
      for (double& v : g0) v = nd(rng);
      std::vector<double> R = H;
      for (int k = 0; k < D; ++k) {
        double* Uk = &R[(size_t)k * D];
        const double ukk = std::sqrt(Uk[k]), r = 1.0 / ukk;
        for (int m = k + 1; m < D; ++m) Uk[m] = Uk[m] * r;
        Uk[k] = ukk;
        for (int i = k + 1; i < D; ++i)
          for (int m = i; m < D; ++m) R[(size_t)i * D + m] = std::fma(-Uk[i], Uk[m], R[(size_t)i * D + m]);
      }
      std::vector<double> F = H;
      if (!chol_solve(F, g0.data(), xs.data(), D)) return 5;
      size_t diff = 0;
      for (int i = 0; i < D; ++i)
        for (int m = i; m < D; ++m) diff += F[(size_t)i * D + m] != R[(size_t)i * D + m];
      printf("D %3d: factor entries differing from the FMA recurrence: %zu\n", D, diff);
      if (diff) return 6;
    }
  }
  // Schur marginal and Cholesky on random SPD augmented systems
  for (int D : {6, 18, 61, 108}) {
    std::vector<double> M((size_t)D * D), A((size_t)(D + 1) * (D + 1), 0.0), g0(D), xs(D);
    for (double& v : M) v = nd(rng);
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        double s = i == j ? D : 0.0;
        for (int k = 0; k < D; ++k) s += M[(size_t)i * D + k] * M[(size_t)j * D + k];
        A[(size_t)i * (D + 1) + j] = s;
      }
    for (int i = 0; i < D; ++i) A[(size_t)i * (D + 1) + D] = A[(size_t)D * (D + 1) + i] = g0[i] = nd(rng);
    A[(size_t)D * (D + 1) + D] = 1e3;
    std::vector<double> out;
    if (D > 6 && !schur_marginal(A, D, 6, out)) return 2;
    std::vector<double> H((size_t)D * D);
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) H[(size_t)i * D + j] = A[(size_t)i * (D + 1) + j];
    std::vector<double> H0 = H;
    if (!chol_solve(H, g0.data(), xs.data(), D)) return 3;
    double rmax = 0;
    for (int i = 0; i < D; ++i) {
      double s = -g0[i];
      for (int j = 0; j < D; ++j) s += H0[(size_t)i * D + j] * xs[j];
      rmax = std::fmax(rmax, std::fabs(s));
    }
    printf("D %3d: chol residual %.2e\n", D, rmax);
    if (!(rmax < 1e-8)) return 4;
  }
  printf("smoother ok\n");
  return 0;
}
