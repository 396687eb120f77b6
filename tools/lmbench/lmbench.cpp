// Host cost of the window LM (smoother.cpp) without the device: a 12-pose window,
// one prior, one dense LinearContainerFactor over the 11 previous poses and 11
// (i, j) pairs whose G is a fixed SPD block (the lin_pairs callback costs nothing).
// Prints microseconds per linearization spent in window_lm itself.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../form_amd/csrc/smoother.hpp"

using namespace fmxh;
namespace fmxh { extern double g_lm_prof[4]; }
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 12;
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd;
  WinGraph g;
  std::vector<Pose> x0(P);
  for (int k = 0; k < P; ++k) {
    g.keys.push_back(k);
    double xi[6];
    for (double& v : xi) v = 0.01 * nd(rng);
    xi[3] += k;
    x0[k] = expmap(xi);
  }
  PriorF pr{0, x0[0], 1e-3};
  g.priors.push_back(&pr);
  LinF L;
  const int n = 6 * (P - 1), m = n + 1;
  for (int k = 0; k < P - 1; ++k) {
    L.keys.push_back(k);
    L.lin.push_back(x0[k]);
  }
  L.info.assign((size_t)m * m, 0.0);
  for (int r = 0; r < 4 * m; ++r) {
    std::vector<double> a(m);
    for (double& v : a) v = nd(rng);
    for (int i = 0; i < m; ++i)
      for (int j = 0; j < m; ++j) L.info[(size_t)i * m + j] += a[i] * a[j];
  }
  g.lins.push_back(&L);
  for (int k = 0; k < P - 1; ++k) g.pairs.push_back({k, P - 1});
  std::vector<double> G0(g.pairs.size() * kPairG);
  for (size_t p = 0; p < g.pairs.size(); ++p) {
    double S[13][13] = {};
    for (int r = 0; r < 40; ++r) {
      double a[13];
      for (double& v : a) v = nd(rng);
      for (int i = 0; i < 13; ++i)
        for (int j = 0; j < 13; ++j) S[i][j] += a[i] * a[j];
    }
    int o = 0;
    for (int i = 0; i < 13; ++i)
      for (int j = i; j < 13; ++j) G0[p * kPairG + o++] = S[i][j];
    G0[p * kPairG + 91] = 0.5 * S[12][12];
  }
  int calls = 0;
  double tcb = 0;
  g.lin_pairs = [&](const std::vector<Pose>& x, double* G) {
    const double t = now();
    std::memcpy(G, G0.data(), G0.size() * sizeof(double));
    // make the error depend on x so the LM iterates: + |translation of the last pose|
    for (size_t p = 0; p < g.pairs.size(); ++p) G[p * kPairG + 90] += 1e-3 * (x[P - 1].m[3] * x[P - 1].m[3]);
    ++calls;
    tcb += now() - t;
  };
  const int reps = 2000;
  double t0 = now();
  int lins = 0, iters = 0;
  for (int r = 0; r < reps; ++r) {
    WinLMResult R = window_lm(g, x0);
    lins += R.lins;
    iters += R.iters;
  }
  const double tt = now() - t0 - tcb;
  printf("P=%d D=%d: %.2f us per linearization (%.2f lins, %.2f iters per LM run), %.1f us per LM run\n", P, 6 * P,
         tt / lins * 1e6, (double)lins / reps, (double)iters / reps, tt / reps * 1e6);
  printf("  chol %.2f us/lin, assemble+callback %.2f us/lin (callback %.2f)\n", g_lm_prof[0] / lins * 1e6, g_lm_prof[1] / lins * 1e6, tcb / lins * 1e6);
  return 0;
}
