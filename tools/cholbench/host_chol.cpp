// Host Cholesky (smoother.cpp chol_solve) time per call vs window size D = 6 x poses:
// the LM solves one per trial.  g++ -O3 -std=c++17 -ffp-contract=off -Iform_amd/csrc
//   tools/cholbench/host_chol.cpp form_amd/csrc/smoother.cpp -o host_chol
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
#include "smoother.hpp"
using namespace fmxh;
int main() {
  std::mt19937 rng(1);
  std::normal_distribution<double> nd;

  for (int D : {66, 84, 102, 120, 138, 156}) {
    std::vector<double> M((size_t)D * D), H((size_t)D * D), g(D), x(D);
    for (auto& v : M) v = nd(rng);
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        double s = i == j ? D : 0;
        for (int k = 0; k < D; ++k) s += M[i * D + k] * M[j * D + k];
        H[i * D + j] = s;
      }
    for (auto& v : g) v = nd(rng);
    const int N = 2000;
    std::vector<double> A;
    double best = 1e9;
    for (int r = 0; r < 5; ++r) {
      auto t0 = std::chrono::steady_clock::now();
      for (int it = 0; it < N; ++it) {
        A = H;
        chol_solve(A, g.data(), x.data(), D);
      }
      double us = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / N * 1e6;
      best = std::min(best, us);
    }
    printf("D %3d: copy + chol_solve %.2f us  (%.1f GFLOP/s)\n", D, best, D * (double)D * D / 3.0 / best * 1e-3);
  }
}
