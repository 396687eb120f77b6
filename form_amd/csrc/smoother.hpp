// smoother.hpp — the window smoother of FORM's default (smoothing) mode, host side:
// ConstraintManager::optimize / marginalize (form/optimization/constraints.cpp:103-203)
// over a DenseLMOptimizer (gtsam.hpp:39-56), with every FeatureFactor linearization
// delegated to the device (window.hip, a callback here).  GTSAM pieces restated from
// their published behaviour (parity unpinned, as the oracle): PriorFactor<Pose3>
// (H = I, e = -Local(x, prior)), LinearContainerFactor around a HessianFactor,
// partial Cholesky elimination, Values::retract (x * Expmap(delta)), and
// LevenbergMarquardtOptimizer with its defaults (lambda0 1e-5, factor 10, upper
// bound 1e5, minModelFidelity 1e-3, rel/abs tol 1e-5, 100 iterations, damping
// H + lambda I).
#pragma once
#include <stdint.h>

#include <functional>
#include <map>
#include <vector>

#include "pose.hpp"

namespace fmxh {

constexpr int kPairG = 92;  // per pair: packed upper 13 x 13 (91) + error

struct PriorF {  // PriorFactor<Pose3>, isotropic sigma (ConstraintManager pose_noise 1e-3)
  uint64_t key;
  Pose mean;
  double sigma;
};
struct LinF {  // LinearContainerFactor holding a HessianFactor over `keys`
  std::vector<uint64_t> keys;
  std::vector<Pose> lin;     // linearization point per key
  std::vector<double> info;  // (6k+1)^2 augmented [G g; g^T f], row-major
};

// One LM problem over the window keys (Values order = ascending key).
struct WinGraph {
  std::vector<uint64_t> keys;
  std::vector<const PriorF*> priors;
  std::vector<const LinF*> lins;
  std::vector<std::pair<int, int>> pairs;  // pair slot -> (key slot i, key slot j)
  // DenseFactor::linearize of every pair at x (key-slot order): G[npairs][kPairG]
  std::function<void(const std::vector<Pose>& x, double* G)> lin_pairs;
  // Optional split form (used when lin_begin is set): lin_begin(x) starts the device
  // linearization, the host assembles the x-dependent non-pair terms, lin_end(G)
  // waits for it and fills G.
  std::function<void(const std::vector<Pose>& x)> lin_begin;
  std::function<void(double* G)> lin_end;
  // Set by window_lm right before a trial's linearization: the trial's predicted cost
  // decrease (the linear model's) and the current cost; -1 for the first linearization.
  // A caller may read them in lin_begin (register_scan: speculate only on a trial the
  // LM will probably stop after).
  mutable double trial_lin_change = -1.0, trial_err = 0.0;
};

struct WinLMResult {
  std::vector<Pose> x;    // final values (key-slot order)
  std::vector<double> G;  // every pair's linearization at x
  int iters = 0;
  int lins = 0;           // lin_pairs calls
};

WinLMResult window_lm(const WinGraph& g, const std::vector<Pose>& x0);

// Dense augmented system over `keys` (any order), columns 6*slot + d, rhs last.
struct DenseSys {
  std::vector<uint64_t> keys;
  std::map<uint64_t, int> slot;
  int D = 0;
  std::vector<double> A;  // (D+1)^2 row-major
  void init(const std::vector<uint64_t>& ks);
  double& at(int r, int c) { return A[(size_t)r * (D + 1) + c]; }
  void add_pair(int si, int sj, const double* G91);
  double add_prior(const PriorF& P, const Pose& x);                       // returns error
  double add_linf(const LinF& L, const std::vector<Pose>& xk);            // x per L.keys
};

// Solve A x = g for SPD A (n x n row-major, overwritten by the factor); false if A is
// not positive definite.
bool chol_solve(std::vector<double>& A, const double* g, double* x, int n);
// sum_k p[k] q[k] (vector partial sums on AVX-512 hosts)
double dot(const double* p, const double* q, int n);

// Schur complement eliminating the first nm columns of an n-column augmented system;
// out = (n - nm + 1)^2.  False if the eliminated block is not positive definite.
bool schur_marginal(const std::vector<double>& A, int n, int nm, std::vector<double>& out);

}  // namespace fmxh
