// smoother.cpp — dense window Levenberg-Marquardt + marginal factors (smoother.hpp).
// Host code; built with -ffp-contract=off like the rest of the pose algebra.
#include "smoother.hpp"

#include <algorithm>
#include <cstring>

namespace fmxh {

void DenseSys::init(const std::vector<uint64_t>& ks) {
  keys = ks;
  slot.clear();
  for (size_t k = 0; k < ks.size(); ++k) slot[ks[k]] = (int)k;
  D = 6 * (int)ks.size();
  A.assign((size_t)(D + 1) * (D + 1), 0.0);
}

// Scatter a pair's packed upper 13 x 13 [H_i H_j b]^T [H_i H_j b] (gtsam.hpp:67-86).
void DenseSys::add_pair(int si, int sj, const double* G) {
  int col[13];
  for (int k = 0; k < 6; ++k) {
    col[k] = 6 * si + k;
    col[6 + k] = 6 * sj + k;
  }
  col[12] = D;
  int o = 0;
  for (int a = 0; a < 13; ++a)
    for (int b = a; b < 13; ++b) {
      const double v = G[o++];
      at(col[a], col[b]) += v;
      if (a != b) at(col[b], col[a]) += v;
    }
}

// PriorFactor<Pose3>::evaluateError: H = I, e = -Logmap(x^-1 * prior), whitened by
// 1/sigma: A = I/sigma, b = -e/sigma = Logmap(x^-1 * prior)/sigma.
double DenseSys::add_prior(const PriorF& P, const Pose& x) {
  double l[6];
  logmap(compose(inverse(x), P.mean), l);
  const double inv = 1.0 / P.sigma;
  const int s = slot.at(P.key);
  double f = 0;
  for (int k = 0; k < 6; ++k) {
    const double b = l[k] * inv;
    at(6 * s + k, 6 * s + k) += inv * inv;
    at(6 * s + k, D) += inv * b;
    at(D, 6 * s + k) += inv * b;
    f += b * b;
  }
  at(D, D) += f;
  return 0.5 * f;
}

// LinearContainerFactor::linearize at x (delta = Local(lin, x) per key):
// G' = G, g' = g - G delta, f' = f + delta^T G delta - 2 delta^T g; error = 0.5 f'.
double DenseSys::add_linf(const LinF& L, const std::vector<Pose>& xk) {
  const int n = 6 * (int)L.keys.size(), m = n + 1;
  std::vector<double> d(n), Gd(n);
  for (size_t k = 0; k < L.keys.size(); ++k) logmap(compose(inverse(L.lin[k]), xk[k]), &d[6 * k]);
  const double* I = L.info.data();
  for (int r = 0; r < n; ++r) {
    double s = 0;
    for (int c = 0; c < n; ++c) s += I[(size_t)r * m + c] * d[c];
    Gd[r] = s;
  }
  double dGd = 0, dg = 0;
  for (int r = 0; r < n; ++r) {
    dGd += d[r] * Gd[r];
    dg += d[r] * I[(size_t)r * m + n];
  }
  std::vector<int> col(m);
  for (size_t k = 0; k < L.keys.size(); ++k)
    for (int e = 0; e < 6; ++e) col[6 * k + e] = 6 * slot.at(L.keys[k]) + e;
  col[n] = D;
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) at(col[r], col[c]) += I[(size_t)r * m + c];
  for (int r = 0; r < n; ++r) {
    const double g = I[(size_t)r * m + n] - Gd[r];
    at(col[r], D) += g;
    at(D, col[r]) += g;
  }
  const double f = I[(size_t)n * m + n] + dGd - 2.0 * dg;
  at(D, D) += f;
  return 0.5 * f;
}

namespace {

// In-place Cholesky of an n x n SPD matrix (row-major, lower factor) + solve.
bool chol_solve(std::vector<double>& H, const double* g, double* x, int n) {
  for (int j = 0; j < n; ++j) {
    double* Hj = &H[(size_t)j * n];
    double s = Hj[j];
    for (int k = 0; k < j; ++k) s -= Hj[k] * Hj[k];
    if (!(s > 0)) return false;
    const double ljj = std::sqrt(s);
    Hj[j] = ljj;
    for (int i = j + 1; i < n; ++i) {
      double* Hi = &H[(size_t)i * n];
      double t = Hi[j];
      for (int k = 0; k < j; ++k) t -= Hi[k] * Hj[k];
      Hi[j] = t / ljj;
    }
  }
  std::vector<double> y(n);
  for (int i = 0; i < n; ++i) {
    const double* Hi = &H[(size_t)i * n];
    double s = g[i];
    for (int k = 0; k < i; ++k) s -= Hi[k] * y[k];
    y[i] = s / Hi[i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < n; ++k) s -= H[(size_t)k * n + i] * x[k];
    x[i] = s / H[(size_t)i * n + i];
  }
  return true;
}

// NonlinearFactorGraph::linearize at x into S; returns the graph error.
double linearize_all(const WinGraph& g, const std::vector<Pose>& x, DenseSys& S, std::vector<double>& G, int& lins) {
  S.init(g.keys);
  G.assign(g.pairs.size() * kPairG, 0.0);
  if (!g.pairs.empty()) {
    g.lin_pairs(x, G.data());
    ++lins;
  }
  double err = 0;
  for (const PriorF* P : g.priors) err += S.add_prior(*P, x[S.slot.at(P->key)]);
  for (const LinF* L : g.lins) {
    std::vector<Pose> xk;
    for (uint64_t k : L->keys) xk.push_back(x[S.slot.at(k)]);
    err += S.add_linf(*L, xk);
  }
  for (size_t p = 0; p < g.pairs.size(); ++p) {
    S.add_pair(g.pairs[p].first, g.pairs[p].second, &G[p * kPairG]);
    err += G[p * kPairG + 91];
  }
  return err;
}

}  // namespace

// LevenbergMarquardtOptimizer over every window pose (NonlinearOptimizer::
// defaultOptimize + iterate/tryLambda).  Each trial is evaluated by a full
// linearization: it yields the error the accept test needs and, when accepted, the
// next iteration's system (one device launch per trial).
WinLMResult window_lm(const WinGraph& g, const std::vector<Pose>& x0) {
  WinLMResult R;
  R.x = x0;
  DenseSys S, Sn;
  std::vector<double> Gn;
  double err = linearize_all(g, R.x, S, R.G, R.lins);
  if (err <= 0.0) return R;
  double lambda = 1e-5;
  const int D = S.D;
  std::vector<double> H((size_t)D * D), gg(D), Hd, dx(D);
  auto iterate = [&]() {
    for (int r = 0; r < D; ++r) {
      std::memcpy(&H[(size_t)r * D], &S.A[(size_t)r * (D + 1)], D * sizeof(double));
      gg[r] = S.at(r, D);
    }
    const double cc = S.at(D, D), oldLin = 0.5 * cc;
    for (;;) {
      Hd = H;
      for (int r = 0; r < D; ++r) Hd[(size_t)r * D + r] += lambda;
      const bool ok = chol_solve(Hd, gg.data(), dx.data(), D);
      bool success = false, stop = false;
      std::vector<Pose> xn;
      double nerr = err;
      if (ok) {
        double dHd = 0, dg = 0;
        for (int r = 0; r < D; ++r) {
          double h = 0;
          const double* Hr = &H[(size_t)r * D];
          for (int c = 0; c < D; ++c) h += Hr[c] * dx[c];
          dHd += dx[r] * h;
          dg += dx[r] * gg[r];
        }
        const double newLin = 0.5 * (dHd - 2 * dg + cc), linChange = oldLin - newLin;
        if (linChange >= 0) {
          xn.resize(R.x.size());
          for (size_t k = 0; k < R.x.size(); ++k) xn[k] = compose(R.x[k], expmap(&dx[6 * k]));
          nerr = linearize_all(g, xn, Sn, Gn, R.lins);
          const double costChange = err - nerr;
          if (linChange > DBL_EPSILON * oldLin) success = (costChange / linChange) > 1e-3;
          else success = true;
          if (std::abs(costChange) < 1e-5 * err) stop = true;
        }
      }
      if (success) {
        lambda = std::max(0.0, lambda / 10.0);
        R.x.swap(xn);
        err = nerr;
        std::swap(S, Sn);
        R.G.swap(Gn);
        return;
      } else if (!stop) {
        lambda *= 10.0;
        if (lambda >= 1e5) return;
      } else {
        return;
      }
    }
  };
  double cur, newErr = err;
  bool conv;
  do {
    cur = newErr;
    iterate();
    ++R.iters;
    newErr = err;
    if (newErr <= 0.0) conv = true;
    else {
      const double absDec = cur - newErr, relDec = absDec / cur;
      conv = (relDec <= 1e-5) || (absDec <= 1e-5);
    }
  } while (R.iters < 100 && !conv && std::isfinite(cur));
  return R;
}

bool schur_marginal(const std::vector<double>& A, int n, int nm, std::vector<double>& out) {
  const int m = n + 1, r = m - nm;
  std::vector<double> L((size_t)nm * nm, 0.0);
  for (int j = 0; j < nm; ++j) {
    double s = A[(size_t)j * m + j];
    for (int k = 0; k < j; ++k) s -= L[(size_t)j * nm + k] * L[(size_t)j * nm + k];
    if (!(s > 0)) return false;
    L[(size_t)j * nm + j] = std::sqrt(s);
    for (int i = j + 1; i < nm; ++i) {
      double t = A[(size_t)i * m + j];
      for (int k = 0; k < j; ++k) t -= L[(size_t)i * nm + k] * L[(size_t)j * nm + k];
      L[(size_t)i * nm + j] = t / L[(size_t)j * nm + j];
    }
  }
  std::vector<double> Y((size_t)nm * r);  // L^-1 A_MR
  for (int c = 0; c < r; ++c)
    for (int i = 0; i < nm; ++i) {
      double s = A[(size_t)i * m + nm + c];
      for (int k = 0; k < i; ++k) s -= L[(size_t)i * nm + k] * Y[(size_t)k * r + c];
      Y[(size_t)i * r + c] = s / L[(size_t)i * nm + i];
    }
  out.assign((size_t)r * r, 0.0);
  for (int a = 0; a < r; ++a)
    for (int b = 0; b < r; ++b) {
      double s = 0;
      for (int k = 0; k < nm; ++k) s += Y[(size_t)k * r + a] * Y[(size_t)k * r + b];
      out[(size_t)a * r + b] = A[(size_t)(nm + a) * m + nm + b] - s;
    }
  return true;
}

}  // namespace fmxh
