// smoother.cpp — dense window Levenberg-Marquardt + marginal factors (smoother.hpp).
// Host code; built with -ffp-contract=off like the rest of the pose algebra.
#include "smoother.hpp"

#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#ifdef FMX_LM_PROF  // diagnostic build: host LM phase times (printed at exit)
#include <chrono>
#include <cstdio>
namespace fmxh {
double g_lm_prof[6];
uint64_t g_lm_n[6];
static const char* kLmProfNames[6] = {"H copy + chol_solve", "trial run (launch .. lin_end)", "accept test",
                                      "after lin_end: add_pair", "iterate prologue", "trial poses"};
struct LmProfPrint {
  ~LmProfPrint() {
    for (int i = 0; i < 6; ++i)
      if (g_lm_n[i]) fprintf(stderr, "lm %-32s %10.1f us total %8llu calls %8.2f us/call\n", kLmProfNames[i],
                             g_lm_prof[i] * 1e6, (unsigned long long)g_lm_n[i], g_lm_prof[i] * 1e6 / g_lm_n[i]);
  }
} g_lm_print;
}  // namespace fmxh
static double lmnow() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define LMP_BEGIN(i) const double _lmp##i = lmnow()
#define LMP_END(i) (fmxh::g_lm_prof[i] += lmnow() - _lmp##i, ++fmxh::g_lm_n[i])
#else
#define LMP_BEGIN(i)
#define LMP_END(i)
#endif

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
  const double f = I[(size_t)n * m + n] + (dGd - 2.0 * dg);
  at(D, D) += f;
  return 0.5 * f;
}

// Cholesky solve of an n x n SPD system (row-major; factor U = L^T kept in the upper
// triangle).  Right-looking, blocked by 6 (one pose): a 6-row panel is factored,
// then the trailing rows take the panel's 6 updates with one load/store per element
// (every element still receives its updates k = 0, 1, ... in order).
// Two paths, chosen once per process: on AVX2+FMA hosts the trailing update runs two
// rows per pass (each panel load feeds both) with fused multiply-adds and the back
// substitution keeps 4 partial sums; elsewhere the plain scalar form, which rounds
// like the oracle's left-looking dot products.  Both are deterministic on a given
// host; they differ from each other (and from the oracle) by FMA rounding only.
namespace {

constexpr int kCholB = 6;

void chol_panel(double* a, int n, int kb, int ke, bool& ok) {
  for (int k = kb; k < ke; ++k) {
    double* __restrict Uk = a + (size_t)k * n;
    const double s = Uk[k];
    if (!(s > 0)) {
      ok = false;
      return;
    }
    const double ukk = std::sqrt(s);
    Uk[k] = ukk;
    for (int m = k + 1; m < n; ++m) Uk[m] = Uk[m] / ukk;
    for (int i = k + 1; i < ke; ++i) {
      double* __restrict Ai = a + (size_t)i * n;
      const double uki = Uk[i];
      for (int m = i; m < n; ++m) Ai[m] -= uki * Uk[m];
    }
  }
}
// FMA form of the panel: scale by the reciprocal, fused updates.
__attribute__((target("avx2,fma"))) void chol_panel_fma(double* a, int n, int kb, int ke, bool& ok) {
  for (int k = kb; k < ke; ++k) {
    double* __restrict Uk = a + (size_t)k * n;
    const double s = Uk[k];
    if (!(s > 0)) {
      ok = false;
      return;
    }
    const double ukk = std::sqrt(s), r = 1.0 / ukk;
    Uk[k] = ukk;
    for (int m = k + 1; m < n; ++m) Uk[m] = Uk[m] * r;
    for (int i = k + 1; i < ke; ++i) {
      double* __restrict Ai = a + (size_t)i * n;
      const double uki = Uk[i];
      for (int m = i; m < n; ++m) Ai[m] = std::fma(-uki, Uk[m], Ai[m]);
    }
  }
}

void chol_trail_plain(double* a, int n, int kb, int ke) {
  const double* U[kCholB];
  for (int t = 0; t < kCholB; ++t) U[t] = a + (size_t)(kb + t) * n;
  for (int i = ke; i < n; ++i) {
    double* __restrict Ai = a + (size_t)i * n;
    double u[kCholB];
    for (int t = 0; t < kCholB; ++t) u[t] = U[t][i];
    for (int m = i; m < n; ++m) {
      double v = Ai[m];
      for (int t = 0; t < kCholB; ++t) v -= u[t] * U[t][m];
      Ai[m] = v;
    }
  }
}

__attribute__((target("avx2,fma"))) void chol_trail_fma(double* a, int n, int kb, int ke) {
  const double* U[kCholB];
  for (int t = 0; t < kCholB; ++t) U[t] = a + (size_t)(kb + t) * n;
  int i = ke;
  for (; i + 2 <= n; i += 2) {
    double* __restrict A0 = a + (size_t)i * n;
    double* __restrict A1 = A0 + n;
    double u0[kCholB], u1[kCholB];
    __m256d b0[kCholB], b1[kCholB];
    for (int t = 0; t < kCholB; ++t) {
      u0[t] = U[t][i];
      u1[t] = U[t][i + 1];
      b0[t] = _mm256_set1_pd(u0[t]);
      b1[t] = _mm256_set1_pd(u1[t]);
    }
    {
      double v = A0[i];
      for (int t = 0; t < kCholB; ++t) v = std::fma(-u0[t], U[t][i], v);
      A0[i] = v;
    }
    int m = i + 1;
    for (; m + 4 <= n; m += 4) {
      __m256d x0 = _mm256_loadu_pd(A0 + m), x1 = _mm256_loadu_pd(A1 + m);
      for (int t = 0; t < kCholB; ++t) {
        const __m256d uu = _mm256_loadu_pd(U[t] + m);
        x0 = _mm256_fnmadd_pd(b0[t], uu, x0);
        x1 = _mm256_fnmadd_pd(b1[t], uu, x1);
      }
      _mm256_storeu_pd(A0 + m, x0);
      _mm256_storeu_pd(A1 + m, x1);
    }
    for (; m < n; ++m) {
      double v0 = A0[m], v1 = A1[m];
      for (int t = 0; t < kCholB; ++t) {
        v0 = std::fma(-u0[t], U[t][m], v0);
        v1 = std::fma(-u1[t], U[t][m], v1);
      }
      A0[m] = v0;
      A1[m] = v1;
    }
  }
  for (; i < n; ++i) {
    double* __restrict Ai = a + (size_t)i * n;
    for (int m = i; m < n; ++m) {
      double v = Ai[m];
      for (int t = 0; t < kCholB; ++t) v = std::fma(-U[t][i], U[t][m], v);
      Ai[m] = v;
    }
  }
}

__attribute__((target("avx2,fma"))) void chol_back_fma(const double* a, int n, const double* y, double* x) {
  for (int i = n - 1; i >= 0; --i) {  // U x = y
    const double* Ui = a + (size_t)i * n;
    __m256d acc = _mm256_setzero_pd();
    int k = i + 1;
    for (; k + 4 <= n; k += 4) acc = _mm256_fmadd_pd(_mm256_loadu_pd(Ui + k), _mm256_loadu_pd(x + k), acc);
    double p[4];
    _mm256_storeu_pd(p, acc);
    double s = y[i] - ((p[0] + p[1]) + (p[2] + p[3]));
    for (; k < n; ++k) s = std::fma(-Ui[k], x[k], s);
    x[i] = s / Ui[i];
  }
}

__attribute__((target("avx512f,fma"))) inline __mmask8 tail_mask(int left) {
  return left >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << left) - 1u);
}

// The trailing rows i0 .. i0 + R - 1 take the 8 updates of panel rows kb .. kb + 7 in a
// register tile: R rows x 3 column vectors (24 columns) per pass, each panel row's
// three vectors loaded once for the R rows (its entries in rows i0 .. as embedded
// broadcasts), then 8-wide (masked) vectors to the row end.  Columns start at the
// vector holding row i0's diagonal; rows below i0 write lower-triangle scratch there.
template <int R>
__attribute__((target("avx512f,fma"))) inline void chol_tile_512(double* a, int n, int kb, int i0) {
  const double* U = a + (size_t)kb * n;
  double* A = a + (size_t)i0 * n;
  int m = i0 & ~7;
  for (; m + 24 <= n; m += 24) {
    __m512d x[R][3];
#pragma GCC unroll 16
    for (int r = 0; r < R; ++r)
#pragma GCC unroll 16
      for (int v = 0; v < 3; ++v) x[r][v] = _mm512_loadu_pd(A + (size_t)r * n + m + 8 * v);
#pragma GCC unroll 16
    for (int t = 0; t < 8; ++t) {
      const double* Ut = U + (size_t)t * n;
      const __m512d u0 = _mm512_loadu_pd(Ut + m), u1 = _mm512_loadu_pd(Ut + m + 8), u2 = _mm512_loadu_pd(Ut + m + 16);
#pragma GCC unroll 16
      for (int r = 0; r < R; ++r) {
        const __m512d b = _mm512_set1_pd(Ut[i0 + r]);
        x[r][0] = _mm512_fnmadd_pd(b, u0, x[r][0]);
        x[r][1] = _mm512_fnmadd_pd(b, u1, x[r][1]);
        x[r][2] = _mm512_fnmadd_pd(b, u2, x[r][2]);
      }
    }
#pragma GCC unroll 16
    for (int r = 0; r < R; ++r)
#pragma GCC unroll 16
      for (int v = 0; v < 3; ++v) _mm512_storeu_pd(A + (size_t)r * n + m + 8 * v, x[r][v]);
  }
  for (; m < n; m += 8) {
    const __mmask8 k = tail_mask(n - m);
    __m512d x[R];
#pragma GCC unroll 16
    for (int r = 0; r < R; ++r) x[r] = _mm512_maskz_loadu_pd(k, A + (size_t)r * n + m);
#pragma GCC unroll 16
    for (int t = 0; t < 8; ++t) {
      const double* Ut = U + (size_t)t * n;
      const __m512d u = _mm512_maskz_loadu_pd(k, Ut + m);
#pragma GCC unroll 16
      for (int r = 0; r < R; ++r) x[r] = _mm512_fnmadd_pd(_mm512_set1_pd(Ut[i0 + r]), u, x[r]);
    }
#pragma GCC unroll 16
    for (int r = 0; r < R; ++r) _mm512_mask_storeu_pd(A + (size_t)r * n + m, k, x[r]);
  }
}

// AVX-512 form (the GPU box's EPYC has it), blocked by 8 rows: (1) the panel's diagonal
// block factored in a local 8 x 8 copy; (2) the panel's strip (columns >= ke) solved in
// registers, the 8 rows of two 8-column vectors at a time (x_k -= U[t][k] x_t for t < k,
// then x_k *= 1 / u_kk); (3) the trailing rows updated in 4-row register tiles
// (chol_tile_512).  Every element still takes its updates k = 0, 1, ... in order as
// fused multiply-adds and each row is scaled by its pivot's reciprocal, so the factor is
// bit for bit the scalar FMA recurrence's (tests/cpp/test_smoother.cpp checks it), as the
// row-at-a-time form it replaces was; the panel no longer round-trips every strip row
// through memory once per pivot.
__attribute__((target("avx512f,fma"))) bool chol_solve_512(double* a, const double* g, double* x, int n) {
  for (int kb = 0; kb < n; kb += 8) {
    const int ke = std::min(n, kb + 8), nb = ke - kb;
    double B[8][8], rk[8];
    for (int i = 0; i < nb; ++i)
      for (int m = i; m < nb; ++m) B[i][m] = a[(size_t)(kb + i) * n + kb + m];
    for (int k = 0; k < nb; ++k) {
      const double s = B[k][k];
      if (!(s > 0)) return false;
      const double ukk = std::sqrt(s), r = 1.0 / ukk;
      for (int m = k + 1; m < nb; ++m) B[k][m] = B[k][m] * r;
      B[k][k] = ukk;
      rk[k] = r;
      for (int i = k + 1; i < nb; ++i)
        for (int m = i; m < nb; ++m) B[i][m] = __builtin_fma(-B[k][i], B[k][m], B[i][m]);
    }
    for (int i = 0; i < nb; ++i)
      for (int m = i; m < nb; ++m) a[(size_t)(kb + i) * n + kb + m] = B[i][m];
    if (ke == n) break;  // (nb == 8 below: only the last panel is short)
    double* P = a + (size_t)kb * n;
    int m = ke;
    for (; m + 16 <= n; m += 16) {
      __m512d x0[8], x1[8];
#pragma GCC unroll 16
      for (int k = 0; k < 8; ++k) {
        __m512d v0 = _mm512_loadu_pd(P + (size_t)k * n + m), v1 = _mm512_loadu_pd(P + (size_t)k * n + m + 8);
#pragma GCC unroll 16
        for (int t = 0; t < k; ++t) {
          const __m512d b = _mm512_set1_pd(B[t][k]);
          v0 = _mm512_fnmadd_pd(b, x0[t], v0);
          v1 = _mm512_fnmadd_pd(b, x1[t], v1);
        }
        const __m512d r = _mm512_set1_pd(rk[k]);
        x0[k] = _mm512_mul_pd(v0, r);
        x1[k] = _mm512_mul_pd(v1, r);
        _mm512_storeu_pd(P + (size_t)k * n + m, x0[k]);
        _mm512_storeu_pd(P + (size_t)k * n + m + 8, x1[k]);
      }
    }
    for (; m < n; m += 8) {
      const __mmask8 msk = tail_mask(n - m);
      __m512d x0[8];
#pragma GCC unroll 16
      for (int k = 0; k < 8; ++k) {
        __m512d v0 = _mm512_maskz_loadu_pd(msk, P + (size_t)k * n + m);
#pragma GCC unroll 16
        for (int t = 0; t < k; ++t) v0 = _mm512_fnmadd_pd(_mm512_set1_pd(B[t][k]), x0[t], v0);
        x0[k] = _mm512_mul_pd(v0, _mm512_set1_pd(rk[k]));
        _mm512_mask_storeu_pd(P + (size_t)k * n + m, msk, x0[k]);
      }
    }
    int i = ke;
    for (; i + 4 <= n; i += 4) chol_tile_512<4>(a, n, kb, i);
    switch (n - i) {
      case 3: chol_tile_512<3>(a, n, kb, i); break;
      case 2: chol_tile_512<2>(a, n, kb, i); break;
      case 1: chol_tile_512<1>(a, n, kb, i); break;
      default: break;
    }
  }
  // forward U^T y = g (y in x), then back U x = y
  std::memcpy(x, g, (size_t)n * sizeof(double));
  for (int k = 0; k < n; ++k) {
    const double* Uk = a + (size_t)k * n;
    const double yk = x[k] / Uk[k];
    x[k] = yk;
    const __m512d b = _mm512_set1_pd(yk);
    int m = k + 1;
    for (; m < n; m += 8) {
      const __mmask8 msk = tail_mask(n - m);
      _mm512_mask_storeu_pd(x + m, msk, _mm512_fnmadd_pd(b, _mm512_maskz_loadu_pd(msk, Uk + m), _mm512_maskz_loadu_pd(msk, x + m)));
    }
  }
  for (int i = n - 1; i >= 0; --i) {
    const double* Ui = a + (size_t)i * n;
    __m512d acc = _mm512_setzero_pd();
    for (int k = i + 1; k < n; k += 8) {
      const __mmask8 msk = tail_mask(n - k);
      acc = _mm512_fmadd_pd(_mm512_maskz_loadu_pd(msk, Ui + k), _mm512_maskz_loadu_pd(msk, x + k), acc);
    }
    x[i] = (x[i] - _mm512_reduce_add_pd(acc)) / Ui[i];
  }
  return true;
}

__attribute__((target("avx512f,fma"))) double dot_512(const double* p, const double* q, int n) {
  __m512d acc = _mm512_setzero_pd();
  for (int k = 0; k < n; k += 8) {
    const __mmask8 msk = tail_mask(n - k);
    acc = _mm512_fmadd_pd(_mm512_maskz_loadu_pd(msk, p + k), _mm512_maskz_loadu_pd(msk, q + k), acc);
  }
  return _mm512_reduce_add_pd(acc);
}

// 0 plain, 1 AVX2+FMA, 2 AVX-512: the host CPU's widest
int simd_level() {
  static const int lv = [] {
    const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
    if (avx2 && __builtin_cpu_supports("avx512f")) return 2;
    return avx2 ? 1 : 0;
  }();
  return lv;
}

}  // namespace

// sum_k p[k] q[k]: vector partial sums on AVX-512 hosts, left to right otherwise
double dot(const double* p, const double* q, int n) {
  if (simd_level() == 2) return dot_512(p, q, n);
  double s = 0;
  for (int k = 0; k < n; ++k) s += p[k] * q[k];
  return s;
}

bool chol_solve(std::vector<double>& A, const double* g, double* x, int n) {
  if (simd_level() == 2) return chol_solve_512(A.data(), g, x, n);
  const bool fma = simd_level() == 1;
  double* a = A.data();
  for (int kb = 0; kb < n; kb += kCholB) {
    const int ke = std::min(n, kb + kCholB);
    bool ok = true;
    if (fma) chol_panel_fma(a, n, kb, ke, ok);
    else chol_panel(a, n, kb, ke, ok);
    if (!ok) return false;
    if (ke - kb == kCholB) {
      if (fma) chol_trail_fma(a, n, kb, ke);
      else chol_trail_plain(a, n, kb, ke);
    } else {
      for (int k = kb; k < ke; ++k) {
        const double* Uk = a + (size_t)k * n;
        for (int i = ke; i < n; ++i) {
          double* Ai = a + (size_t)i * n;
          const double uki = Uk[i];
          for (int m = i; m < n; ++m) Ai[m] -= uki * Uk[m];
        }
      }
    }
  }
  std::vector<double> y(g, g + n);  // forward: U^T y = g
  for (int k = 0; k < n; ++k) {
    const double* Uk = a + (size_t)k * n;
    y[k] = y[k] / Uk[k];
    const double yk = y[k];
    for (int m = k + 1; m < n; ++m) y[m] -= Uk[m] * yk;
  }
  if (fma) {
    chol_back_fma(a, n, y.data(), x);
    return true;
  }
  for (int i = n - 1; i >= 0; --i) {  // back: U x = y
    const double* Ui = a + (size_t)i * n;
    double s = y[i];
    for (int k = i + 1; k < n; ++k) s -= Ui[k] * x[k];
    x[i] = s / Ui[i];
  }
  return true;
}

namespace {

// NonlinearFactorGraph::linearize at x into S; returns the graph error.  The
// x-independent information blocks (prior H = I/sigma^2, the linear factors' G) are
// summed once per LM run into `base` in factor order; each linearization starts from
// a copy of it and adds the rest (rhs / constant terms, then the pairs) in the same
// factor order, so every element sees the same sequence of additions as a fresh sum.
struct Assembler {
  const WinGraph& g;
  DenseSys base;
  explicit Assembler(const WinGraph& gr) : g(gr) {
    base.init(g.keys);
    const int D = base.D;
    for (const PriorF* P : g.priors) {
      const double inv = 1.0 / P->sigma;
      const int s = base.slot.at(P->key);
      for (int k = 0; k < 6; ++k) base.at(6 * s + k, 6 * s + k) += inv * inv;
    }
    for (const LinF* L : g.lins) {
      const int n = 6 * (int)L->keys.size(), m = n + 1;
      std::vector<int> col(n);
      for (size_t k = 0; k < L->keys.size(); ++k)
        for (int e = 0; e < 6; ++e) col[6 * k + e] = 6 * base.slot.at(L->keys[k]) + e;
      const double* I = L->info.data();
      for (int r = 0; r < n; ++r) {
        double* row = &base.A[(size_t)col[r] * (D + 1)];
        for (int c = 0; c < n; ++c) row[col[c]] += I[(size_t)r * m + c];
      }
    }
  }
  // S back to the base system.  A linearization changes only the entries the pairs'
  // 6 x 6 blocks ((i,i), (i,j), (j,i), (j,j)) and the rhs row / column cover (the prior
  // and linear factors' information is in the base; their rhs terms go to the last
  // row / column), so only those are copied back from the base — the same values a
  // full copy would give, at a fraction of the D^2 doubles.
  void reset(DenseSys& S) const {
    const int D = base.D, ld = D + 1;
    auto blk = [&](int si, int sj) {
      for (int r = 0; r < 6; ++r)
        std::memcpy(&S.A[(size_t)(6 * si + r) * ld + 6 * sj], &base.A[(size_t)(6 * si + r) * ld + 6 * sj],
                    6 * sizeof(double));
    };
    for (const auto& pr : g.pairs) {
      blk(pr.first, pr.first);
      blk(pr.first, pr.second);
      blk(pr.second, pr.first);
      blk(pr.second, pr.second);
    }
    for (int r = 0; r < D; ++r) S.A[(size_t)r * ld + D] = base.A[(size_t)r * ld + D];
    std::memcpy(&S.A[(size_t)D * ld], &base.A[(size_t)D * ld], ld * sizeof(double));
  }
  // started: the caller already issued lin_begin(x) (window_lm's first linearization,
  // launched before this Assembler was built)
  double run(const std::vector<Pose>& x, DenseSys& S, std::vector<double>& G, int& lins, bool started = false) const {
    const bool split = !g.pairs.empty() && g.lin_begin;
    if (split && !started) g.lin_begin(x);  // device work overlaps everything below up to lin_end
    if (S.D != base.D || S.keys != base.keys) S = base;
    else reset(S);
    G.assign(g.pairs.size() * kPairG, 0.0);
    if (!split && !g.pairs.empty()) {
      g.lin_pairs(x, G.data());
      ++lins;
    }
    const int D = S.D;
    double err = 0;
    for (const PriorF* P : g.priors) {  // rhs part of DenseSys::add_prior
      double l[6];
      logmap(compose(inverse(x[S.slot.at(P->key)]), P->mean), l);
      const double inv = 1.0 / P->sigma;
      const int s = S.slot.at(P->key);
      double f = 0;
      for (int k = 0; k < 6; ++k) {
        const double b = l[k] * inv;
        S.at(6 * s + k, D) += inv * b;
        S.at(D, 6 * s + k) += inv * b;
        f += b * b;
      }
      S.at(D, D) += f;
      err += 0.5 * f;
    }
    for (const LinF* L : g.lins) {  // rhs part of DenseSys::add_linf
      const int n = 6 * (int)L->keys.size(), m = n + 1;
      double d[6 * 64];
      std::vector<double> dv;
      double* dp = d;
      if (n > 6 * 64) {
        dv.resize(n);
        dp = dv.data();
      }
      for (size_t k = 0; k < L->keys.size(); ++k)
        logmap(compose(inverse(L->lin[k]), x[S.slot.at(L->keys[k])]), dp + 6 * k);
      const double* I = L->info.data();
      double dGd = 0, dg = 0;
      for (int r = 0; r < n; ++r) {
        const double* Ir = I + (size_t)r * m;
        const double sr = dot(Ir, dp, n);  // (I d)_r: vector partial sums on AVX-512 hosts
        const int cr = 6 * S.slot.at(L->keys[r / 6]) + r % 6;
        const double gr = Ir[n] - sr;
        S.at(cr, D) += gr;
        S.at(D, cr) += gr;
        dGd += dp[r] * sr;
        dg += dp[r] * Ir[n];
      }
      const double f = I[(size_t)n * m + n] + (dGd - 2.0 * dg);
      S.at(D, D) += f;
      err += 0.5 * f;
    }
    if (split) {
      g.lin_end(G.data());
      ++lins;
    }
    LMP_BEGIN(3);
    for (size_t p = 0; p < g.pairs.size(); ++p) {
      S.add_pair(g.pairs[p].first, g.pairs[p].second, &G[p * kPairG]);
      err += G[p * kPairG + 91];
    }
    LMP_END(3);
    return err;
  }
};

}  // namespace

// LevenbergMarquardtOptimizer over every window pose (NonlinearOptimizer::
// defaultOptimize + iterate/tryLambda).  Each trial is evaluated by a full
// linearization: it yields the error the accept test needs and, when accepted, the
// next iteration's system (one device launch per trial).
WinLMResult window_lm(const WinGraph& g, const std::vector<Pose>& x0) {
  WinLMResult R;
  R.x = x0;
  const bool split = !g.pairs.empty() && g.lin_begin;
  if (split) g.lin_begin(R.x);  // the first linearization runs while the base system is built
  const Assembler asmb(g);
  DenseSys S, Sn;
  std::vector<double> Gn;
  double err = asmb.run(R.x, S, R.G, R.lins, split);
  if (err <= 0.0) return R;
  double lambda = 1e-5;
  const int D = S.D;
  std::vector<double> gg(D), Hd((size_t)D * D), dx(D);
  auto iterate = [&]() {
    // H is the leading D x D block of S.A (row stride D + 1), read in place
    LMP_BEGIN(4);
    for (int r = 0; r < D; ++r) gg[r] = S.at(r, D);
    const double cc = S.at(D, D), oldLin = 0.5 * cc;
    LMP_END(4);
    for (;;) {
      LMP_BEGIN(0);
      for (int r = 0; r < D; ++r) {
        std::memcpy(&Hd[(size_t)r * D], &S.A[(size_t)r * (D + 1)], D * sizeof(double));
        Hd[(size_t)r * D + r] += lambda;
      }
      const bool ok = chol_solve(Hd, gg.data(), dx.data(), D);
      LMP_END(0);
      bool success = false, stop = false;
      std::vector<Pose> xn;
      double nerr = err;
      if (ok) {
        LMP_BEGIN(2);
        double dHd = 0, dg = 0;
        for (int r = 0; r < D; ++r) {
          const double h = dot(&S.A[(size_t)r * (D + 1)], dx.data(), D);
          dHd += dx[r] * h;
          dg += dx[r] * gg[r];
        }
        const double newLin = 0.5 * (dHd - 2 * dg + cc), linChange = oldLin - newLin;
        LMP_END(2);
        if (linChange >= 0) {
          LMP_BEGIN(5);
          xn.resize(R.x.size());
          for (size_t k = 0; k < R.x.size(); ++k) xn[k] = compose(R.x[k], expmap(&dx[6 * k]));
          LMP_END(5);
          LMP_BEGIN(1);
          g.trial_lin_change = linChange;
          g.trial_err = err;
          nerr = asmb.run(xn, Sn, Gn, R.lins);
          g.trial_lin_change = -1.0;
          LMP_END(1);
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
