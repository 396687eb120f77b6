// form_oracle.cpp — CPU restatement of FORM's scan-to-submap registration path.
//
// TEST INFRASTRUCTURE ONLY (see form_oracle.h): the checker for the HIP path and the
// CPU baseline timed by bench.py.  Parity vs the reference's OUTPUTS is unpinned:
// the reference cannot be built here and ships no golden vectors.
//
// Every function cites the reference file:line it restates.  Floating-point
// expression order follows the reference's Eigen/SSE2 evaluation (the reference
// CMakeLists.txt sets no -march, so x86-64 SSE2, no FMA):
//   * Vector4{f,d}::squaredNorm with a zero pad  ->  (dx*dx + dz*dz) + dy*dy
//   * Matrix3d * Vector3d                        ->  ((R0 p0 + R1 p1) + R2 p2)
// Build with -ffp-contract=off (oracle/Makefile).
#include "form_oracle.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

// ----------------------------------------------------------------------------
// parallel_for on a persistent worker pool: mirrors the reference's tbb::parallel_for
// sites (extraction.tpp:99-118 normals, matcher.hpp:86-100 match queries) and GTSAM's
// TBB-parallel NonlinearFactorGraph::linearize over the pair factors.  Like TBB's
// arena the workers live across calls (spinning briefly, then sleeping) and take
// chunks from a shared counter, the caller working too; spawning nthreads std::threads
// per call would cost milliseconds at 256 threads and misstate the CPU baseline.
// Every site writes results by index, so the chunking never changes a result.
// ----------------------------------------------------------------------------
class Pool {
 public:
  explicit Pool(int n) : nthreads_(n) {
    for (int t = 1; t < n; ++t) th_.emplace_back([this] { worker(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    for (auto& x : th_) x.join();
  }
  void run(size_t n, const std::function<void(size_t, size_t)>& fn) {
    std::lock_guard<std::mutex> call(call_m_);  // one parallel region at a time per pool
    fn_ = &fn;
    n_ = n;
    grain_ = std::max<size_t>(1, n / (4 * (size_t)nthreads_));
    next_.store(0);
    pending_.store((int)th_.size());
    {
      std::lock_guard<std::mutex> g(m_);
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    work();
    while (pending_.load() != 0) std::this_thread::yield();
  }

 private:
  void work() {
    for (;;) {
      const size_t b = next_.fetch_add(grain_);
      if (b >= n_) return;
      (*fn_)(b, std::min(n_, b + grain_));
    }
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      uint64_t g = gen_.load();
      for (int spin = 0; g == seen && spin < 20000; ++spin) g = gen_.load();  // ~tens of us
      if (g == seen) {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_.load() != seen; });
        g = gen_.load();
      }
      seen = g;
      if (stop_) return;
      work();
      pending_.fetch_sub(1);
    }
  }
  int nthreads_;
  std::vector<std::thread> th_;
  std::mutex m_, call_m_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<size_t> next_{0};
  std::atomic<int> pending_{0};
  const std::function<void(size_t, size_t)>* fn_ = nullptr;
  size_t n_ = 0, grain_ = 1;
  bool stop_ = false;
};

Pool& pool_for(int nthreads) {
  static std::mutex m;
  static std::map<int, std::unique_ptr<Pool>> pools;
  std::lock_guard<std::mutex> g(m);
  auto& p = pools[nthreads];
  if (!p) p = std::make_unique<Pool>(nthreads);
  return *p;
}

// min_n: below it the call runs serially (per-element work too small to share); the
// pair-factor sites pass 2 (each pair is thousands of rows).
void parallel_for(size_t n, int nthreads, const std::function<void(size_t, size_t)>& fn, size_t min_n = 256) {
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
  if (nthreads == 1 || n < min_n) {
    fn(0, n);
    return;
  }
  pool_for(nthreads).run(n, fn);
}

// ----------------------------------------------------------------------------
// SE(3) in GTSAM conventions (external API, restated; unpinned): Pose3 = (R, t),
// compose a*b = (Ra Rb, Ra tb + ta), transformFrom(p) = R p + t, inverse =
// (R^T, R^T(-t)); Expmap/Logmap with tangent [w; v] (GTSAM_POSE3_EXPMAP default).
// ----------------------------------------------------------------------------
struct Pose {
  double R[3][3];
  double t[3];
};

Pose pose_identity() {
  Pose p{};
  for (int i = 0; i < 3; ++i) p.R[i][i] = 1.0;
  return p;
}
Pose pose_from34(const double* a) {
  Pose p;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) p.R[i][j] = a[4 * i + j];
    p.t[i] = a[4 * i + 3];
  }
  return p;
}
void pose_to34(const Pose& p, double* a) {
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) a[4 * i + j] = p.R[i][j];
    a[4 * i + 3] = p.t[i];
  }
}
inline void matvec(const double R[3][3], const double v[3], double o[3]) {
  for (int i = 0; i < 3; ++i) o[i] = (R[i][0] * v[0] + R[i][1] * v[1]) + R[i][2] * v[2];
}
inline void matTvec(const double R[3][3], const double v[3], double o[3]) {
  for (int i = 0; i < 3; ++i) o[i] = (R[0][i] * v[0] + R[1][i] * v[1]) + R[2][i] * v[2];
}
inline void xform(const Pose& T, const double p[3], double o[3]) {
  double r[3];
  matvec(T.R, p, r);
  for (int i = 0; i < 3; ++i) o[i] = r[i] + T.t[i];
}
Pose compose(const Pose& a, const Pose& b) {
  Pose c;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      c.R[i][j] = (a.R[i][0] * b.R[0][j] + a.R[i][1] * b.R[1][j]) + a.R[i][2] * b.R[2][j];
  xform(a, b.t, c.t);
  return c;
}
Pose inverse(const Pose& a) {
  Pose c;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) c.R[i][j] = a.R[j][i];
  double nt[3] = {-a.t[0], -a.t[1], -a.t[2]};
  matvec(c.R, nt, c.t);
  return c;
}
void skew(const double w[3], double W[3][3]) {
  W[0][0] = 0;     W[0][1] = -w[2]; W[0][2] = w[1];
  W[1][0] = w[2];  W[1][1] = 0;     W[1][2] = -w[0];
  W[2][0] = -w[1]; W[2][1] = w[0];  W[2][2] = 0;
}
void cross(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
void rot_expmap(const double w[3], double R[3][3]) {
  double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  double W[3][3], W2[3][3];
  skew(w, W);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) W2[i][j] = W[i][0] * W[0][j] + W[i][1] * W[1][j] + W[i][2] * W[2][j];
  double A, B;
  if (th2 <= DBL_EPSILON) {
    A = 1.0;
    B = 0.5;
  } else {
    double th = std::sqrt(th2);
    A = std::sin(th) / th;
    B = (1.0 - std::cos(th)) / th2;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i][j] = (i == j ? 1.0 : 0.0) + A * W[i][j] + B * W2[i][j];
}
void rot_logmap(const double R[3][3], double w[3]) {
  const double tr = R[0][0] + R[1][1] + R[2][2];
  const double R32 = R[2][1], R23 = R[1][2], R13 = R[0][2], R31 = R[2][0], R21 = R[1][0],
               R12 = R[0][1];
  if (tr + 1.0 < 1e-10) {  // angle ~ pi
    double W[3];
    if (std::abs(R[2][2] + 1.0) > 1e-10) {
      double s = M_PI / std::sqrt(2.0 + 2.0 * R[2][2]);
      W[0] = s * R[0][2]; W[1] = s * R[1][2]; W[2] = s * (1.0 + R[2][2]);
    } else if (std::abs(R[1][1] + 1.0) > 1e-10) {
      double s = M_PI / std::sqrt(2.0 + 2.0 * R[1][1]);
      W[0] = s * R[0][1]; W[1] = s * (1.0 + R[1][1]); W[2] = s * R[2][1];
    } else {
      double s = M_PI / std::sqrt(2.0 + 2.0 * R[0][0]);
      W[0] = s * (1.0 + R[0][0]); W[1] = s * R[1][0]; W[2] = s * R[2][0];
    }
    w[0] = W[0]; w[1] = W[1]; w[2] = W[2];
    return;
  }
  double mag;
  const double tr_3 = tr - 3.0;
  if (tr_3 < -1e-7) {
    double theta = std::acos((tr - 1.0) / 2.0);
    mag = theta / (2.0 * std::sin(theta));
  } else {
    mag = 0.5 - tr_3 * tr_3 / 12.0;
  }
  w[0] = mag * (R32 - R23);
  w[1] = mag * (R13 - R31);
  w[2] = mag * (R21 - R12);
}
Pose pose_expmap(const double xi[6]) {
  Pose T;
  const double* w = xi;
  const double* v = xi + 3;
  rot_expmap(w, T.R);
  double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  double wxv[3], wxwxv[3];
  cross(w, v, wxv);
  cross(w, wxv, wxwxv);
  double a, b;
  if (th2 <= DBL_EPSILON) {
    a = 0.5;
    b = 1.0 / 6.0;
  } else {
    double th = std::sqrt(th2);
    a = (1.0 - std::cos(th)) / th2;
    b = (th - std::sin(th)) / (th2 * th);
  }
  for (int i = 0; i < 3; ++i) T.t[i] = v[i] + a * wxv[i] + b * wxwxv[i];
  return T;
}
void pose_logmap(const Pose& T, double xi[6]) {
  double w[3];
  rot_logmap(T.R, w);
  double t = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  xi[0] = w[0]; xi[1] = w[1]; xi[2] = w[2];
  if (t < 1e-10) {
    xi[3] = T.t[0]; xi[4] = T.t[1]; xi[5] = T.t[2];
    return;
  }
  double wn[3] = {w[0] / t, w[1] / t, w[2] / t};
  double W[3][3];
  skew(wn, W);
  double Tan = std::tan(0.5 * t);
  double WT[3], WWT[3];
  matvec(W, T.t, WT);
  matvec(W, WT, WWT);
  for (int i = 0; i < 3; ++i) xi[3 + i] = T.t[i] - (0.5 * t) * WT[i] + (1 - t / (2. * Tan)) * WWT[i];
}
// GTSAM Rot3::normalized (used by constraints.cpp:93-95): orthogonalize rows.
void rot_normalize(double R[3][3]) {
  double det = R[0][0] * (R[1][1] * R[2][2] - R[1][2] * R[2][1]) -
               R[0][1] * (R[1][0] * R[2][2] - R[1][2] * R[2][0]) +
               R[0][2] * (R[1][0] * R[2][1] - R[1][1] * R[2][0]);
  if (std::fabs(det - 1) < 1e-12) return;
  double x[3] = {R[0][0], R[0][1], R[0][2]}, y[3] = {R[1][0], R[1][1], R[1][2]};
  double err = x[0] * y[0] + x[1] * y[1] + x[2] * y[2];
  double xo[3], yo[3], zo[3];
  for (int i = 0; i < 3; ++i) {
    xo[i] = x[i] - (err / 2) * y[i];
    yo[i] = y[i] - (err / 2) * x[i];
  }
  cross(xo, yo, zo);
  double sx = 0.5 * (3 - (xo[0] * xo[0] + xo[1] * xo[1] + xo[2] * xo[2]));
  double sy = 0.5 * (3 - (yo[0] * yo[0] + yo[1] * yo[1] + yo[2] * yo[2]));
  double sz = 0.5 * (3 - (zo[0] * zo[0] + zo[1] * zo[1] + zo[2] * zo[2]));
  for (int i = 0; i < 3; ++i) {
    R[0][i] = sx * xo[i];
    R[1][i] = sy * yo[i];
    R[2][i] = sz * zo[i];
  }
}

// ----------------------------------------------------------------------------
// Stage 1 — FeatureExtractor (form/feature/extraction.tpp)
// ----------------------------------------------------------------------------
// PointXYZf::squaredNorm = vec4().squaredNorm() in float (utils.hpp:81-83); with
// SSE2 Packet4f and a zero pad it evaluates (x*x + z*z) + y*y.
inline float sqnorm4f(float x, float y, float z) { return (x * x + z * z) + y * y; }
inline float dist2f(const float* a, const float* b) {
  float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
  return (dx * dx + dz * dz) + dy * dy;
}

struct Extractor {
  const orc_extract_params& P;
  const float* s;  // R*C float4
  size_t R, C, k;
  explicit Extractor(const orc_extract_params& p, const float* xyzw)
      : P(p), s(xyzw), R(p.num_rows), C(p.num_columns), k(p.neighbor_points) {}
  const float* pt(size_t i) const { return s + 4 * i; }

  // compute_valid_points, extraction.tpp:136-180
  std::vector<uint8_t> valid_points() const {
    std::vector<uint8_t> mask(R * C, 1);
    for (size_t r = 0; r < R; ++r)
      for (size_t c = 0; c < C; ++c) {
        size_t idx = r * C + c;
        if (c < k || c >= C - k) {
          mask[idx] = 0;
          continue;
        }
        const float* p = pt(idx);
        const double range2 = sqnorm4f(p[0], p[1], p[2]);
        if (range2 < P.min_norm_squared || range2 > P.max_norm_squared) {
          mask[idx] = 0;
          for (size_t i = 1; i <= k; ++i) {
            mask[idx - i] = 0;
            mask[idx + i] = 0;
          }
          continue;
        }
      }
    return mask;
  }
  // compute_point_valid_points, extraction.tpp:182-222
  std::vector<uint8_t> point_valid_points() const {
    std::vector<uint8_t> mask(R * C, 1);
    for (size_t r = 0; r < R; ++r)
      for (size_t c = 0; c < C; ++c) {
        size_t idx = r * C + c;
        if (c < k || c >= C - k) {
          mask[idx] = 0;
          continue;
        }
        const float* p = pt(idx);
        const double range2 = sqnorm4f(p[0], p[1], p[2]);
        if (range2 < P.min_norm_squared || range2 > P.max_norm_squared) mask[idx] = 0;
      }
    return mask;
  }
  // compute_curvature, extraction.tpp:226-261 (double accumulate, float result)
  struct Curv {
    size_t index;
    float curvature;
  };
  std::vector<Curv> curvature(const std::vector<uint8_t>& mask) const {
    std::vector<Curv> out;
    out.reserve(R * C);
    for (size_t idx = 0; idx < R * C; ++idx) {
      if (!mask[idx]) {
        out.push_back({idx, FLT_MAX});
        continue;
      }
      double dx = -(2.0 * k) * (double)pt(idx)[0];
      double dy = -(2.0 * k) * (double)pt(idx)[1];
      double dz = -(2.0 * k) * (double)pt(idx)[2];
      for (size_t n = 1; n <= k; ++n) {
        dx = dx + (double)pt(idx - n)[0] + (double)pt(idx + n)[0];
        dy = dy + (double)pt(idx - n)[1] + (double)pt(idx + n)[1];
        dz = dz + (double)pt(idx - n)[2] + (double)pt(idx + n)[2];
      }
      out.push_back({idx, (float)(dx * dx + dy * dy + dz * dz)});
    }
    return out;
  }
  // extract_planar, extraction.tpp:332-358
  void extract_planar(size_t b, size_t e, const std::vector<Curv>& cv,
                      std::vector<uint32_t>& out, std::vector<uint8_t>& used) const {
    size_t n_feat = 0;
    for (size_t i = b; i < e; ++i) {
      const Curv c = cv[i];
      if (used[c.index] && (double)c.curvature < P.planar_threshold) {
        out.push_back((uint32_t)c.index);
        for (size_t n = 0; n < k; ++n) {
          used[c.index + n] = 0;
          used[c.index - n] = 0;
        }
        n_feat++;
      }
      if (n_feat > P.planar_feats_per_sector) break;
    }
  }
  // extract_point, extraction.tpp:360-399 (including the per-offset break quirk)
  void extract_point(size_t b, size_t e, std::vector<uint32_t>& out,
                     std::vector<uint8_t>& mask) const {
    size_t n_feat = 0;
    if (P.point_feats_per_sector == 0) return;
    std::vector<size_t> unused;
    for (size_t idx = b; idx < e; ++idx)
      if (mask[idx]) unused.push_back(idx);
    size_t factor = 1 + unused.size() / P.point_feats_per_sector;
    for (size_t off = 0; off < factor; ++off) {
      for (size_t ui = off; ui < unused.size(); ui += factor) {
        const size_t idx = unused[ui];
        if (mask[idx]) {
          out.push_back((uint32_t)idx);
          for (size_t n = 0; n < k; ++n) {
            mask[idx + n] = 0;
            mask[idx - n] = 0;
          }
          n_feat++;
        }
        if (n_feat > P.point_feats_per_sector) break;
      }
    }
  }
  // find_closest, extraction.tpp:402-420 (float dist promoted to double, strict <)
  long find_closest(const float* p, size_t b, size_t e, const std::vector<uint8_t>& valid) const {
    long best = -1;
    double md = std::numeric_limits<double>::max();
    for (size_t idx = b; idx < e; ++idx) {
      if (!valid[idx]) continue;
      const double d2 = dist2f(pt(idx), p);
      if (d2 < md) {
        md = d2;
        best = (long)idx;
      }
    }
    return best;
  }
  // find_neighbors, extraction.tpp:422-448 (+ direction first, stop at first miss)
  void find_neighbors(size_t idx, std::vector<const float*>& out) const {
    const float* p = pt(idx);
    const double r2 = P.radius * P.radius;
    for (size_t i = 1; i <= k; ++i) {
      const float* q = pt(idx + i);
      if ((double)dist2f(q, p) < r2) out.push_back(q);
      else break;
    }
    for (size_t i = 1; i <= k; ++i) {
      const float* q = pt(idx - i);
      if ((double)dist2f(q, p) < r2) out.push_back(q);
      else break;
    }
  }
  // compute_normal, extraction.tpp:263-329
  bool compute_normal(size_t idx, const std::vector<uint8_t>& valid, float nrm[3]) const {
    const size_t row = idx / C;
    const float* p = pt(idx);
    std::vector<const float*> nb;
    nb.reserve(40);
    find_neighbors(idx, nb);
    bool other = false;
    if (row > 0) {
      long ci = find_closest(p, C * (row - 1), C * row, valid);
      if (ci >= 0) {
        other = true;
        nb.push_back(pt(ci));
        find_neighbors((size_t)ci, nb);
      }
    }
    if (row < R - 1) {
      long ci = find_closest(p, C * (row + 1), C * (row + 2), valid);
      if (ci >= 0) {
        other = true;
        nb.push_back(pt(ci));
        find_neighbors((size_t)ci, nb);
      }
    }
    if (!other || nb.size() < P.min_points) return false;
    // A = (q - p) / n (float), Cov = A^T A (float, sequential over rows)
    const float nf = (float)nb.size();
    float cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (const float* q : nb) {
      float a[3];
      for (int d = 0; d < 3; ++d) a[d] = (q[d] - p[d]) / nf;
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) cov[r][c] = cov[r][c] + a[r] * a[c];
    }
    // smallest eigenvector; Eigen::SelfAdjointEigenSolver<Matrix3f> in the reference,
    // restated as a cyclic Jacobi sweep in double (sign is arbitrary in both).
    double A[3][3], V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) A[r][c] = cov[r][c];
    for (int sweep = 0; sweep < 64; ++sweep) {
      double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
      double dia = A[0][0] * A[0][0] + A[1][1] * A[1][1] + A[2][2] * A[2][2];
      if (off <= 1e-36 * dia || off == 0.0) break;
      for (int pp = 0; pp < 2; ++pp)
        for (int qq = pp + 1; qq < 3; ++qq) {
          double apq = A[pp][qq];
          if (apq == 0.0) continue;
          double theta = (A[qq][qq] - A[pp][pp]) / (2.0 * apq);
          double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
          double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
          for (int m = 0; m < 3; ++m) {  // A <- J^T A J
            double amp = A[m][pp], amq = A[m][qq];
            A[m][pp] = c * amp - s * amq;
            A[m][qq] = s * amp + c * amq;
          }
          for (int m = 0; m < 3; ++m) {
            double apm = A[pp][m], aqm = A[qq][m];
            A[pp][m] = c * apm - s * aqm;
            A[qq][m] = s * apm + c * aqm;
          }
          for (int m = 0; m < 3; ++m) {
            double vmp = V[m][pp], vmq = V[m][qq];
            V[m][pp] = c * vmp - s * vmq;
            V[m][qq] = s * vmp + c * vmq;
          }
        }
    }
    int mi = 0;
    if (A[1][1] < A[mi][mi]) mi = 1;
    if (A[2][2] < A[mi][mi]) mi = 2;
    double n[3] = {V[0][mi], V[1][mi], V[2][mi]};
    double nn = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    for (int d = 0; d < 3; ++d) n[d] /= nn;
    // deterministic sign: towards the sensor (n . p <= 0)
    double dp = n[0] * p[0] + n[1] * p[1] + n[2] * p[2];
    if (dp > 0)
      for (int d = 0; d < 3; ++d) n[d] = -n[d];
    for (int d = 0; d < 3; ++d) nrm[d] = (float)n[d];
    return true;
  }
};

// ----------------------------------------------------------------------------
// Stage 2 — VoxelMap (form/mapping/map.{hpp,tpp})
// ----------------------------------------------------------------------------
struct Key {
  int x, y, z;
  bool operator==(const Key& o) const { return x == o.x && y == o.y && z == o.z; }
};
struct KeyHash {  // kiss-icp hash, map.hpp:37-42
  size_t operator()(const Key& k) const {
    uint32_t a = (uint32_t)k.x, b = (uint32_t)k.y, c = (uint32_t)k.z;
    return (size_t)(a * 73856093u ^ b * 19349669u ^ c * 83492791u);
  }
};
struct Rec {
  double p[3];
  double n[3];
  uint64_t scan;
};
const int kShifts[27][3] = {  // map.tpp:54-68, fixed order
    {0, 0, 0},   {1, 0, 0},   {-1, 0, 0},  {0, 1, 0},   {0, -1, 0},  {0, 0, 1},  {0, 0, -1},
    {1, 1, 0},   {1, -1, 0},  {-1, 1, 0},  {-1, -1, 0}, {1, 0, 1},   {1, 0, -1}, {-1, 0, 1},
    {-1, 0, -1}, {0, 1, 1},   {0, 1, -1},  {0, -1, 1},  {0, -1, -1}, {1, 1, 1},  {1, 1, -1},
    {1, -1, 1},  {1, -1, -1}, {-1, 1, 1},  {-1, 1, -1}, {-1, -1, 1}, {-1, -1, -1}};

struct VMap {
  double w;
  int kind;  // 0 planar, 1 point
  std::unordered_map<Key, std::vector<Rec>, KeyHash> data;
  std::map<uint64_t, Pose> poses;
  // computeCoords, map.tpp:35-38
  Key coords(const double p[3]) const {
    return {(int)std::floor(p[0] / w), (int)std::floor(p[1] / w), (int)std::floor(p[2] / w)};
  }
  // to_voxel_map inner loop (map.tpp:139-143) + push_back (map.tpp:41-52)
  void add_scan(uint64_t scan, const Pose& T, const float* f, uint32_t n) {
    poses[scan] = T;
    const int stride = kind == 0 ? 6 : 3;
    for (uint32_t i = 0; i < n; ++i) {
      Rec r;
      double lp[3] = {f[stride * i], f[stride * i + 1], f[stride * i + 2]};
      xform(T, lp, r.p);  // PlanarFeat::transform_in_place, features.hpp:137-140
      if (kind == 0) {
        double ln[3] = {f[stride * i + 3], f[stride * i + 4], f[stride * i + 5]};
        matvec(T.R, ln, r.n);
      } else {
        r.n[0] = r.n[1] = r.n[2] = 0;
      }
      r.scan = scan;
      data[coords(r.p)].push_back(r);
    }
  }
  // find_closest, map.tpp:70-91 (27 shifts, insertion order, strict <)
  bool find_closest(const double q[3], Rec& best, double& bd) const {
    Key c = coords(q);
    bd = std::numeric_limits<double>::max();
    bool found = false;
    for (const auto& s : kShifts) {
      auto it = data.find(Key{c.x + s[0], c.y + s[1], c.z + s[2]});
      if (it == data.end()) continue;
      for (const Rec& r : it->second) {
        double dx = r.p[0] - q[0], dy = r.p[1] - q[1], dz = r.p[2] - q[2];
        double d2 = (dx * dx + dz * dz) + dy * dy;
        if (d2 < bd) {
          bd = d2;
          best = r;
          found = true;
        }
      }
    }
    return found;
  }
};

// ----------------------------------------------------------------------------
// Stage 3 — PlanePoint / PointPoint evaluateError (factor.cpp:30-128) and the
// whitened augmented-Hessian reduction of DenseFactor::linearize (gtsam.hpp:67-86,
// FastIsotropic::WhitenSystem gtsam.hpp:129-139: A *= 1/sigma, b *= 1/sigma).
// ----------------------------------------------------------------------------
// One plane row: r and H = [H_i (6) | H_j (6)]
void plane_row(const Pose& Ti, const Pose& Tj, const double* pi, const double* ni,
               const double* pj, double& r, double H[12]) {
  double wn[3], wpi[3], wpj[3], v[3];
  matvec(Ti.R, ni, wn);
  xform(Ti, pi, wpi);
  xform(Tj, pj, wpj);
  for (int d = 0; d < 3; ++d) v[d] = wpj[d] - wpi[d];
  r = (wn[0] * v[0] + wn[1] * v[1]) + wn[2] * v[2];
  double RTn[3], RTv[3], RjTn[3];
  matTvec(Ti.R, wn, RTn);
  matTvec(Ti.R, v, RTv);
  H[0] = RTn[1] * pi[2] - RTn[2] * pi[1] - RTv[1] * ni[2] + RTv[2] * ni[1];
  H[1] = RTn[2] * pi[0] - RTn[0] * pi[2] - RTv[2] * ni[0] + RTv[0] * ni[2];
  H[2] = RTn[0] * pi[1] - RTn[1] * pi[0] - RTv[0] * ni[1] + RTv[1] * ni[0];
  H[3] = -RTn[0];
  H[4] = -RTn[1];
  H[5] = -RTn[2];
  matTvec(Tj.R, wn, RjTn);
  H[6] = -RjTn[1] * pj[2] + RjTn[2] * pj[1];
  H[7] = -RjTn[2] * pj[0] + RjTn[0] * pj[2];
  H[8] = -RjTn[0] * pj[1] + RjTn[1] * pj[0];
  H[9] = RjTn[0];
  H[10] = RjTn[1];
  H[11] = RjTn[2];
}
// One point pair: 3 rows (x, y, z interleaved, factor.cpp:96-124)
void point_rows(const Pose& Ti, const Pose& Tj, const double* pi, const double* pj,
                double r[3], double H[3][12]) {
  double wpi[3], wpj[3];
  xform(Ti, pi, wpi);
  xform(Tj, pj, wpj);
  for (int a = 0; a < 3; ++a) {
    r[a] = wpj[a] - wpi[a];
    const double* Ri = Ti.R[a];
    const double Rn[3] = {Ri[0] * -1.0, Ri[1] * -1.0, Ri[2] * -1.0};
    H[a][0] = Rn[2] * pi[1] - Rn[1] * pi[2];
    H[a][1] = Rn[0] * pi[2] - Rn[2] * pi[0];
    H[a][2] = Rn[1] * pi[0] - Rn[0] * pi[1];
    H[a][3] = Rn[0];
    H[a][4] = Rn[1];
    H[a][5] = Rn[2];
    const double* Rj = Tj.R[a];
    H[a][6] = Rj[2] * pj[1] - Rj[1] * pj[2];
    H[a][7] = Rj[0] * pj[2] - Rj[2] * pj[0];
    H[a][8] = Rj[1] * pj[0] - Rj[0] * pj[1];
    H[a][9] = Rj[0];
    H[a][10] = Rj[1];
    H[a][11] = Rj[2];
  }
}
// Accumulate whitened row into packed upper triangle.
inline void accum(const double H[12], double r, double inv, int single, double* G) {
  double a[13];
  int m;
  if (single) {
    for (int c = 0; c < 6; ++c) a[c] = H[6 + c] * inv;
    a[6] = -r * inv;
    m = 7;
  } else {
    for (int c = 0; c < 12; ++c) a[c] = H[c] * inv;
    a[12] = -r * inv;
    m = 13;
  }
  int o = 0;
  for (int i = 0; i < m; ++i)
    for (int j = i; j < m; ++j) G[o++] += a[i] * a[j];
}

struct PairData {
  std::vector<double> ppi, pni, ppj;  // plane rows (3 doubles each)
  std::vector<double> tpi, tpj;       // point pairs
  uint32_t np() const { return (uint32_t)(ppi.size() / 3); }
  uint32_t nt() const { return (uint32_t)(tpi.size() / 3); }
};

void linearize_pair(const PairData& d, const Pose& Ti, const Pose& Tj, double sigma,
                    int single, double* G, double* err) {
  const double inv = 1.0 / sigma;
  const int ng = single ? 28 : 91;
  for (int i = 0; i < ng; ++i) G[i] = 0;
  double e = 0;
  for (uint32_t k = 0; k < d.np(); ++k) {
    double r, H[12];
    plane_row(Ti, Tj, &d.ppi[3 * k], &d.pni[3 * k], &d.ppj[3 * k], r, H);
    accum(H, r, inv, single, G);
    e += (r * inv) * (r * inv);
  }
  for (uint32_t k = 0; k < d.nt(); ++k) {
    double r[3], H[3][12];
    point_rows(Ti, Tj, &d.tpi[3 * k], &d.tpj[3 * k], r, H);
    for (int a = 0; a < 3; ++a) {
      accum(H[a], r[a], inv, single, G);
      e += (r[a] * inv) * (r[a] * inv);
    }
  }
  *err = 0.5 * e;
}
double error_pair(const PairData& d, const Pose& Ti, const Pose& Tj, double sigma) {
  const double inv = 1.0 / sigma;
  double e = 0;
  for (uint32_t k = 0; k < d.np(); ++k) {
    double r, H[12];
    plane_row(Ti, Tj, &d.ppi[3 * k], &d.pni[3 * k], &d.ppj[3 * k], r, H);
    e += (r * inv) * (r * inv);
  }
  for (uint32_t k = 0; k < d.nt(); ++k) {
    double r[3], H[3][12];
    point_rows(Ti, Tj, &d.tpi[3 * k], &d.tpj[3 * k], r, H);
    for (int a = 0; a < 3; ++a) e += (r[a] * inv) * (r[a] * inv);
  }
  return 0.5 * e;
}

// 6x6 Cholesky solve (dense, as gfg.optimizeDensely() for one variable)
bool chol_solve6(const double H[6][6], const double g[6], double x[6]) {
  double L[6][6] = {};
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = H[i][j];
      for (int k = 0; k < j; ++k) s -= L[i][k] * L[j][k];
      if (i == j) {
        if (s <= 0) return false;
        L[i][i] = std::sqrt(s);
      } else {
        L[i][j] = s / L[j][j];
      }
    }
  double y[6];
  for (int i = 0; i < 6; ++i) {
    double s = g[i];
    for (int k = 0; k < i; ++k) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < 6; ++k) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
  return true;
}

}  // namespace

namespace {
// Single-pose Levenberg-Marquardt on X(j) with every map pose fixed: the
// disable_smoothing mode (constraints.cpp:103-111, 235-250; BinaryFactorWrapper
// gtsam.hpp:144-170) driven by a restatement of GTSAM's NonlinearOptimizer::
// defaultOptimize + LevenbergMarquardtOptimizer::iterate/tryLambda with GTSAM's
// defaults (lambda0 1e-5, factor 10, upper bound 1e5, minModelFidelity 1e-3,
// rel/abs tol 1e-5, maxIterations 100).  External algorithm: parity unpinned.
struct LM {
  const std::vector<std::pair<Pose, const PairData*>>& pairs;
  double sigma;
  double lambda = 1e-5;
  double error_at(const Pose& Tj) const {
    double e = 0;
    for (auto& pr : pairs) e += error_pair(*pr.second, pr.first, Tj, sigma);
    return e;
  }
  // returns the new state (T, err) after one iterate()
  void iterate(Pose& T, double& err) {
    double Hs[6][6] = {}, g[6] = {}, c = 0;
    for (auto& pr : pairs) {
      double G[28], e;
      linearize_pair(*pr.second, pr.first, T, sigma, 1, G, &e);
      int o = 0;
      double full[7][7];
      for (int i = 0; i < 7; ++i)
        for (int j = i; j < 7; ++j) full[i][j] = full[j][i] = G[o++];
      for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < 6; ++j) Hs[i][j] += full[i][j];
        g[i] += full[i][6];
      }
      c += full[6][6];
    }
    const double oldLin = 0.5 * c;
    while (true) {
      double Hd[6][6];
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) Hd[i][j] = Hs[i][j] + (i == j ? lambda : 0.0);
      double dx[6];
      bool ok = chol_solve6(Hd, g, dx);
      bool success = false, stop = false;
      Pose Tn = T;
      double nerr = err;
      if (ok) {
        double dHd = 0, dg = 0;
        for (int i = 0; i < 6; ++i) {
          double h = 0;
          for (int j = 0; j < 6; ++j) h += Hs[i][j] * dx[j];
          dHd += dx[i] * h;
          dg += dx[i] * g[i];
        }
        double newLin = 0.5 * (dHd - 2 * dg + c);
        double linChange = oldLin - newLin;
        if (linChange >= 0) {
          Tn = compose(T, pose_expmap(dx));
          nerr = error_at(Tn);
          double costChange = err - nerr;
          if (linChange > DBL_EPSILON * oldLin) success = (costChange / linChange) > 1e-3;
          else success = true;
          if (std::abs(costChange) < 1e-5 * err) stop = true;
        }
      }
      if (success) {
        lambda = std::max(0.0, lambda / 10.0);
        T = Tn;
        err = nerr;
        return;
      } else if (!stop) {
        lambda *= 10.0;
        if (lambda >= 1e5) return;
      } else {
        return;
      }
    }
  }
  Pose optimize(const Pose& T0, int* iters_out) {
    Pose T = T0;
    double err = error_at(T);
    int iters = 0;
    if (err <= 0.0) {
      *iters_out = 0;
      return T;
    }
    double cur, newErr = err;
    bool conv;
    do {
      cur = newErr;
      iterate(T, err);
      ++iters;
      newErr = err;
      if (newErr <= 0.0) conv = true;
      else {
        double absDec = cur - newErr, relDec = absDec / cur;
        conv = (relDec <= 1e-5) || (absDec <= 1e-5);
      }
    } while (iters < 100 && !conv && std::isfinite(cur));
    *iters_out = iters;
    return T;
  }
};

// ----------------------------------------------------------------------------
// Smoothing mode — ConstraintManager's default (disable_smoothing = false,
// constraints.hpp:54-56): Levenberg-Marquardt over EVERY window pose with a dense
// solve (DenseLMOptimizer, gtsam.hpp:39-56: gfg.optimizeDensely()) on the graph of
// get_graph(fast) (constraints.cpp:252-308):
//   * m_other_factors: the prior on X(0) (step, constraints.cpp:217-220) and the
//     marginal LinearContainerFactors left by marginalize (:120-203);
//   * fast: the current scan's FeatureFactors + m_fast_linear, ONE HessianFactor of
//     every previous pair linearized at m_values when first needed (:268-288);
//   * full: every pair's FeatureFactor (:294-305).
// External GTSAM algorithms restated from their published behaviour (parity
// unpinned): PriorFactor<Pose3> (H = I, e = -Local(x, prior)), LinearContainerFactor
// (error / linearize of a HessianFactor at delta = Local(lin, x)), HessianFactor
// augmented information [G g; g^T f], partial Cholesky elimination, Values::retract
// (x * Expmap(delta)), LM damping H + lambda*I (diagonalDamping = false).
// ----------------------------------------------------------------------------
using Values = std::map<uint64_t, Pose>;

struct PriorF {  // PriorFactor<Pose3>, isotropic sigma (pose_noise = 1e-3, constraints.hpp:63)
  uint64_t key;
  Pose mean;
  double sigma;
};
struct LinF {  // LinearContainerFactor around a HessianFactor over `keys`
  std::vector<uint64_t> keys;
  std::vector<Pose> lin;     // linearization point per key
  std::vector<double> info;  // (6k+1)^2 augmented information [G g; g^T f], row-major
};
struct PairRef {  // one FeatureFactor(X(i), X(j)) (factor.cpp:131-186)
  uint64_t i, j;
  const PairData* d;
};

// Dense augmented system [H g; g^T c] over the window keys (Values order).
struct Sys {
  std::vector<uint64_t> keys;
  std::map<uint64_t, int> slot;
  int D = 0;
  std::vector<double> A;
  void init(const std::vector<uint64_t>& ks) {
    keys = ks;
    slot.clear();
    for (size_t k = 0; k < ks.size(); ++k) slot[ks[k]] = (int)k;
    D = 6 * (int)ks.size();
    A.assign((size_t)(D + 1) * (D + 1), 0.0);
  }
  double& at(int r, int c) { return A[(size_t)r * (D + 1) + c]; }
  // column of augmented index a of a factor whose key slots are ks (last = rhs)
  void add_block(const std::vector<int>& cols, const double* info) {  // info full (m x m)
    const int m = (int)cols.size();
    for (int a = 0; a < m; ++a)
      for (int b = 0; b < m; ++b) at(cols[a], cols[b]) += info[a * m + b];
  }
};

// LinearContainerFactor::linearize: G' = G, g' = g - G d, f' = f + d^T G d - 2 d^T g.
void linf_at(const LinF& L, const Values& x, std::vector<double>& out, double* err) {
  const int n = 6 * (int)L.keys.size(), m = n + 1;
  std::vector<double> d(n);
  for (size_t k = 0; k < L.keys.size(); ++k)
    pose_logmap(compose(inverse(L.lin[k]), x.at(L.keys[k])), &d[6 * k]);
  out = L.info;
  std::vector<double> Gd(n, 0.0);
  for (int r = 0; r < n; ++r) {
    double s = 0;
    for (int c = 0; c < n; ++c) s += L.info[r * m + c] * d[c];
    Gd[r] = s;
  }
  double dGd = 0, dg = 0;
  for (int r = 0; r < n; ++r) {
    dGd += d[r] * Gd[r];
    dg += d[r] * L.info[r * m + n];
  }
  for (int r = 0; r < n; ++r) {
    out[r * m + n] -= Gd[r];
    out[n * m + r] -= Gd[r];
  }
  out[n * m + n] += dGd - 2.0 * dg;
  if (err) *err = 0.5 * out[n * m + n];  // HessianFactor::error(delta) = 0.5 (f - 2 d^T g + d^T G d)
}

// PriorFactor<Pose3>::evaluateError: H = I, e = -Logmap(x^-1 * prior); whitened 1/sigma.
void prior_at(const PriorF& P, const Pose& x, double info[49], double* err) {
  double l[6];
  pose_logmap(compose(inverse(x), P.mean), l);
  const double inv = 1.0 / P.sigma;
  double a[7][7] = {};
  for (int k = 0; k < 6; ++k) a[k][k] = inv;  // A = I / sigma
  double b[6];
  for (int k = 0; k < 6; ++k) b[k] = l[k] * inv;  // b = -e / sigma
  std::fill(info, info + 49, 0.0);
  for (int r = 0; r < 6; ++r) {
    info[r * 7 + r] = inv * inv;
    info[r * 7 + 6] = info[6 * 7 + r] = inv * b[r];
  }
  double f = 0;
  for (int k = 0; k < 6; ++k) f += b[k] * b[k];
  info[48] = f;
  if (err) *err = 0.5 * f;
  (void)a;
}

// Cholesky solve of an n x n SPD system (row-major); false when not positive definite.
bool chol_solve(std::vector<double> H, const std::vector<double>& g, std::vector<double>& x, int n) {
  for (int j = 0; j < n; ++j) {
    double s = H[(size_t)j * n + j];
    for (int k = 0; k < j; ++k) s -= H[(size_t)j * n + k] * H[(size_t)j * n + k];
    if (!(s > 0)) return false;
    const double ljj = std::sqrt(s);
    H[(size_t)j * n + j] = ljj;
    for (int i = j + 1; i < n; ++i) {
      double t = H[(size_t)i * n + j];
      for (int k = 0; k < j; ++k) t -= H[(size_t)i * n + k] * H[(size_t)j * n + k];
      H[(size_t)i * n + j] = t / ljj;
    }
  }
  std::vector<double> y(n);
  for (int i = 0; i < n; ++i) {
    double s = g[i];
    for (int k = 0; k < i; ++k) s -= H[(size_t)i * n + k] * y[k];
    y[i] = s / H[(size_t)i * n + i];
  }
  x.assign(n, 0.0);
  for (int i = n - 1; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < n; ++k) s -= H[(size_t)k * n + i] * x[k];
    x[i] = s / H[(size_t)i * n + i];
  }
  return true;
}

// Columns of a pair's 13 x 13 augmented block in the window system.
std::vector<int> pair_cols(const Sys& S, uint64_t i, uint64_t j) {
  std::vector<int> c(13);
  const int si = S.slot.at(i), sj = S.slot.at(j);
  for (int k = 0; k < 6; ++k) {
    c[k] = 6 * si + k;
    c[6 + k] = 6 * sj + k;
  }
  c[12] = S.D;
  return c;
}
void unpack91(const double* G, double full[169]) {
  int o = 0;
  for (int a = 0; a < 13; ++a)
    for (int b = a; b < 13; ++b) full[a * 13 + b] = full[b * 13 + a] = G[o++];
}

struct WindowGraph {
  std::vector<const PriorF*> priors;
  std::vector<const LinF*> lins;
  std::vector<PairRef> pairs;
  double sigma;
  int nthreads;

  // NonlinearFactorGraph::linearize at x into the dense window system; returns the error.
  // Pair factors are linearized in parallel (GTSAM's TBB linearize), summed in order.
  double linearize(const Values& x, Sys& S) const {
    std::vector<uint64_t> ks;
    for (auto& [k, T] : x) ks.push_back(k);
    S.init(ks);
    std::vector<double> G(91 * pairs.size()), e(pairs.size());
    parallel_for(pairs.size(), nthreads, [&](size_t b, size_t en) {
      for (size_t p = b; p < en; ++p)
        linearize_pair(*pairs[p].d, x.at(pairs[p].i), x.at(pairs[p].j), sigma, 0, &G[91 * p], &e[p]);
    }, 2);
    double err = 0;
    for (auto* P : priors) {
      double info[49], pe;
      prior_at(*P, x.at(P->key), info, &pe);
      std::vector<int> cols(7);
      for (int k = 0; k < 6; ++k) cols[k] = 6 * S.slot.at(P->key) + k;
      cols[6] = S.D;
      S.add_block(cols, info);
      err += pe;
    }
    for (auto* L : lins) {
      std::vector<double> info;
      double le;
      linf_at(*L, x, info, &le);
      std::vector<int> cols;
      for (uint64_t k : L->keys)
        for (int d = 0; d < 6; ++d) cols.push_back(6 * S.slot.at(k) + d);
      cols.push_back(S.D);
      S.add_block(cols, info.data());
      err += le;
    }
    double full[169];
    for (size_t p = 0; p < pairs.size(); ++p) {
      unpack91(&G[91 * p], full);
      S.add_block(pair_cols(S, pairs[p].i, pairs[p].j), full);
      err += e[p];
    }
    return err;
  }
  double error(const Values& x) const {
    std::vector<double> e(pairs.size());
    parallel_for(pairs.size(), nthreads, [&](size_t b, size_t en) {
      for (size_t p = b; p < en; ++p) e[p] = error_pair(*pairs[p].d, x.at(pairs[p].i), x.at(pairs[p].j), sigma);
    }, 2);
    double err = 0;
    for (auto* P : priors) {
      double info[49], pe;
      prior_at(*P, x.at(P->key), info, &pe);
      err += pe;
    }
    for (auto* L : lins) {
      std::vector<double> info;
      double le;
      linf_at(*L, x, info, &le);
      err += le;
    }
    for (double v : e) err += v;
    return err;
  }
};

Values retract(const Values& x, const std::vector<double>& dx) {  // Values::retract
  Values o;
  size_t k = 0;
  for (auto& [key, T] : x) o[key] = compose(T, pose_expmap(&dx[6 * k++]));
  return o;
}

// LevenbergMarquardtOptimizer (GTSAM defaults, as LM above) over every window pose.
Values window_lm(const WindowGraph& g, const Values& x0, int* iters_out) {
  double lambda = 1e-5;
  Values x = x0;
  double err = g.error(x);
  int iters = 0;
  if (err <= 0.0) {
    *iters_out = 0;
    return x;
  }
  auto iterate = [&]() {
    Sys S;
    g.linearize(x, S);
    const int D = S.D;
    std::vector<double> H((size_t)D * D), gg(D);
    for (int r = 0; r < D; ++r) {
      for (int c = 0; c < D; ++c) H[(size_t)r * D + c] = S.at(r, c);
      gg[r] = S.at(r, D);
    }
    const double cc = S.at(D, D), oldLin = 0.5 * cc;
    while (true) {
      std::vector<double> Hd = H, dx;
      for (int r = 0; r < D; ++r) Hd[(size_t)r * D + r] += lambda;
      const bool ok = chol_solve(Hd, gg, dx, D);
      bool success = false, stop = false;
      Values xn;
      double nerr = err;
      if (ok) {
        double dHd = 0, dg = 0;
        for (int r = 0; r < D; ++r) {
          double h = 0;
          for (int c = 0; c < D; ++c) h += H[(size_t)r * D + c] * dx[c];
          dHd += dx[r] * h;
          dg += dx[r] * gg[r];
        }
        const double newLin = 0.5 * (dHd - 2 * dg + cc), linChange = oldLin - newLin;
        if (linChange >= 0) {
          xn = retract(x, dx);
          nerr = g.error(xn);
          const double costChange = err - nerr;
          if (linChange > DBL_EPSILON * oldLin) success = (costChange / linChange) > 1e-3;
          else success = true;
          if (std::abs(costChange) < 1e-5 * err) stop = true;
        }
      }
      if (success) {
        lambda = std::max(0.0, lambda / 10.0);
        x = xn;
        err = nerr;
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
    ++iters;
    newErr = err;
    if (newErr <= 0.0) conv = true;
    else {
      const double absDec = cur - newErr, relDec = absDec / cur;
      conv = (relDec <= 1e-5) || (absDec <= 1e-5);
    }
  } while (iters < 100 && !conv && std::isfinite(cur));
  *iters_out = iters;
  return x;
}

// Schur complement of the augmented system eliminating the first nm columns (partial
// Cholesky elimination, GaussianFactorGraph::eliminatePartialMultifrontal): returns
// the (n - nm + 1)^2 augmented information on the rest; false if the eliminated block
// is not positive definite.
bool schur(const std::vector<double>& A, int n, int nm, std::vector<double>& out) {
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
  // Y = L^-1 A_MR  (nm x r)
  std::vector<double> Y((size_t)nm * r);
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

// KeyScanner::step (keyscanner.cpp:29-91), restated for the oracle pipeline.
struct KScan {
  uint64_t idx;
  size_t unused = 0, size = 0;
};
struct KeyScanner {
  const orc_params& P;
  std::deque<KScan> recent, key;
  explicit KeyScanner(const orc_params& p) : P(p) {}
  uint64_t oldest_rf() const { return recent.empty() ? 0 : recent.front().idx; }
  std::vector<uint64_t> step(uint64_t idx, size_t size, const std::function<size_t(uint64_t)>& conn) {
    if (idx == 0) key.push_back({idx, 0, size});
    else recent.push_back({idx, 0, size});
    std::vector<uint64_t> marg;
    if (recent.size() > P.max_num_recent_scans) {
      KScan rf = recent.front();
      recent.pop_front();
      double ratio = (double)conn(rf.idx) / (double)(rf.size * recent.size());
      if (ratio > P.keyscan_match_ratio) key.push_back(rf);
      else marg.push_back(rf.idx);
    }
    std::set<uint64_t> fin;
    for (auto& kf : key) {
      if (conn(kf.idx) > 0) kf.unused = 0;
      else ++kf.unused;
      if ((int64_t)kf.unused > P.max_steps_unused_keyscan) {
        marg.push_back(kf.idx);
        fin.insert(kf.idx);
      }
    }
    key.erase(std::remove_if(key.begin(), key.end(), [&](const KScan& f) { return fin.count(f.idx) > 0; }),
              key.end());
    if (P.max_num_keyscans > 0 && (int64_t)key.size() > P.max_num_keyscans) {
      marg.push_back(key.front().idx);
      key.pop_front();
    }
    return marg;
  }
};

struct Estimator {
  orc_params P;
  int nthreads;
  KeyScanner ks;
  uint64_t scan = 0;
  bool init = false;
  std::map<uint64_t, Pose> values;
  // keypoint store (local frames): planar 6 floats, point 3 floats
  std::map<uint64_t, std::vector<float>> kp_planar, kp_point;
  // m_constraints[j][i] -> (planar count, point count)
  std::map<uint64_t, std::map<uint64_t, std::pair<size_t, size_t>>> cons;
  // smoothing-mode state (ConstraintManager members, constraints.hpp:74-101)
  std::map<uint64_t, std::map<uint64_t, PairData>> pdata;  // m_constraints[j][i] rows
  std::vector<PriorF> priors;                              // m_other_factors: priors
  std::vector<LinF> margs;                                 // m_other_factors: marginals
  bool have_fast = false;                                  // m_fast_linear
  LinF fast;
  explicit Estimator(const orc_params& p, int nt) : P(p), nthreads(nt), ks(P) {}

  // Linearize `prs` (+ priors / linear factors) at `values` into a Sys over `order`.
  void linearize_into(Sys& S, const std::vector<uint64_t>& order, const std::vector<PairRef>& prs,
                      const std::vector<const PriorF*>& pri, const std::vector<const LinF*>& lfs) const {
    WindowGraph g{pri, lfs, prs, P.planar_constraint_sigma, nthreads};
    Values sub;
    for (uint64_t k : order) sub[k] = values.at(k);
    g.linearize(sub, S);  // Values order (sorted)
    if (order != S.keys) {  // permute into `order`
      Sys T;
      T.init(order);
      std::vector<int> map(S.D + 1);
      for (size_t k = 0; k < S.keys.size(); ++k)
        for (int d = 0; d < 6; ++d) map[6 * k + d] = 6 * T.slot.at(S.keys[k]) + d;
      map[S.D] = T.D;
      for (int r = 0; r <= S.D; ++r)
        for (int c = 0; c <= S.D; ++c) T.at(map[r], map[c]) = S.at(r, c);
      S = T;
    }
  }
  // ConstraintManager::optimize (constraints.cpp:103-118) in smoothing mode
  Values optimize_window(bool fast_mode, int* iters) {
    std::vector<const PriorF*> pri;
    std::vector<const LinF*> lfs;
    for (auto& p : priors) pri.push_back(&p);
    for (auto& m : margs) lfs.push_back(&m);
    std::vector<PairRef> prs;
    for (auto& [j, m] : pdata)
      for (auto& [i, d] : m) {
        if (d.np() + d.nt() == 0) continue;  // is_empty (constraints.cpp:34-37)
        if (fast_mode && j != scan) continue;
        prs.push_back({i, j, &d});
      }
    if (fast_mode) {
      if (!have_fast) {  // m_fast_linear: every previous pair at m_values (:268-288)
        std::vector<PairRef> prev;
        std::set<uint64_t> ks;
        for (auto& [j, m] : pdata)
          for (auto& [i, d] : m)
            if (j != scan && d.np() + d.nt() > 0) {
              prev.push_back({i, j, &d});
              ks.insert(i);
              ks.insert(j);
            }
        fast = LinF{};
        if (!prev.empty()) {
          std::vector<uint64_t> order(ks.begin(), ks.end());
          Sys S;
          linearize_into(S, order, prev, {}, {});
          fast.keys = order;
          for (uint64_t k : order) fast.lin.push_back(values.at(k));
          fast.info = S.A;
        }
        have_fast = true;
      }
      if (!fast.keys.empty()) lfs.push_back(&fast);
    }
    WindowGraph g{pri, lfs, prs, P.planar_constraint_sigma, nthreads};
    return window_lm(g, values, iters);
  }
  // ConstraintManager::marginalize (constraints.cpp:120-203): every factor touching a
  // marginalized key is linearized at m_values and the keys are eliminated; the
  // marginal on the remaining keys becomes a LinearContainerFactor.
  void marginalize(const std::vector<uint64_t>& marg) {
    std::set<uint64_t> M;
    for (uint64_t m : marg)
      if (values.count(m)) M.insert(m);
    if (M.empty()) return;
    std::set<uint64_t> keys(M.begin(), M.end());
    std::vector<PriorF> dp;
    std::vector<LinF> dl;
    for (auto it = priors.begin(); it != priors.end();)
      if (M.count(it->key)) {
        dp.push_back(*it);
        it = priors.erase(it);
      } else ++it;
    for (auto it = margs.begin(); it != margs.end();) {
      bool hit = false;
      for (uint64_t k : it->keys) hit |= M.count(k) > 0;
      if (hit) {
        for (uint64_t k : it->keys) keys.insert(k);
        dl.push_back(std::move(*it));
        it = margs.erase(it);
      } else ++it;
    }
    std::vector<PairRef> prs;
    for (auto& [j, m] : pdata)
      for (auto& [i, d] : m)
        if (d.np() + d.nt() > 0 && (M.count(i) || M.count(j))) {
          prs.push_back({i, j, &d});
          keys.insert(i);
          keys.insert(j);
        }
    std::vector<uint64_t> order(M.begin(), M.end()), rest;
    for (uint64_t k : keys)
      if (!M.count(k)) rest.push_back(k);
    order.insert(order.end(), rest.begin(), rest.end());
    std::vector<const PriorF*> pri;
    std::vector<const LinF*> lfs;
    for (auto& p : dp) pri.push_back(&p);
    for (auto& l : dl) lfs.push_back(&l);
    Sys S;
    linearize_into(S, order, prs, pri, lfs);
    LinF L;
    if (!rest.empty() && schur(S.A, S.D, 6 * (int)M.size(), L.info)) {
      L.keys = rest;
      for (uint64_t k : rest) L.lin.push_back(values.at(k));
      margs.push_back(std::move(L));
    }
  }

  // ConstraintManager::predict_next, constraints.cpp:71-101
  Pose predict_next() const {
    if (!init) return pose_identity();
    uint64_t s = scan + 1;
    bool pe = s > 0 && values.count(s - 1), ppe = s > 1 && values.count(s - 2);
    if (pe && ppe) {
      Pose prev = values.at(s - 1), pp = values.at(s - 2);
      Pose pr = compose(prev, compose(inverse(pp), prev));
      rot_normalize(pr.R);
      return pr;
    } else if (pe) {
      return values.at(s - 1);
    }
    return pose_identity();
  }
  size_t num_recent_connections(uint64_t s, uint64_t oldest) const {
    size_t c = 0;
    for (auto& [j, m] : cons) {
      if (j < oldest) continue;
      auto it = m.find(s);
      if (it != m.end()) c += it->second.first + it->second.second;
    }
    return c;
  }

  int register_scan(const float* xyzw, size_t n, double* pose_out, uint32_t* stats, double* tms) {
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    const auto& E = P.extraction;
    if (n != (size_t)E.num_rows * (size_t)E.num_columns) return -1;
    // step(), constraints.cpp:206-223
    Pose pred = predict_next();
    if (init) ++scan;
    init = true;
    values[scan] = pred;
    have_fast = false;  // step() resets m_fast_linear (constraints.cpp:214)
    if (scan == 0) priors.push_back({0, pred, 1e-3});  // addPrior (:217-220)
    cons[scan];  // get_constraints creates buckets for every other scan in values
    for (auto& [i, T] : values)
      if (i != scan) cons[scan][i] = {0, 0};
    // extract
    const size_t cap_sel = (size_t)E.num_rows * E.num_sectors * (E.planar_feats_per_sector + 1);
    std::vector<uint32_t> sel(cap_sel), pidx(n);
    std::vector<uint8_t> ok(cap_sel);
    std::vector<float> nrm(3 * cap_sel);
    uint32_t nsel = 0, npt = 0;
    orc_extract(&E, xyzw, n, nthreads, sel.data(), &nsel, ok.data(), nrm.data(), pidx.data(), &npt,
                nullptr, nullptr, nullptr);
    std::vector<float> qpl, qpt;
    for (uint32_t i = 0; i < nsel; ++i)
      if (ok[i]) {
        const float* p = xyzw + 4 * (size_t)sel[i];
        qpl.insert(qpl.end(), {p[0], p[1], p[2], nrm[3 * i], nrm[3 * i + 1], nrm[3 * i + 2]});
      }
    for (uint32_t i = 0; i < npt; ++i) {
      const float* p = xyzw + 4 * (size_t)pidx[i];
      qpt.insert(qpt.end(), {p[0], p[1], p[2]});
    }
    const uint32_t nq[2] = {(uint32_t)(qpl.size() / 6), (uint32_t)(qpt.size() / 3)};
    auto t1 = clk::now();
    // to_voxel_map x2 (form.cpp:61-65), voxel width = max_dist_matching
    VMap maps[2] = {{P.max_dist_matching, 0, {}, {}}, {P.max_dist_matching, 1, {}, {}}};
    for (auto& [s, v] : kp_planar) maps[0].add_scan(s, values.at(s), v.data(), (uint32_t)(v.size() / 6));
    for (auto& [s, v] : kp_point) maps[1].add_scan(s, values.at(s), v.data(), (uint32_t)(v.size() / 3));
    auto t2 = clk::now();
    // ICP loop, form.cpp:67-89
    std::map<uint64_t, PairData> local_pairs;
    std::map<uint64_t, PairData>& pairs = P.disable_smoothing ? local_pairs : pdata[scan];
    std::vector<uint8_t> found[2];
    std::vector<double> d2s[2];
    int icp = 0, lm_total = 0;
    for (uint32_t it = 0; it < P.max_num_rematches; ++it) {
      ++icp;
      Pose before = values.at(scan);
      double bj[12];
      pose_to34(before, bj);
      for (auto& [i, pd] : pairs) pd = PairData{};
      for (int I = 0; I < 2; ++I) {
        if (nq[I] == 0) continue;  // matcher.hpp:72-74
        const std::vector<float>& Q = I == 0 ? qpl : qpt;
        found[I].assign(nq[I], 0);
        d2s[I].assign(nq[I], 0);
        std::vector<uint64_t> sc(nq[I]);
        std::vector<double> pi(3 * nq[I]), ni(3 * nq[I]);
        orc_map_match(&maps[I], Q.data(), nq[I], bj, nthreads, found[I].data(), sc.data(),
                      d2s[I].data(), pi.data(), ni.data());
        const double md2 = P.max_dist_matching * P.max_dist_matching;
        for (uint32_t q = 0; q < nq[I]; ++q) {
          if (!(d2s[I][q] < md2)) continue;
          PairData& pd = pairs[sc[q]];
          const int st = I == 0 ? 6 : 3;
          const double pj[3] = {Q[st * q], Q[st * q + 1], Q[st * q + 2]};
          if (I == 0) {
            pd.ppi.insert(pd.ppi.end(), &pi[3 * q], &pi[3 * q + 3]);
            pd.pni.insert(pd.pni.end(), &ni[3 * q], &ni[3 * q + 3]);
            pd.ppj.insert(pd.ppj.end(), pj, pj + 3);
          } else {
            pd.tpi.insert(pd.tpi.end(), &pi[3 * q], &pi[3 * q + 3]);
            pd.tpj.insert(pd.tpj.end(), pj, pj + 3);
          }
        }
      }
      int li = 0;
      Pose after;
      if (P.disable_smoothing) {
        std::vector<std::pair<Pose, const PairData*>> lp;
        for (auto& [i, pd] : pairs)
          if (pd.np() + pd.nt() > 0) lp.push_back({values.at(i), &pd});
        LM lm{lp, P.planar_constraint_sigma};
        after = lm.optimize(before, &li);
      } else {
        after = optimize_window(true, &li).at(scan);
      }
      lm_total += li;
      double xi[6];
      pose_logmap(compose(inverse(before), after), xi);
      double dn = 0;
      for (double x : xi) dn += x * x;
      if (std::sqrt(dn) < P.new_pose_threshold) break;
      values[scan] = after;
    }
    // optimize(false) (form.cpp:92-93)
    if (!P.disable_smoothing) {
      int li = 0;
      values = optimize_window(false, &li);  // update_values (same size: replace)
      lm_total += li;
    } else {
      std::vector<std::pair<Pose, const PairData*>> lp;
      for (auto& [i, pd] : pairs)
        if (pd.np() + pd.nt() > 0) lp.push_back({values.at(i), &pd});
      LM lm{lp, P.planar_constraint_sigma};
      int li = 0;
      values[scan] = lm.optimize(values.at(scan), &li);
      lm_total += li;
    }
    // record constraint counts of the last ICP iteration
    size_t mpl = 0, mpt = 0;
    for (auto& [i, pd] : pairs) {
      cons[scan][i] = {pd.np(), pd.nt()};
      mpl += pd.np();
      mpt += pd.nt();
    }
    auto t3 = clk::now();
    // insert_matches (map.tpp:148-165) from the last match call
    const double mind2 = P.min_dist_map * P.min_dist_map;
    for (int I = 0; I < 2; ++I) {
      if (nq[I] == 0) continue;
      auto& store = I == 0 ? kp_planar[scan] : kp_point[scan];
      const std::vector<float>& Q = I == 0 ? qpl : qpt;
      const int st = I == 0 ? 6 : 3;
      for (uint32_t q = 0; q < nq[I]; ++q)
        if (!found[I][q] || d2s[I][q] > mind2) store.insert(store.end(), &Q[st * q], &Q[st * q + st]);
    }
    // KeyScanner::step + marginalize (form.cpp:98-111)
    auto marg = ks.step(scan, nq[0] + nq[1],
                        [&](uint64_t i) { return num_recent_connections(i, ks.oldest_rf()); });
    if (!P.disable_smoothing) marginalize(marg);
    for (uint64_t m : marg) {
      values.erase(m);
      cons.erase(m);
      for (auto& [j, mm] : cons) mm.erase(m);
      pdata.erase(m);
      for (auto& [j, mm] : pdata) mm.erase(m);
      kp_planar.erase(m);
      kp_point.erase(m);
    }
    pose_to34(values.at(scan), pose_out);
    if (stats) {
      stats[0] = nq[0];
      stats[1] = nq[1];
      stats[2] = icp;
      stats[3] = lm_total;
      stats[4] = (uint32_t)mpl;
      stats[5] = (uint32_t)mpt;
    }
    if (tms) {
      auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      tms[0] = ms(t0, t1);
      tms[1] = ms(t1, t2);
      tms[2] = ms(t2, t3);
      tms[3] = ms(t0, clk::now());
    }
    return 0;
  }
};
}  // namespace

// ============================================================================
// C API
// ============================================================================
extern "C" {

void orc_default_params(orc_params* p) {
  std::memset(p, 0, sizeof(*p));
  auto& e = p->extraction;  // extraction.hpp:59-88
  e.neighbor_points = 5;
  e.num_sectors = 6;
  e.planar_threshold = 1.0;
  e.planar_feats_per_sector = 50;
  e.point_feats_per_sector = 3;
  e.radius = 1.0;
  e.min_points = 5;
  e.min_norm_squared = 1.0;
  e.max_norm_squared = 100.0 * 100.0;
  e.num_columns = 1024;
  e.num_rows = 64;
  p->max_dist_matching = 0.8;  // matcher.hpp:32-41
  p->new_pose_threshold = 1e-4;
  p->max_num_rematches = 30;
  p->planar_constraint_sigma = 0.1;  // constraints.hpp:60
  p->disable_smoothing = 0;          // constraints.hpp:56 default: smoothing (1: single-pose ablation)
  p->max_num_keyscans = 50;          // keyscanner.hpp:55-64
  p->max_steps_unused_keyscan = 10;
  p->max_num_recent_scans = 10;
  p->keyscan_match_ratio = 0.1;
  p->min_dist_map = 0.1;  // map.hpp:97-100
}

int orc_extract(const orc_extract_params* p, const float* xyzw, size_t n_points, int nthreads,
                uint32_t* sel_idx, uint32_t* n_sel, uint8_t* normal_ok, float* normals,
                uint32_t* point_idx, uint32_t* n_point, uint8_t* planar_mask,
                uint8_t* point_mask, float* curvature_out) {
  // extract, extraction.tpp:29-132
  const size_t R = p->num_rows, C = p->num_columns;
  if (n_points != R * C) return -1;  // extraction.tpp:141-145 throws
  Extractor X(*p, xyzw);
  const size_t pps = C / p->num_sectors;
  auto valid = X.valid_points();
  auto curv = X.curvature(valid);
  if (curvature_out)
    for (size_t i = 0; i < R * C; ++i) curvature_out[i] = curv[i].curvature;
  std::vector<uint32_t> planar;
  std::vector<uint8_t> used = valid;
  for (size_t r = 0; r < R; ++r)
    for (size_t s = 0; s < p->num_sectors; ++s) {
      const size_t b = r * C + s * pps;
      const size_t e = (s == p->num_sectors - 1) ? (r + 1) * C : b + pps;
      // std::sort is unstable (extraction.tpp:57-58); restated with the index as the
      // tie-break so the order is defined (parity hazard 1).
      std::sort(curv.begin() + b, curv.begin() + e, [](const Extractor::Curv& a, const Extractor::Curv& c) {
        return a.curvature < c.curvature || (a.curvature == c.curvature && a.index < c.index);
      });
      X.extract_planar(b, e, curv, planar, used);
    }
  auto vpm = X.point_valid_points();
  if (planar_mask) std::memcpy(planar_mask, valid.data(), R * C);
  if (point_mask) std::memcpy(point_mask, vpm.data(), R * C);
  for (size_t i = 0; i < R * C; ++i) vpm[i] = (used[i] == valid[i]) && vpm[i];
  std::vector<uint32_t> points;
  for (size_t r = 0; r < R; ++r)
    for (size_t s = 0; s < p->num_sectors; ++s) {
      const size_t b = r * C + s * pps;
      const size_t e = (s == p->num_sectors - 1) ? (r + 1) * C : b + pps;
      X.extract_point(b, e, points, vpm);
    }
  // normals: tbb::parallel_for site (extraction.tpp:99-118)
  parallel_for(planar.size(), nthreads, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) normal_ok[i] = X.compute_normal(planar[i], valid, normals + 3 * i) ? 1 : 0;
  });
  std::memcpy(sel_idx, planar.data(), planar.size() * 4);
  *n_sel = (uint32_t)planar.size();
  std::memcpy(point_idx, points.data(), points.size() * 4);
  *n_point = (uint32_t)points.size();
  return 0;
}

void* orc_map_new(double w, int kind) { return new VMap{w, kind, {}, {}}; }
void orc_map_free(void* m) { delete static_cast<VMap*>(m); }
void orc_map_add_scan(void* m, uint64_t scan, const double pose34[12], const float* f, uint32_t n) {
  static_cast<VMap*>(m)->add_scan(scan, pose_from34(pose34), f, n);
}
uint64_t orc_map_num_voxels(void* m) { return static_cast<VMap*>(m)->data.size(); }

void orc_map_match(void* mp, const float* Q, uint32_t nq, const double pose_j34[12], int nthreads,
                   uint8_t* found, uint64_t* scan, double* d2, double* pi, double* ni) {
  // Matcher::match, matcher.hpp:67-112
  const VMap& M = *static_cast<VMap*>(mp);
  const Pose Tj = pose_from34(pose_j34);
  const int st = M.kind == 0 ? 6 : 3;
  parallel_for(nq, nthreads, [&](size_t b, size_t e) {
    for (size_t q = b; q < e; ++q) {
      double lp[3] = {Q[st * q], Q[st * q + 1], Q[st * q + 2]}, wp[3];
      xform(Tj, lp, wp);
      Rec best;
      double bd;
      bool f = M.find_closest(wp, best, bd);
      found[q] = f;
      d2[q] = bd;
      if (f) {
        Pose inv = inverse(M.poses.at(best.scan));  // matcher.hpp:92-96 round trip
        xform(inv, best.p, &pi[3 * q]);
        matvec(inv.R, best.n, &ni[3 * q]);
        scan[q] = best.scan;
      } else {
        scan[q] = ~0ull;
        for (int d = 0; d < 3; ++d) pi[3 * q + d] = ni[3 * q + d] = 0;
      }
    }
  });
}

void orc_linearize(uint32_t K, const uint32_t* np, const double* ppi, const double* pni,
                   const double* ppj, const uint32_t* nt, const double* tpi, const double* tpj,
                   const double* poses_i, const double* poses_j, double sigma, int single,
                   double* G, double* err) {
  size_t op = 0, ot = 0;
  const int ng = single ? 28 : 91;
  for (uint32_t k = 0; k < K; ++k) {
    PairData d;
    d.ppi.assign(ppi + 3 * op, ppi + 3 * (op + np[k]));
    d.pni.assign(pni + 3 * op, pni + 3 * (op + np[k]));
    d.ppj.assign(ppj + 3 * op, ppj + 3 * (op + np[k]));
    d.tpi.assign(tpi + 3 * ot, tpi + 3 * (ot + nt[k]));
    d.tpj.assign(tpj + 3 * ot, tpj + 3 * (ot + nt[k]));
    op += np[k];
    ot += nt[k];
    linearize_pair(d, pose_from34(poses_i + 12 * k), pose_from34(poses_j + 12 * k), sigma, single,
                   G + (size_t)ng * k, err + k);
  }
}

void orc_factor_rows(uint32_t np, const double* ppi, const double* pni, const double* ppj,
                     uint32_t nt, const double* tpi, const double* tpj, const double pose_i[12],
                     const double pose_j[12], double* r, double* J) {
  Pose Ti = pose_from34(pose_i), Tj = pose_from34(pose_j);
  size_t row = 0;
  for (uint32_t k = 0; k < np; ++k, ++row) plane_row(Ti, Tj, ppi + 3 * k, pni + 3 * k, ppj + 3 * k, r[row], J + 12 * row);
  for (uint32_t k = 0; k < nt; ++k) {
    double rr[3], H[3][12];
    point_rows(Ti, Tj, tpi + 3 * k, tpj + 3 * k, rr, H);
    for (int a = 0; a < 3; ++a, ++row) {
      r[row] = rr[a];
      std::memcpy(J + 12 * row, H[a], 12 * sizeof(double));
    }
  }
}

void orc_pose_expmap(const double xi[6], double out[12]) { pose_to34(pose_expmap(xi), out); }
void orc_pose_logmap(const double T[12], double xi[6]) { pose_logmap(pose_from34(T), xi); }
void orc_pose_compose(const double a[12], const double b[12], double out[12]) {
  pose_to34(compose(pose_from34(a), pose_from34(b)), out);
}
void orc_pose_inverse(const double a[12], double out[12]) { pose_to34(inverse(pose_from34(a)), out); }

void* orc_estimator_new(const orc_params* p, int nthreads) { return new Estimator(*p, nthreads); }
void orc_estimator_free(void* e) { delete static_cast<Estimator*>(e); }
int orc_register_scan(void* e, const float* xyzw, size_t n, double pose_out[12], uint32_t* stats,
                      double* times_ms) {
  return static_cast<Estimator*>(e)->register_scan(xyzw, n, pose_out, stats, times_ms);
}

// FORM::map() (bindings.cpp:96-119) = KeypointMap::to_voxel_map (map.tpp:128-146) of the
// stored keypoints of feature type `kind` at the current values, in push_back order
// (scans ascending, keypoint order; the grouping into voxels is left to the caller).
// Returns the record count; xyz (3n), nrm (3n, planar only) and scans (n) may be NULL.
uint32_t orc_estimator_map(void* ev, int kind, double* xyz, double* nrm, uint64_t* scans) {
  Estimator& e = *static_cast<Estimator*>(ev);
  const auto& kp = kind == 0 ? e.kp_planar : e.kp_point;
  const int stride = kind == 0 ? 6 : 3;
  uint32_t n = 0;
  for (auto& [s, f] : kp) {
    const Pose& T = e.values.at(s);  // values.at<Pose3>(X(scan_index)), map.tpp:137
    for (size_t i = 0; i < f.size() / stride; ++i, ++n) {
      double lp[3] = {f[stride * i], f[stride * i + 1], f[stride * i + 2]};
      if (xyz) xform(T, lp, xyz + 3 * (size_t)n);  // PlanarFeat::transform, features.hpp:137-140
      if (nrm && kind == 0) {
        double ln[3] = {f[stride * i + 3], f[stride * i + 4], f[stride * i + 5]};
        matvec(T.R, ln, nrm + 3 * (size_t)n);
      }
      if (scans) scans[n] = s;
    }
  }
  return n;
}

}  // extern "C"
