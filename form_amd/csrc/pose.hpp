// pose.hpp — host pose algebra in GTSAM conventions (Pose3 = (R, t), tangent [w; v],
// right perturbation, GTSAM_POSE3_EXPMAP chart) for the register_scan host adapter and
// the window smoother.  Compiled with -ffp-contract=off (the reference's SSE2 rounding).
#pragma once
#include <cfloat>
#include <cmath>

namespace fmxh {
struct Pose {
  double m[12];  // row-major [R | t]
};
inline Pose identity() {
  Pose p{};
  p.m[0] = p.m[5] = p.m[10] = 1.0;
  return p;
}
inline Pose compose(const Pose& a, const Pose& b) {  // gtsam Pose3::operator*
  Pose c;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      c.m[4 * i + j] = (a.m[4 * i] * b.m[j] + a.m[4 * i + 1] * b.m[4 + j]) + a.m[4 * i + 2] * b.m[8 + j];
    c.m[4 * i + 3] = ((a.m[4 * i] * b.m[3] + a.m[4 * i + 1] * b.m[7]) + a.m[4 * i + 2] * b.m[11]) + a.m[4 * i + 3];
  }
  return c;
}
inline Pose inverse(const Pose& a) {  // (R^T, R^T(-t))
  Pose c;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) c.m[4 * i + j] = a.m[4 * j + i];
  const double nt[3] = {-a.m[3], -a.m[7], -a.m[11]};
  for (int i = 0; i < 3; ++i) c.m[4 * i + 3] = (c.m[4 * i] * nt[0] + c.m[4 * i + 1] * nt[1]) + c.m[4 * i + 2] * nt[2];
  return c;
}
inline void cross(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
inline Pose expmap(const double xi[6]) {  // gtsam Pose3::Expmap, tangent [w; v]
  const double* w = xi;
  const double* v = xi + 3;
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  double A, B, a, b;
  if (th2 <= DBL_EPSILON) {
    A = 1.0;
    B = 0.5;
    a = 0.5;
    b = 1.0 / 6.0;
  } else {
    const double th = std::sqrt(th2);
    A = std::sin(th) / th;
    B = (1.0 - std::cos(th)) / th2;
    a = B;
    b = (th - std::sin(th)) / (th2 * th);
  }
  const double W[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
  Pose T;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const double w2 = W[i][0] * W[0][j] + W[i][1] * W[1][j] + W[i][2] * W[2][j];
      T.m[4 * i + j] = (i == j ? 1.0 : 0.0) + A * W[i][j] + B * w2;
    }
  double wxv[3], wxwxv[3];
  cross(w, v, wxv);
  cross(w, wxv, wxwxv);
  for (int i = 0; i < 3; ++i) T.m[4 * i + 3] = v[i] + a * wxv[i] + b * wxwxv[i];
  return T;
}
inline void logmap(const Pose& T, double xi[6]) {  // gtsam Pose3::Logmap
  const double* m = T.m;
  const double tr = m[0] + m[5] + m[10];
  double w[3];
  if (tr + 1.0 < 1e-10) {
    if (std::abs(m[10] + 1.0) > 1e-10) {
      const double s = M_PI / std::sqrt(2.0 + 2.0 * m[10]);
      w[0] = s * m[2]; w[1] = s * m[6]; w[2] = s * (1.0 + m[10]);
    } else if (std::abs(m[5] + 1.0) > 1e-10) {
      const double s = M_PI / std::sqrt(2.0 + 2.0 * m[5]);
      w[0] = s * m[1]; w[1] = s * (1.0 + m[5]); w[2] = s * m[9];
    } else {
      const double s = M_PI / std::sqrt(2.0 + 2.0 * m[0]);
      w[0] = s * (1.0 + m[0]); w[1] = s * m[4]; w[2] = s * m[8];
    }
  } else {
    const double tr_3 = tr - 3.0;
    double mag;
    if (tr_3 < -1e-7) {
      const double th = std::acos((tr - 1.0) / 2.0);
      mag = th / (2.0 * std::sin(th));
    } else {
      mag = 0.5 - tr_3 * tr_3 / 12.0;
    }
    w[0] = mag * (m[9] - m[6]);
    w[1] = mag * (m[2] - m[8]);
    w[2] = mag * (m[4] - m[1]);
  }
  const double t = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  xi[0] = w[0]; xi[1] = w[1]; xi[2] = w[2];
  const double tt[3] = {m[3], m[7], m[11]};
  if (t < 1e-10) {
    xi[3] = tt[0]; xi[4] = tt[1]; xi[5] = tt[2];
    return;
  }
  const double wn[3] = {w[0] / t, w[1] / t, w[2] / t};
  double WT[3], WWT[3];
  cross(wn, tt, WT);
  cross(wn, WT, WWT);
  const double Tan = std::tan(0.5 * t);
  for (int i = 0; i < 3; ++i) xi[3 + i] = tt[i] - (0.5 * t) * WT[i] + (1 - t / (2. * Tan)) * WWT[i];
}
inline void normalize_rot(Pose& P) {  // gtsam Rot3::normalized (constraints.cpp:93-95)
  double* R = P.m;
  const double det = R[0] * (R[5] * R[10] - R[6] * R[9]) - R[1] * (R[4] * R[10] - R[6] * R[8]) +
                     R[2] * (R[4] * R[9] - R[5] * R[8]);
  if (std::fabs(det - 1) < 1e-12) return;
  const double x[3] = {R[0], R[1], R[2]}, y[3] = {R[4], R[5], R[6]};
  const double err = x[0] * y[0] + x[1] * y[1] + x[2] * y[2];
  double xo[3], yo[3], zo[3];
  for (int i = 0; i < 3; ++i) {
    xo[i] = x[i] - (err / 2) * y[i];
    yo[i] = y[i] - (err / 2) * x[i];
  }
  cross(xo, yo, zo);
  const double sx = 0.5 * (3 - (xo[0] * xo[0] + xo[1] * xo[1] + xo[2] * xo[2]));
  const double sy = 0.5 * (3 - (yo[0] * yo[0] + yo[1] * yo[1] + yo[2] * yo[2]));
  const double sz = 0.5 * (3 - (zo[0] * zo[0] + zo[1] * zo[1] + zo[2] * zo[2]));
  for (int i = 0; i < 3; ++i) {
    R[i] = sx * xo[i];
    R[4 + i] = sy * yo[i];
    R[8 + i] = sz * zo[i];
  }
}

inline bool chol_solve6(const double H[6][6], const double g[6], double x[6]) {
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

}  // namespace fmxh
