// factor_rows.hpp — per-correspondence residual + Jacobian rows and the whitened
// outer-product accumulation shared by the linearization kernels (linearize.hip,
// window.hip).  Device code; included inside namespace fmx { namespace { ... } }.
//   PlanePoint::evaluateError  (form/feature/factor.cpp:30-80)
//   PointPoint::evaluateError  (form/feature/factor.cpp:82-128)
//   DenseFactor::linearize + FastIsotropic::WhitenSystem (gtsam.hpp:67-86, 129-139)
#pragma once

template <int MODE>
struct LinShape;
template <>
struct LinShape<0> {  // full binary factor
  static constexpr int M = 13, NG = 91;
};
template <>
struct LinShape<1> {  // single pose (H_j only)
  static constexpr int M = 7, NG = 28;
};
template <>
struct LinShape<2> {  // error only
  static constexpr int M = 0, NG = 1;
};

template <int MODE, int N>
__device__ __forceinline__ void accum_row(const double (&H)[12], double r, double inv, double (&acc)[N]) {
  static_assert(N >= LinShape<MODE>::NG, "accumulator too small");
  if constexpr (MODE == 2) {
    const double w = r * inv;
    acc[0] += w * w;
  } else {
    constexpr int M = LinShape<MODE>::M;
    double a[M];
    if constexpr (MODE == 0) {
#pragma unroll
      for (int c = 0; c < 12; ++c) a[c] = H[c] * inv;
    } else {
#pragma unroll
      for (int c = 0; c < 6; ++c) a[c] = H[6 + c] * inv;
    }
    a[M - 1] = -r * inv;
    int o = 0;
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = i; j < M; ++j) acc[o++] += a[i] * a[j];
  }
}

// PlanePoint row (factor.cpp:37-77), tangent [w; v], right perturbation.
template <int MODE>
__device__ __forceinline__ void plane_row(const double* Ti, const double* Tj, const double pi[3],
                                          const double ni[3], const double pj[3], double& r, double (&H)[12]) {
  double wn[3], wpi[3], wpj[3], v[3];
  d_rot(Ti, ni[0], ni[1], ni[2], wn);
  d_xform(Ti, pi[0], pi[1], pi[2], wpi);
  d_xform(Tj, pj[0], pj[1], pj[2], wpj);
  v[0] = wpj[0] - wpi[0];
  v[1] = wpj[1] - wpi[1];
  v[2] = wpj[2] - wpi[2];
  r = (wn[0] * v[0] + wn[1] * v[1]) + wn[2] * v[2];
  if constexpr (MODE == 0) {
    double RTn[3], RTv[3];
    d_rotT(Ti, wn[0], wn[1], wn[2], RTn);
    d_rotT(Ti, v[0], v[1], v[2], RTv);
    H[0] = RTn[1] * pi[2] - RTn[2] * pi[1] - RTv[1] * ni[2] + RTv[2] * ni[1];
    H[1] = RTn[2] * pi[0] - RTn[0] * pi[2] - RTv[2] * ni[0] + RTv[0] * ni[2];
    H[2] = RTn[0] * pi[1] - RTn[1] * pi[0] - RTv[0] * ni[1] + RTv[1] * ni[0];
    H[3] = -RTn[0];
    H[4] = -RTn[1];
    H[5] = -RTn[2];
  }
  if constexpr (MODE != 2) {
    double Rn[3];
    d_rotT(Tj, wn[0], wn[1], wn[2], Rn);
    H[6] = -Rn[1] * pj[2] + Rn[2] * pj[1];
    H[7] = -Rn[2] * pj[0] + Rn[0] * pj[2];
    H[8] = -Rn[0] * pj[1] + Rn[1] * pj[0];
    H[9] = Rn[0];
    H[10] = Rn[1];
    H[11] = Rn[2];
  }
}

// PointPoint rows (factor.cpp:87-124): residual component a and its 12 columns.
template <int MODE>
__device__ __forceinline__ void point_row(const double* Ti, const double* Tj, const double pi[3],
                                          const double pj[3], const double wpi[3], const double wpj[3], int a,
                                          double& r, double (&H)[12]) {
  r = wpj[a] - wpi[a];
  if constexpr (MODE == 0) {
    const double R0 = Ti[4 * a] * -1.0, R1 = Ti[4 * a + 1] * -1.0, R2 = Ti[4 * a + 2] * -1.0;
    H[0] = R2 * pi[1] - R1 * pi[2];
    H[1] = R0 * pi[2] - R2 * pi[0];
    H[2] = R1 * pi[0] - R0 * pi[1];
    H[3] = R0;
    H[4] = R1;
    H[5] = R2;
  }
  if constexpr (MODE != 2) {
    const double R0 = Tj[4 * a], R1 = Tj[4 * a + 1], R2 = Tj[4 * a + 2];
    H[6] = R2 * pj[1] - R1 * pj[2];
    H[7] = R0 * pj[2] - R2 * pj[0];
    H[8] = R1 * pj[0] - R0 * pj[1];
    H[9] = R0;
    H[10] = R1;
    H[11] = R2;
  }
}

