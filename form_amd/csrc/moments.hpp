// moments.hpp — DenseFactor::linearize of a FeatureFactor pair (gtsam.hpp:67-86,
// factor.cpp:30-128) from its row moments, on the host.
//
// Every plane / point row's whitened a = [H_i H_j -r] / sigma is linear in 16 features
// taken once at reference poses (window.hip, k_win_moments), with coefficients that
// depend only on the pair's two poses.  So with Phi = sum_rows phi phi^T (per pair and
// row type) the pair's packed 13 x 13 information at ANY poses is C Phi C^T: a few
// thousand flops per pair instead of a pass over its rows on the device.  The smoother's
// LM trials (register_scan) evaluate it here, with no device round trip.
//
//   plane rows, features [r0, n x q0 (3), n (3), n_b p_j,d (9)], q0 = p_j in frame i at
//   the reference poses, r0 = n.(q0 - p_i):
//     H_i = [n x q, -n], H_j = [p_j x M^T n, M^T n], r = n.(q - p_i),
//     q = M p_j + v = q0 + (M - M0) p_j + (v - v0),  M = R_i^T R_j, v = R_i^T (t_j - t_i)
//   point rows, features [e0 (3), p_i (3), p_j (3), 1], e0 = the world residual at the
//   reference poses; per world axis a (factor.cpp:87-124):
//     H_i = [p_i x (-R_i[a]), -R_i[a]], H_j = [p_j x R_j[a], R_j[a]],
//     r_a = e0_a + (R_j - R_j0)[a] p_j - (R_i - R_i0)[a] p_i + (t_j - t_j0 - t_i + t_i0)_a
// The residual enters through the per-row r0 / e0 (small), never as a difference of
// large moments, so the result keeps full fp64 precision (tests/test_moments.py).
#pragma once
#include <stdint.h>

#include <vector>

#include "pose.hpp"

namespace fmxh {

constexpr int kMomFeat = 16;    // features per row
constexpr int kMomPacked = 136;  // packed upper 16 x 16
constexpr int kMomPairD = 2 * kMomPacked;  // per pair: plane moments, then point moments

// A set of pairs' moments laid out for evaluation (eight pairs per SIMD block, structure
// of arrays), built once per set (mom_prepare) and evaluated at many poses (mom_eval):
// an LM relinearizes the same pairs at every trial.
struct MomBatch {
  int n = 0;
  std::vector<double> data;  // per block of 8 pairs: kMomBlockD doubles (moments.cpp)
};
// mom[k]: pair k's kMomPairD moments, taken at reference poses (Ti0[k], Tj0[k]).
void mom_prepare(MomBatch& b, int n, const double* const* mom, const Pose* const* Ti0, const Pose* const* Tj0);
// Packed 13 x 13 information (91) + error (0.5 G[12][12]) of every pair of b at poses
// (Ti[k], Tj[k]); inv = 1 / sigma.  G: n x 92.
void mom_eval(const MomBatch& b, const Pose* const* Ti, const Pose* const* Tj, double inv, double* G);

}  // namespace fmxh
