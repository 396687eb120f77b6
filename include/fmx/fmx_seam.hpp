// fmx_seam.hpp — the GTSAM plugin seam of FORM's smoother, without GTSAM.
//
// FORM's factors reach GTSAM through DenseFactor::linearize (form/optimization/
// gtsam.hpp:67-86): evaluateError gives the whitened A = [H_i H_j] and b = -r, and the
// factor returns HessianFactor(JacobianFactor(A, b)), i.e. the blocks of
// [A b]^T [A b].  fmx_linearize computes exactly that matrix for every pair of a graph
// in one launch, packed (the upper triangle of the 13 x 13, 91 doubles per pair; the
// disable_smoothing ablation's BinaryFactorWrapper, gtsam.hpp:144-170, the 7 x 7 of
// [H_j b], 28 doubles).  This header holds the two pieces a GTSAM-side factor needs,
// as plain C++17 over plain arrays (INTEGRATION.md §2 shows the factor itself):
//
//   * unpack13 / unpack7: packed G -> the arguments of GTSAM's constructor
//       HessianFactor(j1, j2, G11, G12, g1, G22, g2, f)   (two keys)
//       HessianFactor(j, G, g, f)                         (one key)
//     with G11 = A_i^T A_i, G12 = A_i^T A_j, G22 = A_j^T A_j, g1 = A_i^T b,
//     g2 = A_j^T b, f = b^T b (the factor's error at the linearization point is f / 2);
//   * FmxBatch: one fmx_linearize for ALL pairs of a graph per set of poses.  GTSAM
//     linearizes every factor of a NonlinearFactorGraph against the same Values, so
//     the first factor's linearize() launches the batch and the others read its cached
//     result; the cache key is the exact bits of the K pose pairs plus the context's
//     correspondence generation (fmx_corr_generation: a re-match or fmx_corr_set at
//     unchanged poses is a new system).
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "fmx/fmx.h"

namespace fmx_seam {

// Index of (r, c), r <= c, in a row-major packed upper triangle of an n x n matrix.
constexpr int packed_index(int n, int r, int c) { return r * n - r * (r - 1) / 2 + (c - r); }
// Symmetric entry (r, c) of a packed n x n.
inline double packed_at(const double* g, int n, int r, int c) {
  return r <= c ? g[packed_index(n, r, c)] : g[packed_index(n, c, r)];
}

// The blocks of one pair's [A_i A_j b]^T [A_i A_j b] (6 x 6 row-major).
struct Hessian2 {
  double G11[36], G12[36], G22[36];
  double g1[6], g2[6];
  double f;
};
// The blocks of the single-pose [A_j b]^T [A_j b].
struct Hessian1 {
  double G[36];
  double g[6];
  double f;
};

// packed 13 x 13 (91 doubles) -> HessianFactor(X(i), X(j), G11, G12, g1, G22, g2, f):
// rows / columns 0-5 belong to X(i), 6-11 to X(j), 12 to b (gtsam.hpp:67-86).
inline Hessian2 unpack13(const double* g91) {
  Hessian2 h{};
  for (int r = 0; r < 6; ++r) {
    for (int c = 0; c < 6; ++c) {
      h.G11[6 * r + c] = packed_at(g91, 13, r, c);
      h.G12[6 * r + c] = packed_at(g91, 13, r, 6 + c);
      h.G22[6 * r + c] = packed_at(g91, 13, 6 + r, 6 + c);
    }
    h.g1[r] = packed_at(g91, 13, r, 12);
    h.g2[r] = packed_at(g91, 13, 6 + r, 12);
  }
  h.f = packed_at(g91, 13, 12, 12);
  return h;
}
// packed 7 x 7 (28 doubles) -> HessianFactor(X(j), G, g, f) (gtsam.hpp:144-170).
inline Hessian1 unpack7(const double* g28) {
  Hessian1 h{};
  for (int r = 0; r < 6; ++r) {
    for (int c = 0; c < 6; ++c) h.G[6 * r + c] = packed_at(g28, 7, r, c);
    h.g[r] = packed_at(g28, 7, r, 6);
  }
  h.f = packed_at(g28, 7, 6, 6);
  return h;
}

// One fmx_linearize per set of poses for every FeatureFactor pair of a graph.  The pairs
// are the context's correspondences (fmx_match or fmx_corr_set): pair k is the factor
// (X(key_i[k]), X(key_j[k])).  PoseOf: callable (uint64_t key, double out[12]) writing
// the pose of `key` in the caller's Values as a row-major 3 x 4 [R | t].
class FmxBatch {
 public:
  FmxBatch(fmx_ctx* ctx, double sigma, bool single_pose) : ctx_(ctx), sigma_(sigma), single_(single_pose) {}

  void set_pairs(const std::vector<uint64_t>& key_i, const std::vector<uint64_t>& key_j) {
    if (key_i.size() != key_j.size()) throw std::invalid_argument("FmxBatch: key lists differ in length");
    ki_ = key_i;
    kj_ = key_j;
    valid_ = false;
  }
  size_t pairs() const { return ki_.size(); }
  int stride() const { return single_ ? 28 : 91; }

  // Packed G of every pair (K x stride()) at the poses pose_of gives; launched once per
  // distinct set of poses, then served from the cache.
  template <class PoseOf>
  const double* linearize_all(PoseOf&& pose_of) {
    const size_t K = ki_.size();
    pi_.resize(12 * K);
    pj_.resize(12 * K);
    for (size_t k = 0; k < K; ++k) {
      pose_of(ki_[k], &pi_[12 * k]);
      pose_of(kj_[k], &pj_[12 * k]);
    }
    uint64_t gen = 0;
    if (fmx_corr_generation(ctx_, &gen) != FMX_OK) throw std::runtime_error("fmx_corr_generation failed");
    if (valid_ && gen == gen_ && pi_ == ci_ && pj_ == cj_) return G_.data();  // doubles compared exactly
    G_.assign((K ? K : 1) * (size_t)stride(), 0.0);
    err_.assign(K ? K : 1, 0.0);
    const fmx_status st = fmx_linearize(ctx_, pi_.data(), pj_.data(), sigma_, single_ ? 1 : 0, G_.data(), err_.data());
    if (st != FMX_OK) throw std::runtime_error(std::string("fmx_linearize: ") + fmx_last_error(ctx_));
    ci_ = pi_;
    cj_ = pj_;
    gen_ = gen;
    valid_ = true;
    ++launches_;
    return G_.data();
  }
  // pair k's blocks from the last linearize_all
  Hessian2 hessian2(size_t k) const { return unpack13(G_.data() + 91 * k); }
  Hessian1 hessian1(size_t k) const { return unpack7(G_.data() + 28 * k); }
  // 0.5 ||r / sigma||^2 of pair k at the cached poses (= f / 2)
  double error(size_t k) const { return err_.at(k); }
  uint64_t launches() const { return launches_; }
  void invalidate() { valid_ = false; }

 private:
  fmx_ctx* ctx_;
  double sigma_;
  bool single_;
  std::vector<uint64_t> ki_, kj_;
  std::vector<double> pi_, pj_, ci_, cj_, G_, err_;
  bool valid_ = false;
  uint64_t gen_ = 0;
  uint64_t launches_ = 0;
};

// The same seam from pair moments (fmx_moments / fmx_moments_contract): the device
// reduces every pair's rows ONCE, at reference poses, into 16 x 16 moments; every later
// linearization — one per LM iteration of GTSAM's optimizer, at whatever Values it
// proposes — is a host contraction with no device round trip (full 13 x 13 only).
// Reload (set_pairs) after every fmx_match / fmx_corr_set: the moments belong to the
// correspondences they were taken from (checked against fmx_corr_generation).
class FmxMomentBatch {
 public:
  FmxMomentBatch(fmx_ctx* ctx, double sigma) : ctx_(ctx), sigma_(sigma) {}

  // pair k = (X(key_i[k]), X(key_j[k])); the moments are taken at pose_of's poses now
  template <class PoseOf>
  void set_pairs(const std::vector<uint64_t>& key_i, const std::vector<uint64_t>& key_j, PoseOf&& pose_of) {
    if (key_i.size() != key_j.size()) throw std::invalid_argument("FmxMomentBatch: key lists differ in length");
    ki_ = key_i;
    kj_ = key_j;
    const size_t K = ki_.size();
    ri_.resize(12 * K);
    rj_.resize(12 * K);
    for (size_t k = 0; k < K; ++k) {
      pose_of(ki_[k], &ri_[12 * k]);
      pose_of(kj_[k], &rj_[12 * k]);
    }
    mom_.assign((K ? K : 1) * 272, 0.0);
    const fmx_status st = fmx_moments(ctx_, ri_.data(), rj_.data(), mom_.data());
    if (st != FMX_OK) throw std::runtime_error(std::string("fmx_moments: ") + fmx_last_error(ctx_));
    if (fmx_corr_generation(ctx_, &gen_) != FMX_OK) throw std::runtime_error("fmx_corr_generation failed");
  }
  size_t pairs() const { return ki_.size(); }

  // packed 13 x 13 G of every pair (K x 91) at pose_of's poses: host only
  template <class PoseOf>
  const double* linearize_all(PoseOf&& pose_of) {
    uint64_t gen = 0;
    if (fmx_corr_generation(ctx_, &gen) != FMX_OK || gen != gen_)
      throw std::logic_error("FmxMomentBatch: the correspondences changed since set_pairs");
    const size_t K = ki_.size();
    pi_.resize(12 * K);
    pj_.resize(12 * K);
    for (size_t k = 0; k < K; ++k) {
      pose_of(ki_[k], &pi_[12 * k]);
      pose_of(kj_[k], &pj_[12 * k]);
    }
    G_.assign((K ? K : 1) * 91, 0.0);
    err_.assign(K ? K : 1, 0.0);
    const fmx_status st = fmx_moments_contract((uint32_t)K, mom_.data(), ri_.data(), rj_.data(), pi_.data(), pj_.data(),
                                               sigma_, G_.data(), err_.data());
    if (st != FMX_OK) throw std::runtime_error("fmx_moments_contract failed");
    return G_.data();
  }
  Hessian2 hessian2(size_t k) const { return unpack13(G_.data() + 91 * k); }
  double error(size_t k) const { return err_.at(k); }

 private:
  fmx_ctx* ctx_;
  double sigma_;
  std::vector<uint64_t> ki_, kj_;
  std::vector<double> ri_, rj_, pi_, pj_, mom_, G_, err_;
  uint64_t gen_ = 0;
};

}  // namespace fmx_seam
