// test_seam.cpp — a C++ caller of the fmx C-ABI (include/fmx/fmx.h) through the GTSAM
// seam header (include/fmx/fmx_seam.hpp), as a GTSAM-side FeatureFactor would use it
// (the reference's seam is DenseFactor::linearize,
// form/optimization/gtsam.hpp:67-86, and BinaryFactorWrapper, :144-170).
//
// Built with g++ -std=c++17 -Wall -Werror (tests/cpp/Makefile); run by
// tests/test_gpu_seam.py on the GPU box.  Checks, per pair of K synthetic FeatureFactors:
//   * the HessianFactor blocks unpack13 gives, reassembled, equal the oracle's packed
//     [A b]^T [A b] (1e-10 relative) AND the product formed here from the oracle's raw
//     rows (A = J / sigma, b = -r / sigma: factor.cpp:30-186, gtsam.hpp:67-86);
//   * the factor error fmx returns is f / 2 (HessianFactor's error at the
//     linearization point);
//   * unpack7 (single_pose = 1) likewise against [A_j b]^T [A_j b];
//   * FmxBatch launches fmx_linearize once per distinct set of poses.
// The oracle (liboracle.so) is test infrastructure: the checker only.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <vector>

#include "fmx/fmx.h"
#include "fmx/fmx_seam.hpp"
#include "form_oracle.h"

namespace {

int g_fail = 0;
void check(bool ok, const char* what, size_t k, double a, double b) {
  if (!ok) {
    std::fprintf(stderr, "FAIL %s pair %zu: %.17g vs %.17g\n", what, k, a, b);
    ++g_fail;
  }
}

// [A b]^T [A b] (n_cols = 12 + 1) of one pair from the oracle's raw residual rows.
std::vector<double> gram_from_rows(const std::vector<double>& r, const std::vector<double>& J, double sigma,
                                   bool single) {
  const size_t rows = r.size();
  const int n = single ? 7 : 13;
  std::vector<double> G((size_t)n * n, 0.0);
  std::vector<double> a(n);
  for (size_t q = 0; q < rows; ++q) {
    for (int c = 0; c < 12; ++c) {
      if (single && c < 6) continue;
      a[single ? c - 6 : c] = J[12 * q + c] / sigma;
    }
    a[n - 1] = -r[q] / sigma;
    for (int u = 0; u < n; ++u)
      for (int v = 0; v < n; ++v) G[(size_t)u * n + v] += a[u] * a[v];
  }
  return G;
}

void rand_pose(std::mt19937_64& g, double out[12], double rot, double tr) {
  std::normal_distribution<double> N(0.0, 1.0);
  double xi[6];
  for (int i = 0; i < 3; ++i) xi[i] = rot * N(g);
  for (int i = 3; i < 6; ++i) xi[i] = tr * N(g);
  orc_pose_expmap(xi, out);
}

}  // namespace

int main() {
  fmx_params prm;
  fmx_default_params(&prm);
  fmx_ctx* ctx = nullptr;
  if (fmx_create(&prm, 0, &ctx) != FMX_OK) {
    std::fprintf(stderr, "fmx_create failed (no HIP device?)\n");
    return 2;
  }
  std::mt19937_64 g(0x464F524D);
  std::uniform_real_distribution<double> U(-20.0, 20.0);
  std::normal_distribution<double> N(0.0, 1.0);
  // K pairs (i_k, j): map scans 0..K-1 against the current scan j = 100
  const uint32_t K = 6;
  std::vector<uint32_t> np(K), nt(K);
  std::vector<double> ppi, pni, ppj, tpi, tpj;
  std::map<uint64_t, std::vector<double>> pose;
  std::vector<uint64_t> key_i, key_j;
  for (uint32_t k = 0; k < K; ++k) {
    np[k] = k == 2 ? 0 : 300 + 97 * k;  // one pair without plane rows
    nt[k] = k == 4 ? 0 : 40 + 13 * k;   // one without point pairs
    for (uint32_t q = 0; q < np[k]; ++q) {
      double n3[3] = {N(g), N(g), N(g)};
      const double nn = std::sqrt(n3[0] * n3[0] + n3[1] * n3[1] + n3[2] * n3[2]);
      for (int d = 0; d < 3; ++d) {
        const double p = U(g);
        ppi.push_back(p);
        pni.push_back(n3[d] / nn);
        ppj.push_back(p + 0.05 * N(g));
      }
    }
    for (uint32_t q = 0; q < nt[k]; ++q)
      for (int d = 0; d < 3; ++d) {
        const double p = U(g);
        tpi.push_back(p);
        tpj.push_back(p + 0.05 * N(g));
      }
    pose[k].resize(12);
    rand_pose(g, pose[k].data(), 0.05, 2.0);
    key_i.push_back(k);
    key_j.push_back(100);
  }
  pose[100].resize(12);
  rand_pose(g, pose[100].data(), 0.05, 2.0);
  if (fmx_corr_set(ctx, K, np.data(), ppi.data(), pni.data(), ppj.data(), nt.data(), tpi.data(), tpj.data()) != FMX_OK) {
    std::fprintf(stderr, "fmx_corr_set: %s\n", fmx_last_error(ctx));
    return 1;
  }
  auto pose_of = [&](uint64_t key, double out[12]) {
    for (int e = 0; e < 12; ++e) out[e] = pose.at(key)[e];
  };
  const double sigma = 0.1;
  for (int single = 0; single < 2; ++single) {
    fmx_seam::FmxBatch batch(ctx, sigma, single != 0);
    batch.set_pairs(key_i, key_j);
    batch.linearize_all(pose_of);
    batch.linearize_all(pose_of);  // same Values: served from the cache
    check(batch.launches() == 1, "cache hit", 0, (double)batch.launches(), 1.0);
    // the correspondences replaced (here: set again) at unchanged poses: a new
    // generation (fmx_corr_generation), so the batch relaunches instead of serving the cache
    if (fmx_corr_set(ctx, K, np.data(), ppi.data(), pni.data(), ppj.data(), nt.data(), tpi.data(), tpj.data()) != FMX_OK)
      return 1;
    batch.linearize_all(pose_of);
    check(batch.launches() == 2, "relaunch on new correspondences", 0, (double)batch.launches(), 2.0);
    // the oracle's packed G and errors at the same poses
    std::vector<double> Pi(12 * K), Pj(12 * K);
    for (uint32_t k = 0; k < K; ++k) {
      pose_of(key_i[k], &Pi[12 * k]);
      pose_of(key_j[k], &Pj[12 * k]);
    }
    const int stride = single ? 28 : 91, n = single ? 7 : 13;
    std::vector<double> Go((size_t)K * stride), eo(K);
    orc_linearize(K, np.data(), ppi.data(), pni.data(), ppj.data(), nt.data(), tpi.data(), tpj.data(), Pi.data(),
                  Pj.data(), sigma, single, Go.data(), eo.data());
    size_t opl = 0, opt = 0;
    for (uint32_t k = 0; k < K; ++k) {
      // this pair's raw rows from the oracle -> [A b]^T [A b] formed here
      const size_t rows = np[k] + 3 * (size_t)nt[k];
      std::vector<double> r(rows), J(12 * rows);
      orc_factor_rows(np[k], &ppi[3 * opl], &pni[3 * opl], &ppj[3 * opl], nt[k], &tpi[3 * opt], &tpj[3 * opt],
                      &Pi[12 * k], &Pj[12 * k], r.data(), J.data());
      opl += np[k];
      opt += nt[k];
      const std::vector<double> Gr = gram_from_rows(r, J, sigma, single != 0);
      // the seam's blocks, reassembled into the full n x n
      std::vector<double> F((size_t)n * n);
      double f;
      if (single) {
        const fmx_seam::Hessian1 h = batch.hessian1(k);
        for (int u = 0; u < 6; ++u) {
          for (int v = 0; v < 6; ++v) F[7 * u + v] = h.G[6 * u + v];
          F[7 * u + 6] = F[7 * 6 + u] = h.g[u];
        }
        f = F[48] = h.f;
      } else {
        const fmx_seam::Hessian2 h = batch.hessian2(k);
        for (int u = 0; u < 6; ++u) {
          for (int v = 0; v < 6; ++v) {
            F[13 * u + v] = h.G11[6 * u + v];
            F[13 * u + 6 + v] = h.G12[6 * u + v];
            F[13 * (6 + v) + u] = h.G12[6 * u + v];  // G21 = G12^T
            F[13 * (6 + u) + 6 + v] = h.G22[6 * u + v];
          }
          F[13 * u + 12] = F[13 * 12 + u] = h.g1[u];
          F[13 * (6 + u) + 12] = F[13 * 12 + 6 + u] = h.g2[u];
        }
        f = F[168] = h.f;
      }
      double scale = 0.0;
      for (double v : Gr) scale = std::max(scale, std::fabs(v));
      for (int u = 0; u < n; ++u)
        for (int v = 0; v < n; ++v) {
          const double o = fmx_seam::packed_at(&Go[(size_t)stride * k], n, u, v);
          check(std::fabs(F[(size_t)n * u + v] - o) <= 1e-10 * scale, single ? "unpack7 vs oracle G" : "unpack13 vs oracle G",
                k, F[(size_t)n * u + v], o);
          check(std::fabs(F[(size_t)n * u + v] - Gr[(size_t)n * u + v]) <= 1e-10 * scale,
                single ? "unpack7 vs rows" : "unpack13 vs rows", k, F[(size_t)n * u + v], Gr[(size_t)n * u + v]);
        }
      check(std::fabs(batch.error(k) - 0.5 * f) <= 1e-12 * f, "error = f/2", k, batch.error(k), 0.5 * f);
      check(std::fabs(batch.error(k) - eo[k]) <= 1e-10 * eo[k], "error vs oracle", k, batch.error(k), eo[k]);
    }
    // a new Values (X(j) moved): one more launch, and a different system
    const double before = batch.error(0);
    pose[100][3] += 0.01;
    batch.linearize_all(pose_of);
    check(batch.launches() == 3, "relaunch on new poses", 0, (double)batch.launches(), 3.0);
    check(batch.error(0) != before, "new poses change the error", 0, batch.error(0), before);
    pose[100][3] -= 0.01;
  }
  // the moment form of the seam: moments once at the current poses, then host-only
  // linearizations at moved poses, against the oracle (1e-10)
  {
    fmx_seam::FmxMomentBatch mb(ctx, sigma);
    mb.set_pairs(key_i, key_j, pose_of);
    for (int step = 0; step < 3; ++step) {
      for (auto& kv : pose) kv.second[3] += 0.004 * (step + 1), kv.second[7] -= 0.002;
      mb.linearize_all(pose_of);
      std::vector<double> Pi(12 * K), Pj(12 * K), Go((size_t)K * 91), eo(K);
      for (uint32_t k = 0; k < K; ++k) {
        pose_of(key_i[k], &Pi[12 * k]);
        pose_of(key_j[k], &Pj[12 * k]);
      }
      orc_linearize(K, np.data(), ppi.data(), pni.data(), ppj.data(), nt.data(), tpi.data(), tpj.data(), Pi.data(),
                    Pj.data(), sigma, 0, Go.data(), eo.data());
      for (uint32_t k = 0; k < K; ++k) {
        double scale = 0.0;
        for (int q = 0; q < 91; ++q) scale = std::max(scale, std::fabs(Go[91 * k + q]));
        const fmx_seam::Hessian2 h = mb.hessian2(k);
        for (int u = 0; u < 6; ++u)
          for (int v = 0; v < 6; ++v)
            check(std::fabs(h.G11[6 * u + v] - fmx_seam::packed_at(&Go[91 * k], 13, u, v)) <= 1e-10 * scale,
                  "moments G11 vs oracle", k, h.G11[6 * u + v], fmx_seam::packed_at(&Go[91 * k], 13, u, v));
        check(std::fabs(mb.error(k) - eo[k]) <= 1e-10 * std::max(eo[k], 1e-300), "moments error vs oracle", k,
              mb.error(k), eo[k]);
      }
    }
    // a re-set of the correspondences invalidates the moments
    if (fmx_corr_set(ctx, K, np.data(), ppi.data(), pni.data(), ppj.data(), nt.data(), tpi.data(), tpj.data()) != FMX_OK)
      return 1;
    bool threw = false;
    try {
      mb.linearize_all(pose_of);
    } catch (const std::logic_error&) {
      threw = true;
    }
    check(threw, "stale moments rejected", 0, threw ? 1.0 : 0.0, 1.0);
  }
  fmx_destroy(ctx);
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  std::printf("seam ok: %u pairs, 13x13 and 7x7 HessianFactor blocks vs oracle and raw rows\n", K);
  return 0;
}
