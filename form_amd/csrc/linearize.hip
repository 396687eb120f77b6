// linearize.hip — stage 3: residual + Jacobian + whitened normal-equation reduction.
//
// Replaces, per correspondence pair (map scan i, current scan j):
//   PlanePoint::evaluateError  (form/feature/factor.cpp:30-80)
//   PointPoint::evaluateError  (form/feature/factor.cpp:82-128)
//   FeatureFactor stacking     (form/feature/factor.cpp:142-186)
//   DenseFactor::linearize + FastIsotropic::WhitenSystem (form/optimization/
//     gtsam.hpp:67-86, 129-139): A = [H_i H_j] / sigma, b = -r / sigma, and the
//     HessianFactor's augmented information G = [A b]^T [A b] (13 x 13, 91 unique
//     doubles), or [H_j b]^T [H_j b] (7 x 7, 28) for the single-pose mode
//     (BinaryFactorWrapper, gtsam.hpp:144-170).
//
// Work split: correspondences are pair-major SoA (voxelmap.hip); a chunk is <= 1024
// plane rows or <= 512 point pairs of ONE pair.  One 256-lane workgroup per chunk:
// each lane accumulates its rows' outer products in fp64 registers, then a wave
// shuffle tree + 4-way LDS sum gives the chunk partial; k_lin_final adds a pair's
// chunk partials in chunk order.  Fixed trees => bitwise-reproducible G.
// HBM-bound: 72 B per plane row and 48 B per point pair against ~300 / ~900 flop.
#include "fmx_device.hpp"
#include "fmx_internal.hpp"

#include <algorithm>
#include <cstring>

namespace fmx {
namespace {

constexpr int kLinThreads = 64;

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

template <int MODE>
__device__ __forceinline__ void accum_row(const double (&H)[12], double r, double inv,
                                          double (&acc)[LinShape<MODE>::NG]) {
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

// One wave per chunk (<= 64 plane rows or <= 64 point pairs of one pair), one row
// (or point pair) per lane; the wave's NG sums go to partials[NG][max_chunks].
template <int MODE>
__global__ __launch_bounds__(kLinThreads) void k_linearize(const Chunk* __restrict__ chunks,
                                                           const uint32_t* __restrict__ n_chunks,
                                                           const double* __restrict__ c_pl, size_t ld_pl,
                                                           const double* __restrict__ c_pt, size_t ld_pt,
                                                           const double* __restrict__ poses, double inv,
                                                           double* __restrict__ partials, size_t ldp) {
  constexpr int NG = LinShape<MODE>::NG;
  const uint32_t ch = blockIdx.x;
  if (ch >= *n_chunks) return;
  const Chunk d = chunks[ch];
  const double* Ti = poses + 24 * d.pair;
  const double* Tj = Ti + 12;
  double acc[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) acc[i] = 0.0;
  double H[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) H[i] = 0.0;
  const uint32_t row = d.begin + threadIdx.x;
  if (row < d.end) {
    if (d.type == 0) {
      const double pi[3] = {c_pl[row], c_pl[ld_pl + row], c_pl[2 * ld_pl + row]};
      const double ni[3] = {c_pl[3 * ld_pl + row], c_pl[4 * ld_pl + row], c_pl[5 * ld_pl + row]};
      const double pj[3] = {c_pl[6 * ld_pl + row], c_pl[7 * ld_pl + row], c_pl[8 * ld_pl + row]};
      double r;
      plane_row<MODE>(Ti, Tj, pi, ni, pj, r, H);
      accum_row<MODE>(H, r, inv, acc);
    } else {
      const double pi[3] = {c_pt[row], c_pt[ld_pt + row], c_pt[2 * ld_pt + row]};
      const double pj[3] = {c_pt[3 * ld_pt + row], c_pt[4 * ld_pt + row], c_pt[5 * ld_pt + row]};
      double wpi[3], wpj[3];
      d_xform(Ti, pi[0], pi[1], pi[2], wpi);
      d_xform(Tj, pj[0], pj[1], pj[2], wpj);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        double r;
        point_row<MODE>(Ti, Tj, pi, pj, wpi, wpj, a, r, H);
        accum_row<MODE>(H, r, inv, acc);
      }
    }
  }
  // butterfly sums: every lane ends with every total; lane i keeps entry i (and i+64)
  double mine0 = 0.0, mine1 = 0.0;
  const int lane = lane_id();
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const double s = wave_sum(acc[i]);
    if (i < 64) {
      if (lane == i) mine0 = s;
    } else {
      if (lane == i - 64) mine1 = s;
    }
  }
  if (lane < NG) partials[(size_t)lane * ldp + ch] = mine0;
  if (lane + 64 < NG) partials[(size_t)(lane + 64) * ldp + ch] = mine1;
}

// One wave per (pair k, entry i): sum the pair's chunk partials (lane-strided, in
// a fixed order, then a fixed butterfly) -> G[k][i]; err[k] = 0.5 * G[k][last].
template <int MODE>
__global__ __launch_bounds__(256) void k_lin_final(const uint32_t* __restrict__ chunk_range,
                                                   const double* __restrict__ partials, size_t ldp,
                                                   double* __restrict__ G, double* __restrict__ err, int K) {
  constexpr int NG = LinShape<MODE>::NG;
  const int item = blockIdx.x * 4 + threadIdx.x / kWave;
  if (item >= K * NG) return;
  const int k = item / NG, i = item % NG;
  const uint32_t b = chunk_range[k], e = chunk_range[k + 1];
  double s = 0.0;
  for (uint32_t c = b + lane_id(); c < e; c += kWave) s += partials[(size_t)i * ldp + c];
  s = wave_sum(s);
  if (lane_id() == 0) {
    if constexpr (MODE == 2) {
      err[k] = 0.5 * s;
    } else {
      G[(size_t)k * NG + i] = s;
      if (i == NG - 1) err[k] = 0.5 * s;
    }
  }
}

}  // namespace

void run_linearize(fmx_ctx* c, const double* poses_i34, const double* poses_j34, double sigma, int mode,
                   double* G_out, double* err_out) {
  if (!c->have_corr) throw StatusError(FMX_E_STATE, "no correspondences (call fmx_match or fmx_corr_set)");
  hipStream_t st = c->stream;
  const int K = (int)c->K;
  if (K == 0) return;
  const int NG = mode == 0 ? 91 : (mode == 1 ? 28 : 1);
  c->h_poses.ensure(24 * (size_t)K);
  for (int k = 0; k < K; ++k) {
    std::memcpy(c->h_poses.p + 24 * k, poses_i34 + 12 * k, 12 * sizeof(double));
    std::memcpy(c->h_poses.p + 24 * k + 12, poses_j34 + 12 * k, 12 * sizeof(double));
  }
  c->poses_ij.ensure(24 * (size_t)K);
  FMX_HIP(hipMemcpyAsync(c->poses_ij.p, c->h_poses.p, 24 * K * sizeof(double), hipMemcpyHostToDevice, st));
  c->partials.ensure((size_t)std::max<uint32_t>(c->max_chunks, 1) * 91 + 1);
  c->G.ensure((size_t)K * 92 + 1);
  double* dG = c->G.p;
  double* dErr = mode == 2 ? dG : dG + (size_t)K * NG;  // error-only: err is the whole output
  const double inv = 1.0 / sigma;  // FastIsotropic invsigma_ (gtsam.hpp:96)
  const uint32_t nb = std::max<uint32_t>(c->max_chunks, 1);
  const size_t ldp = nb;
  if (c->counts_pending && c->prof.on) match_counts_fetch(c);  // exact byte model for the profile
  const double bytes = 72.0 * c->rows_pl + 48.0 * c->rows_pt + 8.0 * NG * K;
  const int nfin = (K * NG + 3) / 4;
  {
    ProfScope ps(c->prof, mode == 2 ? PROF_ERROR : PROF_LINEARIZE, bytes, st);
    if (mode == 0)
      hipLaunchKernelGGL(k_linearize<0>, dim3(nb), dim3(kLinThreads), 0, st, c->chunks.p, c->n_chunks.p, c->c_pl.p,
                         c->ld_pl, c->c_pt.p, c->ld_pt, c->poses_ij.p, inv, c->partials.p, ldp);
    else if (mode == 1)
      hipLaunchKernelGGL(k_linearize<1>, dim3(nb), dim3(kLinThreads), 0, st, c->chunks.p, c->n_chunks.p, c->c_pl.p,
                         c->ld_pl, c->c_pt.p, c->ld_pt, c->poses_ij.p, inv, c->partials.p, ldp);
    else
      hipLaunchKernelGGL(k_linearize<2>, dim3(nb), dim3(kLinThreads), 0, st, c->chunks.p, c->n_chunks.p, c->c_pl.p,
                         c->ld_pl, c->c_pt.p, c->ld_pt, c->poses_ij.p, inv, c->partials.p, ldp);
    FMX_HIP(hipGetLastError());
  }
  {
    ProfScope ps(c->prof, PROF_LIN_FINAL, 8.0 * NG * (double)nb + 8.0 * NG * K, st);
    if (mode == 0)
      hipLaunchKernelGGL(k_lin_final<0>, dim3(nfin), dim3(256), 0, st, c->chunk_range.p, c->partials.p, ldp, dG, dErr, K);
    else if (mode == 1)
      hipLaunchKernelGGL(k_lin_final<1>, dim3(nfin), dim3(256), 0, st, c->chunk_range.p, c->partials.p, ldp, dG, dErr, K);
    else
      hipLaunchKernelGGL(k_lin_final<2>, dim3(nfin), dim3(256), 0, st, c->chunk_range.p, c->partials.p, ldp, dG, dErr, K);
    FMX_HIP(hipGetLastError());
  }
  const size_t nout = (size_t)K * (mode == 2 ? 1 : NG + 1);
  c->h_G.ensure(nout);
  FMX_HIP(hipMemcpyAsync(c->h_G.p, dG, nout * sizeof(double), hipMemcpyDeviceToHost, st));
  FMX_HIP(hipStreamSynchronize(st));
  match_counts_fetch(c);  // already copied; no extra wait
  if (mode == 2) {
    if (err_out) std::memcpy(err_out, c->h_G.p, K * sizeof(double));
  } else {
    if (G_out) std::memcpy(G_out, c->h_G.p, (size_t)K * NG * sizeof(double));
    if (err_out) std::memcpy(err_out, c->h_G.p + (size_t)K * NG, K * sizeof(double));
  }
}

void upload_corr(fmx_ctx* c, uint32_t K, const uint32_t* np, const double* ppi, const double* pni,
                 const double* ppj, const uint32_t* nt, const double* tpi, const double* tpj) {
  hipStream_t st = c->stream;
  uint64_t Np = 0, Nt = 0;
  for (uint32_t k = 0; k < K; ++k) {
    Np += np[k];
    Nt += nt[k];
  }
  c->K = K;
  c->ld_pl = Np + 1;
  c->ld_pt = Nt + 1;
  c->c_pl.ensure(9 * c->ld_pl);
  c->c_pt.ensure(6 * c->ld_pt);
  c->h_corr.ensure(9 * c->ld_pl + 6 * c->ld_pt);
  double* hp = c->h_corr.p;
  double* ht = hp + 9 * c->ld_pl;
  for (uint64_t r = 0; r < Np; ++r)
    for (int d = 0; d < 3; ++d) {
      hp[d * c->ld_pl + r] = ppi[3 * r + d];
      hp[(3 + d) * c->ld_pl + r] = pni[3 * r + d];
      hp[(6 + d) * c->ld_pl + r] = ppj[3 * r + d];
    }
  for (uint64_t r = 0; r < Nt; ++r)
    for (int d = 0; d < 3; ++d) {
      ht[d * c->ld_pt + r] = tpi[3 * r + d];
      ht[(3 + d) * c->ld_pt + r] = tpj[3 * r + d];
    }
  FMX_HIP(hipMemcpyAsync(c->c_pl.p, hp, 9 * c->ld_pl * sizeof(double), hipMemcpyHostToDevice, st));
  FMX_HIP(hipMemcpyAsync(c->c_pt.p, ht, 6 * c->ld_pt * sizeof(double), hipMemcpyHostToDevice, st));
  // chunk table (pair-major), same layout k_pair_offsets writes
  std::vector<Chunk> ch;
  std::vector<uint32_t> cr(K + 1);
  uint64_t op = 0, ot = 0;
  for (uint32_t k = 0; k < K; ++k) {
    cr[k] = (uint32_t)ch.size();
    for (uint32_t r = 0; r < np[k]; r += kPlaneChunk)
      ch.push_back(Chunk{0, k, (uint32_t)(op + r), (uint32_t)(op + std::min<uint64_t>(np[k], r + kPlaneChunk))});
    for (uint32_t r = 0; r < nt[k]; r += kPointChunk)
      ch.push_back(Chunk{1, k, (uint32_t)(ot + r), (uint32_t)(ot + std::min<uint64_t>(nt[k], r + kPointChunk))});
    op += np[k];
    ot += nt[k];
  }
  cr[K] = (uint32_t)ch.size();
  const uint32_t nch = (uint32_t)ch.size();
  c->chunks.ensure(nch + 1);
  c->chunk_range.ensure(K + 1);
  c->n_chunks.ensure(1);
  c->pair_counts.ensure(2 * (size_t)K + 1);
  c->h_meta.ensure(4 * (size_t)nch + 2 * (K + 1) + 2 * (size_t)K + 4);
  uint32_t* hm = c->h_meta.p;
  std::memcpy(hm, ch.data(), nch * sizeof(Chunk));
  std::memcpy(hm + 4 * nch, cr.data(), (K + 1) * sizeof(uint32_t));
  hm[4 * nch + K + 1] = nch;
  std::memcpy(hm + 4 * nch + K + 2, np, K * sizeof(uint32_t));
  std::memcpy(hm + 4 * nch + 2 * K + 2, nt, K * sizeof(uint32_t));
  FMX_HIP(hipMemcpyAsync(c->chunks.p, hm, nch * sizeof(Chunk), hipMemcpyHostToDevice, st));
  FMX_HIP(hipMemcpyAsync(c->chunk_range.p, hm + 4 * nch, (K + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  FMX_HIP(hipMemcpyAsync(c->n_chunks.p, hm + 4 * nch + K + 1, sizeof(uint32_t), hipMemcpyHostToDevice, st));
  FMX_HIP(hipMemcpyAsync(c->pair_counts.p, hm + 4 * nch + K + 2, 2 * K * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  FMX_HIP(hipStreamSynchronize(st));  // staging buffers may be reused after return
  c->max_chunks = std::max<uint32_t>(nch, 1);
  c->rows_pl = Np;
  c->rows_pt = Nt;
  c->counts_pending = false;
  c->have_corr = true;
  c->have_match = false;
}

}  // namespace fmx
