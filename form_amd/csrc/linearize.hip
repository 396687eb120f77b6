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

#include "factor_rows.hpp"

// One wave per chunk (<= kPlaneChunk plane rows or <= kPointChunk point pairs of one
// pair, strided over the lanes); the wave's NG sums go to partials[NG][max_chunks].
template <int MODE>
__global__ __launch_bounds__(kLinThreads) void k_linearize(const Chunk* __restrict__ chunks,
                                                           const uint32_t* __restrict__ n_chunks,
                                                           const double* __restrict__ c_pl, size_t ld_pl,
                                                           const double* __restrict__ c_pt, size_t ld_pt,
                                                           const double* __restrict__ poses, double inv,
                                                           double* __restrict__ partials, size_t ldp,
                                                           const IcpDev* __restrict__ icp, Pose34 tjv, int tj_by_value) {
  constexpr int NG = LinShape<MODE>::NG;
  if (icp && (icp->icp_done || icp->phase == 2)) return;  // device LM finished
  const uint32_t ch = blockIdx.x;
  if (ch >= *n_chunks) return;
  const Chunk d = chunks[ch];
  // poses: [K][Ti | Tj] (general API), or the map poses [K][Ti] with Tj from the
  // device LM state (current / trial pose) or passed by value
  const bool mapi = icp || tj_by_value;
  const double* Ti = mapi ? poses + 12 * d.pair : poses + 24 * d.pair;
  const double* Tj = icp ? (icp->phase == 0 ? icp->T : icp->Tn) : (tj_by_value ? tjv.m : Ti + 12);
  double acc[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) acc[i] = 0.0;
  double H[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) H[i] = 0.0;
  for (uint32_t row = d.begin + threadIdx.x; row < d.end; row += kLinThreads) {
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

// ============================================================================ device LM
// Single-pose Levenberg-Marquardt (GTSAM LevenbergMarquardtOptimizer defaults, the
// same algorithm as the host DeviceLM in fmx_api.cpp and the oracle) and the ICP
// loop control of form.cpp:67-93, run by single-lane kernels against IcpDev so the
// host syncs once per ICP iteration instead of once per linearization.

__device__ __forceinline__ void dpose_compose(const double* a, const double* b, double* o) {
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) o[4 * i + j] = (a[4 * i] * b[j] + a[4 * i + 1] * b[4 + j]) + a[4 * i + 2] * b[8 + j];
    o[4 * i + 3] = ((a[4 * i] * b[3] + a[4 * i + 1] * b[7]) + a[4 * i + 2] * b[11]) + a[4 * i + 3];
  }
}
__device__ __forceinline__ void dpose_inverse(const double* a, double* o) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) o[4 * i + j] = a[4 * j + i];
  const double nt[3] = {-a[3], -a[7], -a[11]};
  for (int i = 0; i < 3; ++i) o[4 * i + 3] = (o[4 * i] * nt[0] + o[4 * i + 1] * nt[1]) + o[4 * i + 2] * nt[2];
}
__device__ __forceinline__ void dcross(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ __forceinline__ void dpose_expmap(const double xi[6], double* T) {
  const double* w = xi;
  const double* v = xi + 3;
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  double A, B, a, b;
  if (th2 <= 2.220446049250313e-16) {
    A = 1.0;
    B = 0.5;
    a = 0.5;
    b = 1.0 / 6.0;
  } else {
    const double th = sqrt(th2);
    A = sin(th) / th;
    B = (1.0 - cos(th)) / th2;
    a = B;
    b = (th - sin(th)) / (th2 * th);
  }
  const double W[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const double w2 = W[i][0] * W[0][j] + W[i][1] * W[1][j] + W[i][2] * W[2][j];
      T[4 * i + j] = (i == j ? 1.0 : 0.0) + A * W[i][j] + B * w2;
    }
  double wxv[3], wxwxv[3];
  dcross(w, v, wxv);
  dcross(w, wxv, wxwxv);
  for (int i = 0; i < 3; ++i) T[4 * i + 3] = v[i] + a * wxv[i] + b * wxwxv[i];
}
__device__ double dpose_lognorm(const double* m) {  // ||Pose3::Logmap(T)||
  const double tr = m[0] + m[5] + m[10];
  double w[3];
  if (tr + 1.0 < 1e-10) {
    if (fabs(m[10] + 1.0) > 1e-10) {
      const double s = M_PI / sqrt(2.0 + 2.0 * m[10]);
      w[0] = s * m[2]; w[1] = s * m[6]; w[2] = s * (1.0 + m[10]);
    } else if (fabs(m[5] + 1.0) > 1e-10) {
      const double s = M_PI / sqrt(2.0 + 2.0 * m[5]);
      w[0] = s * m[1]; w[1] = s * (1.0 + m[5]); w[2] = s * m[9];
    } else {
      const double s = M_PI / sqrt(2.0 + 2.0 * m[0]);
      w[0] = s * (1.0 + m[0]); w[1] = s * m[4]; w[2] = s * m[8];
    }
  } else {
    const double tr_3 = tr - 3.0;
    double mag;
    if (tr_3 < -1e-7) {
      const double th = acos((tr - 1.0) / 2.0);
      mag = th / (2.0 * sin(th));
    } else {
      mag = 0.5 - tr_3 * tr_3 / 12.0;
    }
    w[0] = mag * (m[9] - m[6]);
    w[1] = mag * (m[2] - m[8]);
    w[2] = mag * (m[4] - m[1]);
  }
  const double t = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  double xi[6] = {w[0], w[1], w[2], m[3], m[7], m[11]};
  if (t >= 1e-10) {
    const double wn[3] = {w[0] / t, w[1] / t, w[2] / t};
    const double tt[3] = {m[3], m[7], m[11]};
    double WT[3], WWT[3];
    dcross(wn, tt, WT);
    dcross(wn, WT, WWT);
    const double Tan = tan(0.5 * t);
    for (int i = 0; i < 3; ++i) xi[3 + i] = tt[i] - (0.5 * t) * WT[i] + (1 - t / (2. * Tan)) * WWT[i];
  }
  double n = 0;
  for (int i = 0; i < 6; ++i) n += xi[i] * xi[i];
  return sqrt(n);
}
__device__ __forceinline__ bool dchol_solve6(const double* H, const double* g, double lambda, double* x) {
  double L[6][6];
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) L[i][j] = 0.0;
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = H[6 * i + j] + (i == j ? lambda : 0.0);
      for (int k = 0; k < j; ++k) s -= L[i][k] * L[j][k];
      if (i == j) {
        if (s <= 0) return false;
        L[i][i] = sqrt(s);
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

// LM state held in registers by the deciding lane (IcpDev fields it touches).
struct LmReg {
  double T[12], Tn[12], H[36], g[6], c, err, lambda, cur, linchg;
  int phase, lm_iters;
};

// Advance the LM state machine until a trial pose is proposed (phase 1) or the
// optimization ends (phase 2).  end_first: finish the current iteration first
// (NonlinearOptimizer::defaultOptimize's convergence test), else propose directly
// (tryLambda's solve: Cholesky of H + lambda I, validity of the linearized decrease,
// increaseLambda on failure, give up at the upper bound 1e5).
__device__ __forceinline__ void lm_advance(LmReg& s, bool end_first) {
  bool end = end_first;
  for (int guard = 0; guard < 256; ++guard) {
    if (end) {
      s.lm_iters++;
      const double newErr = s.err;
      bool conv;
      if (newErr <= 0.0) conv = true;
      else {
        const double absDec = s.cur - newErr, relDec = absDec / s.cur;
        conv = (relDec <= 1e-5) || (absDec <= 1e-5);
      }
      if (conv || s.lm_iters >= 100 || !isfinite(s.cur)) {
        s.phase = 2;
        return;
      }
      s.cur = newErr;
      end = false;
    }
    const double oldLin = 0.5 * s.c;
    double dx[6];
    if (dchol_solve6(s.H, s.g, s.lambda, dx)) {
      double dHd = 0, dg = 0;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        double h = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) h += s.H[6 * i + j] * dx[j];
        dHd += dx[i] * h;
        dg += dx[i] * s.g[i];
      }
      const double newLin = 0.5 * (dHd - 2 * dg + s.c);
      const double linChange = oldLin - newLin;
      if (linChange >= 0) {
        double E[12];
        dpose_expmap(dx, E);
        dpose_compose(s.T, E, s.Tn);
        s.linchg = linChange;
        s.phase = 1;
        return;
      }
    }
    s.lambda *= 10.0;  // step not valid: increaseLambda
    if (s.lambda >= 1e5) end = true;
  }
  s.phase = 2;
}

// One LM decision (GTSAM LevenbergMarquardtOptimizer, see lm_advance) on a register
// copy of the state, from the summed 7 x 7 system S (packed upper) and error e.
__device__ __forceinline__ void lm_decide(IcpDev* __restrict__ s, const double* S /* LDS */, double e) {
  LmReg r;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    r.T[i] = s->T[i];
    r.Tn[i] = s->Tn[i];
  }
#pragma unroll
  for (int i = 0; i < 36; ++i) r.H[i] = s->H[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) r.g[i] = s->g[i];
  r.c = s->c;
  r.err = s->err;
  r.lambda = s->lambda;
  r.cur = s->cur;
  r.linchg = s->linchg;
  r.phase = s->phase;
  r.lm_iters = s->lm_iters;
  double H[36], g[6], c = 0;
  {
    int o = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = i; j < 7; ++j) {
        const double v = S[o++];
        if (i < 6 && j < 6) {
          H[6 * i + j] = v;
          H[6 * j + i] = v;
        } else if (i < 6) {
          g[i] = v;
        } else {
          c = v;
        }
      }
  }
  if (r.phase == 0) {  // initial linearization at T
#pragma unroll
    for (int i = 0; i < 36; ++i) r.H[i] = H[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) r.g[i] = g[i];
    r.c = c;
    r.err = e;
    if (e <= 0.0) r.phase = 2;
    else {
      r.cur = e;
      lm_advance(r, false);
    }
  } else {  // trial linearized at Tn: tryLambda's accept test (minModelFidelity 1e-3)
    const double oldLin = 0.5 * r.c;
    const double costChange = r.err - e;
    bool success;
    if (r.linchg > 2.220446049250313e-16 * oldLin) success = (costChange / r.linchg) > 1e-3;
    else success = true;
    const bool stop = fabs(costChange) < 1e-5 * r.err;
    if (success) {
      r.lambda = fmax(0.0, r.lambda / 10.0);
#pragma unroll
      for (int i = 0; i < 12; ++i) r.T[i] = r.Tn[i];
#pragma unroll
      for (int i = 0; i < 36; ++i) r.H[i] = H[i];
#pragma unroll
      for (int i = 0; i < 6; ++i) r.g[i] = g[i];
      r.c = c;
      r.err = e;
      lm_advance(r, true);
    } else if (!stop) {
      r.lambda *= 10.0;
      lm_advance(r, r.lambda >= 1e5);
    } else {
      lm_advance(r, true);
    }
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    s->T[i] = r.T[i];
    s->Tn[i] = r.Tn[i];
  }
#pragma unroll
  for (int i = 0; i < 36; ++i) s->H[i] = r.H[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) s->g[i] = r.g[i];
  s->c = r.c;
  s->err = r.err;
  s->lambda = r.lambda;
  s->cur = r.cur;
  s->linchg = r.linchg;
  s->phase = r.phase;
  s->lm_iters = r.lm_iters;
  s->lins++;
}

// ---------------------------------------------------------------- fused total
// register_scan's linearization (single pose): the sum over ALL pairs of
// [H_j b]^T [H_j b] (28 doubles) and the error, in one launch.  16 waves per block,
// one 64-row chunk each.  Each wave reduce-scatters its 28 (+4 pad) sums across the
// lanes (5 halving steps + 1: 32 shuffles instead of 28 butterflies), the block adds
// its waves in order, the block partial goes out with sc1 (write-through) stores,
// each block takes an agent-scope ticket, and the last block sums the block partials
// with sc1 loads in a fixed order (MI355X_MICROARCH.md, inter-workgroup hand-off,
// row 1: no fences needed).  Host mode writes G and err to mapped memory; device mode
// (DEVLM) takes the LM decision in the same block.
// Host mode: 16 waves per block.  Device-LM mode: 4 waves, so the inlined LM
// decision gets 256 VGPRs without spilling (the grid is < 1 block per CU anyway).
constexpr int kTotWavesHost = 16, kTotWavesDev = 4;
constexpr int kTotLd = 32;  // doubles per block partial (28 used)
template <bool DEVLM>
constexpr int tot_waves() { return DEVLM ? kTotWavesDev : kTotWavesHost; }

// v[0..31] summed over the wave; afterwards lanes 2i and 2i+1 hold entry i in v[0].
__device__ __forceinline__ double wave_reduce_scatter32(double (&v)[32]) {
  const int lane = lane_id();
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int half = 16 >> k;
    const bool hi = (lane >> (5 - k)) & 1;
#pragma unroll
    for (int j = 0; j < half; ++j) {
      const double a = v[j], b = v[j + half];
      const double send = hi ? a : b;
      const double keep = hi ? b : a;
      v[j] = keep + __shfl_xor(send, 32 >> k, 64);
    }
  }
  return v[0] + __shfl_xor(v[0], 1, 64);
}

// Rows in query order (the match outputs, no pair sort): query gq < nq_pl is a plane
// row (p_i = m_pi, n_i = m_ni, p_j = q_pl), else a point pair (p_i = m_pi, p_j =
// q_pt); m_pair < 0 (not accepted) contributes nothing; T_i = poses[m_pair].
struct QoRows {
  const int32_t* pair;
  const double4* pi;
  const double4* ni;
  const float4* q_pl;
  const float4* q_pt;
  uint32_t nq_pl, nq;
};

template <bool DEVLM>
__global__ __launch_bounds__(tot_waves<DEVLM>() * kWave) void k_linearize_total(
    QoRows qo, const double* __restrict__ poses, double inv, double* __restrict__ bpart, uint32_t* __restrict__ ticket,
    double* __restrict__ out, IcpDev* __restrict__ icp, Pose34 tjv, uint32_t* __restrict__ flag, uint32_t seq) {
  constexpr int NG = 28;
  constexpr int kTotWaves = tot_waves<DEVLM>();
  constexpr int kTotGroups = kTotWaves * kWave / NG;  // final reduction: lane groups x 28 entries
  if (icp && (icp->icp_done || icp->phase == 2)) return;  // uniform: device LM finished
  const int w = threadIdx.x / kWave, lane = lane_id();
  const uint32_t ch = blockIdx.x * kTotWaves + w;
  double acc[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) acc[i] = 0.0;
  const uint32_t gq = ch * kWave + lane;
  const int32_t pair = gq < qo.nq ? qo.pair[gq] : -1;
  if (pair >= 0) {
    const double* Ti = poses + 12 * pair;
    const double* Tj = icp ? (icp->phase == 0 ? icp->T : icp->Tn) : tjv.m;
    double H[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) H[i] = 0.0;
    const double4 p4 = qo.pi[gq];
    const double pi[3] = {p4.x, p4.y, p4.z};
    {
      if (gq < qo.nq_pl) {
        const double4 n4 = qo.ni[gq];
        const float4 q = qo.q_pl[gq];
        const double ni[3] = {n4.x, n4.y, n4.z};
        const double pj[3] = {(double)q.x, (double)q.y, (double)q.z};
        double r;
        plane_row<1>(Ti, Tj, pi, ni, pj, r, H);
        accum_row<1>(H, r, inv, acc);
      } else {
        const float4 q = qo.q_pt[gq - qo.nq_pl];
        const double pj[3] = {(double)q.x, (double)q.y, (double)q.z};
        double wpi[3], wpj[3];
        d_xform(Ti, pi[0], pi[1], pi[2], wpi);
        d_xform(Tj, pj[0], pj[1], pj[2], wpj);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          double r;
          point_row<1>(Ti, Tj, pi, pj, wpi, wpj, a, r, H);
          accum_row<1>(H, r, inv, acc);
        }
      }
    }
  }
  __shared__ double sw[kTotWaves][NG];
  __shared__ double sq[kTotGroups][NG];
  __shared__ double sS[NG + 1];
  __shared__ int s_last;
  const double mine = wave_reduce_scatter32(acc);  // entry lane / 2
  if ((lane & 1) == 0 && (lane >> 1) < NG) sw[w][lane >> 1] = mine;
  __syncthreads();
  if (threadIdx.x < NG) {
    const int t = threadIdx.x;
    double bp = sw[0][t];
#pragma unroll
    for (int i = 1; i < kTotWaves; ++i) bp += sw[i][t];
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(bpart + (size_t)blockIdx.x * kTotLd + t),
                       (unsigned long long)__double_as_longlong(bp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  // last block: lane group j (36 of them) sums entry e of blocks j, j + 36, ...;
  // then the 36 group sums in order
  const int nblk = gridDim.x;
  if (threadIdx.x < kTotGroups * NG) {
    const int e = threadIdx.x % NG, j = threadIdx.x / NG;
    double s = 0.0;
    for (int b = j; b < nblk; b += kTotGroups)
      s += __longlong_as_double((long long)__hip_atomic_load(
          reinterpret_cast<const unsigned long long*>(bpart + (size_t)b * kTotLd + e), __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_AGENT));
    sq[j][e] = s;
  }
  __syncthreads();
  if (threadIdx.x < NG) {
    const int e = threadIdx.x;
    double s = sq[0][e];
#pragma unroll
    for (int j = 1; j < kTotGroups; ++j) s += sq[j][e];
    sS[e] = s;
    if (!icp) host_store(out + e, s);
    if (e == NG - 1) {
      sS[NG] = 0.5 * s;
      if (!icp) host_store(out + NG, 0.5 * s);
    }
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (flag) publish_flag(flag, seq);  // out[] was stored by this wave
  }
  __syncthreads();
  if constexpr (DEVLM) {
    if (threadIdx.x == 0) lm_decide(icp, sS, sS[NG]);
  }
}

// form.cpp:71-72: before = current pose; LM restarts (lambda0) from it.
__global__ void k_icp_begin(IcpDev* s) {
  if (s->icp_done) return;
  for (int i = 0; i < 12; ++i) s->Tbefore[i] = s->T[i] = s->Tcur[i];
  s->phase = 0;
  s->lambda = 1e-5;
  s->lm_iters = 0;
  s->icp_iters++;
}
// form.cpp:83-88 (end != 0): stop if ||before.localCoordinates(after)|| < threshold,
// else update_current_pose(after).  Then one wave copies the state to pinned host
// memory and publishes the completion word (the host's once-per-ICP-iteration read).
__global__ __launch_bounds__(64) void k_icp_end(IcpDev* s, int end, double thr, IcpDev* host, uint32_t* flag,
                                                uint32_t seq) {
  if (threadIdx.x == 0 && end && !(s->icp_done || s->phase != 2 || s->ended == s->icp_iters)) {
    s->ended = s->icp_iters;
    s->lm_total += s->lm_iters;
    double Bi[12], D[12];
    dpose_inverse(s->Tbefore, Bi);
    dpose_compose(Bi, s->T, D);
    if (dpose_lognorm(D) < thr) s->icp_done = 1;
    else
      for (int i = 0; i < 12; ++i) s->Tcur[i] = s->T[i];
  }
  __syncthreads();
  static_assert(sizeof(IcpDev) % 4 == 0, "IcpDev copied as words");
  const uint32_t* src = reinterpret_cast<const uint32_t*>(s);
  uint32_t* dst = reinterpret_cast<uint32_t*>(host);
  for (int i = threadIdx.x; i < (int)(sizeof(IcpDev) / 4); i += 64) host_store(dst + i, src[i]);
  if (threadIdx.x == 0) publish_flag(flag, seq);  // the single wave made every store
}
// optimize(false) after an unconverged loop: LM from the current pose.
__global__ void k_lm_begin(IcpDev* s) {
  for (int i = 0; i < 12; ++i) s->T[i] = s->Tcur[i];
  s->phase = 0;
  s->lambda = 1e-5;
  s->lm_iters = 0;
}

}  // namespace

static void linearize_impl(fmx_ctx* c, const double* poses_i34, const double* poses_j34, const double* tj_val,
                           double sigma, int mode, double* G_out, double* err_out) {
  if (!c->have_corr) throw StatusError(FMX_E_STATE, "no correspondences (call fmx_match or fmx_corr_set)");
  hipStream_t st = c->stream;
  const int K = (int)c->K;
  if (K == 0) return;
  const int NG = mode == 0 ? 91 : (mode == 1 ? 28 : 1);
  Pose34 tjv{};
  const int tj_by_value = tj_val ? 1 : 0;
  const double* dposes = c->map_poses_p;
  if (tj_val) {
    std::memcpy(tjv.m, tj_val, sizeof(tjv.m));
  } else {
    c->h_poses.ensure(24 * (size_t)K);
    for (int k = 0; k < K; ++k) {
      std::memcpy(c->h_poses.p + 24 * k, poses_i34 + 12 * k, 12 * sizeof(double));
      std::memcpy(c->h_poses.p + 24 * k + 12, poses_j34 + 12 * k, 12 * sizeof(double));
    }
    c->poses_ij.ensure(24 * (size_t)K);
    FMX_HIP(hipMemcpyAsync(c->poses_ij.p, c->h_poses.p, 24 * K * sizeof(double), hipMemcpyHostToDevice, st));
    dposes = c->poses_ij.p;
  }
  c->partials.ensure((size_t)std::max<uint32_t>(c->max_chunks, 1) * 91 + 1);
  const size_t nout = (size_t)K * (mode == 2 ? 1 : NG + 1);
  c->h_G.ensure(nout + 1);
  double* dG = c->h_G.d;  // k_lin_final writes G / err into mapped host memory (no copy op)
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
                         c->ld_pl, c->c_pt.p, c->ld_pt, dposes, inv, c->partials.p, ldp,
                         (const IcpDev*)nullptr, tjv, tj_by_value);
    else if (mode == 1)
      hipLaunchKernelGGL(k_linearize<1>, dim3(nb), dim3(kLinThreads), 0, st, c->chunks.p, c->n_chunks.p, c->c_pl.p,
                         c->ld_pl, c->c_pt.p, c->ld_pt, dposes, inv, c->partials.p, ldp,
                         (const IcpDev*)nullptr, tjv, tj_by_value);
    else
      hipLaunchKernelGGL(k_linearize<2>, dim3(nb), dim3(kLinThreads), 0, st, c->chunks.p, c->n_chunks.p, c->c_pl.p,
                         c->ld_pl, c->c_pt.p, c->ld_pt, dposes, inv, c->partials.p, ldp,
                         (const IcpDev*)nullptr, tjv, tj_by_value);
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
  stream_wait(c);
  match_counts_fetch(c);  // already copied; no extra wait
  if (mode == 2) {
    if (err_out) std::memcpy(err_out, c->h_G.p, K * sizeof(double));
  } else {
    if (G_out) std::memcpy(G_out, c->h_G.p, (size_t)K * NG * sizeof(double));
    if (err_out) std::memcpy(err_out, c->h_G.p + (size_t)K * NG, K * sizeof(double));
  }
}

void run_linearize(fmx_ctx* c, const double* poses_i34, const double* poses_j34, double sigma, int mode,
                   double* G_out, double* err_out) {
  linearize_impl(c, poses_i34, poses_j34, nullptr, sigma, mode, G_out, err_out);
}
void run_linearize_mapj(fmx_ctx* c, const double* pose_j34, double sigma, int mode, double* G_out, double* err_out) {
  if (!c->have_map) throw StatusError(FMX_E_STATE, "no map");
  linearize_impl(c, nullptr, nullptr, pose_j34, sigma, mode, G_out, err_out);
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

namespace fmx {

// blocks of k_linearize_total over the last query-order match (64 queries per wave)
// (+ the partial / ticket buffers it needs; the ticket starts at 0 and the last block
// resets it)
static uint32_t tot_blocks(fmx_ctx* c, int waves) {
  const uint32_t nch = (c->n_qo + kWave - 1) / kWave;
  const uint32_t nblk = std::max<uint32_t>((nch + waves - 1) / waves, 1);
  c->bpart.ensure((size_t)nblk * kTotLd);
  ensure_zeroed(c->ticket, 1, c->stream);
  return nblk;
}
static QoRows qo_rows(fmx_ctx* c) {
  return QoRows{c->m_pair.p, reinterpret_cast<const double4*>(c->m_pi.p), reinterpret_cast<const double4*>(c->m_ni.p),
                c->q_pl_pos.p, c->q_pt_pos.p, c->n_qpl, c->n_qo};
}

void icp_launch(fmx_ctx* c, int what) {
  hipStream_t st = c->stream;
  if (what == 0) hipLaunchKernelGGL(k_icp_begin, dim3(1), dim3(1), 0, st, c->icp.p);
  else if (what == 1 || what == 3) {  // 1: end the ICP iteration + read back; 3: read back only
    const uint32_t seq = next_flag(c);
    hipLaunchKernelGGL(k_icp_end, dim3(1), dim3(64), 0, st, c->icp.p, what == 1 ? 1 : 0, c->P.new_pose_threshold,
                       c->h_icp.d, c->h_flag.d, seq);
    FMX_HIP(hipGetLastError());
    wait_flag(c, c->h_flag.p, seq);
    return;
  } else hipLaunchKernelGGL(k_lm_begin, dim3(1), dim3(1), 0, st, c->icp.p);
  FMX_HIP(hipGetLastError());
}

// `rounds` x (fused linearize + reduce + LM decision); no host sync.
void lm_rounds(fmx_ctx* c, int rounds) {
  hipStream_t st = c->stream;
  const uint32_t nblk = tot_blocks(c, kTotWavesDev);
  const double inv = 1.0 / c->P.planar_constraint_sigma;
  const QoRows qo = qo_rows(c);
  for (int r = 0; r < rounds; ++r) {
    ProfScope ps(c->prof, PROF_LINEARIZE, 4.0 * c->n_qo + 80.0 * c->rows_pl + 48.0 * c->rows_pt, st);
    // K = 0 or no queries still launches: the LM decides on the empty system
    hipLaunchKernelGGL(k_linearize_total<true>, dim3(nblk), dim3(kTotWavesDev * kWave), 0, st, qo, c->map_poses_p,
                       inv, c->bpart.p, c->ticket.p, (double*)nullptr, c->icp.p, Pose34{}, (uint32_t*)nullptr, 0u);
    FMX_HIP(hipGetLastError());
  }
}

// register_scan's host-LM linearization: out[0..27] = sum over pairs of the packed
// 7 x 7 [H_j b]^T [H_j b] at pose_j, out[28] = error.  One launch, one wait.
void run_linearize_total(fmx_ctx* c, const double* pose_j34, double sigma, double* out) {
  if (!c->have_map) throw StatusError(FMX_E_STATE, "no map");
  if (!c->have_qo) throw StatusError(FMX_E_STATE, "no query-order match");
  hipStream_t st = c->stream;
  for (int i = 0; i < 29; ++i) out[i] = 0.0;
  if (c->K == 0 || c->n_qo == 0) return;
  const uint32_t nblk = tot_blocks(c, kTotWavesHost);
  Pose34 tjv;
  std::memcpy(tjv.m, pose_j34, sizeof(tjv.m));
  c->h_G.ensure(32);
  const uint32_t seq = next_flag(c);
  if (c->counts_pending && c->prof.on) match_counts_fetch(c);  // exact byte model for the profile
  {
    // bytes: pair id per query + (p_i, n_i 32 B each, p_j 16 B) per accepted plane row,
    // (p_i 32 B, p_j 16 B) per accepted point pair
    ProfScope ps(c->prof, PROF_LINEARIZE, 4.0 * c->n_qo + 80.0 * c->rows_pl + 48.0 * c->rows_pt, st);
    hipLaunchKernelGGL(k_linearize_total<false>, dim3(nblk), dim3(kTotWavesHost * kWave), 0, st, qo_rows(c),
                       c->map_poses_p, 1.0 / sigma, c->bpart.p, c->ticket.p, c->h_G.d, (IcpDev*)nullptr, tjv,
                       c->h_flag.d, seq);
    FMX_HIP(hipGetLastError());
  }
  wait_flag(c, c->h_flag.p, seq);
  match_counts_fetch(c, false);  // the match kernel finished before this one started
  std::memcpy(out, c->h_G.p, 29 * sizeof(double));
}

}  // namespace fmx
