// window.hip — smoothing mode (ConstraintManager's default, disable_smoothing = false,
// form/optimization/constraints.hpp:54-56): the window's correspondence store and the
// batched linearization of MANY FeatureFactors per launch.
//
// The reference keeps every scan's matches as PlanePoint/PointPoint buffers per pair
// (m_constraints[j][i], constraints.hpp:95-101) until scan i or j is marginalized, and
// GTSAM linearizes them factor by factor:
//   * fast mode  — the current scan's FeatureFactors every LM iteration of the ICP
//                  loop (get_graph(true), constraints.cpp:257-266);
//   * full mode  — every pair every LM iteration of optimize(false)
//                  (constraints.cpp:294-305, form.cpp:92);
//   * m_fast_linear / marginalize — every previous (resp. dropped) pair once per scan
//                  (constraints.cpp:268-288, 164-167).
// Here: a device arena of pair-major SoA rows (plane p_i, n_i, p_j = 9 doubles; point
// p_i, p_j = 6 doubles, the same layout the sorted match writes), one segment per
// scan j, and k_win_linearize: DenseFactor::linearize (gtsam.hpp:67-86) of a list of
// pairs in ONE launch, 13 x 13 augmented information (91 doubles) + error per pair.
//
// k_win_linearize: one wave per chunk (<= kWinPlaneRows plane rows or kWinPointPairs
// point pairs of one pair, 64 per step, the next step's rows loaded while one
// computes), the 13 x 13 sums on the fp64 matrix cores (stage_and_mfma), agent-
// scope partial stores (visible across XCD L2s), a per-pair ticket whose last chunk
// sums the pair's partials in chunk order (deterministic) and stores that pair's G to
// pinned host memory (write-through) and drains; a ticket over pairs lets the last
// finisher publish the completion word.  HBM-bound: 72 B per plane row, 48 B per
// point pair, ~300 / ~900 flop.
#include "fmx_device.hpp"
#include "fmx_internal.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace fmx {
namespace {

#include "factor_rows.hpp"

constexpr int kWinWaves = kPlaneChunk / kWave;  // waves per block: one chunk, one 64-row step per wave
// (128-row chunks measured slower, 0.22 vs 0.19 ms per scan; a one-wave block, 64 rows,
// is not a supported configuration: its C4 stream came out different — 2.4x the probes
// and candidates per match query, not a parity-tested build; profiles/r3_ab_c4_window_rows.txt)
static_assert(kPlaneChunk == kPointChunk && kPlaneChunk % kWave == 0 && kWinWaves >= 2 && kWinWaves <= 16,
              "window chunking");
constexpr int kFinBatch = 16;   // chunk partials in flight per thread in the pair finisher
constexpr int kWinLd = 96;      // doubles per chunk partial (91 used)
constexpr int kWinG = 92;       // per pair: 91 G entries + error
constexpr int kLdsStride = 13;  // doubles per staged row (13 entries; the pad lanes read 0)
constexpr int kPairedPoses = -2;  // WinArgs::implicit_j: fmx_linearize's per-pair (T_i, T_j) table

typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void agent_store(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double agent_load(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

struct WinArgs {
  const Chunk* chunks;
  const uint32_t* n_chunks;     // device count (chunks of the sorted match) ...
  uint32_t n_chunks_host;       // ... or this when n_chunks is null
  const uint32_t* chunk_range;  // [npairs + 1]
  int npairs;
  const double* c_pl;
  size_t ld_pl;
  const double* c_pt;
  size_t ld_pt;
  const double* dposes;  // pose table in device memory, or null: by value (WinPoses)
  int implicit_j;        // >= 0: chunk.pair indexes pose i, pose j = implicit_j;
                         // kPairedPoses: pair k's poses are table entries 2k (i) and 2k + 1 (j);
                         // else the slots packed in chunk.type
  double inv;            // 1 / sigma (FastIsotropic invsigma_, gtsam.hpp:96)
  double* partials;      // [chunk][kWinLd]
  uint32_t* pair_ticket; // [pair], self-resetting
  uint32_t* done_ticket; // self-resetting
  double* hostG;         // pinned mapped [pair][kWinG]
  uint32_t* flag;
  uint32_t seq;
  uint64_t* dbg;  // FMX_WIN_TIMING: per-wave s_memrealtime stamps [chunk][8], else null
};

#define WSTAMP(i)                                                            \
  do {                                                                       \
    if (a.dbg && threadIdx.x == 0) a.dbg[(size_t)ch * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// The augmented information of a chunk, sum_rows a a^T with a = [H_i H_j -r] / sigma
// (13 wide, padded to 16), is a 16 x 16 x rows fp64 GEMM: one v_mfma_f64_16x16x4_f64
// per 4 rows.  Each lane builds one row's a-vector (64 rows per wave step), stages
// its 13 entries in LDS, and lane l feeds a_{4t + l/16}[l % 16] (0 for l % 16 >= 13)
// as BOTH operands of MFMA t (A[i][k] = a_k[i], B[k][j] = a_k[j]); the 16 x 16 result
// accumulates in 4 registers per lane (row (l >> 4) + 4 r, column l & 15): no
// cross-lane reduction, no 91 accumulators.  The 16 operand reads are issued before
// the MFMA chain (one LDS wait per step).
__device__ __forceinline__ void stage_and_mfma(double* __restrict__ rows /* this wave's LDS */, const double (&av)[13],
                                               bool valid, f64x4 (&acc)[4]) {
  const int lane = lane_id();
  double* mine = rows + lane * kLdsStride;
#pragma unroll
  for (int i = 0; i < 13; ++i) mine[i] = valid ? av[i] : 0.0;
  __builtin_amdgcn_wave_barrier();
  const int col = lane & 15;
  const double* src = rows + (lane >> 4) * kLdsStride + (col < 13 ? col : 0);
  double v[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] = src[4 * t * kLdsStride];
#pragma unroll
  for (int t = 0; t < 16; ++t) {  // four independent chains: a dependent f64 MFMA waits ~3x its issue time
    const double x = col < 13 ? v[t] : 0.0;
    acc[t & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, acc[t & 3], 0, 0, 0);
  }
  __builtin_amdgcn_wave_barrier();
}

// One block (kWinWaves waves) per chunk (<= kPlaneChunk plane rows or kPointChunk
// point pairs of one pair); wave w takes rows [64 w, 64 w + 64) of it, one step.
// The waves' 16 x 16 sums meet in LDS (fixed wave order).  A pair of one chunk: the
// block writes G to pinned host memory itself; more: block partials (agent-scope
// stores), a per-pair ticket, the pair's last chunk sums the partials in chunk order.
// Then a ticket over the pairs with rows lets the last finisher publish the word.
// NP: by-value pose capacity (kernel-argument bytes: a smaller block launches faster)
template <int NP>
__global__ __launch_bounds__(kWinWaves * kWave) void k_win_linearize(WinArgs a, WinPosesN<NP> wp) {
  __shared__ double s_rows[kWinWaves][kWave * kLdsStride];
  __shared__ double s_g[kWinWaves][92];
  __shared__ uint32_t s_t;
  const int w = threadIdx.x / kWave, lane = lane_id(), tid = threadIdx.x;
  const uint32_t ch = blockIdx.x;
  const uint32_t nch = a.n_chunks ? *a.n_chunks : a.n_chunks_host;
  // the chunk descriptor in the same round as the count (a device count: ch < grid <=
  // the table's capacity, an entry past the count is read and never used; a host count:
  // only entries below it)
  Chunk d{};
  if (a.n_chunks || ch < a.n_chunks_host) d = a.chunks[ch];
  if (nch == 0) {  // nothing to linearize: publish at once
    if (blockIdx.x == 0 && tid == 0) publish_flag(a.flag, a.seq);
    return;
  }
  if (ch >= nch) return;
  WSTAMP(0);
  const uint32_t type = d.type & 0xFFu;
  const int slot = (int)d.pair;
  // the pair's chunk range, in flight with the rows (used after the block sum); wave 0
  // also counts the pairs with rows for the done ticket now, off the finisher's chain
  const uint32_t cb = a.chunk_range[slot], ce = a.chunk_range[slot + 1];
  uint32_t n_ne = 0;
  if (w == 0)
    for (int k0 = 0; k0 < a.npairs; k0 += kWave) {
      const int k = k0 + lane;
      const bool ne = k < a.npairs && a.chunk_range[k + 1] > a.chunk_range[k];
      n_ne += (uint32_t)__popcll(__ballot(ne));
    }
  int pi, pj;
  if (a.implicit_j >= 0) {
    pi = slot;
    pj = a.implicit_j;
  } else if (a.implicit_j == kPairedPoses) {
    pi = 2 * slot;
    pj = 2 * slot + 1;
  } else {
    pi = (int)((d.type >> 8) & 0xFFFu);
    pj = (int)(d.type >> 20);
  }
  const double* Ti = a.dposes ? a.dposes + 12 * pi : wp.m[pi];
  const double* Tj = a.dposes ? a.dposes + 12 * pj : wp.m[pj];
  f64x4 accs[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) accs[i] = f64x4{0.0, 0.0, 0.0, 0.0};
  const uint32_t row = d.begin + w * kWave + lane;
  if (d.begin + w * kWave < d.end) {  // wave-uniform: this wave has rows
    WSTAMP(7);
    double* rows = s_rows[w];
    double H[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) H[i] = 0.0;
    double av[13];
    const bool valid = row < d.end;
    if (type == 0) {
      double c[9];
      if (valid) {
#pragma unroll
        for (int q = 0; q < 9; ++q) c[q] = a.c_pl[row + q * a.ld_pl];
        const double pi3[3] = {c[0], c[1], c[2]}, ni3[3] = {c[3], c[4], c[5]}, pj3[3] = {c[6], c[7], c[8]};
        double r;
        plane_row<0>(Ti, Tj, pi3, ni3, pj3, r, H);
#pragma unroll
        for (int q = 0; q < 12; ++q) av[q] = H[q] * a.inv;
        av[12] = -r * a.inv;
      }
      stage_and_mfma(rows, av, valid, accs);
    } else {
      double c[6] = {0, 0, 0, 0, 0, 0};
      if (valid) {
#pragma unroll
        for (int q = 0; q < 6; ++q) c[q] = a.c_pt[row + q * a.ld_pt];
      }
      const double pi3[3] = {c[0], c[1], c[2]}, pj3[3] = {c[3], c[4], c[5]};
      double wpi[3], wpj[3];
      d_xform(Ti, pi3[0], pi3[1], pi3[2], wpi);
      d_xform(Tj, pj3[0], pj3[1], pj3[2], wpj);
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        if (valid) {
          double r;
          point_row<0>(Ti, Tj, pi3, pj3, wpi, wpj, ax, r, H);
#pragma unroll
          for (int q = 0; q < 12; ++q) av[q] = H[q] * a.inv;
          av[12] = -r * a.inv;
        }
        stage_and_mfma(rows, av, valid, accs);
      }
    }
  }
  // wave sums (packed upper 13 x 13) -> LDS; block sum in wave order
  const f64x4 acc = (accs[0] + accs[1]) + (accs[2] + accs[3]);
  {
    const int col = lane & 15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = (lane >> 4) + 4 * r;
      if (rr <= col && col < 13) s_g[w][rr * 13 - rr * (rr - 1) / 2 + (col - rr)] = acc[r];
    }
  }
  __syncthreads();
  WSTAMP(1);
  double bsum = 0.0;
  if (tid < 91) {
    bsum = s_g[0][tid];
#pragma unroll
    for (int i = 1; i < kWinWaves; ++i) bsum += s_g[i][tid];
  }
  if (ce - cb > 1) {
    if (tid < 91) agent_store(a.partials + (size_t)ch * kWinLd + tid, bsum);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) s_t = __hip_atomic_fetch_add(a.pair_ticket + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    WSTAMP(2);
    if (s_t != ce - cb - 1) return;
    // the pair's last chunk sums the partials: wave w takes chunks cb + w, cb + w + W,
    // ... (in order) for entries lane and lane + 64, 2 x kFinBatch loads in flight per
    // lane; the W wave sums then meet in LDS in wave order (a fixed order: deterministic)
    {
      const int e1 = lane + kWave;
      const bool has1 = e1 < 91;
      double s0 = 0.0, s1 = 0.0;
      for (uint32_t c0 = cb + w; c0 < ce; c0 += kFinBatch * kWinWaves) {
        double x0[kFinBatch], x1[kFinBatch];
#pragma unroll
        for (int u = 0; u < kFinBatch; ++u) {
          const uint32_t cc = c0 + u * kWinWaves;
          const double* src = a.partials + (size_t)cc * kWinLd;
          x0[u] = cc < ce ? agent_load(src + lane) : 0.0;
          x1[u] = cc < ce && has1 ? agent_load(src + e1) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kFinBatch; ++u) {
          s0 += x0[u];
          s1 += x1[u];
        }
      }
      s_g[w][lane] = s0;
      if (has1) s_g[w][e1] = s1;
    }
    __syncthreads();
    if (tid < 91) {
      bsum = s_g[0][tid];
#pragma unroll
      for (int i = 1; i < kWinWaves; ++i) bsum += s_g[i][tid];
    }
    if (tid == 0) __hip_atomic_store(a.pair_ticket + slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  WSTAMP(3);
  // G of this pair straight to pinned host memory (write-through), error = 0.5 G[12][12]
  double* G = a.hostG + (size_t)slot * kWinG;
  if (tid < 91) host_store(G + tid, bsum);
  if (tid == 90) host_store(G + 91, 0.5 * bsum);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this pair's host stores are performed
  __syncthreads();
  WSTAMP(4);
  if (w != 0) return;
  // n_ne: the pairs with rows (the others have no chunk and never finish; the host
  // zeroes them)
  uint32_t t = 0;
  if (lane == 0) t = __hip_atomic_fetch_add(a.done_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = __shfl(t, 0, 64);
  WSTAMP(5);
  if (t != n_ne - 1) return;
  // Cross-wave / cross-block ordering (fmx_device.hpp, "several finishers"): every
  // wave of every pair finisher issued its G stores as system-scope write-through
  // stores and waited for their acknowledgement (vmcnt(0)) before the block barrier
  // that precedes its ticket; an acknowledged write-through store has left the GPU
  // caches, so all G stores are host-visible before the last ticket is taken and
  // this word is stored.  publish
  if (lane == 0) {
    __hip_atomic_store(a.done_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    publish_flag(a.flag, a.seq);
  }
  WSTAMP(6);
}

// ---------------------------------------------------------------- pair moments
// The ICP loop's LM relinearizes the current scan's pairs at every trial (fast mode,
// constraints.cpp:257-266) and the final LM every stored pair (:294-305).  Each row's
// whitened a = [H_i H_j -r] / sigma is LINEAR in 16 per-row features taken once at
// reference poses (T_i0, T_j0), with coefficients that depend only on the pair's poses:
//   plane rows (factor.cpp:37-77), q0 = R_i0^T (R_j0 p_j + t_j0 - t_i0) (p_j in frame i):
//     phi = [ r0 = n.(q0 - p_i), n x q0 (3), n (3), n_b p_j,d (9) ]
//     since H_i = [n x q, -n], H_j = [p_j x M^T n, M^T n], r = n.(q - p_i) with
//     q = M p_j + v, M = R_i^T R_j, v = R_i^T (t_j - t_i) = q0 + dM p_j + dv;
//   point rows (factor.cpp:87-124), e0 = (R_j0 p_j + t_j0) - (R_i0 p_i + t_i0):
//     phi = [ e0 (3), p_i (3), p_j (3), 1, 0 x 6 ] (the three axes share it).
// So a pair's DenseFactor::linearize (gtsam.hpp:67-86) at ANY poses is C Phi C^T with
// Phi = sum_rows phi phi^T (16 x 16) — contracted on the host (moments.cpp) without a
// device round trip.  The residual enters through r0 / e0 (taken per row), not as a
// difference of large moments, so the contraction keeps full precision.
// k_win_moments: the same launch geometry as k_win_linearize (one block per <= 256-row
// chunk of one pair, fp64 MFMA sums, per-pair ticket + ordered finisher); out: per pair
// Phi_plane then Phi_point, packed upper 16 x 16 (136 each), to pinned host memory.
constexpr int kMomF = 16;                // features per row
constexpr int kMomP = 136;               // packed upper 16 x 16
constexpr int kMomLd = 144;              // doubles per chunk partial (136 used)
constexpr int kMomStride = 17;           // doubles per staged row (odd: no LDS bank conflicts)

__device__ __forceinline__ void stage_and_mfma16(double* __restrict__ rows, const double (&f)[kMomF], bool valid,
                                                 f64x4 (&acc)[4]) {
  const int lane = lane_id();
  double* mine = rows + lane * kMomStride;
#pragma unroll
  for (int i = 0; i < kMomF; ++i) mine[i] = valid ? f[i] : 0.0;
  __builtin_amdgcn_wave_barrier();
  const double* src = rows + (lane >> 4) * kMomStride + (lane & 15);
  double v[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) v[t] = src[4 * t * kMomStride];
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(v[t], v[t], acc[t & 3], 0, 0, 0);
  __builtin_amdgcn_wave_barrier();
}

template <int NP>
__global__ __launch_bounds__(kWinWaves * kWave) void k_win_moments(WinArgs a, WinPosesN<NP> wp) {
  __shared__ double s_rows[kWinWaves][kWave * kMomStride];
  __shared__ double s_g[kWinWaves][2 * kMomP];
  __shared__ uint32_t s_t;
  const int w = threadIdx.x / kWave, lane = lane_id(), tid = threadIdx.x;
  const uint32_t ch = blockIdx.x;
  const uint32_t nch = a.n_chunks ? *a.n_chunks : a.n_chunks_host;
  Chunk d{};
  if (a.n_chunks || ch < a.n_chunks_host) d = a.chunks[ch];
  if (nch == 0) {
    if (blockIdx.x == 0 && tid == 0) publish_flag(a.flag, a.seq);
    return;
  }
  if (ch >= nch) return;
  const uint32_t type = d.type & 0xFFu;
  const int slot = (int)d.pair;
  const uint32_t cb = a.chunk_range[slot], ce = a.chunk_range[slot + 1];
  int pi, pj;
  if (a.implicit_j >= 0) {
    pi = slot;
    pj = a.implicit_j;
  } else if (a.implicit_j == kPairedPoses) {
    pi = 2 * slot;
    pj = 2 * slot + 1;
  } else {
    pi = (int)((d.type >> 8) & 0xFFFu);
    pj = (int)(d.type >> 20);
  }
  const double* Ti = a.dposes ? a.dposes + 12 * pi : wp.m[pi];
  const double* Tj = a.dposes ? a.dposes + 12 * pj : wp.m[pj];
  f64x4 accs[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) accs[i] = f64x4{0.0, 0.0, 0.0, 0.0};
  const uint32_t row = d.begin + w * kWave + lane;
  if (d.begin + w * kWave < d.end) {  // wave-uniform
    const bool valid = row < d.end;
    double f[kMomF];
#pragma unroll
    for (int i = 0; i < kMomF; ++i) f[i] = 0.0;
    if (valid) {
      if (type == 0) {
        double c[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) c[q] = a.c_pl[row + q * a.ld_pl];
        double wj[3], q0[3];
        d_xform(Tj, c[6], c[7], c[8], wj);
        d_rotT(Ti, wj[0] - Ti[3], wj[1] - Ti[7], wj[2] - Ti[11], q0);
        const double n0 = c[3], n1 = c[4], n2 = c[5];
        f[0] = (n0 * (q0[0] - c[0]) + n1 * (q0[1] - c[1])) + n2 * (q0[2] - c[2]);
        f[1] = n1 * q0[2] - n2 * q0[1];
        f[2] = n2 * q0[0] - n0 * q0[2];
        f[3] = n0 * q0[1] - n1 * q0[0];
        f[4] = n0;
        f[5] = n1;
        f[6] = n2;
#pragma unroll
        for (int b = 0; b < 3; ++b)
#pragma unroll
          for (int e = 0; e < 3; ++e) f[7 + 3 * b + e] = c[3 + b] * c[6 + e];
      } else {
        double c[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) c[q] = a.c_pt[row + q * a.ld_pt];
        double wi[3], wj[3];
        d_xform(Ti, c[0], c[1], c[2], wi);
        d_xform(Tj, c[3], c[4], c[5], wj);
        f[0] = wj[0] - wi[0];
        f[1] = wj[1] - wi[1];
        f[2] = wj[2] - wi[2];
#pragma unroll
        for (int q = 0; q < 6; ++q) f[3 + q] = c[q];
        f[9] = 1.0;
      }
    }
    stage_and_mfma16(s_rows[w], f, valid, accs);
  }
  // wave sums (packed upper 16 x 16) -> LDS; block sum in wave order
  const f64x4 acc = (accs[0] + accs[1]) + (accs[2] + accs[3]);
  {
    const int col = lane & 15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = (lane >> 4) + 4 * r;
      if (rr <= col) s_g[w][rr * 16 - rr * (rr - 1) / 2 + (col - rr)] = acc[r];
    }
  }
  __syncthreads();
  double bsum = 0.0;
  if (tid < kMomP) {
    bsum = s_g[0][tid];
#pragma unroll
    for (int i = 1; i < kWinWaves; ++i) bsum += s_g[i][tid];
  }
  // this pair's sums by type (entry tid < 136): plane rows, point pairs
  double out_pl = 0.0, out_pt = 0.0;
  if (ce - cb > 1) {
    if (tid < kMomP) agent_store(a.partials + (size_t)ch * kMomLd + tid, bsum);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) s_t = __hip_atomic_fetch_add(a.pair_ticket + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_t != ce - cb - 1) return;
    // the pair's last chunk sums the partials by type, in chunk order: wave w takes
    // chunks cb + w, cb + w + W, ...; lane holds entries lane, lane + 64, lane + 128
    // (< 136) of each type; the wave sums meet in LDS in wave order
    {
      double sp[3] = {0.0, 0.0, 0.0}, st[3] = {0.0, 0.0, 0.0};
      for (uint32_t c0 = cb + w; c0 < ce; c0 += kFinBatch * kWinWaves) {
        double x[kFinBatch][3];
        uint32_t ty[kFinBatch];
#pragma unroll
        for (int u = 0; u < kFinBatch; ++u) {
          const uint32_t cc = c0 + u * kWinWaves;
          const double* src = a.partials + (size_t)cc * kMomLd;
          ty[u] = cc < ce ? (a.chunks[cc].type & 0xFFu) : 2u;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const int e = lane + 64 * k;
            x[u][k] = cc < ce && e < kMomP ? agent_load(src + e) : 0.0;
          }
        }
#pragma unroll
        for (int u = 0; u < kFinBatch; ++u)
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            sp[k] += ty[u] == 0u ? x[u][k] : 0.0;
            st[k] += ty[u] == 1u ? x[u][k] : 0.0;
          }
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int e = lane + 64 * k;
        if (e < kMomP) {
          s_g[w][e] = sp[k];
          s_g[w][kMomP + e] = st[k];
        }
      }
    }
    __syncthreads();
    if (tid < kMomP) {
      out_pl = s_g[0][tid];
      out_pt = s_g[0][kMomP + tid];
#pragma unroll
      for (int i = 1; i < kWinWaves; ++i) {
        out_pl += s_g[i][tid];
        out_pt += s_g[i][kMomP + tid];
      }
    }
    if (tid == 0) __hip_atomic_store(a.pair_ticket + slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    out_pl = type == 0 ? bsum : 0.0;
    out_pt = type == 1 ? bsum : 0.0;
  }
  // this pair's Phi (both types) straight to pinned host memory (write-through)
  double* G = a.hostG + (size_t)slot * (2 * kMomP);
  if (tid < kMomP) {
    host_store(G + tid, out_pl);
    host_store(G + kMomP + tid, out_pt);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (w != 0) return;
  uint32_t n_ne = 0;
  for (int k0 = 0; k0 < a.npairs; k0 += kWave) {
    const int k = k0 + lane;
    const bool ne = k < a.npairs && a.chunk_range[k + 1] > a.chunk_range[k];
    n_ne += (uint32_t)__popcll(__ballot(ne));
  }
  uint32_t t = 0;
  if (lane == 0) t = __hip_atomic_fetch_add(a.done_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = __shfl(t, 0, 64);
  if (t != n_ne - 1) return;
  if (lane == 0) {  // every finisher's host stores were acknowledged before its ticket (as k_win_linearize)
    __hip_atomic_store(a.done_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    publish_flag(a.flag, a.seq);
  }
}

// Copy n_pl plane rows (9 comps) and n_pt point pairs (6 comps) between SoA buffers.
__global__ void k_rows_copy(const double* __restrict__ spl, size_t lds_pl, uint64_t so_pl, double* __restrict__ dpl,
                            size_t ldd_pl, uint64_t do_pl, uint32_t n_pl, const double* __restrict__ spt, size_t lds_pt,
                            uint64_t so_pt, double* __restrict__ dpt, size_t ldd_pt, uint64_t do_pt, uint32_t n_pt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t npl = (uint64_t)n_pl * 9, npt = (uint64_t)n_pt * 6;
  if (i < npl) {
    const uint32_t comp = (uint32_t)(i / n_pl), r = (uint32_t)(i % n_pl);
    dpl[comp * ldd_pl + do_pl + r] = spl[comp * lds_pl + so_pl + r];
  } else if (i < npl + npt) {
    const uint64_t k = i - npl;
    const uint32_t comp = (uint32_t)(k / n_pt), r = (uint32_t)(k % n_pt);
    dpt[comp * ldd_pt + do_pt + r] = spt[comp * lds_pt + so_pt + r];
  }
}

void rows_copy(hipStream_t st, const double* spl, size_t lds_pl, uint64_t so_pl, double* dpl, size_t ldd_pl,
               uint64_t do_pl, uint32_t n_pl, const double* spt, size_t lds_pt, uint64_t so_pt, double* dpt,
               size_t ldd_pt, uint64_t do_pt, uint32_t n_pt) {
  const uint64_t n = (uint64_t)n_pl * 9 + (uint64_t)n_pt * 6;
  if (n == 0) return;
  const uint32_t nb = (uint32_t)((n + 255) / 256);
  hipLaunchKernelGGL(k_rows_copy, dim3(nb), dim3(256), 0, st, spl, lds_pl, so_pl, dpl, ldd_pl, do_pl, n_pl, spt,
                     lds_pt, so_pt, dpt, ldd_pt, do_pt, n_pt);
  FMX_HIP(hipGetLastError());
}

// FMX_WIN_TIMING diagnostics: per launch, the spread of the waves' stamps relative to
// the first wave start (us, 100 MHz s_memrealtime), averaged over launches at exit.
struct WinTiming {
  double sum[8] = {0}, n = 0, span = 0;
  ~WinTiming() {
    if (n == 0) return;
    static const char* nm[8] = {"start(max)", "computed", "ticket", "fin_loaded", "fin_stored", "done_ticket",
                                "published", "chunk_read"};
    fprintf(stderr, "k_win_linearize timing over %.0f launches (us after the first wave start, max over waves):\n", n);
    for (int i = 0; i < 8; ++i) fprintf(stderr, "  %-12s %8.2f\n", nm[i], sum[i] / n);
    fprintf(stderr, "  span         %8.2f\n", span / n);
  }
};
static WinTiming& win_timing() {
  static WinTiming t;
  return t;
}
bool win_timing_on() {
  static const bool on = std::getenv("FMX_WIN_TIMING") != nullptr;
  return on;
}
void win_timing_collect(fmx_ctx* c, uint32_t grid_chunks) {
  WinStore& W = c->win;
  FMX_HIP(hipStreamSynchronize(c->stream));
  std::vector<uint64_t> h((size_t)grid_chunks * 8);
  FMX_HIP(hipMemcpy(h.data(), W.dbg.p, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  uint64_t t0 = ~0ull, mx[8] = {0};
  for (uint32_t ch = 0; ch < grid_chunks; ++ch)
    if (h[ch * 8]) t0 = std::min(t0, h[ch * 8]);
  if (t0 == ~0ull) return;
  for (uint32_t ch = 0; ch < grid_chunks; ++ch)
    for (int i = 0; i < 8; ++i)
      if (h[ch * 8 + i]) mx[i] = std::max(mx[i], h[ch * 8 + i] - t0);
  WinTiming& T = win_timing();
  for (int i = 0; i < 8; ++i) T.sum[i] += mx[i] * 0.01;
  T.span += *std::max_element(mx, mx + 7) * 0.01;
  T.n += 1;
  FMX_HIP(hipMemset(W.dbg.p, 0, h.size() * sizeof(uint64_t)));
}

// Launch k_win_linearize (win_start); wait for its word and copy npairs x 92 doubles
// out (win_finish).  The host assembles the x-dependent non-pair terms in between.
// out_dev (sharded fmx_linearize): G to this device buffer instead, the completion word
// to a device scratch word; the caller all-reduces and copies (no win_finish).
// mom: k_win_moments instead (per pair 2 x 136 doubles of moments, to W.hM)
void win_start(fmx_ctx* c, WinArgs a, uint32_t grid_chunks, const double* poses, int nposes, double bytes,
               double* out_dev = nullptr, bool mom = false, hipStream_t st_launch = nullptr) {
  WinStore& W = c->win;
  if (W.pending) win_finish(c, nullptr);  // an abandoned one (error path): drain it first
  hipStream_t st = st_launch ? st_launch : c->stream;
  WinPoses wp;
  WinPosesN<kWinSmallArgPoses> wps;
  if (nposes <= kWinSmallArgPoses) {
    std::memcpy(wps.m, poses, (size_t)nposes * 12 * sizeof(double));
    a.dposes = nullptr;
  } else if (nposes <= kWinMaxArgPoses) {
    std::memcpy(wp.m, poses, (size_t)nposes * 12 * sizeof(double));
    a.dposes = nullptr;
  } else {
    W.hposes.ensure(12 * (size_t)nposes);
    std::memcpy(W.hposes.p, poses, (size_t)nposes * 12 * sizeof(double));
    W.dposes.ensure(12 * (size_t)nposes);
    FMX_HIP(hipMemcpyAsync(W.dposes.p, W.hposes.p, (size_t)nposes * 12 * sizeof(double), hipMemcpyHostToDevice, st));
    a.dposes = W.dposes.p;
  }
  const int np = std::max(a.npairs, 1);
  W.partials.ensure((size_t)std::max<uint32_t>(grid_chunks, 1) * (mom ? kMomLd : kWinLd));
  ensure_zeroed(W.pticket, (size_t)np, st);
  ensure_zeroed(W.dticket, 1, st);
  W.hG.ensure((size_t)np * kWinG);
  if (mom) W.hM.ensure((size_t)np * 2 * kMomP);
  a.partials = W.partials.p;
  a.pair_ticket = W.pticket.p;
  a.done_ticket = W.dticket.p;
  a.hostG = mom ? W.hM.d : W.hG.d;
  a.seq = next_flag(c);
  a.flag = c->h_flag.d;
  if (out_dev) {
    W.dflag.ensure(1);
    a.hostG = out_dev;
    a.flag = W.dflag.p;
  }
  a.dbg = nullptr;
  if (win_timing_on()) {
    if (W.dbg.cap < (size_t)grid_chunks * 8) {
      W.dbg.ensure((size_t)grid_chunks * 8);
      FMX_HIP(hipMemset(W.dbg.p, 0, W.dbg.cap * sizeof(uint64_t)));
    }
    a.dbg = W.dbg.p;
  }
  const uint32_t blocks = std::max<uint32_t>(grid_chunks, 1);
  {
    HostScope hs(12);
    ProfScope ps(c->prof, mom ? PROF_MOMENTS : PROF_WINDOW, bytes, st);
    if (mom) {
      if (nposes <= kWinSmallArgPoses)
        hipLaunchKernelGGL(k_win_moments<kWinSmallArgPoses>, dim3(blocks), dim3(kWinWaves * kWave), 0, st, a, wps);
      else
        hipLaunchKernelGGL(k_win_moments<kWinMaxArgPoses>, dim3(blocks), dim3(kWinWaves * kWave), 0, st, a, wp);
    } else if (nposes <= kWinSmallArgPoses) {
      hipLaunchKernelGGL(k_win_linearize<kWinSmallArgPoses>, dim3(blocks), dim3(kWinWaves * kWave), 0, st, a, wps);
    } else {
      hipLaunchKernelGGL(k_win_linearize<kWinMaxArgPoses>, dim3(blocks), dim3(kWinWaves * kWave), 0, st, a, wp);
    }
    FMX_HIP(hipGetLastError());
  }
  W.pending = out_dev == nullptr;
  W.pending_st = st;
  W.pending_seq = a.seq;
  W.pending_np = a.npairs;
  W.pending_mom = mom;
  W.pending_grid = grid_chunks;
}

}  // namespace

void win_finish(fmx_ctx* c, double* G_out) {
  WinStore& W = c->win;
  if (!W.pending) throw StatusError(FMX_E_STATE, "win_finish: no window linearization in flight");
  W.pending = false;
  {
    HostScope hs(13);
    wait_flag(c, c->h_flag.p, W.pending_seq, W.pending_st);
  }
  if (G_out) {
    if (W.pending_mom) std::memcpy(G_out, W.hM.p, (size_t)W.pending_np * 2 * kMomP * sizeof(double));
    else std::memcpy(G_out, W.hG.p, (size_t)W.pending_np * kWinG * sizeof(double));
  }
  if (win_timing_on() && !W.pending_mom) win_timing_collect(c, W.pending_grid);
}

namespace {
}  // namespace

// ---------------------------------------------------------------- store maintenance
// Append the current scan's sorted correspondences (the last fmx match, sorted mode,
// counts fetched) as segment j: pairs (map_scans[k], j) with rows, i ascending.
void win_persist(fmx_ctx* c, uint64_t j) {
  WinStore& W = c->win;
  hipStream_t st = c->stream;
  if (!c->have_corr) throw StatusError(FMX_E_STATE, "win_persist: no sorted match");
  run_pair_scatter(c);
  uint64_t npl = 0, npt = 0;
  for (uint32_t k = 0; k < c->K; ++k) {
    npl += c->cnt_pl[k];
    npt += c->cnt_pt[k];
  }
  win_reserve(c, npl, npt);
  WinSeg s;
  s.pl_off = W.tail_pl;
  s.pt_off = W.tail_pt;
  s.pl_n = (uint32_t)npl;
  s.pt_n = (uint32_t)npt;
  uint64_t op = 0, ot = 0;
  for (uint32_t k = 0; k < c->K; ++k) {
    if (c->cnt_pl[k] + c->cnt_pt[k] > 0)
      s.pairs.push_back(WinPair{c->map_scans[k], j, s.pl_off + op, s.pt_off + ot, c->cnt_pl[k], c->cnt_pt[k]});
    op += c->cnt_pl[k];
    ot += c->cnt_pt[k];
  }
  rows_copy(st, c->c_pl.p, c->ld_pl, 0, W.pl[W.cur].p, W.cap_pl, s.pl_off, (uint32_t)npl, c->c_pt.p, c->ld_pt, 0,
            W.pt[W.cur].p, W.cap_pt, s.pt_off, (uint32_t)npt);
  W.tail_pl += npl;
  W.tail_pt += npt;
  W.segs[j] = std::move(s);
}

// Room for (npl, npt) more rows at the tail: compact the live segments into the other
// arena (growing both when the live rows fill more than half of it).
void win_reserve(fmx_ctx* c, uint64_t npl, uint64_t npt) {
  WinStore& W = c->win;
  hipStream_t st = c->stream;
  if (W.cap_pl == 0) {
    W.cap_pl = std::max<uint64_t>(c->P.keypoint_pool_capacity, 1u << 20);
    W.cap_pt = std::max<uint64_t>(W.cap_pl / 4, 1u << 18);
    for (int b = 0; b < 2; ++b) {
      W.pl[b].ensure(9 * W.cap_pl);
      W.pt[b].ensure(6 * W.cap_pt);
    }
    W.cap_pl = W.pl[0].cap / 9;  // DBuf over-allocates: use it
    W.cap_pt = W.pt[0].cap / 6;
  }
  if (W.tail_pl + npl <= W.cap_pl && W.tail_pt + npt <= W.cap_pt) return;
  uint64_t live_pl = npl, live_pt = npt;
  for (auto& [j, s] : W.segs) {
    live_pl += s.pl_n;
    live_pt += s.pt_n;
  }
  const int nxt = 1 - W.cur;
  uint64_t cap_pl = W.cap_pl, cap_pt = W.cap_pt;
  while (2 * live_pl > cap_pl) cap_pl *= 2;
  while (2 * live_pt > cap_pt) cap_pt *= 2;
  if (cap_pl != W.cap_pl || cap_pt != W.cap_pt) {  // grow: both arenas (contents move below)
    W.pl[nxt].ensure(9 * cap_pl);
    W.pt[nxt].ensure(6 * cap_pt);
  }
  const uint64_t ncap_pl = cap_pl != W.cap_pl ? W.pl[nxt].cap / 9 : W.cap_pl;
  const uint64_t ncap_pt = cap_pt != W.cap_pt ? W.pt[nxt].cap / 6 : W.cap_pt;
  uint64_t tpl = 0, tpt = 0;
  for (auto& [j, s] : W.segs) {
    rows_copy(st, W.pl[W.cur].p, W.cap_pl, s.pl_off, W.pl[nxt].p, ncap_pl, tpl, s.pl_n, W.pt[W.cur].p, W.cap_pt,
              s.pt_off, W.pt[nxt].p, ncap_pt, tpt, s.pt_n);
    for (auto& p : s.pairs) {
      p.pl_off = p.pl_off - s.pl_off + tpl;
      p.pt_off = p.pt_off - s.pt_off + tpt;
    }
    s.pl_off = tpl;
    s.pt_off = tpt;
    tpl += s.pl_n;
    tpt += s.pt_n;
  }
  W.cur = nxt;
  W.tail_pl = tpl;
  W.tail_pt = tpt;
  if (ncap_pl != W.cap_pl || ncap_pt != W.cap_pt) {  // the old arena grows too (free space only)
    W.pl[1 - nxt].ensure(9 * ncap_pl);
    W.pt[1 - nxt].ensure(6 * ncap_pt);
  }
  W.cap_pl = ncap_pl;
  W.cap_pt = ncap_pt;
  W.chunks_valid = false;
}

// KeypointMap / ConstraintManager erase of scan s (constraints.cpp:195-203): its
// segment and every pair (s, j) of the other segments.  Rows stay until compaction.
void win_remove(fmx_ctx* c, uint64_t s) {
  WinStore& W = c->win;
  W.segs.erase(s);
  for (auto& [j, seg] : W.segs)
    seg.pairs.erase(std::remove_if(seg.pairs.begin(), seg.pairs.end(), [&](const WinPair& p) { return p.i == s; }),
                    seg.pairs.end());
  W.chunks_valid = false;
}

// Every stored pair (j ascending, i ascending): the full-mode factor list.
std::vector<WinPair> win_pairs(fmx_ctx* c) {
  std::vector<WinPair> out;
  for (auto& [j, s] : c->win.segs)
    for (auto& p : s.pairs) out.push_back(p);
  return out;
}

// Chunk table for the stored pairs `prs` (slots = list order) with pose slots into
// `keys`; uploaded once per pair set (the LM's linearizations reuse it).
void win_set_pairs(fmx_ctx* c, const std::vector<WinPair>& prs, const std::vector<uint64_t>& keys) {
  WinStore& W = c->win;
  hipStream_t st = c->stream;
  std::map<uint64_t, uint32_t> slot;
  for (size_t k = 0; k < keys.size(); ++k) slot[keys[k]] = (uint32_t)k;
  if (keys.size() > 0xFFF) throw StatusError(FMX_E_INVAL, "window larger than 4095 poses");
  if (W.tail_pl > 0xFFFFFFFFull || W.tail_pt > 0xFFFFFFFFull)
    throw StatusError(FMX_E_OOM, "window store exceeds 2^32 rows");
  std::vector<Chunk> ch;
  std::vector<uint32_t> cr(prs.size() + 1);
  uint64_t rows_pl = 0, rows_pt = 0;
  for (size_t k = 0; k < prs.size(); ++k) {
    const WinPair& p = prs[k];
    cr[k] = (uint32_t)ch.size();
    const uint32_t tag = (slot.at(p.i) << 8) | (slot.at(p.j) << 20);
    for (uint32_t r = 0; r < p.pl_n; r += kPlaneChunk)
      ch.push_back(Chunk{0u | tag, (uint32_t)k, (uint32_t)(p.pl_off + r),
                         (uint32_t)(p.pl_off + std::min<uint32_t>(p.pl_n, r + kPlaneChunk))});
    for (uint32_t r = 0; r < p.pt_n; r += kPointChunk)
      ch.push_back(Chunk{1u | tag, (uint32_t)k, (uint32_t)(p.pt_off + r),
                         (uint32_t)(p.pt_off + std::min<uint32_t>(p.pt_n, r + kPointChunk))});
    rows_pl += p.pl_n;
    rows_pt += p.pt_n;
  }
  cr[prs.size()] = (uint32_t)ch.size();
  const size_t nch = ch.size();
  // one upload: [chunks (4 words each)][chunk_range]; the pinned staging buffer is
  // reused only after the previous upload's event (no stream synchronization)
  const size_t words = 4 * nch + cr.size();
  if (W.meta_ev_pending) FMX_HIP(hipEventSynchronize(W.meta_ev));
  W.meta.ensure(words + 4);
  W.hmeta.ensure(words + 4);
  std::memcpy(W.hmeta.p, ch.data(), nch * sizeof(Chunk));
  std::memcpy(W.hmeta.p + 4 * nch, cr.data(), cr.size() * sizeof(uint32_t));
  FMX_HIP(hipMemcpyAsync(W.meta.p, W.hmeta.p, words * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  if (!W.meta_ev) FMX_HIP(hipEventCreateWithFlags(&W.meta_ev, hipEventDisableTiming));
  FMX_HIP(hipEventRecord(W.meta_ev, st));
  W.meta_ev_pending = true;
  W.chunks_p = reinterpret_cast<const Chunk*>(W.meta.p);
  W.chunk_range_p = W.meta.p + 4 * nch;
  W.nch = (uint32_t)nch;
  W.npairs = (int)prs.size();
  W.rows_pl = rows_pl;
  W.rows_pt = rows_pt;
  W.chunks_valid = true;
}

// DenseFactor::linearize of every pair of the last win_set_pairs at poses[key slot]:
// G_out[npairs][92] = 91 packed-upper 13 x 13 entries + error.  G_out null: launch
// only; win_finish(c, G_out) waits and copies.
void win_linearize_stored(fmx_ctx* c, const double* poses, int nposes, double sigma, double* G_out) {
  WinStore& W = c->win;
  if (!W.chunks_valid) throw StatusError(FMX_E_STATE, "win_linearize_stored: pair set not uploaded");
  WinArgs a{};
  a.chunks = W.chunks_p;
  a.n_chunks = nullptr;
  a.n_chunks_host = W.nch;
  a.chunk_range = W.chunk_range_p;
  a.npairs = W.npairs;
  a.c_pl = W.pl[W.cur].p;
  a.ld_pl = W.cap_pl;
  a.c_pt = W.pt[W.cur].p;
  a.ld_pt = W.cap_pt;
  a.implicit_j = -1;
  a.inv = 1.0 / sigma;
  win_start(c, a, W.nch, poses, nposes, 72.0 * W.rows_pl + 48.0 * W.rows_pt + 8.0 * kWinG * W.npairs);
  if (G_out) win_finish(c, G_out);
}

// Same for the current scan's K pairs straight from the sorted match (device-built
// chunk table): poses[k] = pose of map_scans[k], poses[K] = the current pose.
// st (null: the context stream): another stream, for a launch whose inputs the host has
// already seen complete (the LM's trial linearizations, whose rows the LM's first
// linearization on the context stream read before them).
void win_linearize_current(fmx_ctx* c, const double* poses, double sigma, double* G_out, hipStream_t st) {
  if (!c->have_corr) throw StatusError(FMX_E_STATE, "win_linearize_current: no sorted match");
  if (c->scatter_pending) st = nullptr;  // its rows are still to be written on the context stream
  run_pair_scatter(c);
  WinArgs a{};
  a.chunks = c->chunks.p;
  a.n_chunks = c->n_chunks.p;
  a.chunk_range = c->chunk_range.p;
  a.npairs = (int)c->K;
  a.c_pl = c->c_pl.p;
  a.ld_pl = c->ld_pl;
  a.c_pt = c->c_pt.p;
  a.ld_pt = c->ld_pt;
  a.implicit_j = (int)c->K;
  a.inv = 1.0 / sigma;
  // exact row counts arrive with the match counts; the byte model uses the last known
  win_start(c, a, c->max_chunks, poses, (int)c->K + 1, 72.0 * c->rows_pl + 48.0 * c->rows_pt + 8.0 * kWinG * c->K,
            nullptr, false, st);
  if (G_out) win_finish(c, G_out);
}

// The moments (k_win_moments) of the current scan's K pairs from the sorted match at the
// reference poses poses[k] (pose of map_scans[k]) and poses[K] (the current pose): out
// (null: launch only, win_finish(c, out) later) = K x 272 doubles, per pair the packed
// upper 16 x 16 plane moments then the point moments.
void win_moments_current(fmx_ctx* c, const double* poses, double* out) {
  if (!c->have_corr) throw StatusError(FMX_E_STATE, "win_moments_current: no sorted match");
  run_pair_scatter(c);
  WinArgs a{};
  a.chunks = c->chunks.p;
  a.n_chunks = c->n_chunks.p;
  a.chunk_range = c->chunk_range.p;
  a.npairs = (int)c->K;
  a.c_pl = c->c_pl.p;
  a.ld_pl = c->ld_pl;
  a.c_pt = c->c_pt.p;
  a.ld_pt = c->ld_pt;
  a.implicit_j = (int)c->K;
  a.inv = 1.0;
  // bytes: rows read (72 B per plane row, 48 B per point pair) + 2 x 136 doubles per pair
  win_start(c, a, c->max_chunks, poses, (int)c->K + 1, 72.0 * c->rows_pl + 48.0 * c->rows_pt + 8.0 * 2 * kMomP * c->K,
            nullptr, true);
  if (out) win_finish(c, out);
}

// fmx_moments: the same for the context's correspondences (fmx_match / fmx_corr_set),
// pair k at the reference poses poses_i[k], poses_j[k] (the GTSAM seam's "linearize once,
// evaluate anywhere" form; fmx_moments_contract).  out: K x 272.
void win_moments_pairs(fmx_ctx* c, const double* poses_i, const double* poses_j, double* out) {
  if (!c->have_corr) throw StatusError(FMX_E_STATE, "no correspondences (call fmx_match or fmx_corr_set)");
  run_pair_scatter(c);
  const int K = (int)c->K;
  if (K == 0) return;
  if (c->comm) throw StatusError(FMX_E_STATE, "fmx_moments is not sharded (no communicator)");
  if (2 * (size_t)K > 0xFFFFFFu) throw StatusError(FMX_E_INVAL, "too many pairs");
  WinStore& W = c->win;
  if (W.pending) win_finish(c, nullptr);
  std::vector<double> table(24 * (size_t)K);
  for (int k = 0; k < K; ++k) {
    std::memcpy(&table[24 * (size_t)k], poses_i + 12 * (size_t)k, 12 * sizeof(double));
    std::memcpy(&table[24 * (size_t)k + 12], poses_j + 12 * (size_t)k, 12 * sizeof(double));
  }
  if (c->counts_pending) match_counts_fetch(c);
  W.hM.ensure((size_t)K * 2 * kMomP);
  std::memset(W.hM.p, 0, (size_t)K * 2 * kMomP * sizeof(double));  // pairs without rows are never written
  WinArgs a{};
  a.chunks = c->chunks.p;
  a.n_chunks = c->n_chunks.p;
  a.chunk_range = c->chunk_range.p;
  a.npairs = K;
  a.c_pl = c->c_pl.p;
  a.ld_pl = c->ld_pl;
  a.c_pt = c->c_pt.p;
  a.ld_pt = c->ld_pt;
  a.implicit_j = kPairedPoses;
  a.inv = 1.0;
  win_start(c, a, c->max_chunks, table.data(), 2 * K, 72.0 * c->rows_pl + 48.0 * c->rows_pt + 8.0 * 2 * kMomP * K,
            nullptr, true);
  win_finish(c, out);
}

// fmx_linearize / fmx_error — the GTSAM seam, DenseFactor::linearize of every pair's
// FeatureFactor (gtsam.hpp:67-86) — on the SAME kernel as register_scan's window
// linearizations: the correspondences of the last sorted match (or fmx_corr_set),
// pair k between poses_i[k] and poses_j[k] (a 2K-entry pose table).  mode 0: G = the
// 13 x 13 augmented information (91); mode 1: the single-pose 7 x 7 (28) =
// [H_j b]^T [H_j b], the trailing 7 x 7 block of the 13 x 13 (BinaryFactorWrapper,
// gtsam.hpp:144-170); mode 2: errors only.  err[k] = 0.5 ||r/sigma||^2.  Pairs
// without rows linearize to zero.
void win_linearize_pairs(fmx_ctx* c, const double* poses_i, const double* poses_j, double sigma, int mode,
                         double* G_out, double* err_out) {
  if (!c->have_corr) throw StatusError(FMX_E_STATE, "no correspondences (call fmx_match or fmx_corr_set)");
  comm_check(c);
  run_pair_scatter(c);  // fmx_match deferred it
  const int K = (int)c->K;
  if (K == 0) return;
  if (2 * (size_t)K > 0xFFFFFFu) throw StatusError(FMX_E_INVAL, "too many pairs");
  WinStore& W = c->win;
  if (W.pending) win_finish(c, nullptr);
  std::vector<double> table(24 * (size_t)K);
  for (int k = 0; k < K; ++k) {
    std::memcpy(&table[24 * (size_t)k], poses_i + 12 * (size_t)k, 12 * sizeof(double));
    std::memcpy(&table[24 * (size_t)k + 12], poses_j + 12 * (size_t)k, 12 * sizeof(double));
  }
  if (c->counts_pending) match_counts_fetch(c);  // exact byte model (rows per type)
  W.hG.ensure((size_t)K * kWinG);
  // pairs without rows are never written: zero them first (sharded: in the device
  // buffer the ranks all-reduce, on the stream ahead of the kernel)
  const bool comm = c->comm != nullptr;
  if (comm) {
    c->d_sum.ensure((size_t)K * kWinG);
    FMX_HIP(hipMemsetAsync(c->d_sum.p, 0, (size_t)K * kWinG * sizeof(double), c->stream));
  } else {
    std::memset(W.hG.p, 0, (size_t)K * kWinG * sizeof(double));
  }
  WinArgs a{};
  a.chunks = c->chunks.p;
  a.n_chunks = c->n_chunks.p;
  a.chunk_range = c->chunk_range.p;
  a.npairs = K;
  a.c_pl = c->c_pl.p;
  a.ld_pl = c->ld_pl;
  a.c_pt = c->c_pt.p;
  a.ld_pt = c->ld_pt;
  a.implicit_j = kPairedPoses;
  a.inv = 1.0 / sigma;  // FastIsotropic invsigma_ (gtsam.hpp:96)
  win_start(c, a, c->max_chunks, table.data(), 2 * K, 72.0 * c->rows_pl + 48.0 * c->rows_pt + 8.0 * kWinG * K,
            comm ? c->d_sum.p : nullptr);
  if (comm) {  // every pair's G (and error) summed over the ranks on this stream
    comm_allreduce_publish(c, c->d_sum.p, (size_t)K * kWinG, W.hG);
  } else {
    win_finish(c, nullptr);
  }
  const double* hg = W.hG.p;
  for (int k = 0; k < K; ++k) {
    const double* g = hg + (size_t)k * kWinG;
    if (err_out) err_out[k] = g[91];
    if (!G_out || mode == 2) continue;
    if (mode == 0) {
      std::memcpy(G_out + (size_t)k * 91, g, 91 * sizeof(double));
    } else {  // rows / columns 6..12 of the packed upper 13 x 13
      double* o = G_out + (size_t)k * 28;
      int q = 0;
      for (int r = 6; r < 13; ++r)
        for (int cc = r; cc < 13; ++cc) o[q++] = g[r * 13 - r * (r - 1) / 2 + (cc - r)];
    }
  }
}

}  // namespace fmx
