// linearize.hip — stage 3 for the single-pose ablation, and the correspondence upload.
//
// Replaces, per correspondence (map scan i, current scan j):
//   PlanePoint::evaluateError  (form/feature/factor.cpp:30-80)
//   PointPoint::evaluateError  (form/feature/factor.cpp:82-128)
//   FeatureFactor stacking     (form/feature/factor.cpp:142-186)
//   DenseFactor::linearize + FastIsotropic::WhitenSystem (form/optimization/
//     gtsam.hpp:67-86, 129-139) wrapped by BinaryFactorWrapper (gtsam.hpp:144-170):
//     [H_j b]^T [H_j b] (7 x 7, 28 unique doubles) with b = -r / sigma.
//
// k_linearize_total: register_scan's linearization in the disable_smoothing mode —
// get_single_graph (constraints.cpp:235-250) is the sum of every pair's FeatureFactor
// at X(j) with X(i) fixed, so the 7 x 7 system is summed over ALL accepted matches in
// query order straight from the match outputs (no pair sort) in one launch.  The
// 13 x 13 per-pair information (the GTSAM seam, fmx_linearize, and the smoothing mode)
// is window.hip's k_win_linearize.  HBM-bound: 80 B per plane row, 48 B per point pair.
#include "fmx_device.hpp"
#include "fmx_internal.hpp"

#include <algorithm>
#include <cstring>

namespace fmx {
namespace {

#include "factor_rows.hpp"

// register_scan's single-pose linearization: the sum over ALL pairs of
// [H_j b]^T [H_j b] (28 doubles) and the error, in one launch.  16 waves per block,
// one 64-row chunk each.  Each wave reduce-scatters its 28 (+4 pad) sums across the
// lanes (5 halving steps + 1: 32 shuffles instead of 28 butterflies), the block adds
// its waves in order, the block partial goes out with agent-scope stores, each block
// takes an agent-scope ticket, and the last block sums the block partials in a fixed
// order (MI355X_MICROARCH.md, inter-workgroup hand-off) and writes G + error to mapped
// host memory behind the completion word.
constexpr int kTotWaves = 16;
constexpr int kTotLd = 32;  // doubles per block partial (28 used)

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

__global__ __launch_bounds__(kTotWaves * kWave) void k_linearize_total(
    QoRows qo, const double* __restrict__ poses, double inv, double* __restrict__ bpart, uint32_t* __restrict__ ticket,
    double* __restrict__ out, Pose34 tjv, uint32_t* __restrict__ flag, uint32_t seq, uint32_t cpw) {
  constexpr int NG = 28;
  constexpr int kTotGroups = kTotWaves * kWave / NG;  // final reduction: lane groups x 28 entries
  const int w = threadIdx.x / kWave, lane = lane_id();
  double acc[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) acc[i] = 0.0;
  // cpw consecutive 64-row chunks per wave (large query sets: one reduce-scatter per
  // cpw chunks instead of per chunk)
  for (uint32_t c = 0; c < cpw; ++c) {
  const uint32_t ch = (blockIdx.x * kTotWaves + w) * cpw + c;
  const uint32_t gq = ch * kWave + lane;
  const int32_t pair = gq < qo.nq ? qo.pair[gq] : -1;
  if (pair >= 0) {
    const double* Ti = poses + 12 * pair;
    const double* Tj = tjv.m;
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
  }  // chunks
  __shared__ double sw[kTotWaves][NG];
  __shared__ double sq[kTotGroups][NG];
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
    host_store(out + e, s);
    if (e == NG - 1) host_store(out + NG, 0.5 * s);
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (flag) publish_flag(flag, seq);  // out[] was stored by this wave (threads 0..28 of wave 0)
  }
}

}  // namespace

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
  // chunk table (pair-major), the layout the sorted match's last block writes
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
  c->scatter_pending = false;
  c->have_match = false;
}

}  // namespace fmx

namespace fmx {

// blocks of k_linearize_total over the last query-order match (64 queries per wave)
// (+ the partial / ticket buffers it needs; the ticket starts at 0 and the last block
// resets it)
constexpr uint32_t kTotTargetWaves = 8192;  // waves enough to fill the chip; beyond, chunks per wave grow
static uint32_t tot_chunks_per_wave(fmx_ctx* c) {
  const uint32_t nch = (c->n_qo + kWave - 1) / kWave;
  return std::max<uint32_t>((nch + kTotTargetWaves - 1) / kTotTargetWaves, 1);
}
static uint32_t tot_blocks(fmx_ctx* c) {
  const uint32_t nch = (c->n_qo + kWave - 1) / kWave, cpw = tot_chunks_per_wave(c);
  const uint32_t nblk = std::max<uint32_t>((nch + kTotWaves * cpw - 1) / (kTotWaves * cpw), 1);
  c->bpart.ensure((size_t)nblk * kTotLd);
  ensure_zeroed(c->ticket, 1, c->stream);
  return nblk;
}
static QoRows qo_rows(fmx_ctx* c) {
  return QoRows{c->m_pair.p, reinterpret_cast<const double4*>(c->m_pi.p), reinterpret_cast<const double4*>(c->m_ni.p),
                c->q_pl_pos.p, c->q_pt_pos.p, c->n_qpl, c->n_qo};
}

// register_scan's single-pose linearization: out[0..27] = sum over pairs of the packed
// 7 x 7 [H_j b]^T [H_j b] at pose_j, out[28] = error.  One launch, one wait.
void run_linearize_total(fmx_ctx* c, const double* pose_j34, double sigma, double* out) {
  if (!c->have_map) throw StatusError(FMX_E_STATE, "no map");
  if (!c->have_qo) throw StatusError(FMX_E_STATE, "no query-order match");
  comm_check(c);
  hipStream_t st = c->stream;
  for (int i = 0; i < 29; ++i) out[i] = 0.0;
  if ((c->K == 0 || c->n_qo == 0) && !c->comm) return;  // sharded: every rank joins the collective
  const uint32_t nblk = tot_blocks(c);
  Pose34 tjv;
  std::memcpy(tjv.m, pose_j34, sizeof(tjv.m));
  c->h_G.ensure(32);
  // sharded (fmx_comm_init): the sums go to a device buffer, are all-reduced there on
  // this stream and copied out; else straight to mapped host memory behind the word
  const bool comm = c->comm != nullptr;
  if (comm) c->d_sum.ensure(32);
  const uint32_t seq = next_flag(c);  // allocates the word on first use
  double* dst = comm ? c->d_sum.p : c->h_G.d;
  uint32_t* flag = comm ? nullptr : c->h_flag.d;
  if (c->counts_pending && c->prof.on) match_counts_fetch(c);  // exact byte model for the profile
  {
    // bytes: pair id per query + (p_i, n_i 32 B each, p_j 16 B) per accepted plane row,
    // (p_i 32 B, p_j 16 B) per accepted point pair
    ProfScope ps(c->prof, PROF_LINEARIZE, 4.0 * c->n_qo + 80.0 * c->rows_pl + 48.0 * c->rows_pt, st);
    hipLaunchKernelGGL(k_linearize_total, dim3(nblk), dim3(kTotWaves * kWave), 0, st, qo_rows(c), c->map_poses_p,
                       1.0 / sigma, c->bpart.p, c->ticket.p, dst, tjv, flag, seq, tot_chunks_per_wave(c));
    FMX_HIP(hipGetLastError());
  }
  if (comm) {
    comm_allreduce_publish(c, c->d_sum.p, 29, c->h_G);
  } else {
    wait_flag(c, c->h_flag.p, seq);
  }
  match_counts_fetch(c, false);  // the match kernel finished before this one started
  std::memcpy(out, c->h_G.p, 29 * sizeof(double));
}


// fmx_linearize_matched on a deferred match at the same pose: match + linearization in
// one launch (k_match's FUSED build), no per-query results materialized; the same
// completion-word / all-reduce handling as run_linearize_total.
void run_match_linearize_total(fmx_ctx* c, const double* pose_j34, double max_dist, double sigma, double* out) {
  if (!c->have_map) throw StatusError(FMX_E_STATE, "no map");
  comm_check(c);
  c->h_G.ensure(32);
  const bool comm = c->comm != nullptr;
  if (comm) c->d_sum.ensure(32);
  const uint32_t seq = next_flag(c);
  run_match_linearize(c, pose_j34, max_dist, sigma, comm ? c->d_sum.p : c->h_G.d, comm ? nullptr : c->h_flag.d, seq);
  if (comm) {
    comm_allreduce_publish(c, c->d_sum.p, 29, c->h_G);
  } else if (c->n_qpl + c->n_qpt == 0) {  // no launch: the zero system was set on the stream
    stream_wait(c);
  } else {
    wait_flag(c, c->h_flag.p, seq);
  }
  if (c->fz_work_pending) {  // profiling: the work counters of this launch (byte model)
    stream_wait(c);
    gl::work_fetch(c);
  }
  std::memcpy(out, c->h_G.p, 29 * sizeof(double));
}

}  // namespace fmx
