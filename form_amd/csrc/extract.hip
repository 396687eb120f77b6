// extract.hip — stage 1: per-scan feature extraction on gfx950.
//
// Restates form::FeatureExtractor::extract (form/feature/extraction.tpp:29-132) as
//   k_extract_rows : one workgroup per scan line.  The row is staged in LDS;
//                    validity masks (:136-222), LOAM curvature (:226-261), the
//                    per-sector greedy planar selection (:44-68, :332-358) and the
//                    point selection (:70-96, :360-399).
//   k_closest      : one wave per selected planar point; wave-wide argmin over
//                    the adjacent scan lines (find_closest, :402-420).
//   k_fit          : one lane per selected planar point; neighbour gather
//                    (find_neighbors, :422-448), A^T A covariance and the smallest
//                    eigenvector (compute_normal, :263-329).
//   k_row_scan / k_write_features : ordered compaction into the query arrays.
//
// Greedy planar selection.  The reference sorts each sector by curvature and
// accepts, in that order, every still-unused point under the threshold, clearing
// +-(k-1) columns around it, until planar_feats_per_sector+1 are accepted.  Here
// the block ranks the candidates by the strict key (curvature, column), then one
// wave walks them in key order 64 at a time: conflicts with accepted points of
// earlier chunks are read from LDS, conflicts inside the chunk are a 64-bit mask
// per lane resolved by ballot rounds.  (Parallel MIS rounds over the whole sector
// were exact too, but curvature is monotone along smooth surfaces, so the rounds
// chained ~pps/k deep.)  Sectors stay sequential: the suppression of sector s
// spills into sector s+1 (parity hazard 5).
#include "fmx_device.hpp"
#include "fmx_internal.hpp"

#include <cfloat>
#include <functional>
#include <cstdlib>

namespace fmx {
namespace {

constexpr int kRowThreads = 1024;  // 16 waves: the row phases are LDS-latency bound

struct ExArgs {
  int R, C, k, S, P, Ppt;
  int row0;            // k_extract_rows: first row of this launch (piecewise launches over a staged scan)
  int cap_pl, cap_pt;  // per-row slot capacities
  double thr, min2, max2, radius2;
  int min_points;
};

// Ordered (stable) block compaction of flag(c) for c in [b, e) into list[0..n).
// Returns n (uniform).  Uses ws[kRowThreads/64 + 1].
template <class F>
__device__ int block_compact(int b, int e, F flag, int* list, int* ws) {
  const int tid = threadIdx.x, w = tid / kWave;
  int base = 0;
  for (int t0 = b; t0 < e; t0 += kRowThreads) {
    const int c = t0 + tid;
    const bool f = c < e && flag(c);
    const uint64_t m = __ballot(f);
    if (lane_id() == 0) ws[w] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int i = 0; i < w; ++i) off += ws[i];
    int tot = 0;
    for (int i = 0; i < kRowThreads / kWave; ++i) tot += ws[i];
    if (f) list[off + __popcll(m & lanemask_lt())] = c;
    __syncthreads();
    base += tot;
  }
  return base;
}

// KC > 0: neighbor_points fixed at compile time (the default 5), so every +-k loop
// unrolls and its LDS reads issue together; KC = 0 reads it from the arguments.
template <int KC, bool PAR>
__global__ __launch_bounds__(kRowThreads) void k_extract_rows(const float4* __restrict__ scan, ExArgs a,
                                                              uint8_t* __restrict__ planar_mask,
                                                              uint32_t* __restrict__ sel_slots,
                                                              uint32_t* __restrict__ pt_slots,
                                                              uint32_t* __restrict__ row_counts) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int C = a.C, r = a.row0 + blockIdx.x, tid = threadIdx.x, k = KC > 0 ? KC : a.k;
  float4* pts = reinterpret_cast<float4*>(smem);
  uint64_t* keys = reinterpret_cast<uint64_t*>(pts + C);  // accepted planar keys (curv bits, column)
  int* list = reinterpret_cast<int*>(keys);                // point phase: compacted columns (aliases keys)
  float* curv = reinterpret_cast<float*>(keys + C);
  uint8_t* flg = reinterpret_cast<uint8_t*>(curv + C);  // bit0 point-valid, bit1 out-of-range, bit2 planar-valid
  uint8_t* used = flg + C;                               // used_points (planar) then point mask
  uint8_t* state = used + C;
  uint8_t* win = state + C;
  __shared__ int ws[kRowThreads / kWave + 1];
  __shared__ int s_cnt;

#ifdef FMX_EXTRACT_TIMING
  uint64_t tstamp[40];
  int nts = 0;
#define TSTAMP() (tstamp[nts < 40 ? nts++ : 39] = wall_clock64())
#else
#define TSTAMP() ((void)0)
#endif
  TSTAMP();
  const float4* row = scan + (size_t)r * C;
  for (int c = tid; c < C; c += kRowThreads) pts[c] = row[c];
  __syncthreads();
  TSTAMP();

  // compute_valid_points / compute_point_valid_points (extraction.tpp:136-222)
  for (int c = tid; c < C; c += kRowThreads) {
    uint8_t f = 0;
    if (c >= k && c < C - k) {
      const float4 p = pts[c];
      const double r2 = (double)sqnorm4f(p.x, p.y, p.z);
      const bool oor = r2 < a.min2 || r2 > a.max2;
      f = oor ? 2 : 1;
    }
    flg[c] = f;
  }
  __syncthreads();
  TSTAMP();
  // planar validity: neighbour invalidation of +-k around out-of-range points
  // (scatter at :170-173, evaluated here as a gather), then the curvature (:226-261).
  for (int c = tid; c < C; c += kRowThreads) {
    bool plv = (flg[c] & 1) != 0;
    if (plv) {  // valid => k <= c < C-k: the neighbour reads stay in the row (no branches, loads batch)
      uint32_t any = 0;
#pragma unroll
      for (int d = 1; d <= k; ++d) any |= (uint32_t)(flg[c - d] | flg[c + d]);
      plv = (any & 2) == 0;
    }
    float cv = FLT_MAX;
    if (plv) {
      const float4 p = pts[c];
      double dx = -(2.0 * k) * (double)p.x;
      double dy = -(2.0 * k) * (double)p.y;
      double dz = -(2.0 * k) * (double)p.z;
#pragma unroll
      for (int n = 1; n <= k; ++n) {
        const float4 qm = pts[c - n], qp = pts[c + n];
        dx = dx + (double)qm.x + (double)qp.x;
        dy = dy + (double)qm.y + (double)qp.y;
        dz = dz + (double)qm.z + (double)qp.z;
      }
      cv = (float)(dx * dx + dy * dy + dz * dz);
    }
    curv[c] = cv;
    win[c] = plv ? 1 : 0;
    planar_mask[(size_t)r * C + c] = plv ? 1 : 0;
  }
  __syncthreads();
  TSTAMP();
  for (int c = tid; c < C; c += kRowThreads) {
    if (win[c]) flg[c] |= 4;
    used[c] = win[c];
  }
  __syncthreads();
  TSTAMP();

  if constexpr (PAR) {
    // ================= sector-parallel selection (pps <= 512, S <= 16) ==============
    // Sectors interact only through suppression spilling k-1 columns over a sector
    // boundary (parity hazard 5).  Every sector is run speculatively at once (wave s
    // = sector s) as if nothing spilled in; then, in sector order, sector s is re-run
    // only if the FINAL selection of sector s-1 suppresses a column that the
    // speculative run of s depended on: for the planar greedy a column it ACCEPTED
    // (removing a candidate the greedy rejected changes nothing), for the point pass
    // a column that was ELIGIBLE (the stride of extract_point depends on |U|).
    const int S = a.S, pps = C / S, P1 = a.P + 1;
    const int w = tid / kWave, lane = lane_id();
    auto sec_b = [&](int s) { return s * pps; };
    auto sec_e = [&](int s) { return s == S - 1 ? C : (s + 1) * pps; };
    int* srt = reinterpret_cast<int*>(pts);                         // sorted candidate columns, per sector at b
    uint32_t* pos = reinterpret_cast<uint32_t*>(srt + C);            // chunk-lane stamps per column
    const int nwd = (C + 63) / 64 + 1;
    uint64_t* accb = reinterpret_cast<uint64_t*>(pts) + C;           // accepted (speculative) bitmap
    int* klist = reinterpret_cast<int*>(accb + nwd);                 // [S][P+1] kept columns in key order
    int* klist2 = klist + S * P1;                                    // [S][P+1] fix-up re-run results
    int* sel_pt = reinterpret_cast<int*>(curv);                      // point selections, per sector at b (after planar)
    __shared__ int s_cntS[16], s_keepS[16], s_nuS[16], s_nptS[16];
    __shared__ int s_keep2[16], s_hiA[16], s_fin[16];
    if (tid < 16) s_cntS[tid] = s_keepS[tid] = s_nuS[tid] = s_nptS[tid] = s_keep2[tid] = s_fin[tid] = 0;
    for (int c = tid; c < C; c += kRowThreads) pos[c] = 0xFFFFFFFFu;
    for (int i = tid; i < nwd; i += kRowThreads) accb[i] = 0;
    __syncthreads();
    // P1: candidates (used && curvature < threshold, :340-342) as keys (curvature
    // bits, column), per sector
    for (int c = tid; c < C; c += kRowThreads)
      if (used[c] && (double)curv[c] < a.thr) {
        const int s = min(c / pps, S - 1);
        keys[sec_b(s) + atomicAdd(&s_cntS[s], 1)] = ((uint64_t)__float_as_uint(curv[c]) << 32) | (uint32_t)c;
      }
    __syncthreads();
    TSTAMP();
    // P2: wave s bitonic-sorts sector s's keys in registers (8 per lane, blocked:
    // element e = lane * 8 + u), pads with ~0
    if (w < S) {
      const int b = sec_b(w), n = s_cntS[w];
      uint64_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = lane * 8 + u < n ? keys[b + lane * 8 + u] : ~0ull;
#pragma unroll
      for (int kk = 2; kk <= 512; kk <<= 1) {
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
          if (j >= 8) {
            const int lj = j >> 3;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int e = lane * 8 + u;
              uint64_t o;  // lane lane ^ lj's element u (DPP / permlane: no LDS traffic)
              switch (lj) {
                case 1: o = xor_lane<1>(v[u]); break;
                case 2: o = xor_lane<2>(v[u]); break;
                case 4: o = xor_lane<4>(v[u]); break;
                case 8: o = xor_lane<8>(v[u]); break;
                case 16: o = xor_lane<16>(v[u]); break;
                default: o = xor_lane<32>(v[u]); break;
              }
              const bool up = (e & kk) == 0, lower = (e & j) == 0;
              v[u] = (up == lower) ? (v[u] < o ? v[u] : o) : (v[u] < o ? o : v[u]);
            }
          } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int pu = u ^ j;
              if (pu > u) {
                const int e = lane * 8 + u;
                const bool up = (e & kk) == 0;
                const uint64_t x = v[u], y = v[pu];
                const bool sw = up ? (x > y) : (x < y);
                v[u] = sw ? y : x;
                v[pu] = sw ? x : y;
              }
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (lane * 8 + u < n) srt[b + lane * 8 + u] = (int)(uint32_t)v[u];
    }
    __syncthreads();
    TSTAMP();
    // planar greedy of sector s by one wave (:343-355), as k_extract_rows; columns
    // [b, blk_hi] are suppressed by the previous sector (blk_hi < b: none)
    // A fix-up re-run resumes at candidate rank `start` with the first `kept0` kept
    // columns already accepted (their decisions cannot change: they precede every
    // suppressed column in key order); its chunk stamps start at `chunk0` so they never
    // equal the stale stamps of the speculative run (chunking may differ).
    auto planar_greedy = [&](int s, int blk_hi, int start, int kept0, uint32_t chunk0, int* out, int* out_keep) {
      const int b = sec_b(s), e = sec_e(s), n = s_cntS[s];
      int kept = kept0;
      uint32_t chunk = chunk0;
      for (int base = start; base < n && kept < P1; base += kWave, ++chunk) {
        const uint32_t stamp = ((uint32_t)s << 14) | chunk;
        const int idx = base + lane;
        const bool in = idx < n;
        const int c = in ? srt[b + idx] : b;
        const int lo = c - (k - 1) < b ? b : c - (k - 1), hi = c + (k - 1) >= e ? e - 1 : c + (k - 1);
        bool und = in && c > blk_hi;
        if (in) {
          pos[c] = (stamp << 6) | (uint32_t)lane;
          const int w0 = lo >> 6, w1 = hi >> 6;
          for (int ww = w0; ww <= w1; ++ww) {
            uint64_t m = accb[ww];
            if (ww == w0) m &= ~0ull << (lo & 63);
            if (ww == w1) m &= ~0ull >> (63 - (hi & 63));
            if (m) und = false;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint64_t conf = 0;
        if (und) {
#pragma unroll
          for (int j = lo; j <= hi; ++j) {
            const uint32_t q = pos[j];
            if ((q >> 6) == stamp && (int)(q & 63) < lane) conf |= 1ull << (q & 63);
          }
        }
        uint64_t A = 0;
        for (;;) {
          const uint64_t U = __ballot(und);
          if (U == 0) break;
          const bool acc = und && (conf & U) == 0;
          A |= __ballot(acc);
          if (acc || (conf & A) != 0) und = false;
        }
        if ((A >> lane) & 1) {
          const int rank = kept + __popcll(A & lanemask_lt());
          if (rank < P1) out[s * P1 + rank] = c;
          atomicOr(reinterpret_cast<unsigned long long*>(&accb[c >> 6]), 1ull << (c & 63));
        }
        kept += __popcll(A);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      if (lane == 0) out_keep[s] = kept < P1 ? kept : P1;
    };
    if (w < S) planar_greedy(w, -1, 0, 0, 0, klist, s_keepS);
    __syncthreads();
    TSTAMP();
    // P4: fix-up.  Sector s's final selection depends on sector s-1's only through the
    // columns [b, hi] that s-1's last kept point suppresses (hi = its column + k - 1).
    // (a) every sector s >= 1 in parallel (wave s): assume s-1's speculative selection
    // is final, and if that suppresses one of s's kept columns, re-run s from there
    // (resume: the kept columns before the first affected one stand) into klist2.
    // (b) wave 0, in sector order: with s-1's actual final selection, keep (a)'s
    // outcome when its assumed hi was right (the usual case: re-runs start at the
    // sector's left edge and rarely move its last kept column), else redo s.
    auto hi_of = [&](const int* lst, int np, int s) {  // suppression reach into sector s, or -1
      int mx = -1;
      for (int i = lane; i < np; i += kWave) mx = max(mx, lst[(s - 1) * P1 + i]);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
      const int hi = min(mx + (k - 1), sec_e(s) - 1);
      return (mx < 0 || hi < sec_b(s)) ? -1 : hi;
    };
    // resume sector s from its speculative selection with [b, hi] suppressed; returns
    // false when none of its kept columns lies in [b, hi] (the speculative one stands)
    auto rerun = [&](int s, int hi, uint32_t chunk0) {
      const int b = sec_b(s), e = sec_e(s), nk = s_keepS[s];
      int r0 = P1;
      for (int i = lane; i < nk; i += kWave)
        if (klist[s * P1 + i] <= hi) r0 = min(r0, i);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) r0 = min(r0, __shfl_xor(r0, o, 64));
      if (r0 >= nk) return false;
      const int col0 = klist[s * P1 + r0];
      int start = 0x7FFFFFFF;  // its candidate rank in the sorted sector
      for (int i = lane; i < s_cntS[s]; i += kWave)
        if (srt[b + i] == col0) start = i;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) start = min(start, __shfl_xor(start, o, 64));
      for (int c = b + lane; c < e; c += kWave)  // the sector's accepted bits := kept[0, r0)
        atomicAnd(reinterpret_cast<unsigned long long*>(&accb[c >> 6]), ~(1ull << (c & 63)));
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int i = lane; i < r0; i += kWave) {
        const int c = klist[s * P1 + i];
        atomicOr(reinterpret_cast<unsigned long long*>(&accb[c >> 6]), 1ull << (c & 63));
        klist2[s * P1 + i] = c;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      planar_greedy(s, hi, start, r0, chunk0, klist2, s_keep2);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      return true;
    };
    __shared__ int s_mxF[16];  // last kept column of each sector's (a) outcome
    auto last_kept = [&](const int* lst, int np, int s) {
      int mx = -1;
      for (int i = lane; i < np; i += kWave) mx = max(mx, lst[s * P1 + i]);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
      return mx;
    };
    if (w >= 1 && w < S) {  // (a)
      const int hi = hi_of(klist, s_keepS[w - 1], w);
      const bool re = hi >= 0 && rerun(w, hi, 512);
      if (lane == 0) {
        s_hiA[w] = hi;
        s_fin[w] = re ? 1 : 0;
      }
    }
    if (w < S) {  // each sector's last kept column after (a)
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int fw = s_fin[w];
      const int mx = last_kept(fw ? klist2 : klist, fw ? s_keep2[w] : s_keepS[w], w);
      if (lane == 0) s_mxF[w] = mx;
    }
    __syncthreads();
    TSTAMP();
    if (w == 0) {  // (b): integer checks; a redo (rare) refreshes the sector's last column
      for (int s = 1; s < S; ++s) {
        const int mx = s_mxF[s - 1];
        const int hi0 = min(mx + (k - 1), sec_e(s) - 1);
        const int hi = (mx < 0 || hi0 < sec_b(s)) ? -1 : hi0;
        if (hi == s_hiA[s]) continue;
        const bool re = hi >= 0 && rerun(s, hi, 1024);
        const int mxn = last_kept(re ? klist2 : klist, re ? s_keep2[s] : s_keepS[s], s);
        if (lane == 0) {
          s_fin[s] = re ? 1 : 0;
          s_mxF[s] = mxn;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
    TSTAMP();
    // P5: suppression used[c +- n], n in [0, k) of every kept point (:347-350)
    for (int t = tid; t < S * P1; t += kRowThreads) {
      const int s = t / P1, i = t % P1;
      if (i < (s_fin[s] ? s_keep2[s] : s_keepS[s])) {
        const int c = s_fin[s] ? klist2[t] : klist[t];
        for (int n = 0; n < k; ++n) {
          used[c + n] = 0;
          used[c - n] = 0;
        }
      }
    }
    __syncthreads();
    int pl_count = 0;
    for (int s = 0; s < S; ++s) {
      const int nk = s_fin[s] ? s_keep2[s] : s_keepS[s];
      const int* lst = s_fin[s] ? klist2 : klist;
      for (int i = tid; i < nk; i += kRowThreads)
        if (pl_count + i < a.cap_pl) sel_slots[(size_t)r * a.cap_pl + pl_count + i] = (uint32_t)lst[s * P1 + i];
      pl_count += nk;
    }
    TSTAMP();
    // ---------------- point features (extraction.tpp:70-96)
    // eligible = (used == planar_valid) && point_valid (:77-79); state[] keeps the
    // eligibility for the fix-up
    for (int c = tid; c < C; c += kRowThreads) {
      const uint8_t f = flg[c];
      const uint8_t el = ((f & 1) && (used[c] == ((f >> 2) & 1))) ? 1 : 0;
      win[c] = el;
      state[c] = el;
    }
    __syncthreads();
    TSTAMP();
    // one sector's extract_point by one wave: U = eligible columns of [b, e) in
    // order (suppressed columns [b, blk_hi] excluded), phase A literal by lane 0,
    // phase B as a register scan; suppression stays inside the sector (what it spills
    // into the next sector is the fix-up's business)
    auto point_pass = [&](int s, int blk_hi) {
      const int b = sec_b(s), e = sec_e(s);
      int nu = 0;
      for (int c0 = b; c0 < e; c0 += kWave) {
        const int c = c0 + lane;
        const bool f = c < e && c > blk_hi && win[c] != 0;
        const uint64_t m = __ballot(f);
        if (f) list[b + nu + __popcll(m & lanemask_lt())] = c;
        nu += __popcll(m);
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      auto suppress = [&](int c) {
        for (int n = 0; n < k; ++n) {
          if (c + n < e) win[c + n] = 0;
          if (c - n >= b) win[c - n] = 0;
        }
      };
      int nf = 0, offA = 0;
      bool stopA = false;
      const int factor = a.Ppt > 0 ? 1 + nu / a.Ppt : 0;
      if (lane == 0 && a.Ppt > 0) {
        for (int off = 0; off < factor && !stopA; ++off) {
          for (int ui = off; ui < nu; ui += factor) {
            const int c = list[b + ui];
            if (win[c]) {
              sel_pt[b + nf] = c;
              suppress(c);
              nf++;
            }
            if (nf > a.Ppt) {
              stopA = true;
              offA = off;
              break;
            }
          }
        }
      }
      nf = __shfl(nf, 0, 64);
      stopA = __shfl((int)stopA, 0, 64) != 0;
      offA = __shfl(offA, 0, 64);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (stopA) {
        const int nA = nf;
        int last = -0x40000000;
        const int ohi = min(factor, nu);  // heads U[o] exist for o < nu only
        for (int o0 = offA + 1; o0 < ohi; o0 += kWave) {
          const int o = o0 + lane;
          const int c = o < ohi ? list[b + o] : 0x7FFFFFFF;
          const int el = o < ohi ? (int)win[c] : 0;
          const int nl = min(kWave, ohi - o0);
          for (int l = 0; l < nl; ++l) {
            const int cl = __builtin_amdgcn_readlane(c, l);
            const int ell = __builtin_amdgcn_readlane(el, l);
            if (ell && cl > last + (k - 1)) {
              if (lane == 0) sel_pt[b + nf] = cl;
              last = cl;
              nf++;
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int i = nA + lane; i < nf; i += kWave) suppress(sel_pt[b + i]);  // phase-B heads (:388-391)
      }
      if (lane == 0) {
        s_nptS[s] = nf;
        s_nuS[s] = nu;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    };
    if (w < S) point_pass(w, -1);
    __syncthreads();
    TSTAMP();
    // Q3: fix-up in sector order (wave 0): the previous sector's final selections
    // suppress [b, mx + k - 1]; if an eligible column lies there, re-run the sector
    if (w == 0) {
      for (int s = 1; s < S; ++s) {
        const int b = sec_b(s), e = sec_e(s);
        const int np = s_nptS[s - 1], bp = sec_b(s - 1);
        int mx = -1;
        for (int i = lane; i < np; i += kWave) mx = max(mx, sel_pt[bp + i]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
        const int hi = min(mx + (k - 1), e - 1);
        if (mx < 0 || hi < b) continue;
        bool hit = false;
        for (int c = b + lane; c <= hi; c += kWave)
          if (state[c]) hit = true;
        if (!__ballot(hit)) continue;
        for (int c = b + lane; c < e; c += kWave) win[c] = state[c];  // eligibility before the speculative run
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        point_pass(s, hi);
      }
    }
    __syncthreads();
    TSTAMP();
    int pt_count = 0;
    for (int s = 0; s < S; ++s) {
      const int np = s_nptS[s], b = sec_b(s);
      for (int i = tid; i < np; i += kRowThreads)  // (bounded: selections are >= k apart)
        if (pt_count + i < a.cap_pt) pt_slots[(size_t)r * a.cap_pt + pt_count + i] = (uint32_t)sel_pt[b + i];
      pt_count += np;
    }
    if (tid == 0) {
      row_counts[2 * r] = (uint32_t)min(pl_count, a.cap_pl);
      row_counts[2 * r + 1] = (uint32_t)min(pt_count, a.cap_pt);
    }
#ifdef FMX_EXTRACT_TIMING
    if (tid == 0 && (r == 5 || r == 64 || r == 120)) {
      int d[16] = {0};
      for (int i = 1; i < nts && i < 17; ++i) d[i - 1] = (int)(tstamp[i] - tstamp[i - 1]);
      printf("PAR row %d: pre %d %d %d %d | cand %d sort %d greedy %d fixA %d fixB %d supp+out %d | elig %d pass %d fix %d\n", r,
             d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9], d[10], d[11], d[12]);
    }
#endif
    return;
  } else {
  // ---------------- planar features: sectors in order (extraction.tpp:44-68)
  // pts[] is dead from here on; its 16C bytes hold the key-sorted candidates srt[C],
  // the chunk-lane map pos[C] ((stamp << 6) | lane) and the accepted bitmap accb.
  int* srt = reinterpret_cast<int*>(pts);
  uint32_t* pos = reinterpret_cast<uint32_t*>(srt + C);
  uint64_t* accb = reinterpret_cast<uint64_t*>(pts) + C;  // byte offset 8C
  for (int c = tid; c < C; c += kRowThreads) pos[c] = 0xFFFFFFFFu;
  const int pps = C / a.S;
  int pl_count = 0;  // uniform
  uint32_t stamp = 0;  // chunk id within the row (uniform)
  for (int s = 0; s < a.S; ++s) {
    const int b = s * pps;
    const int e = (s == a.S - 1) ? C : b + pps;
    // candidates (used && curvature < threshold, :340-342) as packed keys
    // (curvature bits, column): curvature >= 0, so the u64 order is (curv, column).
    if (tid == 0) s_cnt = 0;
    for (int c = b + tid; c < e; c += kRowThreads) state[c] = 0;
    for (int w = (b >> 6) + tid; w <= ((e - 1) >> 6); w += kRowThreads) accb[w] = 0;
    __syncthreads();
    for (int c = b + tid; c < e; c += kRowThreads)
      if (used[c] && (double)curv[c] < a.thr)
        keys[atomicAdd(&s_cnt, 1)] = ((uint64_t)__float_as_uint(curv[c]) << 32) | (uint32_t)c;
    __syncthreads();
    const int n_c = s_cnt;
    if (s < 2) TSTAMP();
    // sort by counting: rank of each key, `sub` adjacent lanes per candidate
    // (each part scans a contiguous, even-aligned range two keys per 16-B read)
    int sub = 1;
    while (sub < 8 && sub * 2 * n_c <= kRowThreads) sub *= 2;
    if (tid == 0 && (n_c & 1)) keys[n_c] = ~0ull;  // pad: never < a key
    __syncthreads();
    for (int t = tid; t < n_c * sub; t += kRowThreads) {
      const int i = t / sub, part = t % sub;
      const uint64_t ki = keys[i];
      const int npair = (n_c + 1) >> 1, per = (npair + sub - 1) / sub;
      const int p0 = part * per, p1 = min(npair, p0 + per);
      const ulonglong2* kp = reinterpret_cast<const ulonglong2*>(keys);
      int rank = 0;
      int j = p0;
      for (; j + 3 < p1; j += 4) {
        const ulonglong2 q0 = kp[j], q1 = kp[j + 1], q2 = kp[j + 2], q3 = kp[j + 3];
        rank += (q0.x < ki) + (q0.y < ki) + (q1.x < ki) + (q1.y < ki) + (q2.x < ki) + (q2.y < ki) +
                (q3.x < ki) + (q3.y < ki);
      }
      for (; j < p1; ++j) {
        const ulonglong2 q = kp[j];
        rank += (q.x < ki) + (q.y < ki);
      }
      for (int o = 1; o < sub; o <<= 1) rank += __shfl_xor(rank, o, 64);
      if (part == 0) srt[rank] = (int)(uint32_t)ki;
    }
    __syncthreads();
    if (s < 2) TSTAMP();
    // Greedy in key order (:343-355), one wave, 64 candidates per chunk: a candidate
    // is accepted iff no accepted candidate of lower key lies within k-1 columns.
    // Earlier chunks: accepted bitmap.  Inside the chunk: each lane maps its column
    // to (stamp, lane) in pos[], reads its +-(k-1) neighbours' lanes into a conflict
    // mask of lower-key lanes, and ballot rounds resolve the chunk.
    if (tid < kWave) {
      const int lane = tid;
      int kept = 0;  // wave-uniform
      for (int base = 0; base < n_c && kept < a.P + 1; base += kWave, ++stamp) {
        const int idx = base + lane;
        const bool in = idx < n_c;
        const int c = in ? srt[idx] : b;
        const int lo = c - (k - 1) < b ? b : c - (k - 1), hi = c + (k - 1) >= e ? e - 1 : c + (k - 1);
        bool und = in;
        if (in) {
          pos[c] = (stamp << 6) | (uint32_t)lane;
          const int w0 = lo >> 6, w1 = hi >> 6;
          for (int w = w0; w <= w1; ++w) {
            uint64_t m = accb[w];
            if (w == w0) m &= ~0ull << (lo & 63);
            if (w == w1) m &= ~0ull >> (63 - (hi & 63));
            if (m) und = false;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint64_t conf = 0;
        if (und) {
#pragma unroll
          for (int j = lo; j <= hi; ++j) {
            const uint32_t q = pos[j];
            if ((q >> 6) == stamp && (int)(q & 63) < lane) conf |= 1ull << (q & 63);
          }
        }
        uint64_t A = 0;
        for (;;) {
          const uint64_t U = __ballot(und);
          if (U == 0) break;
          const bool acc = und && (conf & U) == 0;
          A |= __ballot(acc);
          if (acc || (conf & A) != 0) und = false;
        }
        if ((A >> lane) & 1) {
          const int rank = kept + __popcll(A & lanemask_lt());
          if (rank < a.P + 1) {
            sel_slots[(size_t)r * a.cap_pl + pl_count + rank] = (uint32_t)c;
            state[c] = 4;
          }
          atomicOr(reinterpret_cast<unsigned long long*>(&accb[c >> 6]), 1ull << (c & 63));
        }
        kept += __popcll(A);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      if (tid == 0) s_cnt = kept < a.P + 1 ? kept : a.P + 1;
    }
    __syncthreads();
    if (s < 2) TSTAMP();
    const int keep = s_cnt;
    // suppression used[c +- n], n in [0, k) (:347-350)
    for (int c = b + tid; c < e; c += kRowThreads) {
      if (state[c] != 4) continue;
      for (int n = 0; n < k; ++n) {
        used[c + n] = 0;
        used[c - n] = 0;
      }
    }
    pl_count += keep;
    __syncthreads();
    TSTAMP();
  }

  // ---------------- point features (extraction.tpp:70-96)
  // eligible = (used == planar_valid) && point_valid  (:77-79)
  for (int c = tid; c < C; c += kRowThreads) {
    const uint8_t f = flg[c];
    win[c] = ((f & 1) && (used[c] == ((f >> 2) & 1))) ? 1 : 0;
  }
  __syncthreads();
  int pt_count = 0;  // uniform (broadcast through s_cnt)
  for (int s = 0; s < a.S; ++s) {
    const int b = s * pps;
    const int e = (s == a.S - 1) ? C : b + pps;
    const int nu = block_compact(b, e, [&](int c) { return win[c] != 0; }, list, ws);
    if (s < 1) TSTAMP();
    if (tid < kWave) {
      // extract_point (:360-399).  Phase A, literal, lane 0: passes off = 0, 1, ...
      // over U[off], U[off+factor], ... until the (Ppt+1)-th accept; the break at
      // :395-396 then leaves exactly one element, U[off], per later pass (phase B).
      int nf = 0, offA = 0;
      bool stopA = false;
      const int factor = a.Ppt > 0 ? 1 + nu / a.Ppt : 0;
      if (tid == 0 && a.Ppt > 0) {
        for (int off = 0; off < factor && !stopA; ++off) {
          for (int ui = off; ui < nu; ui += factor) {
            const int c = list[ui];
            if (win[c]) {
              pt_slots[(size_t)r * a.cap_pt + pt_count + nf] = (uint32_t)c;
              for (int n = 0; n < k; ++n) {
                win[c + n] = 0;
                win[c - n] = 0;
              }
              nf++;
            }
            if (nf > a.Ppt) {
              stopA = true;
              offA = off;
              break;
            }
          }
        }
      }
      nf = __shfl(nf, 0, 64);
      stopA = __shfl((int)stopA, 0, 64) != 0;
      offA = __shfl(offA, 0, 64);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (stopA) {
        // Phase B: heads U[o], o = offA+1 .. factor-1, are consecutive in U (column
        // order).  A head is taken iff still eligible after phase A (win[]) and more
        // than k-1 columns past the last taken head: a 1-D greedy scanned from
        // registers, 64 heads per chunk, state kept wave-uniform.
        int last = -0x40000000;
        const int ohi = min(factor, nu);  // heads U[o] exist for o < nu only
        for (int o0 = offA + 1; o0 < ohi; o0 += kWave) {
          const int o = o0 + tid;
          const int c = o < ohi ? list[o] : 0x7FFFFFFF;
          const int el = o < ohi ? (int)win[c] : 0;
          const int nl = min(kWave, ohi - o0);
          for (int l = 0; l < nl; ++l) {
            const int cl = __builtin_amdgcn_readlane(c, l);
            const int ell = __builtin_amdgcn_readlane(el, l);
            if (ell && cl > last + (k - 1)) {
              if (tid == 0) pt_slots[(size_t)r * a.cap_pt + pt_count + nf] = (uint32_t)cl;
              last = cl;
              nf++;
            }
          }
        }
        // suppression of the phase-B heads (spills into the next sector, :388-391)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      if (tid == 0) s_cnt = pt_count + nf;
    }
    __syncthreads();
    if (s < 1) TSTAMP();
    // apply phase-B suppression from the written slots (phase A already applied)
    {
      const int n0 = pt_count, n1 = s_cnt;
      for (int i = n0 + tid; i < n1; i += kRowThreads) {
        const int c = (int)pt_slots[(size_t)r * a.cap_pt + i];
        for (int n = 0; n < k; ++n) {
          win[c + n] = 0;
          win[c - n] = 0;
        }
      }
    }
    __syncthreads();
    pt_count = s_cnt;
    __syncthreads();
    TSTAMP();
  }
  if (tid == 0) {
    row_counts[2 * r] = (uint32_t)pl_count;
    row_counts[2 * r + 1] = (uint32_t)pt_count;
  }
#ifdef FMX_EXTRACT_TIMING
  if (tid == 0 && (r == 5 || r == 64 || r == 120)) {
    int d[24] = {0};
    for (int i = 1; i < nts && i < 24; ++i) d[i - 1] = (int)(tstamp[i] - tstamp[i - 1]);
    printf("row %d ticks: %d %d %d %d | %d %d %d %d %d %d %d %d %d %d %d %d %d %d %d %d %d %d %d %d\n", r, d[0], d[1],
           d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9], d[10], d[11], d[12], d[13], d[14], d[15], d[16], d[17],
           d[18], d[19], d[20], d[21], d[22], d[23]);
  }
#endif
  }  // !PAR
}

// Per-row 64-column block AABBs of the planar-valid points (one wave per block),
// used to prune find_closest exactly.  Empty block: lo = +inf, hi = -inf.
__global__ __launch_bounds__(256) void k_row_blocks(const float4* __restrict__ scan,
                                                    const uint8_t* __restrict__ mask, int R, int C,
                                                    float4* __restrict__ blo, float4* __restrict__ bhi) {
  const int nblk = (C + kWave - 1) / kWave;
  const int wv = blockIdx.x * 4 + threadIdx.x / kWave;
  if (wv >= R * nblk) return;
  const int r = wv / nblk, bk = wv % nblk;
  const int j = bk * kWave + lane_id();
  float lx = INFINITY, ly = INFINITY, lz = INFINITY, hx = -INFINITY, hy = -INFINITY, hz = -INFINITY;
  if (j < C && mask[(size_t)r * C + j]) {
    const float4 p = scan[(size_t)r * C + j];
    lx = hx = p.x;
    ly = hy = p.y;
    lz = hz = p.z;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lx = fminf(lx, __shfl_xor(lx, o, 64));
    ly = fminf(ly, __shfl_xor(ly, o, 64));
    lz = fminf(lz, __shfl_xor(lz, o, 64));
    hx = fmaxf(hx, __shfl_xor(hx, o, 64));
    hy = fmaxf(hy, __shfl_xor(hy, o, 64));
    hz = fmaxf(hz, __shfl_xor(hz, o, 64));
  }
  if (lane_id() == 0) {
    blo[wv] = make_float4(lx, ly, lz, 0.f);
    bhi[wv] = make_float4(hx, hy, hz, 0.f);
  }
}

// find_closest (extraction.tpp:402-420) over rows r-1 and r+1: one wave per slot.
// Exact argmin with the reference's semantics (float distance promoted to double,
// strict <, first index on ties): the block holding the query's own column is
// scanned first, then only blocks whose box lower bound, shrunk by 1e-5 relative
// (>> the few-ulp error of the fp32 distance), does not exceed the running best.
__global__ __launch_bounds__(256) void k_closest(const float4* __restrict__ scan,
                                                 const uint8_t* __restrict__ mask,
                                                 const uint32_t* __restrict__ sel_slots,
                                                 const uint32_t* __restrict__ row_counts, int R, int C,
                                                 int cap, const float4* __restrict__ blo,
                                                 const float4* __restrict__ bhi, int2* __restrict__ closest) {
  const int wv = blockIdx.x * (256 / kWave) + threadIdx.x / kWave;
  const int r = wv / cap, slot = wv % cap;
  if (r >= R) return;
  if ((uint32_t)slot >= row_counts[2 * r]) return;
  const int lane = lane_id();
  const int nblk = (C + kWave - 1) / kWave;
  const int c = (int)sel_slots[(size_t)r * cap + slot];
  const float4 p = scan[(size_t)r * C + c];
  int res[2];
  for (int dir = 0; dir < 2; ++dir) {
    const int rr = dir == 0 ? r - 1 : r + 1;
    res[dir] = -1;
    if (rr < 0 || rr >= R) continue;
    const float4* row = scan + (size_t)rr * C;
    const uint8_t* mrow = mask + (size_t)rr * C;
    float best = 0.f;
    int bj = -1;
    auto scan_block = [&](int bk) {
      const int j = bk * kWave + lane;
      float d = 0.f;
      int dj = -1;
      if (j < C && mrow[j]) {
        d = dist2f(row[j], p);
        if (d <= FLT_MAX) dj = j;  // reference: double(d) < DBL_MAX
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float od = __shfl_xor(d, o, 64);
        const int oj = __shfl_xor(dj, o, 64);
        if (oj >= 0 && (dj < 0 || od < d || (od == d && oj < dj))) {
          d = od;
          dj = oj;
        }
      }
      if (dj >= 0 && (bj < 0 || d < best || (d == best && dj < bj))) {
        best = d;
        bj = dj;
      }
    };
    const int own = c / kWave;
    scan_block(own);
    // lane l owns block l (and l + 64, ... for very wide rows)
    for (int b0 = 0; b0 < nblk; b0 += kWave) {
      const int bk = b0 + lane;
      double lb = INFINITY;
      if (bk < nblk && bk != own) {
        const float4 lo = blo[(size_t)rr * nblk + bk], hi = bhi[(size_t)rr * nblk + bk];
        if (lo.x <= hi.x) {  // non-empty
          const double qx = p.x, qy = p.y, qz = p.z;
          const double ex = fmax(fmax((double)lo.x - qx, qx - (double)hi.x), 0.0);
          const double ey = fmax(fmax((double)lo.y - qy, qy - (double)hi.y), 0.0);
          const double ez = fmax(fmax((double)lo.z - qz, qz - (double)hi.z), 0.0);
          lb = (ex * ex + ey * ey + ez * ez) * (1.0 - 1e-5);
        }
      }
      uint64_t cand = __ballot(bk < nblk && bk != own && lb < INFINITY && (bj < 0 || lb <= (double)best));
      while (cand) {
        const int l = __ffsll((unsigned long long)cand) - 1;
        cand &= cand - 1;
        // re-check against the (possibly improved) best before scanning
        const double lbl = __shfl(lb, l, 64);
        if (bj >= 0 && lbl > (double)best) continue;
        scan_block(b0 + l);
      }
    }
    res[dir] = bj < 0 ? -1 : rr * C + bj;
  }
  if (lane == 0) closest[(size_t)r * cap + slot] = make_int2(res[0], res[1]);
}

// Cyclic Jacobi on the symmetric 3x3 covariance in double; returns the unit
// eigenvector of the smallest eigenvalue (Eigen::SelfAdjointEigenSolver col(0)).
__device__ __forceinline__ void smallest_eigvec(const float cov[3][3], double n[3]) {
  double A[3][3], V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) A[i][j] = (double)cov[i][j];
  for (int sweep = 0; sweep < 64; ++sweep) {
    const double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
    const double dia = A[0][0] * A[0][0] + A[1][1] * A[1][1] + A[2][2] * A[2][2];
    if (off <= 1e-36 * dia || off == 0.0) break;
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
#pragma unroll
      for (int qq = pp + 1; qq < 3; ++qq) {
        const double apq = A[pp][qq];
        if (apq == 0.0) continue;
        const double theta = (A[qq][qq] - A[pp][pp]) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double cc = 1.0 / sqrt(t * t + 1.0), ss = t * cc;
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          const double amp = A[m][pp], amq = A[m][qq];
          A[m][pp] = cc * amp - ss * amq;
          A[m][qq] = ss * amp + cc * amq;
        }
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          const double apm = A[pp][m], aqm = A[qq][m];
          A[pp][m] = cc * apm - ss * aqm;
          A[qq][m] = ss * apm + cc * aqm;
        }
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          const double vmp = V[m][pp], vmq = V[m][qq];
          V[m][pp] = cc * vmp - ss * vmq;
          V[m][qq] = ss * vmp + cc * vmq;
        }
      }
    }
  }
  int mi = 0;  // first smallest diagonal entry (no dynamic indexing: no scratch)
  double dm = A[0][0];
  if (A[1][1] < dm) {
    mi = 1;
    dm = A[1][1];
  }
  if (A[2][2] < dm) mi = 2;
  double v0 = mi == 0 ? V[0][0] : (mi == 1 ? V[0][1] : V[0][2]);
  double v1 = mi == 0 ? V[1][0] : (mi == 1 ? V[1][1] : V[1][2]);
  double v2 = mi == 0 ? V[2][0] : (mi == 1 ? V[2][1] : V[2][2]);
  const double nn = sqrt(v0 * v0 + v1 * v1 + v2 * v2);
  n[0] = v0 / nn;
  n[1] = v1 / nn;
  n[2] = v2 / nn;
}

// compute_normal (extraction.tpp:263-329): one lane per selected planar point.
__device__ int fit_one(const float4* __restrict__ scan, const uint32_t* __restrict__ sel_slots,
                       const int2* __restrict__ closest, const ExArgs& a, float4* __restrict__ nrm_slots,
                       int r, int slot);

// Block (r, part): slots part*blockDim .. of row r; the row's found-normal count is
// a block count (__syncthreads_count) + one atomic per block.
__global__ __launch_bounds__(256) void k_fit(const float4* __restrict__ scan,
                                             const uint32_t* __restrict__ sel_slots,
                                             const uint32_t* __restrict__ row_counts,
                                             const int2* __restrict__ closest, ExArgs a,
                                             float4* __restrict__ nrm_slots,
                                             uint32_t* __restrict__ row_ok) {
  const int r = blockIdx.y;
  const int slot = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = (uint32_t)slot < row_counts[2 * r];
  const int found = active ? fit_one(scan, sel_slots, closest, a, nrm_slots, r, slot) : 0;
  const int nfound = __syncthreads_count(found);
  if (threadIdx.x == 0 && nfound) atomicAdd(&row_ok[2 * r], (uint32_t)nfound);  // pair [2r, 2r+1], see k_row_scan
}

__device__ int fit_one(const float4* __restrict__ scan, const uint32_t* __restrict__ sel_slots,
                       const int2* __restrict__ closest, const ExArgs& a, float4* __restrict__ nrm_slots,
                       int r, int slot) {
  const int C = a.C, k = a.k;
  const size_t idx = (size_t)r * C + sel_slots[(size_t)r * a.cap_pl + slot];
  const float4 p = scan[idx];
  const int2 cl = closest[(size_t)r * a.cap_pl + slot];
  const double r2 = a.radius2;
  // visit(q): the neighbour sequence of the reference, in push order
  auto walk = [&](auto&& visit) {
    auto nbrs = [&](size_t j) {  // find_neighbors(j) (:422-448)
      const float4 pj = scan[j];
      for (int i = 1; i <= k; ++i) {
        const float4 q = scan[j + i];
        if ((double)dist2f(q, pj) < r2) visit(q);
        else break;
      }
      for (int i = 1; i <= k; ++i) {
        const float4 q = scan[j - i];
        if ((double)dist2f(q, pj) < r2) visit(q);
        else break;
      }
    };
    nbrs(idx);
    if (cl.x >= 0) {
      visit(scan[cl.x]);
      nbrs((size_t)cl.x);
    }
    if (cl.y >= 0) {
      visit(scan[cl.y]);
      nbrs((size_t)cl.y);
    }
  };
  int cnt = 0;
  walk([&](float4) { ++cnt; });
  float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
  if ((cl.x >= 0 || cl.y >= 0) && cnt >= a.min_points) {
    const float nf = (float)cnt;
    float cov[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    walk([&](float4 q) {
      const float ax = (q.x - p.x) / nf, ay = (q.y - p.y) / nf, az = (q.z - p.z) / nf;
      const float av[3] = {ax, ay, az};
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) cov[i][j] = cov[i][j] + av[i] * av[j];
    });
    double n[3];
    smallest_eigvec(cov, n);
    const double dp = (n[0] * (double)p.x + n[1] * (double)p.y) + n[2] * (double)p.z;
    if (dp > 0) {
      n[0] = -n[0];
      n[1] = -n[1];
      n[2] = -n[2];
    }
    out = make_float4((float)n[0], (float)n[1], (float)n[2], 1.0f);  // w = 1: normal found
  }
  nrm_slots[(size_t)r * a.cap_pl + slot] = out;
  return out.w != 0.f ? 1 : 0;
}

// find_closest + compute_normal for one scan line in one workgroup (C <= 2048):
// rows r-1, r, r+1 (float4) and the planar masks of r+-1 are staged in LDS, so the
// argmin scans and the neighbour walks read LDS instead of chains of dependent
// global loads.  Same semantics as k_closest + k_fit (which serve wider rows):
//   closest: one wave per selected point, own 64-column block first, then every
//            block whose AABB lower bound (shrunk 1e-5) does not exceed the best;
//   fit:     one lane per selected point, the reference's neighbour push order.
// The row's found-normal count is stored directly (one block per row).
constexpr int kNrmThreads = 1024;
constexpr int kNrmMaxC = 2048;

template <int KC>
__global__ __launch_bounds__(kNrmThreads) void k_normals(const float4* __restrict__ scan,
                                                         const uint8_t* __restrict__ mask,
                                                         const uint32_t* __restrict__ sel_slots,
                                                         const uint32_t* __restrict__ row_counts, ExArgs a,
                                                         float4* __restrict__ nrm_slots,
                                                         uint32_t* __restrict__ row_ok) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int C = a.C, R = a.R, r = blockIdx.x, k = KC > 0 ? KC : a.k;
  const int half = blockIdx.y;  // two workgroups per line split its selected points
  const int nblk = (C + kWave - 1) / kWave;
  // rows r-1, r, r+1; in rows r+-1 the pad component .w holds the planar mask (1/0).
  // One float4 of padding per 64 columns (px): column jj of different 64-column
  // blocks then falls in different LDS banks (blocks would otherwise be 1 KB apart).
  const int CP = C + (C >> 6) + 1;
  auto px = [](int j) { return j + (j >> 6); };
  float4* s_row = reinterpret_cast<float4*>(smem);          // [3][CP]
  float4* s_lo = s_row + 3 * CP;                            // [2][nblk]
  float4* s_hi = s_lo + 2 * nblk;                           // [2][nblk]
  int2* s_cl = reinterpret_cast<int2*>(s_hi + 2 * nblk);    // [cap_pl] closest columns in r-1 / r+1
  unsigned long long* s_best = reinterpret_cast<unsigned long long*>(s_cl + a.cap_pl);  // [cap_pl]
  uint32_t* s_items = reinterpret_cast<uint32_t*>(s_best + a.cap_pl);                   // [cap_pl * nblk]
  int* s_col = reinterpret_cast<int*>(s_items + (size_t)a.cap_pl * nblk);              // [cap_pl] selected columns
  const int tid = threadIdx.x;
  __shared__ int s_found;
  __shared__ int s_nitems;
  if (tid == 0) s_found = 0;
#ifdef FMX_NRM_TIMING
  uint64_t ts[5], tp[12];
  int ntp = 0;
  ts[0] = wall_clock64();
#endif
  for (int s = 0; s < 3; ++s) {
    const int rr = r - 1 + s;
    if (rr < 0 || rr >= R) continue;
    const float4* src = scan + (size_t)rr * C;
    const uint8_t* msk = mask + (size_t)rr * C;
    for (int c = tid; c < C; c += kNrmThreads) {
      float4 q = src[c];
      if (s != 1) q.w = msk[c] ? 1.f : 0.f;
      s_row[s * CP + px(c)] = q;
    }
  }
  __syncthreads();
#ifdef FMX_NRM_TIMING
  ts[1] = wall_clock64();
#endif
  // AABBs of the planar-valid points per 64-column block of rows r-1 / r+1: 16
  // threads per block, 4 columns each, then a 16-lane min/max (empty: lo = +inf,
  // hi = -inf); the selected columns of row r go to LDS meanwhile
  const int nsel_all = (int)row_counts[2 * r];
  const int hs = (nsel_all + 1) / 2;
  const int s_beg = half * hs, nsel = min(nsel_all, s_beg + hs);  // this block: slots [s_beg, nsel)
  for (int s = s_beg + tid; s < nsel; s += kNrmThreads) s_col[s] = (int)sel_slots[(size_t)r * a.cap_pl + s];
  for (int t0 = 0; t0 < 2 * nblk * 16; t0 += kNrmThreads) {
    const int t = t0 + tid;
    const int wb = t / 16, part = t % 16;
    float lx = INFINITY, ly = INFINITY, lz = INFINITY, hx = -INFINITY, hy = -INFINITY, hz = -INFINITY;
    if (wb < 2 * nblk) {
      const int d = wb / nblk, bk = wb % nblk;
      const int rr = d == 0 ? r - 1 : r + 1;
      if (rr >= 0 && rr < R) {
        const float4* row = s_row + (d == 0 ? 0 : 2) * CP;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int jcol = bk * kWave + part * 4 + u;
          if (jcol < C) {
            const float4 q = row[px(jcol)];
            if (q.w != 0.f) {
              lx = fminf(lx, q.x);
              ly = fminf(ly, q.y);
              lz = fminf(lz, q.z);
              hx = fmaxf(hx, q.x);
              hy = fmaxf(hy, q.y);
              hz = fmaxf(hz, q.z);
            }
          }
        }
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      lx = fminf(lx, __shfl_xor(lx, o, 16));
      ly = fminf(ly, __shfl_xor(ly, o, 16));
      lz = fminf(lz, __shfl_xor(lz, o, 16));
      hx = fmaxf(hx, __shfl_xor(hx, o, 16));
      hy = fmaxf(hy, __shfl_xor(hy, o, 16));
      hz = fmaxf(hz, __shfl_xor(hz, o, 16));
    }
    if (wb < 2 * nblk && part == 0) {
      s_lo[wb] = make_float4(lx, ly, lz, 0.f);
      s_hi[wb] = make_float4(hx, hy, hz, 0.f);
    }
  }
  __syncthreads();
#ifdef FMX_NRM_TIMING
  ts[2] = wall_clock64();
#endif
  // find_closest (:402-420) over rows r-1 / r+1, the whole workgroup per row: the
  // argmin over a candidate's points is an LDS atomicMin of the key (fp32 distance
  // bits << 32 | column) — distances are >= 0, so the key orders like the reference
  // (smaller distance, then first index).  Phase 1: the candidate's own 64-column
  // block; phase 2: list every other block whose AABB lower bound (shrunk 1e-5) does
  // not exceed that best (conservative: the final best can only be smaller); phase
  // 3: the listed blocks.  Exact, with three barriers per row instead of a serial
  // chain per candidate.
#pragma unroll 1
  for (int d = 0; d < 2; ++d) {
    const int rr = d == 0 ? r - 1 : r + 1;
    const bool have = rr >= 0 && rr < R;
    const float4* row = s_row + (d == 0 ? 0 : 2) * CP;
    for (int s = s_beg + tid; s < nsel; s += kNrmThreads) s_best[s] = ~0ull;
    if (tid == 0) s_nitems = 0;
    __syncthreads();
#ifdef FMX_NRM_TIMING
    tp[ntp < 12 ? ntp++ : 11] = wall_clock64();
#endif
    // key of column j for query p (~0 when not a candidate); one thread folds its
    // columns in a register and issues a single atomicMin per candidate
    auto key = [&](const float4& p, int j) -> unsigned long long {
      const float4 q = row[px(j)];
      const float dd = dist2f(q, p);
      if (q.w == 0.f || !(dd <= FLT_MAX)) return ~0ull;  // reference: double(d) < DBL_MAX
      return ((unsigned long long)__float_as_uint(dd) << 32) | (unsigned)j;
    };
    // work items are laid out candidate-fastest so the lanes of a wave update
    // different candidates' keys (no same-address LDS atomics within a wave)
    // threads = 256 candidate lanes x 4 column groups (no runtime divisions)
    const int tl = tid & 255, tg = tid >> 8;
    if (have) {
      for (int s = s_beg + tl; s < nsel; s += 256) {
        const int c = s_col[s];
        const float4 p = s_row[CP + px(c)];
        const int j0 = (c / kWave) * kWave;
        unsigned long long kb = ~0ull;
#pragma unroll 4
        for (int jj = tg; jj < kWave; jj += 4)
          if (j0 + jj < C) kb = min(kb, key(p, j0 + jj));
        if (kb != ~0ull) atomicMin(&s_best[s], kb);
      }
    }
    __syncthreads();
#ifdef FMX_NRM_TIMING
    tp[ntp < 12 ? ntp++ : 11] = wall_clock64();
#endif
    if (have) {
      const int nsr = (nsel - s_beg + 255) & ~255;  // whole 256-lane rounds: ballots see full waves
      for (int sb = 0; sb < nsr * ((nblk + 3) / 4); sb += 256) {
        const int s = s_beg + (sb % nsr) + tl, bk = (sb / nsr) * 4 + tg;
        bool keep = false;
        if (s < nsel && bk < nblk) {
          const int c = s_col[s];
          const float4 lo = s_lo[d * nblk + bk], hi = s_hi[d * nblk + bk];
          if (bk != c / kWave && lo.x <= hi.x) {  // not the own block, not empty
            // fp32 bound: pruning only has to be conservative, and the 1e-5 shrink
            // dwarfs the few-ulp fp32 error of the bound and of the distances
            const float4 p = s_row[CP + px(c)];
            const float ex = fmaxf(fmaxf(lo.x - p.x, p.x - hi.x), 0.f);
            const float ey = fmaxf(fmaxf(lo.y - p.y, p.y - hi.y), 0.f);
            const float ez = fmaxf(fmaxf(lo.z - p.z, p.z - hi.z), 0.f);
            const float lb = (ex * ex + ey * ey + ez * ez) * (1.f - 1e-5f);
            const unsigned long long b = s_best[s];
            keep = b == ~0ull || lb <= __uint_as_float((uint32_t)(b >> 32));
          }
        }
        const uint64_t m = __ballot(keep);  // one counter add per wave
        int base = 0;
        if (lane_id() == 0 && m) base = atomicAdd(&s_nitems, __popcll(m));
        base = __shfl(base, 0, 64);
        if (keep) s_items[base + __popcll(m & lanemask_lt())] = (uint32_t)(s * 64 + bk);  // nblk <= 32
      }
    }
    __syncthreads();
#ifdef FMX_NRM_TIMING
    tp[ntp < 12 ? ntp++ : 11] = wall_clock64();
#endif
    const int nitems = s_nitems;

    for (int q = tl; q < nitems; q += 256) {
      const uint32_t it = s_items[q];
      const int s = (int)(it >> 6), bk = (int)(it & 63);
      const float4 p = s_row[CP + px(s_col[s])];
      unsigned long long kb = ~0ull;
#pragma unroll 4
      for (int jj = tg; jj < kWave; jj += 4)
        if (bk * kWave + jj < C) kb = min(kb, key(p, bk * kWave + jj));
      if (kb != ~0ull) atomicMin(&s_best[s], kb);
    }
    __syncthreads();
#ifdef FMX_NRM_TIMING
    tp[ntp < 12 ? ntp++ : 11] = wall_clock64();
#endif
    for (int s = s_beg + tid; s < nsel; s += kNrmThreads) {
      const unsigned long long b = s_best[s];
      const int col = b == ~0ull ? -1 : (int)(uint32_t)b;
      if (d == 0) s_cl[s].x = col;
      else s_cl[s].y = col;
    }
  }
  __syncthreads();
#ifdef FMX_NRM_TIMING
  ts[3] = wall_clock64();
#endif
  // compute_normal (:263-329), one lane per selected point; points addressed as
  // (LDS row 0/1/2, column): every walk stays inside its row (valid columns lie in
  // [k, C-k) and the walk is at most k long)
  int found = 0;
  for (int slot = s_beg + tid; slot < nsel; slot += kNrmThreads) {
    const int c = s_col[slot];
    const float4 p = s_row[CP + px(c)];
    const int2 cl = s_cl[slot];
    const double r2 = a.radius2;
    auto walk = [&](auto&& visit) {
      auto nbrs = [&](const float4* row, int j) {  // find_neighbors (:422-448)
        const float4 pj = row[px(j)];
        for (int i = 1; i <= k; ++i) {
          const float4 q = row[px(j + i)];
          if ((double)dist2f(q, pj) < r2) visit(q);
          else break;
        }
        for (int i = 1; i <= k; ++i) {
          const float4 q = row[px(j - i)];
          if ((double)dist2f(q, pj) < r2) visit(q);
          else break;
        }
      };
      nbrs(s_row + CP, c);
      if (cl.x >= 0) {
        visit(s_row[px(cl.x)]);
        nbrs(s_row, cl.x);
      }
      if (cl.y >= 0) {
        visit(s_row[2 * CP + px(cl.y)]);
        nbrs(s_row + 2 * CP, cl.y);
      }
    };
    int cnt = 0;
    walk([&](float4) { ++cnt; });
    float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((cl.x >= 0 || cl.y >= 0) && cnt >= a.min_points) {
      const float nf = (float)cnt;
      float cov[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
      walk([&](float4 q) {
        const float ax = (q.x - p.x) / nf, ay = (q.y - p.y) / nf, az = (q.z - p.z) / nf;
        const float av[3] = {ax, ay, az};
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int jj = 0; jj < 3; ++jj) cov[i][jj] = cov[i][jj] + av[i] * av[jj];
      });
      double n[3];
      smallest_eigvec(cov, n);
      const double dp = (n[0] * (double)p.x + n[1] * (double)p.y) + n[2] * (double)p.z;
      if (dp > 0) {
        n[0] = -n[0];
        n[1] = -n[1];
        n[2] = -n[2];
      }
      out = make_float4((float)n[0], (float)n[1], (float)n[2], 1.0f);  // w = 1: normal found
      ++found;
    }
    nrm_slots[(size_t)r * a.cap_pl + slot] = out;
  }
  if (found) atomicAdd(&s_found, found);
  __syncthreads();
  if (tid == 0) row_ok[2 * r + half] = (uint32_t)s_found;  // k_row_scan adds the pair
#ifdef FMX_NRM_TIMING
  ts[4] = wall_clock64();
  if (tid == 0 && half == 0 && (r == 5 || r == 64 || r == 100))
    printf("nrm row %d nsel %d: load %d aabb %d closest %d fit %d | %d %d %d %d %d %d %d %d\n", r, nsel,
           (int)(ts[1] - ts[0]), (int)(ts[2] - ts[1]), (int)(ts[3] - ts[2]), (int)(ts[4] - ts[3]), (int)(tp[0] - ts[2]),
           (int)(tp[1] - tp[0]), (int)(tp[2] - tp[1]), (int)(tp[3] - tp[2]), (int)(tp[4] - tp[3]), (int)(tp[5] - tp[4]),
           (int)(tp[6] - tp[5]), (int)(tp[7] - tp[6]));
#endif
}

// per-row offsets of {planar with normal, points, planar selected}: one block
__global__ __launch_bounds__(1024) void k_row_scan(const uint32_t* row_counts, const uint32_t* row_ok, int R,
                                                   uint32_t* row_off /* [3][R+1] */, uint32_t* host_totals,
                                                   uint32_t* flag, uint32_t seq) {
  __shared__ uint32_t ws[16];
  __shared__ uint32_t carry[3];
  if (threadIdx.x < 3) carry[threadIdx.x] = 0;
  __syncthreads();
  for (int r0 = 0; r0 < R; r0 += 1024) {
    const int r = r0 + threadIdx.x;
    for (int t = 0; t < 3; ++t) {
      uint32_t v = 0;
      if (r < R) v = t == 0 ? row_ok[2 * r] + row_ok[2 * r + 1] : (t == 1 ? row_counts[2 * r + 1] : row_counts[2 * r]);
      const uint32_t incl = wave_incl_scan(v);
      const int w = threadIdx.x / kWave;
      if (lane_id() == 63) ws[w] = incl;
      __syncthreads();
      uint32_t off = 0, tot = 0;
      for (int i = 0; i < 16; ++i) {
        if (i < w) off += ws[i];
        tot += ws[i];
      }
      if (r < R) row_off[t * (R + 1) + r] = carry[t] + off + incl - v;
      __syncthreads();
      if (threadIdx.x == 0) carry[t] += tot;
      __syncthreads();
    }
  }
  if (threadIdx.x < 3) {
    row_off[threadIdx.x * (R + 1) + R] = carry[threadIdx.x];
    host_store(host_totals + threadIdx.x, carry[threadIdx.x]);  // mapped host memory: no copy op
  }
  if (threadIdx.x == 0) publish_flag(flag, seq);  // lanes 0-2 of this wave stored the totals
}

// ordered compaction of row slots into the query arrays (block per row)
__global__ __launch_bounds__(256) void k_write_features(const float4* __restrict__ scan, ExArgs a,
                                                        const uint32_t* __restrict__ row_counts,
                                                        const uint32_t* __restrict__ row_off,
                                                        const uint32_t* __restrict__ sel_slots,
                                                        const uint32_t* __restrict__ pt_slots,
                                                        const float4* __restrict__ nrm_slots,
                                                        float4* __restrict__ pl_pos, float4* __restrict__ pl_nrm,
                                                        uint32_t* __restrict__ pl_idx,
                                                        float4* __restrict__ pt_pos, uint32_t* __restrict__ pt_idx) {
  __shared__ int ws[4];
  const int r = blockIdx.x, tid = threadIdx.x, w = tid / kWave;
  const int R = a.R, C = a.C;
  const uint32_t nsel = row_counts[2 * r], npt = row_counts[2 * r + 1];
  uint32_t base = row_off[r];
  for (uint32_t s0 = 0; s0 < nsel; s0 += 256) {
    const uint32_t s = s0 + tid;
    const bool ok = s < nsel && nrm_slots[(size_t)r * a.cap_pl + s].w != 0.f;
    const uint64_t m = __ballot(ok);
    if (lane_id() == 0) ws[w] = __popcll(m);
    __syncthreads();
    uint32_t off = base, tot = 0;
    for (int i = 0; i < 4; ++i) {
      if (i < w) off += ws[i];
      tot += ws[i];
    }
    if (ok) {
      const uint32_t o = off + __popcll(m & lanemask_lt());
      const uint32_t idx = (uint32_t)r * C + sel_slots[(size_t)r * a.cap_pl + s];
      const float4 p = scan[idx];
      const float4 n = nrm_slots[(size_t)r * a.cap_pl + s];
      pl_pos[o] = make_float4(p.x, p.y, p.z, 0.f);
      pl_nrm[o] = make_float4(n.x, n.y, n.z, 0.f);
      pl_idx[o] = idx;
    }
    __syncthreads();
    base += tot;
  }
  const uint32_t pbase = row_off[(R + 1) + r];
  for (uint32_t s = tid; s < npt; s += 256) {
    const uint32_t idx = (uint32_t)r * C + pt_slots[(size_t)r * a.cap_pt + s];
    const float4 p = scan[idx];
    pt_pos[pbase + s] = make_float4(p.x, p.y, p.z, 0.f);
    pt_idx[pbase + s] = idx;
  }
}

}  // namespace

namespace {
// A host scan DMA'd as packed x, y, z (stage.hpp pack3: a PointXYZf's pad is always 0,
// utils.hpp:38-46, and no kernel reads it) back in the float4 layout the extraction
// reads: one lane per point, three dword loads (a wave reads 768 contiguous bytes each).
__global__ __launch_bounds__(256) void k_unpack_xyz(const float* __restrict__ p3, float4* __restrict__ out, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = make_float4(p3[3 * (size_t)i], p3[3 * (size_t)i + 1], p3[3 * (size_t)i + 2], 0.0f);
}
}  // namespace

void unpack_xyz(fmx_ctx* c, const float* d_packed, float4* d_out, size_t n, hipStream_t st) {
  if (!n) return;
  ProfScope ps(c->prof, PROF_UNPACK, 28.0 * n, st);
  hipLaunchKernelGGL(k_unpack_xyz, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, d_packed, d_out, (uint32_t)n);
  FMX_HIP(hipGetLastError());
}

// The arguments and scratch of one extraction (every buffer ensured before any launch:
// a regrowth's hipFree synchronizes the device).
static ExArgs extract_setup(fmx_ctx* c, int R, int C) {
  const auto& E = c->P.extraction;
  ExArgs a;
  a.R = R;
  a.C = C;
  a.k = (int)E.neighbor_points;
  a.S = (int)E.num_sectors;
  a.P = (int)E.planar_feats_per_sector;
  a.Ppt = (int)E.point_feats_per_sector;
  a.row0 = 0;
  a.cap_pl = a.S * (a.P + 1);
  a.cap_pt = a.k > 0 ? C / a.k + 1 : C;
  a.thr = E.planar_threshold;
  a.min2 = E.min_norm_squared;
  a.max2 = E.max_norm_squared;
  a.radius2 = E.radius * E.radius;
  a.min_points = (int)E.min_points;
  const size_t N = (size_t)R * C;
  c->planar_mask.ensure(N);
  c->sel_slots.ensure((size_t)R * a.cap_pl);
  c->pt_slots.ensure((size_t)R * a.cap_pt);
  c->row_counts.ensure(2 * (size_t)R);
  c->row_ok.ensure(2 * (size_t)R);  // found normals per line: [2r] + [2r+1]
  c->row_off.ensure(3 * ((size_t)R + 1));
  c->closest.ensure((size_t)R * a.cap_pl);
  c->nrm_slots.ensure((size_t)R * a.cap_pl);
  c->rows = R;
  c->cols = C;
  if (!c->lds_attr_set) {
    const int lmax = 4096 * (16 + 4 + 4 + 4 + 4);
    const void* kern[4] = {reinterpret_cast<const void*>(k_extract_rows<5, false>),
                           reinterpret_cast<const void*>(k_extract_rows<0, false>),
                           reinterpret_cast<const void*>(k_extract_rows<5, true>),
                           reinterpret_cast<const void*>(k_extract_rows<0, true>)};
    for (const void* kf : kern) FMX_HIP(hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, lmax));
    c->lds_attr_set = true;
  }
  return a;
}

// k_extract_rows over rows [r0, r1) (one 1024-thread block per line).
static void launch_rows(fmx_ctx* c, const float4* d_scan, ExArgs a, int r0, int r1, hipStream_t st) {
  if (r1 <= r0) return;
  const int R = a.R, C = a.C;
  const size_t N = (size_t)R * C;
  const size_t lds = (size_t)C * (16 + 4 + 4 + 4 + 4);
  // sector-parallel selection when every sector sorts in one wave's registers (<= 512
  // columns), there is a wave per sector, sectors are longer than the suppression
  // reach, and the kept lists fit the dead point area of LDS
  const int pps = C / a.S;
  const size_t nwd = (size_t)(C + 63) / 64 + 1;
  const bool par = pps <= 512 && a.S <= 16 && pps >= 2 * a.k &&
                   8 * (size_t)C + 8 * nwd + 2 * 4 * (size_t)a.S * (a.P + 1) <= 16 * (size_t)C;
  a.row0 = r0;
  const dim3 grid(r1 - r0);
  ProfScope ps(c->prof, PROF_EXTRACT_ROWS, (16.0 * N + N) * (r1 - r0) / R, st);
  if (par) {
    if (a.k == 5)
      hipLaunchKernelGGL((k_extract_rows<5, true>), grid, dim3(kRowThreads), lds, st, d_scan, a, c->planar_mask.p,
                         c->sel_slots.p, c->pt_slots.p, c->row_counts.p);
    else
      hipLaunchKernelGGL((k_extract_rows<0, true>), grid, dim3(kRowThreads), lds, st, d_scan, a, c->planar_mask.p,
                         c->sel_slots.p, c->pt_slots.p, c->row_counts.p);
  } else {
    if (a.k == 5)
      hipLaunchKernelGGL((k_extract_rows<5, false>), grid, dim3(kRowThreads), lds, st, d_scan, a, c->planar_mask.p,
                         c->sel_slots.p, c->pt_slots.p, c->row_counts.p);
    else
      hipLaunchKernelGGL((k_extract_rows<0, false>), grid, dim3(kRowThreads), lds, st, d_scan, a, c->planar_mask.p,
                         c->sel_slots.p, c->pt_slots.p, c->row_counts.p);
  }
  FMX_HIP(hipGetLastError());
}

ExLaunch extract_launch(fmx_ctx* c, const float4* d_scan, int R, int C, hipStream_t st, uint32_t* tot_h,
                        uint32_t* tot_d, uint32_t* flag_h, uint32_t* flag_d, uint32_t seq) {
  ExArgs a = extract_setup(c, R, C);
  launch_rows(c, d_scan, a, 0, R, st);
  a.row0 = 0;
  const size_t N = (size_t)R * C;
  const int nslots = R * a.cap_pl;
  const int nblk = (C + 63) / 64;
  // k_normals: one workgroup per line, rows r-1..r+1 in LDS (160 KB per CU, minus
  // the kernel's few static bytes)
  const size_t lds_n = (size_t)3 * (C + (C >> 6) + 1) * 16 + (size_t)4 * nblk * 16 + (size_t)a.cap_pl * 20 +
                       (size_t)a.cap_pl * nblk * 4;
  constexpr size_t kNrmLdsMax = 160 * 1024 - 256;
  if (C <= kNrmMaxC && lds_n <= kNrmLdsMax) {
    if (!c->nrm_attr_set) {
      FMX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_normals<5>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kNrmLdsMax));
      FMX_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_normals<0>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kNrmLdsMax));
      c->nrm_attr_set = true;
    }
    ProfScope ps(c->prof, PROF_FIT, 48.0 * N + 2.0 * N + 16.0 * nslots, st);
    if (a.k == 5)
      hipLaunchKernelGGL(k_normals<5>, dim3(R, 2), dim3(kNrmThreads), lds_n, st, d_scan, c->planar_mask.p, c->sel_slots.p,
                         c->row_counts.p, a, c->nrm_slots.p, c->row_ok.p);
    else
      hipLaunchKernelGGL(k_normals<0>, dim3(R, 2), dim3(kNrmThreads), lds_n, st, d_scan, c->planar_mask.p, c->sel_slots.p,
                         c->row_counts.p, a, c->nrm_slots.p, c->row_ok.p);
    FMX_HIP(hipGetLastError());
  } else {
    FMX_HIP(hipMemsetAsync(c->row_ok.p, 0, 2 * R * sizeof(uint32_t), st));
    c->blk_lo.ensure((size_t)R * nblk);
    c->blk_hi.ensure((size_t)R * nblk);
    {
      ProfScope ps(c->prof, PROF_CLOSEST, 16.0 * N + N + 8.0 * nslots, st);
      hipLaunchKernelGGL(k_row_blocks, dim3((R * nblk + 3) / 4), dim3(256), 0, st, d_scan, c->planar_mask.p, R, C,
                         c->blk_lo.p, c->blk_hi.p);
      hipLaunchKernelGGL(k_closest, dim3((nslots + 3) / 4), dim3(256), 0, st, d_scan, c->planar_mask.p,
                         c->sel_slots.p, c->row_counts.p, R, C, a.cap_pl, c->blk_lo.p, c->blk_hi.p, c->closest.p);
    }
    {
      ProfScope ps(c->prof, PROF_FIT, 0.0, st);
      hipLaunchKernelGGL(k_fit, dim3((a.cap_pl + 255) / 256, R), dim3(256), 0, st, d_scan, c->sel_slots.p,
                         c->row_counts.p, c->closest.p, a, c->nrm_slots.p, c->row_ok.p);
    }
  }
  {
    ProfScope ps(c->prof, PROF_COMPACT, 0.0, st);
    hipLaunchKernelGGL(k_row_scan, dim3(1), dim3(1024), 0, st, c->row_counts.p, c->row_ok.p, R, c->row_off.p,
                       tot_d, flag_d, seq);
  }
  FMX_HIP(hipGetLastError());
  // k_write_features needs only the device row offsets, and its outputs are sized for
  // the worst case (so a wrong total can never become an out-of-bounds write): it is
  // queued before the host blocks on the totals (written to mapped host memory by
  // k_row_scan), and so is any independent work of the caller (register_scan: the
  // map build on the side stream)
  const size_t max_pl = (size_t)R * a.cap_pl, max_pt = (size_t)R * a.cap_pt;
  c->q_pl_pos.ensure(max_pl + 1);
  c->q_pl_nrm.ensure(max_pl + 1);
  c->q_pl_idx.ensure(max_pl + 1);
  c->q_pt_pos.ensure(max_pt + 1);
  c->q_pt_idx.ensure(max_pt + 1);
  {
    ProfScope ps(c->prof, PROF_COMPACT, 32.0 * c->n_qpl + 16.0 * c->n_qpt, st);  // byte model: last totals
    hipLaunchKernelGGL(k_write_features, dim3(R), dim3(256), 0, st, d_scan, a, c->row_counts.p, c->row_off.p,
                       c->sel_slots.p, c->pt_slots.p, c->nrm_slots.p, c->q_pl_pos.p, c->q_pl_nrm.p,
                       c->q_pl_idx.p, c->q_pt_pos.p, c->q_pt_idx.p);
  }
  FMX_HIP(hipGetLastError());
  ExLaunch L;
  L.seq = seq;
  L.flag = flag_h;
  L.tot = tot_h;
  L.max_pl = max_pl;
  L.max_pt = max_pt;
  L.st = st;
  return L;
}

void extract_collect(fmx_ctx* c, const ExLaunch& L, fmx_feature_counts* out) {
  wait_flag(c, L.flag, L.seq, L.st);
  const uint32_t npl = L.tot[0], npt = L.tot[1], nsel = L.tot[2];
  if (npl > L.max_pl || npt > L.max_pt || nsel > L.max_pl) throw StatusError(FMX_E_HIP, "implausible feature totals");
  c->n_qpl = npl;
  c->n_qpt = npt;
  c->n_sel = nsel;
  if (out) {
    out->planar = npl;
    out->point = npt;
    out->planar_selected = nsel;
  }
}

void run_extract(fmx_ctx* c, const float4* d_scan, int R, int C, fmx_feature_counts* out,
                 const std::function<void()>& while_waiting) {
  c->h_u32.ensure(8);
  const uint32_t seq = next_flag(c);
  const ExLaunch L = extract_launch(c, d_scan, R, C, c->stream, c->h_u32.p, c->h_u32.d, c->h_flag.p, c->h_flag.d, seq);
  if (while_waiting) while_waiting();
  extract_collect(c, L, out);
}

}  // namespace fmx
