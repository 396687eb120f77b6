// voxelmap.hip — stage 2: device voxel-hash submap and nearest-neighbour matching.
//
// Replaces tsl::robin_map<Vector3i, std::vector<Point>> (form/mapping/map.hpp:66-94)
// and the TBB matcher (form/optimization/matcher.hpp:67-112):
//   build  : KeypointMap::to_voxel_map (map.tpp:128-146) — transform every window
//            keypoint to the world frame (double), insert its voxel key
//            floor(p / w) (map.tpp:35-38) into an open-addressed table (atomic CAS,
//            linear probing, load <= 0.5), count per voxel, exclusive-scan the
//            counts, scatter records voxel-contiguously.  One 16-B probe yields
//            {key, first, count}.
//   match  : VoxelMap::find_closest (map.tpp:70-91) — the 27 neighbour voxels,
//            squared distance (dx*dx + dz*dz) + dy*dy in double; ties broken by the
//            record's build order (the reference keeps the first in shift/insertion
//            order; identical except for exact distance ties, parity hazard 10).
//            Voxels whose box lies farther than the acceptance bound are skipped:
//            only d^2 < max_dist^2 (acceptance, matcher.hpp:103-105) and
//            d^2 > min_dist_map^2 (insertion, map.tpp:160-163) are observable, and
//            with w = max_dist_matching every point within that bound lies in the
//            27 voxels, so the decisions equal the reference's.
//   pairs  : bucketing per map scan (matcher.hpp:103-111) as a stable counting sort
//            (block histograms -> offsets -> ranked scatter) into pair-major SoA.
//   insert : KeypointMap::insert_matches (map.tpp:148-165) as an ordered compaction.
#include "fmx_device.hpp"
#include "fmx_internal.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#ifndef FMX_VM_NS
#define FMX_VM_NS g8
#endif
#ifndef FMX_DENSE_MIN
#define FMX_DENSE_MIN 128
#endif
#ifndef FMX_SUB_AXIS
#define FMX_SUB_AXIS 4
#endif
#ifndef FMX_MATCH_WAVES
#define FMX_MATCH_WAVES 4  // waves per SIMD k_match is compiled for (register budget 128)
#endif
#ifndef FMX_MATCH_WAVES_PLAIN
#if defined(FMX_MATCH_GROUP) && FMX_MATCH_GROUP == 1
#define FMX_MATCH_WAVES_PLAIN 7  // ... without the dense-cell walk, one lane per query (71 VGPRs;
                                 // C5 match 0.243 -> 0.230 ms per launch, 8 waves spill)
#else
#define FMX_MATCH_WAVES_PLAIN 6  // ... and without the dense-cell walk (register budget 80)
#endif
#endif
#ifndef FMX_MATCH_DEPTH_PLAIN
#if defined(FMX_MATCH_GROUP) && FMX_MATCH_GROUP == 1
#define FMX_MATCH_DEPTH_PLAIN 1  // ... one lane per query (C5): two in flight spilled a record per
                                 // candidate to scratch at 7 waves (48 B of scratch traffic per query,
                                 // ~95 MB per whole-map launch); one: whole-map launch 0.754 -> 0.698 ms
                                 // per registration, local 0.805 -> 0.774 (profiles/r5_c5_ab.txt)
#else
#define FMX_MATCH_DEPTH_PLAIN 2  // record loads in flight per lane without the dense-cell walk
#endif
#endif
#ifndef FMX_MATCH_WAVES_FUSED
#define FMX_MATCH_WAVES_FUSED FMX_MATCH_WAVES_PLAIN  // ... the fused match + linearization (C5)
#endif
#define FMX_MATCH_ATTR                                                                                        \
  __attribute__((amdgpu_waves_per_eu(DENSE ? FMX_MATCH_WAVES : (FUSED ? FMX_MATCH_WAVES_FUSED : FMX_MATCH_WAVES_PLAIN), \
                                     8)))
#ifndef FMX_MATCH_DEPTH
#define FMX_MATCH_DEPTH 4
#endif

#ifndef FMX_CERT_DIAG
#define FMX_CERT_DIAG 0  // diagnostic build (with FMX_WARM_CERT=0): count the warm queries a certificate settles
#endif
#ifndef FMX_WARM_CERT
#define FMX_WARM_CERT 1  // warm queries whose certificate holds skip the search (A/B switch;
                         // an FMX_CERT_DIAG build sets it to 0 so that every query is searched)
#endif
#define FMX_CERT_ANY (FMX_CERT_DIAG || FMX_WARM_CERT)
#ifndef FMX_TAIL_ONEPASS
#define FMX_TAIL_ONEPASS 1  // the match's last block: all its scans in one round of loads (A/B switch)
#endif

namespace fmx {
// This file is compiled twice (Makefile): FMX_MATCH_GROUP 8 -> fmx::g8 and 1 -> fmx::gl;
// run_match picks one per launch (fmx_api.cpp, match_group_for).
namespace FMX_VM_NS {
namespace {

__device__ __forceinline__ int find_seg(const Seg* segs, int K, uint32_t rec) {
  int lo = 0, hi = K - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].off <= rec) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Both feature types in one launch (the fused VoxMap layout, fmx_internal.hpp):
// record rec < n0 is planar record rec, else point record rec - n0; each type has its
// own table section (point bricks at off1) and segment list.
//
// The build (map.tpp:128-146 + push_back :41-52), five launches, no table clear:
//   k_map_insert  one lane per record: world transform, voxel key; the first lane of the
//                 wave's records of one brick finds or claims the brick (epoch-tagged CAS,
//                 linear probing); a claimed brick's claim slot is its claimer's record
//                 index, written into the brick with the slot's cell counts zeroed; every
//                 record notes its brick and cell
//   k_map_count   one lane per record: the brick's claim slot, one count atomic per
//                 (wave, cell) group on the slot's counts (the returned count is the
//                 record's rank in the cell)
//   k_map_alloc   four claim slots per lane: the cells' record ranges (block scan + one
//                 atomic per block and type) into the brick and, with the header slots of
//                 a dense cell added, over the slot's counts (the scatter's bases)
//   k_map_scatter one lane per record: the record at its cell's base + rank
//   k_map_dense   one block per dense cell (> kDenseMin records): counting sort of
//                 its records into 4 x 4 x 4 sub-cells, header = the sub-cell ends
// Claim slots are listed in insertion order: consecutive records are mostly neighbours, so the counts,
// the ranges and the scatter's bases are read and written near one another instead of
// at the table's hashed positions, and the scatter reads no brick (20.6 GB
// per 50M-record build with per-bucket counts, their random lines and the scatter's
// brick reads a large share of it).
// The order of records inside a cell (and of the cells' ranges) follows the atomics,
// so it varies from build to build; nothing observable depends on it: k_match's
// argmin is over the total order (d^2, reference shift rank, build order).
struct BuildState {  // per build, two alternating copies (the other is cleared)
  uint32_t nclaim;   // (unused: claim slots are record indices)
  uint32_t cur[2];   // record slot cursors (planar from 0, point from BuildArgs::pt_base)
  uint32_t err;      // range error: a record outside the packable key range
  uint32_t ndense;   // dense cells
  uint32_t pad[3];
};
constexpr int kDenseMin = FMX_DENSE_MIN;  // records that make a cell dense
constexpr int kSubPerAxis = FMX_SUB_AXIS;  // dense cells: 4 x 4 x 4 sub-cells of w / 4
constexpr int kSubCells = kSubPerAxis * kSubPerAxis * kSubPerAxis;
constexpr int kHdr = (kSubCells * 4 + 31) / 32;  // header slots (double4) holding the u32 sub-cell ends
constexpr int kDenseThreads = 1024;
constexpr int kDenseRecs = 8;             // records per thread: dense cells up to 8192 records are sorted
constexpr uint32_t kUnsorted = 0xFFFFFFFFu;  // header[0] of a dense cell too large to sort
constexpr uint32_t kDenseGrid = 1024;     // k_map_dense blocks (each loops over the dense list)
constexpr int kAllocThreads = 1024;       // k_map_alloc: one cursor atomic per block and type
constexpr uint32_t kNoBrick = 0xFFFFFFFFu;  // a claim slot whose record claimed no brick

struct BuildArgs {
  const float4* pool_pos[2];
  const float4* pool_nrm;  // planar only
  const Seg* segs[2];
  int K;
  const double* poses;
  uint32_t n0, n;  // planar records, all records
  uint32_t pt_base;  // first point slot: planar records + the most header slots they can need
  double w;
  Brick* bricks;
  uint32_t* ccnt;   // [claim slot][8]: cell record counts (insert), then cell bases (alloc)
  uint64_t mask[2];
  uint64_t off1;  // first point brick
  uint32_t epoch;
  uint2* rinfo;     // per record: claim slot * 8 + cell or ~0, rank in the cell
  uint32_t* claim;  // per claim slot (= record index): the brick its record claimed, or kNoBrick
  uint32_t* dense;  // dense cells
  BuildState* st;
  BuildState* st_next;
  unsigned long long* info;  // pinned host word: epoch << 32 | dense cells (k_match<DENSE> choice)
  double4* pos;
  double4* nrm;
  uint32_t rsh;  // record stride: 1 << rsh bytes (5: separate pos / nrm arrays, 6: interleaved)
};

// Record slot i of a record array with stride 1 << rsh bytes.  Small maps keep
// positions and normals in two arrays (32-B stride: a walk over a cell reads 2
// positions per 64-B line); large maps (C5) interleave them (64-B stride, nrm = pos +
// 32 B): a candidate record's line then also holds its normal, so the winner's normal
// costs no second random line (whole-map PMC traffic 1.37x the byte model).
__device__ __forceinline__ double4& rec_at(double4* base, uint32_t i, uint32_t rsh) {
  return *reinterpret_cast<double4*>(reinterpret_cast<char*>(base) + ((size_t)i << rsh));
}
__device__ __forceinline__ const double4& rec_at(const double4* base, uint32_t i, uint32_t rsh) {
  return *reinterpret_cast<const double4*>(reinterpret_cast<const char*>(base) + ((size_t)i << rsh));
}

// world position (and normal) of build-order record rec
struct RecW {
  double p[3], n[3];
  uint32_t seg;
  int t;
};
__device__ __forceinline__ RecW rec_world(const BuildArgs& a, uint32_t rec, bool with_nrm) {
  RecW o;
  o.t = rec < a.n0 ? 0 : 1;
  const uint32_t r = o.t == 0 ? rec : rec - a.n0;
  const Seg* segs = a.segs[o.t];
  const int s = find_seg(segs, a.K, r);
  const Seg sg = segs[s];
  const double* T = a.poses + 12 * s;
  const float4 lp = a.pool_pos[o.t][sg.pool_off + (r - sg.off)];
  d_xform(T, (double)lp.x, (double)lp.y, (double)lp.z, o.p);  // PlanarFeat::transform (features.hpp:137-140)
  if (with_nrm && o.t == 0) {
    const float4 ln = a.pool_nrm[sg.pool_off + (r - sg.off)];
    d_rot(T, (double)ln.x, (double)ln.y, (double)ln.z, o.n);
  }
  o.seg = (uint32_t)s;
  return o;
}

// Lanes of a wave holding equal values, grouped: for each lane (valid ones only) the
// group's first lane and the lane's rank among the group's lanes; that first lane
// also gets the group's size.  One round per distinct value (VALU only), so the
// group's atomics are issued once per group, by its first lane, all groups at once.
__device__ __forceinline__ void wave_group(bool valid, unsigned long long v, int& leader, uint32_t& rank,
                                           uint32_t& size) {
  uint64_t todo = __ballot(valid);
  leader = -1;
  rank = 0;
  size = 0;
  while (todo) {
    const int l = __ffsll((unsigned long long)todo) - 1;
    const unsigned long long lv =
        ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const bool in = valid && v == lv;
    const uint64_t m = __ballot(in);
    if (in) {
      leader = l;
      rank = (uint32_t)__popcll(m & lanemask_lt());
    }
    if (lane_id() == l) size = (uint32_t)__popcll(m);
    todo &= ~m;
  }
}

__global__ __launch_bounds__(256) void k_map_insert(BuildArgs a) {
  const uint32_t rec = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < sizeof(BuildState) / 4)  // the next build's state
    reinterpret_cast<uint32_t*>(a.st_next)[threadIdx.x] = 0u;
  if (blockIdx.x * blockDim.x >= a.n) return;  // (whole waves past the records; the rest stay for the groups)
  bool valid = rec < a.n;
  int cx = 0, cy = 0, cz = 0, t = 0;
  if (valid) {
    const RecW R = rec_world(a, rec, false);
    cx = (int)floor(R.p[0] / a.w), cy = (int)floor(R.p[1] / a.w), cz = (int)floor(R.p[2] / a.w);
    t = R.t;
    if (!key_in_range(cx, cy, cz)) {
      atomicOr(&a.st->err, 1u);
      a.rinfo[rec] = make_uint2(0xFFFFFFFFu, 0u);
      valid = false;
    }
  }
  // records of one brick (consecutive records are mostly neighbours): its first lane
  // probes / claims for the group
  const unsigned long long key = brick_key(cx, cy, cz, a.epoch) ^ (unsigned long long)t << 63;  // (bit 63: type, grouping only)
  int bl;
  uint32_t brank, bsize;
  wave_group(valid, key, bl, brank, bsize);
  const bool prober = valid && brank == 0;
  const unsigned long long bkey = brick_key(cx, cy, cz, a.epoch);
  const uint64_t boff = t == 0 ? 0 : a.off1;
  Brick* bricks = a.bricks + boff;
  const uint64_t mask = a.mask[t];
  uint64_t h = mix64(bkey) & mask;
  bool claimed = false;
  if (prober) {
    for (;;) {  // more buckets than records: a bucket of another epoch always exists
      const unsigned long long cur = __hip_atomic_load(&bricks[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == bkey) break;
      if (key_epoch(cur) != a.epoch) {  // empty for this build: claim it
        const unsigned long long prev = atomicCAS(&bricks[h].key, cur, bkey);
        if (prev == cur) {
          claimed = true;
          break;
        }
        if (prev == bkey) break;
        continue;  // another brick took the bucket: look at it again
      }
      h = (h + 1) & mask;
    }
  }
  // a claimed brick's claim slot is its claimer's record index: no counter (one atomic per
  // wave on a single word serialized the build — C5 insert 9.1 ms for 50M records, C4
  // ~20 us; round 5).  The slot goes into the brick (k_map_count reads it), its cell counts
  // are zeroed, and every record's slot entry says whether it claimed
  if (claimed) {
    bricks[h].slot = rec;
    uint4* cc = reinterpret_cast<uint4*>(a.ccnt + (size_t)rec * 8);
    cc[0] = make_uint4(0, 0, 0, 0);
    cc[1] = make_uint4(0, 0, 0, 0);
  }
  if (rec < a.n) a.claim[rec] = claimed ? (uint32_t)(boff + h) : kNoBrick;
  h = (uint64_t)__shfl((unsigned long long)h, bl < 0 ? 0 : bl, 64);  // the group's bucket
  if (valid) a.rinfo[rec] = make_uint2((uint32_t)((boff + h) * 8 + brick_cell(cx, cy, cz)), 0u);
}

// One lane per record, after k_map_insert (every claimer's slot is in its brick): the
// record's cell in its brick's claim slot, counted with one atomic per (wave, cell) group
// (the returned count is the record's rank in the cell).  Two launches instead of a
// claim lock: a lock held while the claimer fills the slot serialized the waves of
// C4's dense cells (insert 22 -> 113 us, round 5).
__global__ __launch_bounds__(256) void k_map_count(BuildArgs a) {
  const uint32_t rec = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x * blockDim.x >= a.n) return;
  uint2 ri = make_uint2(0xFFFFFFFFu, 0u);
  if (rec < a.n) ri = a.rinfo[rec];
  const bool valid = ri.x != 0xFFFFFFFFu;
  // the wave's records of one cell: its first lane reads the brick's slot and counts
  int cl;
  uint32_t crank, csize;
  wave_group(valid, ri.x, cl, crank, csize);
  uint32_t cell = 0, cbase = 0;
  if (valid && crank == 0) {
    cell = a.bricks[ri.x >> 3].slot * 8 + (ri.x & 7);
    cbase = atomicAdd(a.ccnt + cell, csize);
  }
  cell = (uint32_t)__shfl((int)cell, cl < 0 ? 0 : cl, 64);
  cbase = (uint32_t)__shfl((int)cbase, cl < 0 ? 0 : cl, 64);
  if (valid) a.rinfo[rec] = make_uint2(cell, cbase + crank);
}

// kAllocPer consecutive claim slots (= record indices) per lane: record ranges of each
// claimed brick's 8 cells, allocated per type from the state's cursors (one atomic per
// block and type), into the brick (k_match) and, as the scatter's per-cell bases (past a
// dense cell's header), over the slot's counts; dense cells reserve kHdr header slots
// and are listed for k_map_dense.  Slots whose record claimed nothing are skipped.
constexpr int kAllocPer = 4;
__global__ __launch_bounds__(kAllocThreads) void k_map_alloc(BuildArgs a) {
  const uint32_t i0 = (blockIdx.x * blockDim.x + threadIdx.x) * kAllocPer;
  uint32_t gb[kAllocPer], tot[kAllocPer], dm[kAllocPer], sz[kAllocPer][8];
  uint32_t vt[2] = {0u, 0u};
#pragma unroll
  for (int u = 0; u < kAllocPer; ++u) {
    const uint32_t i = i0 + u;
    gb[u] = i < a.n ? a.claim[i] : kNoBrick;
    tot[u] = 0;
    dm[u] = 0;
    if (gb[u] != kNoBrick) {
      const uint4* cp = reinterpret_cast<const uint4*>(a.ccnt + (size_t)i * 8);
      const uint4 c0 = cp[0], c1 = cp[1];
      const uint32_t c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool d = c[k] > (uint32_t)kDenseMin;
        dm[u] |= (d ? 1u : 0u) << k;
        sz[u][k] = c[k] + (d ? kHdr : 0);
        tot[u] += sz[u][k];
      }
      vt[gb[u] >= a.off1 ? 1 : 0] += tot[u];
    }
  }
  // per type: block-wide exclusive scan of the lanes' range totals, one atomic per block
  __shared__ uint32_t s_w[2][kAllocThreads / kWave];
  __shared__ uint32_t s_b[2];
  const int w = threadIdx.x / kWave;
  uint32_t incl[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    incl[tt] = wave_incl_scan(vt[tt]);
    if (lane_id() == 63) s_w[tt][w] = incl[tt];
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint32_t bt = 0;
    for (int q = 0; q < kAllocThreads / kWave; ++q) bt += s_w[threadIdx.x][q];
    s_b[threadIdx.x] = bt ? atomicAdd(&a.st->cur[threadIdx.x], bt) : 0u;
  }
  __syncthreads();
  uint32_t run[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    uint32_t wo = s_b[tt];
    for (int q = 0; q < w; ++q) wo += s_w[tt][q];
    run[tt] = wo + incl[tt] - vt[tt] + (tt == 1 ? a.pt_base : 0u);
  }
#pragma unroll
  for (int u = 0; u < kAllocPer; ++u) {
    if (gb[u] == kNoBrick) continue;
    const int t = gb[u] >= a.off1 ? 1 : 0;
    Brick& B = a.bricks[gb[u]];
    uint32_t r = run[t], first[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      B.beg[k] = r;
      first[k] = r + (((dm[u] >> k) & 1) ? kHdr : 0);
      r += sz[u][k];
    }
    B.beg[8] = r;
    B.dense = dm[u];
    run[t] = r;
    uint4* cp = reinterpret_cast<uint4*>(a.ccnt + (size_t)(i0 + u) * 8);
    cp[0] = make_uint4(first[0], first[1], first[2], first[3]);
    cp[1] = make_uint4(first[4], first[5], first[6], first[7]);
    if (dm[u]) {
      const uint32_t o = atomicAdd(&a.st->ndense, (uint32_t)__popc(dm[u]));
      uint32_t j = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if ((dm[u] >> k) & 1) a.dense[o + j++] = gb[u] * 8 + k;
    }
  }
}

// .w of a record: the BITS of a u64 (never a value: only loaded, stored and moved) —
// build order (k_match tie-break) in the low 32, the segment above them, so the match
// epilogue needs no seg[] lookup and a candidate's tie key costs no f64 -> u64
// conversion (~8 VALU per candidate when .w held the value)
__device__ __forceinline__ double rec_tag(uint32_t rec, uint32_t seg) {
  return __longlong_as_double((long long)((unsigned long long)seg << 32 | rec));
}
__device__ __forceinline__ unsigned long long tag_bits(double w) { return (unsigned long long)__double_as_longlong(w); }

__global__ __launch_bounds__(256) void k_map_scatter(BuildArgs a) {
  const uint32_t rec = blockIdx.x * blockDim.x + threadIdx.x;
  if (rec >= a.n) return;
  const uint2 ri = a.rinfo[rec];
  if (ri.x == 0xFFFFFFFFu) return;
  const uint32_t o = a.ccnt[ri.x] + ri.y;  // the cell's first record slot (alloc) + rank
  const RecW R = rec_world(a, rec, true);
  rec_at(a.pos, o, a.rsh) = make_double4(R.p[0], R.p[1], R.p[2], rec_tag(rec, R.seg));
  if (R.t == 0) rec_at(a.nrm, o, a.rsh) = make_double4(R.n[0], R.n[1], R.n[2], 0.0);
}

// sub-cell of a position inside cell origin o (per axis), width sw = w / 4
__device__ __forceinline__ int sub_axis(double p, double o, double sw) {
  const int i = (int)floor((p - o) / sw);
  return i < 0 ? 0 : (i > kSubPerAxis - 1 ? kSubPerAxis - 1 : i);
}

// One block per dense cell: records (in registers) counting-sorted by sub-cell in
// place; the header's 64 u32 are the sub-cells' end offsets relative to the first
// record after the header.  Cells over kDenseThreads * kDenseRecs records stay
// unsorted (header[0] = kUnsorted: k_match scans them whole).
__device__ void dense_sort_cell(const BuildArgs& a, uint32_t cell, uint32_t* s_cnt, uint32_t* s_off) {
  const Brick& B = a.bricks[cell >> 3];
  const uint32_t c = cell & 7;
  const uint32_t beg = B.beg[c], n = B.beg[c + 1] - beg - kHdr, first = beg + kHdr;
  const bool planar = (cell >> 3) < a.off1;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(&rec_at(a.pos, beg, a.rsh));  // 256 B in kHdr (>= 4) slots
  const int tid = threadIdx.x;
  if (n > (uint32_t)(kDenseThreads * kDenseRecs)) {
    if (tid == 0) hdr[0] = kUnsorted;
    return;
  }
  if (tid < kSubCells) s_cnt[tid] = 0;
  // the cell's origin from any of its records (all of them map to this cell)
  const double4 p0 = rec_at(a.pos, first, a.rsh);
  const double ox = floor(p0.x / a.w) * a.w, oy = floor(p0.y / a.w) * a.w, oz = floor(p0.z / a.w) * a.w;
  const double sw = a.w / kSubPerAxis;
  __syncthreads();
  double4 rp[kDenseRecs], rn[kDenseRecs];
  uint32_t rs[kDenseRecs];
#pragma unroll
  for (int u = 0; u < kDenseRecs; ++u) {
    const uint32_t i = (uint32_t)(u * kDenseThreads + tid);
    if (i < n) {
      rp[u] = rec_at(a.pos, first + i, a.rsh);
      if (planar) rn[u] = rec_at(a.nrm, first + i, a.rsh);
      const uint32_t sub = (uint32_t)(sub_axis(rp[u].x, ox, sw) + kSubPerAxis * sub_axis(rp[u].y, oy, sw) +
                                      kSubPerAxis * kSubPerAxis * sub_axis(rp[u].z, oz, sw));
      rs[u] = sub | (atomicAdd(&s_cnt[sub], 1u) << 8);
    }
  }
  __syncthreads();
  static_assert(kSubCells <= kWave, "one wave scans the sub-cell counts");
  if (tid < kWave) {  // exclusive scan of the sub-cell counts by wave 0
    const uint32_t v = tid < kSubCells ? s_cnt[tid] : 0u;
    const uint32_t incl = wave_incl_scan(v);
    if (tid < kSubCells) {
      s_off[tid] = incl - v;
      hdr[tid] = incl;  // sub-cell end
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kDenseRecs; ++u) {
    const uint32_t i = (uint32_t)(u * kDenseThreads + tid);
    if (i < n) {
      const uint32_t o = first + s_off[rs[u] & 0xFF] + (rs[u] >> 8);
      rec_at(a.pos, o, a.rsh) = rp[u];
      if (planar) rec_at(a.nrm, o, a.rsh) = rn[u];
    }
  }
}

__global__ __launch_bounds__(kDenseThreads) void k_map_dense(BuildArgs a) {
  const uint32_t nd = __hip_atomic_load(&a.st->ndense, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x == 0 && threadIdx.x == 0) host_store(a.info, ((unsigned long long)a.epoch << 32) | nd);
  __shared__ uint32_t s_cnt[kSubCells];
  __shared__ uint32_t s_off[kSubCells];
  for (uint32_t di = blockIdx.x; di < nd; di += gridDim.x) {
    dense_sort_cell(a, a.dense[di], s_cnt, s_off);
    __syncthreads();
  }
}

struct MapView {
  const Brick* bricks;
  uint64_t mask;
  const double4* pos;
  const double4* nrm;
  uint32_t epoch;
  uint32_t rsh;  // record stride shift (rec_at)
};

// Cell shifts searched around the query's cell: [0] own cell, [1,7) the 6 face
// neighbours and [7,27) the 12 edges + 8 corners — the first 27 in the reference's
// fixed order (map.tpp:54-68) — then [27,125) the 98 cells of ring 2, used when the
// map is built on cells of w/2 (ring 2 is then still within the bound w).
__device__ __constant__ int c_shift[125][3] = {
    {0, 0, 0}, {1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1},
    {1, 1, 0}, {1, -1, 0}, {-1, 1, 0}, {-1, -1, 0}, {1, 0, 1}, {1, 0, -1}, {-1, 0, 1},
    {-1, 0, -1}, {0, 1, 1}, {0, 1, -1}, {0, -1, 1}, {0, -1, -1}, {1, 1, 1}, {1, 1, -1},
    {1, -1, 1}, {1, -1, -1}, {-1, 1, 1}, {-1, 1, -1}, {-1, -1, 1}, {-1, -1, -1}, {-2, 0, 0},
    {0, -2, 0}, {0, 0, -2}, {0, 0, 2}, {0, 2, 0}, {2, 0, 0}, {-2, -1, 0}, {-2, 0, -1},
    {-2, 0, 1}, {-2, 1, 0}, {-1, -2, 0}, {-1, 0, -2}, {-1, 0, 2}, {-1, 2, 0}, {0, -2, -1},
    {0, -2, 1}, {0, -1, -2}, {0, -1, 2}, {0, 1, -2}, {0, 1, 2}, {0, 2, -1}, {0, 2, 1},
    {1, -2, 0}, {1, 0, -2}, {1, 0, 2}, {1, 2, 0}, {2, -1, 0}, {2, 0, -1}, {2, 0, 1},
    {2, 1, 0}, {-2, -1, -1}, {-2, -1, 1}, {-2, 1, -1}, {-2, 1, 1}, {-1, -2, -1}, {-1, -2, 1},
    {-1, -1, -2}, {-1, -1, 2}, {-1, 1, -2}, {-1, 1, 2}, {-1, 2, -1}, {-1, 2, 1}, {1, -2, -1},
    {1, -2, 1}, {1, -1, -2}, {1, -1, 2}, {1, 1, -2}, {1, 1, 2}, {1, 2, -1}, {1, 2, 1},
    {2, -1, -1}, {2, -1, 1}, {2, 1, -1}, {2, 1, 1}, {-2, -2, 0}, {-2, 0, -2}, {-2, 0, 2},
    {-2, 2, 0}, {0, -2, -2}, {0, -2, 2}, {0, 2, -2}, {0, 2, 2}, {2, -2, 0}, {2, 0, -2},
    {2, 0, 2}, {2, 2, 0}, {-2, -2, -1}, {-2, -2, 1}, {-2, -1, -2}, {-2, -1, 2}, {-2, 1, -2},
    {-2, 1, 2}, {-2, 2, -1}, {-2, 2, 1}, {-1, -2, -2}, {-1, -2, 2}, {-1, 2, -2}, {-1, 2, 2},
    {1, -2, -2}, {1, -2, 2}, {1, 2, -2}, {1, 2, 2}, {2, -2, -1}, {2, -2, 1}, {2, -1, -2},
    {2, -1, 2}, {2, 1, -2}, {2, 1, 2}, {2, 2, -1}, {2, 2, 1}, {-2, -2, -2}, {-2, -2, 2},
    {-2, 2, -2}, {-2, 2, 2}, {2, -2, -2}, {2, -2, 2}, {2, 2, -2}, {2, 2, 2},
};

// Component ax of shift s.  Ring 1 (s < 27) is decoded from bit masks (bit s of kShP[ax]
// set: +1, of kShN[ax]: -1) — pure ALU: a lane-indexed c_shift load is a dependent
// memory round of its own in every probe step; ring 2 reads the table.
constexpr uint32_t kShP[3] = {0x781982u, 0x1998288u, 0x2aaa820u}, kShN[3] = {0x7806604u, 0x6660510u, 0x5555040u};
__device__ __forceinline__ int shift_c(int s, int ax) {
  if (s < 27) return (int)((kShP[ax] >> s) & 1u) - (int)((kShN[ax] >> s) & 1u);
  return c_shift[s][ax];
}

// rank of each reference voxel shift (dx, dy, dz) in {-1, 0, 1}^3 in the reference's
// order (map.tpp:54-68), indexed (dx + 1) * 9 + (dy + 1) * 3 + (dz + 1)
__device__ __constant__ uint8_t c_refrank[27] = {
    26, 10, 25, 14, 2, 13, 24, 9, 23, 18, 4, 17, 6, 0, 5, 16, 3, 15, 22, 8, 21, 12, 1, 11, 20, 7, 19,
};

struct MatchArgs {
  double Tj[12];
  double w;       // cell width of the built map (voxel width / subdivision)
  int rings;      // neighbour rings to search (= subdivision)
  double bound;  // prune bound on d^2 (+inf: no pruning)
  double max_d2, min_d2;
  uint32_t nq_pl, nq_pt, nb_pl, nb_pt;  // queries; planar / point blocks
  int K;
  int sorted;  // 1: pair histogram for the pair sort; 0: per-pair counts only
  int tiles;   // sorted: per-(type, pair, tile) counts, scanned by the last block (kTilesTail,
               // k_pair_scatter_t) or by the pair scatter itself (kTilesScatter, k_pair_scatter_s)
  uint32_t ntl_pl, ntl_pt;  // tiles (kTileBlocks match blocks each) per type
  uint32_t* thist_clear;    // kTilesScatter: the count table's other half, cleared by block 0
  uint32_t thist_clear_n;
  // warm start (fmx_ctx::m_rec): the NN record per query of an earlier match on the same
  // map and query set (null: cold), this launch's NN records (null: not kept), and the
  // largest warm distance^2 that may bound the search (a record that close to the query
  // lies inside the searched cells, so it is a legal candidate)
  const uint32_t* warm;
  uint32_t* rec;
  double warm_lim;
  // per query, its own cell as the last match found it (packed cell coordinates, record
  // range, dense bit; fmx_ctx::m_cell): read when `warm` is set, rewritten with rec
  uint4* cell;
#if FMX_CERT_ANY
  // warm certificate (VERDICT r3 "next round" 5): per query the previous match's
  // second-best bound B2 (fp32, never above the truth: every record other than its NN
  // was at d^2 >= B2, or could not be examined), and that match's pose
  float* cert_b2;
  double Tprev[12];
  int cert_ok;  // cert_b2 holds the bounds of the match that wrote the warm records
                // (an 8-lane match on this map and query set; the one-lane build keeps none)
#endif
  // profiled launches only (else null): the launch's total probes / candidates, summed
  // in prof_acc (agent scope, self-resetting) and stored by the last block to prof_work
  // (its pinned slot of the profiler's work ring: the byte model of THIS launch)
  uint32_t* prof_acc;
  uint32_t* prof_work;
};

// kGroup lanes cooperate on one query: lane g of the group visits shifts
// g, g+kGroup, ... (3-4 of the 27 voxels), then the group min-reduces
// (d^2, build order).  ~8x the threads of a lane-per-query kernel: at per-scan
// sizes (~4e4 queries) the chip would otherwise hold ~2 waves per CU and every
// probe's latency would be exposed.
#ifndef FMX_MATCH_GROUP
#define FMX_MATCH_GROUP 8
#endif
constexpr int kGroup = FMX_MATCH_GROUP;  // lanes per query (16 made the kernel 15% faster but register_scan slower)
constexpr int kQPB = 256 / kGroup;  // queries per block: 256 threads, so every block of a scan is resident at once
constexpr int kMatchThreads = kQPB * kGroup;  // 256
#ifndef FMX_SMALL_CELL
#define FMX_SMALL_CELL 2
#endif
constexpr int kSmallCell = FMX_SMALL_CELL;  // neighbour cells with at most this many records: one lane folds them
// Tiled pair sort: a tile = kTileBlocks match blocks of one type = 1024 queries, one
// k_pair_scatter_t block; the match counts matches per (type, pair, tile).
#ifndef FMX_TILE_Q
#define FMX_TILE_Q 1024  // queries per pair-scatter tile (A/B switch)
#endif
constexpr int kTileBlocks = FMX_TILE_Q / kQPB > 0 ? FMX_TILE_Q / kQPB : 1;
constexpr int kTileQ = kTileBlocks * kQPB;  // 1024
constexpr int kTileMaxPairs = (int)kMatchTileMaxPairs;  // LDS bound of the tiled path (wider windows: per-block path)
constexpr int kWorkWords = 8;               // per-block match work / diagnostic words
// Who scans the (type, pair, tile) counts of a tiled match: the match's last block
// (kTilesTail), or every pair-scatter block its own share plus one extra scatter block
// for the per-pair tables and insert offsets (kTilesScatter: the match has no serial
// tail; used while the whole count table fits the scatter's LDS, kScatterTab words).
constexpr int kTilesTail = 1, kTilesScatter = 2;
constexpr uint32_t kScatterTab = 6144;

// Outputs of the tiled pair sort's last-block pass (consumed by later launches).
struct SortOut {
  uint32_t* hist_off;     // [type][pair][tile] exclusive offsets (each type from 0)
  uint32_t* pair_counts;  // [type][K]
  uint32_t* pair_base;    // [type][K]
  uint32_t* chunk_range;  // [K + 1]
  Chunk* chunks;
  uint32_t* n_chunks;
};

// Exclusive scan of one value per thread over a kMatchThreads block; total returned.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* ws, uint32_t& total) {
  const uint32_t incl = wave_incl_scan(v);
  const int w = threadIdx.x / kWave;
  if (lane_id() == 63) ws[w] = incl;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (int i = 0; i < kMatchThreads / kWave; ++i) {
    if (i < w) off += ws[i];
    tot += ws[i];
  }
  __syncthreads();
  total = tot;
  return off + incl - v;
}

// Exclusive scan of n values of the last block's tail, get(i) -> value, put(i, offset):
// each thread takes a contiguous run of kRun entries per pass, all its reads issued
// before the scan (one dependent round per pass instead of one per 256 entries); carry
// is added to every offset; returns carry + the total.
template <int kRun, class Get, class Put>
__device__ __forceinline__ uint32_t block_scan_runs(uint32_t n, uint32_t carry, Get get, Put put, uint32_t* ws) {
  for (uint32_t s0 = 0; s0 < n; s0 += kMatchThreads * kRun) {
    const uint32_t b = s0 + threadIdx.x * kRun;
    uint32_t v[kRun];
#pragma unroll
    for (int u = 0; u < kRun; ++u) v[u] = b + u < n ? get(b + u) : 0u;
    uint32_t sum = 0;
#pragma unroll
    for (int u = 0; u < kRun; ++u) sum += v[u];
    uint32_t tot;
    uint32_t ex = carry + block_excl_scan(sum, ws, tot);
#pragma unroll
    for (int u = 0; u < kRun; ++u) {
      if (b + u < n) put(b + u, ex);
      ex += v[u];
    }
    carry += tot;
  }
  return carry;
}

// What k_pair_base does, for the tiled sort (K <= kTileMaxPairs), from the per-type
// first rows s_pb (filled by the caller's scan of the (type, pair, tile) counts):
// per-pair counts and first rows, the host copy of the counts, the linearize chunk table.
__device__ void pair_sort_finish(const MatchArgs& a, const SortOut& so, uint32_t* __restrict__ host_counts,
                                 uint32_t (*s_pb)[kTileMaxPairs + 1]) {
  __shared__ uint32_t ws[kMatchThreads / kWave];
  __shared__ uint32_t s_cr[kTileMaxPairs + 1];
  const int K = a.K;
  __syncthreads();
  uint32_t carry = 0;
  for (int k0 = 0; k0 < K; k0 += kMatchThreads) {
    const int k = k0 + threadIdx.x;
    uint32_t nch = 0;
    if (k < K) {
      const uint32_t b_pl = s_pb[0][k], npl = s_pb[0][k + 1] - b_pl;
      const uint32_t b_pt = s_pb[1][k], npt = s_pb[1][k + 1] - b_pt;
      so.pair_counts[k] = npl;
      so.pair_counts[K + k] = npt;
      host_store(host_counts + k, npl);  // mapped host memory
      host_store(host_counts + K + k, npt);
      so.pair_base[k] = b_pl;
      so.pair_base[K + k] = b_pt;
      nch = (npl + kPlaneChunk - 1) / kPlaneChunk + (npt + kPointChunk - 1) / kPointChunk;
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan(nch, ws, tot);
    if (k < K) s_cr[k] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) s_cr[K] = carry;
  __syncthreads();
  for (int k = threadIdx.x; k <= K; k += kMatchThreads) so.chunk_range[k] = s_cr[k];
  // descriptors: chunk -> pair by binary search over s_cr
  for (uint32_t ci = threadIdx.x; ci < carry; ci += kMatchThreads) {
    int lo = 0, hi = K - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_cr[mid] <= ci) lo = mid;
      else hi = mid - 1;
    }
    const int k = lo;
    const uint32_t j = ci - s_cr[k];
    const uint32_t b_pl = s_pb[0][k], npl = s_pb[0][k + 1] - b_pl;
    const uint32_t b_pt = s_pb[1][k], npt = s_pb[1][k + 1] - b_pt;
    const uint32_t ncpl = (npl + kPlaneChunk - 1) / kPlaneChunk;
    if (j < ncpl) {
      const uint32_t r = j * kPlaneChunk;
      so.chunks[ci] = Chunk{0, (uint32_t)k, b_pl + r, b_pl + min(npl, r + kPlaneChunk)};
    } else {
      const uint32_t r = (j - ncpl) * kPointChunk;
      so.chunks[ci] = Chunk{1, (uint32_t)k, b_pt + r, b_pt + min(npt, r + kPointChunk)};
    }
  }
  if (threadIdx.x == 0) *so.n_chunks = carry;
}

// The match kernel's last block, tiled sort: scan the (type, pair, tile) counts (read
// and reset), then pair_sort_finish.
__device__ void pair_sort_tail(const MatchArgs& a, uint32_t* __restrict__ thist, const SortOut& so,
                               uint32_t* __restrict__ host_counts, uint32_t (*s_pb)[kTileMaxPairs + 1]) {
  __shared__ uint32_t ws[kMatchThreads / kWave];
  const int K = a.K;
  for (int t = 0; t < 2; ++t) {
    const uint32_t ntl = t ? a.ntl_pt : a.ntl_pl;
    const size_t base = t ? (size_t)K * a.ntl_pl : 0;
    const uint32_t n = (uint32_t)K * ntl;
    const uint32_t carry = block_scan_runs<4>(
        n, 0u,
        [&](uint32_t i) { return __hip_atomic_exchange(thist + base + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); },
        [&](uint32_t i, uint32_t o) {
          so.hist_off[base + i] = o;
          if (i % ntl == 0) s_pb[t][i / ntl] = o;
        },
        ws);
    for (int k = threadIdx.x; k < K; k += kMatchThreads)
      if (ntl == 0) s_pb[t][k] = 0;
    if (threadIdx.x == 0) s_pb[t][K] = carry;
  }
  pair_sort_finish(a, so, host_counts, s_pb);
}

// Exclusive scans of four values per thread over a kMatchThreads block at once (one
// pair of barriers for all four); totals returned.
__device__ __forceinline__ void block_excl_scan4(const uint32_t (&v)[4], uint32_t (&ex)[4], uint32_t (&tot)[4],
                                                 uint32_t (*ws)[4]) {
  uint32_t incl[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) incl[q] = wave_incl_scan(v[q]);
  const int w = threadIdx.x / kWave;
  if (lane_id() == kWave - 1)
#pragma unroll
    for (int q = 0; q < 4; ++q) ws[w][q] = incl[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t off = 0, t = 0;
#pragma unroll
    for (int i = 0; i < kMatchThreads / kWave; ++i) {
      const uint32_t x = ws[i][q];
      if (i < w) off += x;
      t += x;
    }
    ex[q] = off + incl[q] - v[q];
    tot[q] = t;
  }
  __syncthreads();
}

// Lanes of a wave holding G-lane group g's bits of a ballot.
template <int G>
__device__ __forceinline__ uint64_t group_bits(uint64_t ballot) {
  if constexpr (G == kWave) return ballot;
  else return (ballot >> ((lane_id() / G) * G)) & ((1ull << G) - 1);
}

#ifndef FMX_COMPACT_SHIFTS
#define FMX_COMPACT_SHIFTS 1  // one-lane-per-query ring-1 search from a per-lane work list (A/B switch)
#endif
#ifndef FMX_F32_BOUNDS
#define FMX_F32_BOUNDS 1  // cell lower bounds in fp32 from the query's in-cell offset (A/B switch)
#endif
#ifndef FMX_WARM_START
#define FMX_WARM_START 1  // bound each search by the previous match's record (compile-time A/B switch)
#endif
#ifndef FMX_RING_LIST  // neighbour shifts admitted once and probed G per round (A/B switch): the
// 8-lane build (C4: same time as the ring-class passes); the one-lane build keeps the
// passes (its plain variant walks per-lane lists instead, and the list code costs it
// 8 spilled VGPRs)
#define FMX_RING_LIST (FMX_MATCH_GROUP != 1)
#endif
#ifndef FMX_PROBE_TOGETHER
#define FMX_PROBE_TOGETHER 1  // brick key and cell range in flight together (A/B switch)
#endif
// The 26 ring-1 cells relative to a query's octant, nearest first: component i along
// the query's i-th nearest axis is +1 (toward its near face), -1 (far face) or 0.
// Cells 0..6 are the near faces, edges and corner; 7..25 hold a far side.  Bit k of
// kRel0P is set when cell k's component 0 is +1, of kRel0N when it is -1, and so on:
// a lane decodes ITS cell without a table load.
constexpr uint32_t kRel0P = 0x581455u, kRel0N = 0x3a32880u, kRel1P = 0xa84866u, kRel1N = 0x3558500u,
                   kRel2P = 0x130a078u, kRel2N = 0x2ce5200u;
constexpr int kRelNear = 7;
__device__ __forceinline__ int shift_axis(uint32_t pos, uint32_t neg, int k) {
  return (int)((pos >> k) & 1u) - (int)((neg >> k) & 1u);
}
// index of ring-1 shift (dx, dy, dz) != 0 in c_shift / the reference's voxel_shifts
// (map.tpp:54-68): faces 1..6, edges 7..18 (xy, xz, yz), corners 19..26
__device__ __forceinline__ int ring1_index(int dx, int dy, int dz) {
  const int nz = (dx != 0) + (dy != 0) + (dz != 0);
  if (nz == 1) return dx != 0 ? 1 + (dx < 0) : (dy != 0 ? 3 + (dy < 0) : 5 + (dz < 0));
  if (nz == 2)
    return dz == 0 ? 7 + 2 * (dx < 0) + (dy < 0) : (dy == 0 ? 11 + 2 * (dx < 0) + (dz < 0) : 15 + 2 * (dy < 0) + (dz < 0));
  return 19 + 4 * (dx < 0) + 2 * (dy < 0) + (dz < 0);
}
// A non-negative double as an fp32 value never above it (round to nearest, then shrink
// by 2^-22 relative: past both roundings); +inf stays +inf.
__device__ __forceinline__ float cdown(double v) { return (float)v * (1.0f - 0x1p-22f); }

// VoxelMap::find_closest (map.tpp:70-91) of one query by a group of G lanes (lane g of
// the group), bounded by the incoming best (a.bound, or +inf).
template <int G, bool DENSE>
__device__ __forceinline__ void nn_search(const MatchArgs& a, const MapView& M, const double (&wq)[3], int g,
                                          uint32_t* hd, double& best, uint32_t& best_rid, uint32_t& best_i,
                                          uint32_t& best_sg,
                                          uint32_t& n_probe, uint32_t& n_cand, uint32_t& n_iter, uint32_t& n_list,
                                          double warm_b = INFINITY, uint32_t* phase = nullptr,
                                          uint4 ocv = uint4{0u, 0x80000000u, 0u, 0u}, uint4* oc_out = nullptr,
                                          float* b2_out = nullptr) {
  // The warm certificate's second-best bound of this search (FMX_CERT_ANY builds): b2,
  // the least of the d^2 of the examined records other than the lane's current best
  // record and the lower bounds of the cells / sub-cells pruned.  fp32, rounded down
  // (cdown): a bound may only be too small.  (The one-lane compact walk is not covered.)
  constexpr bool kCert = FMX_CERT_ANY && G > 1;
  float b2 = INFINITY;
  const int bx = (int)floor(wq[0] / a.w), by = (int)floor(wq[1] / a.w), bz = (int)floor(wq[2] / a.w);
  // argmin key (d^2, tie): tie = the reference shift rank of the record's voxel
  // (map.tpp:54-68, 77-88: the first voxel in shift order wins an exact tie) << 27 |
  // the record's build order (= insertion order inside a voxel, map.tpp:41-52)
  const int sh = a.rings >= 2 ? 1 : 0;  // cells of w/2: reference voxel = cell >> 1
  auto srank = [&](int sx, int sy, int sz) -> uint32_t {
    const int dx = ((bx + sx) >> sh) - (bx >> sh), dy = ((by + sy) >> sh) - (by >> sh),
              dz = ((bz + sz) >> sh) - (bz >> sh);
    return (uint32_t)c_refrank[(dx + 1) * 9 + (dy + 1) * 3 + (dz + 1)] << 27;
  };
  // the tie rank of shift s: on an unsubdivided map the shift IS the reference voxel
  // shift, whose rank is its index (c_shift[0..26] = voxel_shifts, map.tpp:54-68)
  auto srank_s = [&](int s) -> uint32_t {
    return sh == 0 && s < 27 ? (uint32_t)s << 27 : srank(shift_c(s, 0), shift_c(s, 1), shift_c(s, 2));
  };
  // one bucket read per probe: key, the cell's two boundaries and its dense bit in
  // flight together; a bucket of another build epoch ends the chain (empty)
  auto walk = [&](unsigned long long key, uint32_t ci, uint64_t h, uint32_t& first, uint32_t& count, bool& dense) {
    first = 0;
    count = 0;
    dense = false;
    for (;;) {
      ++n_probe;
      const Brick* b = M.bricks + h;
      const unsigned long long k = b->key;
      const uint32_t b0 = b->beg[ci], b1 = b->beg[ci + 1], dm = b->dense;
      // one lane per query: the cell's range is read with the key, not after its
      // compare (the compiler sinks these loads into the hit branch: a second dependent
      // round; C5 -2..4 %).  The 8-lane build keeps the sunk loads (its registers are
      // tighter: C4 match +3 % with them hoisted).
      if constexpr (G == 1 && FMX_PROBE_TOGETHER) {
        asm volatile("" ::"v"(b0), "v"(b1));
        if constexpr (DENSE) asm volatile("" ::"v"(dm));
      }
      if (k == key) {
        first = b0;
        count = b1 - b0;
        dense = (dm >> ci) & 1;
        return;
      }
      if (key_epoch(k) != M.epoch) return;
      h = (h + 1) & M.mask;
    }
  };
  auto probe = [&](int sx, int sy, int sz, uint32_t& first, uint32_t& count, bool& dense) {
    const int X = bx + sx, Y = by + sy, Z = bz + sz;
    const unsigned long long key = brick_key(X, Y, Z, M.epoch);
    walk(key, brick_cell(X, Y, Z), mix64(key) & M.mask, first, count, dense);
  };
  // a record is one double4: world position + its build order in .w (rec_tag), so a
  // candidate test is one 32-B load
  auto fold = [&](const double4& p, uint32_t i, uint32_t rk) {
    const double dx = p.x - wq[0], dy = p.y - wq[1], dz = p.z - wq[2];
    const double d2 = (dx * dx + dz * dz) + dy * dy;
    const unsigned long long t = tag_bits(p.w);
    const uint32_t tk = rk | ((uint32_t)t & 0x07FFFFFFu);  // build order: low bits
    if (d2 <= best && (d2 < best || tk < best_rid)) {
      if (kCert && best_i != 0xFFFFFFFFu) b2 = fminf(b2, cdown(best));  // the displaced record
      best = d2;
      best_rid = tk;
      best_i = i;
      best_sg = (uint32_t)(t >> 32);  // the record's segment, for the epilogue's pose loads
    } else if (kCert) {
      b2 = fminf(b2, cdown(d2));
    }
  };
  // The same argmin in three reductions instead of one over (d^2, tie, index) moves:
  // min d^2 (fp64 min), then the least tie key among the lanes holding that d^2, then
  // the index among the lanes holding both (every such lane holds the same record: a
  // record's (d^2, tie key) is unique; its segment rides along).  A lane without a
  // candidate holds the bound it
  // started from and tie / index ~0, so it never displaces one (~26 VALU per call
  // instead of ~42: C4 k_match is VALU-limited).
  auto group_min = [&]() {
    if constexpr (G == 1) return;
    else if constexpr (G > 16) {
      double m = best;
      for (int o = 1; o < G; o <<= 1) m = fmin(m, __shfl_xor(m, o, G));
      uint32_t r = best == m ? best_rid : 0xFFFFFFFFu;
      for (int o = 1; o < G; o <<= 1) r = min(r, (uint32_t)__shfl_xor((int)r, o, G));
      const bool win = best == m && best_rid == r;
      if (kCert && !win && best_i != 0xFFFFFFFFu) b2 = fminf(b2, cdown(best));  // a lane's record that lost the argmin
      uint32_t i = win ? best_i : 0xFFFFFFFFu, sg = win ? best_sg : 0xFFFFFFFFu;
      for (int o = 1; o < G; o <<= 1) i = min(i, (uint32_t)__shfl_xor((int)i, o, G));
      for (int o = 1; o < G; o <<= 1) sg = min(sg, (uint32_t)__shfl_xor((int)sg, o, G));
      best = m;
      best_rid = r;
      best_i = i;
      best_sg = sg;
    } else {
      auto dmin = [&](auto ctrl_tag) {
        constexpr int CTRL = decltype(ctrl_tag)::value;
        const long long bb = __double_as_longlong(best);
        const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)bb, CTRL, 0xF, 0xF, false);
        const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(bb >> 32), CTRL, 0xF, 0xF, false);
        best = fmin(best, __longlong_as_double((long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo)));
      };
      auto umin = [&](uint32_t& v, auto ctrl_tag) {
        constexpr int CTRL = decltype(ctrl_tag)::value;
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false));
      };
      const double mine = best;
      const bool rec_mine = best_i != 0xFFFFFFFFu;
      if constexpr (G >= 16) dmin(std::integral_constant<int, 0x140>{});  // row_mirror: l <-> 15-l
      if constexpr (G >= 8) dmin(std::integral_constant<int, 0x141>{});   // row_half_mirror
      if constexpr (G >= 4) dmin(std::integral_constant<int, 0x4E>{});    // quad_perm [2,3,0,1]
      if constexpr (G >= 2) dmin(std::integral_constant<int, 0xB1>{});    // quad_perm [1,0,3,2]
      uint32_t r = mine == best ? best_rid : 0xFFFFFFFFu;
      if constexpr (G >= 16) umin(r, std::integral_constant<int, 0x140>{});
      if constexpr (G >= 8) umin(r, std::integral_constant<int, 0x141>{});
      if constexpr (G >= 4) umin(r, std::integral_constant<int, 0x4E>{});
      if constexpr (G >= 2) umin(r, std::integral_constant<int, 0xB1>{});
      const bool win = mine == best && best_rid == r;
      if (kCert && !win && rec_mine) b2 = fminf(b2, cdown(mine));  // a lane's record that lost the argmin
      uint32_t i = win ? best_i : 0xFFFFFFFFu, sg = win ? best_sg : 0xFFFFFFFFu;
      if constexpr (G >= 16) umin(i, std::integral_constant<int, 0x140>{});
      if constexpr (G >= 8) umin(i, std::integral_constant<int, 0x141>{});
      if constexpr (G >= 4) umin(i, std::integral_constant<int, 0x4E>{});
      if constexpr (G >= 2) umin(i, std::integral_constant<int, 0xB1>{});
      if constexpr (G >= 16) umin(sg, std::integral_constant<int, 0x140>{});
      if constexpr (G >= 8) umin(sg, std::integral_constant<int, 0x141>{});
      if constexpr (G >= 4) umin(sg, std::integral_constant<int, 0x4E>{});
      if constexpr (G >= 2) umin(sg, std::integral_constant<int, 0xB1>{});
      best_rid = r;
      best_i = i;
      best_sg = sg;
    }
  };
  // Records of one cell, walked by the whole group (group-uniform arguments).  A
  // dense cell (k_map_dense) starts with a header of its 64 sub-cell ends: the
  // query's own sub-cell first, then every other sub-cell whose box lower bound does
  // not exceed the best so far, each group-walked (lane g holds sub-cells g, g + G, ...
  // for the bounds; the header copy in LDS `hd` is shared by the group).
  // Lower bounds (cell and sub-cell pruning) in fp32 from the query's offset inside its
  // own cell, qo (the double subtraction wq - b * w, then one rounding): every bound is
  // a distance to a plane of the cell grid, shortened by a slack of 1e-6 w — well over
  // the fp32 error of qo and of the bound's few operations (< 1e-6 relative of w) — so a
  // bound never exceeds the true distance^2 and pruning never drops the winner.  fp64
  // bounds cost ~3x the VALU issue slots of these (C4 k_match is ~60 % VALU-busy per
  // SIMD at 4 waves).
  const float wf = (float)a.w, swf = wf * (1.0f / kSubPerAxis), slk = 1e-6f * wf;
  float qo[3] = {0.0f, 0.0f, 0.0f};
  if (FMX_F32_BOUNDS || DENSE) {
    qo[0] = (float)(wq[0] - bx * a.w);
    qo[1] = (float)(wq[1] - by * a.w);
    qo[2] = (float)(wq[2] - bz * a.w);
  }
  // Records of one cell, walked by the whole group (group-uniform arguments).  A
  // dense cell (k_map_dense) starts with a header of its 64 sub-cell ends: the
  // query's own sub-cell first, then every other sub-cell whose box lower bound does
  // not exceed the best so far, each group-walked (lane g holds sub-cells g, g + G, ...
  // for the bounds; the header copy in LDS `hd` is shared by the group).  sx, sy, sz:
  // the cell's shift from the query's cell.
  auto scan_cell = [&](uint32_t first, uint32_t count, bool dense, int sx, int sy, int sz, uint32_t rk) {
    if constexpr (!DENSE) {  // no dense cell in the map: the cell's records, split over the lanes
      constexpr int D = FMX_MATCH_DEPTH_PLAIN;
      const uint32_t end = first + count;
      n_cand += count / G + (g < (int)(count % G) ? 1 : 0);
      uint32_t i = first + g;
      for (; i + (D - 1) * G < end; i += D * G) {
        double4 pr[D];
#pragma unroll
        for (int d = 0; d < D; ++d) pr[d] = rec_at(M.pos, i + d * G, M.rsh);
#pragma unroll
        for (int d = 0; d < D; ++d) fold(pr[d], i + d * G, rk);
      }
      for (; i < end; i += G) fold(rec_at(M.pos, i, M.rsh), i, rk);
      group_min();
      return;
    }
    constexpr int kPer = kSubCells / G;  // sub-cells per lane
    const uint32_t* hdr = reinterpret_cast<const uint32_t*>(&rec_at(M.pos, first, M.rsh));
    const uint32_t base = dense ? first + kHdr : first;
    // the query's offset from this cell's origin, per axis
    const float ox = qo[0] - sx * wf, oy = qo[1] - sy * wf, oz = qo[2] - sz * wf;
    // per sub-cell lower bound: distance^2 to the sub-cell's box (fp32, slack as above)
    auto axis_lb = [&](float q, int i) {
      const float lo = i * swf, hi = lo + swf;
      const float d = fmaxf(fmaxf(lo - q, q - hi), 0.0f);
      const float m = fmaxf(d - slk, 0.0f);
      return m * m;
    };
    auto sub_lb = [&](int sub) {
      return (double)(axis_lb(ox, sub % kSubPerAxis) + axis_lb(oy, (sub / kSubPerAxis) % kSubPerAxis) +
                      axis_lb(oz, sub / (kSubPerAxis * kSubPerAxis)));
    };
    auto sub_beg = [&](int sub) { return sub == 0 ? 0u : hd[sub - 1]; };
    // A dense cell's header in hd[] (LDS; coalesced copy: lane g copies entries
    // [g * kPer, (g + 1) * kPer)), read in the same round as its sorted marker (entry 0):
    // a sorted cell's sub-cell ranges; any other cell is one range.  The s_waitcnt +
    // memory clobbers order the copy after the previous cell's reads and before the
    // other lanes' reads.
    bool sorted = false;
    if (DENSE && dense) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (kPer >= 4) {
#pragma unroll
        for (int u = 0; u < kPer; u += 4)
          *reinterpret_cast<uint4*>(hd + g * kPer + u) = *reinterpret_cast<const uint4*>(hdr + g * kPer + u);
      } else {
#pragma unroll
        for (int u = 0; u < kPer; ++u) hd[g * kPer + u] = hdr[g * kPer + u];
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      sorted = hd[0] != kUnsorted;
      if (sorted && g == 0) n_probe += kHdr * 32 / 64;  // the header's 64-B lines (byte model)
    }
    // the query's (nearest) sub-cell: only the visiting order depends on it
    auto sub_of = [&](float q) {
      const int i = (int)floorf(q * (kSubPerAxis / wf));
      return i < 0 ? 0 : (i > kSubPerAxis - 1 ? kSubPerAxis - 1 : i);
    };
    const int qs = sub_of(ox) + kSubPerAxis * sub_of(oy) + kSubPerAxis * kSubPerAxis * sub_of(oz);
    // Walk 0: the whole cell, or (sorted) the query's own / nearest sub-cell.  Walk 1
    // (sorted only): every other sub-cell whose box can still hold a closer record.
    // A walk is ONE virtual range — the chosen ranges' records concatenated in
    // sub-cell order, split over the group's lanes, FMX_MATCH_DEPTH loads in flight
    // per lane across range boundaries — then one group min.
    for (int wk = 0; wk < (sorted ? 2 : 1); ++wk) {
      uint64_t mask = 0;
      uint32_t tot = 0;
      if (!sorted) {
        mask = 1;
        tot = first + count - base;
      } else if (wk == 0) {
        const uint32_t s0 = sub_beg(qs), e0 = hd[qs];
        if (e0 > s0 && sub_lb(qs) <= best) {
          mask = 1ull << qs;
          tot = e0 - s0;
        } else if (kCert && e0 > s0) {
          b2 = fminf(b2, cdown(sub_lb(qs)));
        }
      } else {  // lane g bounds sub-cells g, g + G, ...; a ballot per stride
#pragma unroll 1
        for (int u = 0; u < kPer; ++u) {
          const int sub = u * G + g;
          const uint32_t s0 = sub_beg(sub), e0 = hd[sub];
          const bool lv = sub != qs && e0 > s0 && sub_lb(sub) <= best;
          if (kCert && !lv && sub != qs && e0 > s0) b2 = fminf(b2, cdown(sub_lb(sub)));
          if (lv) tot += e0 - s0;
          mask |= group_bits<G>(__ballot(lv)) << (u * G);
        }
#pragma unroll
        for (int o = 1; o < G; o <<= 1) tot += __shfl_xor(tot, o, G);
      }
      if (tot == 0) continue;
      int k = __ffsll((unsigned long long)mask) - 1;
      uint32_t ks = sorted ? sub_beg(k) : 0u, ke = sorted ? hd[k] : tot, vbase = 0;  // (not sorted: never advances)
      auto locate = [&](uint32_t v) {  // v ascending per lane
        while (v - vbase >= ke - ks) {
          vbase += ke - ks;
          mask &= mask - 1;
          k = __ffsll((unsigned long long)mask) - 1;
          ks = sub_beg(k);
          ke = hd[k];
        }
        return base + ks + (v - vbase);
      };
      n_cand += tot / G + ((uint32_t)g < tot % G ? 1 : 0);
      constexpr int D = FMX_MATCH_DEPTH;
      uint32_t v = g;
      for (; v + (D - 1) * G < tot; v += D * G) {
        uint32_t ix[D];
        double4 pr[D];
#pragma unroll
        for (int d = 0; d < D; ++d) ix[d] = locate(v + d * G);
#pragma unroll
        for (int d = 0; d < D; ++d) pr[d] = rec_at(M.pos, ix[d], M.rsh);
#pragma unroll
        for (int d = 0; d < D; ++d) fold(pr[d], ix[d], rk);
      }
      for (; v < tot; v += G) {
        const uint32_t i = locate(v);
        fold(rec_at(M.pos, i, M.rsh), i, rk);
      }
      group_min();
    }
  };
  const bool inr = key_in_range(bx, by, bz);
  // the own cell's identity for the per-query cell cache: 21 bits per coordinate (in
  // range: |coordinate| < 2^18), bit 63 clear (set: no entry)
  const uint2 own_key = make_uint2((uint32_t)(bx & 0x1FFFFF) | (uint32_t)(by & 0x7FF) << 21,
                                   (uint32_t)((by >> 11) & 0x3FF) | (uint32_t)(bz & 0x1FFFFF) << 10);
#if !FMX_F32_BOUNDS
  // lower bound on d^2 from the query to any point of the cell at shift s (fp64)
  auto shift_lb = [&](int s) {
    double lb = 0.0;
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
      const int sa = shift_c(s, ax);
      const int ba = ax == 0 ? bx : (ax == 1 ? by : bz);
      const double hi = (ba + 1) * a.w - wq[ax], lo = wq[ax] - ba * a.w;
      const double e = sa > 0 ? hi + (sa - 1) * a.w : (sa < 0 ? lo + (-sa - 1) * a.w : 0.0);
      const double m = fmax(e - 1e-9, 0.0);
      lb += m * m;
    }
    return lb;
  };
#else
  // lower bound on d^2 from the query to any point of the cell at shift s (fp32 from
  // qo, slack as above)
  auto shift_lb = [&](int s) {
    float lb = 0.0f;
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
      const int sa = shift_c(s, ax);
      const float lo = qo[ax], hi = wf - qo[ax];
      const float e = sa > 0 ? hi + (sa - 1) * wf : (sa < 0 ? lo + (-sa - 1) * wf : 0.0f);
      const float m = fmaxf(e - slk, 0.0f);
      lb += m * m;
    }
    return (double)lb;
  };
#endif
  // The cells in passes of increasing lower bound — the query's own cell (shift 0,
  // visited first by the reference too), ring-1 faces (shifts 1..6), ring-1 edges +
  // corners (7..26), then ring 2 (27..124) when the map uses half-width cells — each
  // pass pruned against the best found so far.  In a pass a lane bounds and probes
  // its shifts in parallel, then the group walks every surviving cell together
  // (records split over the lanes), re-checking each bound against the shared best.
  // One loop over the passes, so the cell walk is emitted once.
  const int npass = a.rings >= 2 ? 4 : 3;
  // One lane per query, plain cells, one ring (the large-set build, C5): after the own
  // cell, each lane walks ITS OWN list of the ring-1 cells whose bound admits them, one
  // cell per step, instead of the wave stepping through all 26 shifts (probing a shift
  // whenever any of its 64 queries needs it).  The wave then takes as many dependent
  // probe + record rounds as its busiest query, not as the union of its queries' cells.
  constexpr bool kCompact = G == 1 && !DENSE && FMX_COMPACT_SHIFTS;
  const bool compact = kCompact && a.rings == 1;
  // One step of the search: lane g bounds and probes shift s (s < 0: none); the cells
  // of at most kSmallCell records are folded by their probing lane, the larger ones
  // walked by the whole group, each bound re-checked against the shared best.
  auto visit = [&](int s, bool own) {
    uint32_t vf = 0, vc = 0;
    bool vd = false;
    double vlb = INFINITY;
    if (inr && s >= 0) {
      const double lb = shift_lb(s);
      if (lb <= best) {  // else conservative: no point inside can win
        if (own && s == 0 && ocv.x == own_key.x && ocv.y == own_key.y) {
          // warm: the own cell as the last match on this map found it (no bucket read)
          vf = ocv.z;
          vc = ocv.w & 0x7FFFFFFFu;
          vd = (ocv.w >> 31) != 0;
        } else {
          probe(shift_c(s, 0), shift_c(s, 1), shift_c(s, 2), vf, vc, vd);
          if (own && s == 0 && oc_out) *oc_out = uint4{own_key.x, own_key.y, vf, vc | (vd ? 0x80000000u : 0u)};
        }
        vlb = lb;
      } else if (kCert) {
        b2 = fminf(b2, cdown(lb));
      }
    } else if (own && s == 0 && oc_out) {
      *oc_out = uint4{0u, 0x80000000u, 0u, 0u};  // no entry
    }
    // the warm bound joins once the own cell's probe is in flight (the probe does not
    // wait for the warm record's load): a record at distance^2 warm_b exists, so no
    // cell, sub-cell or record farther than that can win — the argmin is unchanged
    if (own) best = fmin(best, warm_b);
    // small cells (<= kSmallCell records): the lane that probed one folds its
    // records itself, every lane's loads in flight together, one group min after;
    // the argmin on (d^2, tie key) does not depend on the folding order
    const bool small = vc != 0 && vc <= (uint32_t)kSmallCell && vlb <= best;
    // (a probed small cell the warm bound has since pruned: its records stay unexamined)
    if (kCert && vc != 0 && vc <= (uint32_t)kSmallCell && !(vlb <= best)) b2 = fminf(b2, cdown(vlb));
    if (small) {
      const uint32_t rk = srank_s(s);
      double4 pr[kSmallCell];
#pragma unroll
      for (int u = 0; u < kSmallCell; ++u)
        if (u < (int)vc) pr[u] = rec_at(M.pos, vf + u, M.rsh);
#pragma unroll
      for (int u = 0; u < kSmallCell; ++u)
        if (u < (int)vc) fold(pr[u], vf + u, rk);
      n_cand += vc;
    }
    if (group_bits<G>(__ballot(small))) group_min();
    uint64_t live = group_bits<G>(__ballot(vc > (uint32_t)kSmallCell));  // larger cells: walked by the group
    while (live) {
      const int l = __ffsll((unsigned long long)live) - 1;
      live &= live - 1;
      const double lb = __shfl(vlb, l, G);
      if (lb > best) {  // best is group-uniform here
        if (kCert) b2 = fminf(b2, cdown(lb));
        continue;
      }
      const uint32_t cnt = __shfl(vc, l, G);
      const uint32_t first = __shfl(vf, l, G);
      const bool dn = __shfl((int)vd, l, G) != 0;
      const int sl = __shfl(s, l, G);
      scan_cell(first, cnt, dn, shift_c(sl, 0), shift_c(sl, 1), shift_c(sl, 2), srank_s(sl));
    }
  };
#if FMX_RING_LIST
  // The query's own cell first (shift 0, visited first by the reference too), then
  // every other shift whose lower bound admits it against the best so far — ring 1
  // (and ring 2 on a map of half-width cells), listed once per group as a bit mask and
  // taken G at a time in shift order (nearer rings first), each re-bounded when taken.
  // A group's admitted cells are thus probed G per dependent round instead of one pass
  // per ring class (faces, then edges + corners, then ring 2), each a round of its own.
  visit(g == 0 ? 0 : -1, true);
#ifdef FMX_DIAG_PHASE
  if (phase) phase[0] = (uint32_t)wall_clock64();
#endif
  if (!compact) {
    const int nsh = a.rings >= 2 ? 124 : 26;
    uint64_t m0 = 0, m1 = 0;  // admitted shifts: bit s - 1
    for (int u = 0; u * G < nsh; ++u) {
      const int s = 1 + u * G + g;
      const double slb = inr && s <= nsh ? shift_lb(s) : INFINITY;
      const bool ad = inr && s <= nsh && slb <= best;
      if (kCert && !ad) b2 = fminf(b2, cdown(slb));
      const uint64_t b = group_bits<G>(__ballot(ad));
      const int bit = u * G;
      if (bit < 64) m0 |= b << bit;
      else m1 |= b << (bit - 64);
    }
#ifdef FMX_DIAG_PHASE
    if (phase) phase[1] = (uint32_t)wall_clock64();
#endif
    while (m0 | m1) {
      int mine = -1;  // this lane's shift of the round: the g-th admitted one left
#pragma unroll
      for (int k = 0; k < G; ++k) {
        if (!(m0 | m1)) break;
        int bit;
        if (m0) {
          bit = __ffsll((unsigned long long)m0) - 1;
          m0 &= m0 - 1;
        } else {
          bit = 64 + __ffsll((unsigned long long)m1) - 1;
          m1 &= m1 - 1;
        }
        if (k == g) mine = bit + 1;
      }
      visit(mine, false);
    }
  }
#ifdef FMX_DIAG_PHASE
  if (phase) phase[2] = (uint32_t)wall_clock64();
#endif
#else
  // The cells in passes of increasing lower bound — the query's own cell (shift 0,
  // visited first by the reference too), ring-1 faces (shifts 1..6), ring-1 edges +
  // corners (7..26), then ring 2 (27..124) when the map uses half-width cells — each
  // pass pruned against the best found so far; in a pass a lane bounds and probes its
  // shifts in parallel (visit).
  for (int ip = 0; ip < (compact ? 1 : npass); ++ip) {
    const int s_begin = ip == 0 ? 0 : (ip == 1 ? 1 : (ip == 2 ? 7 : 27));
    const int s_end = ip == 0 ? 1 : (ip == 1 ? 7 : (ip == 2 ? 27 : 125));
    for (int s0 = s_begin; s0 < s_end; s0 += G)  // one shift per lane per chunk
      visit(s0 + g < s_end ? s0 + g : -1, ip == 0);
  }
#endif
  if constexpr (kCompact) {
    if (compact && inr) {
      // Per axis: the query's squared distance (1e-9 slack) to its cell's
      // near and far face, rounded down to fp32, and the near side's sign; the axes
      // sorted by near distance.  The 26 ring-1 cells are listed RELATIVE to that
      // frame, nearest first (kRel*: the near faces, edges and corner of the query's
      // octant, then every cell with a far side, whose bound is at least the smallest
      // far term >= (w/2)^2).  A shift's bound is the sum of its axes' terms; the test
      // against best allows for the fp32 sum's rounding (threshold rounded up,
      // x (1 + 2^-20)), so a cell is skipped only when its true bound exceeds the best: the
      // winner is unchanged (the argmin on (d^2, tie) does not depend on visit order).
      // nr / fr: near / far terms in sorted order; cd: per sorted slot i, bits 3i..3i+1
      // the grid axis and bit 3i+2 set when the near face is the low one
      float nr[3], fr[3];
      uint32_t cd[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int ba = k == 0 ? bx : (k == 1 ? by : bz);
        const double lo = fmax(wq[k] - ba * a.w - 1e-9, 0.0), hi = fmax((ba + 1) * a.w - wq[k] - 1e-9, 0.0);
        const float l2 = __double2float_rd(lo * lo), h2 = __double2float_rd(hi * hi);
        nr[k] = fminf(l2, h2);
        fr[k] = fmaxf(l2, h2);
        cd[k] = (uint32_t)k | (h2 <= l2 ? 0u : 4u);
      }
      auto cswap = [&](int i, int j) {  // sort the axes by near term (3-element network)
        if (nr[j] < nr[i]) {
          float t = nr[i]; nr[i] = nr[j]; nr[j] = t;
          t = fr[i]; fr[i] = fr[j]; fr[j] = t;
          const uint32_t u = cd[i]; cd[i] = cd[j]; cd[j] = u;
        }
      };
      cswap(0, 1);
      cswap(1, 2);
      cswap(0, 1);
      const uint32_t code = cd[0] | cd[1] << 3 | cd[2] << 6;
      auto term = [&](int i, int r) { return r > 0 ? nr[i] : (r < 0 ? fr[i] : 0.0f); };
      auto thresh = [&]() { return __double2float_ru(best) * (1.0f + 0x1p-20f); };
      auto list = [&](int k0, int k1) {  // the cells k0..k1-1 admitted by the current best
        const float bt = thresh();
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < 26; ++k)
          if (k >= k0 && k < k1 &&
              (term(0, shift_axis(kRel0P, kRel0N, k)) + term(1, shift_axis(kRel1P, kRel1N, k))) +
                      term(2, shift_axis(kRel2P, kRel2N, k)) <= bt)
            m |= 1u << k;
        return m;
      };
      uint32_t todo = list(0, kRelNear);
      n_list += __popc(todo);
      bool far_listed = false;
      for (;;) {
        // this lane's next admitted cell (bounds re-checked against the current best)
        int k = -1;
        for (;;) {
          if (!todo) {
            if (far_listed || thresh() < fminf(fminf(fr[0], fr[1]), fr[2])) break;  // no far-side cell can win
            far_listed = true;
            todo = list(kRelNear, 26);
            n_list += __popc(todo);
            continue;
          }
          const int kk = __ffs(todo) - 1;
          todo &= todo - 1;
          const int r0 = shift_axis(kRel0P, kRel0N, kk), r1 = shift_axis(kRel1P, kRel1N, kk),
                    r2 = shift_axis(kRel2P, kRel2N, kk);
          if ((term(0, r0) + term(1, r1)) + term(2, r2) <= thresh()) {
            k = kk;
            break;
          }
        }
        if (k < 0) break;
        ++n_iter;
        // back to grid axes
        int d[3] = {0, 0, 0};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const uint32_t c = code >> (3 * i);
          const int r = shift_axis(i == 0 ? kRel0P : (i == 1 ? kRel1P : kRel2P),
                                   i == 0 ? kRel0N : (i == 1 ? kRel1N : kRel2N), k);
          const int q = (c & 4u) ? -r : r;
          const uint32_t a3 = c & 3u;
          d[0] += a3 == 0 ? q : 0;
          d[1] += a3 == 1 ? q : 0;
          d[2] += a3 == 2 ? q : 0;
        }
        const int dx = d[0], dy = d[1], dz = d[2];
        uint32_t vf = 0, vc = 0;
        bool vd = false;
        probe(dx, dy, dz, vf, vc, vd);
        const uint32_t rk = (uint32_t)ring1_index(dx, dy, dz) << 27;  // one ring: the rank is the shift index
        if (vc <= (uint32_t)kSmallCell) {
          double4 pr[kSmallCell];
#pragma unroll
          for (int u = 0; u < kSmallCell; ++u)
            if (u < (int)vc) pr[u] = rec_at(M.pos, vf + u, M.rsh);
#pragma unroll
          for (int u = 0; u < kSmallCell; ++u)
            if (u < (int)vc) fold(pr[u], vf + u, rk);
          n_cand += vc;
        } else {
          scan_cell(vf, vc, false, dx, dy, dz, rk);
        }
      }
    }
  }
  if constexpr (kCert) {
    float v = b2;
#pragma unroll
    for (int o = 1; o < G; o <<= 1) v = fminf(v, __shfl_xor(v, o, G));
    if (b2_out) *b2_out = fminf(v, cdown(a.bound));  // records beyond the search bound were never examined
  }
}

// DENSE = false: the map has no dense cell (known from the build's pinned info word),
// so the sub-cell walk is compiled out (fewer registers, more waves in flight).
//

#include "factor_rows.hpp"

// FUSED: the match and the single-pose linearization at the SAME pose in one launch,
// for callers that only want the summed 7 x 7 system (fmx_match without counts, then
// fmx_linearize_matched at the match pose: the sharded C5 loop).  No per-query result
// is written: each lane moves its accepted match back to the map scan's frame
// (matcher.hpp:92-96) and builds the whitened row(s) a = [H_j b] / sigma of its
// PlanePoint / PointPoint (factor.cpp:30-128, gtsam.hpp:67-86, 144-170) exactly as
// k_linearize_total would from the stored results; the wave's rows go through LDS
// into v_mfma_f64_16x16x4_f64 (A^T A of 64 rows x 7 columns in 4 registers per lane),
// waves meet in LDS in a fixed order, block partials + ticket, and the last block sums
// the partials in block order (deterministic) into G + error.
struct FusedArgs {
  const double* poses;  // map scan poses [K][12] (T_i)
  double inv;           // 1 / sigma
  double* bpart;        // [block][32]
  double* gpart;        // [block group][32]
  uint32_t* gticket;    // [block group], self-resetting
  uint32_t* ticket;     // self-resetting
  double* out;          // 28 G entries + error (pinned host memory, or a device buffer to all-reduce)
  uint32_t* flag;       // completion word (null: none)
  uint32_t seq;
};
constexpr int kFzLd = 32;    // doubles per block partial (28 used)
constexpr uint32_t kFzGroup = 64;  // blocks per first-level reduction group
// Sum entry e (< 28) of n partials src[i * kFzLd + e], i in [0, n), in a fixed order:
// the block's first 9 * 28 threads take strided subsets (several loads in flight
// each), then 28 threads add the 9 subset sums in order.  Returns the sum in threads
// tid < 28 (entry tid); every thread of the block must call it.
__device__ __forceinline__ double fz_sum_partials(const double* src, uint32_t n, double (*sq)[28]) {
  constexpr int kSub = kMatchThreads / 28;
  const int tid = threadIdx.x;
  if (tid < kSub * 28) {
    const int e = tid % 28, j = tid / 28;
    double sum = 0.0;
#pragma unroll 8
    for (uint32_t b = j; b < n; b += kSub)
      sum += __longlong_as_double((long long)__hip_atomic_load(
          reinterpret_cast<const unsigned long long*>(src + (size_t)b * kFzLd + e), __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_AGENT));
    sq[j][e] = sum;
  }
  __syncthreads();
  double sum = 0.0;
  if (tid < 28) {
    sum = sq[0][tid];
#pragma unroll
    for (int j = 1; j < kSub; ++j) sum += sq[j][tid];
  }
  __syncthreads();
  return sum;
}
constexpr int kFzStride = 7;  // doubles per staged row
typedef double f64x4 __attribute__((ext_vector_type(4)));

// sum over the wave's 64 staged rows of a a^T (7 x 7 in the top-left of a 16 x 16 MFMA
// tile): lane l feeds a_{4t + l/16}[l % 16] (0 past column 6) as both operands of MFMA t
__device__ __forceinline__ void fz_stage_mfma(double* __restrict__ rows, const double (&av)[7], bool valid,
                                              f64x4 (&acc)[2]) {
  const int lane = lane_id();
  double* mine = rows + lane * kFzStride;
#pragma unroll
  for (int i = 0; i < 7; ++i) mine[i] = valid ? av[i] : 0.0;
  __builtin_amdgcn_wave_barrier();
  const int col = lane & 15;
  const double* src = rows + (lane >> 4) * kFzStride + (col < 7 ? col : 0);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    double v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = src[4 * (8 * h + t) * kFzStride];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const double x = col < 7 ? v[t] : 0.0;
      acc[t & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, acc[t & 1], 0, 0, 0);
    }
  }
  __builtin_amdgcn_wave_barrier();
}

// The result of query q (one lane): the match moved back to its scan's frame
// (matcher.hpp:92-96), acceptance (:103-105), insert decision (map.tpp:160-163); the
// query-order outputs are stored, the insert flag returned and the pair (-1: none) set.
__device__ __forceinline__ bool match_result(const MatchArgs& a, const MapView& M, bool planar, uint32_t q, double best,
                                             uint32_t best_i, uint32_t sg, const double* __restrict__ inv_poses,
                                             int32_t* __restrict__ m_pair, double* __restrict__ m_d2,
                                             double4* __restrict__ m_pi, double4* __restrict__ m_ni,
                                             uint8_t* __restrict__ m_ins, int32_t& pair_out, bool cert = false) {
  const bool found = best_i != 0xFFFFFFFFu;
  int32_t pair = -1;
  double4 pi = make_double4(0, 0, 0, 0), ni = make_double4(0, 0, 0, 0);
  if (found) {
    // the record, its normal and its segment's inverse pose in flight together (the
    // segment came with the argmin)
    const double4 p = rec_at(M.pos, best_i, M.rsh);
    const double4 n = planar ? rec_at(M.nrm, best_i, M.rsh) : make_double4(0, 0, 0, 0);
    const double* Ti = inv_poses + 12 * sg;  // match.point.transform_in_place(pose.inverse()), matcher.hpp:95
    double o[3];
    d_xform(Ti, p.x, p.y, p.z, o);
    pi = make_double4(o[0], o[1], o[2], 0.0);
    if (planar) {
      d_rot(Ti, n.x, n.y, n.z, o);
      ni = make_double4(o[0], o[1], o[2], 0.0);
    }
    if (best < a.max_d2) pair = (int32_t)sg;
  }
  const uint32_t gq = planar ? q : a.nq_pl + q;
  m_pair[gq] = pair;
  m_d2[gq] = found ? best : DBL_MAX;
  m_pi[gq] = pi;
  if (planar) m_ni[q] = ni;
  const bool ins = !found || best > a.min_d2;
  m_ins[gq] = (ins ? 1 : 0) | (cert ? 2 : 0);  // bit 0: insert (k_insert); bit 1: settled by the warm certificate
  if (a.rec) a.rec[gq] = best_i;  // the next match's warm start
  pair_out = pair;
  return ins;
}

// The last block's bookkeeping of a match (every block's counts are in): the pair
// counts (counts mode, zeroing mcnt), the per-block insert counts scanned into k_insert
// offsets + totals, the tiled pair sort's tail.
// Per-block words ins_blk[b]: the block's insert count (bits 0-9), certified queries
// (10-19) and warm queries (20-29) — the counts fit 10 bits (<= 256 queries per block).
// Returns the launch's certified / warm totals (valid in thread 0).
constexpr uint32_t kInsMask = 0x3FFu;
__device__ __forceinline__ uint32_t blk_word(uint32_t ins, uint32_t cert, uint32_t warm) {
  return ins | cert << 10 | warm << 20;
}
__device__ __forceinline__ uint2 block_sum2(uint32_t x, uint32_t y) {
  __shared__ uint32_t s2[2][kMatchThreads / kWave];
  x = wave_sum(x);
  y = wave_sum(y);
  if (lane_id() == 0) {
    s2[0][threadIdx.x / kWave] = x;
    s2[1][threadIdx.x / kWave] = y;
  }
  __syncthreads();
  uint2 t = make_uint2(0u, 0u);
  if (threadIdx.x == 0)
    for (int i = 0; i < kMatchThreads / kWave; ++i) {
      t.x += s2[0][i];
      t.y += s2[1][i];
    }
  __syncthreads();  // s2 is read before a following call may overwrite it
  return t;
}
__device__ inline uint2 match_tail(const MatchArgs& a, uint32_t* __restrict__ mcnt, uint32_t* __restrict__ host_counts,
                                   uint32_t* __restrict__ ins_blk, uint32_t* __restrict__ ins_off,
                                   uint32_t* __restrict__ thist, const SortOut& so) {
  if (!a.sorted)
    for (int i = threadIdx.x; i < 2 * a.K; i += kMatchThreads)
      host_store(host_counts + i, __hip_atomic_exchange(mcnt + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  __shared__ uint32_t ws[kMatchThreads / kWave];
  __shared__ uint32_t s_pb[2][kTileMaxPairs + 1];  // tiled sort: per type, first row of pair k, [K] = total
  const bool tiled = a.sorted && a.tiles;
  const uint32_t nth0 = tiled ? (uint32_t)a.K * a.ntl_pl : 0u, nth1 = tiled ? (uint32_t)a.K * a.ntl_pt : 0u;
  constexpr int R = 8;
  if (FMX_TAIL_ONEPASS && max(max(a.nb_pl, a.nb_pt), max(nth0, nth1)) <= (uint32_t)(kMatchThreads * R)) {
    // every scan in one pass: the four inputs (insert counts per type, (pair, tile)
    // counts per type) in ONE round of loads, then one four-way block scan
    __shared__ uint32_t ws4[kMatchThreads / kWave][4];
    const uint32_t b = threadIdx.x * R;
    uint32_t v[4][R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const uint32_t i = b + u;
      v[0][u] = i < a.nb_pl ? __hip_atomic_load(ins_blk + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      v[1][u] = i < a.nb_pt ? __hip_atomic_load(ins_blk + a.nb_pl + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      v[2][u] = i < nth0 ? __hip_atomic_exchange(thist + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      v[3][u] = i < nth1 ? __hip_atomic_exchange(thist + nth0 + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    }
    uint32_t cs = 0, wsum = 0;  // the blocks' certified / warm counts (upper fields of ins_blk)
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        cs += (v[q][u] >> 10) & kInsMask;
        wsum += v[q][u] >> 20;
        v[q][u] &= kInsMask;
      }
    uint32_t sum[4], ex[4], tot[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sum[q] = 0;
#pragma unroll
      for (int u = 0; u < R; ++u) sum[q] += v[q][u];
    }
    block_excl_scan4(sum, ex, tot, ws4);
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const uint32_t i = b + u;
      if (i < a.nb_pl) ins_off[i] = ex[0];
      if (i < a.nb_pt) ins_off[a.nb_pl + i] = ex[1];
      ex[0] += v[0][u];
      ex[1] += v[1][u];
    }
    if (threadIdx.x == 0) {
      host_store(host_counts + 2 * a.K, tot[0]);
      host_store(host_counts + 2 * a.K + 1, tot[1]);
    }
    if (tiled) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const uint32_t ntl = t ? a.ntl_pt : a.ntl_pl, n = t ? nth1 : nth0, base = t ? nth0 : 0u;
        uint32_t e = ex[2 + t];
#pragma unroll
        for (int u = 0; u < R; ++u) {
          const uint32_t i = b + u;
          if (i < n) {
            so.hist_off[base + i] = e;
            if (i % ntl == 0) s_pb[t][i / ntl] = e;
          }
          e += v[2 + t][u];
        }
        for (int k = threadIdx.x; k < a.K; k += kMatchThreads)
          if (ntl == 0) s_pb[t][k] = 0;
        if (threadIdx.x == 0) s_pb[t][a.K] = tot[2 + t];
      }
      pair_sort_finish(a, so, host_counts, s_pb);
    }
    return block_sum2(cs, wsum);
  }
  uint32_t cs = 0, wsum = 0;
  for (uint32_t i = threadIdx.x; i < a.nb_pl + a.nb_pt; i += kMatchThreads) {
    const uint32_t x = __hip_atomic_load(ins_blk + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    cs += (x >> 10) & kInsMask;
    wsum += x >> 20;
  }
  const uint2 cw = block_sum2(cs, wsum);
  __syncthreads();
  for (int tt = 0; tt < 2; ++tt) {  // planar blocks [0, nb_pl), point blocks [nb_pl, nb)
    const uint32_t b0 = tt == 0 ? 0u : a.nb_pl, n = tt == 0 ? a.nb_pl : a.nb_pt;
    const uint32_t tot = block_scan_runs<8>(
        n, 0u,
        [&](uint32_t i) {
          return __hip_atomic_load(ins_blk + b0 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kInsMask;
        },
        [&](uint32_t i, uint32_t o) { ins_off[b0 + i] = o; }, ws);
    if (threadIdx.x == 0) host_store(host_counts + 2 * a.K + tt, tot);
  }
  if (tiled) pair_sort_tail(a, thist, so, host_counts, s_pb);
  return cw;
}

template <bool DENSE, bool FUSED = false>
__global__ __launch_bounds__(kMatchThreads) FMX_MATCH_ATTR void k_match(MatchArgs a, MapView mp, MapView mt,
                                                         const float4* __restrict__ q_pl,
                                                         const float4* __restrict__ q_pt,
                                                         const double* __restrict__ inv_poses,
                                                         int32_t* __restrict__ m_pair, double* __restrict__ m_d2,
                                                         double4* __restrict__ m_pi, double4* __restrict__ m_ni,
                                                         uint8_t* __restrict__ m_ins, uint32_t* __restrict__ hist,
                                                         uint32_t* __restrict__ work,
                                                         uint32_t* __restrict__ mcnt, uint32_t* __restrict__ mticket,
                                                         uint32_t* __restrict__ host_counts,
                                                         uint32_t* __restrict__ ins_blk, uint32_t* __restrict__ ins_off,
                                                         uint32_t* __restrict__ thist, SortOut so, FusedArgs fz) {
  extern __shared__ uint32_t s_hist[];  // [K]
  const double* Tj = a.Tj;
  const uint32_t bq = blockIdx.x;  // this workgroup's query block
  const bool planar = bq < a.nb_pl;
  const uint32_t bt = planar ? bq : bq - a.nb_pl;  // the block's index in its type
  const uint32_t qi = bt * kQPB + threadIdx.x / kGroup;  // the block's first query + the group
  const int g = threadIdx.x % kGroup;
  const uint32_t nq = planar ? a.nq_pl : a.nq_pt;
  const MapView& M = planar ? mp : mt;
  __shared__ uint32_t s_ins;
  __shared__ uint32_t s_hdr[DENSE ? kQPB : 1][kSubCells];  // dense-cell headers, one per query
  for (int k = threadIdx.x; k < a.K; k += kMatchThreads) s_hist[k] = 0;
  if (threadIdx.x == 0) s_ins = 0;
  __syncthreads();
  const uint32_t t_begin = (uint32_t)wall_clock64();
  uint32_t n_probe = 0, n_cand = 0, n_iter = 0, n_list = 0;  // (walk counts: FMX_DIAG_WALK builds only)
  auto world_query = [&](uint32_t q, double (&wq)[3]) {
    const float4 lq = planar ? q_pl[q] : q_pt[q];
    d_xform(Tj, (double)lq.x, (double)lq.y, (double)lq.z, wq);  // kp->transform(init), matcher.hpp:89
  };
  auto emit = [&](uint32_t q, double best, uint32_t best_i, uint32_t sg, bool cert) {
    int32_t pair;
    const bool ins =
        match_result(a, M, planar, q, best, best_i, sg, inv_poses, m_pair, m_d2, m_pi, m_ni, m_ins, pair, cert);
    if (ins) atomicAdd(&s_ins, 1u);
    if (pair >= 0) atomicAdd(&s_hist[pair], 1u);
  };
  double best = a.bound;
  uint32_t best_i = 0xFFFFFFFFu, best_sg = 0;
#ifdef FMX_DIAG_PHASE
  uint32_t phase[4] = {t_begin, t_begin, t_begin, t_begin};  // query loaded, passes 0..2 done
#else
  uint32_t* phase = nullptr;
#endif
#if FMX_CERT_ANY
  bool cert_q = false, warm_q = false, viol_q = false;
  float b2q = INFINITY;
#endif
  if (qi < nq) {
    double wq[3];
    world_query(qi, wq);
#ifdef FMX_DIAG_PHASE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    phase[0] = (uint32_t)wall_clock64();
#endif
    uint32_t best_rid = 0xFFFFFFFFu;
    // warm start: the earlier match's NN record of this query, at the new pose (the same
    // (dx^2 + dz^2) + dy^2 as fold); it bounds the search, it is not taken as the result
    double warm_b = INFINITY;
    const uint32_t gq = planar ? qi : a.nq_pl + qi;
    // (the fused launch keeps no warm state: compiled out there)
    constexpr bool kWarm = FMX_WARM_START && !FUSED;
    uint4 ocv = uint4{0u, 0x80000000u, 0u, 0u};
    if (kWarm && a.warm && a.cell) ocv = a.cell[gq];
    [[maybe_unused]] uint32_t warm_r = 0xFFFFFFFFu;
    if (kWarm && a.warm) {
      const uint32_t r = a.warm[gq];
      warm_r = r;
      if (r != 0xFFFFFFFFu) {
        const double4 p = rec_at(M.pos, r, M.rsh);
        const double dx = p.x - wq[0], dy = p.y - wq[1], dz = p.z - wq[2];
        const double d2 = (dx * dx + dz * dz) + dy * dy;
        if (d2 <= a.warm_lim) warm_b = d2;
#if FMX_CERT_ANY
        // the certificate: the query moved by delta since the previous match (same
        // own cell: same 27 cells); its NN then had distance d1 and every other
        // candidate >= sqrt(B2), so if sqrt(B2) - delta > d1 + delta the NN is unchanged
        // (strictly: no tie), and the search would return it again
        if ((FMX_CERT_DIAG || FMX_WARM_CERT) && a.cert_ok && a.rings == 1 && !FUSED && kGroup > 1) {
          const float4 lq = planar ? q_pl[qi] : q_pt[qi];
          double wo[3];
          d_xform(a.Tprev, (double)lq.x, (double)lq.y, (double)lq.z, wo);
          const double ex = wo[0] - p.x, ey = wo[1] - p.y, ez = wo[2] - p.z;
          const double d1o = (ex * ex + ez * ez) + ey * ey;
          const double mx = wq[0] - wo[0], my = wq[1] - wo[1], mz = wq[2] - wo[2];
          const double delta = sqrt(mx * mx + my * my + mz * mz);
          const int cx = (int)floor(wq[0] / a.w), cy = (int)floor(wq[1] / a.w), cz = (int)floor(wq[2] / a.w);
          const bool same = (int)floor(wo[0] / a.w) == cx && (int)floor(wo[1] / a.w) == cy &&
                            (int)floor(wo[2] / a.w) == cz;
          const double rb = sqrt((double)a.cert_b2[gq]) - delta;
          cert_q = same && rb > sqrt(d1o) + delta + 1e-7;
#if FMX_WARM_CERT
          // one-launch mode: a certified query (group-uniform) takes its previous NN and
          // skips the search (the search keeps a record only within the bound: d2 <= bound)
          cert_q = cert_q && d2 <= a.bound;
          if (cert_q) {
            best = d2;
            best_i = r;
            best_sg = (uint32_t)(tag_bits(p.w) >> 32);
            b2q = cdown(rb * rb);
          }
#endif
        }
#endif
      }
    }
#if FMX_WARM_CERT
    if (!cert_q)
#endif
    nn_search<kGroup, DENSE>(a, M, wq, g, s_hdr[DENSE ? threadIdx.x / kGroup : 0], best, best_rid, best_i, best_sg, n_probe,
                             n_cand, n_iter, n_list, warm_b,
#ifdef FMX_DIAG_PHASE
                             phase + 1,
#else
                             phase,
#endif
                             ocv, kWarm && a.cell && g == 0 ? a.cell + gq : nullptr
#if FMX_CERT_ANY
                             , &b2q
#endif
    );
#if FMX_CERT_ANY
    if (a.cert_b2 && g == 0 && kGroup > 1) a.cert_b2[gq] = b2q;
    warm_q = warm_r != 0xFFFFFFFFu;
    viol_q = cert_q && best_i != warm_r;
#endif
  }
  // work counters for the algorithmic-byte model and the match diagnostics (one plain
  // store per block, summed on the host): probes, candidate records, the largest
  // per-query candidate count of the block, block start / end (100 MHz wall clock)
  __shared__ uint32_t s_work[3][kMatchThreads / kWave];
  uint32_t qc = n_cand;  // this query's candidates: sum over its group
#pragma unroll
  for (int o = 1; o < kGroup; o <<= 1) qc += __shfl_xor(qc, o, 64);
#pragma unroll
  for (int o = kGroup; o < kWave; o <<= 1) qc = max(qc, (uint32_t)__shfl_xor(qc, o, 64));
  const uint32_t wp = wave_sum(n_probe), wc = wave_sum(n_cand);
  if (lane_id() == 0) {
    s_work[0][threadIdx.x / kWave] = wp;
    s_work[1][threadIdx.x / kWave] = wc;
    s_work[2][threadIdx.x / kWave] = qc;
  }
#ifdef FMX_DIAG_PHASE  // per block: the latest wave's end of each phase (ticks after the block's start)
  __shared__ uint32_t s_ph[4];
  if (threadIdx.x < 4) s_ph[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) atomicMax(&s_ph[k], phase[k] - t_begin);
#endif
#if FMX_CERT_ANY  // per block: certifiable queries, certified but changed NN (must be 0), warm queries
  __shared__ uint32_t s_cert[3];
  if (threadIdx.x < 3) s_cert[threadIdx.x] = 0;
  __syncthreads();
  if (qi < nq && g == 0) {
    if (cert_q) atomicAdd(&s_cert[0], 1u);
    if (viol_q) atomicAdd(&s_cert[1], 1u);
    if (warm_q) atomicAdd(&s_cert[2], 1u);
  }
#endif
#ifdef FMX_DIAG_WALK  // per block: sum over waves of the wave's walk rounds, lanes' walk steps, listed cells
  __shared__ uint32_t s_walk[3][kMatchThreads / kWave];
  {
    uint32_t wr = n_iter;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) wr = max(wr, (uint32_t)__shfl_xor(wr, o, 64));
    const uint32_t wi = wave_sum(n_iter), wl = wave_sum(n_list);
    if (lane_id() == 0) {
      s_walk[0][threadIdx.x / kWave] = wr;
      s_walk[1][threadIdx.x / kWave] = wi;
      s_walk[2][threadIdx.x / kWave] = wl;
    }
  }
#endif
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tp = 0, tc = 0, mq = 0;
    for (int i = 0; i < kMatchThreads / kWave; ++i) {
      tp += s_work[0][i];
      tc += s_work[1][i];
      mq = max(mq, s_work[2][i]);
    }
    uint4* w4 = reinterpret_cast<uint4*>(work) + 2 * bq;
    uint32_t d0 = 0, d1 = 0, d2 = 0;
#ifdef FMX_DIAG_WALK
    for (int i = 0; i < kMatchThreads / kWave; ++i) {
      d0 += s_walk[0][i];
      d1 += s_walk[1][i];
      d2 += s_walk[2][i];
    }
#endif
#ifdef FMX_DIAG_PHASE
    d0 = min(s_ph[0], 0xFFFFu) | min(s_ph[1], 0xFFFFu) << 16;
    d1 = min(s_ph[2], 0xFFFFu) | min(s_ph[3], 0xFFFFu) << 16;
#endif
#if FMX_CERT_ANY
    d0 = s_cert[0];
    d1 = s_cert[1];
    d2 = s_cert[2];
#endif
    const uint32_t t_end = (uint32_t)wall_clock64();
    w4[0] = make_uint4(tp, tc, mq, d0);
    w4[1] = make_uint4(t_begin, t_end, d1, d2);
    // (a profiled launch's probe / candidate totals: the last block sums these words; the
    // fused launch, whose blocks have no tail, adds them up as it goes)
    if (FUSED && a.prof_work) {
      __hip_atomic_fetch_add(a.prof_acc, tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(a.prof_acc + 1, tc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  if constexpr (!FUSED) {
#if FMX_WARM_CERT
    if (qi < nq && g == 0) emit(qi, best, best_i, best_sg, cert_q);
#else
    if (qi < nq && g == 0) emit(qi, best, best_i, best_sg, false);
#endif
  } else {
    static_assert(kGroup == 1, "the fused match + linearization runs one lane per query");
    // this lane's accepted match in its map scan's frame, then its row(s)
    const bool acc_q = qi < nq && best_i != 0xFFFFFFFFu && best < a.max_d2;
    double pi[3] = {0, 0, 0}, ni[3] = {0, 0, 0}, pj[3] = {0, 0, 0};
    const double* Ti = fz.poses;
    if (acc_q) {
      const double4 p = rec_at(M.pos, best_i, M.rsh);
      const double4 n = planar ? rec_at(M.nrm, best_i, M.rsh) : make_double4(0, 0, 0, 0);
      const uint32_t sg = best_sg;  // (with the argmin: the pose loads need not wait for p)
      const double* Tinv = inv_poses + 12 * sg;  // matcher.hpp:95
      d_xform(Tinv, p.x, p.y, p.z, pi);
      if (planar) d_rot(Tinv, n.x, n.y, n.z, ni);
      Ti = fz.poses + 12 * sg;
      const float4 lq = planar ? q_pl[qi] : q_pt[qi];
      pj[0] = (double)lq.x;
      pj[1] = (double)lq.y;
      pj[2] = (double)lq.z;
    }
    __shared__ double s_rows[kMatchThreads / kWave][kWave * kFzStride];
    __shared__ double s_g[kMatchThreads / kWave][28];
    double* rows = s_rows[threadIdx.x / kWave];
    f64x4 accs[2] = {f64x4{0.0, 0.0, 0.0, 0.0}, f64x4{0.0, 0.0, 0.0, 0.0}};
    double H[12], av[7];
#pragma unroll
    for (int i = 0; i < 12; ++i) H[i] = 0.0;
#ifdef FMX_DIAG_NOEPI  // diagnostic build: no rows (instruction-count split of the kernel)
    accs[0][0] = acc_q ? 1e-300 * (pi[0] + ni[0] + Ti[0]) : 0.0;
#else
    if (planar) {  // block-uniform: a block holds one feature type
      double r = 0.0;
      if (acc_q) plane_row<1>(Ti, Tj, pi, ni, pj, r, H);
#pragma unroll
      for (int c = 0; c < 6; ++c) av[c] = H[6 + c] * fz.inv;
      av[6] = -r * fz.inv;
      fz_stage_mfma(rows, av, acc_q, accs);
    } else {
      double wpi[3], wpj[3];
      d_xform(Ti, pi[0], pi[1], pi[2], wpi);
      d_xform(Tj, pj[0], pj[1], pj[2], wpj);
      for (int ax = 0; ax < 3; ++ax) {
        double r = 0.0;
        if (acc_q) point_row<1>(Ti, Tj, pi, pj, wpi, wpj, ax, r, H);
#pragma unroll
        for (int c = 0; c < 6; ++c) av[c] = H[6 + c] * fz.inv;
        av[6] = -r * fz.inv;
        fz_stage_mfma(rows, av, acc_q, accs);
      }
    }
#endif
    const f64x4 acc = accs[0] + accs[1];
    {
      const int col = lane_id() & 15;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane_id() >> 4) + 4 * r;
        if (rr <= col && col < 7) s_g[threadIdx.x / kWave][rr * 7 - rr * (rr - 1) / 2 + (col - rr)] = acc[r];
      }
    }
    __syncthreads();
    const int tid = threadIdx.x;
    if (tid < 28) {
      double bp = s_g[0][tid];
#pragma unroll
      for (int i = 1; i < kMatchThreads / kWave; ++i) bp += s_g[i][tid];
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(fz.bpart + (size_t)blockIdx.x * kFzLd + tid),
                         (unsigned long long)__double_as_longlong(bp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // two-level deterministic reduction: the last block of each group of kFzGroup
    // blocks sums the group's partials (block order), the last group finisher sums the
    // group partials (group order) into G + error
    __shared__ int s_flast;
    __shared__ double s_q[kMatchThreads / 28][28];
    const uint32_t grp = blockIdx.x / kFzGroup, ngrp = (gridDim.x + kFzGroup - 1) / kFzGroup;
    const uint32_t gsize = min(kFzGroup, gridDim.x - grp * kFzGroup);
    if (tid == 0)
      s_flast = __hip_atomic_fetch_add(fz.gticket + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1;
    __syncthreads();
    if (!s_flast) return;
    const double gs = fz_sum_partials(fz.bpart + (size_t)grp * kFzGroup * kFzLd, gsize, s_q);
    if (tid < 28)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(fz.gpart + (size_t)grp * kFzLd + tid),
                         (unsigned long long)__double_as_longlong(gs), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_store(fz.gticket + grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_flast = __hip_atomic_fetch_add(fz.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngrp - 1;
    }
    __syncthreads();
    if (!s_flast) return;
    const double tot = fz_sum_partials(fz.gpart, ngrp, s_q);
    if (tid < 28) {
#ifdef FMX_DIAG_NOEPI  // keep the diagnostic build's system solvable
      host_store(fz.out + tid, tot + (tid == 0 || tid == 7 || tid == 13 || tid == 18 || tid == 22 || tid == 25 ? 1.0 : 0.0));
#else
      host_store(fz.out + tid, tot);
#endif
      if (tid == 27) host_store(fz.out + 28, 0.5 * tot);  // error = 0.5 ||r / sigma||^2
    }
    if (tid == 0) {
      if (a.prof_work) {  // the launch's probes / candidates -> its profiler slot
        host_store(a.prof_work, __hip_atomic_exchange(a.prof_acc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        host_store(a.prof_work + 1, __hip_atomic_exchange(a.prof_acc + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
      __hip_atomic_store(fz.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (fz.flag) publish_flag(fz.flag, fz.seq);  // fz.out was stored by this wave (threads 0..27)
    }
    return;
  }
  __syncthreads();  // every emit's LDS counts are in
  // this block's insert count (k_insert offsets) and certified / warm queries, one
  // agent-visible word summed by the last block (per-block adds into one launch-wide
  // counter measured +9 us per C4 launch: every block's atomic on the same address)
#if FMX_CERT_ANY
  if (threadIdx.x == 0)
    __hip_atomic_store(ins_blk + bq, blk_word(s_ins, s_cert[0], s_cert[2]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  if (threadIdx.x == 0) __hip_atomic_store(ins_blk + bq, s_ins, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
  const int t = planar ? 0 : 1;
  if (a.sorted && a.tiles) {
    // per-(type, pair, tile) counts: agent-scope adds, scanned by the last block
    const size_t hbase = planar ? (size_t)0 : (size_t)a.K * a.ntl_pl;
    const uint32_t ntl = planar ? a.ntl_pl : a.ntl_pt;
    const uint32_t tile = bt / kTileBlocks;
    for (int k = threadIdx.x; k < a.K; k += kMatchThreads)
      if (s_hist[k])
        __hip_atomic_fetch_add(thist + hbase + (size_t)k * ntl + tile, s_hist[k], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    // block 0 clears the other half of the count table for the next tiled match on this
    // set (what read it — this set's previous scatter or last block — ran before this
    // launch, in stream order)
    if (blockIdx.x == 0)
      for (uint32_t i = threadIdx.x; i < a.thist_clear_n; i += kMatchThreads) a.thist_clear[i] = 0u;
    // kTilesScatter: no last block — the pair scatter scans the counts
    // (k_pair_scatter_s), so the launch ends with its last query block
    if (a.tiles == kTilesScatter) return;
  } else if (a.sorted) {
    // pair-major layout [type][pair][block]: one exclusive scan gives every block's
    // destination offset (k_pair_base / k_pair_scatter)
    const size_t hbase = planar ? (size_t)0 : (size_t)a.K * a.nb_pl;
    const uint32_t nbt = planar ? a.nb_pl : a.nb_pt;
    for (int k = threadIdx.x; k < a.K; k += kMatchThreads) hist[hbase + (size_t)k * nbt + bt] = s_hist[k];
  } else {
    // counts only: agent-scope adds into mcnt[type][pair]
    for (int k = threadIdx.x; k < a.K; k += kMatchThreads)
      if (s_hist[k])
        __hip_atomic_fetch_add(mcnt + (size_t)t * a.K + k, s_hist[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // a ticket per block (its agent-scope stores / adds are complete first: vmcnt(0) +
  // barrier); the last block publishes the pair counts (counts mode, zeroing mcnt
  // for the next launch) and scans the per-block insert counts into offsets + totals
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int s_last;
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(mticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  const uint2 cw = match_tail(a, mcnt, host_counts, ins_blk, ins_off, thist, so);
  uint2 pc = make_uint2(0u, 0u);
  if (a.prof_work) {  // profiled: the blocks' probe / candidate words, summed
    uint32_t tp = 0, tc = 0;
    for (uint32_t b = threadIdx.x; b < gridDim.x; b += kMatchThreads) {
      tp += __hip_atomic_load(work + kWorkWords * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tc += __hip_atomic_load(work + kWorkWords * b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    pc = block_sum2(tp, tc);
  }
  if (threadIdx.x == 0) {  // certified / warm queries of this launch -> host
    host_store(host_counts + 2 * a.K + 2, cw.x);
    host_store(host_counts + 2 * a.K + 3, cw.y);
    if (a.prof_work) {  // the launch's probes / candidates / certified / warm -> its profiler slot
      host_store(a.prof_work, pc.x);
      host_store(a.prof_work + 1, pc.y);
      host_store(a.prof_work + 2, cw.x);
      host_store(a.prof_work + 3, cw.y);
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(mticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct HistIn {
  const uint32_t* h;
  __device__ uint32_t operator()(size_t i) const { return h[i]; }
};
struct HistOut {
  uint32_t* o;
  __device__ void operator()(size_t i, uint32_t v) const { o[i] = v; }
};

// One block: from the scanned pair-major histogram, per-pair counts and first rows
// (per type), host copy of the counts, and the linearize chunk table (pair-major:
// plane chunks then point chunks of each pair).
__global__ __launch_bounds__(1024) void k_pair_base(int K, uint32_t nb_pl, uint32_t nb_pt,
                                                    const uint32_t* __restrict__ hoff, const uint32_t* __restrict__ total,
                                                    uint32_t* __restrict__ pair_counts, uint32_t* __restrict__ pair_base,
                                                    uint32_t* __restrict__ chunk_range, Chunk* __restrict__ chunks,
                                                    uint32_t* __restrict__ n_chunks,
                                                    uint32_t* __restrict__ host_counts) {
  __shared__ uint32_t ws[16];
  __shared__ uint32_t carry;
  const size_t npl_all = (size_t)K * nb_pl, n_all = npl_all + (size_t)K * nb_pt;
  // start offset of section (t, k) in the scanned array; sections of empty types
  // (nb = 0) start where the next section starts
  auto sec = [&](int t, int k) -> uint32_t {
    const size_t i = t == 0 ? (size_t)k * nb_pl : npl_all + (size_t)k * nb_pt;
    return i < n_all ? hoff[i] : *total;
  };
  const uint32_t tot_pl = K > 0 ? sec(1, 0) : 0u;  // planar total = start of the point part
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int k0 = 0; k0 < K; k0 += 1024) {
    const int k = k0 + threadIdx.x;
    uint32_t npl = 0, npt = 0, b_pl = 0, b_pt = 0;
    if (k < K) {
      b_pl = sec(0, k);
      const uint32_t e_pl = k + 1 < K ? sec(0, k + 1) : tot_pl;
      b_pt = sec(1, k);
      const uint32_t e_pt = k + 1 < K ? sec(1, k + 1) : *total;
      npl = e_pl - b_pl;
      npt = e_pt - b_pt;
      b_pt -= tot_pl;
      pair_counts[k] = npl;
      pair_counts[K + k] = npt;
      host_store(host_counts + k, npl);  // mapped host memory
      host_store(host_counts + K + k, npt);
      pair_base[k] = b_pl;
      pair_base[K + k] = b_pt;
    }
    const uint32_t nch = (npl + kPlaneChunk - 1) / kPlaneChunk + (npt + kPointChunk - 1) / kPointChunk;
    const uint32_t incl = wave_incl_scan(nch);
    const int w = threadIdx.x / kWave;
    if (lane_id() == 63) ws[w] = incl;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int i = 0; i < 16; ++i) {
      if (i < w) off += ws[i];
      tot += ws[i];
    }
    if (k < K) chunk_range[k] = carry + off + incl - nch;
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) chunk_range[K] = carry;
  __syncthreads();
  // descriptors, every thread a strided share: chunk -> pair by binary search
  const uint32_t nch_all = carry;
  for (uint32_t ci = threadIdx.x; ci < nch_all; ci += 1024) {
    int lo = 0, hi = K - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (chunk_range[mid] <= ci) lo = mid;
      else hi = mid - 1;
    }
    const int k = lo;
    const uint32_t j = ci - chunk_range[k];
    const uint32_t npl = pair_counts[k], npt = pair_counts[K + k];
    const uint32_t ncpl = (npl + kPlaneChunk - 1) / kPlaneChunk;
    if (j < ncpl) {
      const uint32_t r = j * kPlaneChunk, b_pl = pair_base[k];
      chunks[ci] = Chunk{0, (uint32_t)k, b_pl + r, b_pl + min(npl, r + kPlaneChunk)};
    } else {
      const uint32_t r = (j - ncpl) * kPointChunk, b_pt = pair_base[K + k];
      chunks[ci] = Chunk{1, (uint32_t)k, b_pt + r, b_pt + min(npt, r + kPointChunk)};
    }
  }
  if (threadIdx.x == 0) *n_chunks = nch_all;
}

// Stable scatter of accepted matches into pair-major SoA correspondences:
// one (partial) wave per match block (kQPB queries), rank by ballot within the wave
// (only the g8 build runs it: match_group_for).
__global__ __launch_bounds__(kQPB) void k_pair_scatter(uint32_t nq_pl, uint32_t nq_pt, uint32_t nb_pl, int K,
                                                     const int32_t* __restrict__ m_pair,
                                                     const double4* __restrict__ m_pi,
                                                     const double4* __restrict__ m_ni,
                                                     const float4* __restrict__ q_pl,
                                                     const float4* __restrict__ q_pt,
                                                     const uint32_t* __restrict__ hist_off,
                                                     uint32_t nb_pt, const uint32_t* __restrict__ pair_base,
                                                     double* __restrict__ c_pl, size_t ld_pl,
                                                     double* __restrict__ c_pt, size_t ld_pt) {
  const bool planar = blockIdx.x < nb_pl;
  const uint32_t qi = (planar ? blockIdx.x : blockIdx.x - nb_pl) * kQPB + threadIdx.x;
  const uint32_t nq = planar ? nq_pl : nq_pt;
  const int32_t pair = qi < nq ? m_pair[planar ? qi : nq_pl + qi] : -1;
  uint32_t rank = 0;
  bool todo = pair >= 0;
  while (__ballot(todo)) {
    const int lead = __ffsll((unsigned long long)__ballot(todo)) - 1;
    const int v = __shfl(pair, lead, 64);
    const uint64_t m = __ballot(todo && pair == v);
    if (todo && pair == v) {
      rank = __popcll(m & lanemask_lt());
      todo = false;
    }
  }
  if (pair < 0) return;
  const int t = planar ? 0 : 1;
  // pair-major scanned histogram; the point part is relative to the planar total
  const size_t npl_all = (size_t)K * nb_pl;
  const uint32_t tot_pl = nb_pt ? hist_off[npl_all] : 0u;  // exclusive prefix at the point section = planar total
  const uint32_t dst = planar ? hist_off[(size_t)pair * nb_pl + blockIdx.x] + rank
                              : hist_off[npl_all + (size_t)pair * nb_pt + (blockIdx.x - nb_pl)] - tot_pl + rank;
  (void)pair_base;
  (void)t;
  const size_t gq = planar ? qi : nq_pl + qi;
  const double4 pi = m_pi[gq];
  if (planar) {
    const double4 ni = m_ni[qi];
    const float4 pj = q_pl[qi];
    c_pl[0 * ld_pl + dst] = pi.x; c_pl[1 * ld_pl + dst] = pi.y; c_pl[2 * ld_pl + dst] = pi.z;
    c_pl[3 * ld_pl + dst] = ni.x; c_pl[4 * ld_pl + dst] = ni.y; c_pl[5 * ld_pl + dst] = ni.z;
    c_pl[6 * ld_pl + dst] = (double)pj.x; c_pl[7 * ld_pl + dst] = (double)pj.y;
    c_pl[8 * ld_pl + dst] = (double)pj.z;
  } else {
    const float4 pj = q_pt[qi];
    c_pt[0 * ld_pt + dst] = pi.x; c_pt[1 * ld_pt + dst] = pi.y; c_pt[2 * ld_pt + dst] = pi.z;
    c_pt[3 * ld_pt + dst] = (double)pj.x; c_pt[4 * ld_pt + dst] = (double)pj.y;
    c_pt[5 * ld_pt + dst] = (double)pj.z;
  }
}

// Tiled stable scatter: one 1024-thread block per tile (kTileBlocks match blocks of
// one type); a query's row = its (pair, tile) offset + the matches of that pair in
// earlier waves of the tile + its ballot rank in its wave.  Query order within a pair.
__global__ __launch_bounds__(kTileQ) void k_pair_scatter_t(uint32_t nq_pl, uint32_t nq_pt, uint32_t ntl_pl,
                                                         uint32_t ntl_pt, int K, const int32_t* __restrict__ m_pair,
                                                         const double4* __restrict__ m_pi,
                                                         const double4* __restrict__ m_ni,
                                                         const float4* __restrict__ q_pl,
                                                         const float4* __restrict__ q_pt,
                                                         const uint32_t* __restrict__ hist_off,
                                                         double* __restrict__ c_pl, size_t ld_pl,
                                                         double* __restrict__ c_pt, size_t ld_pt) {
  __shared__ uint32_t s_cnt[kTileQ / kWave][kTileMaxPairs];
  __shared__ uint32_t s_hoff[kTileMaxPairs];
  const bool planar = blockIdx.x < ntl_pl;
  const uint32_t tile = planar ? blockIdx.x : blockIdx.x - ntl_pl;
  const uint32_t qi = tile * kTileQ + threadIdx.x;
  const uint32_t nq = planar ? nq_pl : nq_pt;
  const int w = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < (kTileQ / kWave) * K; i += kTileQ) s_cnt[i / K][i % K] = 0;
  // every load up front, in one round: the row's fields with its pair, and the tile's
  // (pair, tile) offsets for every pair (to LDS; the ranking and the per-wave scan run
  // while they fly)
  for (int k = threadIdx.x; k < K; k += kTileQ)
    s_hoff[k] = hist_off[planar ? (size_t)k * ntl_pl + tile : (size_t)K * ntl_pl + (size_t)k * ntl_pt + tile];
  const size_t gq = planar ? qi : nq_pl + qi;
  const bool in = qi < nq;
  const int32_t pair = in ? m_pair[gq] : -1;
  const double4 pi = in ? m_pi[gq] : make_double4(0, 0, 0, 0);
  const double4 ni = in && planar ? m_ni[qi] : make_double4(0, 0, 0, 0);
  const float4 pj = in ? (planar ? q_pl[qi] : q_pt[qi]) : make_float4(0, 0, 0, 0);
  __syncthreads();
  uint32_t rank = 0;
  bool todo = pair >= 0;
  while (__ballot(todo)) {
    const int lead = __ffsll((unsigned long long)__ballot(todo)) - 1;
    const int v = __shfl(pair, lead, 64);
    const uint64_t m = __ballot(todo && pair == v);
    if (todo && pair == v) {
      rank = __popcll(m & lanemask_lt());
      todo = false;
    }
    if (lane_id() == lead) s_cnt[w][v] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += kTileQ) {  // per pair: exclusive scan over the waves
    uint32_t run = 0;
#pragma unroll
    for (int i = 0; i < kTileQ / kWave; ++i) {
      const uint32_t c = s_cnt[i][k];
      s_cnt[i][k] = run;
      run += c;
    }
  }
  __syncthreads();
  if (pair < 0) return;
  const uint32_t dst = s_hoff[pair] + s_cnt[w][pair] + rank;
  if (planar) {
    c_pl[0 * ld_pl + dst] = pi.x; c_pl[1 * ld_pl + dst] = pi.y; c_pl[2 * ld_pl + dst] = pi.z;
    c_pl[3 * ld_pl + dst] = ni.x; c_pl[4 * ld_pl + dst] = ni.y; c_pl[5 * ld_pl + dst] = ni.z;
    c_pl[6 * ld_pl + dst] = (double)pj.x; c_pl[7 * ld_pl + dst] = (double)pj.y;
    c_pl[8 * ld_pl + dst] = (double)pj.z;
  } else {
    c_pt[0 * ld_pt + dst] = pi.x; c_pt[1 * ld_pt + dst] = pi.y; c_pt[2 * ld_pt + dst] = pi.z;
    c_pt[3 * ld_pt + dst] = (double)pj.x; c_pt[4 * ld_pt + dst] = (double)pj.y;
    c_pt[5 * ld_pt + dst] = (double)pj.z;
  }
}

// ---- the tiled pair sort without a match tail (kTilesScatter)
// Exclusive scan of one value per thread over an NT-thread block; total returned.
template <int NT>
__device__ __forceinline__ uint32_t blk_excl_scan(uint32_t v, uint32_t* ws, uint32_t& total) {
  const uint32_t incl = wave_incl_scan(v);
  const int w = threadIdx.x / kWave;
  if (lane_id() == kWave - 1) ws[w] = incl;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / kWave; ++i) {
    const uint32_t x = ws[i];
    off += i < w ? x : 0u;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return off + incl - v;
}

struct ScatterArgs {
  uint32_t nq_pl, nq_pt, ntl_pl, ntl_pt;
  int K;
  const int32_t* m_pair;
  const double4* m_pi;
  const double4* m_ni;
  const float4* q_pl;
  const float4* q_pt;
  const uint32_t* thist;  // [type][pair][tile] match counts: [0, K ntl_pl) planar, then point
  double* c_pl;
  size_t ld_pl;
  double* c_pt;
  size_t ld_pt;
  // the meta block's outputs: per-pair counts / first rows [type][K], the window chunk
  // table, the pinned host copy (pair counts, insert totals, certified / warm queries)
  uint32_t* pair_counts;
  uint32_t* pair_base;
  uint32_t* chunk_range;
  Chunk* chunks;
  uint32_t* n_chunks;
  uint32_t* host_counts;
  const uint32_t* ins_blk;  // per match block: insert count | certified << 10 | warm << 20
  uint32_t* ins_off;        // -> k_insert offsets (per type, from 0)
  uint32_t nb_pl, nb_pt;
  const uint32_t* work;  // profiled launches: per-match-block work words (probes, candidates) ...
  uint32_t* prof_work;   // ... summed into the launch's profiler slot (null: not profiled)
};

// Sum over tiles of row k of a [pair][tile] count table in LDS (one wave; every lane
// returns the totals): *pre = the tiles before `tile`.
__device__ __forceinline__ uint32_t tile_row_sum(const uint32_t* tab, uint32_t ntl, uint32_t tile, uint32_t& pre) {
  uint32_t t = 0, p = 0;
  for (uint32_t t0 = 0; t0 < ntl; t0 += kWave) {
    const uint32_t i = t0 + lane_id();
    const uint32_t v = i < ntl ? tab[i] : 0u;
    t += v;
    p += i < tile ? v : 0u;
  }
  pre = wave_sum(p);
  return wave_sum(t);
}

// The meta block of k_pair_scatter_s (the grid's last): what the match's last block did
// for kTilesTail — per-pair counts and first rows, the window chunk table, insert
// offsets — running beside the tile blocks instead of after every query block.
__device__ void scatter_meta(const ScatterArgs& a, uint32_t* s_tab) {
  constexpr int NT = kTileQ, NW = NT / kWave;
  __shared__ uint32_t ws[NW];
  __shared__ uint32_t s_tot[2][kTileMaxPairs];
  __shared__ uint32_t s_cr[kTileMaxPairs + 1];
  __shared__ uint32_t s_cw[NW][4];
  const int K = a.K, w = threadIdx.x / kWave, lane = lane_id();
  const uint32_t n0 = (uint32_t)K * a.ntl_pl, n = n0 + (uint32_t)K * a.ntl_pt;
  for (uint32_t i = threadIdx.x; i < n; i += NT) s_tab[i] = a.thist[i];
  // the launch's certified / warm queries and (profiled) probes / candidates, in the
  // same round of loads
  const uint32_t nb = a.nb_pl + a.nb_pt;
  uint32_t cs = 0, wm = 0, tp = 0, tc = 0;
  for (uint32_t b = threadIdx.x; b < nb; b += NT) {
    const uint32_t x = a.ins_blk[b];
    cs += (x >> 10) & 0x3FFu;
    wm += x >> 20;
    if (a.prof_work) {
      tp += a.work[kWorkWords * b];
      tc += a.work[kWorkWords * b + 1];
    }
  }
  cs = wave_sum(cs);
  wm = wave_sum(wm);
  tp = wave_sum(tp);
  tc = wave_sum(tc);
  if (lane == 0) {
    s_cw[w][0] = cs;
    s_cw[w][1] = wm;
    s_cw[w][2] = tp;
    s_cw[w][3] = tc;
  }
  __syncthreads();
  for (int it = w; it < 2 * K; it += NW) {  // per (type, pair): its total over the tiles
    const int t = it / K, k = it % K;
    const uint32_t ntl = t ? a.ntl_pt : a.ntl_pl;
    uint32_t pre;
    const uint32_t tot = tile_row_sum(s_tab + (t ? n0 : 0u) + (uint32_t)k * ntl, ntl, 0u, pre);
    if (lane == 0) s_tot[t][k] = tot;
  }
  __syncthreads();
  // per pair: counts (device + host), first rows per type, chunks (plane then point)
  uint32_t carry_pl = 0, carry_pt = 0, carry_ch = 0;
  for (int k0 = 0; k0 < K; k0 += NT) {
    const int k = k0 + threadIdx.x;
    const uint32_t npl = k < K ? s_tot[0][k] : 0u, npt = k < K ? s_tot[1][k] : 0u;
    const uint32_t nch = (npl + kPlaneChunk - 1) / kPlaneChunk + (npt + kPointChunk - 1) / kPointChunk;
    uint32_t t0, t1, t2;
    const uint32_t b_pl = carry_pl + blk_excl_scan<NT>(npl, ws, t0);
    const uint32_t b_pt = carry_pt + blk_excl_scan<NT>(npt, ws, t1);
    const uint32_t b_ch = carry_ch + blk_excl_scan<NT>(nch, ws, t2);
    if (k < K) {
      a.pair_counts[k] = npl;
      a.pair_counts[K + k] = npt;
      a.pair_base[k] = b_pl;
      a.pair_base[K + k] = b_pt;
      host_store(a.host_counts + k, npl);  // mapped host memory
      host_store(a.host_counts + K + k, npt);
      s_cr[k] = b_ch;
      s_tot[0][k] = b_pl;  // (first rows, for the descriptors below)
      s_tot[1][k] = b_pt;
    }
    carry_pl += t0;
    carry_pt += t1;
    carry_ch += t2;
  }
  if (threadIdx.x == 0) s_cr[K] = carry_ch;
  __syncthreads();
  for (int k = threadIdx.x; k <= K; k += NT) a.chunk_range[k] = s_cr[k];
  for (uint32_t ci = threadIdx.x; ci < carry_ch; ci += NT) {  // chunk -> pair by binary search
    int lo = 0, hi = K - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_cr[mid] <= ci) lo = mid;
      else hi = mid - 1;
    }
    const int k = lo;
    const uint32_t j = ci - s_cr[k];
    const uint32_t b_pl = s_tot[0][k], b_pt = s_tot[1][k];
    const uint32_t e_pl = k + 1 < K ? s_tot[0][k + 1] : carry_pl, e_pt = k + 1 < K ? s_tot[1][k + 1] : carry_pt;
    const uint32_t cpl = e_pl - b_pl, cpt = e_pt - b_pt;
    const uint32_t ncpl = (cpl + kPlaneChunk - 1) / kPlaneChunk;
    if (j < ncpl) {
      const uint32_t r = j * kPlaneChunk;
      a.chunks[ci] = Chunk{0, (uint32_t)k, b_pl + r, b_pl + min(cpl, r + kPlaneChunk)};
    } else {
      const uint32_t r = (j - ncpl) * kPointChunk;
      a.chunks[ci] = Chunk{1, (uint32_t)k, b_pt + r, b_pt + min(cpt, r + kPointChunk)};
    }
  }
  if (threadIdx.x == 0) *a.n_chunks = carry_ch;
  // insert offsets per type (k_insert), from each type's first block
  for (int t = 0; t < 2; ++t) {
    const uint32_t b0 = t ? a.nb_pl : 0u, nbt = t ? a.nb_pt : a.nb_pl;
    uint32_t carry = 0;
    for (uint32_t i0 = 0; i0 < nbt; i0 += NT) {
      const uint32_t i = i0 + threadIdx.x;
      const uint32_t v = i < nbt ? a.ins_blk[b0 + i] & 0x3FFu : 0u;
      uint32_t tot;
      const uint32_t ex = carry + blk_excl_scan<NT>(v, ws, tot);
      if (i < nbt) a.ins_off[b0 + i] = ex;
      carry += tot;
    }
    if (threadIdx.x == 0) host_store(a.host_counts + 2 * K + t, carry);
  }
  if (threadIdx.x == 0) {
    uint32_t c4[4] = {0, 0, 0, 0};
    for (int i = 0; i < NW; ++i)
      for (int q = 0; q < 4; ++q) c4[q] += s_cw[i][q];
    host_store(a.host_counts + 2 * K + 2, c4[0]);
    host_store(a.host_counts + 2 * K + 3, c4[1]);
    if (a.prof_work) {  // the launch's probes / candidates / certified / warm -> its profiler slot
      host_store(a.prof_work, c4[2]);
      host_store(a.prof_work + 1, c4[3]);
      host_store(a.prof_work + 2, c4[0]);
      host_store(a.prof_work + 3, c4[1]);
    }
  }
}

// Tiled stable scatter for kTilesScatter: tile blocks as k_pair_scatter_t, each finding
// its own (pair, tile) offsets from the match's count table (its type's table to LDS in
// the same round of loads as its rows; a wave per pair sums the pair's tiles and those
// before this one; the pairs' first rows by one exclusive scan of the totals), plus the
// meta block (scatter_meta).  Query order within a pair, deterministic.
__global__ __launch_bounds__(kTileQ) void k_pair_scatter_s(ScatterArgs a) {
  constexpr int NW = kTileQ / kWave;
  __shared__ uint32_t s_tab[kScatterTab];
  __shared__ uint32_t s_cnt[NW][kTileMaxPairs];
  __shared__ uint32_t s_pre[kTileMaxPairs], s_tot[kTileMaxPairs];
  const uint32_t ntiles = a.ntl_pl + a.ntl_pt;
  if (blockIdx.x == ntiles) {
    scatter_meta(a, s_tab);
    return;
  }
  const int K = a.K;
  const bool planar = blockIdx.x < a.ntl_pl;
  const uint32_t tile = planar ? blockIdx.x : blockIdx.x - a.ntl_pl;
  const uint32_t ntl = planar ? a.ntl_pl : a.ntl_pt;
  const uint32_t qi = tile * kTileQ + threadIdx.x;
  const uint32_t nq = planar ? a.nq_pl : a.nq_pt;
  const int w = threadIdx.x / kWave, lane = lane_id();
  // every load up front, in one round: the type's count table, the row's fields
  const uint32_t* tab = a.thist + (planar ? 0u : (uint32_t)K * a.ntl_pl);
  for (uint32_t i = threadIdx.x; i < (uint32_t)K * ntl; i += kTileQ) s_tab[i] = tab[i];
  for (int i = threadIdx.x; i < NW * K; i += kTileQ) s_cnt[i / K][i % K] = 0;
  const size_t gq = planar ? qi : a.nq_pl + qi;
  const bool in = qi < nq;
  const int32_t pair = in ? a.m_pair[gq] : -1;
  const double4 pi = in ? a.m_pi[gq] : make_double4(0, 0, 0, 0);
  const double4 ni = in && planar ? a.m_ni[qi] : make_double4(0, 0, 0, 0);
  const float4 pj = in ? (planar ? a.q_pl[qi] : a.q_pt[qi]) : make_float4(0, 0, 0, 0);
  __syncthreads();
  // per pair: its total and its matches in earlier tiles
  for (int k = w; k < K; k += NW) {
    uint32_t pre;
    const uint32_t tot = tile_row_sum(s_tab + (uint32_t)k * ntl, ntl, tile, pre);
    if (lane == 0) {
      s_tot[k] = tot;
      s_pre[k] = pre;
    }
  }
  uint32_t rank = 0;
  bool todo = pair >= 0;
  while (__ballot(todo)) {
    const int lead = __ffsll((unsigned long long)__ballot(todo)) - 1;
    const int v = __shfl(pair, lead, 64);
    const uint64_t m = __ballot(todo && pair == v);
    if (todo && pair == v) {
      rank = __popcll(m & lanemask_lt());
      todo = false;
    }
    if (lane == lead) s_cnt[w][v] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (w == 0) {  // the pairs' first rows (exclusive scan of the totals) + this tile's offsets
    uint32_t carry = 0;
    for (int k0 = 0; k0 < K; k0 += kWave) {
      const int k = k0 + lane;
      const uint32_t v = k < K ? s_tot[k] : 0u;
      const uint32_t incl = wave_incl_scan(v);
      if (k < K) s_pre[k] += carry + incl - v;
      carry += __shfl(incl, kWave - 1, 64);
    }
  }
  for (int k = threadIdx.x; k < K; k += kTileQ) {  // per pair: exclusive scan over the waves
    uint32_t run = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const uint32_t c = s_cnt[i][k];
      s_cnt[i][k] = run;
      run += c;
    }
  }
  __syncthreads();
  if (pair < 0) return;
  const uint32_t dst = s_pre[pair] + s_cnt[w][pair] + rank;
  if (planar) {
    double* c = a.c_pl;
    const size_t ld = a.ld_pl;
    c[0 * ld + dst] = pi.x; c[1 * ld + dst] = pi.y; c[2 * ld + dst] = pi.z;
    c[3 * ld + dst] = ni.x; c[4 * ld + dst] = ni.y; c[5 * ld + dst] = ni.z;
    c[6 * ld + dst] = (double)pj.x; c[7 * ld + dst] = (double)pj.y; c[8 * ld + dst] = (double)pj.z;
  } else {
    double* c = a.c_pt;
    const size_t ld = a.ld_pt;
    c[0 * ld + dst] = pi.x; c[1 * ld + dst] = pi.y; c[2 * ld + dst] = pi.z;
    c[3 * ld + dst] = (double)pj.x; c[4 * ld + dst] = (double)pj.y; c[5 * ld + dst] = (double)pj.z;
  }
}

// KeypointMap::insert_matches (map.tpp:148-165) for both feature types in one
// launch: wave b covers the 64 queries of match block b and appends those whose NN
// distance exceeded min_dist_map (m_ins) to the type's keypoint store, in query
// order, at the block offset the match kernel's last block scanned (ins_off).
struct InsArgs {
  uint32_t nq_pl, nq_pt, nb_pl;
  const uint8_t* ins;       // [nq_pl + nq_pt]
  const uint32_t* ins_off;  // [nb] per match block, per type
  const float4* q_pl;
  const float4* q_pl_nrm;
  const float4* q_pt;
  float4* d_pl_pos;  // pool ends
  float4* d_pl_nrm;
  float4* d_pt_pos;
};
__global__ __launch_bounds__(kQPB) void k_insert(InsArgs a) {
  const uint32_t b = blockIdx.x;
  const bool planar = b < a.nb_pl;
  const uint32_t qi = (planar ? b : b - a.nb_pl) * kQPB + threadIdx.x;
  const uint32_t nq = planar ? a.nq_pl : a.nq_pt;
  const bool f = qi < nq && (a.ins[planar ? qi : a.nq_pl + qi] & 1) != 0;
  const uint64_t m = __ballot(f);
  // a match block of several waves (large-set build): earlier waves' counts first
  constexpr int kW = (kQPB + kWave - 1) / kWave;
  uint32_t wbase = 0;
  if constexpr (kW > 1) {
    __shared__ uint32_t s_w[kW];
    const int w = threadIdx.x / kWave;
    if (lane_id() == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    for (int i = 0; i < w; ++i) wbase += s_w[i];
  }
  if (!f) return;
  const uint32_t o = a.ins_off[b] + wbase + (uint32_t)__popcll(m & lanemask_lt());
  if (planar) {
    a.d_pl_pos[o] = a.q_pl[qi];
    a.d_pl_nrm[o] = a.q_pl_nrm[qi];
  } else {
    a.d_pt_pos[o] = a.q_pt[qi];
  }
}

uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

}  // namespace

// ---------------------------------------------------------------------------- host
void run_map_build(fmx_ctx* c, const std::vector<uint64_t>& scans, const double* poses34, double w,
                   hipStream_t stream) {
  hipStream_t st = stream ? stream : c->stream;
  HostScope* hs_prep = new HostScope(6);
  const int K = (int)scans.size();
  const int Kc = std::max(K, 1);
  c->map_scans = scans;
  c->voxel_w = w;
  c->K = (uint32_t)K;
  // internal cell = w / subdivision (<= 2).  Searching +-subdivision cells covers the
  // ball of radius w, so decisions bounded by w are unchanged; when min_dist_map > w the
  // reference's exact 27 voxels of width w are needed (subdivision 1).
  int m = c->P.voxel_subdivision == 0 ? 1 : (int)std::min<uint32_t>(c->P.voxel_subdivision, 2u);
  if (c->P.min_dist_map > w) m = 1;
  c->cell_m = m;
  c->cell_w = w / m;
  // one packed upload: poses [K][12], inverses [K][12] (GTSAM Pose3::inverse:
  // (R^T, R^T(-t)), same expression order as the device transforms), segments of
  // both feature types [2][K] (Seg = 16 B = 2 doubles)
  const size_t n_d = 24 * (size_t)Kc + 2 * 2 * (size_t)Kc;
  c->h_mapposes.ensure(n_d);
  double* hp = c->h_mapposes.p;
  for (int k = 0; k < K; ++k) {
    const double* T = poses34 + 12 * k;
    std::memcpy(hp + 12 * k, T, 12 * sizeof(double));
    double* I = hp + 12 * (Kc + k);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) I[4 * i + j] = T[4 * j + i];
    const double nt[3] = {-T[3], -T[7], -T[11]};
    for (int i = 0; i < 3; ++i) I[4 * i + 3] = (I[4 * i] * nt[0] + I[4 * i + 1] * nt[1]) + I[4 * i + 2] * nt[2];
  }
  Seg* hseg = reinterpret_cast<Seg*>(hp + 24 * (size_t)Kc);
  uint32_t nrec[2];
  for (int t = 0; t < 2; ++t) {
    Pool& pool = c->pool[t];
    uint32_t n = 0;
    for (int k = 0; k < Kc; ++k) {
      uint32_t cnt = 0, po = 0;
      if (k < K) {
        auto it = pool.ranges.find(scans[k]);
        if (it != pool.ranges.end()) {
          cnt = it->second.second;
          po = (uint32_t)it->second.first;
        }
      }
      hseg[t * Kc + k] = Seg{n, cnt, po, 0};
      n += cnt;
    }
    nrec[t] = n;
  }
  c->map_blob.ensure(n_d);
  delete hs_prep;
  FMX_HIP(hipMemcpyAsync(c->map_blob.p, hp, n_d * sizeof(double), hipMemcpyHostToDevice, st));
  c->map_poses_p = c->map_blob.p;
  c->map_inv_p = c->map_blob.p + 12 * (size_t)Kc;
  const Seg* dseg = reinterpret_cast<const Seg*>(c->map_blob.p + 24 * (size_t)Kc);
  // fused build of both types: one brick table (planar bricks, then point bricks),
  // one record numbering, five launches (k_map_insert / count / alloc / scatter / dense)
  VoxMap& M = c->map;
  const uint32_t n = nrec[0] + nrec[1];
  if (n >= (1u << 27)) throw StatusError(FMX_E_SIZE, "voxel map: more than 2^27 records (k_match tie key)");
  // bricks: more buckets than records, so a bucket of another epoch always ends a probe
  // (a brick holds >= 1 record; real scans fill a few percent of the buckets)
  for (int t = 0; t < 2; ++t) {
    M.n[t] = nrec[t];
    M.cap[t] = next_pow2(std::max<uint64_t>((uint64_t)nrec[t] + 1, 256));
  }
  const uint64_t slots = M.cap[0] + M.cap[1];  // buckets
  const bool grown = 4 * slots > M.table.cap || M.state.cap < 4;
  M.table.ensure(4 * slots);
  M.ccnt.ensure(8 * ((size_t)n + 1));  // claim slots <= probing lanes <= records
  M.state.ensure(4);  // two BuildState of 32 B
  if (grown || M.epoch >= kEpochMax) {  // fresh storage or epoch wrap: clear everything once
    FMX_HIP(hipMemsetAsync(M.table.p, 0, M.table.cap * sizeof(uint4), st));
    FMX_HIP(hipMemsetAsync(M.state.p, 0, M.state.cap * sizeof(uint4), st));
    M.epoch = 0;
  }
  M.epoch += 1;
  BuildState* bst = reinterpret_cast<BuildState*>(M.state.p);
  c->map_err_p = &bst[M.epoch & 1].err;
  c->map_err_checked = false;
  M.rinfo.ensure(n + 1);
  M.claim.ensure(n + 1);
  M.dense.ensure(n / kDenseMin + 1);
  // planar slots [0, pt_base): records + the header slots of at most n0 / (kDenseMin + 1)
  // dense cells; point slots from pt_base
  const uint32_t pt_base = nrec[0] + nrec[0] / (kDenseMin + 1) * kHdr;
  const size_t rslots = (size_t)pt_base + nrec[1] + nrec[1] / (kDenseMin + 1) * kHdr + 1;
  // record layout (rec_at): interleaved pos + normal for large maps
  M.rsh = n >= interleave_min() ? 6u : 5u;
  if (M.rsh == 6) {
    M.pos.ensure(2 * rslots);
    M.nrm_p = M.pos.p + 1;
  } else {
    M.pos.ensure(rslots);
    M.nrm.ensure((size_t)pt_base + 1);
    M.nrm_p = M.nrm.p;
  }
  // algorithmic bytes, SURVEY.md §8(d) B_build = 2 (32 M_pl + 16 M_pt) + 16 S: read the
  // local records and write the world-sorted ones (32 B per planar record: position +
  // normal as read, 16 B per point record; the same again written), + 16 B per hash slot
  // with S = 2 M slots (load 0.5).  The build as written moves more: insert and scatter
  // both read the local records, the world records are fp64 (64 / 32 B), the table is
  // touched per probe and per claim — DESIGN.md §Map build compares it with the PMC bytes.
  const double bytes = 2.0 * (32.0 * nrec[0] + 16.0 * nrec[1]) + 16.0 * 2.0 * n;
  ProfScope ps(c->prof, PROF_MAP_BUILD, bytes, st);
  HostScope* hs_l = new HostScope(7);
  BuildArgs ba;
  ba.pool_pos[0] = c->pool[0].pos.p;
  ba.pool_pos[1] = c->pool[1].pos.p;
  ba.pool_nrm = c->pool[0].nrm.p;
  ba.segs[0] = dseg;
  ba.segs[1] = dseg + Kc;
  ba.K = K;
  ba.poses = c->map_poses_p;
  ba.n0 = nrec[0];
  ba.n = n;
  ba.pt_base = pt_base;
  ba.w = c->cell_w;
  ba.bricks = reinterpret_cast<Brick*>(M.table.p);
  ba.ccnt = M.ccnt.p;
  ba.mask[0] = M.cap[0] - 1;
  ba.mask[1] = M.cap[1] - 1;
  ba.off1 = M.cap[0];
  ba.epoch = M.epoch;
  ba.rinfo = M.rinfo.p;
  ba.claim = M.claim.p;
  ba.dense = M.dense.p;
  ba.st = bst + (M.epoch & 1);
  ba.st_next = bst + ((M.epoch + 1) & 1);
  ba.pos = M.pos.p;
  ba.nrm = M.nrm_p;
  ba.rsh = M.rsh;
  if (!c->h_mapinfo.p) {
    c->h_mapinfo.ensure(1);
    c->h_mapinfo.p[0] = 0;
  }
  ba.info = c->h_mapinfo.d;
  const uint32_t nb = std::max<uint32_t>((n + 255) / 256, 1);  // >= 1: block 0 clears the next state
  hipLaunchKernelGGL(k_map_insert, dim3(nb), dim3(256), 0, st, ba);
  FMX_HIP(hipGetLastError());
  if (n > 0) {
    hipLaunchKernelGGL(k_map_count, dim3(nb), dim3(256), 0, st, ba);
    FMX_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_map_alloc, dim3((n + kAllocThreads * kAllocPer - 1) / (kAllocThreads * kAllocPer)),
                       dim3(kAllocThreads), 0, st, ba);
    FMX_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_map_scatter, dim3(nb), dim3(256), 0, st, ba);
    FMX_HIP(hipGetLastError());
    const uint32_t nbd = std::min<uint32_t>(n / (kDenseMin + 1) + 1, kDenseGrid);
    hipLaunchKernelGGL(k_map_dense, dim3(nbd), dim3(kDenseThreads), 0, st, ba);
    FMX_HIP(hipGetLastError());
  }
  delete hs_l;
  c->have_map = true;
  c->have_match = false;
  c->have_qo = false;
}

// The pair-major row scatter of the last sorted match (k_pair_scatter_t over the
// tiles, or k_pair_scatter per match block for windows wider than kTileMaxPairs).
void run_pair_scatter(fmx_ctx* c) {
  if (!c->scatter_pending) return;
  c->scatter_pending = false;
  const PairScatter& s = c->ps;
  const uint32_t nb = s.nb_pl + s.nb_pt;
  hipStream_t st = c->stream;
  if (nb > 0 && s.tiles == kTilesScatter) {  // tile blocks (if any pair) + the meta block
    ScatterArgs a;
    a.nq_pl = c->n_qpl;
    a.nq_pt = c->n_qpt;
    a.ntl_pl = c->K ? s.ntl_pl : 0u;
    a.ntl_pt = c->K ? s.ntl_pt : 0u;
    a.K = (int)c->K;
    a.m_pair = c->m_pair.p;
    a.m_pi = c->m_pi.p;
    a.m_ni = c->m_ni.p;
    a.q_pl = c->q_pl_pos.p;
    a.q_pt = c->q_pt_pos.p;
    a.thist = c->thist.p + s.thist_off;
    a.c_pl = c->c_pl.p;
    a.ld_pl = c->ld_pl;
    a.c_pt = c->c_pt.p;
    a.ld_pt = c->ld_pt;
    a.pair_counts = c->pair_counts.p;
    a.pair_base = c->pair_base.p;
    a.chunk_range = c->chunk_range.p;
    a.chunks = c->chunks.p;
    a.n_chunks = c->n_chunks.p;
    a.host_counts = c->h_counts.d;
    a.ins_blk = c->ins_blk.p;
    a.ins_off = c->ins_off.p;
    a.nb_pl = s.nb_pl;
    a.nb_pt = s.nb_pt;
    a.work = c->work.p;
    a.prof_work = s.prof_work;
    ProfScope ps(c->prof, PROF_PAIR_SORT, 0.0, st);
    hipLaunchKernelGGL(k_pair_scatter_s, dim3(a.ntl_pl + a.ntl_pt + 1), dim3(kTileQ), 0, st, a);
    FMX_HIP(hipGetLastError());
    return;
  }
  if (nb == 0 || c->K == 0) return;
  ProfScope ps(c->prof, PROF_PAIR_SORT, 0.0, st);
  if (s.tiles)
    hipLaunchKernelGGL(k_pair_scatter_t, dim3(s.ntl_pl + s.ntl_pt), dim3(kTileQ), 0, st, c->n_qpl, c->n_qpt, s.ntl_pl,
                       s.ntl_pt, s.K, c->m_pair.p, c->m_pi.p, c->m_ni.p, c->q_pl_pos.p, c->q_pt_pos.p, c->hist_off.p,
                       c->c_pl.p, c->ld_pl, c->c_pt.p, c->ld_pt);
  else if (kQPB > kWave)  // (match_group_for sends wide windows to the g8 build)
    throw StatusError(FMX_E_STATE, "per-block pair scatter needs one wave per match block");
  else
    hipLaunchKernelGGL(k_pair_scatter, dim3(nb), dim3(kQPB), 0, st, c->n_qpl, c->n_qpt, s.nb_pl, s.K, c->m_pair.p,
                       c->m_pi.p, c->m_ni.p, c->q_pl_pos.p, c->q_pt_pos.p, c->hist_off.p, s.nb_pt, c->pair_base.p,
                       c->c_pl.p, c->ld_pl, c->c_pt.p, c->ld_pt);
  FMX_HIP(hipGetLastError());
}

void run_match(fmx_ctx* c, const double* pose_j34, double max_dist, double min_dist_map, bool sorted,
               bool defer_scatter) {
  hipStream_t st = c->stream;
  const int K = std::max<int>((int)c->K, 1);
  MatchArgs a;
  if (pose_j34) std::memcpy(a.Tj, pose_j34, sizeof(a.Tj));
  else std::memset(a.Tj, 0, sizeof(a.Tj));
  a.w = c->cell_w;
  a.rings = c->cell_m;
  a.max_d2 = max_dist * max_dist;
  a.min_d2 = min_dist_map * min_dist_map;
  const double obs = std::max(a.max_d2, a.min_d2);
  const double reach = c->cell_m * c->cell_w;  // = the map's voxel width
  check_match_reach(c, max_dist, min_dist_map);
  a.bound = obs <= reach * reach ? obs : INFINITY;
  // warm start from the last match on this map and query set (m_rec, stream order); an
  // unbounded search (a.bound = inf) takes a warm record only well inside the reach
  a.warm_lim = std::isfinite(a.bound) ? a.bound : 0.99 * reach * reach;
  {
    const uint32_t* before = c->m_rec.p;
    c->m_rec.ensure((size_t)c->n_qpl + c->n_qpt + 1);
    const bool warm = c->warm_rec_gen == c->warm_gen && c->m_rec.p == before;
    const uint4* cbefore = c->m_cell.p;
    c->m_cell.ensure((size_t)c->n_qpl + c->n_qpt + 1);
    a.warm = warm && c->m_cell.p == cbefore ? c->m_rec.p : nullptr;
    a.rec = c->m_rec.p;
    a.cell = c->m_cell.p;
    c->warm_rec_gen = c->warm_gen;
#if FMX_CERT_ANY
    const float* cb = c->cert_b2.p;
    c->cert_b2.ensure((size_t)c->n_qpl + c->n_qpt + 1);
    if (c->cert_b2.p != cb) a.warm = nullptr;  // regrown: no previous bounds
    a.cert_b2 = c->cert_b2.p;
    std::memcpy(a.Tprev, c->cert_pose, sizeof(a.Tprev));
    std::memcpy(c->cert_pose, a.Tj, sizeof(a.Tj));
    a.cert_ok = a.warm && c->cert_gen == c->warm_gen && kGroup > 1 ? 1 : 0;
    c->cert_gen = kGroup > 1 ? c->warm_gen : 0;  // this launch's bounds (the 8-lane build writes them)
#endif
  }
  a.nq_pl = c->n_qpl;
  a.nq_pt = c->n_qpt;
  a.nb_pl = (c->n_qpl + kQPB - 1) / kQPB;
  const uint32_t nb_pt = (c->n_qpt + kQPB - 1) / kQPB;
  a.nb_pt = nb_pt;
  a.K = (int)c->K;
  a.sorted = sorted ? 1 : 0;
  a.ntl_pl = (a.nb_pl + kTileBlocks - 1) / kTileBlocks;
  a.ntl_pt = (nb_pt + kTileBlocks - 1) / kTileBlocks;
  // wider windows: per-block histograms; a count table that fits the scatter's LDS: no
  // match tail (the scatter scans it)
  const uint64_t tab = (uint64_t)c->K * (a.ntl_pl + a.ntl_pt);
  a.tiles = !sorted || c->K > (uint32_t)kTileMaxPairs ? 0 : tab <= kScatterTab ? kTilesScatter : kTilesTail;
  const uint32_t nq = c->n_qpl + c->n_qpt;
  c->m_pair.ensure(nq + 1);
  c->m_d2.ensure(nq + 1);
  c->m_pi.ensure(nq + 1);
  c->m_ni.ensure(c->n_qpl + 1);
  c->m_ins.ensure(nq + 1);
  const uint32_t nb = a.nb_pl + nb_pt;
  c->hist.ensure((size_t)(nb + 1) * K);
  c->hist_off.ensure((size_t)(nb + 1) * K);
  c->pair_counts.ensure(2 * (size_t)K);
  c->h_counts.ensure(2 * (size_t)K + 4);
  c->pair_base.ensure(2 * (size_t)K);
  c->chunk_range.ensure(K + 1);
  const uint32_t maxch = c->n_qpl / kPlaneChunk + c->n_qpt / kPointChunk + 2 * K + 2;
  c->chunks.ensure(maxch);
  c->n_chunks.ensure(1);
  c->max_chunks = maxch;
  c->ld_pl = c->n_qpl + 1;
  c->ld_pt = c->n_qpt + 1;
  c->c_pl.ensure(9 * c->ld_pl);
  c->c_pt.ensure(6 * c->ld_pt);
  c->work.ensure(kWorkWords * (size_t)nb + 8);
  c->work_blocks = nb;
  ensure_zeroed(c->mcnt, 2 * (size_t)K, st);
  ensure_zeroed(c->mticket, 1, st);
  c->ins_blk.ensure(nb + 1);
  c->ins_off.ensure(nb + 1);
  // the count table in two halves: a tiled launch adds into one and clears the other
  // (read by this set's previous tiled match or its scatter) for the next
  ensure_zeroed(c->thist, 2 * ((size_t)K * (a.ntl_pl + a.ntl_pt) + 1), st);
  const size_t half = c->thist.cap / 2;
  if (a.tiles && nb > 0) c->thist_par ^= 1u;  // (no launch without queries: nothing added or cleared)
  uint32_t* thist_cur = c->thist.p + c->thist_par * half;
  a.thist_clear = c->thist.p + (1u - c->thist_par) * half;
  a.thist_clear_n = a.tiles ? (uint32_t)half : 0u;
  c->hist_off.ensure((size_t)K * (a.ntl_pl + a.ntl_pt) + 1);
  const SortOut so{c->hist_off.p, c->pair_counts.p, c->pair_base.p, c->chunk_range.p, c->chunks.p, c->n_chunks.p};
  c->h_counts.ensure(2 * (size_t)K + 4);
  auto view = [&](int t) {  // type t's table section over the shared record arrays
    VoxMap& M = c->map;
    return MapView{reinterpret_cast<const Brick*>(M.table.p) + (t == 0 ? 0 : M.cap[0]), M.cap[t] ? M.cap[t] - 1 : 0,
                   M.pos.p, M.nrm_p, M.epoch, M.rsh};
  };
  // Algorithmic bytes of a match launch: query read (16 B) +
  // result write (pair 4 + d2 8 + p_i 32 [+ n_i 32] + flag 1) + the warm state: NN
  // record index and own-cell entry written (4 + 16 B), and on a warm launch also read,
  // with the warm record itself (4 + 16 + 32 B); + one 64-B line per hash probe (a brick;
  // a dense cell's 256-B header counts as 4 probes) + per candidate record tested its
  // line (32 B double4: position + build order/segment; 64 B when interleaved with the
  // normal) — those two from the counts THIS launch
  // publishes to its profiler slot (prof_collect adds them)
  const double bytes = 16.0 * nq + 45.0 * nq + 32.0 * c->n_qpl + (a.rec ? 20.0 * nq : 0.0) + (a.warm ? 52.0 * nq : 0.0);
  const int pslot = nb > 0 ? prof_ring_slot(c) : -1;
  ensure_zeroed(c->mprof, 2, st);
  a.prof_acc = c->mprof.p;
  a.prof_work = pslot >= 0 ? c->prof.wring.d + 4 * (size_t)pslot : nullptr;
  // the sub-cell walk only when the map may hold dense cells: the build's pinned info
  // word (written by k_map_dense) says "none" for this very build (same epoch)
  bool dense = c->map.n[0] + c->map.n[1] > 0;
  if (dense && c->h_mapinfo.p) {
    const unsigned long long w = __atomic_load_n(c->h_mapinfo.p, __ATOMIC_ACQUIRE);
    if ((uint32_t)(w >> 32) == c->map.epoch && (uint32_t)w == 0) dense = false;
  }
  if (nb > 0) {
    ProfScope ps(c->prof, PROF_MATCH, bytes, st);
    ps.ring = pslot;
    ps.warm = a.warm ? 1 : 0;
    ps.queries = nq;
    {
      auto kern = dense ? k_match<true> : k_match<false>;
      hipLaunchKernelGGL(kern, dim3(nb), dim3(kMatchThreads), K * sizeof(uint32_t), st, a,
                         view(0), view(1), c->q_pl_pos.p, c->q_pt_pos.p, c->map_inv_p, c->m_pair.p, c->m_d2.p, c->m_pi.p,
                         c->m_ni.p, c->m_ins.p, c->hist.p, c->work.p, c->mcnt.p, c->mticket.p, c->h_counts.d,
                         c->ins_blk.p, c->ins_off.p, thist_cur, so, FusedArgs{});
      FMX_HIP(hipGetLastError());
    }
  }
  // no queries: no launch, so zero the counts and insert totals the kernel would write
  if (nb == 0) FMX_HIP(hipMemsetAsync(c->h_counts.d, 0, (2 * (size_t)c->K + 4) * sizeof(uint32_t), st));
  c->match_nb_pl = a.nb_pl;
  c->match_nb = nb;
  c->n_qo = nq;  // query-order rows (k_linearize_total) in both modes
  // Pair-major correspondences: the counts, offsets and chunk table come from the match
  // kernel's last block (tiled) or from the scan + k_pair_base (wider windows) right
  // away; the row scatter itself may be deferred (defer_scatter: fmx_match, whose
  // caller may only read the query-order outputs) until run_pair_scatter.
  c->ps = PairScatter{a.nb_pl, nb_pt, a.ntl_pl, a.ntl_pt, a.K, a.tiles, (uint32_t)(thist_cur - c->thist.p),
                      a.prof_work};
  c->scatter_pending = false;
  if (sorted && !a.tiles) {
    ProfScope ps(c->prof, PROF_PAIR_SORT, 0.0, st);
    const size_t nh = (size_t)a.K * nb;
    c->scan_scratch.ensure(scan_scratch_size(nh) + 4);
    c->dev_u32.ensure(8);
    if (nh > 0) exclusive_scan(HistIn{c->hist.p}, HistOut{c->hist_off.p}, nh, c->scan_scratch.p, c->dev_u32.p + 5, st);
    else FMX_HIP(hipMemsetAsync(c->dev_u32.p + 5, 0, 4, st));
    hipLaunchKernelGGL(k_pair_base, dim3(1), dim3(1024), 0, st, a.K, a.nb_pl, nb_pt, c->hist_off.p, c->dev_u32.p + 5,
                       c->pair_counts.p, c->pair_base.p, c->chunk_range.p, c->chunks.p, c->n_chunks.p,
                       c->h_counts.d);
    FMX_HIP(hipGetLastError());
  } else if (sorted && nb == 0) {  // no launch: an empty chunk table
    FMX_HIP(hipMemsetAsync(c->n_chunks.p, 0, sizeof(uint32_t), st));
    FMX_HIP(hipMemsetAsync(c->chunk_range.p, 0, (size_t)(a.K + 1) * sizeof(uint32_t), st));
  }
  if (sorted) {
    c->scatter_pending = true;
    if (!defer_scatter) run_pair_scatter(c);
  }
  // per-pair counts reach pinned host memory from k_pair_base; consumed at the next sync
  c->work_copied = c->prof.on;
  if (c->prof.on) {  // per-block work counters, only needed for the profile's byte model
    c->h_work.ensure(kWorkWords * (size_t)nb + 8);
    if (nb)
      FMX_HIP(hipMemcpyAsync(c->h_work.p, c->work.p, kWorkWords * (size_t)nb * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  }
  c->counts_pending = true;
  c->have_match = true;
  c->have_corr = sorted;  // pair-major correspondences for fmx_linearize
  c->have_qo = true;      // query-order correspondences for register_scan
}

// The match at pose_j fused with its single-pose linearization (k_match<.., FUSED>):
// the summed 7 x 7 + error to dst (28 + 1 doubles), completion word `flag` (null: none).
// No per-query results are written, so the context's match state is left as it was.
void run_match_linearize(fmx_ctx* c, const double* pose_j34, double max_dist, double sigma, double* dst,
                         uint32_t* flag, uint32_t seq) {
  hipStream_t st = c->stream;
  MatchArgs a;
  std::memcpy(a.Tj, pose_j34, sizeof(a.Tj));
  a.w = c->cell_w;
  a.rings = c->cell_m;
  a.max_d2 = max_dist * max_dist;
  a.min_d2 = c->P.min_dist_map * c->P.min_dist_map;
  const double reach = c->cell_m * c->cell_w;  // = the map's voxel width
  if (a.max_d2 > reach * reach && c->cell_m > 1)
    throw StatusError(FMX_E_INVAL, "max_dist exceeds the voxel width of a subdivided map");
  // only acceptance is observable here: the search is bounded by max_dist alone
  a.bound = a.max_d2 <= reach * reach ? a.max_d2 : INFINITY;
  // no warm start here: measured (profiles/r3_ab_c5_warm_*.txt) the C5 searches barely
  // prune further (probes per query 1.724 either way), and keeping 4 B per query cost
  // the HBM-bound whole-map set 2-3 % (0.75 -> 0.77 ms per registration)
  a.warm = nullptr;
  a.rec = nullptr;
  a.cell = nullptr;
  a.warm_lim = 0.0;
#if FMX_CERT_ANY
  a.cert_b2 = nullptr;
#endif
  a.nq_pl = c->n_qpl;
  a.nq_pt = c->n_qpt;
  a.nb_pl = (c->n_qpl + kQPB - 1) / kQPB;
  a.nb_pt = (c->n_qpt + kQPB - 1) / kQPB;
  a.K = (int)c->K;
  a.sorted = 0;
  a.tiles = 0;
  a.ntl_pl = a.ntl_pt = 0;
  const uint32_t nb = a.nb_pl + a.nb_pt;
  // work words of its own: a settled match's (work, h_work) may still be waiting for
  // match_counts_fetch, which must not see this launch's counters
  c->fz_work.ensure(kWorkWords * (size_t)nb + 8);
  c->fz_work_blocks = nb;
  const uint32_t ngrp = (nb + kFzGroup - 1) / kFzGroup;
  c->bpart.ensure((size_t)(nb + ngrp + 1) * kFzLd);
  ensure_zeroed(c->ticket, 1, st);
  ensure_zeroed(c->fz_tickets, ngrp + 1, st);
  if (nb == 0) {  // nothing to match: a zero system
    FMX_HIP(hipMemsetAsync(dst, 0, 29 * sizeof(double), st));
    return;
  }
  auto view = [&](int t) {
    VoxMap& M = c->map;
    return MapView{reinterpret_cast<const Brick*>(M.table.p) + (t == 0 ? 0 : M.cap[0]), M.cap[t] ? M.cap[t] - 1 : 0,
                   M.pos.p, M.nrm_p, M.epoch, M.rsh};
  };
  bool dense = c->map.n[0] + c->map.n[1] > 0;
  if (dense && c->h_mapinfo.p) {
    const unsigned long long w = __atomic_load_n(c->h_mapinfo.p, __ATOMIC_ACQUIRE);
    if ((uint32_t)(w >> 32) == c->map.epoch && (uint32_t)w == 0) dense = false;
  }
  const FusedArgs fz{c->map_poses_p, 1.0 / sigma, c->bpart.p, c->bpart.p + (size_t)nb * kFzLd, c->fz_tickets.p,
                     c->ticket.p, dst, flag, seq};
  const SortOut so{};
  // bytes: query read (16 B) + the accepted match's normal (32 B, planar; in the winner's
  // own line when records are interleaved) + 32 * 8 B block partials + 64 B per probe and
  // per candidate the bytes of its record line (prof_collect: this launch's own counts
  // from its profiler slot)
  const double nq = (double)c->n_qpl + c->n_qpt;
  const double bytes = 16.0 * nq + (c->map.rsh == 6 ? 0.0 : 32.0 * c->n_qpl) + 256.0 * nb;
  const int pslot = prof_ring_slot(c);
  ensure_zeroed(c->mprof, 2, st);
  a.prof_acc = c->mprof.p;
  a.prof_work = pslot >= 0 ? c->prof.wring.d + 4 * (size_t)pslot : nullptr;
  ProfScope ps(c->prof, PROF_MATCH_LIN, bytes, st);
  ps.ring = pslot;
  ps.queries = nq;
#if FMX_MATCH_GROUP == 1
  {
    auto kern = dense ? k_match<true, true> : k_match<false, true>;
    hipLaunchKernelGGL(kern, dim3(nb), dim3(kMatchThreads),
                       std::max<int>(a.K, 1) * sizeof(uint32_t), st, a, view(0), view(1), c->q_pl_pos.p,
                       c->q_pt_pos.p, c->map_inv_p, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, c->fz_work.p,
                       nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, so, fz);
    FMX_HIP(hipGetLastError());
  }
#else
  (void)view;
  (void)fz;
  (void)a;
  throw StatusError(FMX_E_STATE, "fused match + linearization needs the one-lane-per-query build");
#endif
  if (c->prof.on) {  // per-block work counters (byte model of the next launch), read by work_fetch
    c->fz_h_work.ensure(kWorkWords * (size_t)nb + 8);
    FMX_HIP(hipMemcpyAsync(c->fz_h_work.p, c->fz_work.p, kWorkWords * (size_t)nb * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, st));
    c->fz_work_pending = true;
  }
}

// The work counters of the last fused launch (copied while profiling): sums for the
// byte model and the match diagnostics.  The caller has waited for the stream.
void work_fetch(fmx_ctx* c) {
  if (!c->fz_work_pending) return;
  double tp = 0, tc = 0;
  for (uint32_t b = 0; b < c->fz_work_blocks; ++b) {
    tp += c->fz_h_work.p[kWorkWords * b];
    tc += c->fz_h_work.p[kWorkWords * b + 1];
  }
  match_diag_add(c->fz_h_work.p, c->fz_work_blocks);
  c->last_probes = tp;
  c->last_cands = tc;
  c->fz_work_pending = false;
}

// Consume the asynchronously copied match counts (caller has synchronized or will).
void match_counts_fetch(fmx_ctx* c, bool wait) {
  if (!c->counts_pending) return;
  // kTilesScatter: the counts come from the pair scatter's meta block
  if (c->scatter_pending && c->ps.tiles == kTilesScatter) {
    run_pair_scatter(c);
    wait = true;
  }
  if (wait) stream_wait(c);
  const int K = std::max<int>((int)c->K, 1);
  c->cnt_pl.assign(c->h_counts.p, c->h_counts.p + c->K);
  c->cnt_pt.assign(c->h_counts.p + c->K, c->h_counts.p + 2 * c->K);
  c->ins_tot[0] = c->h_counts.p[2 * c->K];
  c->ins_tot[1] = c->h_counts.p[2 * c->K + 1];
  c->cert_tot[0] = c->h_counts.p[2 * c->K + 2];
  c->cert_tot[1] = c->h_counts.p[2 * c->K + 3];
  c->rows_pl = c->rows_pt = 0;
  for (uint32_t k = 0; k < c->K; ++k) {
    c->rows_pl += c->cnt_pl[k];
    c->rows_pt += c->cnt_pt[k];
  }
  (void)K;
  if (c->work_copied) {  // (a match made before profiling was switched on has none)
    double tp = 0, tc = 0;
    for (uint32_t b = 0; b < c->work_blocks; ++b) {
      tp += c->h_work.p[kWorkWords * b];
      tc += c->h_work.p[kWorkWords * b + 1];
    }
    match_diag_add(c->h_work.p, c->work_blocks);
    c->last_probes = tp;
    c->last_cands = tc;
  }
  c->counts_pending = false;
}

void run_insert(fmx_ctx* c, uint64_t scan, uint32_t* n_inserted) {
  if (!c->have_match) throw StatusError(FMX_E_STATE, "no match to insert from");
  hipStream_t st = c->stream;
  match_counts_fetch(c);  // insert totals of the last match (no wait if already fetched)
  const uint32_t tot[2] = {c->ins_tot[0], c->ins_tot[1]};
  for (int t = 0; t < 2; ++t) {
    const uint32_t nq = t == 0 ? c->n_qpl : c->n_qpt;
    if (tot[t] > nq) throw StatusError(FMX_E_HIP, "implausible insert total");
    if (c->pool[t].used + tot[t] > c->pool[t].pos.cap) throw StatusError(FMX_E_OOM, "keypoint pool capacity exceeded");
  }
  InsArgs ia;
  ia.nq_pl = c->n_qpl;
  ia.nq_pt = c->n_qpt;
  ia.nb_pl = c->match_nb_pl;
  ia.ins = c->m_ins.p;
  ia.ins_off = c->ins_off.p;
  ia.q_pl = c->q_pl_pos.p;
  ia.q_pl_nrm = c->q_pl_nrm.p;
  ia.q_pt = c->q_pt_pos.p;
  ia.d_pl_pos = c->pool[0].pos.p + c->pool[0].used;
  ia.d_pl_nrm = c->pool[0].nrm.p + c->pool[0].used;
  ia.d_pt_pos = c->pool[1].pos.p + c->pool[1].used;
  if (c->match_nb > 0) {
    ProfScope ps(c->prof, PROF_INSERT, 33.0 * c->n_qpl + 17.0 * c->n_qpt, st);
    hipLaunchKernelGGL(k_insert, dim3(c->match_nb), dim3(kQPB), 0, st, ia);
    FMX_HIP(hipGetLastError());
  }
  for (int t = 0; t < 2; ++t) {
    Pool& pool = c->pool[t];
    auto& rg = pool.ranges[scan];
    if (rg.second == 0) rg.first = pool.used;
    else if (rg.first + rg.second != pool.used) throw StatusError(FMX_E_STATE, "non-contiguous insert for scan");
    rg.second += tot[t];
    pool.used += tot[t];
  }
  if (n_inserted) {
    n_inserted[0] = tot[0];
    n_inserted[1] = tot[1];
  }
}

}  // namespace FMX_VM_NS
}  // namespace fmx
