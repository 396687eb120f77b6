// fmx_internal.hpp — context layout and kernel-launcher interfaces of libfmx.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <stdint.h>

#include <algorithm>
#include <map>
#include <stdexcept>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "fmx/fmx.h"
#include "stage.hpp"

namespace fmx {

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct StatusError : std::runtime_error {
  fmx_status st;
  StatusError(fmx_status s, const std::string& m) : std::runtime_error(m), st(s) {}
};

#define FMX_HIP(call)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      throw ::fmx::HipError(std::string(#call) + ": " + hipGetErrorString(e_));              \
  } while (0)

inline std::atomic<uint64_t>& dbuf_reallocs() {  // diagnostic (FMX_HOST_TIMING prints it); contexts may
  static std::atomic<uint64_t> n{0};              // live on several host threads
  return n;
}
// Growable device buffer (grows only; contents are not preserved across growth).
template <class T>
struct DBuf {
  T* p = nullptr;
  size_t cap = 0;
  void ensure(size_t n) {
    if (n <= cap) return;
    ++dbuf_reallocs();
    static const bool log = std::getenv("FMX_REALLOC_LOG") != nullptr;  // diagnostic: regrowths
    if (log && p) fprintf(stderr, "dbuf regrow %zu -> %zu elements of %zu B\n", cap, n, sizeof(T));
    if (p) (void)hipFree(p);  // synchronizes the device: grow geometrically so it stays rare
    p = nullptr;
    // at least 256k elements (<= 8 MB for the widest element): the per-scan buffers of
    // a 128 x 2048 stream never regrow once the window has filled (a regrowth's
    // hipFree serializes the device mid-scan)
    size_t c = std::max<size_t>(2 * n + 64, (size_t)1 << 18);
    FMX_HIP(hipMalloc(&p, c * sizeof(T)));
    cap = c;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};
// Grow b to >= n elements; new storage is zeroed on stream st (for self-resetting
// device counters).
template <class T>
void ensure_zeroed(DBuf<T>& b, size_t n, hipStream_t st) {
  if (n <= b.cap) return;
  b.ensure(n);
  FMX_HIP(hipMemsetAsync(b.p, 0, b.cap * sizeof(T), st));
}
template <class T>
struct HBuf {  // pinned host memory, also mapped into the device address space
  T* p = nullptr;
  T* d = nullptr;  // device-visible alias: kernels write small results here directly
  size_t cap = 0;
  void ensure(size_t n) {
    if (n <= cap) return;
    if (p) (void)hipHostFree(p);
    size_t c = n + n / 4 + 64;
    FMX_HIP(hipHostMalloc(&p, c * sizeof(T), hipHostMallocMapped | hipHostMallocCoherent));
    void* dp = nullptr;
    FMX_HIP(hipHostGetDevicePointer(&dp, p, 0));
    d = static_cast<T*>(dp);
    cap = c;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// A ring of events (fmx_ctx's cross-stream ordering): record() takes the next event,
// last() is the most recently recorded one.
struct EvRing {
  static constexpr int kN = 8;
  hipEvent_t e[kN] = {};
  int cur = 0;
  void create() {
    for (auto& x : e)
      if (!x) FMX_HIP(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  }
  void destroy() {
    for (auto& x : e)
      if (x) (void)hipEventDestroy(x);
    for (auto& x : e) x = nullptr;
  }
  hipEvent_t record(hipStream_t st) {
    cur = (cur + 1) % kN;
    FMX_HIP(hipEventRecord(e[cur], st));
    return e[cur];
  }
  hipEvent_t last() const { return e[cur]; }
};

// Profiled kernel classes (bench.py roofline).
enum ProfId {
  PROF_EXTRACT_ROWS = 0,
  PROF_CLOSEST,
  PROF_FIT,
  PROF_COMPACT,
  PROF_MAP_BUILD,
  PROF_MATCH,
  PROF_PAIR_SORT,
  PROF_LINEARIZE,
  PROF_INSERT,
  PROF_WINDOW,
  PROF_MATCH_LIN,
  PROF_UNPACK,
  PROF_MOMENTS,
  PROF_COUNT
};

// Per-launch work words of a profiled match (probes, candidates), written by the
// launch's last block to pinned memory: each launch's byte model uses its OWN counts
// (fmx_api.cpp prof_collect), no launch is charged another's.
constexpr uint32_t kProfRing = 8192;
struct ProfPending {
  int id;
  hipEvent_t a, b;
  double bytes;
  int ring = -1;    // match launches: slot in Prof::wring, else -1
  int warm = 0;     // ... 1: a warm-started launch (an earlier match on this map and query set)
  double queries = 0;
};
struct Prof {
  bool on = false;
  double ms[PROF_COUNT] = {};
  uint64_t launches[PROF_COUNT] = {};
  double bytes[PROF_COUNT] = {};
  // match work since the last reset, [cold, warm] x {launches, queries, probes, candidates,
  // certified queries, warm queries}
  double mwork[2][6] = {};
  std::vector<ProfPending> pending;
  std::vector<hipEvent_t> free_events;
  HBuf<uint32_t> wring;  // [kProfRing][4]: probes, candidates, certified, warm (pinned, mapped)
  uint32_t wnext = 0;    // next slot; slots in use = pending entries with ring >= 0
};

// Scoped kernel timer: HIP events on the context stream around one launch group.
struct ProfScope {
  Prof& pr;
  int id;
  double bytes;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  int ring = -1, warm = 0;  // a match launch's work slot (prof_ring_slot) and class
  double queries = 0;
  ProfScope(Prof& p, int i, double by, hipStream_t s);
  ~ProfScope();
};

// Keypoint store of one feature type: device pool + per-scan ranges (host side).
struct Pool {
  DBuf<float4> pos, nrm;  // nrm unused for point features
  bool planar = true;
  uint64_t used = 0;
  std::map<uint64_t, std::pair<uint64_t, uint32_t>> ranges;  // scan -> (offset, count)
};

// One built voxel map (VoxelMap<P>, map.hpp:66-94) in HBM, both feature types
// (voxelmap.hip): table = planar bricks [0, cap[0]), point bricks [cap[0], cap[0] +
// cap[1]); records planar [0, n[0]) then point [n[0], n[0] + n[1]) (+ the sub-cell
// headers of dense cells), grouped by cell; normals for planar records only.
struct VoxMap {
  DBuf<uint4> table;            // fmx::Brick (epoch-tagged keys: no clear between builds)
  DBuf<uint32_t> ccnt;          // per claim slot: 8 cell counts, then the cells' first record slots
  DBuf<uint4> state;            // two alternating BuildState (voxelmap.hip)
  uint32_t epoch = 0;           // build epoch of the current map (1..63)
  uint64_t cap[2] = {0, 0};     // powers of two
  uint32_t n[2] = {0, 0};
  DBuf<uint2> rinfo;            // per build-order record: cell, rank in the cell
  DBuf<uint32_t> claim, dense;  // claimed bricks, dense cells of the last build
  DBuf<double4> pos, nrm;       // grouped by cell
  uint32_t rsh = 5;             // record stride 1 << rsh bytes: 5 = pos / nrm arrays, 6 = interleaved in pos
  double4* nrm_p = nullptr;     // normals: nrm.p, or pos.p + 1 when interleaved
};
// Maps of at least this many records interleave positions and normals (voxelmap.hip,
// rec_at).
constexpr uint32_t kInterleaveMin = 4u << 20;
inline uint32_t interleave_min() { return kInterleaveMin; }

struct Seg {
  uint32_t off;       // first build-order record
  uint32_t n;         // records
  uint32_t pool_off;  // offset in the pool
  uint32_t pad;
};

// Launch geometry of a sorted match's pending row scatter (run_pair_scatter).
struct PairScatter {
  uint32_t nb_pl = 0, nb_pt = 0, ntl_pl = 0, ntl_pt = 0;
  int K = 0;
  int tiles = 0;              // 0 per-block histograms; 1 counts scanned by the match's last block; 2 by the scatter
  uint32_t thist_off = 0;     // the count table half the match added into
  uint32_t* prof_work = nullptr;  // the match's profiler slot (tiles == 2: filled by the scatter)
};

struct Chunk {
  uint32_t type;  // bits 0-7: 0 plane rows, 1 point pairs; window chunks: pose slot i
                  // in bits 8-19, pose slot j in bits 20-31
  uint32_t pair;
  uint32_t begin;
  uint32_t end;
};
// Linearize chunk sizes: rows strided over the 64 lanes of one wave.
#ifndef FMX_WIN_ROWS
#define FMX_WIN_ROWS 256  // rows per window-kernel block (one 64-row step per wave)
#endif
constexpr int kPlaneChunk = FMX_WIN_ROWS;  // plane rows per chunk (one block of the window kernel)
constexpr int kPointChunk = FMX_WIN_ROWS;  // point pairs per chunk (three rows each)

// ---- smoothing-mode window store (window.hip)
constexpr int kWinMaxArgPoses = 36;    // pose table by value up to this many poses
constexpr int kWinSmallArgPoses = 16;  // ... in a smaller kernel-argument block up to this many
template <int N>
struct WinPosesN {
  double m[N][12];
};
using WinPoses = WinPosesN<kWinMaxArgPoses>;
struct WinPair {  // one FeatureFactor(X(i), X(j))'s rows in the arena
  uint64_t i, j;
  uint64_t pl_off, pt_off;
  uint32_t pl_n, pt_n;
};
struct WinSeg {  // scan j's correspondences (the last match of its ICP loop)
  uint64_t pl_off = 0, pt_off = 0;
  uint32_t pl_n = 0, pt_n = 0;
  std::vector<WinPair> pairs;  // i ascending
};
struct WinStore {
  DBuf<double> pl[2], pt[2];  // ping-pong arenas: plane [9][cap_pl], point [6][cap_pt]
  int cur = 0;
  uint64_t cap_pl = 0, cap_pt = 0, tail_pl = 0, tail_pt = 0;
  std::map<uint64_t, WinSeg> segs;
  // uploaded pair set (win_set_pairs)
  DBuf<uint32_t> meta;  // [chunks (4 words each)][chunk_range]
  const Chunk* chunks_p = nullptr;
  const uint32_t* chunk_range_p = nullptr;
  hipEvent_t meta_ev = nullptr;  // the last upload from hmeta
  bool meta_ev_pending = false;
  uint32_t nch = 0;
  int npairs = 0;
  uint64_t rows_pl = 0, rows_pt = 0;
  bool chunks_valid = false;
  // launch scratch
  DBuf<double> partials, dposes;
  DBuf<uint64_t> dbg;  // FMX_WIN_TIMING stamps
  DBuf<uint32_t> pticket, dticket, dflag;  // dflag: the completion word of a sharded launch
  bool pending = false;  // a k_win_linearize launched by win_start, not yet finished
  bool pending_mom = false;  // ... a k_win_moments (its results in hM)
  uint32_t pending_seq = 0, pending_grid = 0;
  hipStream_t pending_st = nullptr;  // the stream the pending launch went to
  int pending_np = 0;
  HBuf<double> hG, hM, hposes;  // hM: per pair 2 x 136 moments (k_win_moments)
  HBuf<uint32_t> hmeta;
};

// A second set of match outputs: register_scan launches speculative matches into it
// (on the side stream) and swaps it in when the speculation was right (fmx_api.cpp,
// swap_match_set).  The members mirror fmx_ctx's match results one to one.
struct MatchSet {
  DBuf<int32_t> m_pair;
  DBuf<double> m_d2;
  DBuf<double4> m_pi, m_ni;
  DBuf<uint8_t> m_ins;
  DBuf<uint32_t> hist, hist_off, thist;
  uint32_t thist_par = 0;
  DBuf<double> c_pl, c_pt;
  DBuf<uint32_t> pair_counts, chunk_range;
  DBuf<Chunk> chunks;
  DBuf<uint32_t> n_chunks, pair_base, work, mcnt, mticket, ins_blk, ins_off;
  HBuf<uint32_t> h_counts, h_work;
  bool have_match = false, have_corr = false, scatter_pending = false, counts_pending = false, have_qo = false;
  size_t ld_pl = 0, ld_pt = 0;
  uint32_t max_chunks = 0, work_blocks = 0, match_nb_pl = 0, match_nb = 0, n_qo = 0;
  bool work_copied = false;
  int match_group = 8;
  PairScatter ps;
  uint64_t rows_pl = 0, rows_pt = 0;
  std::vector<uint32_t> cnt_pl, cnt_pt;
  double last_probes = 0, last_cands = 0;
  uint32_t ins_tot[2] = {0, 0};
  uint32_t cert_tot[2] = {0, 0};
};

// An extraction launched on stream `st`: its totals and completion word go to mapped
// pinned memory (tot / flag); extract_collect waits for them.
struct ExLaunch {
  uint32_t seq = 0;
  const volatile uint32_t* flag = nullptr;
  const uint32_t* tot = nullptr;
  size_t max_pl = 0, max_pt = 0;
  hipStream_t st = nullptr;
};

}  // namespace fmx

constexpr int kStatsN = 14;  // fmx_last_stats entries

struct fmx_ctx {
  fmx_params P{};
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;                    // map build, overlapped with extraction
  hipStream_t side2 = nullptr;                   // pipelined extraction of the announced next scan
  hipStream_t lin = nullptr;                     // the ICP loop's LM trial linearizations (beside the speculative match)
  // stream -> side -> stream ordering.  Rings of events: each record takes the next one
  // and a wait uses the last recorded, so an event is never re-recorded while an earlier
  // cross-stream wait on it may still be pending in the runtime (a re-record right after
  // a hipStreamWaitEvent was seen to corrupt the HIP runtime's state when the host moved
  // fast between them)
  fmx::EvRing ev_fork, ev_join;
  std::string err;
  fmx::Prof prof;

  // ---- extraction scratch
  fmx::DBuf<float4> scan;
  fmx::DBuf<uint8_t> planar_mask;
  fmx::DBuf<uint32_t> sel_slots, pt_slots, row_counts, row_ok, row_off;
  fmx::DBuf<int2> closest;
  fmx::DBuf<float4> nrm_slots, blk_lo, blk_hi;
  fmx::DBuf<uint32_t> scan_scratch, dev_u32;  // dev_u32: small device scalars
  size_t scan_scratch_half = 0;
  fmx::HBuf<uint32_t> h_u32;
  int rows = 0, cols = 0;

  // ---- current query set (scan being registered)
  uint64_t q_scan = 0;
  uint32_t n_qpl = 0, n_qpt = 0, n_sel = 0;
  fmx::DBuf<float4> q_pl_pos, q_pl_nrm, q_pt_pos;
  fmx::DBuf<uint32_t> q_pl_idx, q_pt_idx;
  bool have_queries = false;

  // ---- pipelined extraction (fmx_next_scan): the scan after the one being registered
  // is extracted on the side stream, during this registration, into a second query set
  // (+ planar mask); the next register_scan swaps it in instead of extracting
  fmx::DBuf<float4> nq_pl_pos, nq_pl_nrm, nq_pt_pos;
  fmx::DBuf<uint32_t> nq_pl_idx, nq_pt_idx;
  fmx::DBuf<uint8_t> n_planar_mask;
  const float* ann_ptr = nullptr;   // announced by fmx_next_scan (device pointer), its size
  size_t ann_n = 0;
  const float* pf_ptr = nullptr;    // the scan whose extraction is queued on the side stream
  size_t pf_n = 0;
  bool pf_launched = false;
  fmx::ExLaunch pf_L;
  uint32_t pf_seq = 0;              // its completion word's sequence number
  fmx::HBuf<uint32_t> h_pf;         // pinned: [0..2] its totals, [4] its completion word
  fmx::EvRing ev_pf, ev_pf_fork;
  uint64_t pf_used = 0, pf_dropped = 0;

  // ---- host-resident scans (stage.hpp): the reference passes the scan as a host
  // std::vector<PointXYZf> (form.hpp:82-83).  Copied into pinned memory by helper
  // threads + the caller, then DMA'd: the sequential path DMAs each completed part at
  // once; an announced host scan (fmx_next_scan) is copied in the background and DMA'd
  // + extracted on side2 once its copy has finished.
  fmx::Stager stager;
  fmx::StageReq st_seq, st_pf[2];
  uint8_t* pin_seq = nullptr;
  uint8_t* pin_pf[2] = {nullptr, nullptr};
  size_t pin_cap = 0;           // bytes of each pinned staging buffer
  bool ann_host = false;        // the announced scan is host memory (staged in st_pf[ann_slot])
  bool ann_pinned = false;      // ... page-locked: DMA'd from the caller's memory, no staging
  int ann_slot = 0, pf_slot = 0;  // pf_slot -1: the queued extraction's DMA read caller memory
  bool pf_host = false;         // the queued extraction's scan was host memory
  fmx::DBuf<float4> pf_scan;    // device copy of a host-announced scan (side2 order)
  fmx::DBuf<float> scan3, pf_scan3;  // packed x, y, z of staged host scans (DMA targets)
  struct ScanBuf {              // fmx_scan_buffer: pinned scan buffers handed to the caller
    float4* p = nullptr;
    size_t cap = 0;
  } scanbuf[3];
  int scanbuf_next = 0;

  // ---- window keypoint store + maps
  fmx::Pool pool[2];
  fmx::VoxMap map;  // both feature types
  std::vector<uint64_t> map_scans;  // pair k -> scan id
  fmx::DBuf<fmx::Seg> segs[2];
  fmx::HBuf<fmx::Seg> h_segs[2];
  fmx::HBuf<double> h_mapposes;
  fmx::DBuf<double> map_blob;                  // poses [K][12], inverses [K][12], segments
  const double* map_poses_p = nullptr;
  const double* map_inv_p = nullptr;
  double voxel_w = 0;   // reference voxel width (max_dist_matching)
  double cell_w = 0;    // internal cell width of the built map
  int cell_m = 1;       // subdivision: rings searched
  bool have_map = false;
  uint32_t* map_err_p = nullptr;  // range-error word of the last build (in map.state)
  bool map_err_checked = false;   // ... already read back (once per build)
  fmx::HBuf<unsigned long long> h_mapinfo;  // pinned: epoch << 32 | dense cells of the last finished build

  // ---- match results (query-indexed; planar then point)
  fmx::DBuf<int32_t> m_pair;
  fmx::DBuf<double> m_d2;
  fmx::DBuf<double4> m_pi, m_ni;
  fmx::DBuf<uint8_t> m_ins;
  fmx::DBuf<uint32_t> hist, hist_off;
  // Warm start: every match writes its NN record per query (m_rec, not part of a
  // MatchSet: each launch reads and rewrites it in place, in stream order).  A later
  // match on the same map and query set starts each query's search bounded by that
  // record's distance at the new pose (any record of the map is a valid bound).
  fmx::DBuf<uint32_t> m_rec;
  fmx::DBuf<uint4> m_cell;    // per query: its own cell as the last match found it (same scheme)
  uint64_t warm_gen = 1;      // bumped by every map build and query-set change
  uint64_t warm_rec_gen = 0;  // warm_gen when m_rec was last written (0: never)
  fmx::DBuf<uint32_t> thist;  // tiled pair sort: per-(type, pair, tile) counts, two halves
  uint32_t thist_par = 0;     // the half the last tiled match added into
  fmx::DBuf<float> cert_b2;   // FMX_CERT_DIAG / FMX_WARM_CERT builds: per query the last match's second-best bound
  double cert_pose[12] = {};  // ... and that match's pose
  uint64_t cert_gen = 0;      // warm_gen when cert_b2 was last written by an 8-lane match (0: none)
  bool have_match = false;

  // ---- sorted correspondences (pair-major SoA) + chunk table
  uint32_t K = 0;
  uint64_t corr_gen = 0;         // bumped by every call that replaces the correspondences (fmx_corr_generation)
  fmx::DBuf<double> c_pl, c_pt;  // [9][cap_pl], [6][cap_pt]
  size_t ld_pl = 0, ld_pt = 0;
  fmx::DBuf<uint32_t> pair_counts;  // [2][K] plane rows, point pairs
  fmx::DBuf<uint32_t> chunk_range;  // [K+1]
  fmx::DBuf<fmx::Chunk> chunks;
  fmx::DBuf<uint32_t> n_chunks;
  uint32_t max_chunks = 0;
  int match_group = 8;  // lanes per query of the last run_match (voxelmap.hip g8 / gl)
  bool have_corr = false;
  fmx::PairScatter ps;          // the last sorted match's scatter (voxelmap.hip)
  bool scatter_pending = false; // ... not yet launched (deferred by fmx_match)
  uint64_t rows_pl = 0, rows_pt = 0;           // correspondences (plane rows, point pairs)
  std::vector<uint32_t> cnt_pl, cnt_pt;         // per pair, host copy after match
  fmx::HBuf<double> h_corr;
  fmx::HBuf<uint32_t> h_meta, h_counts;
  fmx::DBuf<uint32_t> pair_base;                // [2][K] first row of each pair
  fmx::DBuf<uint32_t> work;                     // match work counters per block (probes, candidates)
  fmx::HBuf<uint32_t> h_work;
  uint32_t work_blocks = 0;
  bool work_copied = false;  // h_work holds the last match's counters (profiling was on)
  double last_probes = 0, last_cands = 0;
  bool counts_pending = false;
  bool nrm_attr_set = false;
  bool lds_attr_set = false;

  // ---- linearize
  fmx::DBuf<double> bpart;                        // k_linearize_total block partials
  fmx::DBuf<uint32_t> ticket;                     // its last-block ticket
  fmx::DBuf<uint32_t> fz_tickets;                 // fused match + linearization: per block-group tickets
  fmx::DBuf<uint32_t> mcnt, mticket;              // query-order match: per-pair counters + ticket
  bool fz_work_pending = false;                   // fused launch's work counters copied, not yet summed
  fmx::DBuf<uint32_t> fz_work;                    // ... its own per-block work words (a settled match's
  fmx::HBuf<uint32_t> fz_h_work;                  // work / h_work may still await match_counts_fetch)
  uint32_t fz_work_blocks = 0;
  fmx::DBuf<uint32_t> ins_blk, ins_off;           // per match block insert counts / offsets
  uint32_t ins_tot[2] = {0, 0};                   // insert totals of the last match
  uint32_t cert_tot[2] = {0, 0};                  // ... its certified / warm query counts
  fmx::DBuf<uint32_t> mprof;                      // profiled match launches' probe / candidate sums (self-resetting)
  uint32_t match_nb_pl = 0, match_nb = 0;         // blocks of the last match
  uint32_t n_qo = 0;                              // queries of the last query-order match
  fmx::HBuf<uint32_t> h_flag;                     // mapped completion word (wait_flag)
  uint32_t flag_seq = 0;
  bool have_qo = false;
  // fmx_match without count outputs on a large query set is not launched at once: if
  // the next consumer is fmx_linearize_matched at the same pose, match and
  // linearization run fused (no per-query results); any other consumer launches the
  // match first (fmx_api.cpp, settle_match)
  struct LazyMatch {
    bool pending = false;
    double pose[12];
    double max_dist = 0.0;
  } lazy;
  fmx::HBuf<double> h_poses, h_G;
  fmx::HBuf<int32_t> h_i32;

  // ---- smoothing-mode window store
  fmx::WinStore win;

  // ---- speculative matches (register_scan, smoothing mode): the match of the pose an
  // LM trial proposes, queued behind the trial's linearization while the host decides;
  // used by the next ICP iteration if it starts from exactly that pose
  fmx::MatchSet spec;
  bool spec_valid = false;
  bool spec_first = false;  // the speculative set holds the scan's first match (not a speculation)
  bool spec_mom = false;    // ... and its pair moments are pending in the window machinery (win_moments_current)
  std::vector<double> spec_mom_ref;  // ... taken at these K + 1 reference poses
  double spec_pose[12] = {};
  uint64_t spec_launched = 0, spec_hits = 0;
  uint64_t spec_map_hits = 0, spec_map_misses = 0;  // speculative map builds kept / rebuilt

  // ---- multi-GPU exchange (comm.cpp): RCCL communicator, or null
  void* comm = nullptr;
  int comm_size = 1, comm_rank = 0;
  bool comm_failed = false;  // an all-reduce failed and aborted the communicator (comm_check)
  fmx::DBuf<double> d_sum;  // device-side linearization sums all-reduced in place
  fmx::HBuf<uint32_t> h_hold;  // FMX_TEST_WITHHOLD_FLAG: the word that releases a withheld publish

  // ---- host estimator state (register_scan)
  struct Est;
  Est* est = nullptr;
  uint64_t stats[kStatsN] = {};
  uint64_t host_waits = 0;  // host waits on device results (stream / completion word) so far
};

namespace fmx {
// Wait for the context stream by polling (hipStreamSynchronize's blocking wake-up
// costs tens of microseconds; the ICP loop waits ~5-15 times per scan).
// Host-side timing (env FMX_HOST_TIMING): accumulated seconds / counts per site,
// printed to stderr at exit.  Diagnostic only.
struct HostTiming {
  bool on = std::getenv("FMX_HOST_TIMING") != nullptr;
  double t[20] = {0};
  uint64_t n[20] = {0};
  ~HostTiming() {
    if (!on) return;
    static const char* names[20] = {"register_scan", "stream_wait", "extract", "map_build", "icp_loop",
                                    "insert+tail", "map_host_prep", "map_launches", "fast_lm", "full_lm",
                                    "lin_callback", "marginalize", "win_launch_call", "win_wait",
                                    "pf_launch", "between_calls", "match_call", "scatter_call", "mom_eval",
                                    "mom_prepare"};
    for (int i = 0; i < 20; ++i)
      if (n[i]) fprintf(stderr, "host %-14s %10.1f us total %8llu calls %8.2f us/call\n", names[i], t[i] * 1e6,
                        (unsigned long long)n[i], t[i] * 1e6 / n[i]);
    fprintf(stderr, "host device-buffer reallocations %llu\n", (unsigned long long)dbuf_reallocs().load());
  }
};
inline HostTiming& host_timing() {
  static HostTiming h;
  return h;
}
// Match-kernel diagnostics (env FMX_MATCH_DIAG; needs the profiled path, which
// downloads the per-block work words): per launch the kernel span, block-duration
// percentiles, when 50/90/99 % of the blocks had finished, and the largest per-query
// candidate counts of the slowest blocks.  Printed to stderr at exit.
struct MatchDiag {
  bool on = std::getenv("FMX_MATCH_DIAG") != nullptr;
  uint64_t launches = 0;
  double span = 0, p50 = 0, p90 = 0, p99 = 0, pmax = 0, f50 = 0, f90 = 0, f99 = 0, mq_all = 0, mq_slow = 0;
  uint64_t mq_hist[8] = {0};
  double walk_rounds = 0, walk_steps = 0, walk_listed = 0, waves = 0;  // FMX_DIAG_WALK builds
  double cert = 0, viol = 0, warmq = 0, cert_slow = 0, warm_slow = 0, cert_bl = 0, blocks = 0;  // FMX_CERT_DIAG builds
  double ph50[4] = {0, 0, 0, 0}, ph99[4] = {0, 0, 0, 0};              // FMX_DIAG_PHASE builds
  ~MatchDiag() {
    if (!on || !launches) return;
    const double n = (double)launches;
#ifdef FMX_DIAG_PHASE
    fprintf(stderr, "match diag: phase ends after block start (p50 / p99 over blocks, us): query %.1f / %.1f, own cell "
                    "%.1f / %.1f, faces %.1f / %.1f, edges+corners %.1f / %.1f\n",
            ph50[0] / n, ph99[0] / n, ph50[1] / n, ph99[1] / n, ph50[2] / n, ph99[2] / n, ph50[3] / n, ph99[3] / n);
#endif
    if (warmq > 0)
      fprintf(stderr,
              "match diag: warm certificate: %.0f of %.0f warm queries certifiable (%.3f), %.0f certified with a "
              "changed NN (must be 0); slowest 1%% of blocks: %.3f of their warm queries; blocks all certifiable: "
              "%.3f\n",
              cert, warmq, cert / warmq, viol, warm_slow > 0 ? cert_slow / warm_slow : 0.0, cert_bl / blocks);
    if (walk_listed > 0)
      fprintf(stderr, "match diag: ring-1 list walk: %.2f rounds per wave, %.3f steps and %.3f listed cells per query\n",
              walk_rounds / waves, walk_steps / (waves * 64), walk_listed / (waves * 64));
    fprintf(stderr,
            "match diag: %llu launches; span %.1f us; block dur p50 %.1f p90 %.1f p99 %.1f max %.1f us; "
            "blocks done at 50/90/99%%: %.1f %.1f %.1f us; max query cands per block: mean %.1f, slowest 1%% %.1f\n",
            (unsigned long long)launches, span / n, p50 / n, p90 / n, p99 / n, pmax / n, f50 / n, f90 / n, f99 / n,
            mq_all / n, mq_slow / n);
    fprintf(stderr, "match diag: block max-query-cands histogram <16 <32 <64 <128 <256 <512 <1024 >=1024:");
    for (uint64_t h : mq_hist) fprintf(stderr, " %llu", (unsigned long long)h);
    fprintf(stderr, "\n");
  }
};
inline MatchDiag& match_diag() {
  static MatchDiag d;
  return d;
}
// w: kWorkWords (8) words per block: probes, cands, max query cands, walk rounds, t_begin, t_end,
// walk steps, listed cells (the walk words: FMX_DIAG_WALK builds, else 0)
inline void match_diag_add(const uint32_t* w, uint32_t nb) {
  MatchDiag& d = match_diag();
  if (!d.on || nb == 0) return;
  uint32_t t0 = w[4];
  for (uint32_t b = 1; b < nb; ++b)
    if ((int32_t)(w[8 * b + 4] - t0) < 0) t0 = w[8 * b + 4];
  std::vector<double> dur(nb), fin(nb);
  std::vector<std::pair<double, uint32_t>> by;
  double mq = 0;
#ifdef FMX_DIAG_PHASE
  for (int k = 0; k < 4; ++k) {
    std::vector<double> v(nb);
    for (uint32_t b = 0; b < nb; ++b) v[b] = ((w[8 * b + 3 + 3 * (k / 2)] >> (16 * (k & 1))) & 0xFFFFu) * 0.01;
    std::sort(v.begin(), v.end());
    d.ph50[k] += v[nb / 2];
    d.ph99[k] += v[std::min<size_t>(nb - 1, (size_t)(0.99 * nb))];
  }
#elif FMX_CERT_DIAG || FMX_WARM_CERT
  for (uint32_t b = 0; b < nb; ++b) {
    d.cert += w[8 * b + 3];
    d.viol += w[8 * b + 6];
    d.warmq += w[8 * b + 7];
    if (w[8 * b + 7] > 0) {
      d.blocks += 1;
      d.cert_bl += w[8 * b + 3] == w[8 * b + 7] ? 1 : 0;
    }
  }
#else
  for (uint32_t b = 0; b < nb; ++b) {
    d.walk_rounds += w[8 * b + 3];
    d.walk_steps += w[8 * b + 6];
    d.walk_listed += w[8 * b + 7];
  }
#endif
  for (uint32_t b = 0; b < nb; ++b) {
    dur[b] = (double)(int32_t)(w[8 * b + 5] - w[8 * b + 4]) * 0.01;  // 100 MHz -> us
    fin[b] = (double)(int32_t)(w[8 * b + 5] - t0) * 0.01;
    by.push_back({dur[b], w[8 * b + 2]});
    d.waves += 4;  // waves per match block (256 threads)
    mq += w[8 * b + 2];
    int h = 0;
    for (uint32_t v = w[8 * b + 2]; v >= 16 && h < 7; v >>= 1) ++h;
    d.mq_hist[h]++;
  }
#if FMX_CERT_DIAG || FMX_WARM_CERT
  {  // the slowest 1 % of blocks: how many of their warm queries certify
    std::vector<std::pair<double, uint32_t>> bd;
    for (uint32_t b = 0; b < nb; ++b) bd.push_back({dur[b], b});
    std::sort(bd.begin(), bd.end());
    const size_t ns = std::max<size_t>(1, nb / 100);
    for (size_t i = nb - ns; i < nb; ++i) {
      d.cert_slow += w[8 * bd[i].second + 3];
      d.warm_slow += w[8 * bd[i].second + 7];
    }
  }
#endif
  std::sort(dur.begin(), dur.end());
  std::sort(fin.begin(), fin.end());
  std::sort(by.begin(), by.end());
  auto pct = [&](const std::vector<double>& v, double q) { return v[std::min<size_t>(v.size() - 1, (size_t)(q * v.size()))]; };
  d.launches++;
  d.span += fin.back();
  d.p50 += pct(dur, 0.5);
  d.p90 += pct(dur, 0.9);
  d.p99 += pct(dur, 0.99);
  d.pmax += dur.back();
  d.f50 += pct(fin, 0.5);
  d.f90 += pct(fin, 0.9);
  d.f99 += pct(fin, 0.99);
  d.mq_all += mq / nb;
  const size_t ns = std::max<size_t>(1, nb / 100);
  double ms = 0;
  for (size_t i = nb - ns; i < nb; ++i) ms += by[i].second;
  d.mq_slow += ms / ns;
}
inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
struct HostScope {
  int id;
  double t0;
  explicit HostScope(int i) : id(i), t0(host_timing().on ? now_s() : 0.0) {}
  ~HostScope() {
    if (host_timing().on) {
      host_timing().t[id] += now_s() - t0;
      host_timing().n[id]++;
    }
  }
};

// Wait for the context stream with a hipStreamQuery spin (hipStreamSynchronize's
// blocking wake-up measured 4-5 % slower on register_scan, C4).
inline void stream_wait(fmx_ctx* c) {
  HostScope hs(1);
  ++c->host_waits;
  for (;;) {
    const hipError_t e = hipStreamQuery(c->stream);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) throw HipError(std::string("hipStreamQuery: ") + hipGetErrorString(e));
  }
}
// Wait until a kernel has published sequence number seq at the mapped host word f
// (its last block stores results, drains, releases at system scope, then stores
// seq).  Cheaper than a stream round trip: the host resumes as soon as the word
// lands, before the kernel retires.  A stream that went idle without the word, or a
// stream error, throws (no silent hang).
// A completion word holds the sequence number of the LAST kernel that published to it.
// Its publishers are in one stream in sequence order, so a word at or past seq means the
// kernel of seq has completed (and its results are in): a result left pending while later
// kernels published (a speculative window launch across an extraction, say) is waited
// for with ">=", never "==" (which would spin until the stream drained, then fail).
inline bool flag_reached(uint32_t f, uint32_t seq) { return (int32_t)(f - seq) >= 0; }
inline void wait_flag(fmx_ctx* c, const volatile uint32_t* f, uint32_t seq, hipStream_t st = nullptr) {
  HostScope hs(1);
  ++c->host_waits;
  for (uint32_t spins = 1;; ++spins) {
    if (flag_reached(*f, seq)) break;
    if ((spins & 0x3FFF) == 0) {
      const hipError_t e = hipStreamQuery(st ? st : c->stream);
      if (e == hipSuccess) {
        if (flag_reached(*f, seq)) break;
        throw HipError("kernel completed without publishing its result flag");
      }
      if (e != hipErrorNotReady) throw HipError(std::string("hipStreamQuery: ") + hipGetErrorString(e));
    }
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
}
// The search reach of a match (run_match, and fmx_match before it defers one): on a
// subdivided map (cell_m > 1) the rings searched cover one reference voxel, so neither
// the acceptance radius nor the insert threshold may exceed the voxel width.
inline bool match_reach_ok(const fmx_ctx* c, double max_dist, double min_dist_map) {
  const double obs = std::max(max_dist * max_dist, min_dist_map * min_dist_map);
  const double reach = c->cell_m * c->cell_w;  // = the map's voxel width
  return !(obs > reach * reach && c->cell_m > 1);
}
inline void check_match_reach(const fmx_ctx* c, double max_dist, double min_dist_map) {
  if (!match_reach_ok(c, max_dist, min_dist_map))
    throw StatusError(FMX_E_INVAL, "max_dist / min_dist_map exceed the voxel width of a subdivided map");
}
inline uint32_t next_flag(fmx_ctx* c) {
  if (!c->h_flag.p) {
    c->h_flag.ensure(1);
    c->h_flag.p[0] = 0;
  }
  return ++c->flag_seq;
}
// voxelmap.hip is built twice: 8 lanes per query (fmx::g8, per-scan query sets) and 1
// (fmx::gl, large query sets: more queries in flight per wave); the fmx:: entry points
// below dispatch on c->match_group, chosen by run_match.
#define FMX_VM_DECLS                                                                                   \
  void run_map_build(fmx_ctx* c, const std::vector<uint64_t>& scans, const double* poses34, double w, \
                     hipStream_t st = nullptr);                                                      \
  void run_match(fmx_ctx* c, const double* pose_j34, double max_dist, double min_dist_map,            \
                 bool sorted = true, bool defer_scatter = false);                                    \
  void run_pair_scatter(fmx_ctx* c);                                                                 \
  void run_insert(fmx_ctx* c, uint64_t scan, uint32_t* n_inserted);                                  \
  void match_counts_fetch(fmx_ctx* c, bool wait = true);                                             \
  void run_match_linearize(fmx_ctx* c, const double* pose_j34, double max_dist, double sigma, double* dst, \
                           uint32_t* flag, uint32_t seq);                                              \
  void work_fetch(fmx_ctx* c);
// Windows of at most this many map scans (pairs) use the tiled pair sort; wider ones a
// per-match-block histogram whose scatter ranks within one wave, so they take the g8
// build (32 queries per block) whatever the query count.
constexpr uint32_t kMatchTileMaxPairs = 256;
namespace g8 { FMX_VM_DECLS }
namespace gl { FMX_VM_DECLS }
#undef FMX_VM_DECLS
// A free slot of the profiler's work ring for a match launch about to be profiled
// (collects pending results first when every slot is taken); -1 when not profiling.
int prof_ring_slot(fmx_ctx* c);
// launchers (extract.hip / voxelmap.hip / linearize.hip)
ExLaunch extract_launch(fmx_ctx* c, const float4* d_scan, int R, int C, hipStream_t st, uint32_t* tot_h,
                        uint32_t* tot_d, uint32_t* flag_h, uint32_t* flag_d, uint32_t seq);
void extract_collect(fmx_ctx* c, const ExLaunch& L, fmx_feature_counts* out);
void run_extract(fmx_ctx* c, const float4* d_scan, int R, int C, fmx_feature_counts* out,
                 const std::function<void()>& while_waiting = nullptr);
// packed x, y, z (a staged host scan) -> float4 points with pad 0, on stream st
void unpack_xyz(fmx_ctx* c, const float* d_packed, float4* d_out, size_t n, hipStream_t st);
// st: stream to build on (default the context stream; register_scan uses the side
// stream so the build overlaps extraction)
void run_map_build(fmx_ctx* c, const std::vector<uint64_t>& scans, const double* poses34, double w,
                   hipStream_t st = nullptr);
// sorted: bucket the accepted matches pair-major into SoA correspondences (fmx_match /
// fmx_linearize, the smoothing mode); otherwise only the per-pair counts are produced
// and the single-pose mode linearizes in query order.
// defer_scatter: the pair-major row scatter waits for run_pair_scatter (fmx_match: the
// caller may read only the query-order outputs, e.g. fmx_linearize_matched).
void run_match(fmx_ctx* c, const double* pose_j34, double max_dist, double min_dist_map, bool sorted = true,
               bool defer_scatter = false);
void run_pair_scatter(fmx_ctx* c);  // no-op unless a sorted match's scatter is pending
void run_insert(fmx_ctx* c, uint64_t scan, uint32_t* n_inserted);
// wait = false: the caller knows the match kernel has completed (a later kernel in
// stream order published a flag)
void match_counts_fetch(fmx_ctx* c, bool wait = true);
int match_group_for(uint64_t nq, uint32_t K);
void run_match_linearize(fmx_ctx* c, const double* pose_j34, double max_dist, double sigma, double* dst,
                         uint32_t* flag, uint32_t seq);
// out[0..27]: summed single-pose system over all pairs at pose_j; out[28]: error
void run_linearize_total(fmx_ctx* c, const double* pose_j34, double sigma, double* out);
void upload_corr(fmx_ctx* c, uint32_t K, const uint32_t* np, const double* ppi, const double* pni,
                 const double* ppj, const uint32_t* nt, const double* tpi, const double* tpj);
// window.hip (smoothing mode): correspondence store maintenance + batched linearization
void win_reserve(fmx_ctx* c, uint64_t npl, uint64_t npt);
void win_persist(fmx_ctx* c, uint64_t j);
void win_remove(fmx_ctx* c, uint64_t s);
std::vector<WinPair> win_pairs(fmx_ctx* c);
void win_set_pairs(fmx_ctx* c, const std::vector<WinPair>& prs, const std::vector<uint64_t>& keys);
void win_linearize_stored(fmx_ctx* c, const double* poses, int nposes, double sigma, double* G_out);
void win_linearize_current(fmx_ctx* c, const double* poses, double sigma, double* G_out, hipStream_t st = nullptr);
void win_finish(fmx_ctx* c, double* G_out);  // completes a win_linearize_* / win_moments_* called with G_out = null
// pair moments (k_win_moments): per pair 2 x 136 doubles (plane, point; packed upper 16 x 16)
constexpr int kMomPair = 272;
void win_moments_current(fmx_ctx* c, const double* poses, double* out);
void win_moments_pairs(fmx_ctx* c, const double* poses_i, const double* poses_j, double* out);
// comm.cpp: RCCL communicator of the sharded path, all-reduce on the context stream
// FORM::map() snapshot (snapshot.hip): world-frame keypoints of feature type t of
// `scans` at `poses`, grouped by voxel of width w; returns the record count
uint32_t map_snapshot(fmx_ctx* c, int t, const std::vector<uint64_t>& scans, const std::vector<double>& poses,
                      double w, std::vector<double>& xyz, std::vector<double>& nrm, std::vector<uint64_t>& sid);
void comm_unique_id(uint8_t id[128]);
void comm_init(fmx_ctx* c, const uint8_t id[128], int nranks, int rank);
void comm_destroy(fmx_ctx* c);
// FMX_E_RCCL after an aborted communicator, until fmx_comm_init (every sharded entry)
void comm_check(const fmx_ctx* c);
void run_match_linearize_total(fmx_ctx* c, const double* pose_j34, double max_dist, double sigma, double* out);
void comm_allreduce_sum(fmx_ctx* c, double* dev, size_t n);  // no-op without a communicator
// all-reduce n device doubles, copy them to host.p (write-through + completion word), wait
void comm_allreduce_publish(fmx_ctx* c, double* dev, size_t n, HBuf<double>& host);
// fmx_linearize / fmx_error on k_win_linearize: mode 0 13 x 13 (91), 1 single-pose 7 x 7 (28), 2 errors only
void win_linearize_pairs(fmx_ctx* c, const double* poses_i34, const double* poses_j34, double sigma, int mode,
                         double* G_out, double* err_out);
}  // namespace fmx
