// fmx_api.cpp — C-ABI entry points (include/fmx/fmx.h) and the host adapter that
// mirrors form::Estimator::register_scan (form/form.cpp:40-114) on top of the
// device stages.  Host code only; built with hipcc -ffp-contract=off so the pose
// algebra rounds like the reference's SSE2 Eigen/GTSAM code.
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <unistd.h>
#include <map>
#include <new>
#include <set>
#include <vector>

#include "fmx_internal.hpp"

using namespace fmx;

namespace fmx {

// ---------------------------------------------------------------- match-path dispatch
// Lanes per query of k_match: 8 while the whole query set is resident at once (a
// C4 scan's ~4e4 queries: more lanes shorten each query's chain of dependent loads,
// and split the walks of dense cells), 1 for large sets (>= 128k queries, e.g. C5's 2M,
// ~2 probes and ~2 candidates per query): they run in many waves of blocks, so more
// queries per wave raise the loads in flight.  C5 match per launch: 4 lanes 0.55 ms,
// 2 lanes 0.40, 1 lane 0.245 (C4: 8 lanes 0.22 vs 4 lanes 0.28 ms per scan).
#ifndef FMX_MATCH_LARGE_MIN
#define FMX_MATCH_LARGE_MIN (128u << 10)  // queries from which the large-set build (fmx::gl) is used
#endif
int match_group_for(uint64_t nq, uint32_t K) {
  return nq >= (uint64_t)(FMX_MATCH_LARGE_MIN) && K <= kMatchTileMaxPairs ? 1 : 8;
}
void run_map_build(fmx_ctx* c, const std::vector<uint64_t>& scans, const double* poses34, double w, hipStream_t st) {
  ++c->warm_gen;  // a new map: no warm start from an earlier match
  g8::run_map_build(c, scans, poses34, w, st);  // the same build in both variants
}
void run_match(fmx_ctx* c, const double* pose_j34, double max_dist, double min_dist_map, bool sorted,
               bool defer_scatter) {
  HostScope hs(16);
  ++c->corr_gen;
  c->match_group = match_group_for((uint64_t)c->n_qpl + c->n_qpt, c->K);
  if (c->match_group != 8) gl::run_match(c, pose_j34, max_dist, min_dist_map, sorted, defer_scatter);
  else g8::run_match(c, pose_j34, max_dist, min_dist_map, sorted, defer_scatter);
}
void run_pair_scatter(fmx_ctx* c) {
  HostScope hs(17);
  if (c->match_group != 8) gl::run_pair_scatter(c);
  else g8::run_pair_scatter(c);
}
void run_insert(fmx_ctx* c, uint64_t scan, uint32_t* n_inserted) {
  if (c->match_group != 8) gl::run_insert(c, scan, n_inserted);
  else g8::run_insert(c, scan, n_inserted);
}
void run_match_linearize(fmx_ctx* c, const double* pose_j34, double max_dist, double sigma, double* dst,
                         uint32_t* flag, uint32_t seq) {
  if (match_group_for((uint64_t)c->n_qpl + c->n_qpt, c->K) != 1)
    throw StatusError(FMX_E_STATE, "fused match + linearization needs the one-lane-per-query build");
  gl::run_match_linearize(c, pose_j34, max_dist, sigma, dst, flag, seq);
}
void match_counts_fetch(fmx_ctx* c, bool wait) {
  if (c->match_group != 8) gl::match_counts_fetch(c, wait);
  else g8::match_counts_fetch(c, wait);
}

// ============================================================================ profiling
static const char* kProfNames[PROF_COUNT] = {"extract_rows", "closest",   "fit",       "compact", "map_build",
                                             "match",        "pair_sort", "linearize", "insert",  "window",
                                             "match_linearize", "unpack", "moments"};

ProfScope::ProfScope(Prof& p, int i, double by, hipStream_t s) : pr(p), id(i), bytes(by), st(s) {
  if (!pr.on) return;
  auto get = [&]() {
    hipEvent_t e;
    if (!pr.free_events.empty()) {
      e = pr.free_events.back();
      pr.free_events.pop_back();
    } else {
      FMX_HIP(hipEventCreate(&e));
    }
    return e;
  };
  a = get();
  b = get();
  FMX_HIP(hipEventRecord(a, st));
}
ProfScope::~ProfScope() {
  if (!a) return;
  (void)hipEventRecord(b, st);
  ProfPending e;
  e.id = id;
  e.a = a;
  e.b = b;
  e.bytes = bytes;
  e.ring = ring;
  e.warm = warm;
  e.queries = queries;
  pr.pending.push_back(e);
}
// every stream of the context: main, side (map build), side2 (pipelined extraction)
static void sync_all(fmx_ctx* c) {
  FMX_HIP(hipStreamSynchronize(c->stream));
  if (c->side) FMX_HIP(hipStreamSynchronize(c->side));
  if (c->side2) FMX_HIP(hipStreamSynchronize(c->side2));
  if (c->lin) FMX_HIP(hipStreamSynchronize(c->lin));
}
// A match launch's algorithmic bytes: the per-launch part known at
// launch time + 64 B per hash probe and per candidate record its line (32 B: position +
// tag; 64 B when the map interleaves the normal with it, which the winner's normal then
// costs nothing more), the counts the launch itself published to its ring slot.
static void prof_collect(fmx_ctx* c) {
  Prof& pr = c->prof;
  if (pr.pending.empty()) return;
  run_pair_scatter(c);  // a tiled match's work counts reach its ring slot from its scatter
  sync_all(c);          // profiled launches run on all three streams
  for (ProfPending& e : pr.pending) {
    float ms = 0.f;
    FMX_HIP(hipEventElapsedTime(&ms, e.a, e.b));
    double bytes = e.bytes;
    if (e.ring >= 0) {
      const uint32_t* w = pr.wring.p + 4 * (size_t)e.ring;
      const double probes = w[0], cands = w[1];
      bytes += 64.0 * probes + (c->map.rsh == 6 ? 64.0 : 32.0) * cands;
      double* m = pr.mwork[e.warm ? 1 : 0];
      m[0] += 1;
      m[1] += e.queries;
      m[2] += probes;
      m[3] += cands;
      m[4] += w[2];
      m[5] += w[3];
    }
    pr.ms[e.id] += ms;
    pr.launches[e.id] += 1;
    pr.bytes[e.id] += bytes;
    pr.free_events.push_back(e.a);
    pr.free_events.push_back(e.b);
  }
  pr.pending.clear();
  pr.wnext = 0;
}
int prof_ring_slot(fmx_ctx* c) {
  Prof& pr = c->prof;
  if (!pr.on) return -1;
  if (!pr.wring.p) pr.wring.ensure(4 * (size_t)kProfRing);
  if (pr.wnext >= kProfRing) prof_collect(c);  // every slot pending: collect (syncs) and reuse
  const int s = (int)pr.wnext++;
  std::memset(pr.wring.p + 4 * (size_t)s, 0, 4 * sizeof(uint32_t));
  return s;
}
}  // namespace fmx

#include "moments.hpp"
#include "pose.hpp"
#include "smoother.hpp"
using namespace fmxh;

namespace {
// KeyScanner::step (form/mapping/keyscanner.cpp:29-91)
struct KScan {
  uint64_t idx;
  size_t unused = 0, size = 0;
};
struct KeyScanner {
  const fmx_params* P = nullptr;
  std::deque<KScan> recent, key;
  uint64_t oldest_rf() const { return recent.empty() ? 0 : recent.front().idx; }
  std::vector<uint64_t> step(uint64_t idx, size_t size, const std::function<size_t(uint64_t)>& conn) {
    if (idx == 0) key.push_back({idx, 0, size});
    else recent.push_back({idx, 0, size});
    std::vector<uint64_t> marg;
    if (recent.size() > P->max_num_recent_scans) {
      KScan rf = recent.front();
      recent.pop_front();
      const double ratio = (double)conn(rf.idx) / (double)(rf.size * recent.size());
      if (ratio > P->keyscan_match_ratio) key.push_back(rf);
      else marg.push_back(rf.idx);
    }
    std::set<uint64_t> fin;
    for (auto& kf : key) {
      if (conn(kf.idx) > 0) kf.unused = 0;
      else ++kf.unused;
      if ((int64_t)kf.unused > P->max_steps_unused_keyscan) {
        marg.push_back(kf.idx);
        fin.insert(kf.idx);
      }
    }
    key.erase(std::remove_if(key.begin(), key.end(), [&](const KScan& f) { return fin.count(f.idx) > 0; }),
              key.end());
    if (P->max_num_keyscans > 0 && (int64_t)key.size() > P->max_num_keyscans) {
      marg.push_back(key.front().idx);
      key.pop_front();
    }
    return marg;
  }
};

// A deferred fmx_match (ctx->lazy): launched now, before anything reads or changes
// the state it depends on.
void settle_match(fmx_ctx* c) {
  if (!c->lazy.pending) return;
  c->lazy.pending = false;
  run_match(c, c->lazy.pose, c->lazy.max_dist, c->P.min_dist_map, true, true);
}
// Entry points that discard the match results (a new query set, an extraction,
// register_scan) drop a deferred match instead of launching it: nothing could read it.
// The results of any earlier match are gone with it (the deferred match replaced them),
// also when the dropping call then fails its own checks: no later reader may take an
// older match's outputs for the dropped one's.
void drop_match(fmx_ctx* c) {
  if (!c->lazy.pending) return;
  c->lazy.pending = false;
  c->have_match = false;
  c->have_qo = false;
  c->have_corr = false;
}

// SETTLE: run a deferred fmx_match first — every entry point but fmx_match itself,
// fmx_linearize_matched (which may consume it fused) and those that read no match
// state (pose, stats, profile counters, fmx_sync: a deferred match is no queued work)
template <bool SETTLE = true, class F>
fmx_status guard(fmx_ctx* c, F&& f) {
  if (!c) return FMX_E_INVAL;
  try {
    FMX_HIP(hipSetDevice(c->device));
    if constexpr (SETTLE) settle_match(c);
    f();
    c->err.clear();
    return FMX_OK;
  } catch (const StatusError& e) {
    c->err = e.what();
    return e.st;
  } catch (const HipError& e) {
    c->err = e.what();
    return FMX_E_HIP;
  } catch (const std::bad_alloc&) {
    c->err = "host allocation failed";
    return FMX_E_OOM;
  } catch (const std::exception& e) {
    c->err = e.what();
    return FMX_E_INVAL;
  }
}

void compact_pool(fmx_ctx* c, int t) {
  Pool& pool = c->pool[t];
  DBuf<float4> npos, nnrm;
  npos.ensure(pool.pos.cap);
  if (t == 0) nnrm.ensure(pool.nrm.cap);
  std::vector<std::pair<uint64_t, uint64_t>> order;  // (offset, scan)
  for (auto& [s, r] : pool.ranges) order.push_back({r.first, s});
  std::sort(order.begin(), order.end());
  uint64_t o = 0;
  for (auto& [off, s] : order) {
    auto& r = pool.ranges[s];
    if (r.second) {
      FMX_HIP(hipMemcpyAsync(npos.p + o, pool.pos.p + off, r.second * sizeof(float4), hipMemcpyDeviceToDevice,
                             c->stream));
      if (t == 0)
        FMX_HIP(hipMemcpyAsync(nnrm.p + o, pool.nrm.p + off, r.second * sizeof(float4), hipMemcpyDeviceToDevice,
                               c->stream));
    }
    r.first = o;
    o += r.second;
  }
  FMX_HIP(hipStreamSynchronize(c->stream));
  pool.pos.release();
  pool.pos = npos;
  if (t == 0) {
    pool.nrm.release();
    pool.nrm = nnrm;
  }
  pool.used = o;
}

void ensure_pool_room(fmx_ctx* c, int t, uint64_t need) {
  Pool& pool = c->pool[t];
  if (pool.used + need <= pool.pos.cap) return;
  compact_pool(c, t);
  if (pool.used + need > pool.pos.cap)
    throw StatusError(FMX_E_OOM, "keypoint pool capacity exceeded (raise keypoint_pool_capacity)");
}

// upload host features into the pool under `scan`
void pool_add(fmx_ctx* c, int t, uint64_t scan, const float* f, uint32_t n) {
  if (n == 0) return;
  ensure_pool_room(c, t, n);
  Pool& pool = c->pool[t];
  std::vector<float4> pos(n), nrm(t == 0 ? n : 0);
  const int st = t == 0 ? 6 : 3;
  for (uint32_t i = 0; i < n; ++i) {
    pos[i] = make_float4(f[st * i], f[st * i + 1], f[st * i + 2], 0.f);
    if (t == 0) nrm[i] = make_float4(f[st * i + 3], f[st * i + 4], f[st * i + 5], 0.f);
  }
  auto& rg = pool.ranges[scan];
  if (rg.second == 0) rg.first = pool.used;
  else if (rg.first + rg.second != pool.used) throw StatusError(FMX_E_STATE, "scan keypoints must be added contiguously");
  FMX_HIP(hipMemcpy(pool.pos.p + pool.used, pos.data(), n * sizeof(float4), hipMemcpyHostToDevice));
  if (t == 0) FMX_HIP(hipMemcpy(pool.nrm.p + pool.used, nrm.data(), n * sizeof(float4), hipMemcpyHostToDevice));
  rg.second += n;
  pool.used += n;
}

// device float4 arrays -> pool under `scan`
void pool_add_device(fmx_ctx* c, int t, uint64_t scan, const float* pos4, const float* nrm4, uint32_t n) {
  if (n == 0) return;
  ensure_pool_room(c, t, n);
  Pool& pool = c->pool[t];
  auto& rg = pool.ranges[scan];
  if (rg.second == 0) rg.first = pool.used;
  else if (rg.first + rg.second != pool.used) throw StatusError(FMX_E_STATE, "scan keypoints must be added contiguously");
  FMX_HIP(hipMemcpyAsync(pool.pos.p + pool.used, pos4, n * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
  if (t == 0)
    FMX_HIP(hipMemcpyAsync(pool.nrm.p + pool.used, nrm4, n * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
  rg.second += n;
  pool.used += n;
}

void set_queries_device(fmx_ctx* c, uint64_t scan, const float* plp, const float* pln, uint32_t npl, const float* ptp,
                        uint32_t npt) {
  c->q_pl_pos.ensure(npl + 1);
  c->q_pl_nrm.ensure(npl + 1);
  c->q_pl_idx.ensure(npl + 1);
  c->q_pt_pos.ensure(npt + 1);
  c->q_pt_idx.ensure(npt + 1);
  if (npl) {
    FMX_HIP(hipMemcpyAsync(c->q_pl_pos.p, plp, npl * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
    FMX_HIP(hipMemcpyAsync(c->q_pl_nrm.p, pln, npl * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
  }
  if (npt) FMX_HIP(hipMemcpyAsync(c->q_pt_pos.p, ptp, npt * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
  FMX_HIP(hipMemsetAsync(c->q_pl_idx.p, 0xFF, (npl + 1) * sizeof(uint32_t), c->stream));
  FMX_HIP(hipMemsetAsync(c->q_pt_idx.p, 0xFF, (npt + 1) * sizeof(uint32_t), c->stream));
  c->n_qpl = npl;
  c->n_qpt = npt;
  c->n_sel = npl;
  c->q_scan = scan;
  c->have_queries = true;
  ++c->warm_gen;  // a new query set: no warm start from an earlier match
  c->have_match = false;
  c->have_qo = false;
}

void set_queries(fmx_ctx* c, uint64_t scan, const float* pl, uint32_t npl, const float* pt, uint32_t npt) {
  std::vector<float4> a(npl + 1), b(npl + 1), d(npt + 1);
  for (uint32_t i = 0; i < npl; ++i) {
    a[i] = make_float4(pl[6 * i], pl[6 * i + 1], pl[6 * i + 2], 0.f);
    b[i] = make_float4(pl[6 * i + 3], pl[6 * i + 4], pl[6 * i + 5], 0.f);
  }
  for (uint32_t i = 0; i < npt; ++i) d[i] = make_float4(pt[3 * i], pt[3 * i + 1], pt[3 * i + 2], 0.f);
  c->q_pl_pos.ensure(npl + 1);
  c->q_pl_nrm.ensure(npl + 1);
  c->q_pl_idx.ensure(npl + 1);
  c->q_pt_pos.ensure(npt + 1);
  c->q_pt_idx.ensure(npt + 1);
  FMX_HIP(hipMemcpy(c->q_pl_pos.p, a.data(), (npl + 1) * sizeof(float4), hipMemcpyHostToDevice));
  FMX_HIP(hipMemcpy(c->q_pl_nrm.p, b.data(), (npl + 1) * sizeof(float4), hipMemcpyHostToDevice));
  FMX_HIP(hipMemcpy(c->q_pt_pos.p, d.data(), (npt + 1) * sizeof(float4), hipMemcpyHostToDevice));
  FMX_HIP(hipMemsetAsync(c->q_pl_idx.p, 0xFF, (npl + 1) * sizeof(uint32_t), c->stream));
  FMX_HIP(hipMemsetAsync(c->q_pt_idx.p, 0xFF, (npt + 1) * sizeof(uint32_t), c->stream));
  c->n_qpl = npl;
  c->n_qpt = npt;
  c->n_sel = npl;
  c->q_scan = scan;
  c->have_queries = true;
  ++c->warm_gen;  // a new query set: no warm start from an earlier match
  c->have_match = false;
  c->have_qo = false;
}

// ---- host-resident scans (stage.hpp)
// Helper threads of the staging copy (FMX_STAGE_THREADS, default 3; 0 = the calling
// thread copies alone), chunk size (FMX_STAGE_CHUNK_KB, default 256) and the number of
// DMAs a sequential scan is split into at most (FMX_STAGE_DMAS, default 4: each
// hipMemcpyAsync call costs the host a few microseconds).
int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}
int stage_threads() {
  static const int v = std::max(0, env_int("FMX_STAGE_THREADS", 3));
  return v;
}
size_t stage_chunk() {
  static const size_t v = (size_t)std::max(4, env_int("FMX_STAGE_CHUNK_KB", 256)) << 10;
  return v;
}
uint32_t stage_dmas() {
  static const uint32_t v = (uint32_t)std::max(1, env_int("FMX_STAGE_DMAS", 4));
  return v;
}
// Pinned staging buffers of `bytes` each (grown only; growing drains every stream and
// staging request first, since DMAs may still read the old ones).
void pinned_ensure(fmx_ctx* c, size_t bytes) {
  if (bytes <= c->pin_cap) return;
  c->stager.retire(&c->st_seq);
  c->stager.retire(&c->st_pf[0]);
  c->stager.retire(&c->st_pf[1]);
  sync_all(c);
  uint8_t** bufs[3] = {&c->pin_seq, &c->pin_pf[0], &c->pin_pf[1]};
  for (uint8_t** b : bufs) {
    if (*b) (void)hipHostFree(*b);
    *b = nullptr;
  }
  c->pin_cap = 0;
  c->ann_ptr = nullptr;  // a staged announcement lived in the old buffers
  for (uint8_t** b : bufs) FMX_HIP(hipHostMalloc(reinterpret_cast<void**>(b), bytes, hipHostMallocDefault));
  c->pin_cap = bytes;
}
// Start the staging copy of `bytes` host bytes into pinned `dst` (helpers, if any).
void stage_submit(fmx_ctx* c, StageReq& r, const void* src, void* dst, size_t bytes) {
  c->stager.retire(&r);
  c->stager.start(stage_threads());
  r.reset(src, dst, bytes, stage_chunk(), /*pack=*/true);  // x, y, z only (stage_host_scan)
  if (c->stager.threads() > 0) c->stager.submit(&r);
}
// Every chunk of r copied (this thread helps) and r released by the helpers.
void stage_finish(fmx_ctx* c, StageReq& r) {
  while (r.work_one()) {
  }
  while (!r.complete()) std::this_thread::yield();
  c->stager.retire(&r);
}
// Page-locked host memory (hipHostMalloc / hipHostRegister, e.g. fmx_scan_buffer or a
// pinned torch tensor): both ends of [p, p + bytes) are checked.  Such a scan is DMA'd
// straight from the caller's memory, without a staging copy.
bool host_pinned(const void* p, size_t bytes) {
  if (!p || !bytes) return false;
  for (const void* q : {p, static_cast<const void*>(static_cast<const uint8_t*>(p) + bytes - 1)}) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, q) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    if (at.type != hipMemoryTypeHost) return false;
  }
  return true;
}
// A host scan for the sequential path, into c->scan on the context stream: a pinned one
// is DMA'd directly; a pageable one is staged by the helpers and this thread as packed
// x, y, z (12 of every 16 bytes: a PointXYZf's pad is always 0, utils.hpp:38-46), each
// completed quarter DMA'd right away, then unpacked on the device (k_unpack_xyz).
const float4* stage_host_scan(fmx_ctx* c, const float* xyzw, size_t n) {
  const size_t bytes = n * sizeof(float4);
  c->scan.ensure(n);
  if (host_pinned(xyzw, bytes)) {
    FMX_HIP(hipMemcpyAsync(c->scan.p, xyzw, bytes, hipMemcpyHostToDevice, c->stream));
    return c->scan.p;
  }
  pinned_ensure(c, bytes);
  // pin_seq's previous DMA was on the context stream ahead of an extraction whose totals
  // the host waited for: it has completed
  StageReq& r = c->st_seq;
  stage_submit(c, r, xyzw, c->pin_seq, bytes);
  c->scan3.ensure(3 * n);
  uint8_t* dev = reinterpret_cast<uint8_t*>(c->scan3.p);
  const uint32_t step = std::max<uint32_t>(1, (r.nchunks + stage_dmas() - 1) / stage_dmas());
  uint32_t issued = 0;
  while (issued < r.nchunks) {
    uint32_t ready = issued;
    while (ready < r.nchunks && r.chunk_done(ready)) ++ready;
    if (ready - issued >= step || ready == r.nchunks) {
      const size_t a = (size_t)issued * r.chunk / 16 * 12, b = std::min(bytes, (size_t)ready * r.chunk) / 16 * 12;
      FMX_HIP(hipMemcpyAsync(dev + a, c->pin_seq + a, b - a, hipMemcpyHostToDevice, c->stream));
      issued = ready;
      continue;
    }
    if (!r.work_one()) std::this_thread::yield();  // help; then wait for the helpers' chunks
  }
  c->stager.retire(&r);
  unpack_xyz(c, c->scan3.p, c->scan.p, n, c->stream);
  return c->scan.p;
}

void pf_drop(fmx_ctx* c);
void do_extract(fmx_ctx* c, const float* xyzw, size_t n, uint64_t scan, int on_dev, fmx_feature_counts* out,
                const std::function<void()>& while_waiting = nullptr) {
  const auto& E = c->P.extraction;
  const size_t R = (size_t)E.num_rows, C = (size_t)E.num_columns;
  if (!xyzw && n) throw StatusError(FMX_E_INVAL, "null scan");
  if (n != R * C)  // extraction.tpp:141-145
    throw StatusError(FMX_E_SIZE, "Provided scan does not match the expected size " + std::to_string(R * C) +
                                      " != " + std::to_string(n));
  if (C > 4096 || C < 2 * E.neighbor_points + 2 || E.num_sectors == 0 || E.num_sectors > C)
    throw StatusError(FMX_E_INVAL, "unsupported scan geometry (columns must be <= 4096)");
  pf_drop(c);  // a queued extraction shares the scratch buffers
  const float4* d = on_dev ? reinterpret_cast<const float4*>(xyzw) : stage_host_scan(c, xyzw, n);
  run_extract(c, d, (int)R, (int)C, out, while_waiting);
  c->q_scan = scan;
  c->have_queries = true;
  ++c->warm_gen;  // a new query set: no warm start from an earlier match
  c->have_match = false;
  c->have_qo = false;
}

// ---- pipelined extraction (fmx_next_scan)
// Exchange the current query set (+ planar mask) with the second one.
void swap_query_set(fmx_ctx* c) {
  using std::swap;
  swap(c->q_pl_pos, c->nq_pl_pos); swap(c->q_pl_nrm, c->nq_pl_nrm); swap(c->q_pt_pos, c->nq_pt_pos);
  swap(c->q_pl_idx, c->nq_pl_idx); swap(c->q_pt_idx, c->nq_pt_idx); swap(c->planar_mask, c->n_planar_mask);
}
// Discard a queued extraction of an announced scan (its buffers are then free again).
void pf_drop(fmx_ctx* c) {
  if (c->pf_launched) {
    FMX_HIP(hipStreamSynchronize(c->side2));
    ++c->pf_dropped;
  }
  c->pf_launched = false;
  c->pf_ptr = nullptr;
}
// Queue the extraction of the announced scan on its own low-priority stream (side2:
// the speculative map build on `side` is not serialized behind it), into the second
// query set, behind everything queued on the context stream so far (the current scan's
// extraction and its first match, which read the current set).  Its results are not
// read until the register_scan of that scan (pf_take).  Placement measured: here or at
// the start of the full LM (optimize(false)) is the same within the box-to-box noise.
// A host-announced scan is launched once its staging copy has finished (force: wait for
// it): register_scan offers the launch after every ICP match and before the full LM,
// and forces it at its end.
void pf_launch(fmx_ctx* c, bool force = true) {
  if (!c->ann_ptr || c->pf_launched) return;
  if (c->ann_host && !c->ann_pinned) {
    StageReq& r = c->st_pf[c->ann_slot];
    if (!force && !r.complete()) return;
    stage_finish(c, r);
  }
  HostScope hs(14);
  const auto& E = c->P.extraction;
  const float4* d = reinterpret_cast<const float4*>(c->ann_ptr);
  c->h_pf.ensure(8);
  if (c->pf_seq == 0) c->h_pf.p[4] = 0;
  c->ev_pf_fork.record(c->stream);
  FMX_HIP(hipStreamWaitEvent(c->side2, c->ev_pf_fork.last(), 0));
  if (c->ann_host) {  // the staged copy -> the device (side2: behind the previous queued extraction's reads)
    c->pf_scan.ensure(c->ann_n);
    if (c->ann_pinned) {
      FMX_HIP(hipMemcpyAsync(c->pf_scan.p, c->ann_ptr, c->ann_n * sizeof(float4), hipMemcpyHostToDevice, c->side2));
    } else {  // staged as packed x, y, z
      c->pf_scan3.ensure(3 * c->ann_n);
      FMX_HIP(hipMemcpyAsync(c->pf_scan3.p, c->pin_pf[c->ann_slot], c->ann_n * 12, hipMemcpyHostToDevice, c->side2));
      unpack_xyz(c, c->pf_scan3.p, c->pf_scan.p, c->ann_n, c->side2);
    }
    d = c->pf_scan.p;
  }
  swap_query_set(c);
  try {
    const uint32_t seq = ++c->pf_seq;
    c->pf_L = extract_launch(c, d, (int)E.num_rows, (int)E.num_columns, c->side2, c->h_pf.p, c->h_pf.d, c->h_pf.p + 4,
                             c->h_pf.d + 4, seq);
  } catch (...) {
    swap_query_set(c);
    throw;
  }
  swap_query_set(c);
  c->ev_pf.record(c->side2);
  c->pf_launched = true;
  c->pf_ptr = c->ann_ptr;
  c->pf_n = c->ann_n;
  c->pf_host = c->ann_host;
  c->pf_slot = c->ann_pinned ? -1 : c->ann_slot;
  c->ann_ptr = nullptr;
}
// register_scan(scan): true if `scan` is the one whose extraction was queued; its query
// set becomes current (the context stream waits for its kernels) and its totals are
// collected.  Any other scan drops the queued extraction.
bool pf_take(fmx_ctx* c, const float* xyzw, size_t n, int on_dev, uint64_t scan, fmx_feature_counts* out) {
  if (!c->pf_launched) return false;
  if ((on_dev != 0) == c->pf_host || xyzw != c->pf_ptr || n != c->pf_n) {
    pf_drop(c);
    return false;
  }
  c->pf_launched = false;
  c->pf_ptr = nullptr;
  swap_query_set(c);
  FMX_HIP(hipStreamWaitEvent(c->stream, c->ev_pf.last(), 0));
  extract_collect(c, c->pf_L, out);
  ++c->pf_used;
  c->q_scan = scan;
  c->have_queries = true;
  ++c->warm_gen;  // a new query set: no warm start from an earlier match
  c->have_match = false;
  c->have_qo = false;
  return true;
}

}  // namespace

// ============================================================================ estimator
struct fmx_ctx::Est {
  bool init = false;
  uint64_t scan = 0;
  std::map<uint64_t, Pose> values;
  std::map<uint64_t, std::map<uint64_t, std::pair<uint32_t, uint32_t>>> cons;
  KeyScanner ks;
  std::vector<double> poses_i, poses_j, G, err;
  // smoothing mode (ConstraintManager members, constraints.hpp:74-101)
  std::vector<PriorF> priors;  // m_other_factors: the prior on X(0)
  std::vector<LinF> margs;     // m_other_factors: marginal LinearContainerFactors
  // every stored pair's linearization at `values` (the last full LM's final state),
  // keyed (j, i): m_fast_linear and marginalize reuse it
  std::map<std::pair<uint64_t, uint64_t>, std::vector<double>> gcache;
  // pair moments (moments.hpp) of every stored pair, keyed (j, i): the rows of scan j's
  // last match, taken at reference poses; under FMX_MOMENTS=1 the LMs linearize the pairs
  // from them on the host
  struct Mom {
    Pose ref_i, ref_j;
    std::vector<double> phi;  // kMomPairD
  };
  std::map<std::pair<uint64_t, uint64_t>, Mom> moms;
  // marginalization of the scans the last keyscan step dropped, deferred to the next
  // register_scan where it runs while that scan's extraction kernels execute
  bool tail_pending = false;
  std::vector<uint64_t> tail_marg;
  // the last scan's constraint counts and map size (fmx_last_stats)
  uint64_t last_mpl = 0, last_mpt = 0, last_map_pl = 0, last_map_pt = 0;
  // speculative map build (smoothing mode): the next scan's map built during this
  // scan's final LM from a trial it will probably end on; valid iff the next scan's
  // map inputs (scans, poses) equal these bit for bit
  bool spec_map = false;
  std::vector<uint64_t> spec_map_scans;
  std::vector<double> spec_map_poses;
};

namespace {

// ConstraintManager::predict_next (constraints.cpp:71-101)
// `gone`: keys the pending marginalization is about to erase (treated as absent).
Pose predict_next(const fmx_ctx::Est& e, const std::vector<uint64_t>& gone = {}) {
  if (!e.init) return identity();
  const uint64_t s = e.scan + 1;
  auto has = [&](uint64_t k) { return e.values.count(k) && std::find(gone.begin(), gone.end(), k) == gone.end(); };
  const bool pe = s > 0 && has(s - 1), ppe = s > 1 && has(s - 2);
  if (pe && ppe) {
    const Pose& prev = e.values.at(s - 1);
    const Pose& pp = e.values.at(s - 2);
    Pose pr = compose(prev, compose(inverse(pp), prev));
    normalize_rot(pr);
    return pr;
  }
  if (pe) return e.values.at(s - 1);
  return identity();
}

// Single-pose LM on X(j), map poses fixed (disable_smoothing, constraints.cpp:103-111,
// 235-250) with GTSAM LevenbergMarquardtOptimizer defaults.  Linearizations run on
// the device (fmx stage 3, 7x7 layout).  Every trial pose is evaluated with a full
// linearization: it returns the error the accept test needs AND, if the step is
// accepted, the next iteration's system — one device round trip per trial, and the
// arithmetic is identical to evaluating the error alone.
struct DeviceLM {
  fmx_ctx* c;
  fmx_ctx::Est& e;
  double sigma;
  double lambda = 1e-5;
  int linearizations = 0;
  // cached linearization
  double Hs[6][6], g[6], cc, err;
  void fill(const Pose& Tj) {
    const uint32_t K = c->K;
    e.poses_i.resize(12 * (size_t)K);
    e.poses_j.resize(12 * (size_t)K);
    for (uint32_t k = 0; k < K; ++k) {
      std::memcpy(&e.poses_i[12 * k], e.values.at(c->map_scans[k]).m, 12 * sizeof(double));
      std::memcpy(&e.poses_j[12 * k], Tj.m, 12 * sizeof(double));
    }
  }
  // linearize at Tj into (H, g, c, err); returns err
  double linearize(const Pose& Tj, double H[6][6], double gg[6], double& c2) {
    const uint32_t K = c->K;
    for (int i = 0; i < 6; ++i) {
      gg[i] = 0;
      for (int j = 0; j < 6; ++j) H[i][j] = 0;
    }
    c2 = 0;
    if (K == 0) return 0.0;
    // window poses = the built map's poses (unchanged during the scan); Tj by value;
    // one fused launch sums the system over all pairs
    double S[29];
    run_linearize_total(c, Tj.m, sigma, S);
    ++linearizations;
    double full[7][7];
    int o = 0;
    for (int i = 0; i < 7; ++i)
      for (int j = i; j < 7; ++j) full[i][j] = full[j][i] = S[o++];
    for (int i = 0; i < 6; ++i) {
      for (int j = 0; j < 6; ++j) H[i][j] = full[i][j];
      gg[i] = full[i][6];
    }
    c2 = full[6][6];
    const double er = S[28];
    return er;
  }
  // one LevenbergMarquardtOptimizer::iterate() from the cached system at T
  void iterate(Pose& T) {
    const double oldLin = 0.5 * cc;
    for (;;) {  // tryLambda
      double Hd[6][6];
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) Hd[i][j] = Hs[i][j] + (i == j ? lambda : 0.0);
      double dx[6];
      const bool ok = chol_solve6(Hd, g, dx);
      bool success = false, stop = false;
      Pose Tn = T;
      double nerr = err, nH[6][6], ng[6], ncc = 0;
      if (ok) {
        double dHd = 0, dg = 0;
        for (int i = 0; i < 6; ++i) {
          double h = 0;
          for (int j = 0; j < 6; ++j) h += Hs[i][j] * dx[j];
          dHd += dx[i] * h;
          dg += dx[i] * g[i];
        }
        const double newLin = 0.5 * (dHd - 2 * dg + cc);
        const double linChange = oldLin - newLin;
        if (linChange >= 0) {
          Tn = compose(T, expmap(dx));
          nerr = linearize(Tn, nH, ng, ncc);
          const double costChange = err - nerr;
          if (linChange > DBL_EPSILON * oldLin) success = (costChange / linChange) > 1e-3;
          else success = true;
          if (std::abs(costChange) < 1e-5 * err) stop = true;
        }
      }
      if (success) {
        lambda = std::max(0.0, lambda / 10.0);
        T = Tn;
        err = nerr;
        std::memcpy(Hs, nH, sizeof(Hs));
        std::memcpy(g, ng, sizeof(g));
        cc = ncc;
        return;
      } else if (!stop) {
        lambda *= 10.0;
        if (lambda >= 1e5) return;
      } else {
        return;
      }
    }
  }
  Pose optimize(const Pose& T0, int* iters) {  // NonlinearOptimizer::defaultOptimize
    lambda = 1e-5;
    Pose T = T0;
    err = linearize(T, Hs, g, cc);
    int it = 0;
    if (err <= 0.0) {
      *iters = 0;
      return T;
    }
    double cur, newErr = err;
    bool conv;
    do {
      cur = newErr;
      iterate(T);
      ++it;
      newErr = err;
      if (newErr <= 0.0) conv = true;
      else {
        const double absDec = cur - newErr, relDec = absDec / cur;
        conv = (relDec <= 1e-5) || (absDec <= 1e-5);
      }
    } while (it < 100 && !conv && std::isfinite(cur));
    *iters = it;
    return T;
  }
};

// ------------------------------------------------------------------ smoothing mode
// Window keys (Values order) and their current poses.
std::vector<uint64_t> window_keys(const fmx_ctx::Est& e) {
  std::vector<uint64_t> k;
  for (auto& [s, T] : e.values) k.push_back(s);
  return k;
}
std::vector<Pose> window_poses(const fmx_ctx::Est& e) {
  std::vector<Pose> x;
  for (auto& [s, T] : e.values) x.push_back(T);
  return x;
}

// m_fast_linear (constraints.cpp:268-288): ONE HessianFactor of every previous pair
// linearized at m_values.  m_values of those keys are the last full LM's final state,
// whose per-pair linearizations are cached (minus the pairs marginalization dropped).
LinF fast_linear(const fmx_ctx::Est& e) {
  LinF L;
  std::set<uint64_t> ks;
  for (auto& [ji, G] : e.gcache) {
    ks.insert(ji.first);
    ks.insert(ji.second);
  }
  if (ks.empty()) return L;
  L.keys.assign(ks.begin(), ks.end());
  DenseSys S;
  S.init(L.keys);
  for (auto& [ji, G] : e.gcache) S.add_pair(S.slot.at(ji.second), S.slot.at(ji.first), G.data());
  for (uint64_t k : L.keys) L.lin.push_back(e.values.at(k));
  L.info.swap(S.A);
  return L;
}

// The window graph's pair linearization in split form: launch, the host assembles the
// non-pair terms, then wait.
template <class B, class E>
void set_lin(WinGraph& g, B begin, E end) {
  g.lin_pairs = [begin, end](const std::vector<Pose>& x, double* G) {
    begin(x);
    end(G);
  };
  g.lin_begin = begin;
  g.lin_end = end;
}

// Exchange the context's match results with the speculative set (fmx::MatchSet).
void swap_match_set(fmx_ctx* c) {
  MatchSet& S = c->spec;
  using std::swap;
  ++c->corr_gen;
  swap(c->m_pair, S.m_pair); swap(c->m_d2, S.m_d2); swap(c->m_pi, S.m_pi); swap(c->m_ni, S.m_ni);
  swap(c->m_ins, S.m_ins); swap(c->hist, S.hist); swap(c->hist_off, S.hist_off); swap(c->thist, S.thist);
  swap(c->thist_par, S.thist_par);
  swap(c->c_pl, S.c_pl); swap(c->c_pt, S.c_pt); swap(c->pair_counts, S.pair_counts);
  swap(c->chunk_range, S.chunk_range); swap(c->chunks, S.chunks); swap(c->n_chunks, S.n_chunks);
  swap(c->pair_base, S.pair_base); swap(c->work, S.work); swap(c->mcnt, S.mcnt); swap(c->mticket, S.mticket);
  swap(c->ins_blk, S.ins_blk); swap(c->ins_off, S.ins_off); swap(c->h_counts, S.h_counts); swap(c->h_work, S.h_work);
  swap(c->have_match, S.have_match); swap(c->have_corr, S.have_corr); swap(c->scatter_pending, S.scatter_pending);
  swap(c->counts_pending, S.counts_pending); swap(c->have_qo, S.have_qo); swap(c->ld_pl, S.ld_pl);
  swap(c->ld_pt, S.ld_pt); swap(c->max_chunks, S.max_chunks); swap(c->work_blocks, S.work_blocks);
  swap(c->work_copied, S.work_copied);
  swap(c->match_nb_pl, S.match_nb_pl); swap(c->match_nb, S.match_nb); swap(c->n_qo, S.n_qo);
  swap(c->match_group, S.match_group); swap(c->ps, S.ps); swap(c->rows_pl, S.rows_pl); swap(c->rows_pt, S.rows_pt);
  swap(c->cnt_pl, S.cnt_pl); swap(c->cnt_pt, S.cnt_pt); swap(c->last_probes, S.last_probes);
  swap(c->last_cands, S.last_cands); swap(c->ins_tot, S.ins_tot); swap(c->cert_tot, S.cert_tot);
}

// Speculative match (smoothing-mode ICP): when an LM trial is probably the LM's last
// and the ICP loop will probably continue from it, the sorted match of the trial's X(j)
// is queued on the context stream right behind the trial's linearization, into the
// speculative set, so it runs while the host takes the LM decision.  If the next ICP
// iteration starts from exactly that pose it takes these results (use_spec_match)
// instead of matching again; results are bit-identical either way.  The speculative
// set is not read by any queued kernel: it was swapped out at the start of this ICP
// iteration and every kernel that read it belongs to earlier, completed iterations.
// mom_ref (moments mode, else null): K + 1 reference poses (the map scans', then X(j) =
// pose_j): the speculative set's pair moments are queued right behind its match and
// scatter (win_moments_current, left pending in the window machinery), so an ICP
// iteration that takes this match finds its moments under way (c->spec_mom).
void spec_match(fmx_ctx* c, const double* pose_j, bool first = false, const double* mom_ref = nullptr) {
  const fmx_params& P = c->P;
  swap_match_set(c);
  try {
    run_match(c, pose_j, P.max_dist_matching, P.min_dist_map, true);
    if (mom_ref) win_moments_current(c, mom_ref, nullptr);
  } catch (...) {
    swap_match_set(c);
    throw;
  }
  swap_match_set(c);
  c->spec_mom = mom_ref != nullptr;
  if (mom_ref) c->spec_mom_ref.assign(mom_ref, mom_ref + 12 * ((size_t)c->K + 1));
  std::memcpy(c->spec_pose, pose_j, sizeof(c->spec_pose));
  c->spec_valid = true;
  c->spec_first = first;
  if (!first) ++c->spec_launched;
}
bool use_spec_match(fmx_ctx* c, const double* pose_j) {
  if (!c->spec_valid || std::memcmp(c->spec_pose, pose_j, sizeof(c->spec_pose)) != 0) return false;
  swap_match_set(c);
  c->spec_valid = false;
  if (!c->spec_first) ++c->spec_hits;
  c->spec_first = false;
  return true;
}

void keyscan_step(fmx_ctx* c, fmx_ctx::Est& e, uint64_t j, uint32_t nfeat);
void record_cons(fmx_ctx* c, fmx_ctx::Est& e, uint64_t j);

// FMX_TRACE (diagnostic): one stderr line per step of the smoothing-mode registration
bool trace_on() {
  static const bool v = std::getenv("FMX_TRACE") != nullptr;
  return v;
}
#define FMX_TRACE_(...)                   \
  do {                                    \
    if (trace_on()) {                     \
      fprintf(stderr, __VA_ARGS__);       \
      fflush(stderr);                     \
    }                                     \
  } while (0)

// The smoother's LMs linearize every trial on the device from the rows (k_win_linearize
// over the sorted match / the window store) — or, with FMX_MOMENTS=1 (opt-in; measured
// neutral on C4 and slower on C2, DESIGN.md "pair moments"), from the pair moments
// (k_win_moments once per ICP iteration, host contractions, moments.cpp) in the ICP loop
// and from the stored pairs' moments in the final LM.
bool lin_rows() {
  static const bool v = std::getenv("FMX_MOMENTS") == nullptr;
  return v;
}

// ICP loop (form.cpp:67-89) + optimize(false) (form.cpp:92-93) in smoothing mode:
// every LM runs over all window poses; the current scan's FeatureFactors linearize
// from the sorted match, the stored pairs from the window store (window.hip).
// fast: m_fast_linear of the window (fast_linear(e)), computed by the caller while the
// extraction kernels run
void smooth_register(fmx_ctx* c, fmx_ctx::Est& e, uint64_t j, uint32_t nfeat, const LinF& fast, uint64_t& icp,
                     uint64_t& lm_it, uint64_t& lins, bool& inserted) {
  const fmx_params& P = c->P;
  const double sigma = P.planar_constraint_sigma;
  const std::vector<uint64_t> keys = window_keys(e);
  std::map<uint64_t, int> slot;
  for (size_t k = 0; k < keys.size(); ++k) slot[keys[k]] = (int)k;
  WinGraph g;
  g.keys = keys;
  for (auto& p : e.priors) g.priors.push_back(&p);
  for (auto& m : e.margs) g.lins.push_back(&m);
  if (!fast.keys.empty()) g.lins.push_back(&fast);
  std::vector<double> table;
  const bool mom = !lin_rows();
  const bool mom_full = mom;  // the final LM from the stored pairs' moments too
  std::vector<double> momv;                  // the current scan's pair moments (K x kMomPairD)
  std::vector<Pose> mref;                    // ... their reference poses: [k] pair k's X(i), [K] X(j)
  std::vector<const double*> mp;             // contraction arguments (moments.hpp)
  std::vector<const Pose*> mri, mrj, mxi, mxj;
  MomBatch mbatch;
  for (uint32_t it = 0; it < P.max_num_rematches; ++it) {
    ++icp;
    const Pose before = e.values.at(j);
    const bool spec_hit = use_spec_match(c, before.m);
    if (!spec_hit) run_match(c, before.m, P.max_dist_matching, P.min_dist_map, true);  // pair-major
    c->spec_valid = false;
    // the taken speculative match's moments are pending (spec_match); a missed one's are
    // drained by the next window launch
    const bool mom_queued = spec_hit && c->spec_mom;
    c->spec_mom = false;
    pf_launch(c, false);  // the announced next scan's extraction, behind this match (host: once staged)
    // get_graph(true): the current scan's K pairs (empty ones linearize to zero)
    g.pairs.clear();
    for (uint32_t k = 0; k < c->K; ++k) g.pairs.push_back({slot.at(c->map_scans[k]), slot.at(j)});
    const int K = (int)c->K;
    // an LM trial the LM will probably stop after (its predicted decrease within the
    // LM's convergence tolerances, rel/abs 1e-5; the actual decrease decides and tracks
    // the prediction closely on this stream, profiles/r2_spec_log.txt): match its X(j)
    // speculatively — the next ICP iteration starts from the LM's final X(j).  A trial
    // predicted to decrease more is followed by another.
    auto maybe_spec = [&](const std::vector<Pose>& x) {
      const Pose& xj = x[slot.at(j)];
      const double lc = g.trial_lin_change, ce = g.trial_err;
      bool last_likely = lc >= 0.0 && (lc <= 1e-5 * ce || lc <= 1e-5);
      if (last_likely) {  // ... and the ICP loop continues from it (form.cpp:83-88)
        double xi[6], dn = 0;
        logmap(compose(inverse(before), xj), xi);
        for (double v : xi) dn += v * v;
        last_likely = std::sqrt(dn) >= P.new_pose_threshold;
      }
      if (last_likely && it + 1 < P.max_num_rematches && std::memcmp(xj.m, before.m, sizeof(xj.m)) != 0) {
        FMX_TRACE_("  spec match\n");
        if (mom) {
          // the next iteration's reference: its LM starts from the window values with
          // X(j) = this trial's (fast mode keeps only X(j), constraints.cpp:257-266)
          std::vector<double> ref(12 * ((size_t)K + 1));
          for (int k = 0; k < K; ++k) std::memcpy(&ref[12 * k], e.values.at(c->map_scans[k]).m, 12 * sizeof(double));
          std::memcpy(&ref[12 * (size_t)K], xj.m, 12 * sizeof(double));
          spec_match(c, xj.m, false, ref.data());
        } else {
          spec_match(c, xj.m);
        }
      }
    };
    bool launched = false, ready = false;  // (moments: captured by the LM's callbacks below)
    int nlin = 0;                          // (rows: this LM's linearizations so far)
    if (mom) {
      // The pairs' moments at the LM's starting values: launched by the LM's first
      // linearization (split form: the host builds the base system and the non-pair
      // terms while the moments kernel runs) and waited for in its lin_end; from then on
      // every linearization of this LM is a host contraction (moments.hpp), no launch.
      auto lin_begin = [&](const std::vector<Pose>& x) {
        HostScope hs(10);
        if (!launched && mom_queued) {  // queued behind the speculative match (spec_match)
          mref.resize((size_t)K + 1);
          for (int k = 0; k <= K; ++k) std::memcpy(mref[k].m, &c->spec_mom_ref[12 * (size_t)k], 12 * sizeof(double));
          momv.resize((size_t)std::max(K, 1) * kMomPairD);
          launched = true;
          FMX_TRACE_("scan %llu it %u: moments queued with the spec match\n", (unsigned long long)j, it);
        }
        if (!launched) {
          mref.resize((size_t)K + 1);
          table.resize(12 * ((size_t)K + 1));
          for (int k = 0; k < K; ++k) mref[k] = x[slot.at(c->map_scans[k])];
          mref[K] = x[slot.at(j)];
          for (int k = 0; k <= K; ++k) std::memcpy(&table[12 * k], mref[k].m, 12 * sizeof(double));
          momv.resize((size_t)std::max(K, 1) * kMomPairD);
          FMX_TRACE_("scan %llu it %u: moments launch K %d chunks %u\n", (unsigned long long)j, it, K, c->max_chunks);
          win_moments_current(c, table.data(), nullptr);  // launch only; win_finish in lin_end
          FMX_TRACE_("  launched\n");
          launched = true;
        }
        maybe_spec(x);
        mxi.resize(K);
        mxj.resize(K);
        for (int k = 0; k < K; ++k) {  // (x outlives the lin_end of this linearization)
          mxi[k] = &x[slot.at(c->map_scans[k])];
          mxj[k] = &x[slot.at(j)];
        }
      };
      auto lin_end = [&](double* G) {
        HostScope hs(10);
        if (!ready) {
          FMX_TRACE_("  wait\n");
          win_finish(c, momv.data());
          FMX_TRACE_("  moments in\n");
          match_counts_fetch(c, false);  // the match finished before the moments
          for (int k = 0; k < K; ++k)  // pairs without rows are never written by the kernel
            if (c->cnt_pl[k] + c->cnt_pt[k] == 0)
              std::fill(&momv[(size_t)k * kMomPairD], &momv[(size_t)(k + 1) * kMomPairD], 0.0);
          mp.resize(K);
          mri.resize(K);
          mrj.assign(K, &mref[K]);
          for (int k = 0; k < K; ++k) {
            mp[k] = &momv[(size_t)k * kMomPairD];
            mri[k] = &mref[k];
          }
          HostScope hp(19);
          mom_prepare(mbatch, K, mp.data(), mri.data(), mrj.data());
          FMX_TRACE_("  prepared\n");
          ready = true;
        }
        HostScope he(18);
        mom_eval(mbatch, mxi.data(), mxj.data(), 1.0 / sigma, G);
        FMX_TRACE_("  eval\n");
      };
      set_lin(g, lin_begin, lin_end);
    } else {
      // split form: launch, the host assembles the non-pair terms, then wait (smoother.hpp).
      // The LM's first linearization goes to the context stream (behind this iteration's
      // match and scatter); its trials to the `lin` stream: their rows were final when the
      // first one's word arrived, and a speculative match queued right after a trial
      // (maybe_spec, on the context stream) then runs beside it instead of behind it.
      auto lin_begin = [&](const std::vector<Pose>& x) {
        table.resize(12 * ((size_t)K + 1));
        for (int k = 0; k < K; ++k) std::memcpy(&table[12 * k], x[slot.at(c->map_scans[k])].m, 12 * sizeof(double));
        std::memcpy(&table[12 * (size_t)K], x[slot.at(j)].m, 12 * sizeof(double));
        HostScope hs(10);
        win_linearize_current(c, table.data(), sigma, nullptr, nlin++ == 0 ? nullptr : c->lin);
        maybe_spec(x);
      };
      auto lin_end = [&](double* G) {
        HostScope hs(10);
        win_finish(c, G);
        match_counts_fetch(c, false);  // the match finished before the linearization
        for (int k = 0; k < K; ++k)
          if (c->cnt_pl[k] + c->cnt_pt[k] == 0) std::fill(G + (size_t)k * kPairG, G + (size_t)(k + 1) * kPairG, 0.0);
      };
      set_lin(g, lin_begin, lin_end);
    }
    HostScope* hs_lm = new HostScope(8);
    FMX_TRACE_("scan %llu it %u: lm\n", (unsigned long long)j, it);
    const WinLMResult R = window_lm(g, window_poses(e));
    FMX_TRACE_("scan %llu it %u: lm done\n", (unsigned long long)j, it);
    delete hs_lm;
    lm_it += R.iters;
    lins += R.lins;
    const Pose after = R.x[slot.at(j)];
    double xi[6];
    logmap(compose(inverse(before), after), xi);
    double dn = 0;
    for (double v : xi) dn += v * v;
    if (std::sqrt(dn) < P.new_pose_threshold) break;
    e.values[j] = after;  // update_current_pose
  }
  // the last match is the scan's constraint set: into the window store (its rows, or
  // its pair moments in FMX_MOMENTS mode)
  record_cons(c, e, j);
  if (mom_full) {
    for (uint32_t k = 0; k < c->K; ++k)
      if (c->cnt_pl[k] + c->cnt_pt[k] > 0) {
        fmx_ctx::Est::Mom& m = e.moms[{j, c->map_scans[k]}];
        m.ref_i = mref[k];
        m.ref_j = mref[c->K];
        m.phi.assign(momv.begin() + (size_t)k * kMomPairD, momv.begin() + (size_t)(k + 1) * kMomPairD);
      }
  } else {
    win_persist(c, j);
  }
  // insert_matches (form.cpp:98-100) reads only the last match (local keypoints and
  // their NN distances), not the poses optimize(false) moves: its kernel goes ahead of
  // the full LM, off the scan's tail
  ensure_pool_room(c, 0, c->n_qpl);
  ensure_pool_room(c, 1, c->n_qpt);
  run_insert(c, j, nullptr);
  inserted = true;
  // keyscan step (form.cpp:104-111): it reads only the constraint counts, so it runs
  // before optimize(false); the next map's scans are known from here on
  keyscan_step(c, e, j, nfeat);
  c->ev_fork.record(c->stream);  // after the insert: the pool is final
  std::vector<uint64_t> map_scans;
  {
    std::set<uint64_t> sset;
    for (int t = 0; t < 2; ++t)
      for (auto& [s, r] : c->pool[t].ranges) sset.insert(s);
    map_scans.assign(sset.begin(), sset.end());
  }
  int spec_builds = 0;
  pf_launch(c, false);  // a host-announced next scan staged by now
  // optimize(false): every stored pair's FeatureFactor (constraints.cpp:294-305)
  std::vector<WinPair> prs;
  if (mom_full) {  // (j ascending, i ascending: the window store's order)
    for (auto& [ji, m] : e.moms) prs.push_back(WinPair{ji.second, ji.first, 0, 0, 0, 0});
  } else {
    prs = win_pairs(c);
  }
  g.lins.clear();
  for (auto& m : e.margs) g.lins.push_back(&m);
  g.pairs.clear();
  for (auto& p : prs) g.pairs.push_back({slot.at(p.i), slot.at(p.j)});
  if (!prs.empty() && !mom_full) win_set_pairs(c, prs, keys);
  // Speculative map build: a trial the LM will probably stop after (predicted decrease
  // within its 1e-5 tolerances, as for the speculative match) gives the poses the next
  // scan's map is built from; build it now on the side stream, behind the insert, while
  // this LM and the next scan's extraction run.  register_scan(j+1) keeps it only if its
  // map inputs are exactly these.
  auto maybe_spec_map = [&](const std::vector<Pose>& x) {
    const double lc = g.trial_lin_change, ce = g.trial_err;
    if (lc >= 0.0 && (lc <= 1e-5 * ce || lc <= 1e-5) && spec_builds < 2 && !map_scans.empty()) {
      ++spec_builds;
      std::vector<double> mpo(12 * map_scans.size());
      for (size_t k = 0; k < map_scans.size(); ++k) std::memcpy(&mpo[12 * k], x[slot.at(map_scans[k])].m, 12 * sizeof(double));
      FMX_TRACE_("  spec map (drain %d)\n", (int)e.spec_map);
      if (e.spec_map) FMX_HIP(hipStreamSynchronize(c->side));  // pinned staging reuse (see register_scan)
      FMX_HIP(hipStreamWaitEvent(c->side, c->ev_fork.last(), 0));
      FMX_TRACE_("  spec map build\n");
      run_map_build(c, map_scans, mpo.data(), P.max_dist_matching, c->side);
      c->ev_join.record(c->side);
      FMX_TRACE_("  spec map queued\n");
      e.spec_map = true;
      e.spec_map_scans = map_scans;
      e.spec_map_poses = std::move(mpo);
    }
  };
  if (mom_full) {
    const size_t np = prs.size();
    mp.resize(np);
    mri.resize(np);
    mrj.resize(np);
    mxi.resize(np);
    mxj.resize(np);
    for (size_t p = 0; p < np; ++p) {
      const fmx_ctx::Est::Mom& m = e.moms.at({prs[p].j, prs[p].i});
      mp[p] = m.phi.data();
      mri[p] = &m.ref_i;
      mrj[p] = &m.ref_j;
    }
    {
      HostScope hp(19);
      mom_prepare(mbatch, (int)np, mp.data(), mri.data(), mrj.data());
    }
    g.lin_begin = nullptr;
    g.lin_end = nullptr;
    g.lin_pairs = [&, np](const std::vector<Pose>& x, double* G) {  // (np: this block's local, by value)
      HostScope hs(10);
      FMX_TRACE_("  full lm lin (lin change %.3e)\n", g.trial_lin_change);
      maybe_spec_map(x);
      for (size_t p = 0; p < np; ++p) {
        mxi[p] = &x[g.pairs[p].first];
        mxj[p] = &x[g.pairs[p].second];
      }
      HostScope he(18);
      mom_eval(mbatch, mxi.data(), mxj.data(), 1.0 / sigma, G);
    };
  } else {
    auto lin_begin = [&](const std::vector<Pose>& x) {
      table.resize(12 * keys.size());
      for (size_t k = 0; k < keys.size(); ++k) std::memcpy(&table[12 * k], x[k].m, 12 * sizeof(double));
      HostScope hs(10);
      win_linearize_stored(c, table.data(), (int)keys.size(), sigma, nullptr);
      maybe_spec_map(x);
    };
    auto lin_end = [&](double* G) {
      HostScope hs(10);
      win_finish(c, G);
    };
    set_lin(g, lin_begin, lin_end);
  }
  FMX_TRACE_("scan %llu: full lm, %zu pairs\n", (unsigned long long)j, prs.size());
  HostScope* hs_lm = new HostScope(9);
  const WinLMResult R = window_lm(g, window_poses(e));
  delete hs_lm;
  FMX_TRACE_("scan %llu: full lm done, %d spec maps\n", (unsigned long long)j, spec_builds);
  lm_it += R.iters;
  lins += R.lins;
  for (size_t k = 0; k < keys.size(); ++k) e.values[keys[k]] = R.x[k];  // update_values
  // gcache = exactly the stored pairs' G at the new values: entries are overwritten in
  // place (their vectors keep their storage), stale ones erased
  std::set<std::pair<uint64_t, uint64_t>> live;
  for (size_t p = 0; p < prs.size(); ++p) {
    const std::pair<uint64_t, uint64_t> k{prs[p].j, prs[p].i};
    e.gcache[k].assign(R.G.begin() + p * kPairG, R.G.begin() + (p + 1) * kPairG);
    live.insert(k);
  }
  for (auto it = e.gcache.begin(); it != e.gcache.end();)
    it = live.count(it->first) ? std::next(it) : e.gcache.erase(it);
}

// ConstraintManager::marginalize (constraints.cpp:120-203): the factors touching the
// marginalized keys (priors, marginal factors, FeatureFactors), linearized at
// m_values, are eliminated onto the remaining keys as a LinearContainerFactor.
void smooth_marginalize(fmx_ctx::Est& e, const std::vector<uint64_t>& marg) {
  HostScope hs(11);
  std::set<uint64_t> M;
  for (uint64_t m : marg)
    if (e.values.count(m)) M.insert(m);
  if (M.empty()) return;
  std::set<uint64_t> keys(M.begin(), M.end());
  std::vector<PriorF> dp;
  std::vector<LinF> dl;
  for (auto it = e.priors.begin(); it != e.priors.end();)
    if (M.count(it->key)) {
      dp.push_back(*it);
      it = e.priors.erase(it);
    } else ++it;
  for (auto it = e.margs.begin(); it != e.margs.end();) {
    bool hit = false;
    for (uint64_t k : it->keys) hit |= M.count(k) > 0;
    if (hit) {
      for (uint64_t k : it->keys) keys.insert(k);
      dl.push_back(std::move(*it));
      it = e.margs.erase(it);
    } else ++it;
  }
  std::vector<std::pair<std::pair<uint64_t, uint64_t>, const std::vector<double>*>> dpairs;
  for (auto& [ji, G] : e.gcache)
    if (M.count(ji.first) || M.count(ji.second)) {
      dpairs.push_back({ji, &G});
      keys.insert(ji.first);
      keys.insert(ji.second);
    }
  std::vector<uint64_t> order(M.begin(), M.end()), rest;
  for (uint64_t k : keys)
    if (!M.count(k)) rest.push_back(k);
  order.insert(order.end(), rest.begin(), rest.end());
  // same factor order as a sorted-Values linearization (priors, linear, pairs), then
  // permuted so the eliminated keys come first
  std::vector<uint64_t> sorted(keys.begin(), keys.end());
  DenseSys S;
  S.init(sorted);
  for (auto& p : dp) S.add_prior(p, e.values.at(p.key));
  for (auto& l : dl) {
    std::vector<Pose> xk;
    for (uint64_t k : l.keys) xk.push_back(e.values.at(k));
    S.add_linf(l, xk);
  }
  for (auto& [ji, G] : dpairs) S.add_pair(S.slot.at(ji.second), S.slot.at(ji.first), G->data());
  DenseSys T;
  T.init(order);
  std::vector<int> map(S.D + 1);
  for (size_t k = 0; k < sorted.size(); ++k)
    for (int d = 0; d < 6; ++d) map[6 * k + d] = 6 * T.slot.at(sorted[k]) + d;
  map[S.D] = T.D;
  for (int r = 0; r <= S.D; ++r)
    for (int cc = 0; cc <= S.D; ++cc) T.at(map[r], map[cc]) = S.at(r, cc);
  LinF L;
  if (!rest.empty() && schur_marginal(T.A, T.D, 6 * (int)M.size(), L.info)) {
    L.keys = rest;
    for (uint64_t k : rest) L.lin.push_back(e.values.at(k));
    e.margs.push_back(std::move(L));
  }
  for (auto it = e.gcache.begin(); it != e.gcache.end();)
    if (M.count(it->first.first) || M.count(it->first.second)) it = e.gcache.erase(it);
    else ++it;
}

size_t num_recent_connections(const fmx_ctx::Est& e, uint64_t s, uint64_t oldest) {  // constraints.cpp:319-336
  size_t cnt = 0;
  for (auto& [j, m] : e.cons) {
    if (j < oldest) continue;
    auto it = m.find(s);
    if (it != m.end()) cnt += it->second.first + it->second.second;
  }
  return cnt;
}

void remove_scan(fmx_ctx* c, uint64_t s) {  // KeypointMap::remove (map.tpp:112-126)
  for (int t = 0; t < 2; ++t) c->pool[t].ranges.erase(s);
}

// The tail of register_scan (form.cpp:104-111): keyscan selection + marginalization
// of the last registered scan.  It changes only host-side window state (which scans
// and factors remain), never the registered poses, so register_scan defers it to the
// next call (where it overlaps that scan's extraction); entry points that read the
// keypoint pool run it first.
// The tail of register_scan (form.cpp:104-111), in two parts.  The keyscan step runs
// as soon as the scan's constraint counts are known (it reads only those): the
// dropped scans leave the keypoint pool, so the next map no longer holds them.  The
// marginalization proper (host-only factor bookkeeping; it moves no pose, so the map
// does not depend on it) is deferred to the next register_scan, where it overlaps
// that scan's extraction; entry points that read the estimator state run it first.
void keyscan_step(fmx_ctx* c, fmx_ctx::Est& e, uint64_t j, uint32_t nfeat) {
  auto marg = e.ks.step(j, nfeat, [&](uint64_t i) { return num_recent_connections(e, i, e.ks.oldest_rf()); });
  for (uint64_t m : marg) remove_scan(c, m);
  e.tail_marg = std::move(marg);
  e.tail_pending = true;
}
// the constraint counts of scan j's last match (ConstraintManager bookkeeping)
void record_cons(fmx_ctx* c, fmx_ctx::Est& e, uint64_t j) {
  match_counts_fetch(c);
  auto& cj = e.cons[j];
  e.last_mpl = e.last_mpt = 0;
  for (uint32_t k = 0; k < c->K; ++k) {
    cj[c->map_scans[k]] = {c->cnt_pl[k], c->cnt_pt[k]};
    e.last_mpl += c->cnt_pl[k];
    e.last_mpt += c->cnt_pt[k];
  }
  e.last_map_pl = c->map.n[0];
  e.last_map_pt = c->map.n[1];
}
void finish_tail(fmx_ctx* c, fmx_ctx::Est& e) {
  if (!e.tail_pending) return;
  e.tail_pending = false;
  const std::vector<uint64_t> marg = std::move(e.tail_marg);
  e.tail_marg.clear();
  if (marg.empty()) return;
  HostScope hs(5);
  const fmx_params& P = c->P;
  if (!P.disable_smoothing) smooth_marginalize(e, marg);
  for (uint64_t m : marg) {
    if (!P.disable_smoothing) win_remove(c, m);
    for (auto it = e.moms.begin(); it != e.moms.end();)  // pairs (m, j) and (i, m)
      it = it->first.first == m || it->first.second == m ? e.moms.erase(it) : std::next(it);
    e.values.erase(m);
    e.cons.erase(m);
    for (auto& [jj, mm] : e.cons) mm.erase(m);
  }
}
void finish_tail(fmx_ctx* c) {
  if (c->est) finish_tail(c, *c->est);
}

void register_scan(fmx_ctx* c, const float* xyzw, size_t n, int on_dev, fmx_feature_counts* out) {
  HostScope hs_all(0);
  // host time spent outside register_scan since the previous call returned (diagnostic)
  static double last_ret = 0.0;
  struct RetStamp {
    ~RetStamp() {
      if (host_timing().on) last_ret = now_s();
    }
  } ret_stamp;
  if (host_timing().on && last_ret > 0.0) {
    host_timing().t[15] += now_s() - last_ret;
    host_timing().n[15]++;
  }
  if (!c->est) {
    c->est = new fmx_ctx::Est();
    c->est->ks.P = &c->P;
  }
  fmx_ctx::Est& e = *c->est;
  const fmx_params& P = c->P;
  const size_t RC = (size_t)P.extraction.num_rows * (size_t)P.extraction.num_columns;
  if (n != RC)
    throw StatusError(FMX_E_SIZE, "Provided scan does not match the expected size " + std::to_string(RC) +
                                      " != " + std::to_string(n));
  const uint64_t j = e.init ? e.scan + 1 : 0;
  FMX_TRACE_("scan %llu: register_scan\n", (unsigned long long)j);
  const uint64_t waits0 = c->host_waits;
  const uint64_t spec0 = c->spec_launched, hits0 = c->spec_hits, pf0 = c->pf_used;
  c->spec_valid = false;  // a new map and query set: no speculation carries over
  // Host work that only needs the estimator state runs while this scan's extraction
  // kernels execute: the previous scan's deferred tail (keyscan step +
  // marginalization), then step(prediction) (constraints.cpp:206-223) and the map
  // build inputs.  to_voxel_map x2, voxel width = max_dist_matching (form.cpp:61-65):
  // the map holds only earlier scans at their current estimates, so it does not
  // depend on this scan's features.
  std::vector<uint64_t> scans;
  std::vector<double> poses;
  // prepare: the keyscan step, prediction and map inputs (the map build is queued right
  // after it); finish: the marginalization proper and the new scan's constraint slots.
  bool map_spec_used = false;
  auto prepare = [&] {
    const Pose pred = predict_next(e, e.tail_pending ? e.tail_marg : std::vector<uint64_t>{});
    std::set<uint64_t> sset;
    for (int t = 0; t < 2; ++t)
      for (auto& [s, r] : c->pool[t].ranges) sset.insert(s);
    scans.assign(sset.begin(), sset.end());
    poses.resize(12 * scans.size());
    for (size_t k = 0; k < scans.size(); ++k) std::memcpy(&poses[12 * k], e.values.at(scans[k]).m, 12 * sizeof(double));
    e.scan = j;
    e.init = true;
    e.values[j] = pred;
    if (j == 0) e.priors.push_back(PriorF{0, pred, 1e-3});  // addPrior (constraints.cpp:217-220)
  };
  LinF fast;
  auto finish = [&] {
    finish_tail(c, e);
    auto& cj = e.cons[j];
    for (auto& [i, T] : e.values)
      if (i != j) cj[i] = {0, 0};
    if (!P.disable_smoothing) fast = fast_linear(e);  // m_fast_linear (constraints.cpp:257-288)
  };
  // The map build goes to the side stream and is queued while the extraction kernels
  // run (extraction occupies one CU per scan line, so the build's kernels take the
  // idle CUs, and its host launch cost hides behind the extraction wait).
  fmx_feature_counts fc{};
  c->ev_fork.record(c->stream);  // after the previous scan's insert
  auto map_inputs = [&] {
    prepare();
    const bool spec_ok = e.spec_map && e.spec_map_scans == scans && e.spec_map_poses.size() == poses.size() &&
                         std::memcmp(e.spec_map_poses.data(), poses.data(), poses.size() * sizeof(double)) == 0;
    if (e.spec_map) ++(spec_ok ? c->spec_map_hits : c->spec_map_misses);
    map_spec_used = spec_ok;
    if (!spec_ok) {
      HostScope hs_map(3);
      // a discarded speculative build may still be reading the pinned pose staging
      // buffer this build rewrites: drain it first (misses are rare)
      if (e.spec_map) FMX_HIP(hipStreamSynchronize(c->side));
      FMX_HIP(hipStreamWaitEvent(c->side, c->ev_fork.last(), 0));
      run_map_build(c, scans, poses.data(), P.max_dist_matching, c->side);
      c->ev_join.record(c->side);
    }
    e.spec_map = false;
  };
  {
    HostScope hs_ex(2);
    if (pf_take(c, xyzw, n, on_dev, j, &fc)) {
      // pipelined: the features were extracted during the previous registration.  The
      // first ICP match (at the prediction) is queued before the host's finish() work,
      // which then overlaps it; the ICP loop takes it as a speculative match.
      map_inputs();
      FMX_HIP(hipStreamWaitEvent(c->stream, c->ev_join.last(), 0));
      if (!P.disable_smoothing) {
        if (!lin_rows()) {  // + the first ICP iteration's moments (its x0: the window values)
          std::vector<double> ref(12 * ((size_t)c->K + 1));
          for (uint32_t k = 0; k < c->K; ++k) std::memcpy(&ref[12 * k], e.values.at(c->map_scans[k]).m, 12 * sizeof(double));
          std::memcpy(&ref[12 * (size_t)c->K], e.values.at(j).m, 12 * sizeof(double));
          spec_match(c, e.values.at(j).m, true, ref.data());
        } else {
          spec_match(c, e.values.at(j).m, true);
        }
      }
      finish();
    } else {
      do_extract(c, xyzw, n, j, on_dev, &fc, [&] {
        map_inputs();
        finish();
      });
    }
  }
  FMX_HIP(hipStreamWaitEvent(c->stream, c->ev_join.last(), 0));
  FMX_TRACE_("scan %llu: extracted %u + %u, map queued\n", (unsigned long long)j, fc.planar, fc.point);
  HostScope* hs_icp = new HostScope(4);
  uint64_t icp = 0, lm_it = 0, lins = 0;
  bool inserted = false;
  if (!P.disable_smoothing) {
    smooth_register(c, e, j, fc.planar + fc.point, fast, icp, lm_it, lins, inserted);
  } else {
    // ICP loop (form.cpp:67-89) with the LM on the host (one sync per linearization)
    DeviceLM lm{c, e, P.planar_constraint_sigma};
    bool converged = false;
    Pose last_after = e.values.at(j);
    for (uint32_t it = 0; it < P.max_num_rematches; ++it) {
      ++icp;
      const Pose before = e.values.at(j);
      run_match(c, before.m, P.max_dist_matching, P.min_dist_map, false);  // query order
      pf_launch(c, false);  // the announced next scan's extraction, behind this match (host: once staged)
      int li = 0;
      const Pose after = lm.optimize(before, &li);
      lm_it += li;
      double xi[6];
      logmap(compose(inverse(before), after), xi);
      double dn = 0;
      for (double x : xi) dn += x * x;
      if (std::sqrt(dn) < P.new_pose_threshold) {
        converged = true;
        last_after = after;
        break;
      }
      e.values[j] = after;  // update_current_pose
    }
    // optimize(false) + update_values (form.cpp:92-93).  In the single-pose mode the
    // graph is the same current-scan factor set (get_single_graph ignores `fast`), so
    // after a converged break it restarts from `before` with the same data and
    // returns `after` again, bit for bit: reuse it.  Otherwise run it.
    if (converged) {
      e.values[j] = last_after;
    } else {
      int li = 0;
      e.values[j] = lm.optimize(e.values.at(j), &li);
      lm_it += li;
    }
    lins = lm.linearizations;
  }
  delete hs_icp;
  pf_launch(c, true);  // an announced host scan whose staging outlasted the ICP loop
  if (!inserted) {  // single-pose mode
    HostScope hs_tail(5);
    record_cons(c, e, j);
    // insert_matches (form.cpp:98-100) from the last match
    ensure_pool_room(c, 0, c->n_qpl);
    ensure_pool_room(c, 1, c->n_qpt);
    run_insert(c, j, nullptr);
    keyscan_step(c, e, j, fc.planar + fc.point);  // marginalization: deferred (finish_tail)
  }
  FMX_TRACE_("scan %llu: done\n", (unsigned long long)j);
  c->stats[0] = icp;
  c->stats[1] = lm_it;
  c->stats[2] = e.last_mpl;
  c->stats[3] = e.last_mpt;
  c->stats[4] = e.last_map_pl;
  c->stats[5] = e.last_map_pt;
  c->stats[6] = lins;
  c->stats[7] = scans.size();
  c->stats[8] = c->host_waits - waits0;
  c->stats[9] = c->spec_launched - spec0;
  c->stats[10] = c->spec_hits - hits0;
  c->stats[11] = map_spec_used ? 1 : 0;
  c->stats[12] = c->pf_used - pf0;
  c->stats[13] = e.values.size();
  if (out) *out = fc;
}

}  // namespace

// ============================================================================ C ABI
extern "C" {

int fmx_abi_version(void) { return FMX_ABI_VERSION; }

void fmx_default_params(fmx_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  auto& e = p->extraction;  // extraction.hpp:59-88
  e.neighbor_points = 5;
  e.num_sectors = 6;
  e.planar_threshold = 1.0;
  e.planar_feats_per_sector = 50;
  e.point_feats_per_sector = 3;
  e.radius = 1.0;
  e.min_points = 5;
  e.min_norm_squared = 1.0;
  e.max_norm_squared = 100.0 * 100.0;
  e.num_columns = 1024;
  e.num_rows = 64;
  p->max_dist_matching = 0.8;  // matcher.hpp:32-41
  p->new_pose_threshold = 1e-4;
  p->max_num_rematches = 30;
  p->planar_constraint_sigma = 0.1;  // constraints.hpp:60
  p->disable_smoothing = 0;  // ConstraintManager default (constraints.hpp:56): smoothing
  p->max_num_keyscans = 50;  // keyscanner.hpp:55-64
  p->max_steps_unused_keyscan = 10;
  p->max_num_recent_scans = 10;
  p->keyscan_match_ratio = 0.1;
  p->min_dist_map = 0.1;  // map.hpp:97-100
  p->keypoint_pool_capacity = 4u << 20;
  p->max_pairs = 1024;
  p->voxel_subdivision = 1;
}


fmx_status fmx_create(const fmx_params* p, int device, fmx_ctx** out) {
  if (!p || !out) return FMX_E_INVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return FMX_E_HIP;
  if (device < 0 || device >= ndev) return FMX_E_INVAL;
  fmx_ctx* c = new (std::nothrow) fmx_ctx();
  if (!c) return FMX_E_OOM;
  c->P = *p;
  c->device = device;
  fmx_status st = guard(c, [&] {
    // the context stream carries the registration's critical path: highest priority
    int prio_lo = 0, prio_hi = 0;
    FMX_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    FMX_HIP(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_hi));
    FMX_HIP(hipStreamCreateWithPriority(&c->lin, hipStreamNonBlocking, prio_hi));
    // The side streams (pipelined extraction, speculative map build) run on a quarter of
    // the CUs: their 1024-thread blocks (k_normals: ~147 KB of LDS each) otherwise occupy
    // every CU while the ICP loop's window linearizations and matches wait for CU room (a
    // linearization overlapping k_normals took 39 instead of 10 us,
    // profiles/r5_c4_trace_unprofiled.txt).  Measured (profiles/r6_ab_side_cus.txt, 3 reps
    // x 120 scans): unmasked 1412, 32 CUs 1316, 64 CUs 1460, 128 CUs 1442 scans/s; the
    // extraction itself, off the critical path, takes ~3.5x as long (and at 32 CUs no
    // longer finishes before the next scan needs it).  Mask bits come in groups of 8 = one
    // CU of each XCD (tools/flagbench/cumaskmap.hip), so any aligned run of 64 bits is 8 CUs
    // of every XCD.  Successive contexts of the process take successive quarters, so that
    // contexts serving concurrent streams do not pile their side work onto the same CUs
    // (4 streams on one GPU: 1421-1667 scans/s with one shared quarter, profiles/
    // r6_end_bench_spread.txt).  FMX_SIDE_CUS: the side streams' CU count (0 = all CUs;
    // several contexts serving concurrent streams measured faster unmasked:
    // profiles/r6_ab_side_cus_streams.txt).
    {
      static std::atomic<uint32_t> ctx_seq{0};
      hipDeviceProp_t pr;
      FMX_HIP(hipGetDeviceProperties(&pr, device));
      const char* cus = std::getenv("FMX_SIDE_CUS");
      const int ncu = pr.multiProcessorCount, n = cus ? std::min(ncu, std::atoi(cus)) : std::max(1, ncu / 4);
      std::vector<uint32_t> m((ncu + 31) / 32, 0u);
      if (n <= 0) {
        std::fill(m.begin(), m.end(), 0xFFFFFFFFu);
      } else {
        const int q = (int)(ctx_seq.fetch_add(1u) % (uint32_t)std::max(1, ncu / n));
        for (int i = ncu - n * (q + 1); i < ncu - n * q; ++i) m[i / 32] |= 1u << (i % 32);
      }
      FMX_HIP(hipExtStreamCreateWithCUMask(&c->side, (uint32_t)m.size(), m.data()));
      FMX_HIP(hipExtStreamCreateWithCUMask(&c->side2, (uint32_t)m.size(), m.data()));
    }
    c->ev_fork.create();
    c->ev_join.create();
    c->ev_pf.create();
    c->ev_pf_fork.create();
    const uint64_t cap = p->keypoint_pool_capacity ? p->keypoint_pool_capacity : (4u << 20);
    c->pool[0].planar = true;
    c->pool[1].planar = false;
    c->pool[0].pos.ensure(cap);
    c->pool[0].nrm.ensure(cap);
    c->pool[1].pos.ensure(cap);
  });
  if (st != FMX_OK) {
    fmx_destroy(c);
    return st;
  }
  *out = c;
  return FMX_OK;
}

void fmx_destroy(fmx_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->side) (void)hipStreamSynchronize(c->side);
  if (c->side2) (void)hipStreamSynchronize(c->side2);
  for (auto& e : c->prof.free_events) (void)hipEventDestroy(e);
  for (auto& pe : c->prof.pending) {
    (void)hipEventDestroy(pe.a);
    (void)hipEventDestroy(pe.b);
  }
  c->prof.wring.release();
  delete c->est;
  comm_destroy(c);
  c->d_sum.release();
  c->h_hold.release();
  // DBuf/HBuf members do not free in their destructors: release explicitly.
  c->scan.release(); c->planar_mask.release(); c->sel_slots.release(); c->pt_slots.release();
  c->row_counts.release(); c->row_ok.release(); c->row_off.release(); c->closest.release();
  c->nrm_slots.release(); c->scan_scratch.release(); c->dev_u32.release(); c->h_u32.release();
  c->q_pl_pos.release(); c->q_pl_nrm.release(); c->q_pt_pos.release(); c->q_pl_idx.release(); c->q_pt_idx.release();
  c->nq_pl_pos.release(); c->nq_pl_nrm.release(); c->nq_pt_pos.release(); c->nq_pl_idx.release(); c->nq_pt_idx.release();
  c->n_planar_mask.release(); c->h_pf.release();
  c->stager.stop();  // no helper touches the staging buffers after this
  for (uint8_t* b : {c->pin_seq, c->pin_pf[0], c->pin_pf[1]})
    if (b) (void)hipHostFree(b);
  c->pf_scan.release();
  c->scan3.release();
  c->pf_scan3.release();
  for (auto& B : c->scanbuf)
    if (B.p) (void)hipHostFree(B.p);
  for (int t = 0; t < 2; ++t) {
    c->pool[t].pos.release(); c->pool[t].nrm.release();
    c->segs[t].release(); c->h_segs[t].release();
  }
  {
    auto& M = c->map;
    M.table.release(); M.ccnt.release(); M.state.release(); M.rinfo.release(); M.claim.release(); M.dense.release();
    M.pos.release(); M.nrm.release();
  }
  c->h_mapposes.release(); c->map_blob.release(); c->h_mapinfo.release();
  c->blk_lo.release(); c->blk_hi.release(); c->h_work.release();
  c->work.release(); c->pair_base.release();
  c->m_pair.release(); c->m_d2.release(); c->m_pi.release(); c->m_ni.release(); c->m_ins.release();
  c->m_rec.release(); c->m_cell.release();
  c->hist.release(); c->hist_off.release(); c->thist.release(); c->c_pl.release(); c->c_pt.release(); c->pair_counts.release();
  c->chunk_range.release(); c->chunks.release(); c->n_chunks.release();
  c->bpart.release(); c->ticket.release(); c->h_poses.release(); c->h_G.release(); c->h_i32.release();
  c->h_corr.release(); c->h_meta.release(); c->h_counts.release(); c->h_flag.release();
  c->mcnt.release(); c->mticket.release(); c->ins_blk.release(); c->ins_off.release();
  c->fz_work.release(); c->fz_h_work.release(); c->fz_tickets.release(); c->mprof.release();
  c->cert_b2.release();
  {
    auto& S = c->spec;
    S.m_pair.release(); S.m_d2.release(); S.m_pi.release(); S.m_ni.release(); S.m_ins.release();
    S.hist.release(); S.hist_off.release(); S.thist.release(); S.c_pl.release(); S.c_pt.release();
    S.pair_counts.release(); S.chunk_range.release(); S.chunks.release(); S.n_chunks.release(); S.pair_base.release();
    S.work.release(); S.mcnt.release(); S.mticket.release(); S.ins_blk.release(); S.ins_off.release();
    S.h_counts.release(); S.h_work.release();
  }
  {
    auto& W = c->win;
    for (int b = 0; b < 2; ++b) { W.pl[b].release(); W.pt[b].release(); }
    W.meta.release(); if (W.meta_ev) (void)hipEventDestroy(W.meta_ev); W.partials.release(); W.dposes.release();
    W.pticket.release(); W.dticket.release(); W.dflag.release(); W.dbg.release(); W.hG.release(); W.hM.release(); W.hposes.release(); W.hmeta.release();
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->side2) (void)hipStreamDestroy(c->side2);
  if (c->lin) (void)hipStreamDestroy(c->lin);
  c->ev_fork.destroy();
  c->ev_join.destroy();
  c->ev_pf.destroy();
  c->ev_pf_fork.destroy();
  delete c;
}

const char* fmx_last_error(const fmx_ctx* c) { return c ? c->err.c_str() : "null context"; }

fmx_status fmx_extract(fmx_ctx* c, const float* xyzw, size_t n, uint64_t scan, int on_dev, fmx_feature_counts* out) {
  return guard<false>(c, [&] {
    drop_match(c);
    do_extract(c, xyzw, n, scan, on_dev, out);
  });
}

fmx_status fmx_extract_download(fmx_ctx* c, float* planar, uint32_t* planar_index, float* point,
                                uint32_t* point_index, uint8_t* planar_mask) {
  return guard(c, [&] {
    if (!c->have_queries) throw StatusError(FMX_E_STATE, "no extraction");
    FMX_HIP(hipStreamSynchronize(c->stream));
    const uint32_t npl = c->n_qpl, npt = c->n_qpt;
    if (planar) {
      std::vector<float4> a(npl), b(npl);
      FMX_HIP(hipMemcpy(a.data(), c->q_pl_pos.p, npl * sizeof(float4), hipMemcpyDeviceToHost));
      FMX_HIP(hipMemcpy(b.data(), c->q_pl_nrm.p, npl * sizeof(float4), hipMemcpyDeviceToHost));
      for (uint32_t i = 0; i < npl; ++i) {
        planar[6 * i] = a[i].x; planar[6 * i + 1] = a[i].y; planar[6 * i + 2] = a[i].z;
        planar[6 * i + 3] = b[i].x; planar[6 * i + 4] = b[i].y; planar[6 * i + 5] = b[i].z;
      }
    }
    if (planar_index) FMX_HIP(hipMemcpy(planar_index, c->q_pl_idx.p, npl * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (point) {
      std::vector<float4> a(npt);
      FMX_HIP(hipMemcpy(a.data(), c->q_pt_pos.p, npt * sizeof(float4), hipMemcpyDeviceToHost));
      for (uint32_t i = 0; i < npt; ++i) {
        point[3 * i] = a[i].x; point[3 * i + 1] = a[i].y; point[3 * i + 2] = a[i].z;
      }
    }
    if (point_index) FMX_HIP(hipMemcpy(point_index, c->q_pt_idx.p, npt * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (planar_mask) {
      if (!c->rows) throw StatusError(FMX_E_STATE, "no device extraction");
      FMX_HIP(hipMemcpy(planar_mask, c->planar_mask.p, (size_t)c->rows * c->cols, hipMemcpyDeviceToHost));
    }
  });
}

fmx_status fmx_set_queries(fmx_ctx* c, uint64_t scan, const float* planar, uint32_t npl, const float* point,
                           uint32_t npt) {
  return guard<false>(c, [&] {
    if ((npl && !planar) || (npt && !point)) throw StatusError(FMX_E_INVAL, "null features");
    drop_match(c);
    set_queries(c, scan, planar, npl, point, npt);
  });
}

fmx_status fmx_keypoints_add(fmx_ctx* c, uint64_t scan, const float* planar, uint32_t npl, const float* point,
                             uint32_t npt) {
  return guard(c, [&] {
    finish_tail(c);
    if ((npl && !planar) || (npt && !point)) throw StatusError(FMX_E_INVAL, "null features");
    pool_add(c, 0, scan, planar, npl);
    pool_add(c, 1, scan, point, npt);
  });
}

fmx_status fmx_keypoints_add_device(fmx_ctx* c, uint64_t scan, const float* plp, const float* pln, uint32_t npl,
                                    const float* ptp, uint32_t npt) {
  return guard(c, [&] {
    finish_tail(c);
    if ((npl && (!plp || !pln)) || (npt && !ptp)) throw StatusError(FMX_E_INVAL, "null features");
    pool_add_device(c, 0, scan, plp, pln, npl);
    pool_add_device(c, 1, scan, ptp, nullptr, npt);
  });
}

fmx_status fmx_set_queries_device(fmx_ctx* c, uint64_t scan, const float* plp, const float* pln, uint32_t npl,
                                  const float* ptp, uint32_t npt) {
  return guard<false>(c, [&] {
    if ((npl && (!plp || !pln)) || (npt && !ptp)) throw StatusError(FMX_E_INVAL, "null features");
    drop_match(c);
    set_queries_device(c, scan, plp, pln, npl, ptp, npt);
  });
}

fmx_status fmx_keypoints_remove(fmx_ctx* c, uint64_t scan) {
  return guard(c, [&] { finish_tail(c); remove_scan(c, scan); });
}

fmx_status fmx_map_build(fmx_ctx* c, const uint64_t* scans, const double* poses, uint32_t n, double w) {
  return guard(c, [&] {
    finish_tail(c);
    if (n && (!scans || !poses)) throw StatusError(FMX_E_INVAL, "null scans/poses");
    if (!(w > 0)) throw StatusError(FMX_E_INVAL, "voxel width must be > 0");
    std::vector<uint64_t> s(scans, scans + n);
    run_map_build(c, s, poses, w);
  });
}

fmx_status fmx_match(fmx_ctx* c, const double pose_j[12], double max_dist, uint32_t* cpl, uint32_t* cpt) {
  return guard<false>(c, [&] {
    c->lazy.pending = false;  // a newer match replaces a deferred one
    ++c->corr_gen;
    if (!c->have_map) throw StatusError(FMX_E_STATE, "fmx_map_build first");
    if (!c->have_queries) throw StatusError(FMX_E_STATE, "no queries (fmx_extract or fmx_set_queries)");
    if (!(max_dist > 0)) throw StatusError(FMX_E_INVAL, "max_dist must be > 0");
    if (!pose_j) throw StatusError(FMX_E_INVAL, "null pose");
    // validated here, not when a deferred match is launched (the error belongs to this call)
    check_match_reach(c, max_dist, c->P.min_dist_map);
    // no count outputs on a large query set (the one-lane-per-query build): deferred,
    // so that fmx_linearize_matched at this pose can run fused with it
    const bool defer = !cpl && !cpt && match_group_for((uint64_t)c->n_qpl + c->n_qpt, c->K) == 1;
    if (defer) {
      c->lazy.pending = true;
      std::memcpy(c->lazy.pose, pose_j, sizeof(c->lazy.pose));
      c->lazy.max_dist = max_dist;
    } else {
      run_match(c, pose_j, max_dist, c->P.min_dist_map, true, true);  // rows scattered when read
    }
    // the map's range-error word is read back once per build; with no count outputs
    // requested the call then returns without waiting (the next consumer of the match
    // results waits for them: fmx_linearize_matched, fmx_match_download, ...)
    if (!c->map_err_checked) {
      c->h_u32.ensure(8);
      FMX_HIP(hipMemcpyAsync(c->h_u32.p, c->map_err_p, 4, hipMemcpyDeviceToHost, c->stream));
      FMX_HIP(hipStreamSynchronize(c->stream));
      if (c->h_u32.p[0]) throw StatusError(FMX_E_RANGE, "voxel coordinate outside the packed-key range");
      c->map_err_checked = true;
    }
    if (!cpl && !cpt) return;
    match_counts_fetch(c);
    if (cpl) std::memcpy(cpl, c->cnt_pl.data(), c->K * sizeof(uint32_t));
    if (cpt) std::memcpy(cpt, c->cnt_pt.data(), c->K * sizeof(uint32_t));
  });
}

fmx_status fmx_match_download(fmx_ctx* c, int32_t* pair, double* d2, double* pi, double* ni) {
  return guard(c, [&] {
    if (!c->have_match) throw StatusError(FMX_E_STATE, "no match results");
    FMX_HIP(hipStreamSynchronize(c->stream));
    const uint32_t nq = c->n_qpl + c->n_qpt;
    if (pair) FMX_HIP(hipMemcpy(pair, c->m_pair.p, nq * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (d2) FMX_HIP(hipMemcpy(d2, c->m_d2.p, nq * sizeof(double), hipMemcpyDeviceToHost));
    if (pi) {
      std::vector<double4> a(nq);
      FMX_HIP(hipMemcpy(a.data(), c->m_pi.p, nq * sizeof(double4), hipMemcpyDeviceToHost));
      for (uint32_t i = 0; i < nq; ++i) {
        pi[3 * i] = a[i].x; pi[3 * i + 1] = a[i].y; pi[3 * i + 2] = a[i].z;
      }
    }
    if (ni) {
      std::vector<double4> a(c->n_qpl);
      FMX_HIP(hipMemcpy(a.data(), c->m_ni.p, c->n_qpl * sizeof(double4), hipMemcpyDeviceToHost));
      for (uint32_t i = 0; i < c->n_qpl; ++i) {
        ni[3 * i] = a[i].x; ni[3 * i + 1] = a[i].y; ni[3 * i + 2] = a[i].z;
      }
    }
  });
}

fmx_status fmx_map_insert(fmx_ctx* c, double min_dist_map, uint32_t* n_inserted) {
  return guard(c, [&] {
    if (!c->have_match) throw StatusError(FMX_E_STATE, "no match results");
    if (min_dist_map != c->P.min_dist_map)
      throw StatusError(FMX_E_INVAL, "min_dist_map must equal the context's (fixed at match time)");
    ensure_pool_room(c, 0, c->n_qpl);
    ensure_pool_room(c, 1, c->n_qpt);
    uint32_t n[2];
    run_insert(c, c->q_scan, n);
    if (n_inserted) {
      n_inserted[0] = n[0];
      n_inserted[1] = n[1];
    }
  });
}

fmx_status fmx_corr_set(fmx_ctx* c, uint32_t K, const uint32_t* np, const double* ppi, const double* pni,
                        const double* ppj, const uint32_t* nt, const double* tpi, const double* tpj) {
  return guard(c, [&] {
    if (K && (!np || !nt)) throw StatusError(FMX_E_INVAL, "null counts");
    ++c->corr_gen;
    upload_corr(c, K, np, ppi, pni, ppj, nt, tpi, tpj);
  });
}

fmx_status fmx_linearize(fmx_ctx* c, const double* pi, const double* pj, double sigma, int single, double* G,
                         double* err) {
  return guard(c, [&] {
    if (!(sigma > 0)) throw StatusError(FMX_E_INVAL, "sigma must be > 0");
    if (c->K && (!pi || !pj)) throw StatusError(FMX_E_INVAL, "null poses");
    win_linearize_pairs(c, pi, pj, sigma, single ? 1 : 0, G, err);
  });
}

fmx_status fmx_moments(fmx_ctx* c, const double* pi, const double* pj, double* mom) {
  return guard(c, [&] {
    if (c->K && (!pi || !pj || !mom)) throw StatusError(FMX_E_INVAL, "null poses / output");
    win_moments_pairs(c, pi, pj, mom);
  });
}

fmx_status fmx_moments_contract(uint32_t K, const double* mom, const double* ri, const double* rj, const double* pi,
                                const double* pj, double sigma, double* G, double* err) {
  if (K == 0) return FMX_OK;
  if (!mom || !ri || !rj || !pi || !pj || !(sigma > 0)) return FMX_E_INVAL;
  try {
    std::vector<const double*> m(K);
    std::vector<const Pose*> a(K), b(K), x(K), y(K);
    for (uint32_t k = 0; k < K; ++k) {
      m[k] = mom + (size_t)kMomPairD * k;
      a[k] = reinterpret_cast<const Pose*>(ri + 12 * (size_t)k);
      b[k] = reinterpret_cast<const Pose*>(rj + 12 * (size_t)k);
      x[k] = reinterpret_cast<const Pose*>(pi + 12 * (size_t)k);
      y[k] = reinterpret_cast<const Pose*>(pj + 12 * (size_t)k);
    }
    std::vector<double> g((size_t)K * 92);
    MomBatch mb;
    mom_prepare(mb, (int)K, m.data(), a.data(), b.data());
    mom_eval(mb, x.data(), y.data(), 1.0 / sigma, g.data());
    for (uint32_t k = 0; k < K; ++k) {
      if (G) std::memcpy(G + 91 * (size_t)k, &g[92 * (size_t)k], 91 * sizeof(double));
      if (err) err[k] = g[92 * (size_t)k + 91];
    }
    return FMX_OK;
  } catch (const std::bad_alloc&) {
    return FMX_E_OOM;
  }
}

fmx_status fmx_error(fmx_ctx* c, const double* pi, const double* pj, double sigma, double* err) {
  return guard(c, [&] {
    if (!(sigma > 0)) throw StatusError(FMX_E_INVAL, "sigma must be > 0");
    if (c->K && (!pi || !pj)) throw StatusError(FMX_E_INVAL, "null poses");
    win_linearize_pairs(c, pi, pj, sigma, 2, nullptr, err);
  });
}

fmx_status fmx_linearize_matched(fmx_ctx* c, const double pose_j[12], double sigma, double out[29]) {
  return guard<false>(c, [&] {
    if (!(sigma > 0)) throw StatusError(FMX_E_INVAL, "sigma must be > 0");
    if (!pose_j || !out) throw StatusError(FMX_E_INVAL, "null pose / output");
    if (c->lazy.pending && std::memcmp(pose_j, c->lazy.pose, sizeof(c->lazy.pose)) == 0) {
      // the deferred match at this very pose: match + linearization fused, no per-query
      // results (the match stays deferred for any later reader)
      run_match_linearize_total(c, pose_j, c->lazy.max_dist, sigma, out);
      return;
    }
    settle_match(c);
    if (!c->have_match) throw StatusError(FMX_E_STATE, "no match results");
    run_linearize_total(c, pose_j, sigma, out);
  });
}

fmx_status fmx_register_points(fmx_ctx* c, const double pose_init[12], double max_dist, double sigma,
                               uint32_t max_iters, double threshold, double pose_out[12], uint32_t* iters) {
  return guard<false>(c, [&] {
    c->lazy.pending = false;  // replaced by this loop's matches
    if (!c->have_map) throw StatusError(FMX_E_STATE, "fmx_map_build first");
    if (!c->have_queries) throw StatusError(FMX_E_STATE, "no queries (fmx_extract or fmx_set_queries)");
    if (!pose_init || !pose_out) throw StatusError(FMX_E_INVAL, "null pose");
    if (!(max_dist > 0) || !(sigma > 0) || !(threshold >= 0)) throw StatusError(FMX_E_INVAL, "bad max_dist / sigma");
    const bool fused = match_group_for((uint64_t)c->n_qpl + c->n_qpt, c->K) == 1;
    Pose T;
    std::memcpy(T.m, pose_init, sizeof(T.m));
    uint32_t it = 0;
    double S[29];
    while (it < max_iters) {
      // Matcher::match at T + the summed single-pose system (all-reduced when sharded)
      if (fused) {
        run_match_linearize_total(c, T.m, max_dist, sigma, S);
        // the last match stays available (launched on demand) when run_match accepts it
        c->lazy.pending = match_reach_ok(c, max_dist, c->P.min_dist_map);
        std::memcpy(c->lazy.pose, T.m, sizeof(T.m));
        c->lazy.max_dist = max_dist;
      } else {
        run_match(c, T.m, max_dist, c->P.min_dist_map, false);
        run_linearize_total(c, T.m, sigma, S);
      }
      ++it;
      // Gauss-Newton on X(j): H dx = g from the packed 7 x 7 [H_j b]^T [H_j b]
      double H[6][6], g[6], dx[6];
      for (int r = 0; r < 7; ++r)
        for (int q = r; q < 7; ++q) {
          const double v = S[r * 7 - r * (r - 1) / 2 + (q - r)];
          if (q < 6) H[r][q] = H[q][r] = v;
          else if (r < 6) g[r] = v;
        }
      if (!chol_solve6(H, g, dx)) throw StatusError(FMX_E_STATE, "singular normal equations (too few matches)");
      T = compose(T, expmap(dx));
      double n2 = 0.0;
      for (double x : dx) n2 += x * x;
      if (std::sqrt(n2) < threshold) break;  // form.cpp:83-88
    }
    std::memcpy(pose_out, T.m, sizeof(T.m));
    if (iters) *iters = it;
  });
}

fmx_status fmx_comm_unique_id(uint8_t id[128]) {
  if (!id) return FMX_E_INVAL;
  try {
    comm_unique_id(id);
    return FMX_OK;
  } catch (const StatusError& e) {
    return e.st;
  } catch (const std::exception&) {
    return FMX_E_RCCL;
  }
}

fmx_status fmx_comm_init(fmx_ctx* c, const uint8_t id[128], int nranks, int rank) {
  return guard(c, [&] {
    if (!id) throw StatusError(FMX_E_INVAL, "null id");
    FMX_HIP(hipStreamSynchronize(c->stream));
    comm_init(c, id, nranks, rank);
  });
}

fmx_status fmx_next_scan(fmx_ctx* c, const float* xyzw, size_t n, int on_dev) {
  return guard<false>(c, [&] {
    // a pageable announcement being withdrawn or replaced: its staging copy still reads
    // the caller's array on the helper threads — finish it before returning, so the
    // caller may free or reuse that memory once this call is back
    auto retire_announced = [&] {
      if (c->ann_ptr && c->ann_host && !c->ann_pinned) c->stager.retire(&c->st_pf[c->ann_slot]);
    };
    if (!xyzw) {  // withdraw the announcement
      retire_announced();
      c->ann_ptr = nullptr;
      return;
    }
    const auto& E = c->P.extraction;
    if (n != (size_t)E.num_rows * (size_t)E.num_columns)
      throw StatusError(FMX_E_SIZE, "Provided scan does not match the expected size " +
                                        std::to_string((size_t)E.num_rows * E.num_columns) + " != " + std::to_string(n));
    retire_announced();
    c->ann_pinned = !on_dev && host_pinned(xyzw, n * sizeof(float4));
    if (!on_dev && !c->ann_pinned) {
      // a pageable host scan: its staging copy into a pinned slot starts now, in the
      // background (the helpers copy it while the caller's next register_scan runs)
      pinned_ensure(c, n * sizeof(float4));
      const int slot = c->ann_ptr && c->ann_host && !c->ann_pinned
                           ? c->ann_slot ^ 1
                           : (c->pf_launched && c->pf_host && c->pf_slot >= 0 ? c->pf_slot ^ 1 : 0);
      // the slot's pinned bytes may still feed the DMA of a queued, not yet taken extraction
      if (c->pf_launched && c->pf_host && c->pf_slot == slot) FMX_HIP(hipStreamSynchronize(c->side2));
      stage_submit(c, c->st_pf[slot], xyzw, c->pin_pf[slot], n * sizeof(float4));
      if (c->stager.threads() == 0) stage_finish(c, c->st_pf[slot]);
      c->ann_slot = slot;
    }
    c->ann_host = !on_dev;
    c->ann_ptr = xyzw;
    c->ann_n = n;
  });
}

fmx_status fmx_scan_buffer(fmx_ctx* c, size_t n, float** out) {
  return guard<false>(c, [&] {
    if (!out || !n) throw StatusError(FMX_E_INVAL, "null output / zero points");
    auto& B = c->scanbuf[c->scanbuf_next];
    if (B.cap < n) {
      // the buffer may feed a queued DMA (a registered or announced scan): drain first
      sync_all(c);
      if (B.p) {
        // an announcement or a queued extraction of a scan in this buffer would otherwise
        // outlive it (a new buffer may even come back at the same address)
        const float* b0 = reinterpret_cast<const float*>(B.p);
        const float* b1 = reinterpret_cast<const float*>(B.p + B.cap);
        if (c->ann_ptr >= b0 && c->ann_ptr < b1) c->ann_ptr = nullptr;
        if (c->pf_launched && c->pf_ptr >= b0 && c->pf_ptr < b1) pf_drop(c);
      }
      if (B.p) (void)hipHostFree(B.p);
      B.p = nullptr;
      B.cap = 0;
      FMX_HIP(hipHostMalloc(reinterpret_cast<void**>(&B.p), n * sizeof(float4), hipHostMallocDefault));
      B.cap = n;
    }
    c->scanbuf_next = (c->scanbuf_next + 1) % 3;
    *out = reinterpret_cast<float*>(B.p);
  });
}

fmx_status fmx_register_scan(fmx_ctx* c, const float* xyzw, size_t n, int on_dev, fmx_feature_counts* out) {
  return guard<false>(c, [&] {
    drop_match(c);
    register_scan(c, xyzw, n, on_dev, out);
  });
}

fmx_status fmx_current_pose(fmx_ctx* c, double pose[12]) {
  return guard<false>(c, [&] {
    if (!c->est || !c->est->init) {
      const Pose I = identity();
      std::memcpy(pose, I.m, sizeof(I.m));
      return;
    }
    std::memcpy(pose, c->est->values.at(c->est->scan).m, 12 * sizeof(double));
  });
}

fmx_status fmx_map_download(fmx_ctx* c, double voxel_width, double* planar, uint64_t* planar_scan,
                            uint32_t* n_planar, double* point, uint64_t* point_scan, uint32_t* n_point) {
  return guard(c, [&] {
    if (!c->est || !c->est->init) throw StatusError(FMX_E_STATE, "no registered scan (fmx_register_scan)");
    if (!(voxel_width > 0)) throw StatusError(FMX_E_INVAL, "voxel width must be > 0");
    if (!n_planar || !n_point) throw StatusError(FMX_E_INVAL, "null count pointers");
    finish_tail(c);  // the reference's register_scan ends with marginalization + KeypointMap::remove
    fmx_ctx::Est& e = *c->est;
    // m_keypoint_map's scans, each at its current estimate (map.tpp:135-137)
    std::set<uint64_t> sset;
    for (int t = 0; t < 2; ++t)
      for (auto& [s, r] : c->pool[t].ranges) sset.insert(s);
    std::vector<uint64_t> scans(sset.begin(), sset.end());
    std::vector<double> poses(12 * scans.size());
    for (size_t k = 0; k < scans.size(); ++k) {
      auto it = e.values.find(scans[k]);
      if (it == e.values.end()) throw StatusError(FMX_E_STATE, "keypoints of a scan without an estimate");
      std::memcpy(&poses[12 * k], it->second.m, 12 * sizeof(double));
    }
    uint32_t cnt[2] = {0, 0};
    for (int t = 0; t < 2; ++t)
      for (uint64_t s : scans) {
        auto it = c->pool[t].ranges.find(s);
        if (it != c->pool[t].ranges.end()) cnt[t] += it->second.second;
      }
    double* outs[2] = {planar, point};
    uint64_t* sids[2] = {planar_scan, point_scan};
    uint32_t* ns[2] = {n_planar, n_point};
    for (int t = 0; t < 2; ++t) {
      if (!outs[t] && !sids[t]) {
        *ns[t] = cnt[t];
        continue;
      }
      if (*ns[t] < cnt[t]) throw StatusError(FMX_E_SIZE, "map_download: buffer smaller than the map");
      std::vector<double> xyz, nrm;
      std::vector<uint64_t> sid;
      const uint32_t m = map_snapshot(c, t, scans, poses, voxel_width, xyz, nrm, sid);
      const int stride = t == 0 ? 6 : 3;
      for (uint32_t r = 0; r < m; ++r) {
        if (outs[t]) {
          std::memcpy(outs[t] + (size_t)stride * r, &xyz[3 * (size_t)r], 3 * sizeof(double));
          if (t == 0) std::memcpy(outs[t] + (size_t)stride * r + 3, &nrm[3 * (size_t)r], 3 * sizeof(double));
        }
        if (sids[t]) sids[t][r] = sid[r];
      }
      *ns[t] = m;
    }
  });
}

fmx_status fmx_last_stats(fmx_ctx* c, uint64_t* stats, int n) {
  return guard<false>(c, [&] {
    if (!stats || n < 0) throw StatusError(FMX_E_INVAL, "null stats");
    for (int k = 0; k < n; ++k) stats[k] = k < kStatsN ? c->stats[k] : 0;
  });
}

fmx_status fmx_match_work(fmx_ctx* c, double work[3]) {
  return guard<false>(c, [&] {  // the last launched match (a fused one counts too)
    match_counts_fetch(c);
    work[0] = (double)c->n_qpl + (double)c->n_qpt;
    work[1] = c->last_probes;
    work[2] = c->last_cands;
  });
}

fmx_status fmx_match_cert(fmx_ctx* c, uint64_t counts[2], uint8_t* certified) {
  return guard(c, [&] {
    if (!c->have_match) throw StatusError(FMX_E_STATE, "no match results");
    match_counts_fetch(c);
    if (counts) {
      counts[0] = c->cert_tot[0];
      counts[1] = c->cert_tot[1];
    }
    if (certified) {
      const uint32_t nq = c->n_qpl + c->n_qpt;
      std::vector<uint8_t> f(nq);
      if (nq) FMX_HIP(hipMemcpy(f.data(), c->m_ins.p, nq, hipMemcpyDeviceToHost));
      for (uint32_t q = 0; q < nq; ++q) certified[q] = (f[q] >> 1) & 1;
    }
  });
}

fmx_status fmx_profile_match_work(fmx_ctx* c, double out[12]) {
  return guard<false>(c, [&] {
    if (!out) throw StatusError(FMX_E_INVAL, "null output");
    prof_collect(c);
    for (int k = 0; k < 2; ++k)
      for (int i = 0; i < 6; ++i) out[6 * k + i] = c->prof.mwork[k][i];
  });
}

fmx_status fmx_corr_generation(fmx_ctx* c, uint64_t* gen) {
  return guard<false>(c, [&] {
    if (!gen) throw StatusError(FMX_E_INVAL, "null output");
    *gen = c->corr_gen;
  });
}

fmx_status fmx_profile_enable(fmx_ctx* c, int on) {
  return guard<false>(c, [&] { c->prof.on = on != 0; });
}
fmx_status fmx_profile_reset(fmx_ctx* c) {
  return guard<false>(c, [&] {
    prof_collect(c);
    for (int i = 0; i < PROF_COUNT; ++i) {
      c->prof.ms[i] = 0;
      c->prof.launches[i] = 0;
      c->prof.bytes[i] = 0;
    }
    std::memset(c->prof.mwork, 0, sizeof(c->prof.mwork));
  });
}
int fmx_profile_count(void) { return PROF_COUNT; }
const char* fmx_profile_name(int k) { return (k >= 0 && k < PROF_COUNT) ? kProfNames[k] : ""; }
fmx_status fmx_profile_read(fmx_ctx* c, double* ms, uint64_t* launches, double* bytes, int n) {
  return guard<false>(c, [&] {
    prof_collect(c);
    for (int i = 0; i < std::min(n, (int)PROF_COUNT); ++i) {
      if (ms) ms[i] = c->prof.ms[i];
      if (launches) launches[i] = c->prof.launches[i];
      if (bytes) bytes[i] = c->prof.bytes[i];
    }
  });
}
fmx_status fmx_sync(fmx_ctx* c) {
  return guard<false>(c, [&] { sync_all(c); });
}

}  // extern "C"
