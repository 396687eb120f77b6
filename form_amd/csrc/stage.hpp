// stage.hpp — host-side staging of caller-owned (pageable) scans into pinned memory.
//
// The reference's boundary takes the scan as a host std::vector<PointXYZf>
// (form/form.hpp:82-83, filled per measurement by FORM::add_lidar,
// python/bindings.cpp:150-159).  A DMA to the device needs page-locked memory, so a
// host scan is first copied into a context-owned pinned buffer.  That copy (4 MiB per
// 128 x 2048 scan) is CPU work: it is split into chunks that a few helper threads and
// the calling thread copy in parallel, and the caller issues the DMA of each completed
// prefix right away (sequential registration), or it runs entirely in the background
// while the previous scan registers (an announced next scan, fmx_next_scan).
#pragma once
#include <dirent.h>
#include <immintrin.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace fmx {

// The CPUs the process may use — the union of its threads' affinity masks when the
// library is loaded (a caller that pinned its registering thread before loading it,
// as bench.py does, still has threads on the launch mask: taskset / numactl / a rank
// binding) — narrowed by FMX_STAGE_CPUS ("0-3,8,10-11") when set.  The staging helpers
// run only on these.  (Round 5: the loading thread's own mask alone was the pinned CPU,
// so every helper ran on the registering thread's CPU: pageable host input 0.98 -> 0.83
// of the device-resident rate.)
inline cpu_set_t capture_load_cpus() {
  cpu_set_t m;
  CPU_ZERO(&m);
  if (sched_getaffinity(0, sizeof(m), &m) != 0) {
    for (int i = 0; i < CPU_SETSIZE; ++i) CPU_SET(i, &m);
  }
  if (DIR* d = opendir("/proc/self/task")) {
    while (const dirent* e = readdir(d)) {
      const int tid = std::atoi(e->d_name);
      cpu_set_t t;
      CPU_ZERO(&t);
      if (tid > 0 && sched_getaffinity(tid, sizeof(t), &t) == 0) CPU_OR(&m, &m, &t);
    }
    closedir(d);
  }
  if (const char* e = std::getenv("FMX_STAGE_CPUS")) {
    cpu_set_t o;
    CPU_ZERO(&o);
    const std::string s(e);
    size_t p = 0;
    while (p < s.size()) {
      const size_t q = s.find(',', p);
      const std::string part = s.substr(p, q == std::string::npos ? std::string::npos : q - p);
      const size_t dash = part.find('-');
      const int lo = std::atoi(part.c_str()), hi = dash == std::string::npos ? lo : std::atoi(part.c_str() + dash + 1);
      for (int c = lo; c <= hi && c < CPU_SETSIZE; ++c)
        if (c >= 0 && CPU_ISSET(c, &m)) CPU_SET(c, &o);
      if (q == std::string::npos) break;
      p = q + 1;
    }
    if (CPU_COUNT(&o) > 0) m = o;
  }
  return m;
}
inline const cpu_set_t g_load_cpus = capture_load_cpus();  // dynamic init at library load

// Where the helpers of a creator running on `creator_cpu` may run: every load-time CPU
// (g_load_cpus) but the creator's; if that leaves nothing, the inherited mask (returns
// false).
inline bool helper_cpus(int creator_cpu, cpu_set_t& out) {
  out = g_load_cpus;
  if (creator_cpu >= 0) CPU_CLR(creator_cpu, &out);
  return CPU_COUNT(&out) > 0;
}

// float4 points -> packed x, y, z.  AVX2 hosts: four points per step, each 16-B point
// shuffled down to its 12 bytes inside a 32-B register pair and stored as 48 contiguous
// bytes (two unaligned 16-B + one 16-B store), ~2x the scalar copy's throughput.
__attribute__((target("avx2"))) inline void pack_xyz_avx2(const float* s4, float* d3, size_t np) {
  size_t p = 0;
  for (; p + 4 <= np; p += 4) {
    const __m128 a = _mm_loadu_ps(s4 + 4 * p), b = _mm_loadu_ps(s4 + 4 * p + 4), c = _mm_loadu_ps(s4 + 4 * p + 8),
                 d = _mm_loadu_ps(s4 + 4 * p + 12);
    // [a0 a1 a2 b0] [b1 b2 c0 c1] [c2 d0 d1 d2]
    const __m128 o0 = _mm_blend_ps(a, _mm_shuffle_ps(b, b, 0x00), 0x8);
    const __m128 o1 = _mm_shuffle_ps(b, c, _MM_SHUFFLE(1, 0, 2, 1));
    const __m128 o2 = _mm_shuffle_ps(_mm_shuffle_ps(c, d, _MM_SHUFFLE(0, 0, 2, 2)), d, _MM_SHUFFLE(2, 1, 2, 0));
    _mm_storeu_ps(d3 + 3 * p, o0);
    _mm_storeu_ps(d3 + 3 * p + 4, o1);
    _mm_storeu_ps(d3 + 3 * p + 8, o2);
  }
  for (; p < np; ++p) {
    d3[3 * p] = s4[4 * p];
    d3[3 * p + 1] = s4[4 * p + 1];
    d3[3 * p + 2] = s4[4 * p + 2];
  }
}
inline void pack_xyz(const float* s4, float* d3, size_t np) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2) {
    pack_xyz_avx2(s4, d3, np);
    return;
  }
  for (size_t p = 0; p < np; ++p) {
    d3[3 * p] = s4[4 * p];
    d3[3 * p + 1] = s4[4 * p + 1];
    d3[3 * p + 2] = s4[4 * p + 2];
  }
}

// One staging request: bytes [0, n) of src -> dst in `chunks` pieces.  Chunks are
// claimed by any thread (helpers or the caller) and flagged when copied.  pack3: src is
// float4 points and dst receives their x, y, z only (12 of every 16 bytes: the pad of a
// PointXYZf is always 0, utils.hpp:38-46, so a quarter of the DMA is dropped); offsets
// and chunk sizes are then counted in source bytes, dst offsets are 3/4 of them.
struct StageReq {
  const uint8_t* src = nullptr;
  uint8_t* dst = nullptr;
  bool pack3 = false;
  size_t bytes = 0, chunk = 0;
  uint32_t nchunks = 0;
  std::atomic<uint32_t> next{0};  // next unclaimed chunk
  std::atomic<uint32_t> ndone{0};
  std::atomic<int> users{0};  // helper threads holding this request (retire waits for 0)
  std::unique_ptr<std::atomic<uint8_t>[]> done;
  uint32_t done_cap = 0;
  bool active = false;  // submitted, not yet waited for (owner's view)

  void reset(const void* s, void* d, size_t n, size_t ch, bool pack = false) {
    src = static_cast<const uint8_t*>(s);
    dst = static_cast<uint8_t*>(d);
    pack3 = pack;
    bytes = n;
    chunk = std::max<size_t>(ch, 4096) & ~(size_t)15;  // whole points
    nchunks = (uint32_t)((n + chunk - 1) / chunk);
    if (nchunks > done_cap) {
      done.reset(new std::atomic<uint8_t>[nchunks]);
      done_cap = nchunks;
    }
    for (uint32_t i = 0; i < nchunks; ++i) done[i].store(0, std::memory_order_relaxed);
    ndone.store(0, std::memory_order_relaxed);
    next.store(0, std::memory_order_release);
  }
  // claim and copy one chunk; false when every chunk has been claimed
  bool work_one() {
    const uint32_t i = next.fetch_add(1, std::memory_order_acq_rel);
    if (i >= nchunks) return false;
    const size_t off = (size_t)i * chunk, len = std::min(chunk, bytes - off);
    if (!pack3) {
      std::memcpy(dst + off, src + off, len);
    } else {
      pack_xyz(reinterpret_cast<const float*>(src + off), reinterpret_cast<float*>(dst + off / 16 * 12), len / 16);
    }
    done[i].store(1, std::memory_order_release);
    ndone.fetch_add(1, std::memory_order_acq_rel);
    return true;
  }
  bool chunk_done(uint32_t i) const { return done[i].load(std::memory_order_acquire) != 0; }
  bool complete() const { return ndone.load(std::memory_order_acquire) == nchunks; }
  bool unclaimed() const { return next.load(std::memory_order_acquire) < nchunks; }
};

// Helper threads that copy the chunks of submitted requests.  They are not pinned to
// the CPU of the thread that creates them (a registering thread is often pinned to one
// CPU; threads inherit that mask): each helper runs on the CPUs the process was given at
// load time (taskset / numactl / a per-rank binding, FMX_STAGE_CPUS) that share the
// never the creator's own (helper_cpus).
class Stager {
 public:
  ~Stager() { stop(); }
  void start(int nthreads) {
    if (!th_.empty() || nthreads <= 0) return;
    const int creator_cpu = sched_getcpu();
    quit_ = false;
    for (int t = 0; t < nthreads; ++t) th_.emplace_back([this, creator_cpu] { loop(creator_cpu); });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
    th_.clear();
    reqs_.clear();
  }
  int threads() const { return (int)th_.size(); }
  void submit(StageReq* r) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      reqs_.push_back(r);
    }
    r->active = true;
    cv_.notify_all();
  }
  // the request's chunks are all copied: forget it (its buffers may be reused)
  void retire(StageReq* r) {
    if (!r->active) return;
    while (!r->complete()) {
      if (!r->work_one()) std::this_thread::yield();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      reqs_.erase(std::remove(reqs_.begin(), reqs_.end(), r), reqs_.end());
    }
    // no helper picks it up any more; wait for the ones still inside work_one's claim
    while (r->users.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    r->active = false;
  }

 private:
  void loop(int creator_cpu) {
    cpu_set_t m;
    if (helper_cpus(creator_cpu, m)) (void)sched_setaffinity(0, sizeof(m), &m);
    for (;;) {
      StageReq* r = nullptr;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] {
          if (quit_) return true;
          for (StageReq* q : reqs_)
            if (q->unclaimed()) return true;
          return false;
        });
        if (quit_) return;
        for (StageReq* q : reqs_)
          if (q->unclaimed()) {
            r = q;
            r->users.fetch_add(1, std::memory_order_acq_rel);
            break;
          }
      }
      if (!r) continue;
      while (r->work_one()) {
      }
      r->users.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  std::vector<std::thread> th_;
  std::vector<StageReq*> reqs_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool quit_ = false;
};

}  // namespace fmx
