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
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace fmx {

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
      const float* s4 = reinterpret_cast<const float*>(src + off);
      float* d3 = reinterpret_cast<float*>(dst + off / 16 * 12);
      const size_t np = len / 16;
      for (size_t p = 0; p < np; ++p) {
        d3[3 * p] = s4[4 * p];
        d3[3 * p + 1] = s4[4 * p + 1];
        d3[3 * p + 2] = s4[4 * p + 2];
      }
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
// CPU; threads inherit that mask): each helper widens its mask to every CPU the cpuset
// allows except the creator's.
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
    cpu_set_t all;
    CPU_ZERO(&all);
    for (int i = 0; i < CPU_SETSIZE; ++i) CPU_SET(i, &all);
    (void)sched_setaffinity(0, sizeof(all), &all);  // the kernel keeps the cpuset's CPUs
    cpu_set_t eff;
    if (creator_cpu >= 0 && sched_getaffinity(0, sizeof(eff), &eff) == 0 && CPU_COUNT(&eff) > 1) {
      CPU_CLR(creator_cpu, &eff);
      (void)sched_setaffinity(0, sizeof(eff), &eff);
    }
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
