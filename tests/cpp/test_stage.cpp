// test_stage.cpp — the host staging of pageable scans (form_amd/csrc/stage.hpp) on the
// CPU: requests copied by helper threads and the caller together, plain and packed
// (float4 -> x, y, z), several requests in flight, reuse after retire, helpers stopped
// and restarted.  Built twice by tests/cpp/Makefile: plain and with
// -fsanitize=thread (data races between the helpers, the caller and retire/reset).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <random>
#include <vector>

#include "stage.hpp"

static int g_fail = 0;
#define CHECK(c)                                                 \
  do {                                                           \
    if (!(c)) {                                                  \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                  \
    }                                                            \
  } while (0)

// the helpers' CPUs are within the process's load-time CPUs (taskset /
// FMX_STAGE_CPUS), never the creator's own, and a one-CPU process keeps its mask.
static int check_helper_cpus() {
  int bad = 0;
  for (int cpu = 0; cpu < CPU_SETSIZE; ++cpu) {
    if (!CPU_ISSET(cpu, &fmx::g_load_cpus)) continue;
    cpu_set_t m;
    const bool set = fmx::helper_cpus(cpu, m);
    if (!set) {
      bad += CPU_COUNT(&fmx::g_load_cpus) > 1;  // only a single-CPU process may keep the inherited mask
      continue;
    }
    if (CPU_ISSET(cpu, &m)) ++bad;
    cpu_set_t x;
    CPU_AND(&x, &m, &fmx::g_load_cpus);
    if (!CPU_EQUAL(&x, &m)) ++bad;
  }
  return bad;
}

// Round 5: a process whose loading thread is pinned to one CPU (bench.py pins its
// registering thread before the library loads) still has its other threads on the
// launch mask; the helpers' mask is their union, not the pinned CPU alone.
static int check_pinned_loader() {
  cpu_set_t all;
  CPU_ZERO(&all);
  if (sched_getaffinity(0, sizeof(all), &all) != 0 || CPU_COUNT(&all) < 2) return 0;  // nothing to check
  std::atomic<bool> go{false};
  std::thread other([&] {  // keeps the launch mask
    while (!go.load()) std::this_thread::yield();
  });
  int first = 0;
  while (!CPU_ISSET(first, &all)) ++first;
  cpu_set_t one;
  CPU_ZERO(&one);
  CPU_SET(first, &one);
  sched_setaffinity(0, sizeof(one), &one);
  const cpu_set_t got = fmx::capture_load_cpus();
  sched_setaffinity(0, sizeof(all), &all);
  go = true;
  other.join();
  cpu_set_t x;
  CPU_AND(&x, &got, &all);
  return CPU_EQUAL(&x, &all) ? 0 : 1;
}

int main() {
  if (check_helper_cpus()) {
    std::printf("helper CPUs outside the load-time mask\n");
    return 1;
  }
  if (!std::getenv("FMX_STAGE_CPUS") && check_pinned_loader()) {
    std::printf("a pinned loading thread narrowed the helpers' mask to its CPU\n");
    return 1;
  }
  std::mt19937 g(7);
  fmx::Stager st;
  fmx::StageReq r[3];
  for (int round = 0; round < 40; ++round) {
    const int threads = round % 4;  // 0: the caller copies alone
    if (round % 10 == 0) st.stop();
    st.start(threads);
    const size_t npts = 1000 + (g() % 70000);
    std::vector<std::vector<float>> src(3, std::vector<float>(4 * npts));
    std::vector<std::vector<float>> dst(3, std::vector<float>(4 * npts, -1.0f));
    for (int k = 0; k < 3; ++k)
      for (auto& v : src[k]) v = (float)(g() % 100000) * 0.01f;
    for (int k = 0; k < 3; ++k) {
      st.retire(&r[k]);
      r[k].reset(src[k].data(), dst[k].data(), npts * 16, 4096 * (1 + k + round % 5), (round + k) % 2 == 1);
      if (st.threads() > 0) st.submit(&r[k]);
    }
    for (int k = 0; k < 3; ++k) {  // the caller helps, then waits, as stage_finish does
      while (r[k].work_one()) {
      }
      while (!r[k].complete()) {
      }
      st.retire(&r[k]);
      for (uint32_t c = 0; c < r[k].nchunks; ++c) CHECK(r[k].chunk_done(c));
      if (!r[k].pack3) {
        CHECK(std::memcmp(src[k].data(), dst[k].data(), npts * 16) == 0);
      } else {
        bool ok = true;
        for (size_t p = 0; p < npts && ok; ++p)
          for (int d = 0; d < 3; ++d) ok &= dst[k][3 * p + d] == src[k][4 * p + d];
        CHECK(ok);
        CHECK(dst[k][3 * npts] == -1.0f);  // nothing past the packed bytes
      }
    }
  }
  st.stop();
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  std::printf("stage ok\n");
  return 0;
}
