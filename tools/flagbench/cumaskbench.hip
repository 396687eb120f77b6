// Where a CU-masked stream's workgroups run on MI355X (hipExtStreamCreateWithCUMask):
// for a few mask patterns over the 256 CU bits, each workgroup records its XCC_ID and
// HW_ID (s_getreg); the host counts the XCDs and (XCD, SE, CU) slots used.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void k_where(uint32_t* out) {
  if (threadIdx.x == 0) {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    // linger so that later workgroups spread over more CUs
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) {}
  }
}
int main() {
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int ncu = pr.multiProcessorCount, nw = (ncu + 31) / 32;
  printf("CUs %d\n", ncu);
  const int NB = 8192;
  uint32_t* d;
  CK(hipMalloc(&d, NB * 8));
  std::vector<uint32_t> h(2 * NB);
  struct M { const char* name; std::vector<uint32_t> m; };
  std::vector<M> ms;
  auto mk = [&](const char* n, auto f) { std::vector<uint32_t> m(nw, 0); for (int i = 0; i < ncu; ++i) if (f(i)) m[i / 32] |= 1u << (i % 32); ms.push_back({n, m}); };
  mk("all", [](int) { return true; });
  mk("top 64 (i >= 192)", [&](int i) { return i >= ncu - 64; });
  mk("first 64 (i < 64)", [](int i) { return i < 64; });
  mk("every 4th (i % 4 == 0)", [](int i) { return i % 4 == 0; });
  mk("i % 32 < 8", [](int i) { return i % 32 < 8; });
  mk("i % 8 == 0", [](int i) { return i % 8 == 0; });
  mk("first 32 (i < 32)", [](int i) { return i < 32; });
  for (auto& m : ms) {
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.m.size(), m.m.data()));
    hipLaunchKernelGGL(k_where, dim3(NB), dim3(64), 0, s, d);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h.data(), d, NB * 8, hipMemcpyDeviceToHost));
    std::set<uint32_t> xccs;
    std::set<uint64_t> slots;
    int per_xcc[8] = {0};
    std::set<uint64_t> cu_xcc[8];
    for (int b = 0; b < NB; ++b) {
      const uint32_t hw = h[2 * b], x = h[2 * b + 1] & 0xF;
      xccs.insert(x);
      const uint32_t cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      const uint64_t key = ((uint64_t)x << 16) | (se << 8) | (sh << 4) | cu;
      slots.insert(key);
      if (x < 8) { ++per_xcc[x]; cu_xcc[x].insert(key); }
    }
    printf("%-24s xcds %zu, distinct (xcd,se,sh,cu) %zu | CUs per XCD:", m.name, xccs.size(), slots.size());
    for (int x = 0; x < 8; ++x) printf(" %zu", cu_xcc[x].size());
    printf("\n");
    CK(hipStreamDestroy(s));
  }
  return 0;
}
