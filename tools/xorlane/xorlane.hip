// GPU self-check of fmx::xor_lane<LJ> (fmx_device.hpp) against lane ^ LJ, 32- and
// 64-bit.  Build: hipcc -O3 --offload-arch=gfx950 -I../../include -I../../form_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include "fmx_device.hpp"

template <int LJ>
__global__ void k(uint32_t* bad) {
  const uint32_t l = __lane_id();
  const uint32_t x = 1000u + l;
  const uint64_t y = ((uint64_t)(7000u + l) << 32) | (3000u + l);
  const uint32_t gx = fmx::xor_lane<LJ>(x);
  const uint64_t gy = fmx::xor_lane<LJ>(y);
  const uint32_t p = l ^ LJ;
  if (gx != 1000u + p || gy != (((uint64_t)(7000u + p) << 32) | (3000u + p))) atomicAdd(bad, 1u);
}

int main() {
  uint32_t* d;
  if (hipMalloc(&d, 4) != hipSuccess) return 2;
  int fails = 0;
  auto run = [&](auto kern, int lj) {
    uint32_t z = 0;
    (void)hipMemcpy(d, &z, 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kern, dim3(4), dim3(256), 0, 0, d);
    (void)hipMemcpy(&z, d, 4, hipMemcpyDeviceToHost);
    printf("xor_lane<%d>: %s (%u bad lanes)\n", lj, z ? "FAIL" : "ok", z);
    fails += z != 0;
  };
  run(k<1>, 1); run(k<2>, 2); run(k<4>, 4); run(k<8>, 8); run(k<16>, 16); run(k<32>, 32);
  (void)hipFree(d);
  return fails ? 1 : 0;
}
