// fmx_device.hpp — device helpers shared by the fmx HIP kernels (gfx950, wave64).
//
// Rounding contract: every .hip file is compiled with -ffp-contract=off, so the
// float/double expressions below round exactly like the reference's SSE2 Eigen
// code (CMakeLists.txt sets no -march; no FMA):
//   PointXYZf::squaredNorm / (a - b).squaredNorm() on vec4 with zero pad
//     -> (dx*dx + dz*dz) + dy*dy          (Packet4f predux: (a0+a2)+(a1+a3))
//   Matrix3d * Vector3d -> ((R0 v0 + R1 v1) + R2 v2) per row.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fmx {

constexpr int kWave = 64;

// ---------------------------------------------------------------- poses
struct Pose34 {  // row-major [R | t]
  double m[12];
};

__device__ __forceinline__ void d_xform(const double* T, double x, double y, double z, double o[3]) {
  o[0] = ((T[0] * x + T[1] * y) + T[2] * z) + T[3];
  o[1] = ((T[4] * x + T[5] * y) + T[6] * z) + T[7];
  o[2] = ((T[8] * x + T[9] * y) + T[10] * z) + T[11];
}
__device__ __forceinline__ void d_rot(const double* T, double x, double y, double z, double o[3]) {
  o[0] = (T[0] * x + T[1] * y) + T[2] * z;
  o[1] = (T[4] * x + T[5] * y) + T[6] * z;
  o[2] = (T[8] * x + T[9] * y) + T[10] * z;
}
// R^T v
__device__ __forceinline__ void d_rotT(const double* T, double x, double y, double z, double o[3]) {
  o[0] = (T[0] * x + T[4] * y) + T[8] * z;
  o[1] = (T[1] * x + T[5] * y) + T[9] * z;
  o[2] = (T[2] * x + T[6] * y) + T[10] * z;
}

__device__ __forceinline__ float sqnorm4f(float x, float y, float z) { return (x * x + z * z) + y * y; }
__device__ __forceinline__ float dist2f(float4 a, float4 b) {
  const float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
  return (dx * dx + dz * dz) + dy * dy;
}

// ---------------------------------------------------------------- wave ops
__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}
template <class T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T u = __shfl_up(v, o, 64);
    if (l >= o) v += u;
  }
  return v;
}
// Value of lane (lane ^ LJ) without the LDS crossbar (ds_bpermute): DPP quad
// permutes for 1 and 2, row shifts + select for 4, a row rotate for 8, the gfx950
// permlane16/32 swaps + select for 16 and 32.  VALU only.
template <int LJ>
__device__ __forceinline__ uint32_t xor_lane(uint32_t x) {
  static_assert(LJ == 1 || LJ == 2 || LJ == 4 || LJ == 8 || LJ == 16 || LJ == 32, "xor distance");
  if constexpr (LJ == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
  if constexpr (LJ == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);
  if constexpr (LJ == 4) {
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xF, 0xF, false);  // row_shl:4 (l <- l+4)
    const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4 (l <- l-4)
    return (__lane_id() & 4) ? dn : up;
  }
  if constexpr (LJ == 8) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false);  // row_ror:8
  if constexpr (LJ == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (__lane_id() & 16) ? r[0] : r[1];
  }
  if constexpr (LJ == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (__lane_id() & 32) ? r[0] : r[1];
  }
  return x;
}
template <int LJ>
__device__ __forceinline__ uint64_t xor_lane(uint64_t v) {
  return ((uint64_t)xor_lane<LJ>((uint32_t)(v >> 32)) << 32) | xor_lane<LJ>((uint32_t)v);
}

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- host completion word
// Results the host polls for go to pinned host memory with SYSTEM-scope stores
// (host_store: sc0 sc1, written through, never left dirty in the GPU L2); the wave
// that made them drains (vmcnt 0) and then stores the completion word the same way
// (publish_flag; host side: wait_flag in fmx_internal.hpp).  MI355X_MICROARCH.md
// lists this write-through form as valid without a release fence; a system release
// (buffer_wbl2) would write back every dirty L2 line of the XCD instead.  Plain
// stores to host memory CAN sit in L2: with plain payload stores and no fence the
// host once read stale totals behind a fresh word.  Call publish_flag from ONE lane
// of the wave that made every host_store it covers — or, when several waves / blocks
// made them (k_win_linearize's pair finishers), after each of those waves waited for
// its own write-through stores (vmcnt(0): acknowledged = left the GPU caches) BEFORE
// the barrier / agent-scope ticket that orders it ahead of the publishing wave.
__device__ __forceinline__ void host_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void host_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void host_store(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void publish_flag(uint32_t* flag, uint32_t seq) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------- device-wide scan
// Exclusive scan of n uint32 values produced by in(i) into out(i, v); *total = sum.
// Three launches (tile reduce, block-sum scan, tile scan): deterministic.
constexpr int kScanThreads = 1024;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanThreads * kScanItems;

template <class In>
__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(In in, size_t n, uint32_t* bsum) {
  __shared__ uint32_t ws[kScanThreads / kWave];
  const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j)
    if (base + j < n) s += in(base + j);
  s = wave_sum(s);
  if (lane_id() == 0) ws[threadIdx.x / kWave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kScanThreads / kWave; ++w) t += ws[w];
    bsum[blockIdx.x] = t;
  }
}

// single block: exclusive scan of nb block sums in place; *total = sum
template <int Dummy = 0>
__global__ __launch_bounds__(kScanThreads) void k_scan_blocks(uint32_t* bsum, uint32_t nb, uint32_t* total) {
  __shared__ uint32_t ws[kScanThreads / kWave];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nb; b0 += kScanThreads) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t v = i < nb ? bsum[i] : 0u;
    const uint32_t incl = wave_incl_scan(v);
    const int w = threadIdx.x / kWave;
    if (lane_id() == 63) ws[w] = incl;
    __syncthreads();
    uint32_t woff = 0, tot = 0;
    for (int k = 0; k < kScanThreads / kWave; ++k) {
      if (k < w) woff += ws[k];
      tot += ws[k];
    }
    const uint32_t c = carry;
    if (i < nb) bsum[i] = c + woff + incl - v;
    __syncthreads();
    if (threadIdx.x == 0) carry = c + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

template <class In, class Out>
__global__ __launch_bounds__(kScanThreads) void k_scan_tiles(In in, Out out, size_t n, const uint32_t* bsum) {
  __shared__ uint32_t ws[kScanThreads / kWave];
  const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    v[j] = base + j < n ? in(base + j) : 0u;
    s += v[j];
  }
  const uint32_t incl = wave_incl_scan(s);
  const int w = threadIdx.x / kWave;
  if (lane_id() == 63) ws[w] = incl;
  __syncthreads();
  uint32_t woff = 0;
  for (int i = 0; i < w; ++i) woff += ws[i];
  uint32_t run = bsum[blockIdx.x] + woff + incl - s;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    if (base + j < n) out(base + j, run);
    run += v[j];
  }
}

// One workgroup scans the whole array tile by tile (coalesced, carry in LDS): one
// launch instead of three, for arrays up to kScanSingleMax.
constexpr size_t kScanSingleMax = (size_t)kScanTile * 4;
template <class In, class Out>
__global__ __launch_bounds__(kScanThreads) void k_scan_single(In in, Out out, size_t n, uint32_t* total) {
  __shared__ uint32_t ws[kScanThreads / kWave];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int w = threadIdx.x / kWave;
  for (size_t t0 = 0; t0 < n; t0 += kScanTile) {
    const size_t base = t0 + (size_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
      v[j] = base + j < n ? in(base + j) : 0u;
      s += v[j];
    }
    const uint32_t incl = wave_incl_scan(s);
    if (lane_id() == 63) ws[w] = incl;
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int i = 0; i < kScanThreads / kWave; ++i) {
      if (i < w) off += ws[i];
      tot += ws[i];
    }
    uint32_t run = carry + off + incl - s;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
      if (base + j < n) out(base + j, run);
      run += v[j];
    }
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

template <class In, class Out>
inline void exclusive_scan(In in, Out out, size_t n, uint32_t* scratch /* >= nb */, uint32_t* total,
                           hipStream_t st) {
  const uint32_t nb = (uint32_t)((n + kScanTile - 1) / kScanTile);
  if (nb == 0) {
    (void)hipMemsetAsync(total, 0, sizeof(uint32_t), st);
    return;
  }
  if (n <= kScanSingleMax) {
    k_scan_single<In, Out><<<1, kScanThreads, 0, st>>>(in, out, n, total);
    return;
  }
  k_scan_reduce<In><<<nb, kScanThreads, 0, st>>>(in, n, scratch);
  k_scan_blocks<0><<<1, kScanThreads, 0, st>>>(scratch, nb, total);
  k_scan_tiles<In, Out><<<nb, kScanThreads, 0, st>>>(in, out, n, scratch);
}
inline size_t scan_scratch_size(size_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

// ---------------------------------------------------------------- voxel keys
// Brick key: the brick coordinates (cell >> 1), 19 bits each with an offset of 2^18,
// under a 6-bit build epoch in bits 57-62.  A bucket whose key carries another epoch
// (0 included: never written) is empty for the current build, so a rebuild needs no
// table clear: the epoch advances instead (the host clears the table once every 63
// builds, when the epoch wraps).  Valid cell coordinates: |c| < 2^19 - 2.
constexpr int kKeyBias = 1 << 18;
constexpr int kEpochShift = 57;
constexpr uint32_t kEpochMax = 63;
__device__ __forceinline__ uint64_t pack_key(int x, int y, int z) {
  return ((uint64_t)(uint32_t)(x + kKeyBias) << 38) | ((uint64_t)(uint32_t)(y + kKeyBias) << 19) |
         (uint64_t)(uint32_t)(z + kKeyBias);
}
__device__ __forceinline__ bool key_in_range(int x, int y, int z) {
  const int L = 2 * kKeyBias - 2;
  return x > -L && x < L && y > -L && y < L && z > -L && z < L;
}
__device__ __forceinline__ uint32_t key_epoch(uint64_t k) { return (uint32_t)(k >> kEpochShift); }
__device__ __forceinline__ uint64_t mix64(uint64_t k) {  // splitmix64 finalizer
  k ^= k >> 30;
  k *= 0xbf58476d1ce4e5b9ull;
  k ^= k >> 27;
  k *= 0x94d049bb133111ebull;
  k ^= k >> 31;
  return k;
}

// Brick: the 2 x 2 x 2 cells (x, y, z) >> 1 of one 64-B bucket — the 27-cell
// neighbourhood of any cell lies in at most 8 bricks, and neighbouring queries share
// them.  Records of cell c (c = (x & 1) | (y & 1) << 1 | (z & 1) << 2) are
// [beg[c], beg[c + 1]); bit c of `dense` marks a cell stored with a sub-cell header
// (voxelmap.hip, dense cells).
struct alignas(64) Brick {
  unsigned long long key;  // epoch | pack_key of the brick coordinates (bit 63: claim in progress)
  uint32_t beg[9];
  uint32_t dense;
  uint32_t slot;  // build only: the brick's slot in the build's claim list (cell counts, then begins)
  uint32_t pad[3];
};
static_assert(sizeof(Brick) == 64, "brick = 64 B");
__device__ __forceinline__ uint64_t brick_key(int x, int y, int z, uint32_t epoch) {
  return ((uint64_t)epoch << kEpochShift) | pack_key(x >> 1, y >> 1, z >> 1);
}
__device__ __forceinline__ uint32_t brick_cell(int x, int y, int z) {
  return (uint32_t)((x & 1) | ((y & 1) << 1) | ((z & 1) << 2));
}

}  // namespace fmx
