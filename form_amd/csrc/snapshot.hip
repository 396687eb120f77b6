// snapshot.hip — the window's keypoints in the world frame, for FORM::map()
// (python/bindings.cpp:96-119): KeypointMap::to_voxel_map of both feature types at the
// current estimates (map.tpp:128-146), voxel width = the caller's (the binding passes
// min_dist_map, bindings.cpp:100).  Visualization only, off the registration path:
// one lane per stored keypoint transforms it with its scan's pose (the same double
// expression order as the map build, PlanarFeat::transform, features.hpp:137-140),
// computes its voxel (computeCoords, map.tpp:35-38), and the host groups the records
// by voxel.  Voxel order is unspecified, as the reference's robin_map iteration; inside
// a voxel records keep push_back order (scans ascending, then keypoint order).
#include "fmx_device.hpp"
#include "fmx_internal.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

namespace fmx {
namespace {

struct SnapSeg {
  uint32_t off;       // first output record
  uint32_t n;         // records
  uint32_t pool_off;  // offset in the pool
  uint32_t pad;
};

__global__ __launch_bounds__(256) void k_map_world(const float4* __restrict__ pos, const float4* __restrict__ nrm,
                                                   const SnapSeg* __restrict__ segs, int K,
                                                   const double* __restrict__ poses, uint32_t n, double w,
                                                   double* __restrict__ out_p, double* __restrict__ out_n,
                                                   int* __restrict__ out_cell) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  int lo = 0, hi = K - 1;  // last segment with off <= r
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].off <= r) lo = mid; else hi = mid - 1;
  }
  const SnapSeg sg = segs[lo];
  const double* T = poses + 12 * lo;
  const float4 lp = pos[sg.pool_off + (r - sg.off)];
  double p[3];
  d_xform(T, (double)lp.x, (double)lp.y, (double)lp.z, p);
  out_p[3 * (size_t)r] = p[0];
  out_p[3 * (size_t)r + 1] = p[1];
  out_p[3 * (size_t)r + 2] = p[2];
  if (out_n) {
    const float4 ln = nrm[sg.pool_off + (r - sg.off)];
    double q[3];
    d_rot(T, (double)ln.x, (double)ln.y, (double)ln.z, q);
    out_n[3 * (size_t)r] = q[0];
    out_n[3 * (size_t)r + 1] = q[1];
    out_n[3 * (size_t)r + 2] = q[2];
  }
  // computeCoords: (p / w).floor() cast to int (map.tpp:35-38)
  out_cell[3 * (size_t)r] = (int)floor(p[0] / w);
  out_cell[3 * (size_t)r + 1] = (int)floor(p[1] / w);
  out_cell[3 * (size_t)r + 2] = (int)floor(p[2] / w);
}

}  // namespace

// World-frame snapshot of feature type t of the keypoint store for `scans` at `poses`
// (K x 12), grouped by voxel of width w.  xyz: 3 doubles per record, nrm (planar) 3
// more; scan ids beside them.  Returns the record count.
uint32_t map_snapshot(fmx_ctx* c, int t, const std::vector<uint64_t>& scans, const std::vector<double>& poses,
                      double w, std::vector<double>& xyz, std::vector<double>& nrm, std::vector<uint64_t>& sid) {
  Pool& pool = c->pool[t];
  const int K = (int)scans.size();
  std::vector<SnapSeg> segs;
  std::vector<double> segposes;
  uint32_t n = 0;
  for (int k = 0; k < K; ++k) {
    auto it = pool.ranges.find(scans[k]);
    if (it == pool.ranges.end() || it->second.second == 0) continue;
    segs.push_back(SnapSeg{n, it->second.second, (uint32_t)it->second.first, 0});
    segposes.insert(segposes.end(), poses.begin() + 12 * k, poses.begin() + 12 * (k + 1));
    n += it->second.second;
  }
  xyz.assign(3 * (size_t)n, 0.0);
  nrm.assign(t == 0 ? 3 * (size_t)n : 0, 0.0);
  sid.assign(n, 0);
  if (n == 0) return 0;
  const bool planar = t == 0;
  const size_t bytes_seg = segs.size() * sizeof(SnapSeg), bytes_pose = segposes.size() * sizeof(double);
  const size_t bytes_out = (size_t)n * (3 * sizeof(double) * (planar ? 2 : 1) + 3 * sizeof(int));
  char* d = nullptr;
  FMX_HIP(hipMalloc(&d, bytes_seg + bytes_pose + bytes_out));
  struct Free {
    char* p;
    ~Free() { (void)hipFree(p); }
  } fr{d};
  SnapSeg* dseg = reinterpret_cast<SnapSeg*>(d);
  double* dpose = reinterpret_cast<double*>(d + bytes_seg);
  double* dp = dpose + segposes.size();
  double* dn = planar ? dp + 3 * (size_t)n : nullptr;
  int* dcell = reinterpret_cast<int*>(dp + 3 * (size_t)n * (planar ? 2 : 1));
  hipStream_t st = c->stream;
  FMX_HIP(hipMemcpyAsync(dseg, segs.data(), bytes_seg, hipMemcpyHostToDevice, st));
  FMX_HIP(hipMemcpyAsync(dpose, segposes.data(), bytes_pose, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_map_world, dim3((n + 255) / 256), dim3(256), 0, st, pool.pos.p, planar ? pool.nrm.p : nullptr,
                     dseg, (int)segs.size(), dpose, n, w, dp, dn, dcell);
  FMX_HIP(hipGetLastError());
  std::vector<double> hp(3 * (size_t)n), hn(planar ? 3 * (size_t)n : 0);
  std::vector<int> hc(3 * (size_t)n);
  FMX_HIP(hipMemcpyAsync(hp.data(), dp, hp.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  if (planar) FMX_HIP(hipMemcpyAsync(hn.data(), dn, hn.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  FMX_HIP(hipMemcpyAsync(hc.data(), dcell, hc.size() * sizeof(int), hipMemcpyDeviceToHost, st));
  FMX_HIP(hipStreamSynchronize(st));
  // group by voxel, push_back order inside a voxel (stable)
  std::vector<uint32_t> ord(n);
  std::iota(ord.begin(), ord.end(), 0u);
  std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
    return std::lexicographical_compare(&hc[3 * (size_t)a], &hc[3 * (size_t)a + 3], &hc[3 * (size_t)b],
                                        &hc[3 * (size_t)b + 3]);
  });
  std::vector<uint64_t> rec_scan(n);
  {
    size_t s = 0;
    for (int k = 0; k < K; ++k) {
      auto it = pool.ranges.find(scans[k]);
      if (it == pool.ranges.end()) continue;
      for (uint32_t i = 0; i < it->second.second; ++i) rec_scan[s++] = scans[k];
    }
  }
  for (uint32_t o = 0; o < n; ++o) {
    const uint32_t r = ord[o];
    std::memcpy(&xyz[3 * (size_t)o], &hp[3 * (size_t)r], 3 * sizeof(double));
    if (planar) std::memcpy(&nrm[3 * (size_t)o], &hn[3 * (size_t)r], 3 * sizeof(double));
    sid[o] = rec_scan[r];
  }
  return n;
}

}  // namespace fmx
