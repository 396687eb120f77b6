/*
 * fmx.h — C-ABI of the MI355X-native scan-to-submap registration path for FORM.
 *
 * Drop-in boundary for form::Estimator's hot path (huangjuite/form).  Every entry
 * point names the reference interface it replaces (file:line under the reference's
 * form/ tree).  Plain pointers and sizes only; no exceptions cross this boundary;
 * errors are status codes + fmx_last_error().  One context = one HIP device + one
 * HIP stream; a context is NOT thread-safe (the reference's register_scan is also
 * driven from a single caller thread, bindings.cpp:147-179).
 *
 * Conventions
 *   - points: PointXYZf layout, 4 x float32 per point (x, y, z, pad), row-major
 *     organized R x C scan (form/utils.hpp:38-46; extraction.tpp:141-145).
 *   - poses: row-major 3x4 double [R | t] (gtsam::Pose3 = (R, t)).
 *   - planar features: 6 floats (x, y, z, nx, ny, nz); point features: 3 floats
 *     (form/feature/features.hpp:31-163 stores the same values as doubles).
 *   - Jacobian columns: GTSAM Pose3 tangent [w; v], right perturbation.
 *   - Augmented Hessian G: packed upper triangle, row-major, of [A b]^T [A b] with
 *     A, b whitened by 1/sigma (gtsam.hpp:67-86, 129-139).  Full mode: 13 x 13 ->
 *     91 doubles (A = [H_i H_j]); single-pose mode: 7 x 7 -> 28 doubles (A = H_j).
 */
#ifndef FMX_FMX_H_
#define FMX_FMX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FMX_ABI_VERSION 1

typedef enum fmx_status {
  FMX_OK = 0,
  FMX_E_INVAL = 1, /* bad argument */
  FMX_E_SIZE = 2,  /* scan size != rows*cols (reference throws, extraction.tpp:141-145) */
  FMX_E_OOM = 3,   /* device allocation failed or a capacity was exceeded */
  FMX_E_HIP = 4,   /* HIP runtime error */
  FMX_E_STATE = 5, /* call out of order (e.g. match before map_build) */
  FMX_E_RANGE = 6, /* voxel coordinate outside the +-2^20 packed-key range */
  FMX_E_RCCL = 7   /* RCCL missing or a collective failed (multi-GPU only) */
} fmx_status;

/* form::FeatureExtractor::Params (form/feature/extraction.hpp:59-88). */
typedef struct fmx_extract_params {
  uint32_t neighbor_points;
  uint32_t num_sectors;
  double planar_threshold;
  uint32_t planar_feats_per_sector;
  uint32_t point_feats_per_sector;
  double radius;
  uint32_t min_points;
  double min_norm_squared;
  double max_norm_squared;
  int32_t num_columns;
  int32_t num_rows;
} fmx_extract_params;

/* form::Estimator::Params (form/form.hpp:42-56) flattened, plus device capacities. */
typedef struct fmx_params {
  fmx_extract_params extraction;
  double max_dist_matching;        /* MatcherParams, matcher.hpp:32-41 */
  double new_pose_threshold;
  uint32_t max_num_rematches;
  double planar_constraint_sigma;  /* ConstraintManager::Params, constraints.hpp:54-70 */
  int32_t disable_smoothing;       /* 0 (default): window smoothing; 1: single-pose ablation */
  int64_t max_num_keyscans;        /* KeyScanner::Params, keyscanner.hpp:55-64 */
  int64_t max_steps_unused_keyscan;
  uint32_t max_num_recent_scans;
  double keyscan_match_ratio;
  double min_dist_map;             /* KeypointMapParams, map.hpp:97-100 */
  /* device capacities (not in the reference: it allocates on demand) */
  uint64_t keypoint_pool_capacity; /* records per feature type kept in the window store */
  uint32_t max_pairs;              /* scans per submap (window size bound) */
  uint32_t voxel_subdivision;      /* device map cells = voxel width / this (1 or 2; 0 = 1):
                                      same matches; 2 tests fewer candidates per query but
                                      probes more cells (slower on C4/C5) */
} fmx_params;

typedef struct fmx_ctx fmx_ctx;

typedef struct fmx_feature_counts {
  uint32_t planar; /* planar features with a normal (extraction.tpp:99-118) */
  uint32_t point;  /* point features (extraction.tpp:120-129) */
  uint32_t planar_selected; /* planar indices before normal estimation */
} fmx_feature_counts;

int fmx_abi_version(void);
void fmx_default_params(fmx_params* p);

/* Estimator(const Params&) (form/form.hpp:74-76, form.cpp:31-38). */
fmx_status fmx_create(const fmx_params* p, int device, fmx_ctx** out);
void fmx_destroy(fmx_ctx* ctx);
const char* fmx_last_error(const fmx_ctx* ctx);

/* ---------------- stage 1: FeatureExtractor::extract ----------------------
 * Replaces FeatureExtractor::extract<PointXYZf> (extraction.hpp:99-101,
 * extraction.tpp:29-132).  xyzw: rows*cols float4; src_on_device != 0 means
 * xyzw is a device pointer on the context's device, else host memory.
 * The features stay device-resident as the context's current query set.
 * Host scans (here, in fmx_register_scan and fmx_next_scan): page-locked memory (from
 * fmx_scan_buffer, hipHostMalloc, hipHostRegister) is DMA'd directly; pageable memory
 * (the reference's std::vector<PointXYZf>, form.hpp:82-83) is first copied into the
 * context's pinned staging memory by a few helper threads and the caller, each part
 * DMA'd as soon as it is copied (FMX_STAGE_THREADS, default 3 helpers).  The pad
 * component must be 0, as every reference PointXYZf's is (utils.hpp:38-46). */
fmx_status fmx_extract(fmx_ctx* ctx, const float* xyzw, size_t n_points, uint64_t scan_idx,
                       int src_on_device, fmx_feature_counts* out);
/* A context-owned page-locked buffer of n_points float4 (PointXYZf layout) that a
 * caller assembling its scans (as FORM::add_lidar does, bindings.cpp:150-159) can fill
 * directly: passed as a host scan (src_on_device = 0) it is DMA'd with no staging copy.
 * Three buffers are handed out in turn: the one returned here is returned again by the
 * third next call, so a caller may fill scan k+1 while scan k registers.  Valid until
 * fmx_destroy, or until a later call asks for more points than that buffer holds: the
 * buffer is then reallocated (after draining every queued DMA from it), and an
 * announcement of a scan in the old buffer is withdrawn. */
fmx_status fmx_scan_buffer(fmx_ctx* ctx, size_t n_points, float** out);
/* Copy the last extraction to host (any pointer may be NULL):
 * planar[6*planar], planar_index[planar] (scan point index), point[3*point],
 * point_index[point], planar_mask[rows*cols] (compute_valid_points, 0/1). */
fmx_status fmx_extract_download(fmx_ctx* ctx, float* planar, uint32_t* planar_index,
                                float* point, uint32_t* point_index, uint8_t* planar_mask);

/* Replace the current query set (the scan being registered) with caller features. */
fmx_status fmx_set_queries(fmx_ctx* ctx, uint64_t scan_idx, const float* planar, uint32_t n_planar,
                           const float* point, uint32_t n_point);

/* Device-resident variants (no host round trip): float4 arrays (x, y, z, pad) that
 * already live on the context's device; normals likewise.  Same semantics as
 * fmx_set_queries / fmx_keypoints_add. */
fmx_status fmx_set_queries_device(fmx_ctx* ctx, uint64_t scan_idx, const float* planar_pos4,
                                  const float* planar_nrm4, uint32_t n_planar, const float* point_pos4,
                                  uint32_t n_point);

/* ---------------- stage 2: KeypointMap / VoxelMap / Matcher ---------------
 * Window keypoint store: KeypointMap::get(scan).push_back / insert_matches /
 * remove (map.tpp:95-126, 148-165).  Features are in the scan's local frame. */
fmx_status fmx_keypoints_add(fmx_ctx* ctx, uint64_t scan_idx, const float* planar,
                             uint32_t n_planar, const float* point, uint32_t n_point);
fmx_status fmx_keypoints_add_device(fmx_ctx* ctx, uint64_t scan_idx, const float* planar_pos4,
                                    const float* planar_nrm4, uint32_t n_planar, const float* point_pos4,
                                    uint32_t n_point);
fmx_status fmx_keypoints_remove(fmx_ctx* ctx, uint64_t scan_idx);
/* KeypointMap::to_voxel_map for both feature types (map.tpp:128-146, form.cpp:61-65):
 * builds the device voxel hash of every stored keypoint of scans[0..n) at the given
 * world poses.  Pair k of later calls refers to scans[k]. */
fmx_status fmx_map_build(fmx_ctx* ctx, const uint64_t* scans, const double* poses34,
                         uint32_t n_scans, double voxel_width);
/* Matcher<PlanarFeat>::match<0> + Matcher<PointFeat>::match<1> (matcher.hpp:67-112):
 * nearest map keypoint of every query at pose_j (VoxelMap::find_closest,
 * map.tpp:70-91), moved back to its scan's frame, accepted if d^2 < max_dist^2 and
 * bucketed per pair on the device.  counts_planar / counts_point (may be NULL):
 * K = n_scans accepted correspondences per pair.  With both NULL the call returns
 * without waiting for the device (once the map build's range check has been read);
 * the calls that read the results wait for them.
 * Deferred match: with both NULL on a large query set (>= 128k queries, windows of
 * <= 256 scans) the match is not launched yet.  Arguments are validated by this call
 * (FMX_E_INVAL / FMX_E_STATE are returned here, never by a later call).  If the next
 * consumer is fmx_linearize_matched at the same pose, match and linearization run as
 * ONE fused launch that writes no per-query results; its 7 x 7 sums are accumulated in
 * a different order than the two-step path (equal to 1e-10 relative, not bit for bit).
 * Any other reader (fmx_match_download, fmx_map_insert, fmx_linearize, ...) launches
 * the deferred match first, so its results are those of an immediate match.  Calls
 * that discard match results (fmx_set_queries*, fmx_extract, fmx_register_scan) drop
 * a deferred match without launching it. */
fmx_status fmx_match(fmx_ctx* ctx, const double pose_j34[12], double max_dist,
                     uint32_t* counts_planar, uint32_t* counts_point);
/* Per-query match results of the last fmx_match, planar queries then point
 * queries (any pointer may be NULL): pair[q] (-1 if not accepted), d2[q]
 * (DBL_MAX when no record lies within
 * max(max_dist, min_dist_map) of the query inside its 27 voxels; with both <= the
 * voxel width the search is bounded by them, otherwise it covers all 27 voxels, so a
 * finite d2 may exceed max_dist^2 — accept/insert decisions equal the reference's), pi[3q], ni[3q] (planar only). */
fmx_status fmx_match_download(fmx_ctx* ctx, int32_t* pair, double* d2, double* pi, double* ni);
/* KeypointMap::insert_matches (map.tpp:148-165): append every query of the last
 * match whose NN distance^2 > min_dist_map^2 to the store under the query scan. */
fmx_status fmx_map_insert(fmx_ctx* ctx, double min_dist_map, uint32_t* n_inserted);

/* ---------------- stage 3: FeatureFactor + DenseFactor::linearize ---------
 * Load correspondences directly (replacing the match output), pair-major:
 * plane rows p_i, n_i, p_j (3 doubles each) and point pairs p_i, p_j.
 * PlanePoint / PointPoint buffers, factor.hpp:43-130. */
fmx_status fmx_corr_set(fmx_ctx* ctx, uint32_t K, const uint32_t* n_plane,
                        const double* plane_pi, const double* plane_ni, const double* plane_pj,
                        const uint32_t* n_point, const double* point_pi, const double* point_pj);
/* A counter that changes whenever the context's correspondences may have been replaced
 * (fmx_match, fmx_corr_set, fmx_register_scan): a caller caching fmx_linearize results per
 * set of poses (fmx_seam.hpp's FmxBatch) keys its cache on it as well. */
fmx_status fmx_corr_generation(fmx_ctx* ctx, uint64_t* gen);
/* DenseFactor::linearize of every pair's FeatureFactor (gtsam.hpp:67-86,
 * factor.cpp:142-186): poses_i / poses_j are K x 12.  G: K x 91 (single_pose=0)
 * or K x 28 (single_pose=1); err: K x 1 = 0.5*||r/sigma||^2 (may be NULL). */
fmx_status fmx_linearize(fmx_ctx* ctx, const double* poses_i34, const double* poses_j34,
                         double sigma, int single_pose, double* G, double* err);
/* Pair moments: DenseFactor::linearize "once, evaluated anywhere".  Every row's whitened
 * [H_i H_j -r] is linear in 16 per-row features taken at reference poses (plane rows:
 * r0 = n.(q0 - p_i), n x q0, n, n (x) p_j with q0 = p_j in frame i; point rows: the world
 * residual e0, p_i, p_j, 1), so a pair's 13 x 13 information at ANY poses is C Phi C^T
 * with Phi = sum over its rows of phi phi^T.  fmx_moments: Phi of every pair of the
 * context's correspondences (fmx_match / fmx_corr_set) at reference poses
 * poses_i[k], poses_j[k] (K x 12 each), on the device (one launch).  mom: K x 272 =
 * per pair the packed upper 16 x 16 of the plane rows, then of the point rows. */
fmx_status fmx_moments(fmx_ctx* ctx, const double* ref_i34, const double* ref_j34, double* mom);
/* Host only (no context, no device): the packed 13 x 13 G (K x 91, may be NULL) and
 * errors 0.5 ||r/sigma||^2 (K, may be NULL) of K pairs at poses (poses_i[k],
 * poses_j[k]) from their moments mom (K x 272) taken at (ref_i[k], ref_j[k]) — equal to
 * fmx_linearize at the same poses up to rounding (gtsam.hpp:67-86, factor.cpp:30-128). */
fmx_status fmx_moments_contract(uint32_t K, const double* mom, const double* ref_i34, const double* ref_j34,
                                const double* poses_i34, const double* poses_j34, double sigma, double* G,
                                double* err);
/* NoiseModelFactor::error of every pair (FeatureFactor::evaluateError without
 * Jacobians), err: K x 1. */
fmx_status fmx_error(fmx_ctx* ctx, const double* poses_i34, const double* poses_j34,
                     double sigma, double* err);
/* The single-pose ablation's whole linear system at X(j) = pose_j34 (X(i) fixed at
 * the built map's poses; fused with a deferred fmx_match at the same pose, see
 * fmx_match): sum over every accepted match of the last fmx_match of the
 * 7 x 7 [H_j b]^T [H_j b] — what GTSAM's LM eliminates from get_single_graph's
 * BinaryFactorWrapper<FeatureFactor>s (constraints.cpp:235-250, gtsam.hpp:40-54,
 * 144-170) — in one launch over the match outputs in query order.  out[0..27]: the
 * packed upper 7 x 7, out[28]: the error 0.5 ||r/sigma||^2. */
fmx_status fmx_linearize_matched(fmx_ctx* ctx, const double pose_j34[12], double sigma, double out[29]);

/* Point-set registration against the built map in the single-pose formulation (the
 * 2M-point C5 configuration): from pose_init, iterate
 *   Matcher::match at X (matcher.hpp:67-112) -> the summed 7 x 7 [H_j b]^T [H_j b]
 *   (gtsam.hpp:67-86, 144-170; all-reduced over the communicator's ranks, below) ->
 *   Gauss-Newton step H dx = g -> X <- X Exp(dx)
 * until ||dx|| < threshold (form.cpp:83-88's break) or max_iters iterations.  The whole
 * loop runs in libfmx (on large query sets each iteration is one fused launch); every
 * rank of a communicator computes the identical iterate.  pose_out: the result, *iters
 * (may be NULL): the iterations run.  FMX_E_STATE if a system is singular. */
fmx_status fmx_register_points(fmx_ctx* ctx, const double pose_init34[12], double max_dist, double sigma,
                               uint32_t max_iters, double threshold, double pose_out34[12], uint32_t* iters);

/* ---------------- multi-GPU: the sharded C5 path -----------
 * One rank per GPU, each with the same voxel map and a contiguous shard of the
 * queries.  fmx_comm_unique_id on one rank; the caller shares the 128 bytes (e.g. a
 * torch.distributed broadcast); fmx_comm_init on every rank (collective).  From then
 * on the context's linearization sums — fmx_linearize_matched's 7 x 7 system and
 * fmx_linearize / fmx_error's per-pair G — are all-reduced (fp64 sum) over the ranks
 * with RCCL on the context's HIP stream, device buffer to device buffer, before they
 * reach the host, so every rank returns the identical global system.  The reference
 * has no multi-device path; this is the north star's "RCCL all-reduce of the normal
 * equations over xGMI".  RCCL is loaded on first use (FMX_E_RCCL if absent).  A wait for
 * an all-reduce is bounded: it polls the stream and ncclCommGetAsyncError and, after
 * FMX_COMM_TIMEOUT_S seconds (environment, default 60), aborts the communicator and
 * returns FMX_E_RCCL.  The communicator is gone then, and every later sharded call
 * (fmx_linearize_matched, fmx_linearize / fmx_error, fmx_register_points) also returns
 * FMX_E_RCCL until fmx_comm_init attaches a new one: this rank holds only a shard of the
 * queries, so a rank-local system must never stand in for the global one. */
fmx_status fmx_comm_unique_id(uint8_t id[128]);
fmx_status fmx_comm_init(fmx_ctx* ctx, const uint8_t id[128], int nranks, int rank);

/* ---------------- host adapter: Estimator::register_scan -------------------
 * form::Estimator::register_scan (form/form.hpp:82-83, form.cpp:40-114): predict,
 * extract, map build, ICP loop (match + LM), final LM, insert_matches, keyscan
 * selection, marginalization.  The smoother runs in ConstraintManager's default
 * smoothing mode (LM over every window pose, constraints.cpp:103-118, 252-308,
 * marginal LinearContainerFactors, constraints.cpp:120-203) or, with
 * params.disable_smoothing, in the single-pose ablation (constraints.cpp:103-111,
 * 235-250).  Every FeatureFactor linearization runs on the device. */
fmx_status fmx_register_scan(fmx_ctx* ctx, const float* xyzw, size_t n_points, int src_on_device,
                             fmx_feature_counts* out);
/* Pipelined extraction (no reference counterpart; an fmx throughput option).
 * Announces the scan that will FOLLOW the one passed to the next fmx_register_scan:
 * that call extracts it (FeatureExtractor::extract, extraction.tpp:29-132) on a side
 * stream while it registers its own scan, and the register_scan of this scan then
 * skips its extraction.  Results are identical either way: extraction depends only on
 * the scan.  The scan may be device-resident (src_on_device = 1) or host memory (0: a
 * pageable scan's staging copy starts at once on the helper threads, and the scan is
 * DMA'd and extracted on the side stream as soon as that copy has finished); it must
 * stay unchanged until its own fmx_register_scan returns.  That call must pass the
 * same pointer with the same src_on_device, else the queued extraction is discarded
 * and the scan extracted in the call.  xyzw = NULL withdraws the announcement.  A
 * withdrawing or replacing call returns only once the staging copy of a withdrawn or
 * replaced pageable scan has finished: from then on its memory is no longer read. */
fmx_status fmx_next_scan(fmx_ctx* ctx, const float* xyzw, size_t n_points, int src_on_device);
/* Estimator::current_lidar_estimate (form/form.hpp:79). */
fmx_status fmx_current_pose(fmx_ctx* ctx, double pose34[12]);
/* FORM::map() (python/bindings.cpp:96-119): KeypointMap::to_voxel_map of both feature
 * types (map.tpp:128-146) at the current window estimates, voxel width voxel_width
 * (the binding passes min_dist_map, bindings.cpp:100), every voxel's points in turn —
 * world frame, planar: 6 doubles (x, y, z, nx, ny, nz), point: 3 doubles, plus the
 * scan id of each (the binding ships it as the point's column, bindings.cpp:31-41).
 * Voxel order is unspecified (the reference iterates a robin_map); inside a voxel,
 * push_back order (scans ascending, then keypoint order).  Two calls: with NULL
 * buffers *n_planar / *n_point receive the sizes; with buffers they are the
 * capacities on entry (FMX_E_SIZE if too small) and the counts on return.  Needs a
 * registered scan (FMX_E_STATE otherwise). */
fmx_status fmx_map_download(fmx_ctx* ctx, double voxel_width, double* planar, uint64_t* planar_scan,
                            uint32_t* n_planar, double* point, uint64_t* point_scan, uint32_t* n_point);

/* Statistics of the last register_scan, the first n of: {icp_iters, lm_iters,
 * matched_planar, matched_point, map_planar, map_point, linearizations, map_scans,
 * host_waits (host<->device round trips: waits on a completion word or the stream),
 * spec_matches (speculative matches launched at LM-trial poses), spec_hits (ICP
 * iterations that used one instead of matching), spec_map (1 when the scan's map was
 * the one built speculatively during the previous scan's final LM, 0 when built at
 * the start of this scan), pipelined (1 when the scan's features were extracted
 * during the previous registration, fmx_next_scan), window_poses (poses in the
 * smoother's window after the scan: the host LM's system is 6 x window_poses)};
 * entries past the known ones read 0. */
fmx_status fmx_last_stats(fmx_ctx* ctx, uint64_t* stats, int n);
/* Work of the last fmx_match (counted by the kernel, available while profiling is
 * enabled): queries, hash probes, candidate records distance-tested. */
fmx_status fmx_match_work(fmx_ctx* ctx, double work[3]);
/* The warm certificate of the last fmx_match (no profiling needed).  A match on the same
 * map and query set as the previous one starts warm; a warm query whose previous nearest
 * record provably stays nearest after the pose step (it kept its cell, and every other
 * record was farther than that record by more than twice the step) skips the search —
 * the result is identical to a search (VoxelMap::find_closest, map.tpp:70-91).
 * counts[0] = certified queries, counts[1] = warm queries (either may be 0);
 * certified (may be NULL): per query (planar then point) 1 if it was certified. */
fmx_status fmx_match_cert(fmx_ctx* ctx, uint64_t counts[2], uint8_t* certified);

/* ---------------- profiling (bench.py roofline) ----------------------------
 * When enabled, each kernel launch is bracketed by HIP events on the context
 * stream.  fmx_profile_read fills, for kernel id k < n: total ms, launches and
 * algorithmic bytes accumulated since the last reset. */
fmx_status fmx_profile_enable(fmx_ctx* ctx, int on);
fmx_status fmx_profile_reset(fmx_ctx* ctx);
int fmx_profile_count(void);
const char* fmx_profile_name(int k);
fmx_status fmx_profile_read(fmx_ctx* ctx, double* ms, uint64_t* launches, double* bytes, int n);
/* Match work of the profiled match launches since the last reset, cold (the first match
 * on a map / query set) then warm: {launches, queries, probes, candidates, certified
 * queries, warm queries} each (fmx_match_cert's counts, summed). */
fmx_status fmx_profile_match_work(fmx_ctx* ctx, double out[12]);

/* Wait for all of the context's device work (its stream and the side streams of the
 * map build and the pipelined extraction). */
fmx_status fmx_sync(fmx_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* FMX_FMX_H_ */
