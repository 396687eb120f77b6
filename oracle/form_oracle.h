/*
 * form_oracle.h — C interface of the CPU oracle for FORM's scan-to-submap path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so, and only as the checker / CPU baseline.
 * The product (form_amd/, libfmx.so) never links, loads or calls anything here.
 *
 * PARITY STATUS: the reference (huangjuite/form) cannot be compiled in this image
 * (Eigen3, GTSAM, oneTBB headers and tsl::robin_map are absent; CMake FetchContent
 * needs network) and it ships no golden vectors (its only test,
 * tests/test_SeparateFactor.cpp, is stale and pins no numbers).  This oracle is a
 * line-by-line CPU restatement of the reference files cited per function in
 * form_oracle.cpp.  It is cross-checked against an independent numpy restatement
 * and against finite-difference Jacobians (tests/), but against reference OUTPUTS
 * it is "parity unpinned".
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same field order as fmx_extract_params (include/fmx/fmx.h) and
 * form::FeatureExtractor::Params (form/feature/extraction.hpp:59-88). */
typedef struct orc_extract_params {
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
} orc_extract_params;

typedef struct orc_params {
  orc_extract_params extraction;
  double max_dist_matching;      /* MatcherParams, matcher.hpp:32-41 */
  double new_pose_threshold;
  uint32_t max_num_rematches;
  double planar_constraint_sigma; /* ConstraintManager::Params, constraints.hpp:54-70 */
  int32_t disable_smoothing;
  int64_t max_num_keyscans;       /* KeyScanner::Params, keyscanner.hpp:55-64 */
  int64_t max_steps_unused_keyscan;
  uint32_t max_num_recent_scans;
  double keyscan_match_ratio;
  double min_dist_map;            /* KeypointMapParams, map.hpp:97-100 */
} orc_params;

void orc_default_params(orc_params* p);

/* ---- stage 1: FeatureExtractor::extract (extraction.tpp:29-132) ----
 * xyzw: R*C float4 (PointXYZf layout), row-major.
 * Outputs (caller-allocated; capacities: sel <= R*S*(P+1), points <= R*C):
 *   sel_idx / n_sel    : planar indices in selection order (row, sector, curvature)
 *   normal_ok[n_sel]   : 1 if compute_normal returned a value
 *   normals[3*n_sel]   : float normal (sign: oriented towards the sensor origin)
 *   point_idx / n_point: point-feature indices in selection order
 *   planar_mask, point_mask (optional, R*C bytes): compute_valid_points /
 *   compute_point_valid_points.  curvature (optional, R*C floats).
 * Returns 0, or -1 on a size mismatch (the reference throws, extraction.tpp:141-145). */
int orc_extract(const orc_extract_params* p, const float* xyzw, size_t n_points,
                int nthreads, uint32_t* sel_idx, uint32_t* n_sel, uint8_t* normal_ok,
                float* normals, uint32_t* point_idx, uint32_t* n_point,
                uint8_t* planar_mask, uint8_t* point_mask, float* curvature);

/* ---- stage 2: VoxelMap / KeypointMap::to_voxel_map / Matcher::match ----
 * A map holds the world-frame keypoints of several scans (map.tpp:128-146).
 * kind = 0 planar (records are 6 floats: xyz, nxyz), 1 point (3 floats). */
void* orc_map_new(double voxel_width, int kind);
void orc_map_free(void* m);
void orc_map_add_scan(void* m, uint64_t scan, const double pose34[12], const float* feats,
                      uint32_t n);
uint64_t orc_map_num_voxels(void* m);
/* Matcher<P>::match<I> (matcher.hpp:67-112) for one query scan at pose_j.
 * Per query q: found[q] (1 if the 27-voxel NN exists), scan[q], d2[q],
 * pi[3q..] / ni[3q..] = matched point (and normal) moved back to its scan's local frame. */
void orc_map_match(void* m, const float* queries, uint32_t nq, const double pose_j34[12],
                   int nthreads, uint8_t* found, uint64_t* scan, double* d2, double* pi,
                   double* ni);

/* ---- stage 3: FeatureFactor + DenseFactor::linearize (factor.cpp:30-186,
 * gtsam.hpp:67-139) ----
 * K pairs; pair k has np[k] plane rows then nt[k] point pairs (3 rows each), packed
 * contiguously in pair order.  poses_i / poses_j: K x 12 (row-major 3x4).
 * single_pose=0: G = K x 91 packed upper triangle of [H_i H_j b]^T [H_i H_j b]
 * single_pose=1: G = K x 28 packed upper triangle of [H_j b]^T [H_j b]
 * err[k] = 0.5*||r/sigma||^2. */
void orc_linearize(uint32_t K, const uint32_t* np, const double* plane_pi,
                   const double* plane_ni, const double* plane_pj, const uint32_t* nt,
                   const double* point_pi, const double* point_pj, const double* poses_i,
                   const double* poses_j, double sigma, int single_pose, double* G,
                   double* err);
/* Raw per-row residuals and 12-column Jacobians of ONE pair (unwhitened). */
void orc_factor_rows(uint32_t np, const double* plane_pi, const double* plane_ni,
                     const double* plane_pj, uint32_t nt, const double* point_pi,
                     const double* point_pj, const double pose_i[12],
                     const double pose_j[12], double* r, double* J);

/* ---- SE(3) helpers (GTSAM Pose3 conventions: tangent [w; v], right perturbation) */
void orc_pose_expmap(const double xi[6], double out34[12]);
void orc_pose_logmap(const double T34[12], double xi[6]);
void orc_pose_compose(const double a[12], const double b[12], double out[12]);
void orc_pose_inverse(const double a[12], double out[12]);

/* ---- full register_scan restatement (form.cpp:40-114) in single-pose mode ---- */
void* orc_estimator_new(const orc_params* p, int nthreads);
void orc_estimator_free(void* e);
/* stats[0..5] = {planar, point, icp_iters, lm_iters, matched_planar, matched_point};
 * times_ms[0..3] = {extract, map_build, icp(match+lm), total} */
int orc_register_scan(void* e, const float* xyzw, size_t n, double pose_out34[12],
                      uint32_t* stats, double* times_ms);
/* FORM::map() restated: the stored keypoints of feature type kind (0 planar, 1 point)
 * in the world frame at the current values, push_back order (scans ascending); returns
 * the count; any output pointer may be NULL. */
uint32_t orc_estimator_map(void* e, int kind, double* xyz, double* nrm, uint64_t* scans);

#ifdef __cplusplus
}
#endif
