/* =====================================================================================
 * pfx.h -- C-ABI of the MI355X-native (gfx950) feature-extraction path.
 *
 * This is the drop-in boundary that replaces the PCL 1.7 calls srv/pcl_feature_extraction
 * makes on its hot path.  Plain pointers and sizes, no torch or PCL
 * types.  Every entry point returns 0 on success; on failure a nonzero pfx_status and the
 * message is available from pfx_last_error(ctx).  PCL's own error behaviour (initCompute
 * failure -> PCL_ERROR + empty output; per-point failure -> NaN fill) is mapped by the C++
 * facade (include/pfx_pcl.hpp) onto these codes.
 *
 * Two families:
 *   pfx_*      host pointers in / host pointers out (synchronous, H2D/D2H inside)
 *   pfx_*_dev  device pointers in / device pointers out, stream-ordered on the ctx stream
 * Arrays are structure-of-arrays float32 (x, y, z / nx, ny, nz), indexed by the caller's
 * point index, exactly the order of PointCloud<T>::points.
 *
 * Replaced reference interfaces (file:line in /root/reference):
 *   pfx_normals*        <- Tools::estimateNormals -> NormalEstimationOMP<PointXYZRGB,Normal>
 *                          ::compute  (include/pcl_feature_extraction/tools.h:22-32)
 *   pfx_fpfh*           <- FPFHEstimation<PointXYZRGB,Normal,FPFHSignature33>::compute via
 *                          Features<T>::compute (features.h:175-196, evaluation.cpp:593-612)
 *   pfx_shot*           <- SHOTEstimationOMP<PointXYZRGB,Normal,SHOT352>::compute
 *                          (features.h:175-196, evaluation.cpp:766-785)
 *   pfx_range_image_planar* <- RangeImagePlanar::createFromPointCloudWithFixedSize
 *                          (keypoints.h:212-216, tools.h:61-77)
 *   pfx_narf_keypoints* <- RangeImageBorderExtractor + NarfKeypoint::compute
 *                          (keypoints.h:219-224)
 *   pfx_radius_search*  <- search::KdTree<PointXYZRGB>::radiusSearch (features.h:192,
 *                          tools.h:29; FLANN order: (d^2, index) ascending, strict d^2 < r^2)
 *   pfx_nearest_descriptors_dev <- Features<T>::getCorrespondences (features.h:255-273):
 *                          KdTreeFLANN<FeatureT>::nearestKSearch(k = 1) per descriptor
 *   pfx_correspondences* <- Features<T>::findCorrespondences (features.h:224-253)
 *   pfx_pcd_*           <- pcl::io::loadPCDFile<PointXYZRGB> (evaluation.cpp:226-235)
 *   pfx_cloud_resolution* <- Keypoints::computeCloudResolution (keypoints.h:401-428)
 *   pfx_iss_keypoints*  <- ISSKeypoint3D<PointXYZRGB,PointXYZRGB>::compute as configured by
 *                          Keypoints::compute's ISS branch (keypoints.h:177-189)
 *   pfx_harris3d_keypoints* <- HarrisKeypoint3D<PointXYZRGB,PointXYZI>::compute + getKeypointsCloud
 *   pfx_harris6d_keypoints* <- HarrisKeypoint6D<PointXYZRGB,PointXYZI>::compute + getKeypointsCloud
 *                          (Keypoints::compute's HARRIS_3D branch, keypoints.h:150-162, 365-395)
 *   pfx_ransac_rejector <- registration::CorrespondenceRejectorSampleConsensus<PointXYZRGB> in
 *                          Features<T>::filterCorrespondences (features.h:282-297)
 * ===================================================================================== */
#ifndef PFX_H_
#define PFX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pfx_ctx pfx_ctx;
typedef int32_t pfx_status;

enum {
  PFX_OK = 0,
  PFX_ERR_INVALID = 1,     /* bad argument (null pointer, negative size, radius <= 0, ...) */
  PFX_ERR_DEVICE = 2,      /* HIP runtime error (message from hipGetErrorString)            */
  PFX_ERR_CAPACITY = 3,    /* caller buffer too small (required size in the out count)      */
  PFX_ERR_UNSUPPORTED = 4  /* parameter combination the path does not implement             */
};

/* NarfKeypoint::Parameters + RangeImageBorderExtractor::Parameters (PCL 1.7 defaults; the
 * reference sets only support_size = 0.2f, keypoints.h:223). */
typedef struct pfx_narf_params {
  float support_size;                            /* -1 (must be set > 0)   */
  int32_t max_no_of_interest_points;             /* -1 = unlimited          */
  float min_distance_between_interest_points;    /* 0.25 (x support_size)   */
  float optimal_distance_to_high_surface_change; /* 0.25                    */
  float min_interest_value;                      /* 0.45                    */
  float min_surface_change_score;                /* 0.2                     */
  /* 1.  The greedy selection then orders the survivors with std::sort on strength, as PCL does:
   * the order of EQUAL strengths is the sort implementation's (the libstdc++ this library is
   * built with; PCL's was an Indigo-era GCC).  It decides the keypoints only when two tied
   * survivors lie closer than min_distance_between_interest_points * support_size:
   * scripts/narf_tie_report.py finds none on the reference's four clouds (their keypoints are
   * independent of the toolchain: tests/test_oracle_narf_ties.py) and 6-11 such pairs on each
   * configs[2] synthetic room, where 4-7 of ~85 keypoints move between the two extreme tie
   * orders (profiles/r05_narf_tie_report.jsonl).  The GPU path and the oracle share this
   * build's order. */
  int32_t do_non_maximum_suppression;
  /* 1 (PCL's default).  Either value computes NarfKeypoint's COMPLETE interest formula
   * (calculateCompleteInterestImage); 1 only skips pixels that provably cannot reach
   * min_interest_value, so 0 and 1 give the same keypoints.  PCL 1.7's own sparse heuristics
   * (calculateSparseInterestImage, source absent here) are NOT reproduced: parity with that
   * mode is unpinned, with a measured sensitivity of 1-2 keypoints per reference cloud
   * (DESIGN.md section 5).  pfx_ctx_last_stats(ctx, "narf_interest_formula") = 0 after every
   * NARF call (0 = complete formula). */
  int32_t calculate_sparse_interest_image;
  int32_t no_of_polynomial_approximations_per_point; /* 0 (only 0 supported) */
  int32_t add_points_on_straight_edges;          /* 0 (only 0 supported)    */
  /* RangeImageBorderExtractor::Parameters */
  int32_t pixel_radius_borders;                  /* 3   */
  int32_t pixel_radius_plane_extraction;         /* 2   */
  int32_t pixel_radius_border_direction;         /* 2   */
  float minimum_border_probability;              /* 0.8 */
  int32_t pixel_radius_principal_curvature;      /* 2   */
} pfx_narf_params;

/* RangeImagePlanar::createFromPointCloudWithFixedSize arguments */
typedef struct pfx_camera {
  int32_t width, height;          /* 640, 480 (keypoints.h:204)     */
  float center_x, center_y;       /* 320, 240 (keypoints.h:205)     */
  float focal_length_x, focal_length_y; /* 525, 525 (keypoints.h:206, both fx) */
  float sensor_pose[16];          /* row-major 4x4 Affine3f (sensor_origin_ * orientation_) */
  int32_t coordinate_frame;       /* 0 = CAMERA_FRAME, 1 = LASER_FRAME */
  float noise_level;              /* 0 */
  float min_range;                /* 0 */
} pfx_camera;

void pfx_narf_params_default(pfx_narf_params* p);
/* The reference's NARF setup (keypoints.h:203-223) with an identity pose */
void pfx_camera_default(pfx_camera* c);

/* ---- context ---------------------------------------------------------------------- */
pfx_status pfx_ctx_create(int device, pfx_ctx** out);
void pfx_ctx_destroy(pfx_ctx* ctx);
const char* pfx_last_error(const pfx_ctx* ctx);
/* Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL is HIP's
 * null stream (torch's default stream).  A new ctx runs on its own non-blocking stream, created
 * by the first call that runs on it (a ctx set to an external stream first never creates one). */
pfx_status pfx_ctx_set_stream(pfx_ctx* ctx, void* hip_stream);
/* Back to the ctx-owned non-blocking stream. */
pfx_status pfx_ctx_use_own_stream(pfx_ctx* ctx);
void* pfx_ctx_get_stream(pfx_ctx* ctx);
/* Frees every device scratch buffer of ctx (grids, neighbour lists, the rarely used overflow
 * scratch of the list builder and the FPFH weighting, NARF images) after synchronising its
 * stream; the next call reallocates what it needs.  Held state (lists kept for
 * pfx_normals_chains_dev / pfx_fpfh_after_normals_dev, prepared FPFH grids) is dropped. */
pfx_status pfx_ctx_trim(pfx_ctx* ctx);
pfx_status pfx_ctx_synchronize(pfx_ctx* ctx);
/* Launch-shape hint, no effect on results: another stream of this process runs latency-critical
 * work on the device at the same time (the overlapped NARF + normal estimation step).
 * NARF's flood fill then runs on 4 instead of 20 waves per CU, so the concurrent grid build
 * and list set-up find free wave slots (1M-pt room: 161.4 -> 162.6 Mpoints/s; alone the
 * interest stage takes 0.63 instead of 0.47 ms, hence off by default). */
pfx_status pfx_ctx_set_shared(pfx_ctx* ctx, int shared);
/* HIP-event timing on the ctx stream (for bench.py's live roofline): enable = 1 times every kernel
 * group, 2 only the stage scopes (one event pair per stage call: "normals", "normals_fast", "iss",
 * "harris3d", ...; the per-kernel pairs cost ~2 % of the headline step in host launch time), 0 off. */
pfx_status pfx_ctx_set_timing(pfx_ctx* ctx, int enable);
pfx_status pfx_ctx_reset_timing(pfx_ctx* ctx);
/* Accumulated device time and launch count of the kernel `name`; syncs the stream. */
pfx_status pfx_ctx_kernel_time(pfx_ctx* ctx, const char* name, double* total_ms,
                               int64_t* launches);
/* Statistics of the last calls on ctx, by name: e.g. "normals_neighbors" (sum over queries of
 * |N_r(q)| of the last normals call -- the per-launch unit count for the neighbour-gather
 * roofline), "narf_keypoints", "narf_interest_formula" (0 = NarfKeypoint's complete formula, the
 * only one implemented; see pfx_narf_params.calculate_sparse_interest_image). */
pfx_status pfx_ctx_last_stats(pfx_ctx* ctx, const char* what, int64_t* value);

/* ---- radius search (FLANN semantics) ---------------------------------------------- */
/* counts[nq] = |{p : d2(q,p) < (float)(r*r)}|; if idx != NULL also the first `cap`
 * neighbours of each query in (d2, index) order, row-major with row stride `cap`. */
pfx_status pfx_radius_search(pfx_ctx* ctx, const float* x, const float* y, const float* z,
                             int64_t n, const float* qx, const float* qy, const float* qz,
                             int64_t nq, double radius, int64_t* counts, int32_t* idx,
                             float* d2, int64_t cap);

/* ---- normals: NormalEstimationOMP (input == surface) ------------------------------- */
pfx_status pfx_normals(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                       double radius, const float viewpoint[3], float* nx, float* ny, float* nz,
                       float* curvature);
pfx_status pfx_normals_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                           int64_t n, double radius, const float viewpoint[3], float* d_nx,
                           float* d_ny, float* d_nz, float* d_curvature);
/* The same computation in two phases, so that a caller can order the points it needs first
 * (results identical to pfx_normals_dev):
 *   lists  -- radius-neighbour lists of every finite point, kept in ctx; outputs NaN-filled;
 *   chains -- the normals of the points with (d_mask[i] != 0) == want (all when d_mask is
 *             null), on ctx's stream, from the lists held by `lists_ctx` (ctx itself or another
 *             context on the same device whose lists phase is ordered before this call).  Two
 *             chains calls with complementary masks may run concurrently on two contexts.
 *             want = 3 / 2: workgroup partition -- every point of a block of 256 consecutive
 *             (cell-ordered) queries that holds any masked point / holds none, so the two passes
 *             stage each block's candidates once between them (the masked points are a subset
 *             of pass 3's). */
pfx_status pfx_normals_lists_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                 int64_t n, double radius, float* d_nx, float* d_ny, float* d_nz,
                                 float* d_curvature);
pfx_status pfx_normals_chains_dev(pfx_ctx* ctx, pfx_ctx* lists_ctx, const uint8_t* d_mask, int32_t want,
                                  const float viewpoint[3], float* d_nx, float* d_ny, float* d_nz,
                                  float* d_curvature);

/* pfx_normals_dev split at its one host round trip, so a consumer (FPFH) can be queued on another
 * stream right behind the estimation: _launch queues grid, lists and chains with no host wait
 * (the chains compute nothing unless the lists turn out whole); _finish validates them (host
 * wait on ctx's stream) and, rarely -- a scan outside the previous scan's widened bounds, a list
 * buffer to grow, the first very long lists -- reruns the exact path, stream-ordered on ctx's
 * stream, and sets *rerun = 1: whatever read the outputs in between must then run again.
 * Results after _finish are pfx_normals_dev's, bit for bit. */
pfx_status pfx_normals_launch_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                  int64_t n, double radius, const float viewpoint[3], float* d_nx,
                                  float* d_ny, float* d_nz, float* d_curvature);
pfx_status pfx_normals_finish_dev(pfx_ctx* ctx, int32_t* rerun);

/* Scheduling hint (no reference counterpart): the next pfx_normals_launch_dev / pfx_normals_dev on
 * ctx makes its stream wait for hip_event (a hipEvent_t already recorded by the caller) after its
 * grid build and list set-up and before its neighbour-list kernels, once.  The list kernels are
 * persistent and fill the device; a short stage on another stream that must not queue behind
 * them (FPFH's surface grid, which NARF's chain then follows) is kept ahead this way.  NULL
 * clears it. */
pfx_status pfx_normals_gate_dev(pfx_ctx* ctx, void* hip_event);
/* Scheduling aid: queue the (speculative) grid of the next pfx_normals_launch_dev /
 * pfx_normals_dev on the same d_x, d_y, d_z, n and radius now, so the caller can issue it before another
 * stream's work (and that work's gate, pfx_normals_gate_dev) and the estimation's lists after.
 * Results are unchanged; any other call in between on ctx discards it. */
pfx_status pfx_normals_grid_launch_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                       int64_t n, double radius);

/* NormalEstimationOMP (tools.h:22-32) over a subset of the cloud: the points with
 * (d_mask[i] != 0) == want get PCL's normal and curvature bit for bit (their neighbours are
 * searched in the whole cloud); every other output entry is left untouched.  Two calls, want = 1
 * then 0, give pfx_normals_dev's result.  Use: FPFH's support (pfx_fpfh_support_ball_dev) first,
 * so FPFHEstimation starts on another stream while the rest is estimated -- the normals are
 * Features::compute's intermediate (features.h:185-187), FPFH reads only the support's.
 * pfx_normals_prepare_dev builds the cloud's grid ahead (coordinates only), e.g. while the mask
 * is still being computed; pfx_normals_subset_dev builds it itself otherwise. */
pfx_status pfx_normals_prepare_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                   int64_t n, double radius);
pfx_status pfx_normals_subset_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                  int64_t n, double radius, const uint8_t* d_mask, int32_t want,
                                  const float viewpoint[3], float* d_nx, float* d_ny, float* d_nz,
                                  float* d_curvature);

/* Opt-in fast mode, NOT parity-exact (BASELINE north_star "MFMA for the 3x3
 * covariance accumulation"): the same neighbour set (FLANN's d2 < (float)(r*r)), but the
 * covariance sums are one MFMA contraction per 16 points -- hit mask x candidate features,
 * centred on the group's first point -- instead of PCL's sequential float chains in FLANN order,
 * so no neighbour list is sorted or stored.  Results differ from pfx_normals by rounding (the
 * sums carry less rounding than PCL's raw-coordinate ones); bench.py --workload fastnormals
 * reports the deviation.  Same NaN rules (< 3 neighbours, non-finite points). */
pfx_status pfx_normals_fast(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                            double radius, const float viewpoint[3], float* nx, float* ny, float* nz,
                            float* curvature);
pfx_status pfx_normals_fast_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                int64_t n, double radius, const float viewpoint[3], float* d_nx,
                                float* d_ny, float* d_nz, float* d_curvature);

/* ---- FPFH-33: FPFHEstimation (surface + normals, queries = input cloud) ------------- */
/* same_as_surface != 0 selects PCL's "input_ == surface_ && indices == all" branch (queries
 * must then be the surface itself).  out: nq x 33 row-major (FPFHSignature33::histogram). */
pfx_status pfx_fpfh(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz,
                    const float* snx, const float* sny, const float* snz, int64_t n_surface,
                    const float* qx, const float* qy, const float* qz, int64_t nq,
                    int same_as_surface, double radius, float* out);
/* _dev: stream-ordered, no host synchronisation; its statistics (pfx_ctx_last_stats) and a
 * neighbourhood beyond the 2^22 capacity (PFX_ERR_CAPACITY) are reported by the next
 * pfx_ctx_synchronize / pfx_ctx_last_stats on this ctx.
 * pfx_fpfh_dev never reuses state of an earlier normal estimation: it builds its own lists. */
pfx_status pfx_fpfh_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                        const float* d_snx, const float* d_sny, const float* d_snz,
                        int64_t n_surface, const float* d_qx, const float* d_qy,
                        const float* d_qz, int64_t nq, int same_as_surface, double radius,
                        float* d_out);
/* Features::compute's sequence (features.h:187-195): pfx_fpfh_dev right after a
 * pfx_normals_dev / pfx_normals_lists_dev on this ctx over the same device cloud.  The caller
 * vouches that (d_sx, d_sy, d_sz) still hold the cloud that normal estimation ran on; with
 * same_as_surface, equal pointers, n_surface and radius, its FLANN-ordered neighbour lists are
 * then reused for the weighting (else they are built as in pfx_fpfh_dev).  Either way the
 * held lists are released, so a second call cannot reuse them. */
pfx_status pfx_fpfh_after_normals_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                                      const float* d_snx, const float* d_sny, const float* d_snz,
                                      int64_t n_surface, const float* d_qx, const float* d_qy,
                                      const float* d_qz, int64_t nq, int same_as_surface, double radius,
                                      float* d_out);

/* Builds the search-surface index of the next pfx_fpfh_dev call on this ctx ahead of time (the
 * surface grid needs only the coordinates, so it can overlap normal estimation -- PCL builds the
 * same tree inside FPFHEstimation::compute, features.h:192-195).  The next pfx_fpfh_dev with the
 * same (d_sx, n_surface, radius) consumes it; the surface must not change in between. */
pfx_status pfx_fpfh_prepare_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                                int64_t n_surface, double radius);
/* Also marks the SPFH point set S of the next pfx_fpfh_dev (input != surface) for these queries
 * (d_qx must be the same pointer, nq the same count): S needs only the coordinates, so it can be
 * found while the normals are still being computed.  Builds the surface grid first if needed. */
pfx_status pfx_fpfh_prepare_queries_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                                        int64_t n_surface, const float* d_qx, const float* d_qy,
                                        const float* d_qz, int64_t nq, double radius);
/* d_mask[i] = 1 for every surface point whose normal FPFHEstimation reads for these queries
 * (the r-neighbours of the SPFH set S = the r-neighbourhoods of the queries, fpfh.hpp), else 0.
 * n_surface bytes.  The next pfx_fpfh_dev on ctx reads only these normals, so the others may
 * still be computed concurrently (pfx_normals_chains_dev with want = 0 on another stream). */
pfx_status pfx_fpfh_support_mask_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                                     int64_t n_surface, const float* d_qx, const float* d_qy,
                                     const float* d_qz, int64_t nq, double radius, uint8_t* d_mask);

/* Conservative form of pfx_fpfh_support_mask_dev: d_mask[i] = 1 for every surface point within
 * 2 * radius of a query (a superset of the normals FPFHEstimation reads, marked in one pass over
 * the queries' 5x5x5 cell blocks instead of one per SPFH point).  Same contract for the next
 * pfx_fpfh_dev on ctx. */
pfx_status pfx_fpfh_support_ball_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                                     int64_t n_surface, const float* d_qx, const float* d_qy,
                                     const float* d_qz, int64_t nq, double radius, uint8_t* d_mask);

/* ---- SHOT-352: SHOTEstimationOMP + SHOTLocalReferenceFrameEstimation ---------------- */
/* desc: nq x 352, rf: nq x 9 (x_axis, y_axis, z_axis) -- SHOT352::{descriptor, rf}. */
pfx_status pfx_shot(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz,
                    const float* snx, const float* sny, const float* snz, int64_t n_surface,
                    const float* qx, const float* qy, const float* qz, int64_t nq,
                    double radius, float* desc, float* rf);
pfx_status pfx_shot_dev(pfx_ctx* ctx, const float* d_sx, const float* d_sy, const float* d_sz,
                        const float* d_snx, const float* d_sny, const float* d_snz,
                        int64_t n_surface, const float* d_qx, const float* d_qy,
                        const float* d_qz, int64_t nq, double radius, float* d_desc,
                        float* d_rf);

/* ---- range image + NARF keypoints ---------------------------------------------------- */
/* out_points: width*height x 4 floats {x, y, z, range} (PointWithRange); unobserved pixels
 * are {NaN, NaN, NaN, -inf}. */
pfx_status pfx_range_image_planar(pfx_ctx* ctx, const float* x, const float* y, const float* z,
                                  int64_t n, const pfx_camera* cam, float* out_points);
/* Keypoint pixel indices (y*width + x), ascending, as NarfKeypoint::compute returns them in
 * PointCloud<int>.  *n_out = number of keypoints; PFX_ERR_CAPACITY if it exceeds cap. */
pfx_status pfx_narf_keypoints(pfx_ctx* ctx, const float* x, const float* y, const float* z,
                              int64_t n, const pfx_camera* cam, const pfx_narf_params* params,
                              int32_t* out, int64_t cap, int64_t* n_out);
pfx_status pfx_narf_keypoints_dev(pfx_ctx* ctx, const float* d_x, const float* d_y,
                                  const float* d_z, int64_t n, const pfx_camera* cam,
                                  const pfx_narf_params* params, int32_t* out, int64_t cap,
                                  int64_t* n_out);
/* Debug/parity access to the NARF intermediates of the last pfx_narf_keypoints* call
 * (host buffers of width*height elements):  "interest" (float), "surface_change" (float),
 * "border_traits" (uint32 bitset, PCL BorderTrait order), "range" (float).            */
pfx_status pfx_narf_debug_image(pfx_ctx* ctx, const char* which, void* out, int64_t count);

/* ---- the reference's keypoint -> cloud mapping (keypoints.h:227-229) ----------------- */
/* k_xyz[i] = cloud[idx[i]] for 0 <= idx[i] < n (the reference indexes the cloud with pixel
 * indices; out-of-range indices are an out-of-bounds read there and are skipped here).
 * d_kx/d_ky/d_kz hold `cap` floats each; more in-range indices than `cap` -> PFX_ERR_CAPACITY
 * (nothing written).  Returns the number of points written in *n_out. */
pfx_status pfx_gather_points_dev(pfx_ctx* ctx, const float* d_x, const float* d_y,
                                 const float* d_z, int64_t n, const int32_t* idx, int64_t k,
                                 float* d_kx, float* d_ky, float* d_kz, int64_t cap, int64_t* n_out);

/* Descriptor matching.  Rows are `dim` floats, `*_stride` floats apart
 * (FPFHSignature33: dim 33, stride 33; PointCloud<SHOT352> read in place: dim 352, stride 361).
 * Distance = FLANN L2_Simple<float> (sequential float sum of squared differences), exact 1-NN;
 * equal distances -> the lowest row (FLANN: first visited, unpinned); a source row with a
 * non-finite value, or no finite target row -> -1 and NaN distance.
 * Both directions in one pass: d_s2t[i] = nearest target row of source row i (+ its squared
 * distance), d_t2s[j] = nearest source row of target row j.  Distance and t2s outputs are
 * nullable.  Stream-ordered except for one host read of the candidate count. */
pfx_status pfx_nearest_descriptors_dev(pfx_ctx* ctx, const float* d_src, int64_t n_src, int64_t src_stride,
                                       const float* d_tgt, int64_t n_tgt, int64_t tgt_stride, int32_t dim,
                                       int32_t* d_s2t, float* d_s2t_dist, int32_t* d_t2s, float* d_t2s_dist);
/* Host-pointer form of one direction (the facade's KdTreeFLANN<FeatureT>::nearestKSearch). */
pfx_status pfx_nearest_descriptors(pfx_ctx* ctx, const float* src, int64_t n_src, int64_t src_stride,
                                   const float* tgt, int64_t n_tgt, int64_t tgt_stride, int32_t dim,
                                   int32_t* s2t, float* s2t_dist);
/* Mutual nearest neighbours (index_query, index_match) in source order.  *n_out = the number
 * of correspondences (host); PFX_ERR_CAPACITY (nothing written) when it exceeds cap. */
pfx_status pfx_correspondences_dev(pfx_ctx* ctx, const float* d_src, int64_t n_src, int64_t src_stride,
                                   const float* d_tgt, int64_t n_tgt, int64_t tgt_stride, int32_t dim,
                                   int32_t* d_query, int32_t* d_match, int64_t cap, int64_t* n_out);
pfx_status pfx_correspondences(pfx_ctx* ctx, const float* src, int64_t n_src, int64_t src_stride,
                               const float* tgt, int64_t n_tgt, int64_t tgt_stride, int32_t dim,
                               int32_t* query, int32_t* match, int64_t cap, int64_t* n_out);

/* ---- PCD v0.7 input ------------------------------------------------- */
typedef struct pfx_pcd_header {
  int64_t points;          /* POINTS (default WIDTH * HEIGHT)                                  */
  int32_t width, height;
  int32_t data;            /* 0 ascii, 1 binary, 2 binary_compressed                            */
  int32_t point_size;      /* binary: bytes per point; ascii: columns per point                 */
  int32_t x_offset, y_offset, z_offset; /* binary: byte offsets; ascii: column indices          */
  int32_t nfields;
  float viewpoint[7];      /* VIEWPOINT tx ty tz qw qx qy qz (sensor_origin_, sensor_orientation_) */
  int64_t data_offset;     /* byte offset of the data block                                     */
} pfx_pcd_header;
/* Header only (host, no device, no context).  x, y, z must be single float32 fields. */
pfx_status pfx_pcd_read_header(const char* path, pfx_pcd_header* out);
/* loadPCDFile: x, y, z of every point into device SoA arrays (caller order = file order, NaN
 * points kept as in PCL's non-dense clouds).  *n_out = POINTS; PFX_ERR_CAPACITY (nothing
 * written) when it exceeds cap.  hdr (nullable) receives the header (viewpoint = the cloud's
 * sensor pose, which NARF's range image uses: keypoints.h:207-210). */
pfx_status pfx_pcd_load_xyz_dev(pfx_ctx* ctx, const char* path, float* d_x, float* d_y, float* d_z,
                                int64_t cap, int64_t* n_out, pfx_pcd_header* hdr);

/* ---- active-list keypoints ------------------------------------------ */
/* Keypoints::computeCloudResolution: mean distance of every finite point to its nearest other
 * point (FLANN kNN k = 2, the first hit being the point itself), 0 without such points. */
pfx_status pfx_cloud_resolution_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                                    double* resolution);
pfx_status pfx_cloud_resolution(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                double* resolution);
/* ISSKeypoint3D::compute (PCL 1.7 iss_3d.hpp): setSalientRadius, setNonMaxRadius,
 * setMinNeighbors, setThreshold21, setThreshold32 (keypoints.h:182-187; no border radius).
 * Keypoint cloud indices in ascending order into idx[0..cap); *n_out = their number
 * (PFX_ERR_CAPACITY, nothing written, when it exceeds cap).  third (nullable, n doubles): the
 * per-point third eigenvalue map (0 where the point is not a candidate).  A parameter that
 * PCL's initCompute rejects (radius, threshold or min neighbours <= 0) -> PFX_ERR_INVALID. */
pfx_status pfx_iss_keypoints_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                                 double salient_radius, double non_max_radius, int32_t min_neighbors,
                                 double threshold21, double threshold32, int32_t* d_idx, int64_t cap,
                                 int64_t* n_out, double* d_third);
pfx_status pfx_iss_keypoints(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                             double salient_radius, double non_max_radius, int32_t min_neighbors,
                             double threshold21, double threshold32, int32_t* idx, int64_t cap, int64_t* n_out,
                             double* third);

/* HarrisKeypoint3D (method HARRIS) + Keypoints::getKeypointsCloud: response over the normals of
 * the radius ball (NormalEstimation at the same radius, viewpoint 0), non-maximum suppression
 * above `threshold`, corner refinement (refine != 0, PCL's default), then every corner snapped
 * to its nearest cloud point when d2 < 0.0001.  idx[0..cap): those cloud indices in corner
 * (= index) order, *n_out their number (PFX_ERR_CAPACITY when it or the corner count exceeds
 * cap).  response (nullable, n floats): per-point intensity; corners (nullable, 3 * cap floats)
 * and n_corners (nullable): the refined corners; corner_idx (nullable, cap int32): the cloud index
 * of each corner's own point (PCL's output intensity = response[corner_idx]).  non_max == 0 ->
 * PFX_ERR_UNSUPPORTED (not used by the reference: keypoints.h:155). */
pfx_status pfx_harris3d_keypoints_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z, int64_t n,
                                      double radius, float threshold, int32_t non_max, int32_t refine,
                                      int32_t* d_idx, int64_t cap, int64_t* n_out, float* d_response,
                                      float* d_corners, int64_t* n_corners, int32_t* d_corner_idx);
pfx_status pfx_harris3d_keypoints(pfx_ctx* ctx, const float* x, const float* y, const float* z, int64_t n,
                                  double radius, float threshold, int32_t non_max, int32_t refine, int32_t* idx,
                                  int64_t cap, int64_t* n_out, float* response, float* corners, int64_t* n_corners,
                                  int32_t* corner_idx);

/* HarrisKeypoint6D (keypoints.h:164-176) + Keypoints::getKeypointsCloud: normals at the radius
 * (viewpoint 0), IntensityGradientEstimation at the radius over the colour intensity
 * float(299 r + 587 g + 114 b) * 0.001f (IntensityFieldAccessor<PointXYZRGB>), gradients of
 * squared length > 200 scaled to unit length and every other gradient (NaN ones included) set
 * to 0 (harris_6d.hpp's else branch), the 6x6 covariance of (normal, gradient) over the
 * radius ball and its fourth eigenvalue as the response (responseTomasi), non-maximum
 * suppression above `threshold`, corner refinement, snap -- outputs as the Harris3D entry.
 * rgb: one packed 0x00RRGGBB word per point (the bits of PointXYZRGB::rgb).  grad (nullable,
 * 3 n floats): the normalised gradient of every point (0 where PCL's normalisation zeroes it). */
pfx_status pfx_harris6d_keypoints_dev(pfx_ctx* ctx, const float* d_x, const float* d_y, const float* d_z,
                                      const uint32_t* d_rgb, int64_t n, double radius, float threshold,
                                      int32_t non_max, int32_t refine, int32_t* d_idx, int64_t cap, int64_t* n_out,
                                      float* d_response, float* d_corners, int64_t* n_corners, float* d_grad,
                                      int32_t* d_corner_idx);
pfx_status pfx_harris6d_keypoints(pfx_ctx* ctx, const float* x, const float* y, const float* z, const uint32_t* rgb,
                                  int64_t n, double radius, float threshold, int32_t non_max, int32_t refine,
                                  int32_t* idx, int64_t cap, int64_t* n_out, float* response, float* corners,
                                  int64_t* n_corners, float* grad, int32_t* corner_idx);

/* ---- RANSAC correspondence rejection --------------------------------- */
/* CorrespondenceRejectorSampleConsensus::getCorrespondences + getBestTransformation (host
 * arrays: the two keypoint clouds and the n correspondences index_query -> index_match):
 * setInlierThreshold(threshold), setMaximumIterations(max_iterations).  keep[0..*n_keep) =
 * positions of the remaining correspondences in input order (all of them when RANSAC finds no
 * model or fewer than 3 inliers, as PCL), transformation = the best model, row-major 4x4
 * (identity in those cases). */
pfx_status pfx_ransac_rejector(pfx_ctx* ctx, const float* sx, const float* sy, const float* sz, int64_t ns,
                               const float* tx, const float* ty, const float* tz, int64_t nt, const int32_t* query,
                               const int32_t* match, int64_t n, double threshold, int32_t max_iterations,
                               int32_t* keep, int64_t* n_keep, float* transformation);

/* ---- multi-GPU scan batch (SURVEY 8(e), configs[4]) ------------------------------------- */
/* Replaces the reference's per-scan loop for the (Narf, FPFH) pair (evaluation.cpp:272-852 over
 * Keypoints::compute, keypoints.h:199-231, and Features<FPFHSignature33>::compute,
 * features.h:175-196) for a C++ host with several GPUs in one process.  pfx_batch_create: the
 * devices (ordinals), two contexts and two streams per device, and an RCCL communicator over them
 * (ncclCommInitAll). */
typedef struct pfx_batch pfx_batch;
pfx_status pfx_batch_create(const int* devices, int n_devices, pfx_batch** out);
void pfx_batch_destroy(pfx_batch* batch);
const char* pfx_batch_last_error(const pfx_batch* batch);
/* n_scans host clouds (x[s], y[s], z[s], n[s] points; SoA float); scan s runs on device
 * s % n_devices: NARF keypoints (cam, params as pfx_narf_keypoints), the in-range pixel indices
 * mapped to cloud points (keypoints.h:229), normals of the whole cloud at normal_radius, FPFH at the
 * keypoints at feature_radius -- each device pipelines its scans over two streams.  The K_s x 33
 * descriptors and K_s cloud indices of every scan are gathered on the first device over RCCL and
 * copied out in scan order: rows[s] = K_s, scan s's rows start at sum_{t<s} K_t of desc
 * (cap_rows x 33) and idx (cap_rows).  Results equal the per-scan entry points bit for bit.
 * PFX_ERR_CAPACITY (rows filled in) when sum K_s > cap_rows. */
/* The batch's host-side plan (no device work; pfx_batch_narf_fpfh follows it): scan s runs on
 * device device_of_scan[s] = s % n_devices as that device's slot slot_of_scan[s] = s / n_devices
 * (its scans pipelined in slot order), and given each scan's descriptor rows K_s, its rows land at
 * row_offset[s] = sum_{t<s} K_t of the gathered output (row_offset has n_scans + 1 entries: the last
 * is the total).  Any output pointer may be NULL.  PFX_ERR_INVALID for n_scans < 0,
 * n_devices <= 0 or a negative K_s. */
pfx_status pfx_batch_plan(int n_scans, int n_devices, const int64_t* rows_per_scan, int32_t* device_of_scan,
                          int32_t* slot_of_scan, int64_t* row_offset);
pfx_status pfx_batch_narf_fpfh(pfx_batch* batch, int n_scans, const float* const* x, const float* const* y,
                               const float* const* z, const int64_t* n, const pfx_camera* cam,
                               const pfx_narf_params* params, double normal_radius, double feature_radius,
                               float* desc, int32_t* idx, int64_t cap_rows, int64_t* rows);

#ifdef __cplusplus
} /* extern "C" */
#endif
#endif /* PFX_H_ */
