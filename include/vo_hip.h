/*
 * vo_hip.h -- C-ABI of the MI355X (gfx950) back end for the feature-matching +
 * sliding-window bundle-adjustment hot path of cteufel13/VisualOdometry.
 *
 * Plain C: pointers, sizes and status codes only.  The Python host package
 * (visualodometry_amd/_lib.py) binds it with ctypes; INTEGRATION.md shows the
 * binding.  Every entry point is host-synchronous unless its name ends in
 * _async, and returns VO_OK (0) or a negative vo_status.
 *
 * Reference interfaces replaced (paths relative to the reference repo root):
 *   vo_match_knn2_ratio   <- FeatureFrontend.match_frames, SIFT branch,
 *                            src/modules/frontend.py:86-111
 *                            (cv2.BFMatcher(cv2.NORM_L2, crossCheck=False)
 *                             .knnMatch(des0, des1, k=2) at :34/:101 and the
 *                             Lowe ratio test at :103-109)
 *   vo_match_knn2         <- the knnMatch(k=2) call alone, frontend.py:101
 *   vo_triangulate        <- triangulate_points, src/modules/frontend.py:115-148
 *   vo_pnp_ransac         <- cv2.solvePnPRansac in the tracking step,
 *                            src/modules/vo.py:135-141
 *   vo_sift_detect_and_compute <- cv2.SIFT_create(...).detectAndCompute,
 *                            src/modules/frontend.py:27-32,55 (vo_sift_detect: its
 *                            extrema stage, for parity)
 *   vo_ba_*               <- new: the reference has no BA (pyceres/pycolmap
 *                            are declared in pyproject.toml:11-12 but never
 *                            imported).  Insertion point: the keyframe hook
 *                            VisualOdometry._create_keyframe,
 *                            src/modules/vo.py:252-288.  Projection model of
 *                            frontend.py:128-140, pose convention T_cw of
 *                            vo.py:260-261.
 */
#ifndef VO_HIP_H
#define VO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VO_ABI_VERSION 1

typedef enum {
  VO_OK = 0,
  VO_ERR_ARG = -1,      /* bad argument / unsupported shape */
  VO_ERR_HIP = -2,      /* HIP runtime error */
  VO_ERR_NOT_SPD = -3,  /* reduced camera system not positive definite */
  VO_ERR_RCCL = -4,     /* RCCL error */
  VO_ERR_NOMEM = -5,    /* device allocation failed */
  VO_ERR_STATE = -6,    /* call out of order (e.g. vo_ba_run before vo_ba_setup) */
  VO_ERR_NODEV = -7     /* no usable gfx950 device */
} vo_status;

typedef struct vo_ctx vo_ctx;

/* ---- library / context -------------------------------------------------- */
int vo_abi_version(void);
/* Thread-local message for the last failing call on this thread. */
const char* vo_last_error(void);
/* Creates a context bound to HIP device `device` with its own stream.  flags: 0.
 * Returns NULL on failure (vo_last_error() says why). */
vo_ctx* vo_create(int device, int flags);
void vo_destroy(vo_ctx* ctx);
/* The context's HIP stream (hipStream_t), for callers that enqueue on it. */
void* vo_stream(vo_ctx* ctx);
int vo_synchronize(vo_ctx* ctx);

/* Device buffers on the context's device (so callers need no second HIP
 * runtime in-process).  Copies are synchronous on the context stream. */
void* vo_device_alloc(vo_ctx* ctx, uint64_t bytes);
int vo_device_free(vo_ctx* ctx, void* ptr);
int vo_memcpy_h2d(vo_ctx* ctx, void* dst, const void* src, uint64_t bytes);
int vo_memcpy_d2h(vo_ctx* ctx, void* dst, const void* src, uint64_t bytes);

/* ---- descriptor matching (knn k=2 + Lowe ratio) --------------------------
 * des0: (n0, dim) float32 row-major, the "query" (previous keyframe) set;
 * des1: (n1, dim) float32 row-major, the "train" (current frame) set.
 * Semantics of OpenCV BFMatcher(NORM_L2).knnMatch(k=2) followed by the
 * reference ratio test:
 *   dist(i,j) = sqrtf(sum_d (a_id - b_jd)^2), the two nearest train rows per
 *   query under the order (dist, j) -- equal distances keep the lower j --,
 *   and pair (i, j1) is kept iff (double)dist1 < ratio * (double)dist2.
 *   Queries with n1 < 2 neighbours emit nothing.  Pairs are written in
 *   ascending query order as int32 (query, train).
 * Descriptors whose values are all integers in [0, 255] (OpenCV SIFT) take the
 * exact int8 MFMA path; any other values take the fp32 path, whose per-pair
 * distance is the k-ordered fmaf chain sum((a-b)^2).
 * out_pairs capacity: 2*n0 int32.  Empty inputs give *out_count = 0.        */
int vo_match_knn2_ratio(vo_ctx* ctx, const float* des0, int n0, const float* des1,
                        int n1, int dim, double ratio, int32_t* out_pairs,
                        int32_t* out_count);

/* Top-2 per query without the ratio test.  idx_out: (n0, 2) int32 (-1 when
 * fewer than 2 neighbours exist), dist_out: (n0, 2) float32 distances
 * (FLT_MAX where idx is -1). */
/* The same with a cached query side: the reference matches every frame against the same
 * keyframe (vo.py:64-65, des0 = the keyframe's descriptors), so a nonzero des0_tag keys a cache
 * of des0's device copy and packed rows.  A call whose (des0 pointer, n0, dim, des0_tag) equal
 * the cached ones skips des0's upload and packing; the caller gives a new tag whenever des0's
 * contents may have changed (0 = no cache).  Results are vo_match_knn2_ratio's. */
int vo_match_knn2_ratio_q(vo_ctx* ctx, const float* des0, int n0, uint64_t des0_tag, const float* des1,
                          int n1, int dim, double ratio, int32_t* out_pairs, int32_t* out_count);
/* Device-resident descriptors (pointers into this process's HIP device memory, e.g. the
 * feature dicts' GPU tensors, which frontend.py:66-67 moves to config.device): no descriptor
 * crosses PCIe, only the pairs come back to the host.  The caller orders the producer of the
 * descriptors before the call (e.g. synchronises its stream).  des0_tag as in _q. */
int vo_match_knn2_ratio_dev(vo_ctx* ctx, const float* d_des0, int n0, uint64_t des0_tag,
                            const float* d_des1, int n1, int dim, double ratio, int32_t* out_pairs,
                            int32_t* out_count);
int vo_match_knn2(vo_ctx* ctx, const float* des0, int n0, const float* des1, int n1,
                  int dim, int32_t* idx_out, float* dist_out);

/* Batched frame pairs, device pointers, enqueued on the context stream.
 * d_des0: (batch, n0, dim), d_des1: (batch, n1, dim) float32 on the device;
 * d_best: (batch, n0) int32 -- the train index kept for each query by the
 * ratio test, or -1.  Nothing is copied to the host. */
int vo_match_batch_async(vo_ctx* ctx, const float* d_des0, const float* d_des1,
                         int batch, int n0, int n1, int dim, double ratio,
                         int32_t* d_best);
/* Descriptor-kind hint for this context's later matcher calls (results never depend on
 * it; the device checks every call's values either way):
 *   VO_DESC_AUTO (0, default) launches both paths' kernels; a call runs the one its
 *     values need (a device-side flag) -- SIFT integers on the int8 MFMA sweep, other
 *     floats on the bf16 MFMA shortlist + exact re-rank;
 *   VO_DESC_SIFT (1): OpenCV SIFT integers expected (FeatureFrontend with the SIFT
 *     extractor, frontend.py:25-34): the float shortlist is not launched, and a call
 *     whose values are not 0..255 integers takes the exact fp32 sweep instead;
 *   VO_DESC_FLOAT (2): SuperPoint-like floats expected: no int8 pack, integer check, int8
 *     sweep or merge is launched; every call takes the bf16 shortlist + exact re-rank (exact
 *     for SIFT integers too), and a call with a non-finite value is answered by the re-rank
 *     kernel's exact scan (the exact fp32 sweep's result). */
#define VO_DESC_AUTO 0
#define VO_DESC_SIFT 1
#define VO_DESC_FLOAT 2
int vo_match_hint(vo_ctx* ctx, int kind);

/* ---- sliding-window bundle adjustment ------------------------------------ */
typedef struct {
  int32_t n_poses;   /* N cameras in the window                               */
  int32_t n_points;  /* L landmarks                                           */
  int32_t n_obs;     /* M observations                                        */
  int32_t n_fixed;   /* poses 0..n_fixed-1 are held fixed (gauge)             */
  double fx, fy, cx, cy;      /* pinhole K, no distortion (frontend.py:139)  */
  double lambda;              /* Levenberg damping added to every block (>=0) */
  const int32_t* point_ptr;   /* (n_points+1) CSR: obs of point p are
                                 point_ptr[p]..point_ptr[p+1]-1               */
  const int32_t* obs_cam;     /* (n_obs) camera index of each observation    */
  const float* obs_uv;        /* (n_obs, 2) pixel measurement (float32, as
                                 FeatureFrontend keypoints, frontend.py:59)   */
} vo_ba_problem;

/* Uploads the observation structure and builds the static execution plan
 * (landmark chunks, per-workgroup camera-pair windows, reduced-system profile).
 * Replaces any previous problem in this context.  *session_out receives the id of
 * this problem (unique in the process); every later vo_ba_* call on it passes that
 * id and fails with VO_ERR_STATE once another vo_ba_setup on the context has replaced
 * the problem (whose sizes the caller's buffers no longer match).  With a
 * communicator (vo_comm_init) every rank reaches the same verdict: a shard that
 * fails its checks on one rank is VO_ERR_ARG on all ranks. */
int vo_ba_setup(vo_ctx* ctx, const vo_ba_problem* prob, uint64_t* session_out);
/* Optional, once per context before its first keyframe (SlidingWindowBA's constructor, with
 * the window and map capacity of the VO configuration): pre-sizes every host and device
 * buffer a window of about n_poses cameras, n_points landmarks and n_obs observations needs
 * (page-locked plan images, device slabs and systems, kernel attributes), so the first
 * vo_ba_setup of the drive (vo.py:252-288, the first keyframe) allocates nothing and faults in
 * no page.  The context has no problem afterwards.  VO_ERR_STATE with a communicator of more
 * than one rank (call it before vo_comm_init). */
int vo_ba_reserve(vo_ctx* ctx, int n_poses, int n_points, int64_t n_obs, int n_fixed);
/* poses: (n_poses, 12) float64 = R_cw row-major (9) then t_cw (3);
 * points: (n_points, 3) float64 -- the sizes of the session's problem. */
int vo_ba_set_state(vo_ctx* ctx, uint64_t session, const double* poses, const double* points);
int vo_ba_get_state(vo_ctx* ctx, uint64_t session, double* poses, double* points);
/* Runs `iters` pure Gauss-Newton iterations (every step accepted) on the
 * device-resident state.  cost_out (iters+1 doubles, may be NULL): sum of
 * squared residuals before each iteration and after the last one.
 * Returns VO_ERR_NOT_SPD (state left at the last good iterate) if the reduced
 * camera system is not positive definite. */
int vo_ba_run(vo_ctx* ctx, uint64_t session, int iters, double* cost_out);
/* Same, enqueued on the context stream with no host synchronisation and no
 * cost read-back (for timing).  Errors surface at the next synchronous call. */
int vo_ba_run_async(vo_ctx* ctx, uint64_t session, int iters);
/* One GN iteration with the intermediate quantities exported (parity tests):
 * S_out: dense (6F, 6F) float64 reduced camera matrix with F = n_poses-n_fixed
 * (may be NULL), b_out: (6F), dc_out: (6F) pose update (may be NULL),
 * cost_out: 1 double.  The state is advanced by the step. */
int vo_ba_gn_step(vo_ctx* ctx, uint64_t session, double* S_out, double* b_out, double* dc_out,
                  double* cost_out);
/* One-call convenience: setup + set_state + run + get_state. */
int vo_ba_solve(vo_ctx* ctx, const vo_ba_problem* prob, double* poses, double* points,
                int iters, double* cost_out);

/* Static plan statistics (for DESIGN.md/bench): fills up to n int64 values:
 * [0] chunks [1] segments [2] slab blocks [3] reduced blocks [4] profile
 * blocks [5] track entries [6] bytes read+written per GN iteration
 * (algorithmic) [7] banded solver in use [8] first-camera groups and
 * [9] chunks the last vo_ba_setup took over from the previous window's plan (the slide)
 * [10] observations per segment the plan was packed for (1: the one-wave K1's plan);
 * [11..22] host time of the last vo_ba_setup's sections in nanoseconds: stream sync, landmark
 * order and track entries, segments, lists and chunk images, the rest of planning, plan checks,
 * image uploads, reduction profile, uploads, buffers, banded-solver tables, attributes.
 * Returns count written. */
int vo_ba_plan_stats(vo_ctx* ctx, int64_t* out, int n);

/* Diagnostic only: in a stamped build of the library (make EXTRA=-DVO_BA_STAMPS=1), K1
 * and K3 record s_memtime phase stamps; returns per-phase shader-cycle sums over
 * all workgroups of the last K1 launch (load, backsub, linobs, reduce, elim,
 * schur_pairs, write, schur_cams, then two unused slots) followed by the K3 phase
 * cycles.  With n < 0 it instead writes up to -n raw per-segment values (10 per
 * segment, the last two the absolute start and end time of that workgroup).
 * Returns the count written (0 when stamps are off). */
int vo_ba_debug_stamps(vo_ctx* ctx, uint64_t* out, int n);

/* ---- kernel timing (HIP events on the context stream) ---------------------
 * When enabled, every kernel launch is bracketed by hipEventRecord on the
 * context stream.  vo_profile_read synchronises and returns, per kernel id,
 * the summed duration in ms and the launch count, then clears the records.
 * Ids: 0 ba_lin (K1), 1 ba_reduce (K2), 2 ba_solve (K3), 3 match_pack,
 *      4 match_i8 (MFMA sweep), 5 match_f32, 6 match_merge, 7 triangulate,
 *      8 pnp_hyp, 9 pnp_score, 10 pnp_final, 11 sift_pyramid (all upsample, blur
 *      and downsample launches of one call), 12 sift_extrema (all octaves),
 *      13 sift_orient, 14 sift_select (sort keys, segmented sort, duplicate removal,
 *      retainBest, compaction), 15 sift_desc, 16 match_rerank (the float path's exact
 *      re-rank; before it had an id of its own it was timed under match_merge),
 *      17 pnp_decide, 18 pnp_hyp_tail, 19 pnp_score_tail (large batches: the replay after
 *      the first hypotheses of every frame, then the rest for the frames still looping). */
#define VO_PROFILE_KERNELS 20
int vo_profile_enable(vo_ctx* ctx, int on);
int vo_profile_read(vo_ctx* ctx, double* ms_out, int64_t* counts_out);

/* Host only: groups observations by landmark (the CSR that vo_ba_problem takes) from a
 * per-observation landmark index, as the keyframe window holds it (reference
 * src/modules/vo.py:252-288 builds the BA problem from the map's observation lists):
 * point_ptr (n_points + 1) and order (n_obs, stable: observations of one landmark keep the
 * caller's order), so that obs_cam[order] / obs_uv[order] are the problem's arrays.
 * With order == NULL it only checks that the observations are already grouped
 * (nondecreasing obs_pt, one pass) and fills point_ptr: returns 1 when they are not
 * (point_ptr then unspecified; call again with an order array).
 * VO_ERR_ARG if an index is out of range. */
int vo_ba_group_by_point(int n_points, int n_obs, const int32_t* obs_pt, int32_t* order, int32_t* point_ptr);
/* Host-only: builds the static plan of `prob` without a device (planner tests,
 * capacity checks).  Fills up to n int64 values: [0] chunks [1] segments
 * [2] slab blocks [3] profile blocks [4] track entries [5] max pairs in a chunk
 * [6] max window slots in a segment [7] max window cameras in a segment
 * [8] free poses F [9] widest profile row span (blocks) [10] two-sided K3
 * layout usable [11] its rows per side m [12] separator rows s [13] bottom rows. 
 * Returns the count written, or VO_ERR_ARG (vo_last_error() says why). */
int vo_ba_plan_probe(const vo_ba_problem* prob, int target_segments, int64_t* out, int n);
/* Host only: a 64-bit FNV-1a digest of every array of the static plan (chunks, segments,
 * slab layout, pair and camera lists, profile, K3 step tables) for `prob`; it pins the plan
 * (and so every kernel's summation order) across planner changes (tests/golden).  The plan is
 * packed for ceil(n_obs / target_segments) observations per segment. */
int vo_ba_plan_digest(const vo_ba_problem* prob, int target_segments, uint64_t* digest);

/* ---- triangulation ----------------------------------- */
/* Replaces triangulate_points (reference src/modules/frontend.py:115-148):
 * cv2.triangulatePoints(P1, P2, pts1.T, pts2.T) (DLT + SVD per point, float32
 * homogeneous output), dehomogenisation in float32, depth in camera 2 > min_depth
 * (:134-135) and the cv2.projectPoints reprojection error in image 2 <
 * max_reproj_err (:139-143).  P1, P2: 3x4 row-major K @ T_cw[:3, :] (as the caller
 * forms them, :127-128); T_cw2: 3x4 row-major [R | t]; K: 3x3 row-major.  pts1,
 * pts2: n x 2 float32.  Writes the float32 triangulation of EVERY point (n x 3) and
 * its mask (n bytes, 1 = kept); the reference returns pts3d[mask], mask.
 * Host buffers; synchronous. */
int vo_triangulate(vo_ctx* ctx, const double* P1, const double* P2, const double* T_cw2,
                   const double* K, const float* pts1, const float* pts2, int n,
                   double min_depth, double max_reproj_err, float* pts3d_out, uint8_t* mask_out);
/* Device-buffer variant (points and outputs in HBM; matrices on the host); enqueued
 * on the context stream, returns without synchronising. */
int vo_triangulate_async(vo_ctx* ctx, const double* P1, const double* P2, const double* T_cw2,
                         const double* K, const float* d_pts1, const float* d_pts2, int n,
                         double min_depth, double max_reproj_err, float* d_pts3d, uint8_t* d_mask);

/* ---- PnP-RANSAC ------------------------------------- */
/* Replaces cv2.solvePnPRansac(objpts, imgpts, K, None, reprojectionError=reproj_err,
 * iterationsCount=iterations, confidence=confidence) with SOLVEPNP_ITERATIVE, as the
 * tracking step calls it (reference src/modules/vo.py:135-141; map points and
 * keypoints are float32, vo.py:130-134).  objpts: n x 3 float32, imgpts: n x 2
 * float32, K: 3x3 row-major (no distortion).  RANSAC of OpenCV 4.12: cv::RNG((uint64)-1)
 * subsets of 5 points, EPnP per subset, float32 squared reprojection error <=
 * (float)(reproj_err^2), best = first model with the most inliers (> 4), the niters
 * update of RANSACUpdateNumIters; then a Levenberg-Marquardt refinement on the
 * inliers.  n == 5: EPnP on all points, all inliers.  n < 5: failure.
 * Outputs: rvec (3), tvec (3) (the pose T_cw, Rodrigues vector), mask (n bytes, 1 =
 * inlier of the best RANSAC model), *success_out = 1/0 (solvePnPRansac's retval).
 * Host buffers; synchronous. */
int vo_pnp_ransac(vo_ctx* ctx, const float* objpts, const float* imgpts, int n, const double* K,
                  int iterations, double reproj_err, double confidence, double* rvec_out,
                  double* tvec_out, uint8_t* mask_out, int32_t* success_out);
/* Batch of frames, points in HBM: frame f owns points offsets[f]..offsets[f+1]-1 of
 * d_objpts (total x 3) / d_imgpts (total x 2); offsets is a HOST array (batch+1,
 * offsets[0] = 0).  d_pose: (batch, 6) float64 = rvec, tvec; d_mask: (total) bytes;
 * d_status: (batch, 2) int32 = success, inlier count.  Enqueued on the context stream
 * (the subsets are regenerated and uploaded only when the frame layout changes). */
int vo_pnp_ransac_batch_async(vo_ctx* ctx, const float* d_objpts, const float* d_imgpts,
                              const int32_t* offsets, int batch, const double* K, int iterations,
                              double reproj_err, double confidence, double* d_pose, uint8_t* d_mask,
                              int32_t* d_status);
/* Host only: the RANSAC subsets the cv::RNG((uint64)-1) stream gives for `count` points
 * (iterations x 5 int32), for parity tests. */
int vo_pnp_subsets(int count, int iterations, int32_t* out);

/* ---- SIFT keypoint detection (the extrema stage) ----- */
/* Replaces the keypoint detection of cv2.SIFT_create(nfeatures, contrastThreshold,
 * edgeThreshold, sigma).detectAndCompute(gray, None) (reference
 * src/modules/frontend.py:27-32,55): doubled base image, Gaussian / DoG pyramid of
 * n_layers + 3 levels per octave, 26-neighbour extrema of DoG levels 1..n_layers beyond a
 * 5-pixel border with |v| > floor(0.5 contrast / n_layers * 255), adjustLocalExtrema
 * (sub-pixel fit, contrast and edge tests): the refined extrema before orientation
 * assignment (vo_sift_detect_and_compute below runs the whole call; this stage is exposed
 * for parity tests).  img: h x w uint8 row-major.
 * Per keypoint, in (octave, candidate level, row, column) order:
 *   kp_f[8]: x, y (input-image pixels), size, response, xi, 0, 0, 0
 *   kp_i[8]: image, OpenCV's octave word (first octave -1), candidate level, level,
 *            row, column (octave pixels, after refinement), candidate row, column.
 * *count receives the number found; at most `capacity` are written.  Host buffers. */
int vo_sift_detect(vo_ctx* ctx, const uint8_t* img, int h, int w, double contrast, double edge, double sigma,
                   int n_layers, int capacity, float* kp_f, int32_t* kp_i, int32_t* count);
/* Batch of equally sized images in HBM (d_imgs: batch x h x w uint8); keypoints of all
 * images appended to d_kpf / d_kpi in no particular order, *d_count (device int32) = total
 * found.  Enqueued on the context stream. */
int vo_sift_detect_batch_async(vo_ctx* ctx, const uint8_t* d_imgs, int batch, int h, int w, double contrast,
                               double edge, double sigma, int n_layers, int capacity, float* d_kpf,
                               int32_t* d_kpi, int32_t* d_count);
/* Parity/debug: the Gaussian (g_out) and DoG (d_out) pyramids of one image in the pitched
 * layout vo_sift_layout describes (g_floats / d_floats = capacities in floats). */
int vo_sift_pyramid(vo_ctx* ctx, const uint8_t* img, int h, int w, double sigma, int n_layers, float* g_out,
                    int64_t g_floats, float* d_out, int64_t d_floats);
/* ---- SIFT detectAndCompute ------------------------- */
/* One keypoint as cv::KeyPoint holds it after detectAndCompute: pt (x, y) and size in
 * input-image pixels, angle in degrees, response, OpenCV's octave word (first octave -1);
 * image = index in the batch. */
typedef struct vo_sift_keypoint {
  float x, y, size, angle, response;
  int32_t octave, image, reserved;
} vo_sift_keypoint;
/* Replaces cv2.SIFT_create(nfeatures, contrastThreshold, edgeThreshold, sigma)
 * .detectAndCompute(gray, None) (reference src/modules/frontend.py:27-32,55; OpenCV 4.12
 * sift.dispatch.cpp / sift.simd.hpp): the detection above, then calcOrientationHist (one
 * keypoint per histogram peak >= 0.8 max), KeyPointsFilter::removeDuplicatedSorted,
 * retainBest(nfeatures) when nfeatures > 0 (every keypoint whose response is >= the
 * nfeatures-th largest), and calcSIFTDescriptor (4 x 4 x 8, clipped at 0.2, scaled to 512,
 * saturate_cast<uchar>, stored as float).  Keypoints come out in removeDuplicatedSorted's
 * order (x asc, y asc, size desc, angle asc, response desc, octave desc); OpenCV's order
 * after retainBest is implementation-defined.  capacity is the size of
 * the output buffers; the oriented keypoints considered before the nfeatures cut start at
 * that capacity and the call retries with 4x more (up to 131072 per image) when they
 * overflow, as OpenCV has no such cap.  *count = the number written; VO_ERR_ARG when more
 * than 131072 oriented keypoints or more than capacity output keypoints.  Host buffers:
 * kps[capacity], desc[capacity x 128]. */
int vo_sift_detect_and_compute(vo_ctx* ctx, const uint8_t* img, int h, int w, int nfeatures, double contrast,
                               double edge, double sigma, int n_layers, int capacity, vo_sift_keypoint* kps,
                               float* desc, int32_t* count);
/* The same call with device outputs: FeatureFrontend.process_image's SIFT branch
 * (frontend.py:51-75) keeps only k.pt and the descriptors and moves both to config.device
 * (:66-67), so the drop-in writes them straight into the caller's GPU buffers (pointers of
 * this process's HIP runtime on the context's GPU, validated before any launch: VO_ERR_ARG
 * otherwise) and only *count crosses PCIe.  d_kps[capacity], d_desc[capacity x 128]. */
int vo_sift_detect_and_compute_dev(vo_ctx* ctx, const uint8_t* img, int h, int w, int nfeatures, double contrast,
                                   double edge, double sigma, int n_layers, int capacity, vo_sift_keypoint* d_kps,
                                   float* d_desc, int32_t* count);
/* Batch of equally sized images in HBM (d_imgs: batch x h x w uint8).  Per image b:
 * d_kps[b * capacity + i], d_desc[(b * capacity + i) * 128], i < d_counts[b]
 * (d_counts[b] < 0 when a capacity overflowed: -d_counts[b] is the working capacity that
 * image asked for, a lower bound when an earlier stage was cut short).  Enqueued on the
 * context stream. */
int vo_sift_detect_and_compute_batch_async(vo_ctx* ctx, const uint8_t* d_imgs, int batch, int h, int w,
                                           int nfeatures, double contrast, double edge, double sigma,
                                           int n_layers, int capacity, vo_sift_keypoint* d_kps, float* d_desc,
                                           int32_t* d_counts);
/* Host only: [n_octaves, G floats per image, DoG floats per image] then per octave
 * [h, w, pitch, G offset, DoG offset]; returns the count of values (writes up to n). */
int vo_sift_layout(int h, int w, int n_layers, int64_t* out, int n);

/* ---- multi-GPU (landmark sharding + RCCL all-reduce) --------------------- */
/* 128-byte RCCL unique id, created on rank 0 and shared by the caller. */
int vo_comm_unique_id(char out[128]);
/* Attaches an RCCL communicator to the context (one process per GPU).  After
 * this, vo_ba_setup expects THIS rank's landmark shard: every rank passes all
 * n_poses cameras but only its own points/observations; each GN iteration
 * all-reduces the partial reduced camera system (S, b, cost) before the
 * redundant dense pose solve, so all ranks hold identical poses. */
int vo_comm_init(vo_ctx* ctx, int nranks, int rank, const char id[128]);
/* (The test-only loopback communicator is declared in vo_hip_testing.h.) */

#ifdef __cplusplus
}
#endif
#endif /* VO_HIP_H */
