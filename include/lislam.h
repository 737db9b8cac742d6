/*
 * lislam — MI355X (gfx950) implementation of the per-scan hot path of
 * himhan34/Intensity_based_LiDAR_SLAM_for_me-: Ouster cloud -> range/intensity images ->
 * LOAM curvature features -> scan-to-scan kNN association -> point-to-line / point-to-plane
 * residual + Jacobian -> Ceres-semantics pose solve.
 *
 * C ABI (plain pointers and sizes; no C++ or torch types).  Every function returns an int
 * status (LISLAM_OK == 0); lislam_last_error() describes the last failure of a context.
 * A context owns one HIP device + stream and is not internally thread safe; use one context
 * per callback thread / GPU (the reference runs one ROS node per process, scanRegistration.cpp:738).
 *
 * Reference interfaces replaced (file:line in the reference tree):
 *   lislam_scan_registration  <- ImageHandler::cloud_handler        src/image_handler.h_ouster:103
 *                                + laserCloudHandler                   src/scanRegistration.cpp:189-658
 *   lislam_odom_step          <- laserOdometry main-loop body          src/laserOdometry.cpp:313-808
 *   lislam_batch_*            <- the same two stages for a batch of scans resident in HBM
 *                                (independent scans / chains of scans)
 *   lislam_eval_factors       <- ceres::CostFunction::Evaluate of LidarEdgeFactor /
 *                                LidarPlaneFactor / LidarPlaneNormFactor
 *                                                                      src/lidarFeaturePointsFunction.hpp:143-293
 *   lislam_map_*              <- KD_TREE Build / Add_Points / Nearest_Search / size / flatten
 *                                                                      src/ikd-Tree/ikd_Tree.h:256-279
 *   lislam_map_associate      <- 5-NN line / plane association        src/laserMapping.cpp:668-796,
 *                                                                      src/mapOptimization.cpp:376-429
 *   lislam_normal_equations / lislam_pose_solve
 *                             <- ceres::Solve(DENSE_QR) of those blocks (laserMapping.cpp:836-845,
 *                                mapOptimization.cpp:433-442)
 *   lislam_voxel_grid         <- pcl::VoxelGrid::filter                (scanRegistration.cpp:583-586,
 *                                laserMapping.cpp:608-616, mapOptimization.cpp:368-370)
 *   lislam_mapopt_step        <- mapOptimization::mapOptimizationCallback ground-map stage
 *                                                                      src/mapOptimization.cpp:99-479
 *   lislam_laser_mapping      <- laserMapping::process optimization    src/laserMapping.cpp:620-850
 *   lislam_lmap_*             <- laserMapping::process with its cube map src/laserMapping.cpp:319-1002
 *   lislam_batch_intensity_odometry / lislam_intensity_tracker_*
 *                             <- feature_tracker::detectfeatures       src/intensity_feature_tracker.cpp:597-738
 *   lislam_ground_extract / lislam_batch_ground
 *                             <- ImageHandler::groundPlaneExtraction   src/image_handler.h_ouster:41-100
 *   lislam_batch_upload / lislam_batch_download_cloud
 *                             <- pcl::fromROSMsg / toROSMsg            src/image_handler.h_ouster:105-106,
 *                                                                      src/scanRegistration.cpp:592-642
 *   lislam_loop_icp           <- loopClosureThread's USE_ICP block     src/intensity_feature_tracker.cpp:217-366
 *   lislam_odom_fuse          <- odomHandler callback                 src/odom_handler_node.cpp:44-132
 */
#ifndef LISLAM_H_
#define LISLAM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LISLAM_OK 0
#define LISLAM_ERR_ARG (-1)      /* invalid argument / unsupported configuration */
#define LISLAM_ERR_DEVICE (-2)   /* HIP runtime error */
#define LISLAM_ERR_CAPACITY (-3) /* caller buffer too small */
#define LISLAM_ERR_STATE (-4)    /* call out of order */

typedef struct lislam_ctx lislam_ctx;
typedef struct lislam_batch lislam_batch;
typedef struct lislam_odom lislam_odom;

/* Parameters the reference reads from the ROS parameter server / compile-time constants. */
typedef struct {
  int32_t n_scans;        /* N_SCANS = image_height (scanRegistration.cpp:692; spot.yaml:8): 16/32/64/128 */
  int32_t width;          /* image_width (spot.yaml:7) */
  float min_range;        /* MINIMUM_RANGE = remove_radius (scanRegistration.cpp:695; spot.yaml:49) */
  int32_t max_iterations; /* ceres max_num_iterations of the odometry solve (laserOdometry.cpp:707) */
  int32_t want_images;    /* materialize image_range / image_intensity / cloud_track (a1) */
} lislam_config;

/* Field layout of a sensor_msgs/PointCloud2 point (fromROSMsg, image_handler.h_ouster:106). */
typedef struct {
  uint32_t point_step; /* bytes per point (Ouster: 48; PCL PointXYZI: 32; packed xyzI: 16) */
  uint32_t off_x, off_y, off_z, off_intensity; /* byte offsets of the float32 fields */
} lislam_point_layout;

/* Features of one scan as published by scanRegistration (scanRegistration.cpp:592-642).
 * Points are float32 (x, y, z, intensity) quadruples; intensity = scanID + 0.1 * relTime.
 * Capacities are in points; on return n_* hold the counts.  Null pointers are skipped. */
typedef struct {
  float* laser_cloud; int32_t cap_laser_cloud; int32_t n_laser_cloud;   /* /velodyne_cloud_2 */
  float* sharp; int32_t cap_sharp; int32_t n_sharp;                     /* /laser_cloud_sharp */
  float* less_sharp; int32_t cap_less_sharp; int32_t n_less_sharp;      /* /laser_cloud_less_sharp */
  float* flat; int32_t cap_flat; int32_t n_flat;                        /* /laser_cloud_flat */
  float* less_flat; int32_t cap_less_flat; int32_t n_less_flat;         /* /laser_cloud_less_flat */
  uint8_t* image_range; uint8_t* image_intensity;                       /* H*W each (cloud_handler) */
  float* cloud_track;                                                   /* H*W*4 (cloud_handler) */
} lislam_scan_out;

/* One frame of features as consumed by laserOdometry (laserOdometry.cpp:336-377). */
typedef struct {
  const float* sharp; int32_t n_sharp;
  const float* less_sharp; int32_t n_less_sharp;
  const float* flat; int32_t n_flat;
  const float* less_flat; int32_t n_less_flat;
} lislam_frame;

/* ---------------------------------------------------------------- context */
int lislam_ctx_create(const lislam_config* cfg, int32_t device, lislam_ctx** out);
int lislam_ctx_destroy(lislam_ctx* ctx);
const char* lislam_last_error(const lislam_ctx* ctx);
int lislam_synchronize(lislam_ctx* ctx);
/* Use an external hipStream_t (e.g. a torch stream) instead of the context's own. */
int lislam_set_stream(lislam_ctx* ctx, void* hip_stream);
int lislam_get_stream(lislam_ctx* ctx, void** hip_stream);

/* ---------------------------------------------------------------- single scan (drop-in) */
/* laserCloudHandler: one organized cloud of n_scans*width points (host memory) -> features. */
int lislam_scan_registration(lislam_ctx* ctx, const void* points, const lislam_point_layout* layout,
                             lislam_scan_out* out);

/* laserOdometry node: state = last corner/surf clouds, para_q/para_t, q_w_curr/t_w_curr. */
int lislam_odom_create(lislam_ctx* ctx, lislam_odom** out);
int lislam_odom_destroy(lislam_odom* od);
/* Process one frame.  para_out[7] = (q_last_curr x,y,z,w, t_last_curr), pose_out[7] = (q_w_curr,
 * t_w_curr), stats_out[8] = corner/plane correspondences of the two outer passes, LM iterations
 * of each pass, termination of each pass (0 max-iterations, 1 convergence, 2 failure). */
int lislam_odom_step(lislam_odom* od, const lislam_frame* frame, double* para_out, double* pose_out,
                     int32_t* stats_out);
/* The reference's default gating (laserOdometry.cpp:403-417): the frame is associated and
 * optimized only when use_aloam != 0 (its sharp cloud's frame_id == "skip_intensity"); otherwise
 * para_q/para_t carry over and the pose accumulates them (:716-717). */
int lislam_odom_step_gated(lislam_odom* od, const lislam_frame* frame, int32_t use_aloam, double* para_out,
                           double* pose_out, int32_t* stats_out);

/* ---------------------------------------------------------------- batch (device resident) */
int lislam_batch_create(lislam_ctx* ctx, int32_t max_scans, lislam_batch** out);
int lislam_batch_destroy(lislam_batch* b);
/* Copy n_scans clouds from host memory (contiguous, n_scans*n_scans_cfg*width points). */
int lislam_batch_upload(lislam_batch* b, const void* points, int32_t n_scans, const lislam_point_layout* layout);
/* The same ingest without blocking the host: the bytes go to the device on the batch's copy
 * stream in chunks of 16 scans, and each chunk is parsed (k_unpack_layout) on the context stream
 * as soon as it has landed, after whatever the context stream was doing before (the previous
 * batch's extraction still reading the input buffer).  So the transfer of the next batch overlaps
 * the processing of the current one.  `points` must stay valid and unchanged until the context
 * stream has passed the upload (lislam_synchronize, or any download); pinned memory makes the
 * copies asynchronous. */
int lislam_batch_upload_async(lislam_batch* b, const void* points, int32_t n_scans, const lislam_point_layout* layout);
/* Device pointer of the packed float4 (x,y,z,intensity) input buffer [max_scans][H*W]. */
int lislam_batch_input_device_ptr(lislam_batch* b, void** dptr);
/* a1..a7 for scans [0, n_scans) of the batch. */
int lislam_batch_extract(lislam_batch* b, int32_t n_scans);
/* a12..a18 for scans [0, n_scans): ceil((n_scans-1)/chain_len) independent chains, chain c is a
 * fresh laserOdometry node over scans [c*chain_len, min((c+1)*chain_len, n_scans-1)]. */
int lislam_batch_odometry(lislam_batch* b, int32_t n_scans, int32_t chain_len);
/* The reference's default gating (laserOdometry.cpp:403-417): pair (k-1, k) is associated and
 * optimized only when use_aloam[k] != 0 — the sharp cloud's frame_id is "skip_intensity", i.e.
 * the intensity tracker skipped scan k (scanRegistration.cpp:603-609; LISLAM_OUT_ORB_STATS[0] ==
 * 0).  Otherwise para keeps the previous estimate and the pose accumulates it (:716-717).
 * use_aloam[n_scans]: host or device memory; a host array is copied before the call returns, so
 * it may be freed then.  lislam_batch_odometry = every use_aloam set. */
int lislam_batch_odometry_gated(lislam_batch* b, int32_t n_scans, int32_t chain_len, const int32_t* use_aloam);
/* Enable per-kernel HIP-event timing: every following extract / odometry call records events on
 * the stream (no host synchronization). */
int lislam_batch_set_timing(lislam_batch* b, int32_t enable);
/* Kernels timed by lislam_batch_kernel_times, in this order. */
#define LISLAM_NUM_KERNELS 7 /* k_scan_front, k_scan_lines, k_scan_compact, k_target_index,
                                k_odom_assoc, k_odom_lm (the latter includes k_odom_init),
                                k_odom_chain (the persistent engine of few long chains: association
                                and solve of every round in one launch) */
/* Synchronize, then return, over the calls recorded since the previous read, the average ms
 * per call spent in each kernel (ms_per_call[LISLAM_NUM_KERNELS]) and the launches per call of
 * each kernel (launches_per_call[LISLAM_NUM_KERNELS], may be null); calls[2] (may be null) =
 * extract / odometry calls averaged.  Clears the record.  (LISLAM_NUM_KERNELS was 6 before the
 * chain engine: size the arrays from the macro.) */
int lislam_batch_kernel_times(lislam_batch* b, float* ms_per_call, int32_t* launches_per_call, int32_t* calls);

#define LISLAM_OUT_IMAGE_RANGE 0     /* uint8  [H*W] */
#define LISLAM_OUT_IMAGE_INTENSITY 1 /* uint8  [H*W] */
#define LISLAM_OUT_CLOUD_TRACK 2     /* float4 [H*W] */
#define LISLAM_OUT_LASER_CLOUD 3     /* float4 [n]   */
#define LISLAM_OUT_CURVATURE 4       /* float  [n]   */
#define LISLAM_OUT_LABEL 5           /* int8   [n]   */
#define LISLAM_OUT_LINE_OFFSETS 6    /* int32  [H+1] */
#define LISLAM_OUT_SHARP 7           /* float4 [n]   */
#define LISLAM_OUT_LESS_SHARP 8      /* float4 [n]   */
#define LISLAM_OUT_FLAT 9            /* float4 [n]   */
#define LISLAM_OUT_LESS_FLAT 10      /* float4 [n]   */
#define LISLAM_OUT_PARA 11           /* double [7]   */
#define LISLAM_OUT_POSE 12           /* double [7]   */
#define LISLAM_OUT_STATS 13          /* int32  [8]   */
#define LISLAM_OUT_ORB_T 14          /* double [7]   T_s2s of pair (scan-1, scan) (q x,y,z,w, t) */
#define LISLAM_OUT_ORB_STATS 15      /* int32  [8]   see lislam_intensity_tracker_step */
#define LISLAM_OUT_ORB_KEYPOINTS 16  /* float  [n][6] of the nfeatures detection */
#define LISLAM_OUT_ORB_POINTS 17     /* float4 [n]   their cloud_track points */
#define LISLAM_OUT_ORB_DESCRIPTORS 18 /* uint8 [n][32] */
#define LISLAM_OUT_GROUND 19         /* float4 [n]   ground cloud x, y, z, 1 (lislam_batch_ground) */
#define LISLAM_OUT_GROUND_PLANE 20   /* float  [4]   segmented plane A, B, C, D */
#define LISLAM_OUT_GROUND_INFO 21    /* int32  [4]   status (1 ground, 0 plane rejected by the n.z >
                                        cos 15 deg test, -1 < 3 candidates, -2 no model, -3 sampling
                                        beyond the device map), RANSAC iterations, best inliers,
                                        refit inliers */
/* Copy one output of one scan to host memory; cap/n count elements of the listed type.  dst null:
 * only *n is set (the element count). */
int lislam_batch_download(lislam_batch* b, int32_t what, int32_t scan, void* dst, int32_t cap, int32_t* n);
/* toROSMsg of a point-cloud output (laser cloud, the four feature clouds, cloud_track, ground,
 * ORB points; scanRegistration.cpp:592-642): cap / n points written into dst in the given
 * PointCloud2 layout (e.g. PCL PointXYZI: point_step 32, x 0, y 4, z 8, intensity 16), packed on
 * the device; bytes outside the four fields are zero.  lislam_batch_upload parses any layout on
 * the device the same way (fromROSMsg). */
int lislam_batch_download_cloud(lislam_batch* b, int32_t what, int32_t scan, void* dst, const lislam_point_layout* layout,
                                int32_t cap, int32_t* n);

/* Odometry schedule of lislam_batch_odometry (results are the same): LISLAM_ENGINE_OFF issues one
 * association and one solve launch per round (chains advance together, one workgroup per chain's
 * solve); LISLAM_ENGINE_ON runs every round of every chain inside ONE persistent launch
 * (k_odom_chain: a device ticket queue orders the association and solve items, no host round trip
 * between scans) — the schedule of few long chains, e.g. the reference's single continuous chain;
 * LISLAM_ENGINE_AUTO (default) picks ON for at most 4 chains. */
#define LISLAM_ENGINE_OFF 0
#define LISLAM_ENGINE_AUTO 1
#define LISLAM_ENGINE_ON 2
int lislam_set_odometry_schedule(lislam_ctx* ctx, int32_t mode);
/* The chain engine's shape for this context's launches (results are the same).
 * queries_per_wave: 1 = one association query per wavefront (64-lane searches: the shortest chain,
 * but one engine's association waves fill half of every CU); 2, 3 = that many 64-lane queries one
 * after another per wavefront; 4 = four at once, one per 16-lane row.  Above 1 each chain is
 * slower but an engine holds a fraction of the waves, so several engines and the next batches'
 * extraction share the GPU.  0 = keep.  depth = engines in flight per device when a launch of this
 * context enters the device's queue (1..6; a launch waits for the one `depth` launches before it);
 * 0 = keep.  Latency (one sequence at a time): 1 / 1, the default (one engine in flight, its item
 * workgroups 12 waves: a pass's queries in one round).  Throughput (several pipelined
 * contexts, e.g. bench.py): 3 / 5.  LISLAM_ENGINE_QPW / LISLAM_ENGINE_DEPTH seed a new context's
 * shape. */
int lislam_set_engine_shape(lislam_ctx* ctx, int32_t queries_per_wave, int32_t depth);
/* status = the number of engine launches of the batch that gave up since the previous status call
 * (one of the engine's bounded device waits expired, e.g. when its two launches could not run
 * together).  An aborted launch is recovered, not refused: the next call that reads or replaces the
 * batch's outputs waits for the engine on the host and re-runs that launch's chains on the
 * per-round schedule (LISLAM_ENGINE_OFF, no device waits) before it goes on, so the outputs are
 * always those of a complete schedule.  Those calls ("settling" calls): lislam_batch_extract,
 * lislam_batch_odometry(_gated), lislam_batch_download, lislam_batch_download_cloud,
 * lislam_batch_kernel_times, lislam_batch_odometry_status / _engine / _abort_code,
 * lislam_batch_mapopt(_corner), lislam_odom_step(_gated) and lislam_synchronize.  The calls that
 * touch only the input points or the ORB / ground stages do not wait for the engine:
 * lislam_batch_upload(_async), lislam_batch_input_device_ptr, lislam_batch_set_timing,
 * lislam_batch_ground, lislam_batch_intensity_odometry.  Reading the count clears it. */
int lislam_batch_odometry_status(lislam_batch* b, int32_t* status);
/* Which schedule the batch's last odometry call ran: 0 per-round launches, 1 the single-launch
 * engine (k_odom_chain), 2 the split engine (k_odom_roles + k_odom_items on CU-masked streams). */
int lislam_batch_odometry_engine(lislam_batch* b, int32_t* kind);
/* The error word of the batch's last aborted engine launch (0: none since the batch's creation):
 * which bounded wait gave up — 1 an association item waiting for the previous pass's items, 2 an
 * item waiting for its pass's pose, 3 a solve role waiting for its pass's items, 4 / 5 the
 * progressive gather's poll / loads, 0x57xx an overflow query out of range. */
int lislam_batch_odometry_abort_code(lislam_batch* b, int32_t* code);
/* The CU-masked streams the library holds on a device (*masked_queues).  Each is a hardware queue
 * of its own, and past about 20 of them in one process every launch slows: a context holds one
 * (its stream, which its ORB front end shares), the chain engine's 4 stream pairs and the per-round
 * schedule's group stream belong to the device (shared by all batches). */
int lislam_device_queue_count(int32_t device, int32_t* masked_queues);

/* Order of equal sort keys in the two std::sort calls of the feature extraction:
 * - each segment's sort by curvature (scanRegistration.cpp:445), which decides which of two
 *   points of equal curvature the sharp / flat walks (:450-568) reach first;
 * - the scan-line VoxelGrid(0.2) of the less-flat cloud (a7, :583-586): PCL 1.10's VoxelGrid
 *   sorts (voxel, point) pairs with std::sort by voxel alone, so a voxel's points are summed in
 *   the order libstdc++'s introsort leaves them.
 * LISLAM_TIES_REFERENCE (the default) replays libstdc++'s order exactly in both (bit-exact
 * selections and centroids); LISLAM_TIES_INDEX breaks ties by point index (faster; centroids
 * differ by float rounding, poses by up to 1e-4 on the bench data, tests/test_oracle.py).
 * Applies to later extractions of ctx. */
#define LISLAM_TIES_REFERENCE 0
#define LISLAM_TIES_INDEX 1
int lislam_set_tie_order(lislam_ctx* ctx, int32_t order);

/* ---------------------------------------------------------------- cost functors */
/* Evaluate n residual blocks at (q[4] = x,y,z,w, t[3]) on the GPU.  kind[i]: 0 LidarEdgeFactor
 * (pts: curr, a, b), 1 LidarPlaneFactor (curr, j, l, m), 2 LidarPlaneNormFactor (curr, n, d);
 * pts holds 12 doubles per block.  Outputs residuals[3n] (unused entries 0) and local-
 * parameterization Jacobians jac[3n x 6] (d/d delta-theta, d/d t), both optional. */
int lislam_eval_factors(lislam_ctx* ctx, int32_t n, const int32_t* kind, const double* pts, const double* q,
                        const double* t, double* residuals, double* jac);
/* ceres::AutoDiffCostFunction<F, R, 4, 3>::Evaluate of the reference functors on the GPU: the
 * Jacobians w.r.t. the raw parameter blocks, jac_q[n][3][4] (q x, y, z, w) and jac_t[n][3][3],
 * as Ceres' Jet differentiation gives them (lidarFeaturePointsFunction.hpp:29,49-54,157,183-190,
 * 208,228-234,252,282-288).  kind[i]: 0 LidarEdgeFactor (pts: curr, a, b), 1 LidarPlaneFactor
 * (curr, j, l, m), 2 LidarPlaneNormFactor (curr, n, d), 3 front_end_residual /
 * FeatureMatchingResidual (curr / src, dst; :21-99), 4 LidarGroundPlaneNormFactor (curr, n, d;
 * q block only, jac_t rows zero; :101-141), 5 LidarEdgeFactor with s != 1 (curr, a, b, s) and
 * 6 LidarPlaneFactor with s != 1 (curr, j, unit normal, s): DISTORTION 1, Identity.slerp(s, q)
 * and s t (:155-162,255-262).  Residual rows past the block's size are zero.  All
 * pointers may be host or device memory; outputs are optional.  include/lislam_factors.h wraps
 * this behind the reference's functor structs and their Create(). */
int lislam_eval_factors_raw(lislam_ctx* ctx, int32_t n, const int32_t* kind, const double* pts, const double* q,
                            const double* t, double* residuals, double* jac_q, double* jac_t);

/* ---------------------------------------------------------------- ORB intensity front end (a8-a11) */
/* cv::ORB::create(nfeatures, 1.2f, 8, 1) detect (with the feature_tracker MASK, H x W u8, 0 =
 * blocked; null = none) + extractPointsAndFilterZeroValue + compute on one intensity image
 * (intensity_feature_tracker.cpp:609-628, :1071-1099).  kp[n][6] = x, y, size, angle (deg),
 * response, octave; desc[n][32]; p3d[n][4] = the cloud_track point (x, y, z, 0).  cloud_track is
 * the organized H*W float4 cloud of ImageHandler::cloud_handler.  Host or device pointers. */
int lislam_orb_detect(lislam_ctx* ctx, const uint8_t* image, const float* cloud_track, const uint8_t* mask, int32_t H,
                      int32_t W, int32_t nfeatures, float* kp, uint8_t* desc, float* p3d, int32_t cap, int32_t* n);
/* BFMatcher(NORM_HAMMING, crossCheck=true).match(query, train) (:631): matches[m][3] = query,
 * train, distance in query order (capacity nq). */
int lislam_orb_match(lislam_ctx* ctx, const uint8_t* qdesc, int32_t nq, const uint8_t* tdesc, int32_t nt,
                     int32_t* matches, int32_t* n_matches);
/* feature_tracker::detectfeatures (intensity_feature_tracker.cpp:597-738): one frame per step,
 * state = the previous frame.  T_s2s[7] = (q x,y,z,w, t) of p2p_calculateRandT (identity when
 * the frame is skipped); stats[8] = good (1) / skipped (0) / first frame (-1), re-detected,
 * keypoints, matches, good matches, LM iterations, LM termination, previous keypoints. */
typedef struct lislam_intensity_tracker lislam_intensity_tracker;
int lislam_intensity_tracker_create(lislam_ctx* ctx, int32_t H, int32_t W, int32_t nfeatures, const uint8_t* mask,
                                    lislam_intensity_tracker** out);
int lislam_intensity_tracker_destroy(lislam_intensity_tracker* t);
int lislam_intensity_tracker_step(lislam_intensity_tracker* t, const uint8_t* image, const float* cloud_track,
                                  double* T_s2s, int32_t* stats);
/* detectfeatures over scans [0, n_scans) of a batch (its a1 images, want_images = 1): scan k is
 * matched against scan k-1 exactly as the tracker would; outputs LISLAM_OUT_ORB_*.  Asynchronous:
 * it returns once its work is queued (on a side stream the context stream then waits for); the
 * sequential re-detection rule (intensity_feature_tracker.cpp:652-687) is decided on the device in
 * LISLAM_ORB_ROUNDS passes (default 1).  Reading an ORB output first checks that the device
 * decision converged, and redoes the batch with host-decided rounds if it did not. */
int lislam_batch_intensity_odometry(lislam_batch* b, int32_t n_scans, int32_t nfeatures, const uint8_t* mask);
/* The last lislam_batch_intensity_odometry's cascade, after its outputs were read: info[0] = 1
 * device-decided and converged, 0 redone with host rounds, -1 host rounds from the start
 * (LISLAM_ORB_HOST_CASCADE=1 or fewer than 2 scans); info[1] = device decision passes. */
int lislam_batch_orb_cascade_info(lislam_batch* b, int32_t* info);

/* ---- ground plane (ImageHandler::groundPlaneExtraction, src/image_handler.h_ouster:41-100):
 * z-band screening [-2, -0.45], PCL SACSegmentation(SACMODEL_PLANE, SAC_RANSAC, 0.01, optimized
 * coefficients) with PCL 1.10's single-thread sampling sequence, the n.z > cos(15 deg) test and
 * the points within 0.03 m of the plane with z < 0 — the GroundPointOut cloud mapOptimization
 * merges with the less-flat cloud (mapOptimization.cpp:136,148).  Outputs LISLAM_OUT_GROUND*. */
int lislam_batch_ground(lislam_batch* b, int32_t n_scans);
/* One organized cloud (the context's n_scans x width, any point layout): ground cloud out[cap][4]
 * (x, y, z, 1), *n_out, plane[4] (A, B, C, D) and info[4] as LISLAM_OUT_GROUND_INFO (each
 * nullable).  Replaces ImageHandler::groundPlaneExtraction's body. */
int lislam_ground_extract(lislam_ctx* ctx, const void* points, const lislam_point_layout* layout, float* out,
                          int32_t cap, int32_t* n_out, float* plane, int32_t* info);

/* ---------------------------------------------------------------- scan-to-map (a19-a21) */
/* A device-resident point map with the semantics of the vendored ikd-Tree
 * (src/ikd-Tree/ikd_Tree.h:256-279): Build, Add_Points with box downsampling, exact k-NN
 * Nearest_Search, and the mapping stages that consume it.  Points are float32 x, y, z; input
 * arrays are n points of `stride` floats (3 = PointXYZ packed, 4 = PointXYZ / PointXYZI as PCL
 * stores them).  Pointers may be host or device memory (copied with hipMemcpyDefault). */
typedef struct lislam_map lislam_map;

typedef struct {
  float downsample_size; /* ikd KD_TREE(delete_param, balance_param, box_length): 0.4 ground map,
                            0.8 corner map (mapOptimization.cpp:504-505) */
  float cell_size;       /* edge of the hash-grid cells the search walks (0: downsample_size);
                            a search accelerator only, results do not depend on it */
} lislam_map_config;

int lislam_map_create(lislam_ctx* ctx, const lislam_map_config* cfg, lislam_map** out);
int lislam_map_destroy(lislam_map* m);
/* KD_TREE::Build (ikd_Tree.cpp:470-492): the map holds exactly these points (ids 0..n-1). */
int lislam_map_build(lislam_map* m, const float* pts, int64_t n, int32_t stride);
/* KD_TREE::Add_Points (ikd_Tree.cpp:569-706).  downsample_on: per box of edge downsample_size
 * only the point nearest the box centre survives, as the reference's sequential loop leaves it.
 * Inputs take ids next_id .. next_id+n-1.  n_added (nullable) = inputs that entered the map. */
int lislam_map_add_points(lislam_map* m, const float* pts, int64_t n, int32_t stride, int32_t downsample_on,
                          int64_t* n_added);
/* KD_TREE::size / validnum. */
int lislam_map_size(lislam_map* m, int64_t* n);
/* KD_TREE::flatten / PCL_Storage: live points as (x, y, z, id bits), storage order. */
int lislam_map_points(lislam_map* m, float* out_xyzi, int64_t cap, int64_t* n);
/* KD_TREE::Nearest_Search (ikd_Tree.cpp:494-547) for n queries: up to k (<= 8) points with
 * squared distance <= max_dist^2 (max_dist <= 0: unbounded), ascending (squared float distance,
 * id).  out_pts[n][k][4] = x, y, z, id bits; out_d2[n][k]; out_found[n] (all nullable). */
int lislam_map_nearest_search(lislam_map* m, const float* queries, int32_t n, int32_t stride, int32_t k,
                              float max_dist, float* out_pts, float* out_d2, int32_t* out_found);

#define LISLAM_MATCH_LINE 0  /* laserMapping corner: 5-NN, PCA line, LidarEdgeFactor (laserMapping.cpp:668-723) */
#define LISLAM_MATCH_PLANE 1 /* 5-NN, QR plane, LidarPlaneNormFactor (laserMapping.cpp:744-796,
                                mapOptimization.cpp:376-429) */
/* Associate n sensor-frame points at pose x = (q x,y,z,w, t) against the map: out_rec[n][9]
 * (line: curr, a, b; plane: curr, n, d, 0, 0) and out_kind[n] (0 edge, 2 plane-norm, -1 none). */
int lislam_map_associate(lislam_map* m, int32_t kind, const float* pts, int32_t n, int32_t stride, const double* x,
                         double* out_rec, int32_t* out_kind);
/* Cost, J^T J (upper, 21) and J^T r (6) = 28 doubles of n records (kinds 0 edge / 1 plane /
 * 2 plane-norm, -1 skipped) under HuberLoss(0.1) at x (SURVEY.md §8(b) eval_normal_eq). */
int lislam_normal_equations(lislam_ctx* ctx, const double* rec, const int32_t* kind, int32_t n, const double* x,
                            double* out28);
/* ceres::Solve (DENSE_QR, max_iterations) of n records at x (in/out, 7 doubles).
 * summary[4] (nullable) = iterations, termination (0 no-convergence, 1 convergence, 2 failure),
 * edge blocks, plane blocks. */
int lislam_pose_solve(lislam_ctx* ctx, const double* rec, const int32_t* kind, int32_t n, double* x,
                      int32_t max_iterations, int32_t* summary);
/* pcl::VoxelGrid (leaf) of n points (x, y, z, intensity, stride 4): per-voxel centroid of all four
 * fields, output ordered by voxel index; points of a voxel summed in input order.  out holds up
 * to n points. */
int lislam_voxel_grid(lislam_ctx* ctx, const float* pts, int32_t n, float leaf, float* out, int32_t* n_out);

/* mapOptimization::mapOptimizationCallback ground-map stage (mapOptimization.cpp:99-479 without
 * the ORB / keyframe-image logic): ground = GroundPointOut (sensor frame, stride 4), odom =
 * q_wodom_curr, t_wodom_curr (7); state = q_wmap_wodom, t_wmap_wodom (7, in/out).  Empty map:
 * Build with the transformed cloud.  Otherwise VoxelGrid(0.8), plane association, Ceres(10 it),
 * transformUpdate on CONVERGENCE, Add_Points(downsample) at the keyframe pose.
 * out_pose = q_w_curr, t_w_curr; summary[3] = planes, iterations, termination (-1: built). */
int lislam_mapopt_step(lislam_map* m, const float* ground, int32_t n, const double* odom, double* state,
                       double* out_pose, int32_t* summary);
/* The same stage with mapOptimization's corner ikd-Tree (corner_ikdtree_, KD_TREE(0.3, 0.6, 0.8),
 * mapOptimization.cpp:195,479,505): the sensor-frame corner cloud (pc_corner, stride 4) goes in
 * at the ground cloud's keyframe pose, Build while that tree is empty, else Add_Points with
 * downsampling (create corner_map with downsample_size 0.8).  corner_map may be null. */
int lislam_mapopt_step_corner(lislam_map* m, lislam_map* corner_map, const float* ground, int32_t n,
                              const float* corner, int32_t nc, const double* odom, double* state, double* out_pose,
                              int32_t* summary);
/* The same stage fed from a batch without a host round trip: GroundPointOut of `scan`
 * (lislam_batch_ground) followed by its less-flat cloud, concatenated on the device
 * (mapOptimization.cpp:136-150).  The map's context must be the batch's. */
int lislam_batch_mapopt(lislam_batch* b, lislam_map* m, int32_t scan, const double* odom, double* state,
                        double* out_pose, int32_t* summary);
/* As lislam_batch_mapopt, with mapOptimization's corner ikd-Tree (corner_map, see
 * lislam_mapopt_step_corner) fed the scan's less-sharp cloud (/laser_cloud_less_sharp, the
 * pc_corner topic, mapOptimizationNode.cpp:63). corner_map NULL = lislam_batch_mapopt. */
int lislam_batch_mapopt_corner(lislam_batch* b, lislam_map* m, lislam_map* corner_map, int32_t scan,
                               const double* odom, double* state, double* out_pose, int32_t* summary);
/* laserMapping::process optimization (laserMapping.cpp:620-850) against a corner map and a surf
 * map: the downsampled current corner / surf clouds (stride 4), pose x (in/out), two outer
 * passes of association + Ceres(4 it).  stats[4] = corner / surf blocks of each pass. */
int lislam_laser_mapping(lislam_map* corner_map, lislam_map* surf_map, const float* corner, int32_t n_corner,
                         const float* surf, int32_t n_surf, double* x, int32_t* stats);

/* ---- laserMapping's cube map (laserMapping.cpp:70-99, 319-1002), device
 * resident: 21 x 21 x 11 cubes of 50 m holding the corner / surf points in map frame. */
typedef struct lislam_lmap lislam_lmap;
/* line_res / plane_res: mapping_line_resolution / mapping_plane_resolution (spot.launch: 0.4 / 0.8). */
int lislam_lmap_create(lislam_ctx* ctx, float line_res, float plane_res, lislam_lmap** out);
int lislam_lmap_destroy(lislam_lmap* m);
/* One laserMapping::process frame without publishing: corner_last / surf_last (stride 4, sensor
 * frame, host or device), odom = q_wodom_curr, t_wodom_curr (7); state (in/out) = q_wmap_wodom,
 * t_wmap_wodom (7); out_pose = q_w_curr, t_w_curr (7).  transformAssociateToMap, cube re-centring,
 * the local map of the valid cubes, VoxelGrid of the current clouds, the optimization of
 * lislam_laser_mapping when the map holds > 10 corner and > 50 surf points, transformUpdate,
 * insertion and the VoxelGrid of every valid cube.  stats[8] (nullable) = corner / surf local-map
 * sizes, corner / surf stack sizes, lislam_laser_mapping's stats (-1 when not optimized). */
int lislam_lmap_step(lislam_lmap* m, const float* corner_last, int32_t nc, const float* surf_last, int32_t ns,
                     const double* odom, double* state, double* out_pose, int32_t* stats);
/* Points per cube (cube index order, 4851 each; either nullable) and a whole cloud (0 corner,
 * 1 surf) as x, y, z, intensity in cube order (out nullable: *n only). */
int lislam_lmap_counts(lislam_lmap* m, int32_t* corner_counts, int32_t* surf_counts);
int lislam_lmap_points(lislam_lmap* m, int32_t which, float* out, int64_t cap, int64_t* n);

/* ---- loop closure and odometry fusion */
/* loop_closure_parameters (config/spot.yaml:26-33) + the ICP settings of
 * intensity_feature_tracker.cpp:219-232. */
typedef struct {
  int32_t use_crop;                   /* USE_CROP (spot.yaml: false) */
  float crop_size;                    /* CROP_SIZE: CropBox [-c, c]^3 (spot.yaml: 200) */
  int32_t use_downsample;             /* USE_DOWNSAMPLE (true) */
  float voxel_size;                   /* VOXEL_SIZE = vf_scan_res (0.25) */
  float max_correspondence_distance;  /* setMaxCorrespondenceDistance (100) */
  int32_t max_iterations;             /* setMaximumIterations (100) */
  double transformation_epsilon;      /* setTransformationEpsilon (1e-6) */
  double euclidean_fitness_epsilon;   /* setEuclideanFitnessEpsilon (1e-6) */
  double fitness_threshold;           /* FITNESS_SCORE = icp_fitness_score (0.5) */
} lislam_icp_config;
/* The USE_ICP block of feature_tracker::loopClosureThread (intensity_feature_tracker.cpp:217-366)
 * with tranformCurrentScanToMap (:167-172) and getSubmapOfhistory (:174-193): cur = the new
 * keyframe's cloud_track (n_cur x, y, z, intensity), T_cur = getTransformMatrix(keyframeId)
 * (row-major 4x4); hist = the history keyframes' clouds concatenated (hist_counts[n_hist]) with
 * their poses T_hist[n_hist][16].  removeNaN, CropBox, VoxelGrid, pcl::IterativeClosestPoint and
 * getFitnessScore on the device.  Outputs (each nullable): T_icp[16] = getFinalTransformation,
 * T_cur2map[16] = T_icp * T_cur (the loop factor's pose_from, :316-321), fitness, info[8] =
 * accepted (1 converged and fitness <= threshold, 0 not, -1 empty submap, -2 <= 10 points after
 * filtering), converged, convergence state (0 none, 1 iterations, 2 transform, 3 absolute MSE,
 * 4 relative MSE, 5 < 3 correspondences), iterations, source points, target points, last
 * correspondences, 0.  Point arrays may be host or device memory. */
int lislam_loop_icp(lislam_ctx* ctx, const lislam_icp_config* cfg, const float* cur, int32_t n_cur, const double* T_cur,
                    const float* hist, const int32_t* hist_counts, int32_t n_hist, const double* T_hist, double* T_icp,
                    double* T_cur2map, double* fitness, int32_t* info);
/* odomHandler's callback (src/odom_handler_node.cpp:44-132) over n synchronized pairs in order:
 * aloam[n][7] = /laser_odom_to_init_aloam, intensity[n][7] = /laser_odom_to_init_intensity
 * (q x,y,z,w, t), skip[n] = 1 when the intensity message's child_frame_id is "/odom_skip";
 * fused[n][7] = the published /laser_odom_to_init.  The fuser keeps the previous poses and
 * odom_cur on the device between calls.  Pointers may be host or device memory. */
typedef struct lislam_odom_fuser lislam_odom_fuser;
int lislam_odom_fuser_create(lislam_ctx* ctx, lislam_odom_fuser** out);
int lislam_odom_fuser_destroy(lislam_odom_fuser* f);
int lislam_odom_fuse(lislam_odom_fuser* f, const double* aloam, const double* intensity, const int32_t* skip, int32_t n,
                     double* fused);

/* HIP-event timing of the mapping kernels of a context (recorded on its stream, no host sync
 * while recording).  lislam_map_kernel_times synchronizes, returns the total ms and launch count
 * per kernel since the previous read (arrays of LISLAM_MAP_NUM_KERNELS, in the order below) and
 * clears the record. */
#define LISLAM_MAP_NUM_KERNELS 22 /* k_knn, k_fit, k_lm_eval, k_lm_step, map rebuild (keys + sort +
                                     gather + cell table), Add_Points downsample (claim + resolve),
                                     k_orb_pyramid, k_orb_fast, k_orb_select, k_orb_finish,
                                     k_orb_blur (the padded-level blur of images too large for
                                     k_orb_pyramid), k_orb_desc, k_orb_match, k_orb_lm,
                                     k_ground_screen, k_ground_ransac, k_ground_extract,
                                     k_lc_step, k_lc_apply, k_fuse, k_orb_roiblur (the ROI blur +
                                     border rows after k_orb_pyramid), k_lm_solve (a whole pose
                                     solve in one launch; k_lm_eval / k_lm_step are no longer
                                     launched) */
int lislam_map_set_timing(lislam_ctx* ctx, int32_t enable);
int lislam_map_kernel_times(lislam_ctx* ctx, float* ms, int32_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* LISLAM_H_ */
