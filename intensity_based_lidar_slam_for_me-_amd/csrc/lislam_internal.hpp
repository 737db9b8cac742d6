// Internal (not exported) kernel argument blocks and launch entry points of liblislam.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <vector>

#include "lislam_device.hpp"

namespace lislam {

constexpr int kMaxLines = 128;               // N_SCANS in {16, 32, 64, 128}
constexpr int kCapSharpPerLine = 12;         // 2 per segment x 6 (scanRegistration.cpp:459)
constexpr int kCapLessSharpPerLine = 120;    // 20 per segment x 6 (:466)
constexpr int kCapFlatPerLine = 24;          // 4 per segment x 6 (:530)
constexpr int kMaxEngineDepth = 6;           // engines in flight per device (lislam_set_engine_shape)

// Device-resident batch of S organized scans and every per-scan output of a1..a7.
struct FeatureArgs {
  const P4* pts;  // [S][N] xyzI, ring-major (u * W + v)
  int S, H, W, N;
  float min_range;
  // a1 outputs (nullable)
  uint8_t* img_range;  // [S][N]
  uint8_t* img_int;    // [S][N]
  P4* track;           // [S][N]
  // a2..a5
  P4* cloud;      // [S][N] laserCloud, scan-grouped
  int* n_cloud;   // [S]
  int* line_off;  // [S][H+1]
  float* curv;    // [S][N]
  int8_t* label;  // [S][N]
  // per-line staging
  P4* stg_sharp;       // [S][H][12]
  P4* stg_less_sharp;  // [S][H][120]
  P4* stg_flat;        // [S][H][24]
  P4* stg_less_flat;   // [S][N] (line regions at line_off)
  int* line_counts;    // [S][H][4]
  // front pass scratch: ranges of 1024 ring-order points
  int fr_R;            // ranges per scan = ceil(N / 1024)
  int* fr_hist;        // [S][R][H] per-range line histogram, then per-range write bases
  int* fr_flip;        // [S][R] first halfPassed flip index of each range; [s][0] = the scan's
  float* fr_ori;       // [S][2] startOri, endOri
  // scratch for lines longer than the LDS fast path
  uint8_t* scr_picked;  // [S][N]
  uint64_t* scr_keys;   // [S][2N]
  int* scr_list;        // [S][N]
  uint8_t* scr_link;    // [S][N]
  // a6/a7 outputs, concatenated in line order
  P4* sharp;       // [S][cap_sharp]
  P4* less_sharp;  // [S][cap_less_sharp]
  P4* flat;        // [S][cap_flat]
  P4* less_flat;   // [S][N]
  int* n_feat;     // [S][4] = sharp, less_sharp, flat, less_flat
  int* feat_loff;  // [S][2][H+1] per-line offsets of less_sharp / less_flat
  int cap_sharp, cap_less_sharp, cap_flat;
  int ties;  // order of equal keys in the segment sorts and the a7 VoxelGrid: LISLAM_TIES_REFERENCE
            // (libstdc++ std::sort's) / LISLAM_TIES_INDEX
};

// Spatial index of a feature cloud: chunks of kChunk consecutive points (in the cloud's own,
// scan-line-major order) and super-chunks of kChunk chunks, each with an AABB whose w lanes hold
// the min / max scan line label int(intensity) of its points.
constexpr int kChunk = 16;
constexpr int kSuper = kChunk * kChunk;

struct TargetIndex {
  // scan-line (original) order: used by the scan-line searches
  float4* chunk;  // [S][nchunk][2] (lo, hi)
  float4* super;  // [S][nsuper][2]
  // Morton (z-order) order: used by the 1-NN; w of a sorted point = original index (int bits)
  float4* sorted;    // [S][cap] points
  float4* nn_chunk;  // [S][nchunk][2]
  float4* nn_super;  // [S][nsuper][2]
  uint64_t* keys;    // [S][2 * cap] sort scratch for clouds beyond the LDS sort
  int cap, nchunk, nsuper;
};

// Scan-to-scan odometry over chains of consecutive scans (a12..a18).  Chain c is a fresh
// laserOdometry node over scans [c*L, min(c*L + L, S-1)]; round r processes pair k = c*L + r + 1
// of every chain in two phases per outer pass (association, then the Ceres-semantics solve).
struct OdomArgs {
  int S, N, H;
  const P4* sharp; const P4* less_sharp; const P4* flat; const P4* less_flat;
  const int* n_feat;
  const int* feat_loff;  // [S][2][H+1] line offsets of less_sharp / less_flat
  TargetIndex idx_ls, idx_lf;
  float4* qpts_sharp;  // [S][cap_sharp] sharp queries in Morton order: x, y, z, query index bits
  float4* qpts_flat;   // [S][cap_flat]    (association wave -> its query in one load)
  int cap_sharp, cap_less_sharp, cap_flat;
  int chain_len;
  int n_chains;
  int c0, cn;      // the chains [c0, c0 + cn) one launch serves (a chain group)
  int max_iterations;  // ceres max_num_iterations (4, laserOdometry.cpp:707)
  const double* init_state;  // [n_chains][14] = para(7) + pose(7) at the chain start, or null
  double* state;             // [n_chains][16] = para(7), q_w(4), t_w(3)
  double* blk;     // [n_chains][cap_sharp + cap_flat][9] residual block records
  int* blk_kind;   // -1 invalid, 0 edge, 1 plane
  // outputs per scan
  double* para;    // [S][7] q_last_curr (x,y,z,w), t_last_curr after this scan
  double* pose;    // [S][7] q_w_curr, t_w_curr in the chain's frame
  int* stats;      // [S][8] corners/planes for outer 0/1, LM iterations 0/1, terminations 0/1
  const int* gate;  // [S] use_aloam per scan (laserOdometry.cpp:403-417), or null = every scan
  // chain engine (k_odom_chain): control words (zeroed before every launch) and the per-query
  // association of the first outer pass, the second pass's starting bounds
  unsigned* eng_ctl;  // [8 + 10 S]
  int eng_qpw, eng_depth;  // the split engine's shape (lislam_set_engine_shape)
  int* warm;          // [n_chains][cap_sharp + cap_flat][4]
  double* eng_part;   // [n_chains][engine_part_rows][32]: each association item's (and overflow query's)
                      // share of the first evaluation
};

// Batched evaluation of the cost functors (lislam_eval_factors).
struct FactorArgs {
  int n;
  const int* kind;     // 0 edge, 1 plane, 2 plane-norm
  const double* pts;   // [n][12]
  const double* x;     // q(4), t(3)
  double* res;         // [n][3] or null
  double* jac;         // [n][3][6] or null
};

// PointCloud2 point layout (point_step and the byte offsets of x, y, z, intensity).
struct WireLayout {
  uint32_t step, ox, oy, oz, oi;
};
void launch_unpack_layout(const uint8_t* raw, int n, const WireLayout& L, P4* out, hipStream_t st);
void launch_pack_layout(const P4* in, int n, const WireLayout& L, uint8_t* raw, hipStream_t st);

// images_ready (nullable): recorded once k_scan_front has written the range / intensity images and
// cloud_track, which is all the ORB front end reads.
void launch_features(const FeatureArgs& a, hipStream_t st, hipEvent_t* ev /*4 or null*/, hipEvent_t images_ready);
void launch_target_index(const OdomArgs& a, int n_scans, hipStream_t st);
// One timed launch of the odometry schedule: kernel id (4 k_odom_assoc, 5 k_odom_lm) and the events
// recorded on its stream right before and after it.
struct OdoTimed {
  int kernel;
  hipEvent_t b, e;
};
// Issues the whole round/phase schedule.  The chains are split into ngroups groups, group g on
// streams[g] (streams[0] = the caller's stream, which the others fork from and join back into),
// so one group's solves overlap another group's association.  fork / join: ngroups events.
// ev (nullable) receives every launch's timing events (from get_event).
void launch_odometry(const OdomArgs& a, const hipStream_t* streams, int ngroups, hipEvent_t fork,
                     const hipEvent_t* join, std::vector<OdoTimed>* ev, hipEvent_t (*get_event)(void*),
                     void* ev_owner);
// The same schedule as ONE persistent launch (k_odom_chain, lislam_odometry.hip): every round of
// the a.n_chains chains, association and solve, sequenced on the device.  Returns the grid size.
int launch_odometry_chain(const OdomArgs& a, hipStream_t st);
// The same engine as two launches (k_odom_roles / k_odom_items on a CU-masked stream pair).
// Nothing is queued on the context stream: the launch takes the device's next engine slot (its
// stream pair, shared by every batch: engine_streams_available), the roles stream waits for `ready`
// (the inputs) and for the launch `depth` before it, the items stream forks from it; join_r /
// join_i mark the end (the caller makes its stream wait for them later); t0 / t1 (nullable): timing
// events; h_abort (nullable): pinned host words the launch's error / sticky abort words are copied
// to at its end, `done` (nullable) recorded after that copy.  0 = nothing queued (no CU masks on
// this device): the caller must run the single-launch engine instead.
int launch_odometry_chain_split(const OdomArgs& a, hipEvent_t ready, hipEvent_t fork, hipEvent_t join_r,
                                hipEvent_t join_i, hipEvent_t t0, hipEvent_t t1, unsigned* h_abort, hipEvent_t done);
// The same launch through the device's engine dispatcher (a host thread per device): the request is
// queued and submit returns at once; the dispatcher launches it, on whichever engine slot is free,
// once its `ready` event has completed and fewer than `depth` engines are in flight — so a chain
// never waits for one particular earlier chain (launch n - depth) while another slot is idle.
// The events are recorded when the dispatcher launches; wait_engine_launched(r) returns once they
// are (before any wait on them).  submit: 0 = nothing queued (no CU masks on this device).
struct EngineRequest {
  OdomArgs a;
  hipEvent_t ready, fork, join_r, join_i, t0, t1, done;
  unsigned* h_abort;
  void* plan = nullptr;  // the launch's parameters, fixed when submitted (its environment knobs included)
  std::atomic<int> state{0};  // 0 none, 1 queued, 2 launched
};
int submit_odometry_chain_split(EngineRequest* r);
void wait_engine_launched(EngineRequest* r);
bool engine_dispatch_enabled();  // LISLAM_ENGINE_DISPATCH (default 1; 0: launch_odometry_chain_split)
bool engine_streams_available(int dev);  // the device has CU-masked streams for the split engine
void release_engine_streams(int dev);    // with the device's last context (also the round-stream pool)
// A stream for the library's other kernels that keeps off the solve roles' CUs (see lislam_odometry.hip).
// Every CU-masked stream is a hardware queue of its own; the library counts them per device
// (masked_queue_count) and destroys them with destroy_stream.
bool work_stream(int dev, hipStream_t* s);
void destroy_stream(hipStream_t s);
int masked_queue_count(int dev);
// The per-round schedule's extra chain-group stream g (>= 1): one per device and group, shared by
// every batch (two pipelined contexts' group-g launches then queue on one hardware queue instead of
// one each); null if it cannot be made.
hipStream_t round_stream(int dev, int g);
// Whether the engine serves a.n_chains chains (launch_odometry otherwise): mode = the context's
// lislam_set_odometry_schedule (LISLAM_ENGINE_*; a context starts from the environment's
// LISLAM_ENGINE if set); AUTO = on for at most 4 chains.
bool use_chain_engine(const OdomArgs& a, int mode);
// Association items per (pass, chain) of the engine for cap_queries = cap_sharp + cap_flat (the
// size of OdomArgs::eng_part's per-chain rows).
int engine_items(int cap_queries);
// Rows per chain of OdomArgs::eng_part: the items' and the stolen overflow queries' (lislam_odometry.hip).
int engine_part_rows(int cap_queries);
void launch_factors(const FactorArgs& a, hipStream_t st);

// AutoDiffCostFunction<F, R, 4, 3>::Evaluate of the functors of lidarFeaturePointsFunction.hpp:
// Jacobians w.r.t. the raw parameter blocks q[4] (x, y, z, w) and t[3], as ceres::Jet computes them.
struct RawFactorArgs {
  int n;
  const int* kind;     // 0 edge, 1 plane, 2 plane-norm, 3 front_end_residual / FeatureMatchingResidual,
                       // 4 LidarGroundPlaneNormFactor (q block only)
  const double* pts;   // [n][12]
  const double* x;     // q(4), t(3)
  double* res;         // [n][3] or null
  double* jq;          // [n][3][4] or null
  double* jt;          // [n][3][3] or null
};
void launch_factors_raw(const RawFactorArgs& a, hipStream_t st);

}  // namespace lislam
