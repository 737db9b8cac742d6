// The device-resident batch and laserOdometry node objects behind the lislam C ABI, shared by
// the ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/lislam.h"
#include "lislam_internal.hpp"

using lislam::FeatureArgs;
using lislam::OdomArgs;

struct lislam_batch {
  lislam_ctx* ctx = nullptr;
  int max_scans = 0, H = 0, W = 0, N = 0;
  int cap_sharp = 0, cap_less_sharp = 0, cap_flat = 0;
  std::vector<void*> allocs;
  FeatureArgs fa{};
  OdomArgs oa{};
  double* d_init = nullptr;
  int* d_gate = nullptr;  // [max_scans] use_aloam of lislam_batch_odometry_gated
  // pinned staging of the odometry's host inputs (init states, use_aloam): the caller's arrays
  // are copied here before the asynchronous upload, so they may be freed on return; stage_ev
  // guards the staging against the next call until the previous upload has run
  void* h_stage = nullptr;
  hipEvent_t stage_ev = nullptr;
  bool stage_busy = false;
  bool timing = false;
  // per-call event sets recorded on the stream while timing is on; read back (and released)
  // by lislam_batch_kernel_times, so the timed region never blocks on the host.
  std::vector<std::vector<hipEvent_t>> ext_ev;
  std::vector<std::vector<lislam::OdoTimed>> odo_ev;
  // chain groups of the odometry schedule: group 0 on the context stream, the others on their own
  // streams (created on first use), forked / joined by events
  static constexpr int kMaxGroups = 4;
  static constexpr int kGroups = 2;  // groups used: one group's solves overlap the other's association
  hipStream_t odo_stream[kMaxGroups] = {};
  hipEvent_t odo_fork = nullptr, odo_join[kMaxGroups] = {};
  std::vector<hipEvent_t> pool;
  int extracted = 0;
  bool engine_ran = false;  // the last odometry call ran the chain engine (lislam_batch_odometry_status)
  // the split engine's fork / join events (its two CU-masked streams are the device's: a pair per
  // engine slot, shared by every batch); split: -1 not tried yet, 0 unavailable (single-launch
  // engine), 1 ready
  int eng_split = -1;
  hipEvent_t eng_fork = nullptr, eng_join_r = nullptr, eng_join_i = nullptr;
  // the split engine is not joined back into the context stream at launch (a join there would also
  // hold back whatever another context queued behind it on a shared hardware queue): eng_pending
  // until the next batch call that touches the batch's buffers, or lislam_synchronize, makes the
  // context stream wait for it.  eng_ready: recorded on the context stream at the end of every
  // lislam_batch_extract (and after odometry's staging copies); the engine starts from it.
  bool eng_pending = false;
  hipEvent_t eng_ready = nullptr;
  // the split launch as queued with the device's engine dispatcher (lislam::submit_odometry_chain_split):
  // its events are recorded when the dispatcher launches it, so every wait on them first waits for that
  lislam::EngineRequest eng_req;
  // Abort recovery.  Every engine launch (split or single) copies its sticky abort word into h_abort
  // (pinned) and records eng_done behind it; eng_check stays set until the next batch call settles
  // it: the host waits for eng_done and, if the engine gave up (a bounded device wait expired), clears
  // the word and re-runs eng_args on the per-round schedule on the context stream before the call
  // goes on, so a caller never sees the aborted launch's outputs.  eng_fallbacks counts those
  // recoveries until lislam_batch_odometry_status reads (and clears) it.
  bool eng_check = false;
  hipEvent_t eng_done = nullptr;
  unsigned* h_abort = nullptr;
  OdomArgs eng_args{};
  int eng_fallbacks = 0;
  unsigned eng_abort_code = 0;  // the error word of the last aborted launch (lislam_batch_odometry_abort_code)
  // recorded inside every lislam_batch_extract once the a1 images exist: the ORB front end waits
  // on it from its own stream, so it overlaps the rest of the extraction and whatever the caller
  // queued on the context stream after it.
  hipEvent_t ev_images = nullptr;
  void* orb = nullptr;  // ORB engine of lislam_batch_intensity_odometry (lislam_orb.hip)
  void* ground = nullptr;
  void* wire = nullptr;        // device staging of PointCloud2 bytes (lislam_batch_upload / download_cloud)
  size_t wire_bytes = 0;
  // lislam_batch_upload_async: the copy stream, a whole-batch staging area, and per 16-scan chunk
  // the "landed" (copy stream) and "parsed" (context stream) events
  hipStream_t copy_stream = nullptr;
  void* ring = nullptr;
  size_t ring_bytes = 0;
  std::vector<hipEvent_t> chunk_landed, chunk_parsed;
  std::vector<char> chunk_used;
  hipEvent_t get_event() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    hipEventCreate(&e);
    return e;
  }
  static hipEvent_t event_cb(void* self) { return static_cast<lislam_batch*>(self)->get_event(); }
};

struct lislam_odom {
  lislam_ctx* ctx = nullptr;
  bool have_last = false;
  double state[14] = {0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0};
  int frames = 0;
  int32_t gate[2] = {1, 1};  // use_aloam of the two scans of a gated step (kept alive for the async copy)
};


// Frees lislam_batch::ground / returns the device source of a ground output (lislam_ground.hip).
void lislam_free_ground(void* p);
int lislam_ground_batch_output(lislam_batch* b, int what, int scan, const void** src, int* cnt, size_t* esz);
// Frees lislam_batch::orb (lislam_orb.hip).
void lislam_free_orb(void* p);
// Device source of the ORB outputs (LISLAM_OUT_ORB_*) of one scan (lislam_orb.hip).
int lislam_orb_batch_output(lislam_batch* b, int what, int scan, const void** src, int* cnt, size_t* esz);
// Resolves a pending device-decided ORB cascade (lislam_orb.hip): waits for its verdict and, if it
// did not converge, redoes the batch from the images it was given.  lislam_batch_extract calls it
// before it overwrites those images.
int orb_settle(lislam_batch* b);
