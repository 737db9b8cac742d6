// The context object behind the lislam C ABI (one HIP device + stream), shared by the ABI
// translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/lislam.h"

// HIP-event timing of the mapping kernels (lislam_map_set_timing / lislam_map_kernel_times):
// events are recorded on the context's stream around each launch and read back only on request.
struct lislam_ktimer {
  bool on = false;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> rec;
  std::vector<hipEvent_t> pool;
  hipEvent_t get() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  ~lislam_ktimer() {
    for (auto& r : rec) { (void)hipEventDestroy(r.second.first); (void)hipEventDestroy(r.second.second); }
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

struct lislam_ctx {
  lislam_config cfg;
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  lislam_batch* single = nullptr;  // 2-scan batch behind lislam_scan_registration / odom_step
  std::vector<lislam_batch*> batches;  // live batches (lislam_synchronize settles their engines)
  void* map_scratch = nullptr;     // device scratch of the stateless mapping entry points
  lislam_ktimer mtimer;            // mapping-kernel timing
  int ties = LISLAM_TIES_REFERENCE;  // lislam_set_tie_order
  int odom_engine = LISLAM_ENGINE_AUTO;     // lislam_set_odometry_schedule
  int eng_qpw = 1, eng_depth = 1;           // lislam_set_engine_shape (the latency shape)
  // lislam_eval_factors(_raw): one grow-only device buffer for the blocks, the parameters and the
  // outputs, reused across calls; the mutex serializes callers (Ceres evaluates residual blocks
  // from num_threads threads)
  std::mutex factor_mu;
  void* factor_buf = nullptr;
  size_t factor_bytes = 0;
};

// kernel ids of lislam_map_kernel_times (LISLAM_CTX_NUM_KERNELS in include/lislam.h)
enum {
  kT_knn = 0, kT_fit, kT_lm_eval, kT_lm_step, kT_rebuild, kT_downsample,
  kT_orb_pyramid, kT_orb_fast, kT_orb_select, kT_orb_finish, kT_orb_blur, kT_orb_desc, kT_orb_match, kT_orb_lm,
  kT_ground_screen, kT_ground_ransac, kT_ground_extract, kT_icp_step, kT_icp_apply, kT_fuse, kT_orb_roiblur,
  kT_lm_solve, kT_count
};

// Records HIP events around the launches of its scope when the context's timer is on.
struct TimedScope {
  lislam_ctx* c;
  int id;
  hipEvent_t b = nullptr;
  TimedScope(lislam_ctx* c_, int id_) : c(c_), id(id_) {
    if (c->mtimer.on) { b = c->mtimer.get(); (void)hipEventRecord(b, c->stream); }
  }
  ~TimedScope() {
    if (!b) return;
    hipEvent_t e = c->mtimer.get();
    (void)hipEventRecord(e, c->stream);
    c->mtimer.rec.push_back({id, {b, e}});
  }
};

namespace lislam {
// Developer timeline (LISLAM_TIMELINE=1): timeline_epoch records a per-device epoch event on s
// once (at the first context's creation); timeline_print writes a timed launch's start / end in ms
// from that epoch to stderr, so the streams of pipelined contexts line up on one clock.
void timeline_epoch(int dev, hipStream_t s);
void timeline_print(int dev, const char* who, const void* obj, int kernel, hipEvent_t b, hipEvent_t e);
}  // namespace lislam

// Frees lislam_ctx::map_scratch (lislam_map.hip).
void lislam_free_map_scratch(void* p);
