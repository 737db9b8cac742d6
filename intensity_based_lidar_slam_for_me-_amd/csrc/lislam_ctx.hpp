// The context object behind the lislam C ABI (one HIP device + stream), shared by the ABI
// translation units.
#pragma once
#include <hip/hip_runtime.h>

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
  void* map_scratch = nullptr;     // device scratch of the stateless mapping entry points
  lislam_ktimer mtimer;            // mapping-kernel timing
};

// Frees lislam_ctx::map_scratch (lislam_map.hip).
void lislam_free_map_scratch(void* p);
