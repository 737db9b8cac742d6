// The context object behind the lislam C ABI (one HIP device + stream), shared by the ABI
// translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/lislam.h"

struct lislam_ctx {
  lislam_config cfg;
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  lislam_batch* single = nullptr;  // 2-scan batch behind lislam_scan_registration / odom_step
  void* map_scratch = nullptr;     // device scratch of the stateless mapping entry points
};

// Frees lislam_ctx::map_scratch (lislam_map.hip).
void lislam_free_map_scratch(void* p);
