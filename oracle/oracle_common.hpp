// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference hot path (himhan34/Intensity_based_LiDAR_SLAM_for_me-).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code,
// and only as the checker / CPU baseline.  The product path (the HIP library) never links it.
//
// Parity status: the reference cannot be compiled here (ROS/PCL/OpenCV/Ceres/Eigen absent and
// its sources are syntactically damaged); it ships no tests and no golden
// vectors.  This restatement is pinned by (1) golden fixtures it generates and commits under
// tests/golden/, (2) exact-kNN cross-checks against scipy.cKDTree, (3) finite-difference
// Jacobian checks of the functors, (4) independent property tests.  Third-party arithmetic at
// the boundary (PCL VoxelGrid/KdTreeFLANN, Ceres 1.14 LM, Eigen QR) is restated from the
// published algorithms and is "parity unpinned" against the real libraries.
#pragma once
#include <cmath>
#include <cstdint>

namespace oracle {

struct P4 {
  float x, y, z, i;
};

// Float transcendental semantics used by the restatement (and by the HIP path): the
// reference calls float atan/atan2 (scanRegistration.cpp:285,334 through <math.h>'s float
// overloads), whose last-ulp behaviour is libm-specific.  We define them as the correctly
// rounded float of the double-precision function; see DESIGN.md "FP semantics".
inline float atan2_f(float y, float x) { return (float)std::atan2((double)y, (double)x); }
inline float atan_f(float v) { return (float)std::atan((double)v); }

}  // namespace oracle
