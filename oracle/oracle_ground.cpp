// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.hpp).
//
// Restatement of ImageHandler::groundPlaneExtraction (src/image_handler.h_ouster:41-100), the
// RANSAC ground cloud that mapOptimization merges with the less-flat cloud
// (src/mapOptimization.cpp:136,148):
//   1. screening: points with z in [-2.0, -0.45] (:49-54), taken in index order (the reference
//      fills the vector from an OpenMP loop with an unsynchronized push_back, :48-54);
//   2. pcl::SACSegmentation<PointXYZ>, SACMODEL_PLANE, SAC_RANSAC, threshold 0.01, optimized
//      coefficients (:57-67).  setAxis / setEpsAngle do not apply to SACMODEL_PLANE.  Restated
//      from PCL 1.10.0 (the libpcl-dev of the ros:noetic base image, Dockerfile:1-8), single
//      thread: SampleConsensusModel seeded with 12345 (random_ = false), boost::mt19937 with
//      uniform_int<>(0, INT_MAX) (= mt19937() >> 1), drawIndexSample's partial Fisher-Yates on
//      the persistent shuffled index list, isSampleGood's collinearity test, plane coefficients
//      from the cross product (Eigen 4-float SSE reductions: (e0 + e2) + (e1 + e3)),
//      countWithinDistance with |n.p + d| < threshold, RandomSampleConsensus::computeModel's
//      adaptive k (probability 0.99, max 50 iterations), selectWithinDistance, then
//      optimizeModelCoefficients: computeMeanAndCovarianceMatrix (float, in inlier order) and
//      pcl::eigen33's smallest-eigenvalue eigenvector (computeRoots closed form);
//   3. the orientation test n . z > cos(15 deg) (:76-77) and the ground cloud: every input point
//      with |A x + B y + C z + D| / |n| <= 0.03 and z < 0, in double (:79-89).
//
// Parity status: PCL is absent here and the reference calls setNumberOfThreads(2 * 6) (:65), which
// with PCL >= 1.11 makes RANSAC's sample order thread-scheduled — parity unpinned against PCL;
// this single-thread restatement is pinned by tests/test_oracle_ground.py (an independent numpy
// transcription of the same steps).  Float atan2 / cos / sin are the correctly rounded floats of
// the double functions (DESIGN.md "FP semantics").
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

#include "oracle_common.hpp"

namespace {

struct V3 {
  float x, y, z;
};

// Eigen 3.3 SSE predux of a 4-float packet: (e0 + e2) + (e1 + e3)
inline float sum4(float e0, float e1, float e2, float e3) { return (e0 + e2) + (e1 + e3); }
// Eigen 3.3 non-vectorized redux of 3 floats: e0 + (e1 + e2)
inline float sum3(float e0, float e1, float e2) { return e0 + (e1 + e2); }

// SampleConsensusModelPlane::computeModelCoefficients (plane through 3 points, normalized)
void plane_from_3(const V3& p0, const V3& p1, const V3& p2, float* c) {
  const float a0 = p1.x - p0.x, a1 = p1.y - p0.y, a2 = p1.z - p0.z;
  const float b0 = p2.x - p0.x, b1 = p2.y - p0.y, b2 = p2.z - p0.z;
  c[0] = a1 * b2 - a2 * b1;
  c[1] = a2 * b0 - a0 * b2;
  c[2] = a0 * b1 - a1 * b0;
  c[3] = 0.f;
  const float z = sum4(c[0] * c[0], c[1] * c[1], c[2] * c[2], c[3] * c[3]);
  if (z > 0.f) {
    const float s = std::sqrt(z);
    for (int k = 0; k < 4; k++) c[k] /= s;
  }
  c[3] = -1.f * sum4(c[0] * p0.x, c[1] * p0.y, c[2] * p0.z, c[3] * 1.f);
}

// isSampleGood: (p1 - p0) / (p2 - p0) not the same in all three coordinates
bool sample_good(const V3& p0, const V3& p1, const V3& p2) {
  const float d0 = (p1.x - p0.x) / (p2.x - p0.x), d1 = (p1.y - p0.y) / (p2.y - p0.y), d2 = (p1.z - p0.z) / (p2.z - p0.z);
  return (d0 != d1) || (d2 != d1);
}

inline float plane_dist(const float* c, const V3& p) { return std::fabs(sum4(c[0] * p.x, c[1] * p.y, c[2] * p.z, c[3] * 1.f)); }

inline float f_atan2(float y, float x) { return (float)std::atan2((double)y, (double)x); }
inline float f_cos(float v) { return (float)std::cos((double)v); }
inline float f_sin(float v) { return (float)std::sin((double)v); }

void compute_roots2(float b, float c, float* r) {
  r[0] = 0.f;
  float d = (float)((double)(b * b) - 4.0 * (double)c);
  if (d < 0.0) d = 0.f;
  const float sd = std::sqrt(d);
  r[2] = 0.5f * (b + sd);
  r[1] = 0.5f * (b - sd);
}

// pcl::computeRoots (common/eigen.hpp) of a symmetric 3x3 (row-major m[9])
void compute_roots(const float* m, float* r) {
  const float m00 = m[0], m01 = m[1], m02 = m[2], m11 = m[4], m12 = m[5], m22 = m[8];
  const float c0 = m00 * m11 * m22 + 2.f * m01 * m02 * m12 - m00 * m12 * m12 - m11 * m02 * m02 - m22 * m01 * m01;
  const float c1 = m00 * m11 - m01 * m01 + m00 * m22 - m02 * m02 + m11 * m22 - m12 * m12;
  const float c2 = m00 + m11 + m22;
  if (std::fabs(c0) < std::numeric_limits<float>::epsilon()) {
    compute_roots2(c2, c1, r);
    return;
  }
  const float s_inv3 = (float)(1.0 / 3.0);
  const float s_sqrt3 = std::sqrt(3.0f);
  const float c2_over_3 = c2 * s_inv3;
  float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
  if (a_over_3 > 0.f) a_over_3 = 0.f;
  const float half_b = 0.5f * (c0 + c2_over_3 * (2.f * c2_over_3 * c2_over_3 - c1));
  float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
  if (q > 0.f) q = 0.f;
  const float rho = std::sqrt(-a_over_3);
  const float theta = f_atan2(std::sqrt(-q), half_b) * s_inv3;
  const float ct = f_cos(theta), st = f_sin(theta);
  r[0] = c2_over_3 + 2.f * rho * ct;
  r[1] = c2_over_3 - rho * (ct + s_sqrt3 * st);
  r[2] = c2_over_3 - rho * (ct - s_sqrt3 * st);
  if (r[0] >= r[1]) std::swap(r[0], r[1]);
  if (r[1] >= r[2]) {
    std::swap(r[1], r[2]);
    if (r[0] >= r[1]) std::swap(r[0], r[1]);
  }
  if (r[0] <= 0.f) compute_roots2(c2, c1, r);
}

// pcl::eigen33: eigenvector of the smallest eigenvalue of a symmetric 3x3 (row-major)
void eigen33_min(const float* mat, float* ev) {
  float scale = 0.f;
  for (int k = 0; k < 9; k++) scale = std::max(scale, std::fabs(mat[k]));
  if (scale <= std::numeric_limits<float>::min()) scale = 1.f;
  float m[9];
  for (int k = 0; k < 9; k++) m[k] = mat[k] / scale;
  float r[3];
  compute_roots(m, r);
  m[0] -= r[0];
  m[4] -= r[0];
  m[8] -= r[0];
  auto cross = [&](int i, int j, float* v) {
    const float* a = m + 3 * i;
    const float* b = m + 3 * j;
    v[0] = a[1] * b[2] - a[2] * b[1];
    v[1] = a[2] * b[0] - a[0] * b[2];
    v[2] = a[0] * b[1] - a[1] * b[0];
  };
  float v1[3], v2[3], v3[3];
  cross(0, 1, v1);
  cross(0, 2, v2);
  cross(1, 2, v3);
  const float l1 = sum3(v1[0] * v1[0], v1[1] * v1[1], v1[2] * v1[2]);
  const float l2 = sum3(v2[0] * v2[0], v2[1] * v2[1], v2[2] * v2[2]);
  const float l3 = sum3(v3[0] * v3[0], v3[1] * v3[1], v3[2] * v3[2]);
  const float* v;
  float l;
  if (l1 >= l2 && l1 >= l3) { v = v1; l = l1; }
  else if (l2 >= l1 && l2 >= l3) { v = v2; l = l2; }
  else { v = v3; l = l3; }
  const float s = std::sqrt(l);
  for (int k = 0; k < 3; k++) ev[k] = v[k] / s;
}

constexpr double kThreshold = 0.01;   // setDistanceThreshold (:61)
constexpr int kMaxIterations = 50;    // SACSegmentation default max_iterations_
constexpr double kProbability = 0.99; // SACSegmentation default probability_
constexpr int kMaxSampleChecks = 1000;

}  // namespace

// Per-cloud result: info[0] status (1 ground plane accepted, 0 plane rejected by the orientation
// test, -1 fewer than 3 candidates / no sample, -2 no model), info[1] RANSAC iterations,
// info[2] best RANSAC inlier count, info[3] refit inlier count; plane[4] = the segmented
// coefficients (A, B, C, D); out (n x 4: x, y, z, 1) the ground cloud, returns its size.
extern "C" int oracle_ground_extract(const float* pts, int n, int stride, float* out, float* plane, int* info) {
  info[0] = -1; info[1] = 0; info[2] = 0; info[3] = 0;
  for (int k = 0; k < 4; k++) plane[k] = 0.f;
  // 1. screening
  std::vector<V3> cand;
  for (int i = 0; i < n; i++) {
    const float* p = pts + (size_t)i * stride;
    if (p[2] >= -2.0 && p[2] <= -0.45) cand.push_back(V3{p[0], p[1], p[2]});
  }
  const int nc = (int)cand.size();
  if (nc < 3) return 0;
  // 2. RANSAC (RandomSampleConsensus::computeModel)
  std::mt19937 rng(12345u);
  auto rnd = [&]() -> int { return (int)(rng() >> 1); };  // boost::uniform_int<>(0, INT_MAX)
  std::vector<int> shuffled(nc);
  for (int i = 0; i < nc; i++) shuffled[i] = i;
  int iterations = 0, best = -INT_MAX;
  double k = 1.0;
  const double log_probability = std::log(1.0 - kProbability);
  const double one_over_indices = 1.0 / (double)nc;
  float model[4] = {0, 0, 0, 0};
  bool have_model = false;
  while (iterations < k) {
    int sel[3];
    bool got = false;
    for (int chk = 0; chk < kMaxSampleChecks && !got; chk++) {
      for (int i = 0; i < 3; i++) std::swap(shuffled[i], shuffled[i + ((size_t)rnd() % (size_t)(nc - i))]);
      for (int i = 0; i < 3; i++) sel[i] = shuffled[i];
      got = sample_good(cand[sel[0]], cand[sel[1]], cand[sel[2]]);
    }
    if (!got) break;  // "No samples could be selected"
    float c[4];
    plane_from_3(cand[sel[0]], cand[sel[1]], cand[sel[2]], c);
    int cnt = 0;
    for (int i = 0; i < nc; i++) cnt += plane_dist(c, cand[i]) < kThreshold;
    if (cnt > best) {
      best = cnt;
      std::memcpy(model, c, sizeof(model));
      have_model = true;
      const double w = (double)best * one_over_indices;
      double p_no_outliers = 1.0 - std::pow(w, 3.0);
      p_no_outliers = std::max(std::numeric_limits<double>::epsilon(), p_no_outliers);
      p_no_outliers = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no_outliers);
      k = log_probability / std::log(p_no_outliers);
    }
    ++iterations;
    if (iterations > kMaxIterations) break;
  }
  info[1] = iterations;
  if (!have_model) { info[0] = -2; return 0; }
  info[2] = best;
  // selectWithinDistance + optimizeModelCoefficients
  float coef[4] = {model[0], model[1], model[2], model[3]};
  float acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  int ni = 0;
  for (int i = 0; i < nc; i++) {
    const V3& p = cand[i];
    if (!(plane_dist(model, p) < kThreshold)) continue;
    acc[0] += p.x * p.x; acc[1] += p.x * p.y; acc[2] += p.x * p.z;
    acc[3] += p.y * p.y; acc[4] += p.y * p.z; acc[5] += p.z * p.z;
    acc[6] += p.x; acc[7] += p.y; acc[8] += p.z;
    ni++;
  }
  info[3] = ni;
  if (ni > 3) {
    for (int e = 0; e < 9; e++) acc[e] /= (float)ni;
    float cov[9];
    cov[0] = acc[0] - acc[6] * acc[6];
    cov[1] = acc[1] - acc[6] * acc[7];
    cov[2] = acc[2] - acc[6] * acc[8];
    cov[4] = acc[3] - acc[7] * acc[7];
    cov[5] = acc[4] - acc[7] * acc[8];
    cov[8] = acc[5] - acc[8] * acc[8];
    cov[3] = cov[1];
    cov[6] = cov[2];
    cov[7] = cov[5];
    float ev[3];
    eigen33_min(cov, ev);
    coef[0] = ev[0]; coef[1] = ev[1]; coef[2] = ev[2]; coef[3] = 0.f;
    coef[3] = -1.f * sum4(coef[0] * acc[6], coef[1] * acc[7], coef[2] * acc[8], coef[3] * 1.f);
  }
  for (int e = 0; e < 4; e++) plane[e] = coef[e];
  // 3. orientation test and the ground cloud (double)
  const double A = coef[0], B = coef[1], C = coef[2], D = coef[3];
  const float nz = sum3(coef[0] * 0.f, coef[1] * 0.f, coef[2] * 1.f);
  if (!((double)nz > std::cos(15 * M_PI / 180))) { info[0] = 0; return 0; }
  info[0] = 1;
  const double nrm = std::sqrt(A * A + B * B + C * C);
  int m = 0;
  for (int i = 0; i < n; i++) {
    const float* p = pts + (size_t)i * stride;
    const double X = p[0], Y = p[1], Z = p[2];
    const double height = std::fabs(A * X + B * Y + C * Z + D) / nrm;
    if (height <= 0.03 && p[2] < -0.0) {
      out[4 * m + 0] = p[0]; out[4 * m + 1] = p[1]; out[4 * m + 2] = p[2]; out[4 * m + 3] = 1.f;
      m++;
    }
  }
  return m;
}
