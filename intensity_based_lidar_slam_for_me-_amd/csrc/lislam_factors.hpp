// Device restatement of the cost functors of src/lidarFeaturePointsFunction.hpp with analytic
// Jacobians in Ceres' local parameterization: columns (d/d delta-theta[3], d/d t[3]) where
// EigenQuaternionParameterization::Plus(q, d) = [sin|d| d/|d|, cos|d|] (x) q, so that
// d(R(q) c)/d delta = -2 [R(q) c]x at delta = 0.  Residuals follow the functors' expression
// order in fp64.  s == 1 in every reference call site (DISTORTION 0, laserOdometry.cpp:82), and
// Identity.slerp(1, q) is +-q, which rotates exactly like q.
#pragma once
#include "lislam_device.hpp"

namespace lislam {

// LidarEdgeFactor (hpp:243-293): r = (lp - a) x (lp - b) / |a - b|, lp = q c + t.
__device__ __forceinline__ void edge_factor(const DQ& q, const D3& t, const D3& c, const D3& pa,
                                            const D3& pb, double* r, double (*J)[6]) {
  const D3 p = qrot(q, c);
  const D3 lp = p + t;
  const D3 nu = cross(lp - pa, lp - pb);
  const D3 de = pa - pb;
  const double nde = sqrt(de.x * de.x + de.y * de.y + de.z * de.z);
  r[0] = nu.x / nde; r[1] = nu.y / nde; r[2] = nu.z / nde;
  if (!J) return;
  // d r / d lp = [d]x with d = (b - a) / |a - b|
  const D3 d{(pb.x - pa.x) / nde, (pb.y - pa.y) / nde, (pb.z - pa.z) / nde};
  const double M[3][3] = {{0, -d.z, d.y}, {d.z, 0, -d.x}, {-d.y, d.x, 0}};
  const double P[3][3] = {{0, 2 * p.z, -2 * p.y}, {-2 * p.z, 0, 2 * p.x}, {2 * p.y, -2 * p.x, 0}};  // -2[p]x
  for (int i = 0; i < 3; i++) {
    for (int cc = 0; cc < 3; cc++) J[i][cc] = M[i][0] * P[0][cc] + M[i][1] * P[1][cc] + M[i][2] * P[2][cc];
    for (int cc = 0; cc < 3; cc++) J[i][3 + cc] = M[i][cc];
  }
}

// LidarPlaneFactor (hpp:143-196) with the constructor's unit normal n: r = (lp - j) . n.
__device__ __forceinline__ void plane_factor(const DQ& q, const D3& t, const D3& c, const D3& pj,
                                             const D3& n, double* r, double* J) {
  const D3 p = qrot(q, c);
  const D3 lp = p + t;
  *r = dot(lp - pj, n);
  if (!J) return;
  const D3 pn = cross(p, n);  // d r / d delta = 2 (p x n)
  J[0] = 2 * pn.x; J[1] = 2 * pn.y; J[2] = 2 * pn.z;
  J[3] = n.x; J[4] = n.y; J[5] = n.z;
}

// LidarPlaneNormFactor (hpp:199-240): r = n . (q c + t) + d.
__device__ __forceinline__ void plane_norm_factor(const DQ& q, const D3& t, const D3& c, const D3& n,
                                                  double dd, double* r, double* J) {
  const D3 p = qrot(q, c);
  const D3 pw = p + t;
  *r = dot(n, pw) + dd;
  if (!J) return;
  const D3 pn = cross(p, n);
  J[0] = 2 * pn.x; J[1] = 2 * pn.y; J[2] = 2 * pn.z;
  J[3] = n.x; J[4] = n.y; J[5] = n.z;
}

// front_end_residual (hpp:21-58): r = q c + t - dst (3 residuals).
__device__ __forceinline__ void p2p_factor(const DQ& q, const D3& t, const D3& c, const D3& dst, double* r,
                                           double (*J)[6]) {
  const D3 p = qrot(q, c);
  const D3 w = p + t;
  r[0] = w.x - dst.x; r[1] = w.y - dst.y; r[2] = w.z - dst.z;
  if (!J) return;
  const double P[3][3] = {{0, 2 * p.z, -2 * p.y}, {-2 * p.z, 0, 2 * p.x}, {2 * p.y, -2 * p.x, 0}};  // -2[p]x
  for (int i = 0; i < 3; i++)
    for (int cc = 0; cc < 3; cc++) { J[i][cc] = P[i][cc]; J[i][3 + cc] = i == cc ? 1.0 : 0.0; }
}

// LidarPlaneFactor constructor: ljm_norm = normalize((j - l) x (j - m)) (Eigen normalize()).
__device__ __forceinline__ D3 plane_normal(const D3& j, const D3& l, const D3& m) {
  D3 n = cross(j - l, j - m);
  const double sq = n.x * n.x + n.y * n.y + n.z * n.z;
  if (sq > 0) { const double rr = sqrt(sq); n.x /= rr; n.y /= rr; n.z /= rr; }
  return n;
}

// ceres::HuberLoss(a) + Corrector (rho'' <= 0 -> sqrt(rho') scaling).  Returns the scale and
// adds 0.5 rho(s) to *cost.
__device__ __forceinline__ double huber_scale(double a, double s, double* cost) {
  const double b = a * a;
  if (s > b) {
    const double rr = sqrt(s);
    *cost += 0.5 * (2.0 * a * rr - b);
    return sqrt(fmax(2.2250738585072014e-308, a / rr));
  }
  *cost += 0.5 * s;
  return 1.0;
}

}  // namespace lislam
