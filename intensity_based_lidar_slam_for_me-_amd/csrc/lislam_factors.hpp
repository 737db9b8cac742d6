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

// ---- DISTORTION 1 (laserOdometry.cpp:82, s = the point's relative time): the functors interpolate
// the pose, q_last_curr = Identity.slerp(s, q), t_last_curr = s t (lidarFeaturePointsFunction.hpp:
// 160-162,260-262).  Evaluated the way ceres::AutoDiffCostFunction does it: a forward-mode dual
// number over the 7 raw parameters (q x y z w, t), with Ceres' jet rules.
struct DJet {
  double a, v[7];
};
__device__ __forceinline__ DJet dj(double x) { DJet r; r.a = x; for (int k = 0; k < 7; k++) r.v[k] = 0.0; return r; }
__device__ __forceinline__ DJet dj(double x, int slot) { DJet r = dj(x); r.v[slot] = 1.0; return r; }
__device__ __forceinline__ DJet operator+(const DJet& f, const DJet& g) {
  DJet r; r.a = f.a + g.a; for (int k = 0; k < 7; k++) r.v[k] = f.v[k] + g.v[k]; return r;
}
__device__ __forceinline__ DJet operator-(const DJet& f, const DJet& g) {
  DJet r; r.a = f.a - g.a; for (int k = 0; k < 7; k++) r.v[k] = f.v[k] - g.v[k]; return r;
}
__device__ __forceinline__ DJet operator-(const DJet& f) {
  DJet r; r.a = -f.a; for (int k = 0; k < 7; k++) r.v[k] = -f.v[k]; return r;
}
__device__ __forceinline__ DJet operator*(const DJet& f, const DJet& g) {
  DJet r; r.a = f.a * g.a; for (int k = 0; k < 7; k++) r.v[k] = f.a * g.v[k] + f.v[k] * g.a; return r;
}
__device__ __forceinline__ DJet operator/(const DJet& f, const DJet& g) {  // a/b + (u - (a/b) v)/b, through 1/b
  const double ginv = 1.0 / g.a, fbyg = f.a * ginv;
  DJet r; r.a = f.a * ginv; for (int k = 0; k < 7; k++) r.v[k] = (f.v[k] - fbyg * g.v[k]) * ginv; return r;
}
__device__ __forceinline__ DJet jsqrt(const DJet& f) {
  const double t = sqrt(f.a), two_t = t + t;
  DJet r; r.a = t; for (int k = 0; k < 7; k++) r.v[k] = f.v[k] / two_t; return r;
}
__device__ __forceinline__ DJet jacos(const DJet& f) {
  const double tmp = -1.0 / sqrt(1.0 - f.a * f.a);
  DJet r; r.a = acos(f.a); for (int k = 0; k < 7; k++) r.v[k] = tmp * f.v[k]; return r;
}
__device__ __forceinline__ DJet jsin(const DJet& f) {
  const double c = cos(f.a);
  DJet r; r.a = sin(f.a); for (int k = 0; k < 7; k++) r.v[k] = c * f.v[k]; return r;
}
struct DJ3 {
  DJet x, y, z;
};
__device__ __forceinline__ DJ3 operator+(const DJ3& a, const DJ3& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ DJ3 operator-(const DJ3& a, const DJ3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ DJ3 jcross(const DJ3& a, const DJ3& b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ DJ3 dj3(const double* p) { return {dj(p[0]), dj(p[1]), dj(p[2])}; }

// Identity.slerp(s, q) (Eigen 3.3 QuaternionBase::slerp with this = (0, 0, 0, 1): this . q = w).
__device__ __forceinline__ void jslerp_identity(double s, const DJet* q, DJet* out) {
  const DJet d = q[3];
  const DJet absD = d.a < 0 ? -d : d;
  DJet scale0, scale1;
  if (absD.a >= 1.0 - 2.220446049250313e-16) {
    scale0 = dj(1.0 - s);
    scale1 = dj(s);
  } else {
    const DJet theta = jacos(absD);
    const DJet sinTheta = jsin(theta);
    scale0 = jsin(dj(1.0 - s) * theta) / sinTheta;
    scale1 = jsin(dj(s) * theta) / sinTheta;
  }
  if (d.a < 0) scale1 = -scale1;
  out[0] = scale1 * q[0]; out[1] = scale1 * q[1]; out[2] = scale1 * q[2]; out[3] = scale0 + scale1 * q[3];
}

// lp = Identity.slerp(s, q) c + s t, Eigen's _transformVector (uv = 2 q.vec x c; c + w uv + q.vec x uv).
__device__ __forceinline__ DJ3 jlast_point(const double* q, const double* t, const double* c, double s) {
  DJet qj[4], ql[4];
  for (int k = 0; k < 4; k++) qj[k] = dj(q[k], k);
  jslerp_identity(s, qj, ql);
  const DJ3 cp = dj3(c), qv{ql[0], ql[1], ql[2]};
  DJ3 uv = jcross(qv, cp);
  uv = uv + uv;
  const DJ3 wuv{ql[3] * uv.x, ql[3] * uv.y, ql[3] * uv.z};
  const DJ3 p = (cp + wuv) + jcross(qv, uv);
  const DJet sj = dj(s);
  const DJ3 tt{sj * dj(t[0], 4), sj * dj(t[1], 5), sj * dj(t[2], 6)};
  return p + tt;
}

// LidarEdgeFactor with s (rec: curr, a, b, s): r = (lp - a) x (lp - b) / |a - b|.
__device__ __forceinline__ void edge_factor_s(const double* q, const double* t, const double* rec, DJet* r) {
  const DJ3 lp = jlast_point(q, t, rec, rec[9]);
  const DJ3 a = dj3(rec + 3), b = dj3(rec + 6);
  const DJ3 nu = jcross(lp - a, lp - b);
  const DJ3 de = a - b;
  const DJet nde = jsqrt(de.x * de.x + de.y * de.y + de.z * de.z);
  r[0] = nu.x / nde; r[1] = nu.y / nde; r[2] = nu.z / nde;
}
// LidarPlaneFactor with s (rec: curr, j, the constructor's unit normal, s): r = (lp - j) . n.
__device__ __forceinline__ void plane_factor_s(const double* q, const double* t, const double* rec, DJet* r) {
  const DJ3 lp = jlast_point(q, t, rec, rec[9]);
  const DJ3 e = lp - dj3(rec + 3), n = dj3(rec + 6);
  r[0] = (e.x * n.x + e.y * n.y) + e.z * n.z;
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
