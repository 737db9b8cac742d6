// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.hpp).
//
// A dual number with the arithmetic rules of ceres::Jet (Ceres 1.14, third party, absent here:
// restated from its published jet.h semantics, parity unpinned), plus the handful of Eigen
// quaternion / vector operations the cost functors of src/lidarFeaturePointsFunction.hpp use,
// restated in the evaluation order Eigen 3.3 uses for 3-vectors on x86-64.
#pragma once
#include <cmath>

namespace oracle {

template <int N>
struct Jet {
  double a;
  double v[N];
  Jet() : a(0) { for (int k = 0; k < N; k++) v[k] = 0; }
  explicit Jet(double x) : a(x) { for (int k = 0; k < N; k++) v[k] = 0; }
  Jet(double x, int slot) : a(x) {
    for (int k = 0; k < N; k++) v[k] = 0;
    v[slot] = 1.0;
  }
};

template <int N> inline Jet<N> operator+(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> r; r.a = f.a + g.a; for (int k = 0; k < N; k++) r.v[k] = f.v[k] + g.v[k]; return r;
}
template <int N> inline Jet<N> operator-(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> r; r.a = f.a - g.a; for (int k = 0; k < N; k++) r.v[k] = f.v[k] - g.v[k]; return r;
}
template <int N> inline Jet<N> operator-(const Jet<N>& f) {
  Jet<N> r; r.a = -f.a; for (int k = 0; k < N; k++) r.v[k] = -f.v[k]; return r;
}
template <int N> inline Jet<N> operator*(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> r; r.a = f.a * g.a; for (int k = 0; k < N; k++) r.v[k] = f.a * g.v[k] + f.v[k] * g.a; return r;
}
template <int N> inline Jet<N> operator*(double s, const Jet<N>& g) {
  Jet<N> r; r.a = s * g.a; for (int k = 0; k < N; k++) r.v[k] = s * g.v[k]; return r;
}
// ceres: (a+u)/(b+v) = a/b + (u - (a/b) v)/b, evaluated through 1/b
template <int N> inline Jet<N> operator/(const Jet<N>& f, const Jet<N>& g) {
  const double ginv = 1.0 / g.a;
  const double fbyg = f.a * ginv;
  Jet<N> r; r.a = f.a * ginv;
  for (int k = 0; k < N; k++) r.v[k] = (f.v[k] - fbyg * g.v[k]) * ginv;
  return r;
}
template <int N> inline Jet<N> sqrt(const Jet<N>& f) {
  const double t = std::sqrt(f.a);
  const double two_t = t + t;
  Jet<N> r; r.a = t; for (int k = 0; k < N; k++) r.v[k] = f.v[k] / two_t; return r;
}
template <int N> inline bool operator<(const Jet<N>& f, double c) { return f.a < c; }
template <int N> inline bool operator>=(const Jet<N>& f, const Jet<N>& g) { return f.a >= g.a; }
// ceres jet.h: abs(f) = f < 0 ? -f : f; acos(f) = [acos a, -1 / sqrt(1 - a^2) v]; sin(f) = [sin a, cos a v]
template <int N> inline Jet<N> abs(const Jet<N>& f) { return f.a < 0 ? -f : f; }
template <int N> inline Jet<N> acos(const Jet<N>& f) {
  const double tmp = -1.0 / std::sqrt(1.0 - f.a * f.a);
  Jet<N> r; r.a = std::acos(f.a); for (int k = 0; k < N; k++) r.v[k] = tmp * f.v[k]; return r;
}
template <int N> inline Jet<N> sin(const Jet<N>& f) {
  const double c = std::cos(f.a);
  Jet<N> r; r.a = std::sin(f.a); for (int k = 0; k < N; k++) r.v[k] = c * f.v[k]; return r;
}
inline double abs(double x) { return std::fabs(x); }
inline double acos(double x) { return std::acos(x); }
inline double sin(double x) { return std::sin(x); }

inline double sqrt(double x) { return std::sqrt(x); }
inline bool lt0(double x) { return x < 0; }
template <int N> inline bool lt0(const Jet<N>& x) { return x.a < 0; }
inline double val(double x) { return x; }
template <int N> inline double val(const Jet<N>& x) { return x.a; }

template <typename T>
struct V3 {
  T x, y, z;
};
template <typename T> inline V3<T> operator+(const V3<T>& a, const V3<T>& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
template <typename T> inline V3<T> operator-(const V3<T>& a, const V3<T>& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <typename T> inline V3<T> cross(const V3<T>& a, const V3<T>& b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
template <typename T> inline T dot(const V3<T>& a, const V3<T>& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <typename T> inline T norm(const V3<T>& a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }

// Quaternion with coefficient storage (x, y, z, w), as Eigen::Quaternion / ceres para_q.
template <typename T>
struct Q4 {
  T x, y, z, w;
};

// Eigen's _transformVector: uv = 2 (q.vec × v); v' = v + w uv + q.vec × uv.
template <typename T> inline V3<T> rotate(const Q4<T>& q, const V3<T>& v) {
  V3<T> qv{q.x, q.y, q.z};
  V3<T> uv = cross(qv, v);
  uv = uv + uv;
  V3<T> wuv{q.w * uv.x, q.w * uv.y, q.w * uv.z};
  return (v + wuv) + cross(qv, uv);
}

// Identity.slerp(s, q) for s == 1 (DISTORTION 0, laserOdometry.cpp:82): Eigen's slerp returns
// exactly +q (or -q when w < 0) with the derivative of q; both rotate identically.
template <typename T> inline Q4<T> slerp_identity_s1(const Q4<T>& q) {
  if (lt0(q.w)) return Q4<T>{-q.x, -q.y, -q.z, -q.w};
  return q;
}

// Identity.slerp(s, q) for any s (DISTORTION 1: laserOdometry.cpp:82 with s = the point's relative
// time): Eigen 3.3's QuaternionBase::slerp, this = (0, 0, 0, 1), so this . q = w and the result is
// scale0 (0, 0, 0, 1) + scale1 q.
template <typename T> inline Q4<T> slerp_identity(double s, const Q4<T>& q) {
  const T one = T(1.0 - 2.220446049250313e-16);
  const T d = q.w;
  const T absD = abs(d);
  T scale0, scale1;
  if (absD >= one) {
    scale0 = T(1.0 - s);
    scale1 = T(s);
  } else {
    const T theta = acos(absD);
    const T sinTheta = sin(theta);
    scale0 = sin(T(1.0 - s) * theta) / sinTheta;
    scale1 = sin(T(s) * theta) / sinTheta;
  }
  if (lt0(d)) scale1 = -scale1;
  return Q4<T>{scale1 * q.x, scale1 * q.y, scale1 * q.z, scale0 + scale1 * q.w};
}

// Quaternion product a*b in the term grouping of Eigen 3.3's SSE2 quat_product<double>.
inline Q4<double> qmul(const Q4<double>& a, const Q4<double>& b) {
  Q4<double> r;
  r.x = (a.w * b.x + a.y * b.z) + (-(a.z * b.y - a.x * b.w));
  r.y = (a.w * b.y + a.y * b.w) + (a.z * b.x - a.x * b.z);
  r.z = (a.w * b.z - a.y * b.x) + (a.z * b.w + a.x * b.y);
  r.w = (a.w * b.w - a.y * b.y) + (-(a.z * b.z + a.x * b.x));
  return r;
}

}  // namespace oracle
