// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.hpp).
//
// Cost functors (src/lidarFeaturePointsFunction.hpp) with Ceres-style autodiff, the residual
// block evaluator and the Ceres 1.14 LM restatement shared by the odometry (oracle_odom.cpp) and
// mapping (oracle_map.cpp) restatements.
#pragma once
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "oracle_common.hpp"
#include "oracle_jet.hpp"

namespace oracle {

// ------------------------------------------------------------------ functors (a15-a17, a11)
// Same constructor arguments and operator()(q, t, residual) shape as the reference functors.
struct EdgeFactor {  // LidarEdgeFactor, lidarFeaturePointsFunction.hpp:243-293
  double cp[3], pa[3], pb[3], s;
  static constexpr int kResiduals = 3;
  template <typename T>
  bool operator()(const T* q, const T* t, T* residual) const {
    V3<T> c{T(cp[0]), T(cp[1]), T(cp[2])};
    V3<T> a{T(pa[0]), T(pa[1]), T(pa[2])};
    V3<T> b{T(pb[0]), T(pb[1]), T(pb[2])};
    const Q4<T> q0{q[0], q[1], q[2], q[3]};
    Q4<T> qq = s == 1.0 ? slerp_identity_s1(q0) : slerp_identity(s, q0);
    V3<T> tt{T(s) * t[0], T(s) * t[1], T(s) * t[2]};
    V3<T> lp = rotate(qq, c) + tt;
    V3<T> nu = cross(lp - a, lp - b);
    V3<T> de = a - b;
    residual[0] = nu.x / norm(de);
    residual[1] = nu.y / norm(de);
    residual[2] = nu.z / norm(de);
    return true;
  }
};

struct PlaneFactor {  // LidarPlaneFactor, lidarFeaturePointsFunction.hpp:143-196
  double cp[3], pj[3], n[3], s;
  static constexpr int kResiduals = 1;
  PlaneFactor() : cp{0, 0, 0}, pj{0, 0, 0}, n{0, 0, 0}, s(1.0) {}
  PlaneFactor(const double* c, const double* j, const double* l, const double* m, double s_) : s(s_) {
    for (int k = 0; k < 3; k++) { cp[k] = c[k]; pj[k] = j[k]; }
    V3<double> jl{j[0] - l[0], j[1] - l[1], j[2] - l[2]};
    V3<double> jm{j[0] - m[0], j[1] - m[1], j[2] - m[2]};
    V3<double> nn = cross(jl, jm);
    double sq = nn.x * nn.x + nn.y * nn.y + nn.z * nn.z;  // Eigen normalize()
    if (sq > 0) { double r = std::sqrt(sq); nn.x /= r; nn.y /= r; nn.z /= r; }
    n[0] = nn.x; n[1] = nn.y; n[2] = nn.z;
  }
  template <typename T>
  bool operator()(const T* q, const T* t, T* residual) const {
    V3<T> c{T(cp[0]), T(cp[1]), T(cp[2])};
    V3<T> j{T(pj[0]), T(pj[1]), T(pj[2])};
    V3<T> nn{T(n[0]), T(n[1]), T(n[2])};
    const Q4<T> q0{q[0], q[1], q[2], q[3]};
    Q4<T> qq = s == 1.0 ? slerp_identity_s1(q0) : slerp_identity(s, q0);
    V3<T> tt{T(s) * t[0], T(s) * t[1], T(s) * t[2]};
    V3<T> lp = rotate(qq, c) + tt;
    residual[0] = dot(lp - j, nn);
    return true;
  }
};

struct PlaneNormFactor {  // LidarPlaneNormFactor, lidarFeaturePointsFunction.hpp:199-240
  double cp[3], n[3], d;
  static constexpr int kResiduals = 1;
  template <typename T>
  bool operator()(const T* q, const T* t, T* residual) const {
    Q4<T> qq{q[0], q[1], q[2], q[3]};
    V3<T> c{T(cp[0]), T(cp[1]), T(cp[2])};
    V3<T> pw = rotate(qq, c) + V3<T>{t[0], t[1], t[2]};
    V3<T> nn{T(n[0]), T(n[1]), T(n[2])};
    residual[0] = dot(nn, pw) + T(d);
    return true;
  }
};

struct P2PFactor {  // front_end_residual, lidarFeaturePointsFunction.hpp:21-58
  double src[3], dst[3];
  static constexpr int kResiduals = 3;
  template <typename T>
  bool operator()(const T* q, const T* t, T* residual) const {
    Q4<T> qq{q[0], q[1], q[2], q[3]};
    V3<T> cp{T(src[0]), T(src[1]), T(src[2])};
    V3<T> p = rotate(qq, cp) + V3<T>{t[0], t[1], t[2]};
    residual[0] = p.x - T(dst[0]);
    residual[1] = p.y - T(dst[1]);
    residual[2] = p.z - T(dst[2]);
    return true;
  }
};

// AutoDiffCostFunction<F, R, 4, 3>::Evaluate: residuals, and the 7-column global Jacobian.
template <typename F>
static void autodiff_eval(const F& f, const double* q, const double* t, double* r, double* J /*R x 7 or null*/) {
  constexpr int R = F::kResiduals;
  if (!J) {
    f(q, t, r);
    return;
  }
  Jet<7> qj[4], tj[3], rj[R];
  for (int k = 0; k < 4; k++) qj[k] = Jet<7>(q[k], k);
  for (int k = 0; k < 3; k++) tj[k] = Jet<7>(t[k], 4 + k);
  f(qj, tj, rj);
  for (int i = 0; i < R; i++) {
    r[i] = rj[i].a;
    for (int k = 0; k < 7; k++) J[i * 7 + k] = rj[i].v[k];
  }
}

// ceres::EigenQuaternionParameterization::ComputeJacobian (4 x 3, row-major), x = [x y z w].
static void quat_plus_jacobian(const double* x, double* P) {
  P[0] = x[3];  P[1] = x[2];  P[2] = -x[1];
  P[3] = -x[2]; P[4] = x[3];  P[5] = x[0];
  P[6] = x[1];  P[7] = -x[0]; P[8] = x[3];
  P[9] = -x[0]; P[10] = -x[1]; P[11] = -x[2];
}

// ceres::EigenQuaternionParameterization::Plus: x' = [sin|d| d/|d|, cos|d|] (x) x.
static void quat_plus(const double* x, const double* d, double* xp) {
  const double nd = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd > 0.0) {
    const double sdd = std::sin(nd) / nd;
    Q4<double> dq{sdd * d[0], sdd * d[1], sdd * d[2], std::cos(nd)};
    Q4<double> xq{x[0], x[1], x[2], x[3]};
    Q4<double> r = qmul(dq, xq);
    xp[0] = r.x; xp[1] = r.y; xp[2] = r.z; xp[3] = r.w;
  } else {
    for (int k = 0; k < 4; k++) xp[k] = x[k];
  }
}

// ------------------------------------------------------------------ residual blocks + evaluator
struct Block {
  int kind;  // 0 edge, 1 plane, 2 plane-norm, 3 point-to-point (front_end_residual)
  EdgeFactor e;
  PlaneFactor p;
  PlaneNormFactor pn;
  P2PFactor pp;
  int nres() const { return (kind == 0 || kind == 3) ? 3 : 1; }
};

// ceres::HuberLoss(a).Evaluate(s, rho)
static void huber(double a, double s, double rho[3]) {
  const double b = a * a;
  if (s > b) {
    const double r = std::sqrt(s);
    rho[0] = 2.0 * a * r - b;
    rho[1] = std::max(std::numeric_limits<double>::min(), a / r);
    rho[2] = -rho[1] / (2.0 * s);
  } else {
    rho[0] = s; rho[1] = 1.0; rho[2] = 0.0;
  }
}

struct Problem {
  std::vector<Block> blocks;
  double huber_a = 0.1;
  int rows() const {
    int n = 0;
    for (const Block& b : blocks) n += b.nres();
    return n;
  }
  // ProgramEvaluator: cost = sum 0.5 rho(|r|^2); with J: loss-corrected r and local J (rows x 6),
  // gradient g = J^T r.  x = [q(4), t(3)].
  bool evaluate(const double* x, double* cost, std::vector<double>* res, std::vector<double>* J,
                double* g) const {
    const double* q = x;
    const double* t = x + 4;
    double P[12];
    quat_plus_jacobian(q, P);
    int row = 0;
    double c = 0;
    if (g) for (int k = 0; k < 6; k++) g[k] = 0;
    for (const Block& b : blocks) {
      const int R = b.nres();
      double r[3], Jg[21];
      double* jp = J ? Jg : nullptr;
      if (b.kind == 0) autodiff_eval(b.e, q, t, r, jp);
      else if (b.kind == 1) autodiff_eval(b.p, q, t, r, jp);
      else if (b.kind == 2) autodiff_eval(b.pn, q, t, r, jp);
      else autodiff_eval(b.pp, q, t, r, jp);
      double sq = 0;
      for (int i = 0; i < R; i++) sq += r[i] * r[i];
      double rho[3];
      huber(huber_a, sq, rho);
      c += 0.5 * rho[0];
      if (res || J) {
        const double scale = std::sqrt(rho[1]);  // Corrector with rho'' <= 0
        for (int i = 0; i < R; i++) {
          double Jl[6];
          if (J) {
            for (int cc = 0; cc < 3; cc++) {
              double acc = 0;
              for (int k = 0; k < 4; k++) acc += Jg[i * 7 + k] * P[k * 3 + cc];
              Jl[cc] = acc;
            }
            for (int cc = 0; cc < 3; cc++) Jl[3 + cc] = Jg[i * 7 + 4 + cc];
            for (int cc = 0; cc < 6; cc++) (*J)[(size_t)(row + i) * 6 + cc] = Jl[cc] * scale;
          }
          if (res) (*res)[row + i] = r[i] * scale;
        }
        if (g && J)
          for (int i = 0; i < R; i++)
            for (int cc = 0; cc < 6; cc++) g[cc] += (*J)[(size_t)(row + i) * 6 + cc] * (*res)[row + i];
      }
      row += R;
    }
    *cost = c;
    return std::isfinite(c);
  }
};

// Householder least squares: argmin |A y - b|, A is m x 6 (m >= 6), row-major.
static bool householder_lsq(std::vector<double> A, std::vector<double> b, int m, double* y) {
  const int n = 6;
  for (int k = 0; k < n; k++) {
    double nrm = 0;
    for (int i = k; i < m; i++) nrm += A[i * n + k] * A[i * n + k];
    nrm = std::sqrt(nrm);
    if (nrm == 0) continue;
    const double alpha = A[k * n + k] > 0 ? -nrm : nrm;
    std::vector<double> v(m - k);
    for (int i = k; i < m; i++) v[i - k] = A[i * n + k];
    v[0] -= alpha;
    double vn = 0;
    for (double e : v) vn += e * e;
    if (vn == 0) continue;
    for (int j = k; j < n; j++) {
      double s = 0;
      for (int i = k; i < m; i++) s += v[i - k] * A[i * n + j];
      s = 2 * s / vn;
      for (int i = k; i < m; i++) A[i * n + j] -= s * v[i - k];
    }
    double s = 0;
    for (int i = k; i < m; i++) s += v[i - k] * b[i];
    s = 2 * s / vn;
    for (int i = k; i < m; i++) b[i] -= s * v[i - k];
  }
  for (int k = n - 1; k >= 0; k--) {
    double s = b[k];
    for (int j = k + 1; j < n; j++) s -= A[k * n + j] * y[j];
    if (A[k * n + k] == 0) return false;
    y[k] = s / A[k * n + k];
  }
  for (int k = 0; k < n; k++)
    if (!std::isfinite(y[k])) return false;
  return true;
}

static void state_plus(const double* x, const double* d, double* xp) {
  quat_plus(x, d, xp);
  for (int k = 0; k < 3; k++) xp[4 + k] = x[4 + k] + d[3 + k];
}

struct SolveSummary {
  int iterations = 0, successful = 0;
  int termination = 0;  // 0 no-convergence, 1 convergence, 2 failure
  double initial_cost = 0, final_cost = 0;
};

// ceres::Solve with TRUST_REGION / LEVENBERG_MARQUARDT / DENSE_QR and Solver::Options defaults
// (initial radius 1e4, min_relative_decrease 1e-3, function/gradient/parameter tolerances
// 1e-6/1e-10/1e-8, jacobi_scaling, monotonic steps).
static SolveSummary ceres_solve(const Problem& prob, double* x /*7*/, int max_iterations) {
  SolveSummary sum;
  const int m = prob.rows();
  if (m == 0) { sum.termination = 1; return sum; }
  std::vector<double> r(m), J((size_t)m * 6), rc(m), Jc((size_t)m * 6);
  double g[6], cost;
  if (!prob.evaluate(x, &cost, &r, &J, g)) { sum.termination = 2; return sum; }
  sum.initial_cost = cost;
  // jacobi scaling from iteration 0's Jacobian
  double scale[6];
  for (int c = 0; c < 6; c++) {
    double s = 0;
    for (int i = 0; i < m; i++) s += J[(size_t)i * 6 + c] * J[(size_t)i * 6 + c];
    scale[c] = 1.0 / (1.0 + std::sqrt(s));
  }
  auto scale_cols = [&](std::vector<double>& JJ) {
    for (int i = 0; i < m; i++)
      for (int c = 0; c < 6; c++) JJ[(size_t)i * 6 + c] *= scale[c];
  };
  auto grad_max_norm = [&](const double* xx, const double* gg) {
    double ng[6], xp[7];
    for (int k = 0; k < 6; k++) ng[k] = -gg[k];
    state_plus(xx, ng, xp);
    double mx = 0;
    for (int k = 0; k < 7; k++) mx = std::max(mx, std::fabs(xx[k] - xp[k]));
    return mx;
  };
  scale_cols(J);
  double radius = 1e4, decrease_factor = 2.0;
  bool reuse_diagonal = false;
  double diag[6];
  if (grad_max_norm(x, g) <= 1e-10) { sum.termination = 1; sum.final_cost = cost; return sum; }
  int invalid_steps = 0;
  for (int it = 1; it <= max_iterations; it++) {
    sum.iterations = it;
    // LevenbergMarquardtStrategy::ComputeStep
    if (!reuse_diagonal) {
      for (int c = 0; c < 6; c++) {
        double s = 0;
        for (int i = 0; i < m; i++) s += J[(size_t)i * 6 + c] * J[(size_t)i * 6 + c];
        diag[c] = std::min(std::max(s, 1e-6), 1e32);
      }
    }
    std::vector<double> A((size_t)(m + 6) * 6, 0.0), b(m + 6, 0.0);
    std::memcpy(A.data(), J.data(), sizeof(double) * m * 6);
    for (int c = 0; c < 6; c++) A[(size_t)(m + c) * 6 + c] = std::sqrt(diag[c] / radius);
    for (int i = 0; i < m; i++) b[i] = r[i];
    double y[6] = {0, 0, 0, 0, 0, 0};
    bool ok = householder_lsq(A, b, m + 6, y);
    reuse_diagonal = true;
    double step[6];
    for (int k = 0; k < 6; k++) step[k] = -y[k];
    // model cost change = -(J step)'(r + J step / 2)
    double mcc = 0;
    if (ok) {
      for (int i = 0; i < m; i++) {
        double mr = 0;
        for (int c = 0; c < 6; c++) mr += J[(size_t)i * 6 + c] * step[c];
        mcc += mr * (r[i] + mr / 2.0);
      }
      mcc = -mcc;
    }
    if (!ok || !(mcc > 0.0)) {  // invalid step: treated as a rejected step
      if (++invalid_steps >= 5) { sum.termination = 2; break; }
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      reuse_diagonal = true;
      continue;
    }
    invalid_steps = 0;
    double delta[6], xc[7];
    for (int k = 0; k < 6; k++) delta[k] = step[k] * scale[k];
    state_plus(x, delta, xc);
    double ccost;
    if (!prob.evaluate(xc, &ccost, nullptr, nullptr, nullptr)) ccost = DBL_MAX;
    // ParameterToleranceReached
    double xn = 0, sn = 0;
    for (int k = 0; k < 7; k++) { xn += x[k] * x[k]; sn += (x[k] - xc[k]) * (x[k] - xc[k]); }
    xn = std::sqrt(xn); sn = std::sqrt(sn);
    if (sn <= 1e-8 * (xn + 1e-8)) { sum.termination = 1; break; }
    // FunctionToleranceReached
    if (std::fabs(cost - ccost) <= 1e-6 * cost) { sum.termination = 1; break; }
    const double rel = (cost - ccost) / mcc;
    if (rel > 1e-3) {
      std::memcpy(x, xc, sizeof(double) * 7);
      prob.evaluate(x, &cost, &r, &J, g);
      scale_cols(J);
      radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rel - 1.0, 3));
      radius = std::min(1e16, radius);
      decrease_factor = 2.0;
      reuse_diagonal = false;
      sum.successful++;
      if (grad_max_norm(x, g) <= 1e-10) { sum.termination = 1; break; }
    } else {
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      reuse_diagonal = true;
    }
    if (radius <= 1e-32) { sum.termination = 1; break; }
  }
  sum.final_cost = cost;
  return sum;
}

}  // namespace oracle
