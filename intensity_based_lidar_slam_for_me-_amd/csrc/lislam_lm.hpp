// Device restatement of ceres::Solve(TRUST_REGION, LEVENBERG_MARQUARDT, DENSE_QR) for one
// 6-DoF pose (EigenQuaternionParameterization q + R^3 t) with Ceres 1.14 Solver::Options
// defaults, shared by the scan-to-scan odometry (laserOdometry.cpp:697-710, max 4 iterations),
// the ground-map optimization (mapOptimization.cpp:433-442, max 10) and laserMapping
// (laserMapping.cpp:836-845, max 4).
//
// A problem is a list of residual-block records (9 doubles) with a kind:
//   0 LidarEdgeFactor(curr, a, b, s=1)         rec = curr, a, b
//   1 LidarPlaneFactor(curr, j, l, m, s=1)     rec = curr, j, unit normal of the constructor
//   2 LidarPlaneNormFactor(curr, n, d)         rec = curr, n, d, -, -
//   3 front_end_residual(src, dst)             rec = src, dst, -, -, -
// every one under the same HuberLoss(0.1) (laserOdometry.cpp:424, laserMapping.cpp:646,
// mapOptimization.cpp:233).  One evaluation = cost, J^T J (21, upper) and J^T r (6) of the
// loss-corrected residuals in the local parameterization = 28 doubles ("acc").  The step logic
// (jacobi scaling fixed at iteration 0, LM diagonal clamp [1e-6, 1e32], initial radius 1e4,
// min_relative_decrease 1e-3, radius update 1/max(1/3, 1-(2 rho-1)^3), function / gradient /
// parameter tolerances 1e-6 / 1e-10 / 1e-8, 5 consecutive invalid steps = FAILURE) runs on one
// thread between evaluations; the augmented DENSE_QR system [J S; sqrt(D/radius)] is solved
// through its normal equations by Cholesky.
#pragma once
#include "lislam_device.hpp"
#include "lislam_factors.hpp"

namespace lislam {

constexpr int kAcc = 28;  // cost, J^T J upper (21), J^T r (6)

__device__ __forceinline__ void accum_row(double* acc, const double* J, double r) {
  int e = 1;
#pragma unroll
  for (int i = 0; i < 6; i++) {
#pragma unroll
    for (int j = i; j < 6; j++) acc[e++] += J[i] * J[j];
  }
#pragma unroll
  for (int i = 0; i < 6; i++) acc[22 + i] += J[i] * r;
}

// One residual block's contribution to acc at (q, t).
__device__ __forceinline__ void block_accum(int kd, const double* r9, const DQ& q, const D3& t, double* acc) {
  const double ha = 0.1;  // HuberLoss(0.1)
  const D3 c{r9[0], r9[1], r9[2]};
  if (kd == 0 || kd == 3) {
    double res[3], J[3][6];
    if (kd == 0)
      edge_factor(q, t, c, D3{r9[3], r9[4], r9[5]}, D3{r9[6], r9[7], r9[8]}, res, J);
    else
      p2p_factor(q, t, c, D3{r9[3], r9[4], r9[5]}, res, J);
    const double sc = huber_scale(ha, res[0] * res[0] + res[1] * res[1] + res[2] * res[2], &acc[0]);
    for (int k = 0; k < 3; k++) {
      double Js[6];
      for (int cc = 0; cc < 6; cc++) Js[cc] = J[k][cc] * sc;
      accum_row(acc, Js, res[k] * sc);
    }
  } else {
    double res, J[6];
    if (kd == 1)
      plane_factor(q, t, c, D3{r9[3], r9[4], r9[5]}, D3{r9[6], r9[7], r9[8]}, &res, J);
    else
      plane_norm_factor(q, t, c, D3{r9[3], r9[4], r9[5]}, r9[6], &res, J);
    const double sc = huber_scale(ha, res * res, &acc[0]);
    for (int cc = 0; cc < 6; cc++) J[cc] *= sc;
    accum_row(acc, J, res * sc);
  }
}

template <int kCtrl>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, kCtrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), kCtrl, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
// sum over the 16 lanes of each row (every lane of the row gets it)
__device__ __forceinline__ double row_sum(double v) {
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);  // row_half_mirror
  v += dpp_d<0x140>(v);  // row_mirror
  return v;
}

struct LM {
  double x[7], xc[7];
  double cost;
  double A[36], g[6];
  double scale[6], diag[6];
  double radius, dfac, mcc;
  int reuse;
  int it, invalid, term;
};

__device__ __forceinline__ void unpack(const double* acc, double* cost, double* A, double* g) {
  *cost = acc[0];
  int e = 1;
  for (int i = 0; i < 6; i++)
    for (int j = i; j < 6; j++) { A[i * 6 + j] = acc[e]; A[j * 6 + i] = acc[e]; e++; }
  for (int i = 0; i < 6; i++) g[i] = acc[22 + i];
}

// EigenQuaternionParameterization::Plus: x' = [sin|d| d/|d|, cos|d|] (x) x.
__device__ __forceinline__ void quat_plus(const double* x, const double* d, double* xp) {
  const double nd = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd > 0.0) {
    double sn, cs;
    sincos(nd, &sn, &cs);
    const double sdd = sn / nd;
    const DQ r = qmul(DQ{sdd * d[0], sdd * d[1], sdd * d[2], cs}, DQ{x[0], x[1], x[2], x[3]});
    xp[0] = r.x; xp[1] = r.y; xp[2] = r.z; xp[3] = r.w;
  } else {
    for (int k = 0; k < 4; k++) xp[k] = x[k];
  }
}
__device__ __forceinline__ void state_plus(const double* x, const double* d, double* xp) {
  quat_plus(x, d, xp);
  for (int k = 0; k < 3; k++) xp[4 + k] = x[4 + k] + d[3 + k];
}
__device__ __forceinline__ double grad_max_norm(const double* x, const double* g) {
  double ng[6], xp[7];
  for (int k = 0; k < 6; k++) ng[k] = -g[k];
  state_plus(x, ng, xp);
  double mx = 0;
  for (int k = 0; k < 7; k++) mx = fmax(mx, fabs(x[k] - xp[k]));
  return mx;
}

// (S A S + diag/radius) y = S g by Cholesky (the normal equations of Ceres' augmented DENSE_QR
// system [J S; sqrt(diag/radius)] y = [r; 0]).  The factor overwrites the packed lower triangle
// of the scaled matrix in place (row i at i (i + 1) / 2): 21 live doubles instead of 72, so the
// step fits the registers of a 16-wave workgroup's thread 0.  Each column divides once (1 / l_jj)
// and the factor and both substitutions multiply by that reciprocal: the serial step is
// issue- and latency-bound on one lane, and an fp64 division is ~10 dependent instructions.
__device__ __forceinline__ bool lm_solve(const LM& s, double* y) {
  double M[21], b[6], inv[6];
  for (int i = 0; i < 6; i++) {
    for (int j = 0; j <= i; j++) M[i * (i + 1) / 2 + j] = s.scale[i] * s.A[i * 6 + j] * s.scale[j];
    M[i * (i + 1) / 2 + i] += s.diag[i] / s.radius;
    b[i] = s.scale[i] * s.g[i];
  }
#pragma unroll
  for (int j = 0; j < 6; j++) {
    double d = M[j * (j + 1) / 2 + j];
#pragma unroll
    for (int k = 0; k < j; k++) d -= M[j * (j + 1) / 2 + k] * M[j * (j + 1) / 2 + k];
    if (!(d > 0)) return false;
    const double ljj = sqrt(d);
    inv[j] = 1.0 / ljj;  // one division per column; the column and both substitutions multiply
    M[j * (j + 1) / 2 + j] = ljj;
#pragma unroll
    for (int i = j + 1; i < 6; i++) {
      double v = M[i * (i + 1) / 2 + j];
#pragma unroll
      for (int k = 0; k < j; k++) v -= M[i * (i + 1) / 2 + k] * M[j * (j + 1) / 2 + k];
      M[i * (i + 1) / 2 + j] = v * inv[j];
    }
  }
  double z[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    double v = b[i];
#pragma unroll
    for (int k = 0; k < i; k++) v -= M[i * (i + 1) / 2 + k] * z[k];
    z[i] = v * inv[i];
  }
#pragma unroll
  for (int i = 5; i >= 0; i--) {
    double v = z[i];
#pragma unroll
    for (int k = i + 1; k < 6; k++) v -= M[k * (k + 1) / 2 + i] * y[k];
    y[i] = v * inv[i];
  }
  for (int i = 0; i < 6; i++)
    if (!isfinite(y[i])) return false;
  return true;
}

// Next candidate into s.xc (TrustRegionMinimizer + LevenbergMarquardtStrategy); false = stop.
__device__ __forceinline__ bool lm_propose(LM& s, int max_it) {
  while (s.it < max_it) {
    s.it++;
    if (!s.reuse)
      for (int c = 0; c < 6; c++) s.diag[c] = fmin(fmax(s.scale[c] * s.scale[c] * s.A[c * 6 + c], 1e-6), 1e32);
    double y[6] = {0, 0, 0, 0, 0, 0};
    const bool ok = lm_solve(s, y);
    s.reuse = 1;
    double step[6];
    for (int k = 0; k < 6; k++) step[k] = -y[k];
    double mcc = 0;
    if (ok) {
      double sg = 0, sAs = 0;
      for (int i = 0; i < 6; i++) {
        sg += step[i] * s.scale[i] * s.g[i];
        double row = 0;
        for (int j = 0; j < 6; j++) row += s.scale[i] * s.A[i * 6 + j] * s.scale[j] * step[j];
        sAs += step[i] * row;
      }
      mcc = -(sg + 0.5 * sAs);
    }
    if (!ok || !(mcc > 0.0)) {  // invalid step: rejected-step radius update, solve again
      if (++s.invalid >= 5) { s.term = 2; return false; }
      s.radius /= s.dfac;
      s.dfac *= 2.0;
      s.reuse = 1;
      continue;
    }
    s.invalid = 0;
    double delta[6];
    for (int k = 0; k < 6; k++) delta[k] = step[k] * s.scale[k];
    state_plus(s.x, delta, s.xc);
    s.mcc = mcc;
    return true;
  }
  s.term = 0;  // NO_CONVERGENCE: max_num_iterations
  return false;
}

// After the evaluation at x0 (acc): initialize, test the gradient and propose the first
// candidate (s.xc).  Returns whether a candidate must be evaluated.
__device__ __forceinline__ bool lm_start(LM& s, const double* x0, const double* acc, int max_it) {
  for (int e = 0; e < 7; e++) s.x[e] = x0[e];
  unpack(acc, &s.cost, s.A, s.g);
  for (int cc = 0; cc < 6; cc++) s.scale[cc] = 1.0 / (1.0 + sqrt(s.A[cc * 6 + cc]));  // jacobi scaling
  s.radius = 1e4; s.dfac = 2.0; s.reuse = 0; s.mcc = 0;
  s.it = 0; s.invalid = 0; s.term = 0;
  bool cont = isfinite(s.cost) && !(grad_max_norm(s.x, s.g) <= 1e-10);
  if (!isfinite(s.cost)) s.term = 2; else if (!cont) s.term = 1;
  if (cont) cont = lm_propose(s, max_it);
  return cont;
}

// After the evaluation at the candidate s.xc (acc): accept / reject, tolerances, next
// candidate.  Returns whether another candidate must be evaluated.
__device__ __forceinline__ bool lm_next(LM& s, const double* acc, int max_it) {
  double ccost = acc[0];
  if (!isfinite(ccost)) ccost = 1.7976931348623157e308;
  bool cont = true;
  double xn = 0, sn = 0;
  for (int e = 0; e < 7; e++) { xn += s.x[e] * s.x[e]; sn += (s.x[e] - s.xc[e]) * (s.x[e] - s.xc[e]); }
  xn = sqrt(xn); sn = sqrt(sn);
  if (sn <= 1e-8 * (xn + 1e-8)) { s.term = 1; cont = false; }                      // parameter_tolerance
  else if (fabs(s.cost - ccost) <= 1e-6 * s.cost) { s.term = 1; cont = false; }   // function_tolerance
  else {
    const double rel = (s.cost - ccost) / s.mcc;
    if (rel > 1e-3) {  // min_relative_decrease: accept
      for (int e = 0; e < 7; e++) s.x[e] = s.xc[e];
      double unused;
      unpack(acc, &unused, s.A, s.g);
      s.cost = ccost;
      const double t3 = 2.0 * rel - 1.0;
      s.radius = fmin(1e16, s.radius / fmax(1.0 / 3.0, 1.0 - t3 * t3 * t3));
      s.dfac = 2.0;
      s.reuse = 0;
      if (grad_max_norm(s.x, s.g) <= 1e-10) { s.term = 1; cont = false; }       // gradient_tolerance
    } else {           // reject
      s.radius /= s.dfac;
      s.dfac *= 2.0;
      s.reuse = 1;
    }
    if (cont && s.radius <= 1e-32) { s.term = 1; cont = false; }
  }
  if (cont) cont = lm_propose(s, max_it);
  return cont;
}

}  // namespace lislam
