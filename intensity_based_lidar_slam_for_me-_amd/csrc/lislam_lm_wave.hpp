// The Ceres-semantics LM step of lislam_lm.hpp (same decisions) as a short dependent chain for one
// wavefront, its state in LDS: the chain engine's solve role (lislam_odometry.hip) and the
// laserMapping / mapOptimization / pose solve (k_lm_evalstep, lislam_map.hip) both take their steps
// with it.  Every lane of the wave runs the same scalar code.
#pragma once
#include <hip/hip_runtime.h>

#include "lislam_lm.hpp"

namespace lislam {

// ---- the step logic of lislam_lm.hpp (Ceres 1.14 LM, same decisions), on every lane of wave 0.
// Written for a short dependent chain (fp64 on gfx950: ~32 cycles per dependent operation):
// - the 6x6 system by its 3x3 blocks: adjugate inverse of the rotation block, Schur complement of
//   the translation block, adjugate again (positive definiteness by the leading minors of both:
//   Sylvester, the same test as a Cholesky's positive pivots);
// - 1 / radius carried beside radius (scaled by the same powers of two and the same factor m);
// - rel by the reciprocal of the model cost change, computed while the candidate is evaluated;
// - the parameter tolerance of a candidate decided while it is evaluated;
// - sin|d|/|d| and cos|d| of EigenQuaternionParameterization's plus by Estrin's scheme.
struct EngLM {
  double x[7], xc[7], A[21], g[6], scale[6], iscale[6], diag[6];
  double cost, radius, ir, dfac, mcc, imcc;
  int reuse, it, invalid, term, ptol;
};

__device__ __forceinline__ double rcp_d(double d) {  // 1 / d to ~1 ulp (d normal, nonzero)
  double y = __builtin_amdgcn_rcp(d);
  y = fma(fma(-d, y, 1.0), y, y);
  y = fma(fma(-d, y, 1.0), y, y);
  return y;
}
__device__ __forceinline__ double rsqrt_d(double d) {  // 1 / sqrt(d), d > 0, to ~1 ulp
  double y = __builtin_amdgcn_rsq(d);
  y = y * fma(-0.5 * d, y * y, 1.5);
  y = y * fma(-0.5 * d, y * y, 1.5);
  return y;
}
__device__ __noinline__ void sincos_slow(double n2, double* sdd, double* cs) {
  const double nd = sqrt(n2);
  double sn;
  sincos(nd, &sn, cs);
  *sdd = sn / nd;
}
// x' = [sin|d| d/|d|, cos|d|] (x) x (quaternion part of the state plus)
__device__ __forceinline__ void eng_quat_plus(const double* x, const double* d, double* xp) {
  const double n2 = fma(d[0], d[0], fma(d[1], d[1], d[2] * d[2]));
  if (!(n2 > 0.0)) {
    for (int k = 0; k < 4; k++) xp[k] = x[k];
    return;
  }
  double sdd, cs;
  if (n2 <= 0.25) {  // Taylor series in n2 to x^16 (truncation < 1e-19), Estrin's scheme
    const double z2 = n2 * n2, z4 = z2 * z2, z8 = z4 * z4;
    sdd = fma(z8, 2.8114572543455206e-15,
              fma(z4, fma(z2, fma(n2, -7.6471637318198164e-13, 1.6059043836821613e-10),
                          fma(n2, -2.5052108385441720e-08, 2.7557319223985893e-06)),
                  fma(z2, fma(n2, -1.9841269841269841e-04, 8.3333333333333333e-03), fma(n2, -1.6666666666666666e-01, 1.0))));
    cs = fma(z8, 4.7794773323873853e-14,
             fma(z4, fma(z2, fma(n2, -1.1470745597729725e-11, 2.0876756987868099e-09),
                         fma(n2, -2.7557319223985888e-07, 2.4801587301587302e-05)),
                 fma(z2, fma(n2, -1.3888888888888889e-03, 4.1666666666666664e-02), fma(n2, -0.5, 1.0))));
  } else {
    sincos_slow(n2, &sdd, &cs);
  }
  const double ax = sdd * d[0], ay = sdd * d[1], az = sdd * d[2];
  // (a, cs) (x) (x0..x3): pairwise sums (depth 3)
  xp[0] = fma(cs, x[0], ax * x[3]) + fma(ay, x[2], -az * x[1]);
  xp[1] = fma(cs, x[1], ay * x[3]) + fma(az, x[0], -ax * x[2]);
  xp[2] = fma(cs, x[2], az * x[3]) + fma(ax, x[1], -ay * x[0]);
  xp[3] = fma(cs, x[3], -ax * x[0]) - fma(ay, x[1], az * x[2]);
}
// grad_max_norm(x, g) <= 1e-10: max_k |x_k - (x (+) -g)_k|
__device__ __forceinline__ bool eng_grad_small(const double* x, const double* g) {
  double mx = 0.0;
  for (int k = 0; k < 3; k++) mx = fmax(mx, fabs(x[4 + k] - (x[4 + k] + -g[3 + k])));
  if (mx > 1e-10) return false;  // the rotation part only raises the maximum
  const double ng[3] = {-g[0], -g[1], -g[2]};
  double xp[4];
  eng_quat_plus(x, ng, xp);
  for (int k = 0; k < 4; k++) mx = fmax(mx, fabs(x[k] - xp[k]));
  return mx <= 1e-10;
}
// packed upper index of (i, j), i <= j
__device__ __forceinline__ constexpr int pu(int i, int j) { return i * 6 - i * (i - 1) / 2 + (j - i); }

// Adjugate of a symmetric 3x3 [[a, b, c], [b, d, e], [c, e, f]]: cofactors (symmetric) and det.
struct Sym3Inv {
  double c00, c01, c02, c11, c12, c22, det;
};
__device__ __forceinline__ Sym3Inv sym3_adj(double a, double b, double c, double d, double e, double f) {
  Sym3Inv r;
  r.c00 = fma(d, f, -e * e);
  r.c01 = fma(c, e, -b * f);
  r.c02 = fma(b, e, -c * d);
  r.c11 = fma(a, f, -c * c);
  r.c12 = fma(b, c, -a * e);
  r.c22 = fma(a, d, -b * b);
  r.det = fma(a, r.c00, fma(b, r.c01, c * r.c02));
  return r;
}

// Solve M y = b, M = A (packed upper, 6x6) + diag(Dr); false = not positive definite.
__device__ __forceinline__ bool solve6(const double* A, const double* Dr, const double* b, double* y) {
  // P (rotation block 0..2), Q (0..2 x 3..5), S (translation block 3..5)
  const double p00 = A[pu(0, 0)] + Dr[0], p01 = A[pu(0, 1)], p02 = A[pu(0, 2)];
  const double p11 = A[pu(1, 1)] + Dr[1], p12 = A[pu(1, 2)], p22 = A[pu(2, 2)] + Dr[2];
  double Q[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) Q[i][j] = A[pu(i, 3 + j)];
  const Sym3Inv P = sym3_adj(p00, p01, p02, p11, p12, p22);
  const double ip = rcp_d(P.det);
  const double adjP[3][3] = {{P.c00, P.c01, P.c02}, {P.c01, P.c11, P.c12}, {P.c02, P.c12, P.c22}};
  // W = P^-1 Q, u1 = P^-1 b1
  double W[3][3], u1[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
#pragma unroll
    for (int j = 0; j < 3; j++) W[i][j] = fma(adjP[i][0], Q[0][j], fma(adjP[i][1], Q[1][j], adjP[i][2] * Q[2][j])) * ip;
    u1[i] = fma(adjP[i][0], b[0], fma(adjP[i][1], b[1], adjP[i][2] * b[2])) * ip;
  }
  // Schur complement S' = S - Q^T W, h = b2 - Q^T u1
  double Sp[3][3], h[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
#pragma unroll
    for (int j = i; j < 3; j++) {
      const double sij = A[pu(3 + i, 3 + j)] + (i == j ? Dr[3 + i] : 0.0);
      Sp[i][j] = sij - fma(Q[0][i], W[0][j], fma(Q[1][i], W[1][j], Q[2][i] * W[2][j]));
    }
    h[i] = b[3 + i] - fma(Q[0][i], u1[0], fma(Q[1][i], u1[1], Q[2][i] * u1[2]));
  }
  const Sym3Inv S = sym3_adj(Sp[0][0], Sp[0][1], Sp[0][2], Sp[1][1], Sp[1][2], Sp[2][2]);
  const double is = rcp_d(S.det);
  const double adjS[3][3] = {{S.c00, S.c01, S.c02}, {S.c01, S.c11, S.c12}, {S.c02, S.c12, S.c22}};
#pragma unroll
  for (int i = 0; i < 3; i++) y[3 + i] = fma(adjS[i][0], h[0], fma(adjS[i][1], h[1], adjS[i][2] * h[2])) * is;
  // y1 = u1 - W y2
#pragma unroll
  for (int i = 0; i < 3; i++) y[i] = u1[i] - fma(W[i][0], y[3], fma(W[i][1], y[4], W[i][2] * y[5]));
  // Sylvester: leading minors of P and of S' positive <=> M positive definite
  return p00 > 0.0 && P.c22 > 0.0 && P.det > 0.0 && Sp[0][0] > 0.0 && S.c22 > 0.0 && S.det > 0.0;
}

typedef __attribute__((address_space(3))) EngLM LdsLM;

// Propose the next candidate into s.xc; false = stop (s.term set).  Ceres solves (S A S + D /
// radius) y = S g and steps -S y (S the Jacobi scaling, D its clamped diagonal).  With z = S y that
// is (A + S^-1 D S^-1 / radius) z = g, step -z, and the model cost change 0.5 (z.g + z.(D' /
// radius) z), D' = S^-1 D S^-1 (s.diag): the same system without scaling the matrix.
// A / g: the current evaluation (registers) -- s.A / s.g hold the same values.
__device__ __forceinline__ bool eng_propose(LdsLM& s, const double* A, const double* g, int max_it) {
  int it = s.it, invalid = s.invalid, reuse = s.reuse;
  double radius = s.radius, ir = s.ir, dfac = s.dfac;
  double diag[6];
#pragma unroll
  for (int e = 0; e < 6; e++) diag[e] = s.diag[e];
  bool out = false;
  int term = 0;
  while (it < max_it) {
    it++;
    if (!reuse)
#pragma unroll
      for (int e = 0; e < 6; e++) diag[e] = fmin(fmax(s.scale[e] * A[pu(e, e)], 1e-6), 1e32) * s.iscale[e];
    reuse = 1;
    double Dr[6], y[6];
#pragma unroll
    for (int e = 0; e < 6; e++) Dr[e] = diag[e] * ir;
    bool ok = solve6(A, Dr, g, y);
    double yb = 0.0, yd = 0.0;
#pragma unroll
    for (int i = 0; i < 6; i++) { ok = ok && isfinite(y[i]); yb = fma(y[i], g[i], yb); yd = fma(y[i] * Dr[i], y[i], yd); }
    const double mcc = ok ? 0.5 * (yb + yd) : 0.0;
    if (!ok || !(mcc > 0.0)) {  // invalid step: rejected-step radius update, solve again
      if (++invalid >= 5) { term = 2; break; }
      radius /= dfac;
      ir *= dfac;  // dfac: a power of two, exact
      dfac *= 2.0;
      continue;
    }
    invalid = 0;
    double delta[6], x[7], xc[7];
#pragma unroll
    for (int k = 0; k < 6; k++) delta[k] = -y[k];
#pragma unroll
    for (int k = 0; k < 7; k++) x[k] = s.x[k];
    eng_quat_plus(x, delta, xc);
#pragma unroll
    for (int k = 0; k < 3; k++) xc[4 + k] = x[4 + k] + delta[3 + k];
#pragma unroll
    for (int k = 0; k < 7; k++) s.xc[k] = xc[k];
    s.mcc = mcc;
    out = true;
    break;
  }
  s.it = it; s.invalid = invalid; s.reuse = reuse;
  s.radius = radius; s.ir = ir; s.dfac = dfac;
#pragma unroll
  for (int e = 0; e < 6; e++) s.diag[e] = diag[e];
  if (!out) s.term = term;  // 0 NO_CONVERGENCE (max_num_iterations) or 2 FAILURE
  return out;
}

// After the evaluation at x0 (first) or at the candidate s.xc (acc, lislam_lm.hpp layout):
// lm_start / lm_next, then one propose.  Returns whether a candidate (s.xc) must be evaluated.
__device__ __forceinline__ bool eng_step(LdsLM& s, const double* x0, const double (&acc)[kAcc], bool first, int max_it) {
  const double* Aa = acc + 1;
  const double* ga = acc + 22;
  if (first) {
    double x[7];
#pragma unroll
    for (int e = 0; e < 7; e++) { x[e] = x0[e]; s.x[e] = x[e]; }
    s.cost = acc[0];
#pragma unroll
    for (int e = 0; e < 21; e++) s.A[e] = Aa[e];
#pragma unroll
    for (int e = 0; e < 6; e++) s.g[e] = ga[e];
#pragma unroll
    for (int e = 0; e < 6; e++) {  // jacobi scaling S = 1 / (1 + sqrt(A_ee)), kept as S^2 and 1 / S^2
      const double r = 1.0 + sqrt(Aa[pu(e, e)]);
      const double sc = 1.0 / r;
      s.scale[e] = sc * sc;
      s.iscale[e] = r * r;
    }
    s.radius = 1e4; s.ir = 1.0 / 1e4; s.dfac = 2.0; s.reuse = 0; s.mcc = 0; s.imcc = 0;
    s.it = 0; s.invalid = 0; s.term = 0; s.ptol = 0;
    if (!isfinite(acc[0])) { s.term = 2; return false; }
    if (eng_grad_small(x, ga)) { s.term = 1; return false; }
    return eng_propose(s, Aa, ga, max_it);
  }
  double ccost = acc[0];
  if (!isfinite(ccost)) ccost = 1.7976931348623157e308;
  const double cost = s.cost;
  if (s.ptol) { s.term = 1; return false; }                                   // parameter_tolerance
  if (fabs(cost - ccost) <= 1e-6 * cost) { s.term = 1; return false; }        // function_tolerance
  const double rel = (cost - ccost) * s.imcc;
  if (rel > 1e-3) {  // min_relative_decrease: accept
    double xc[7];
#pragma unroll
    for (int e = 0; e < 7; e++) { xc[e] = s.xc[e]; s.x[e] = xc[e]; }
#pragma unroll
    for (int e = 0; e < 21; e++) s.A[e] = Aa[e];
#pragma unroll
    for (int e = 0; e < 6; e++) s.g[e] = ga[e];
    s.cost = ccost;
    const double t3 = fma(2.0, rel, -1.0);
    const double m = fmax(1.0 / 3.0, 1.0 - t3 * t3 * t3);
    const double radius = fmin(1e16, s.radius / m);
    s.radius = radius;
    s.ir = fmax(1e-16, s.ir * m);
    s.dfac = 2.0;
    s.reuse = 0;
    if (eng_grad_small(xc, ga)) { s.term = 1; return false; }                 // gradient_tolerance
    if (radius <= 1e-32) { s.term = 1; return false; }
    return eng_propose(s, Aa, ga, max_it);
  }
  // reject: the current point's matrix (s.A, s.g) with a smaller radius
  const double dfac = s.dfac;
  s.radius = s.radius / dfac;
  s.ir = s.ir * dfac;
  s.dfac = dfac * 2.0;
  s.reuse = 1;
  if (s.radius <= 1e-32) { s.term = 1; return false; }
  double A[21], g[6];
#pragma unroll
  for (int e = 0; e < 21; e++) A[e] = s.A[e];
#pragma unroll
  for (int e = 0; e < 6; e++) g[e] = s.g[e];
  return eng_propose(s, A, g, max_it);
}

// While the candidate is evaluated (wave 0): 1 / mcc and the parameter tolerance of the step.
__device__ __forceinline__ void eng_step_post(LdsLM& s) {
  double xn = 0.0, sn = 0.0;
#pragma unroll
  for (int e = 0; e < 7; e++) {
    const double xe = s.x[e], d = xe - s.xc[e];
    xn = fma(xe, xe, xn);
    sn = fma(d, d, sn);
  }
  s.ptol = sqrt(sn) <= 1e-8 * (sqrt(xn) + 1e-8);
  s.imcc = 1.0 / s.mcc;
}

}  // namespace lislam
