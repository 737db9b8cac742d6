// lislam scan-to-scan odometry on gfx950 (a12..a18 of SURVEY.md §8(a)), forced geometric mode.
//
// One 256-thread workgroup owns one chain of consecutive scans — a fresh laserOdometry node
// started at the chain's first scan (laserOdometry.cpp:382-389), carrying para_q/para_t as the
// initial guess from pair to pair (:130-135) and accumulating the pose (:716-717).  Per pair:
//   2 outer passes (:417) of
//     association  — TransformToStart (:147-172), exact 1-NN in the previous less-sharp /
//                    less-flat cloud (KdTreeFLANN, :452/:574) by LDS-tiled brute force with the
//                    FLANN float distance, then the scan-line searches (:467-520, :589-646) with
//                    the reference's visit order, strict '<' and 'break' semantics;
//     solve        — ceres::Solve(DENSE_QR, max 4 it) restated as a device-side trust-region
//                    Levenberg-Marquardt: every evaluation is one pass over the residual blocks
//                    computing cost, J^T J (21) and J^T r (6) of the Huber-corrected analytic
//                    LidarEdgeFactor / LidarPlaneFactor residuals in fp64, reduced across the
//                    workgroup; thread 0 runs the 6x6 step logic.
#include <hip/hip_runtime.h>

#include "lislam_device.hpp"
#include "lislam_factors.hpp"
#include "lislam_internal.hpp"

namespace lislam {

constexpr int kOdomThreads = 256;
constexpr int kOdomWaves = kOdomThreads / 64;
constexpr int kTile = 1024;  // target points per LDS tile
constexpr int kQPT = 4;      // queries per thread per round
constexpr double kDistSq = 25.0;
constexpr double kNearby = 2.5;

struct OdomShared {
  P4 tile[kTile];
  double red[kOdomWaves][28];
  double x[7];       // point at which the next evaluation runs
  double acc[28];    // reduced cost, JtJ (21, upper-triangular row-major), g (6)
  int flag;
  int cnt[2];
};

__device__ __forceinline__ P4 transform_to_start(const P4& pi, const double* x) {
  const DQ q{x[0], x[1], x[2], x[3]};
  const D3 u = qrot(q, D3{(double)pi.x, (double)pi.y, (double)pi.z}) + D3{1.0 * x[4], 1.0 * x[5], 1.0 * x[6]};
  return P4{(float)u.x, (float)u.y, (float)u.z, pi.i};
}

__device__ __forceinline__ float flann_d2(const P4& q, const P4& p) {
  const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
  return dx * dx + dy * dy + dz * dz;
}

__device__ __forceinline__ double line_d2(const P4& p, const P4& sel) {  // laserOdometry.cpp:478
  return (double)((p.x - sel.x) * (p.x - sel.x) + (p.y - sel.y) * (p.y - sel.y) + (p.z - sel.z) * (p.z - sel.z));
}

// Exact 1-NN of up to kQPT queries per thread against target[0..n) (ties: lowest index).
__device__ void nn1_tiled(OdomShared& sh, const P4* target, int n, const P4* qsel, int nq_this,
                          float* best, int* bi) {
  for (int k = 0; k < kQPT; k++) { best[k] = 3.4e38f; bi[k] = -1; }
  for (int t0 = 0; t0 < n; t0 += kTile) {
    const int m = min(kTile, n - t0);
    __syncthreads();
    for (int j = threadIdx.x; j < m; j += kOdomThreads) sh.tile[j] = ld4(target + t0 + j);
    __syncthreads();
    for (int j = 0; j < m; j++) {
      const P4 p = sh.tile[j];
#pragma unroll
      for (int k = 0; k < kQPT; k++) {
        const float d = flann_d2(qsel[k], p);
        if (k < nq_this && d < best[k]) { best[k] = d; bi[k] = t0 + j; }
      }
    }
  }
}

// ------------------------------------------------------------------ block records
// record r (9 doubles): edge  -> c, a, b          (LidarEdgeFactor(curr, a, b, s=1))
//                       plane -> c, j, unit normal (LidarPlaneFactor ctor normalizes, hpp:151-152)
__device__ void associate(OdomShared& sh, const OdomArgs& a, int k, const double* x, double* blk, int* kind) {
  const int tid = threadIdx.x;
  const P4* cur_s = a.sharp + (size_t)k * a.cap_sharp;
  const P4* cur_f = a.flat + (size_t)k * a.cap_flat;
  const P4* lastC = a.less_sharp + (size_t)(k - 1) * a.cap_less_sharp;
  const P4* lastS = a.less_flat + (size_t)(k - 1) * a.N;
  const int ns = a.n_feat[k * 4 + 0], nf = a.n_feat[k * 4 + 2];
  const int nC = a.n_feat[(k - 1) * 4 + 1], nS = a.n_feat[(k - 1) * 4 + 3];
  int ncorner = 0, nplane = 0;
  // ---- corners
  for (int r0 = 0; r0 < ns; r0 += kOdomThreads * kQPT) {
    P4 sel[kQPT];
    int qi[kQPT];
    int nq = 0;
    for (int k2 = 0; k2 < kQPT; k2++) {
      qi[k2] = r0 + k2 * kOdomThreads + tid;
      sel[k2] = P4{0, 0, 0, 0};
      if (qi[k2] < ns) { sel[k2] = transform_to_start(ld4(cur_s + qi[k2]), x); nq = k2 + 1; }
    }
    float best[kQPT];
    int bi[kQPT];
    nn1_tiled(sh, lastC, nC, sel, nq, best, bi);
    for (int k2 = 0; k2 < kQPT; k2++) {
      const int q = qi[k2];
      if (q >= ns) continue;
      int min2 = -1;
      const int closest = bi[k2];
      if (closest >= 0 && (double)best[k2] < kDistSq) {
        const int cid = int(ld4(lastC + closest).i);
        double best2 = kDistSq;
        for (int j = closest + 1; j < nC; ++j) {
          const P4 p = ld4(lastC + j);
          const int pid = int(p.i);
          if (pid <= cid) continue;
          if ((double)pid > cid + kNearby) break;
          const double d = line_d2(p, sel[k2]);
          if (d < best2) { best2 = d; min2 = j; }
        }
        for (int j = closest - 1; j >= 0; --j) {
          const P4 p = ld4(lastC + j);
          const int pid = int(p.i);
          if (pid >= cid) continue;
          if ((double)pid < cid - kNearby) break;
          const double d = line_d2(p, sel[k2]);
          if (d < best2) { best2 = d; min2 = j; }
        }
      }
      double* r = blk + (size_t)q * 9;
      if (min2 >= 0) {
        const P4 c = ld4(cur_s + q), pa = ld4(lastC + closest), pb = ld4(lastC + min2);
        r[0] = c.x; r[1] = c.y; r[2] = c.z; r[3] = pa.x; r[4] = pa.y; r[5] = pa.z;
        r[6] = pb.x; r[7] = pb.y; r[8] = pb.z;
        kind[q] = 0;
        ncorner++;
      } else {
        kind[q] = -1;
      }
    }
  }
  // ---- surfs
  for (int r0 = 0; r0 < nf; r0 += kOdomThreads * kQPT) {
    P4 sel[kQPT];
    int qi[kQPT];
    int nq = 0;
    for (int k2 = 0; k2 < kQPT; k2++) {
      qi[k2] = r0 + k2 * kOdomThreads + tid;
      sel[k2] = P4{0, 0, 0, 0};
      if (qi[k2] < nf) { sel[k2] = transform_to_start(ld4(cur_f + qi[k2]), x); nq = k2 + 1; }
    }
    float best[kQPT];
    int bi[kQPT];
    nn1_tiled(sh, lastS, nS, sel, nq, best, bi);
    for (int k2 = 0; k2 < kQPT; k2++) {
      const int q = qi[k2];
      if (q >= nf) continue;
      int min2 = -1, min3 = -1;
      const int closest = bi[k2];
      if (closest >= 0 && (double)best[k2] < kDistSq) {
        const int cid = int(ld4(lastS + closest).i);
        double best2 = kDistSq, best3 = kDistSq;
        for (int j = closest + 1; j < nS; ++j) {
          const P4 p = ld4(lastS + j);
          const int pid = int(p.i);
          if ((double)pid > cid + kNearby) break;
          const double d = line_d2(p, sel[k2]);
          if (pid <= cid && d < best2) { best2 = d; min2 = j; }
          else if (pid > cid && d < best3) { best3 = d; min3 = j; }
        }
        for (int j = closest - 1; j >= 0; --j) {
          const P4 p = ld4(lastS + j);
          const int pid = int(p.i);
          if ((double)pid < cid - kNearby) break;
          const double d = line_d2(p, sel[k2]);
          if (pid >= cid && d < best2) { best2 = d; min2 = j; }
          else if (pid < cid && d < best3) { best3 = d; min3 = j; }
        }
      }
      double* r = blk + (size_t)(a.cap_sharp + q) * 9;
      int* kd = kind + a.cap_sharp + q;
      if (min2 >= 0 && min3 >= 0) {
        const P4 c = ld4(cur_f + q), pj = ld4(lastS + closest), pl = ld4(lastS + min2), pm = ld4(lastS + min3);
        const D3 j{pj.x, pj.y, pj.z}, l{pl.x, pl.y, pl.z}, m{pm.x, pm.y, pm.z};
        const D3 nrm = plane_normal(j, l, m);
        r[0] = c.x; r[1] = c.y; r[2] = c.z; r[3] = j.x; r[4] = j.y; r[5] = j.z;
        r[6] = nrm.x; r[7] = nrm.y; r[8] = nrm.z;
        *kd = 1;
        nplane++;
      } else {
        *kd = -1;
      }
    }
  }
  // counts (corner_correspondence / plane_correspondence)
  if (tid == 0) { sh.cnt[0] = 0; sh.cnt[1] = 0; }
  __syncthreads();
  if (ncorner) atomicAdd(&sh.cnt[0], ncorner);
  if (nplane) atomicAdd(&sh.cnt[1], nplane);
  __syncthreads();
}

// ------------------------------------------------------------------ evaluation
// Analytic local Jacobian: lp = R(q) c + t, d lp / d t = I, d lp / d delta = -2 [R(q)c]x
// (EigenQuaternionParameterization plus: q <- [sin|d| d/|d|, cos|d|] (x) q).
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

__device__ void evaluate(OdomShared& sh, const OdomArgs& a, int ns, int nf, const double* blk, const int* kind) {
  double acc[28];
#pragma unroll
  for (int e = 0; e < 28; e++) acc[e] = 0;
  const DQ q{sh.x[0], sh.x[1], sh.x[2], sh.x[3]};
  const D3 t{sh.x[4], sh.x[5], sh.x[6]};
  const double ha = 0.1;  // HuberLoss(0.1), laserOdometry.cpp:424
  const int total = a.cap_sharp + nf;
  for (int idx = threadIdx.x; idx < total; idx += kOdomThreads) {
    if (idx >= ns && idx < a.cap_sharp) continue;
    const int kd = kind[idx];
    if (kd < 0) continue;
    const double* r9 = blk + (size_t)idx * 9;
    const D3 c{r9[0], r9[1], r9[2]};
    if (kd == 0) {
      double res[3], J[3][6];
      edge_factor(q, t, c, D3{r9[3], r9[4], r9[5]}, D3{r9[6], r9[7], r9[8]}, res, J);
      const double sc = huber_scale(ha, res[0] * res[0] + res[1] * res[1] + res[2] * res[2], &acc[0]);
      for (int i = 0; i < 3; i++) {
        double Js[6];
        for (int cc = 0; cc < 6; cc++) Js[cc] = J[i][cc] * sc;
        accum_row(acc, Js, res[i] * sc);
      }
    } else {
      double res, J[6];
      plane_factor(q, t, c, D3{r9[3], r9[4], r9[5]}, D3{r9[6], r9[7], r9[8]}, &res, J);
      const double sc = huber_scale(ha, res * res, &acc[0]);
      for (int cc = 0; cc < 6; cc++) J[cc] *= sc;
      accum_row(acc, J, res * sc);
    }
  }
  // workgroup reduction
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < 28; e++) {
    double v = acc[e];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) sh.red[wave][e] = v;
  }
  __syncthreads();
  if (threadIdx.x < 28) {
    double v = 0;
    for (int w = 0; w < kOdomWaves; w++) v += sh.red[w][threadIdx.x];
    sh.acc[threadIdx.x] = v;
  }
  __syncthreads();
}

// ------------------------------------------------------------------ LM state (thread 0)
struct LM {
  double x[7], xc[7];
  double cost;
  double A[36], g[6];  // J^T J, J^T r at x (unscaled)
  double scale[6], diag[6];
  double radius, dfac;
  bool reuse;
  int it, invalid, successful, term;
};

__device__ void unpack(const double* acc, double* cost, double* A, double* g) {
  *cost = acc[0];
  int e = 1;
  for (int i = 0; i < 6; i++)
    for (int j = i; j < 6; j++) { A[i * 6 + j] = acc[e]; A[j * 6 + i] = acc[e]; e++; }
  for (int i = 0; i < 6; i++) g[i] = acc[22 + i];
}

__device__ void quat_plus(const double* x, const double* d, double* xp) {
  const double nd = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd > 0.0) {
    const double sdd = sin(nd) / nd;
    const DQ r = qmul(DQ{sdd * d[0], sdd * d[1], sdd * d[2], cos(nd)}, DQ{x[0], x[1], x[2], x[3]});
    xp[0] = r.x; xp[1] = r.y; xp[2] = r.z; xp[3] = r.w;
  } else {
    for (int k = 0; k < 4; k++) xp[k] = x[k];
  }
}
__device__ void state_plus(const double* x, const double* d, double* xp) {
  quat_plus(x, d, xp);
  for (int k = 0; k < 3; k++) xp[4 + k] = x[4 + k] + d[3 + k];
}
__device__ double grad_max_norm(const double* x, const double* g) {
  double ng[6], xp[7];
  for (int k = 0; k < 6; k++) ng[k] = -g[k];
  state_plus(x, ng, xp);
  double mx = 0;
  for (int k = 0; k < 7; k++) mx = fmax(mx, fabs(x[k] - xp[k]));
  return mx;
}

// Solve (S A S + diag(D)) y = S g by Cholesky; false if not positive definite / not finite.
__device__ bool lm_solve(const LM& s, double* y) {
  double M[36], b[6];
  for (int i = 0; i < 6; i++) {
    for (int j = 0; j < 6; j++) M[i * 6 + j] = s.scale[i] * s.A[i * 6 + j] * s.scale[j];
    M[i * 6 + i] += s.diag[i] / s.radius;
    b[i] = s.scale[i] * s.g[i];
  }
  double L[36] = {0};
  for (int j = 0; j < 6; j++) {
    double d = M[j * 6 + j];
    for (int k = 0; k < j; k++) d -= L[j * 6 + k] * L[j * 6 + k];
    if (!(d > 0)) return false;
    const double ljj = sqrt(d);
    L[j * 6 + j] = ljj;
    for (int i = j + 1; i < 6; i++) {
      double v = M[i * 6 + j];
      for (int k = 0; k < j; k++) v -= L[i * 6 + k] * L[j * 6 + k];
      L[i * 6 + j] = v / ljj;
    }
  }
  double z[6];
  for (int i = 0; i < 6; i++) {
    double v = b[i];
    for (int k = 0; k < i; k++) v -= L[i * 6 + k] * z[k];
    z[i] = v / L[i * 6 + i];
  }
  for (int i = 5; i >= 0; i--) {
    double v = z[i];
    for (int k = i + 1; k < 6; k++) v -= L[k * 6 + i] * y[k];
    y[i] = v / L[i * 6 + i];
  }
  for (int i = 0; i < 6; i++)
    if (!isfinite(y[i])) return false;
  return true;
}

// Proposes the next candidate into s.xc; returns false when the solve terminates.
// Mirrors TrustRegionMinimizer + LevenbergMarquardtStrategy (Ceres 1.14 defaults).
__device__ bool lm_propose(LM& s, int max_it, double* mcc_out) {
  while (s.it < max_it) {
    s.it++;
    if (!s.reuse)
      for (int c = 0; c < 6; c++)
        s.diag[c] = fmin(fmax(s.scale[c] * s.scale[c] * s.A[c * 6 + c], 1e-6), 1e32);
    double y[6];
    const bool ok = lm_solve(s, y);
    s.reuse = true;
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
    if (!ok || !(mcc > 0.0)) {  // invalid step -> rejected-step radius update, try again
      if (++s.invalid >= 5) { s.term = 2; return false; }
      s.radius /= s.dfac;
      s.dfac *= 2.0;
      s.reuse = true;
      continue;
    }
    s.invalid = 0;
    double delta[6];
    for (int k = 0; k < 6; k++) delta[k] = step[k] * s.scale[k];
    state_plus(s.x, delta, s.xc);
    *mcc_out = mcc;
    return true;
  }
  s.term = 0;  // NO_CONVERGENCE (max iterations)
  return false;
}

__global__ __launch_bounds__(kOdomThreads) void k_odom_chain(OdomArgs a) {
  __shared__ OdomShared sh;
  const int c = blockIdx.x;
  const int k0 = c * a.chain_len;
  const int k1 = min(k0 + a.chain_len, a.S - 1);
  double* blk = a.blk + (size_t)c * (a.cap_sharp + a.cap_flat) * 9;
  int* kind = a.blk_kind + (size_t)c * (a.cap_sharp + a.cap_flat);
  // node state (thread 0 owns it; broadcast through sh.x)
  double para[7] = {0, 0, 0, 1, 0, 0, 0};
  DQ qw{0, 0, 0, 1};
  D3 tw{0, 0, 0};
  if (a.init_state) {  // resume a node (lislam_odom_step)
    const double* is = a.init_state + (size_t)c * 14;
    for (int e = 0; e < 7; e++) para[e] = is[e];
    qw = DQ{is[7], is[8], is[9], is[10]};
    tw = D3{is[11], is[12], is[13]};
  }
  if (threadIdx.x == 0 && c == 0 && !a.init_state) {
    for (int e = 0; e < 7; e++) { a.para[e] = para[e]; a.pose[e] = e == 3 ? 1.0 : 0.0; }
    for (int e = 0; e < 8; e++) a.stats[e] = 0;
  }
  for (int k = k0 + 1; k <= k1; k++) {
    const int ns = a.n_feat[k * 4 + 0], nf = a.n_feat[k * 4 + 2];
    int st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int outer = 0; outer < 2; outer++) {
      if (threadIdx.x == 0)
        for (int e = 0; e < 7; e++) sh.x[e] = para[e];
      __syncthreads();
      double xl[7];
      for (int e = 0; e < 7; e++) xl[e] = sh.x[e];
      associate(sh, a, k, xl, blk, kind);
      __threadfence_block();
      st[outer * 2 + 0] = sh.cnt[0];
      st[outer * 2 + 1] = sh.cnt[1];
      LM s;
      bool go = sh.cnt[0] + sh.cnt[1] > 0;
      double mcc = 0;
      // iteration 0: evaluate at x
      if (go) {
        __syncthreads();
        evaluate(sh, a, ns, nf, blk, kind);
        if (threadIdx.x == 0) {
          for (int e = 0; e < 7; e++) s.x[e] = para[e];
          unpack(sh.acc, &s.cost, s.A, s.g);
          for (int cc = 0; cc < 6; cc++) s.scale[cc] = 1.0 / (1.0 + sqrt(s.A[cc * 6 + cc]));
          s.radius = 1e4; s.dfac = 2.0; s.reuse = false;
          s.it = 0; s.invalid = 0; s.successful = 0; s.term = 0;
          bool cont = isfinite(s.cost) && !(grad_max_norm(s.x, s.g) <= 1e-10);
          if (!isfinite(s.cost)) s.term = 2; else if (!cont) s.term = 1;
          if (cont) cont = lm_propose(s, a.max_iterations, &mcc);
          sh.flag = cont;
          if (cont)
            for (int e = 0; e < 7; e++) sh.x[e] = s.xc[e];
        }
        __syncthreads();
        go = sh.flag;
      }
      while (go) {
        evaluate(sh, a, ns, nf, blk, kind);  // cost + J^T J + J^T r at the candidate
        if (threadIdx.x == 0) {
          double ccost, cA[36], cg[6];
          unpack(sh.acc, &ccost, cA, cg);
          if (!isfinite(ccost)) ccost = 1.7976931348623157e308;
          bool cont = true;
          double xn = 0, sn = 0;
          for (int e = 0; e < 7; e++) { xn += s.x[e] * s.x[e]; sn += (s.x[e] - s.xc[e]) * (s.x[e] - s.xc[e]); }
          xn = sqrt(xn); sn = sqrt(sn);
          if (sn <= 1e-8 * (xn + 1e-8)) { s.term = 1; cont = false; }                      // parameter tol
          else if (fabs(s.cost - ccost) <= 1e-6 * s.cost) { s.term = 1; cont = false; }   // function tol
          else {
            const double rel = (s.cost - ccost) / mcc;
            if (rel > 1e-3) {  // accept
              for (int e = 0; e < 7; e++) s.x[e] = s.xc[e];
              s.cost = ccost;
              for (int e = 0; e < 36; e++) s.A[e] = cA[e];
              for (int e = 0; e < 6; e++) s.g[e] = cg[e];
              const double t3 = 2.0 * rel - 1.0;
              s.radius = fmin(1e16, s.radius / fmax(1.0 / 3.0, 1.0 - t3 * t3 * t3));
              s.dfac = 2.0;
              s.reuse = false;
              s.successful++;
              if (grad_max_norm(s.x, s.g) <= 1e-10) { s.term = 1; cont = false; }
            } else {           // reject
              s.radius /= s.dfac;
              s.dfac *= 2.0;
              s.reuse = true;
            }
            if (cont && s.radius <= 1e-32) { s.term = 1; cont = false; }
          }
          if (cont) cont = lm_propose(s, a.max_iterations, &mcc);
          sh.flag = cont;
          if (cont)
            for (int e = 0; e < 7; e++) sh.x[e] = s.xc[e];
        }
        __syncthreads();
        go = sh.flag;
      }
      if (threadIdx.x == 0 && (st[outer * 2] + st[outer * 2 + 1]) > 0) {
        for (int e = 0; e < 7; e++) para[e] = s.x[e];
        st[4 + outer] = s.it;
        st[6 + outer] = s.term;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      // t_w_curr = t_w_curr + q_w_curr * t_last_curr; q_w_curr = q_w_curr * q_last_curr
      tw = tw + qrot(qw, D3{para[4], para[5], para[6]});
      qw = qmul(qw, DQ{para[0], para[1], para[2], para[3]});
      double* op = a.para + (size_t)k * 7;
      double* ow = a.pose + (size_t)k * 7;
      for (int e = 0; e < 7; e++) op[e] = para[e];
      ow[0] = qw.x; ow[1] = qw.y; ow[2] = qw.z; ow[3] = qw.w; ow[4] = tw.x; ow[5] = tw.y; ow[6] = tw.z;
      for (int e = 0; e < 8; e++) a.stats[(size_t)k * 8 + e] = st[e];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_eval_factors(FactorArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const DQ q{a.x[0], a.x[1], a.x[2], a.x[3]};
  const D3 t{a.x[4], a.x[5], a.x[6]};
  const double* p = a.pts + (size_t)i * 12;
  const D3 c{p[0], p[1], p[2]};
  double r[3] = {0, 0, 0}, J[3][6] = {{0}};
  if (a.kind[i] == 0) {
    edge_factor(q, t, c, D3{p[3], p[4], p[5]}, D3{p[6], p[7], p[8]}, r, J);
  } else if (a.kind[i] == 1) {
    const D3 n = plane_normal(D3{p[3], p[4], p[5]}, D3{p[6], p[7], p[8]}, D3{p[9], p[10], p[11]});
    plane_factor(q, t, c, D3{p[3], p[4], p[5]}, n, r, J[0]);
  } else {
    plane_norm_factor(q, t, c, D3{p[3], p[4], p[5]}, p[6], r, J[0]);
  }
  if (a.res)
    for (int k = 0; k < 3; k++) a.res[(size_t)i * 3 + k] = r[k];
  if (a.jac)
    for (int k = 0; k < 3; k++)
      for (int cc = 0; cc < 6; cc++) a.jac[((size_t)i * 3 + k) * 6 + cc] = J[k][cc];
}

void launch_factors(const FactorArgs& a, hipStream_t st) {
  if (a.n > 0) hipLaunchKernelGGL(k_eval_factors, dim3((a.n + 255) / 256), dim3(256), 0, st, a);
}

void launch_odometry(const OdomArgs& a, hipStream_t st, hipEvent_t* ev) {
  if (ev) (void)hipEventRecord(ev[0], st);
  if (a.n_chains > 0) hipLaunchKernelGGL(k_odom_chain, dim3(a.n_chains), dim3(kOdomThreads), 0, st, a);
  if (ev) (void)hipEventRecord(ev[1], st);
}

}  // namespace lislam
