// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.hpp).
//
// Restatement of scan-to-scan odometry in the forced-geometric mode:
//   a12 TransformToStart                     src/laserOdometry.cpp:147-172
//   a13 corner association (1-NN + lines)    src/laserOdometry.cpp:446-565
//   a14 surf association                     src/laserOdometry.cpp:568-689
//   a15 LidarEdgeFactor                      src/lidarFeaturePointsFunction.hpp:243-293
//   a16 LidarPlaneFactor                     src/lidarFeaturePointsFunction.hpp:143-196
//   a17 LidarPlaneNormFactor                 src/lidarFeaturePointsFunction.hpp:199-240
//   a18 2 x Ceres(DENSE_QR, 4 it), pose accumulation, cloud swap
//                                            src/laserOdometry.cpp:403-437,697-717,793-808
// pcl::KdTreeFLANN 1-NN (a22) is restated as an exact kd-tree search returning the
// lexicographically smallest (float squared distance, index); FLANN's own order among exact
// distance ties is unknowable here (parity unpinned; ties have measure zero on the synthetic
// data).  The Ceres 1.14 Levenberg-Marquardt loop is restated from its published trust-region
// minimizer (jacobi scaling, LM diagonal, DENSE_QR on the augmented system, step acceptance,
// function/parameter/gradient tolerances) — parity unpinned against the real library.
#include <algorithm>
#include <cfloat>
#include <cstring>
#include <limits>
#include <vector>

#include "oracle_common.hpp"
#include "oracle_jet.hpp"
#include "oracle_solver.hpp"

namespace oracle {

// ------------------------------------------------------------------ exact 1-NN (a22)
struct KdTree {
  const P4* pts = nullptr;
  int n = 0;
  std::vector<int> idx;
  struct Node { int lo, hi, dim, left, right; float split; };
  std::vector<Node> nodes;
  int build(int lo, int hi) {
    Node nd{lo, hi, -1, -1, -1, 0.f};
    const int me = (int)nodes.size();
    nodes.push_back(nd);
    if (hi - lo <= 15) return me;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = lo; i < hi; i++) {
      const P4& p = pts[idx[i]];
      const float c[3] = {p.x, p.y, p.z};
      for (int k = 0; k < 3; k++) { mn[k] = std::min(mn[k], c[k]); mx[k] = std::max(mx[k], c[k]); }
    }
    int dim = 0;
    for (int k = 1; k < 3; k++) if (mx[k] - mn[k] > mx[dim] - mn[dim]) dim = k;
    const int mid = (lo + hi) / 2;
    auto key = [&](int a) { const P4& p = pts[a]; return dim == 0 ? p.x : dim == 1 ? p.y : p.z; };
    std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi,
                     [&](int a, int b) { return key(a) < key(b); });
    const float split = key(idx[mid]);
    const int l = build(lo, mid);
    const int r = build(mid, hi);
    nodes[me].dim = dim; nodes[me].split = split; nodes[me].left = l; nodes[me].right = r;
    return me;
  }
  void init(const P4* p, int count) {
    pts = p; n = count;
    idx.resize(n);
    for (int i = 0; i < n; i++) idx[i] = i;
    nodes.clear();
    if (n > 0) build(0, n);
  }
  // float squared distance in FLANN's L2_Simple order ((dx^2 + dy^2) + dz^2)
  static float d2(const P4& a, const P4& b) {
    float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
    return dx * dx + dy * dy + dz * dz;
  }
  void search(int node, const P4& q, float& best, int& besti) const {
    const Node& nd = nodes[node];
    if (nd.dim < 0) {
      for (int i = nd.lo; i < nd.hi; i++) {
        const int j = idx[i];
        const float d = d2(q, pts[j]);
        if (d < best || (d == best && j < besti)) { best = d; besti = j; }
      }
      return;
    }
    const float qc = nd.dim == 0 ? q.x : nd.dim == 1 ? q.y : q.z;
    const double diff = (double)qc - (double)nd.split;
    const int first = diff < 0 ? nd.left : nd.right;
    const int second = diff < 0 ? nd.right : nd.left;
    search(first, q, best, besti);
    // conservative pruning: float distances may round below the exact bound
    if (diff * diff <= (double)best * (1.0 + 1e-5) + 1e-30) search(second, q, best, besti);
  }
  int nearest(const P4& q, float* dist) const {
    float best = FLT_MAX;
    int bi = -1;
    if (n > 0) search(0, q, best, bi);
    *dist = best;
    return bi;
  }
};

// ------------------------------------------------------------------ odometry
struct Frame {
  const P4* sharp; int n_sharp;
  const P4* less_sharp; int n_less_sharp;
  const P4* flat; int n_flat;
  const P4* less_flat; int n_less_flat;
};

// TransformToStart with s = 1 (laserOdometry.cpp:147-172): double math, stored as float.
static P4 transform_to_start(const P4& pi, const double* q, const double* t) {
  Q4<double> qq = slerp_identity_s1(Q4<double>{q[0], q[1], q[2], q[3]});
  V3<double> p{(double)pi.x, (double)pi.y, (double)pi.z};
  V3<double> u = rotate(qq, p) + V3<double>{1.0 * t[0], 1.0 * t[1], 1.0 * t[2]};
  return P4{(float)u.x, (float)u.y, (float)u.z, pi.i};
}

static inline double sqd_float(const P4& a, const P4& b) {  // evaluated in float (:478-483)
  return (double)((a.x - b.x) * (a.x - b.x) + (a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z));
}

struct OdomStats { int corner[2], plane[2]; int lm_iter[2]; };

static void associate_and_solve(const Frame& cur, const P4* cornerLast, int nCL, const KdTree& kdC,
                                const P4* surfLast, int nSL, const KdTree& kdS, double* para,
                                OdomStats& st) {
  const double DIST_SQ = 25.0, NEARBY = 2.5;
  for (int opti = 0; opti < 2; opti++) {
    Problem prob;
    int nc = 0, np = 0;
    for (int i = 0; i < cur.n_sharp; i++) {
      P4 sel = transform_to_start(cur.sharp[i], para, para + 4);
      float d;
      int ci = kdC.nearest(sel, &d);
      int closest = -1, min2 = -1;
      if (ci >= 0 && (double)d < DIST_SQ) {
        closest = ci;
        const int cid = int(cornerLast[closest].i);
        double best2 = DIST_SQ;
        for (int j = closest + 1; j < nCL; ++j) {
          if (int(cornerLast[j].i) <= cid) continue;
          if ((double)int(cornerLast[j].i) > cid + NEARBY) break;
          double dd = sqd_float(cornerLast[j], sel);
          if (dd < best2) { best2 = dd; min2 = j; }
        }
        for (int j = closest - 1; j >= 0; --j) {
          if (int(cornerLast[j].i) >= cid) continue;
          if ((double)int(cornerLast[j].i) < cid - NEARBY) break;
          double dd = sqd_float(cornerLast[j], sel);
          if (dd < best2) { best2 = dd; min2 = j; }
        }
      }
      if (min2 >= 0) {
        Block b;
        b.kind = 0;
        const P4& c = cur.sharp[i];
        const P4& a = cornerLast[closest];
        const P4& bb = cornerLast[min2];
        b.e = EdgeFactor{{c.x, c.y, c.z}, {a.x, a.y, a.z}, {bb.x, bb.y, bb.z}, 1.0};
        prob.blocks.push_back(b);
        nc++;
      }
    }
    for (int i = 0; i < cur.n_flat; i++) {
      P4 sel = transform_to_start(cur.flat[i], para, para + 4);
      float d;
      int ci = kdS.nearest(sel, &d);
      int closest = -1, min2 = -1, min3 = -1;
      if (ci >= 0 && (double)d < DIST_SQ) {
        closest = ci;
        const int cid = int(surfLast[closest].i);
        double best2 = DIST_SQ, best3 = DIST_SQ;
        for (int j = closest + 1; j < nSL; ++j) {
          if ((double)int(surfLast[j].i) > cid + NEARBY) break;
          double dd = sqd_float(surfLast[j], sel);
          if (int(surfLast[j].i) <= cid && dd < best2) { best2 = dd; min2 = j; }
          else if (int(surfLast[j].i) > cid && dd < best3) { best3 = dd; min3 = j; }
        }
        for (int j = closest - 1; j >= 0; --j) {
          if ((double)int(surfLast[j].i) < cid - NEARBY) break;
          double dd = sqd_float(surfLast[j], sel);
          if (int(surfLast[j].i) >= cid && dd < best2) { best2 = dd; min2 = j; }
          else if (int(surfLast[j].i) < cid && dd < best3) { best3 = dd; min3 = j; }
        }
        if (min2 >= 0 && min3 >= 0) {
          const P4& c = cur.flat[i];
          const P4& a = surfLast[closest];
          const P4& b2 = surfLast[min2];
          const P4& b3 = surfLast[min3];
          const double cc[3] = {c.x, c.y, c.z}, aa[3] = {a.x, a.y, a.z};
          const double bb[3] = {b2.x, b2.y, b2.z}, dd[3] = {b3.x, b3.y, b3.z};
          Block b;
          b.kind = 1;
          b.p = PlaneFactor(cc, aa, bb, dd, 1.0);
          prob.blocks.push_back(b);
          np++;
        }
      }
    }
    st.corner[opti] = nc;
    st.plane[opti] = np;
    SolveSummary s = ceres_solve(prob, para, 4);
    st.lm_iter[opti] = s.iterations;
  }
}

}  // namespace oracle

using namespace oracle;

extern "C" {

// Runs a fresh laserOdometry node (forced geometric mode) over n frames.  Feature clouds are
// passed concatenated with per-frame offsets (off arrays have n+1 entries, in points).
// out_pose[7n] = world pose (qx,qy,qz,qw,tx,ty,tz) after each frame (laserOdometry.cpp:716-744);
// out_rel[7n] = para_q/para_t after each frame; out_stats[6n] = corner/plane counts and LM
// iterations for the two outer passes.  Returns 0.
// use_aloam (nullable = every frame, the forced geometric mode): frame f > 0 is optimized only
// when use_aloam[f] != 0 (laserOdometry.cpp:403-417: the sharp cloud's frame_id ==
// "skip_intensity"); otherwise para keeps the previous estimate and the pose still accumulates
// (:716-717).
int oracle_odometry_chain_gated(int n, const float* sharp, const int* sharp_off, const float* less_sharp,
                                const int* less_sharp_off, const float* flat, const int* flat_off,
                                const float* less_flat, const int* less_flat_off, const int* use_aloam,
                                double* out_pose, double* out_rel, int* out_stats);

int oracle_odometry_chain(int n, const float* sharp, const int* sharp_off, const float* less_sharp,
                          const int* less_sharp_off, const float* flat, const int* flat_off,
                          const float* less_flat, const int* less_flat_off, double* out_pose,
                          double* out_rel, int* out_stats) {
  return oracle_odometry_chain_gated(n, sharp, sharp_off, less_sharp, less_sharp_off, flat, flat_off, less_flat,
                                     less_flat_off, nullptr, out_pose, out_rel, out_stats);
}

int oracle_odometry_chain_gated(int n, const float* sharp, const int* sharp_off, const float* less_sharp,
                                const int* less_sharp_off, const float* flat, const int* flat_off,
                                const float* less_flat, const int* less_flat_off, const int* use_aloam,
                                double* out_pose, double* out_rel, int* out_stats) {
  double para[7] = {0, 0, 0, 1, 0, 0, 0};
  Q4<double> qw{0, 0, 0, 1};
  double tw[3] = {0, 0, 0};
  const P4* S = reinterpret_cast<const P4*>(sharp);
  const P4* LS = reinterpret_cast<const P4*>(less_sharp);
  const P4* F = reinterpret_cast<const P4*>(flat);
  const P4* LF = reinterpret_cast<const P4*>(less_flat);
  const P4* cornerLast = nullptr;
  const P4* surfLast = nullptr;
  int nCL = 0, nSL = 0;
  KdTree kdC, kdS;
  for (int f = 0; f < n; f++) {
    Frame fr{S + sharp_off[f], sharp_off[f + 1] - sharp_off[f],
             LS + less_sharp_off[f], less_sharp_off[f + 1] - less_sharp_off[f],
             F + flat_off[f], flat_off[f + 1] - flat_off[f],
             LF + less_flat_off[f], less_flat_off[f + 1] - less_flat_off[f]};
    OdomStats st{{0, 0}, {0, 0}, {0, 0}};
    if (f > 0) {
      if (!use_aloam || use_aloam[f]) associate_and_solve(fr, cornerLast, nCL, kdC, surfLast, nSL, kdS, para, st);
      // t_w_curr = t_w_curr + q_w_curr * t_last_curr; q_w_curr = q_w_curr * q_last_curr
      V3<double> tr = rotate(qw, V3<double>{para[4], para[5], para[6]});
      tw[0] = tw[0] + tr.x; tw[1] = tw[1] + tr.y; tw[2] = tw[2] + tr.z;
      qw = qmul(qw, Q4<double>{para[0], para[1], para[2], para[3]});
    }
    if (out_pose) {
      double* o = out_pose + 7 * f;
      o[0] = qw.x; o[1] = qw.y; o[2] = qw.z; o[3] = qw.w; o[4] = tw[0]; o[5] = tw[1]; o[6] = tw[2];
    }
    if (out_rel) std::memcpy(out_rel + 7 * f, para, sizeof(para));
    if (out_stats) {
      int* o = out_stats + 6 * f;
      o[0] = st.corner[0]; o[1] = st.plane[0]; o[2] = st.corner[1]; o[3] = st.plane[1];
      o[4] = st.lm_iter[0]; o[5] = st.lm_iter[1];
    }
    cornerLast = fr.less_sharp; nCL = fr.n_less_sharp;
    surfLast = fr.less_flat; nSL = fr.n_less_flat;
    kdC.init(cornerLast, nCL);
    kdS.init(surfLast, nSL);
  }
  return 0;
}

// Exact 1-NN of each query in target (kd-tree), for the a22 cross-checks.
int oracle_nn1(const float* target, int n, const float* queries, int m, int* out_idx, float* out_d2) {
  KdTree kd;
  kd.init(reinterpret_cast<const P4*>(target), n);
  const P4* Q = reinterpret_cast<const P4*>(queries);
  for (int i = 0; i < m; i++) out_idx[i] = kd.nearest(Q[i], &out_d2[i]);
  return 0;
}

// Evaluate one functor (kind 0 edge(curr,a,b), 1 plane(curr,j,l,m), 2 plane-norm(curr,n,d))
// at (q, t): residuals r[R] and the global Jacobian J[R x 7] (q: 4 columns, t: 3).
int oracle_eval_factor(int kind, const double* pts, const double* q, const double* t, double* r,
                       double* J) {
  if (kind == 0) {
    EdgeFactor e{{pts[0], pts[1], pts[2]}, {pts[3], pts[4], pts[5]}, {pts[6], pts[7], pts[8]}, 1.0};
    autodiff_eval(e, q, t, r, J);
  } else if (kind == 1) {
    PlaneFactor p(pts, pts + 3, pts + 6, pts + 9, 1.0);
    autodiff_eval(p, q, t, r, J);
  } else {
    PlaneNormFactor p{{pts[0], pts[1], pts[2]}, {pts[3], pts[4], pts[5]}, pts[6]};
    autodiff_eval(p, q, t, r, J);
  }
  return 0;
}

}  // extern "C"
