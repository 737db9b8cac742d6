// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.hpp).
//
// Restatement of the scan-to-map stages of the hot path:
//   a21 ikd-Tree  Build                 src/ikd-Tree/ikd_Tree.cpp:470-492
//                 Add_Points (box downsampling)                  :569-706
//                 Search_by_range (half-open box predicate)      :1607-1645
//                 Nearest_Search / Search (k-NN, max_dist)       :494-547, :1381-1604
//                 calc_dist / same_point                         :2224-2235, :2216-2220
//   a20 mapOptimization ground-plane association, Ceres(DENSE_QR, 10 it), transformUpdate on
//       CONVERGENCE, Add_Points of the keyframe cloud   src/mapOptimization.cpp:364-479, :730-746
//   a19 laserMapping corner (5-NN line, PCA) / surf (5-NN plane, QR) association and
//       2 x Ceres(4 it)                                 src/laserMapping.cpp:640-850
//
// The ikd-Tree's kd layout (balance / lazy rebuild) decides how points are found, not which:
// this restatement keeps the tree's point set (lazy delete = the point leaves the set) and
// answers Search_by_range with ikd's half-open predicate (min <= p < max on every axis) and
// Nearest_Search with an exact kd-tree k-NN ordered by (float squared distance, point id).  ikd's
// own order among exactly equal distances follows its tree layout and is unknowable here (ties
// have measure zero on the synthetic data).  Point ids: Build numbers the points 0..n-1; every
// Add_Points call reserves ids next_id .. next_id+n-1 for its inputs in order (an input keeps its
// id if it enters the tree; a stored point that wins a downsample box keeps its own id).
// Eigen's ColPivHouseholderQR (5x3 plane fit, laserMapping.cpp:771, mapOptimization.cpp:407) and
// SelfAdjointEigenSolver (3x3 line fit, laserMapping.cpp:700) are restated from the published
// algorithms (column-pivoted Householder QR; cyclic Jacobi): parity unpinned against Eigen at the
// last-ulp level, which the 1e-4 pose tolerance absorbs.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "oracle_common.hpp"
#include "oracle_solver.hpp"

namespace oracle {

struct MapPoint {
  float x, y, z;
  int id;
  bool dead = false;
};

// ikd_Tree.cpp:2224-2235 (left-to-right float sum)
static inline float calc_dist(float ax, float ay, float az, float bx, float by, float bz) {
  return (ax - bx) * (ax - bx) + (ay - by) * (ay - by) + (az - bz) * (az - bz);
}

// ------------------------------------------------------------------ exact k-NN (kd-tree)
struct KnnTree {
  std::vector<MapPoint> pts;
  struct Node {
    float lo[3], hi[3];
    int begin, end, left, right;
  };
  std::vector<Node> nodes;
  std::vector<int> order;

  void build(const std::vector<MapPoint>& p) {
    pts = p;
    nodes.clear();
    order.resize(pts.size());
    for (size_t i = 0; i < pts.size(); i++) order[i] = (int)i;
    if (!pts.empty()) build_rec(0, (int)pts.size());
  }
  int build_rec(int b, int e) {
    Node nd;
    nd.begin = b; nd.end = e; nd.left = nd.right = -1;
    for (int k = 0; k < 3; k++) { nd.lo[k] = FLT_MAX; nd.hi[k] = -FLT_MAX; }
    for (int i = b; i < e; i++) {
      const MapPoint& q = pts[order[i]];
      const float c[3] = {q.x, q.y, q.z};
      for (int k = 0; k < 3; k++) { nd.lo[k] = std::min(nd.lo[k], c[k]); nd.hi[k] = std::max(nd.hi[k], c[k]); }
    }
    const int id = (int)nodes.size();
    nodes.push_back(nd);
    if (e - b > 8) {
      int ax = 0;
      float w = -1;
      for (int k = 0; k < 3; k++)
        if (nd.hi[k] - nd.lo[k] > w) { w = nd.hi[k] - nd.lo[k]; ax = k; }
      const int m = (b + e) / 2;
      std::nth_element(order.begin() + b, order.begin() + m, order.begin() + e, [&](int u, int v) {
        const float cu = ax == 0 ? pts[u].x : ax == 1 ? pts[u].y : pts[u].z;
        const float cv = ax == 0 ? pts[v].x : ax == 1 ? pts[v].y : pts[v].z;
        return cu < cv || (cu == cv && u < v);
      });
      const int l = build_rec(b, m);
      const int r = build_rec(m, e);
      nodes[id].left = l;
      nodes[id].right = r;
    }
    return id;
  }
  // float lower bound of calc_dist over the box (monotone rounding: never above a member's distance)
  static float box_dist(const Node& n, const float* q) {
    float d = 0;
    for (int k = 0; k < 3; k++) {
      float g = 0;
      if (q[k] < n.lo[k]) g = q[k] - n.lo[k];
      else if (q[k] > n.hi[k]) g = q[k] - n.hi[k];
      d += g * g;
    }
    return d;
  }
  struct Best {
    float d;
    int id, idx;
  };
  static bool less(const Best& a, const Best& b) { return a.d < b.d || (a.d == b.d && a.id < b.id); }
  void search(int ni, const float* q, int k, float maxd2, std::vector<Best>& best) const {
    const Node& n = nodes[ni];
    const float bd = box_dist(n, q);
    if (bd > maxd2) return;
    if ((int)best.size() == k && bd > best.back().d) return;
    if (n.left < 0) {
      for (int i = n.begin; i < n.end; i++) {
        const MapPoint& p = pts[order[i]];
        const float d = calc_dist(q[0], q[1], q[2], p.x, p.y, p.z);
        if (d > maxd2) continue;
        Best c{d, p.id, order[i]};
        if ((int)best.size() < k) {
          best.insert(std::upper_bound(best.begin(), best.end(), c, less), c);
        } else if (less(c, best.back())) {
          best.pop_back();
          best.insert(std::upper_bound(best.begin(), best.end(), c, less), c);
        }
      }
      return;
    }
    const float dl = box_dist(nodes[n.left], q), dr = box_dist(nodes[n.right], q);
    if (dl <= dr) {
      search(n.left, q, k, maxd2, best);
      search(n.right, q, k, maxd2, best);
    } else {
      search(n.right, q, k, maxd2, best);
      search(n.left, q, k, maxd2, best);
    }
  }
};

// ------------------------------------------------------------------ the ikd-Tree point set
struct IkdMap {
  float downsample_size = 0.2f;  // KD_TREE(delete_param, balance_param, box_length)
  std::vector<MapPoint> pts;     // live points
  int next_id = 0;
  // search accelerator only: cell (edge = downsample_size) -> indices into pts
  std::unordered_map<uint64_t, std::vector<int>> grid;
  KnnTree tree;
  bool dirty = true;
  int n_dead = 0;

  static uint64_t key(int ix, int iy, int iz) {
    return ((uint64_t)(uint32_t)(ix + (1 << 20)) << 42) | ((uint64_t)(uint32_t)(iy + (1 << 20)) << 21) |
           (uint64_t)(uint32_t)(iz + (1 << 20));
  }
  int cell(float v) const { return (int)std::floor(v / downsample_size); }
  void insert(const MapPoint& p) {
    pts.push_back(p);
    grid[key(cell(p.x), cell(p.y), cell(p.z))].push_back((int)pts.size() - 1);
    dirty = true;
  }
  void reindex() {
    grid.clear();
    for (size_t i = 0; i < pts.size(); i++) grid[key(cell(pts[i].x), cell(pts[i].y), cell(pts[i].z))].push_back((int)i);
    dirty = true;
  }
  // Build (ikd_Tree.cpp:470-492): the tree holds exactly the given points.
  void build(const float* p, int n, int stride) {
    pts.clear();
    n_dead = 0;
    next_id = 0;
    for (int i = 0; i < n; i++) pts.push_back(MapPoint{p[i * stride], p[i * stride + 1], p[i * stride + 2], next_id++});
    reindex();
  }
  // Search_by_range (ikd_Tree.cpp:1607-1645): live points with min <= p < max on every axis,
  // ascending id (ikd's traversal order is unknowable; only ties depend on it).
  void search_by_range(const float* bmin, const float* bmax, std::vector<int>& out) const {
    out.clear();
    const int c0[3] = {cell(bmin[0]) - 1, cell(bmin[1]) - 1, cell(bmin[2]) - 1};
    const int c1[3] = {cell(bmax[0]) + 1, cell(bmax[1]) + 1, cell(bmax[2]) + 1};
    for (int ix = c0[0]; ix <= c1[0]; ix++)
      for (int iy = c0[1]; iy <= c1[1]; iy++)
        for (int iz = c0[2]; iz <= c1[2]; iz++) {
          auto it = grid.find(key(ix, iy, iz));
          if (it == grid.end()) continue;
          for (int i : it->second) {
            const MapPoint& q = pts[i];
            if (q.dead) continue;
            if (bmin[0] <= q.x && bmax[0] > q.x && bmin[1] <= q.y && bmax[1] > q.y && bmin[2] <= q.z && bmax[2] > q.z)
              out.push_back(i);
          }
        }
    std::sort(out.begin(), out.end(), [&](int a, int b) { return pts[a].id < pts[b].id; });
  }
  void remove(const std::vector<int>& idx) {  // Delete_by_range: the points leave the set
    for (int i : idx) pts[i].dead = true;
    n_dead += (int)idx.size();
    dirty = true;
  }
  void compact() {
    if (n_dead == 0) return;
    std::vector<MapPoint> keep;
    keep.reserve(pts.size() - n_dead);
    for (const MapPoint& p : pts)
      if (!p.dead) keep.push_back(p);
    pts.swap(keep);
    n_dead = 0;
    reindex();
  }
  int live() const { return (int)pts.size() - n_dead; }
  // Add_Points (ikd_Tree.cpp:569-706), processed point by point as the reference does.
  int add_points(const float* p, int n, int stride, bool downsample_on) {
    const int base = next_id;
    next_id += n;
    int counter = 0;
    std::vector<int> S;
    for (int i = 0; i < n; i++) {
      MapPoint np{p[i * stride], p[i * stride + 1], p[i * stride + 2], base + i};
      if (!downsample_on) {
        insert(np);
        continue;
      }
      const float L = downsample_size;
      float bmin[3], bmax[3], mid[3];
      const float c[3] = {np.x, np.y, np.z};
      for (int k = 0; k < 3; k++) {
        bmin[k] = std::floor(c[k] / L) * L;
        bmax[k] = bmin[k] + L;
        mid[k] = (float)(bmin[k] + (bmax[k] - bmin[k]) / 2.0);
      }
      search_by_range(bmin, bmax, S);
      float min_dist = calc_dist(np.x, np.y, np.z, mid[0], mid[1], mid[2]);
      MapPoint result = np;
      for (int s : S) {
        const float d = calc_dist(pts[s].x, pts[s].y, pts[s].z, mid[0], mid[1], mid[2]);
        if (d < min_dist) { min_dist = d; result = pts[s]; }
      }
      const bool same = std::fabs(np.x - result.x) < 1e-6f && std::fabs(np.y - result.y) < 1e-6f &&
                        std::fabs(np.z - result.z) < 1e-6f;
      if (S.size() > 1 || same) {
        if (!S.empty()) remove(S);
        insert(result);
        counter++;
      }
    }
    return counter;
  }
  void ensure_tree() {
    if (dirty) { compact(); tree.build(pts); dirty = false; }
  }
  // Nearest_Search (ikd_Tree.cpp:494-547): up to k points with dist <= max_dist^2, ascending.
  int nearest(const float* q, int k, double max_dist, MapPoint* out, float* d2) {
    ensure_tree();
    std::vector<KnnTree::Best> best;
    const float maxd2 = std::isinf(max_dist) ? INFINITY : (float)(max_dist * max_dist);
    if (!tree.nodes.empty()) tree.search(0, q, k, maxd2, best);
    for (size_t j = 0; j < best.size(); j++) {
      out[j] = tree.pts[best[j].idx];
      d2[j] = best[j].d;
    }
    return (int)best.size();
  }
};

// ------------------------------------------------------------------ fits
// Eigen::ColPivHouseholderQR<Matrix<double,5,3>>::compute + solve(b = -1): column-pivoted
// Householder QR, norm downdating, rank from the threshold, R^-1 Q^T b, un-permuted.
static void colpiv_qr_solve_5x3(const double A_in[5][3], double x[3]) {
  const int R = 5, C = 3;
  double A[5][3];
  std::memcpy(A, A_in, sizeof(A));
  double upd[3], dir[3], tau[3];
  int trans[3];
  double maxn = 0;
  for (int j = 0; j < C; j++) {
    double s = 0;
    for (int i = 0; i < R; i++) s += A[i][j] * A[i][j];
    upd[j] = dir[j] = std::sqrt(s);
    maxn = std::max(maxn, upd[j]);
  }
  const double eps = DBL_EPSILON;
  const double thr = (maxn * eps) * (maxn * eps) / R;
  const double downdate = std::sqrt(eps);
  int nonzero = C;
  for (int k = 0; k < C; k++) {
    int big = k;
    for (int j = k + 1; j < C; j++)
      if (upd[j] > upd[big]) big = j;
    const double bsq = upd[big] * upd[big];
    if (nonzero == C && bsq < thr * (R - k)) nonzero = k;
    trans[k] = big;
    if (k != big) {
      for (int i = 0; i < R; i++) std::swap(A[i][k], A[i][big]);
      std::swap(upd[k], upd[big]);
      std::swap(dir[k], dir[big]);
    }
    // makeHouseholderInPlace on A[k..R-1][k]
    const double c0 = A[k][k];
    double tail = 0;
    for (int i = k + 1; i < R; i++) tail += A[i][k] * A[i][k];
    double beta;
    if (tail <= DBL_MIN) {
      tau[k] = 0;
      beta = c0;
      for (int i = k + 1; i < R; i++) A[i][k] = 0;
    } else {
      beta = std::sqrt(c0 * c0 + tail);
      if (c0 >= 0) beta = -beta;
      for (int i = k + 1; i < R; i++) A[i][k] = A[i][k] / (c0 - beta);
      tau[k] = (beta - c0) / beta;
    }
    A[k][k] = beta;
    // applyHouseholderOnTheLeft to the trailing columns
    for (int j = k + 1; j < C; j++) {
      if (tau[k] == 0) continue;
      double t = A[k][j];
      for (int i = k + 1; i < R; i++) t += A[i][k] * A[i][j];
      A[k][j] -= tau[k] * t;
      for (int i = k + 1; i < R; i++) A[i][j] -= tau[k] * A[i][k] * t;
    }
    for (int j = k + 1; j < C; j++) {
      if (upd[j] == 0) continue;
      double t = std::fabs(A[k][j]) / upd[j];
      t = (1 + t) * (1 - t);
      t = t < 0 ? 0 : t;
      const double t2 = t * (upd[j] / dir[j]) * (upd[j] / dir[j]);
      if (t2 <= downdate) {
        double s = 0;
        for (int i = k + 1; i < R; i++) s += A[i][j] * A[i][j];
        dir[j] = upd[j] = std::sqrt(s);
      } else {
        upd[j] *= std::sqrt(t);
      }
    }
  }
  int perm[3] = {0, 1, 2};
  for (int k = 0; k < C; k++) std::swap(perm[k], perm[trans[k]]);
  double c[5] = {-1, -1, -1, -1, -1};
  for (int k = 0; k < nonzero; k++) {
    if (tau[k] == 0) continue;
    double t = c[k];
    for (int i = k + 1; i < R; i++) t += A[i][k] * c[i];
    c[k] -= tau[k] * t;
    for (int i = k + 1; i < R; i++) c[i] -= tau[k] * A[i][k] * t;
  }
  for (int i = nonzero - 1; i >= 0; i--) {  // column-oriented back substitution
    c[i] /= A[i][i];
    for (int r = 0; r < i; r++) c[r] -= A[r][i] * c[i];
  }
  for (int i = 0; i < C; i++) x[perm[i]] = i < nonzero ? c[i] : 0.0;
}

// Plane of 5 neighbours (laserMapping.cpp:756-788, mapOptimization.cpp:398-420): A n = -1,
// d = 1/|n|, n normalized, valid iff |n.p + d| <= 0.2 for all five.
static bool plane_fit(const MapPoint* nb, double n[3], double* d) {
  double A[5][3];
  for (int j = 0; j < 5; j++) { A[j][0] = nb[j].x; A[j][1] = nb[j].y; A[j][2] = nb[j].z; }
  colpiv_qr_solve_5x3(A, n);
  const double nn = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  *d = 1 / nn;
  if (nn > 0) { n[0] /= nn; n[1] /= nn; n[2] /= nn; }
  for (int j = 0; j < 5; j++)
    if (std::fabs(n[0] * nb[j].x + n[1] * nb[j].y + n[2] * nb[j].z + *d) > 0.2) return false;
  return true;
}

// Symmetric 3x3 eigen-decomposition by cyclic Jacobi; eigenvalues ascending, v[:, k] the vectors.
static void sym_eig3(const double M[3][3], double w[3], double V[3][3]) {
  double a[3][3];
  std::memcpy(a, M, sizeof(a));
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) V[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 32; sweep++) {
    const double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    if (off == 0.0) break;
    for (int p = 0; p < 2; p++)
      for (int q = p + 1; q < 3; q++) {
        if (a[p][q] == 0.0) continue;
        const double theta = (a[q][q] - a[p][p]) / (2.0 * a[p][q]);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; k++) {  // a = J^T a J
          const double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; k++) {
          const double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 3; k++) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
  int ord[3] = {0, 1, 2};
  for (int i = 0; i < 3; i++)
    for (int j = i + 1; j < 3; j++)
      if (a[ord[j]][ord[j]] < a[ord[i]][ord[i]]) std::swap(ord[i], ord[j]);
  double W[3][3];
  for (int k = 0; k < 3; k++) {
    w[k] = a[ord[k]][ord[k]];
    for (int i = 0; i < 3; i++) W[i][k] = V[i][ord[k]];
  }
  std::memcpy(V, W, sizeof(W));
}

// Line of 5 neighbours (laserMapping.cpp:681-723): centroid, covariance, principal direction;
// valid iff lambda_2 > 3 lambda_1; a, b = centroid -/+ 0.1 v.
static bool line_fit(const MapPoint* nb, double pa[3], double pb[3]) {
  double c[3] = {0, 0, 0};
  for (int j = 0; j < 5; j++) { c[0] = c[0] + nb[j].x; c[1] = c[1] + nb[j].y; c[2] = c[2] + nb[j].z; }
  for (int k = 0; k < 3; k++) c[k] = c[k] / 5.0;
  double M[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  for (int j = 0; j < 5; j++) {
    const double z[3] = {nb[j].x - c[0], nb[j].y - c[1], nb[j].z - c[2]};
    for (int r = 0; r < 3; r++)
      for (int s = 0; s < 3; s++) M[r][s] = M[r][s] + z[r] * z[s];
  }
  double w[3], V[3][3];
  sym_eig3(M, w, V);
  if (!(w[2] > 3 * w[1])) return false;
  for (int k = 0; k < 3; k++) {
    pa[k] = 0.1 * V[k][2] + c[k];
    pb[k] = -0.1 * V[k][2] + c[k];
  }
  return true;
}

// Eigen q * v (_transformVector), as in the odometry restatement.
static void qrot(const double* q, const double* v, double* o) {
  const double u[3] = {2 * (q[1] * v[2] - q[2] * v[1]), 2 * (q[2] * v[0] - q[0] * v[2]), 2 * (q[0] * v[1] - q[1] * v[0])};
  const double c[3] = {q[1] * u[2] - q[2] * u[1], q[2] * u[0] - q[0] * u[2], q[0] * u[1] - q[1] * u[0]};
  for (int k = 0; k < 3; k++) o[k] = (v[k] + q[3] * u[k]) + c[k];
}

// pointAssociateToMap (laserMapping.cpp:138-147) / mapOptimization.cpp:385: double transform,
// stored as float.
static void to_world(const double* x, const float* p, float* w) {
  const double v[3] = {p[0], p[1], p[2]};
  double o[3];
  qrot(x, v, o);
  for (int k = 0; k < 3; k++) w[k] = (float)(o[k] + x[4 + k]);
}

// Association of one query against a map: kind 0 corner (line), 1 surf (plane).
// Record layout (9 doubles): edge = curr(3), a(3), b(3); plane-norm = curr(3), n(3), d, 0, 0.
static bool associate(IkdMap& m, int kind, const float* p, const double* x, double* rec) {
  float w[3];
  to_world(x, p, w);
  MapPoint nb[5];
  float d2[5];
  const int found = m.nearest(w, 5, INFINITY, nb, d2);
  if (found < 5 || !(d2[4] < 1.0)) return false;
  rec[0] = p[0]; rec[1] = p[1]; rec[2] = p[2];
  if (kind == 0) return line_fit(nb, rec + 3, rec + 6);
  double n[3], d;
  if (!plane_fit(nb, n, &d)) return false;
  rec[3] = n[0]; rec[4] = n[1]; rec[5] = n[2]; rec[6] = d; rec[7] = 0; rec[8] = 0;
  return true;
}

// kind 0 LidarEdgeFactor(curr, a, b, 1.0), 2 LidarPlaneNormFactor(curr, n, d); -1 none.
static void add_block(Problem& P, int kind, const double* rec) {
  if (kind < 0) return;
  Block b{};
  if (kind == 0) {
    b.kind = 0;
    for (int k = 0; k < 3; k++) { b.e.cp[k] = rec[k]; b.e.pa[k] = rec[3 + k]; b.e.pb[k] = rec[6 + k]; }
    b.e.s = 1.0;
  } else {
    b.kind = 2;
    for (int k = 0; k < 3; k++) { b.pn.cp[k] = rec[k]; b.pn.n[k] = rec[3 + k]; }
    b.pn.d = rec[6];
  }
  P.blocks.push_back(b);
}

}  // namespace oracle

using namespace oracle;

extern "C" {

void* oracle_map_create(float downsample_size) {
  IkdMap* m = new IkdMap();
  m->downsample_size = downsample_size;
  return m;
}
void oracle_map_destroy(void* h) { delete static_cast<IkdMap*>(h); }
void oracle_map_build(void* h, const float* p, int n, int stride) { static_cast<IkdMap*>(h)->build(p, n, stride); }
int oracle_map_add_points(void* h, const float* p, int n, int stride, int downsample) {
  return static_cast<IkdMap*>(h)->add_points(p, n, stride, downsample != 0);
}
int oracle_map_size(void* h) { return static_cast<IkdMap*>(h)->live(); }
// Live points (x, y, z, id as float bits) in ascending id.
int oracle_map_points(void* h, float* out) {
  IkdMap* m = static_cast<IkdMap*>(h);
  m->compact();
  std::vector<MapPoint> v = m->pts;
  std::sort(v.begin(), v.end(), [](const MapPoint& a, const MapPoint& b) { return a.id < b.id; });
  for (size_t i = 0; i < v.size(); i++) {
    out[i * 4 + 0] = v[i].x; out[i * 4 + 1] = v[i].y; out[i * 4 + 2] = v[i].z;
    std::memcpy(&out[i * 4 + 3], &v[i].id, 4);
  }
  return (int)v.size();
}
// Batched Nearest_Search: out_pts[n][k][4] (x, y, z, id bits), out_d2[n][k], out_found[n].
void oracle_map_knn(void* h, const float* q, int n, int stride, int k, double max_dist, float* out_pts, float* out_d2,
                    int* out_found) {
  IkdMap* m = static_cast<IkdMap*>(h);
  std::vector<MapPoint> nb(k);
  std::vector<float> d2(k);
  for (int i = 0; i < n; i++) {
    const int f = m->nearest(q + (size_t)i * stride, k, max_dist, nb.data(), d2.data());
    out_found[i] = f;
    for (int j = 0; j < k; j++) {
      float* o = out_pts + ((size_t)i * k + j) * 4;
      if (j < f) {
        o[0] = nb[j].x; o[1] = nb[j].y; o[2] = nb[j].z;
        std::memcpy(&o[3], &nb[j].id, 4);
        out_d2[(size_t)i * k + j] = d2[j];
      } else {
        o[0] = o[1] = o[2] = 0; o[3] = 0;
        out_d2[(size_t)i * k + j] = INFINITY;
      }
    }
  }
}
// Association records (9 doubles) and block kinds (0 edge, 2 plane-norm, -1 none) for n
// sensor-frame queries at pose x (q4, t3); kind 0 = corner (line), 1 = surf (plane).
void oracle_map_associate(void* h, int kind, const float* p, int n, int stride, const double* x, double* rec,
                          int* out_kind) {
  IkdMap* m = static_cast<IkdMap*>(h);
  for (int i = 0; i < n; i++) {
    double* r = rec + (size_t)i * 9;
    for (int e = 0; e < 9; e++) r[e] = 0;
    out_kind[i] = associate(*m, kind, p + (size_t)i * stride, x, r) ? (kind == 0 ? 0 : 2) : -1;
  }
}
// Ceres solve over given records (kind per block 0 edge / 2 plane-norm / -1 skipped), Huber(0.1).
// summary[0] iterations, [1] termination.
void oracle_map_solve(const double* rec, const int* kind, int n, double* x, int max_iterations, int* summary) {
  Problem P;
  P.huber_a = 0.1;
  for (int i = 0; i < n; i++) add_block(P, kind[i], rec + (size_t)i * 9);
  SolveSummary s = ceres_solve(P, x, max_iterations);
  summary[0] = s.iterations;
  summary[1] = s.termination;
}

// One mapOptimization ground step (mapOptimization.cpp:99-479 minus the ORB / keyframe image
// logic): ground = GroundPointOut (sensor frame, xyz stride 4), odom = q_wodom_curr, t_wodom_curr
// (7), state = q_wmap_wodom, t_wmap_wodom (7, in/out).  First call (empty map): Build with the
// transformed raw cloud (:185-192).  Otherwise VoxelGrid(0.8) (:368-370), plane association
// (:376-429), Ceres(10 it) (:433-442), transformUpdate on CONVERGENCE (:448-450, :740-746) and
// Add_Points(downsample) of the voxelized cloud at the keyframe pose (:453-475).
// out_pose = q_w_curr, t_w_curr after the step; summary = planes, iterations, termination.
int oracle_voxel_grid(const float* xyzi, int n, float leaf, int canonical, float* out, int* n_out);
void oracle_mapopt_step_corner(void* h, void* hc, const float* ground, int n, const float* corner, int nc,
                               const double* odom, double* state, double* out_pose, int* summary);

void oracle_mapopt_step(void* h, const float* ground, int n, const double* odom, double* state, double* out_pose,
                        int* summary) {
  oracle_mapopt_step_corner(h, nullptr, ground, n, nullptr, 0, odom, state, out_pose, summary);
}

// With mapOptimization's corner ikd-Tree (corner_ikdtree_, KD_TREE(0.3, 0.6, 0.8),
// mapOptimization.cpp:505): pc_corner transformed by the same keyframe pose as the ground cloud,
// Build on the first keyframe (:193-195), Add_Points(downsample) afterwards (:477-479).
void oracle_mapopt_step_corner(void* h, void* hc, const float* ground, int n, const float* corner, int nc,
                               const double* odom, double* state, double* out_pose, int* summary) {
  IkdMap* m = static_cast<IkdMap*>(h);
  IkdMap* cm = static_cast<IkdMap*>(hc);
  const double* qo = odom;
  const double* to = odom + 4;
  double* qm = state;
  double* tm = state + 4;
  // transformAssociateToMap (:730-736)
  Q4<double> qw = qmul(Q4<double>{qm[0], qm[1], qm[2], qm[3]}, Q4<double>{qo[0], qo[1], qo[2], qo[3]});
  double x[7] = {qw.x, qw.y, qw.z, qw.w, 0, 0, 0};
  double tr[3];
  qrot(qm, to, tr);
  for (int k = 0; k < 3; k++) x[4 + k] = tr[k] + tm[k];
  summary[0] = summary[1] = 0;
  summary[2] = -1;
  auto transformed = [&](const float* src, int cnt, const double* pose, std::vector<float>& dst) {
    // pcl::transformPointCloud with the 4x4 of (q, t): float points, double matrix products
    dst.assign((size_t)cnt * 4, 0.f);
    for (int i = 0; i < cnt; i++) to_world(pose, src + (size_t)i * 4, &dst[(size_t)i * 4]);
  };
  // Build on the ground map's first keyframe, Add_Points(downsample) afterwards, whatever the
  // corner tree holds (an empty first pc_corner leaves it empty until a later Add_Points)
  auto corner_update = [&](const double* pose, bool first) {
    if (!cm || nc <= 0) return;
    std::vector<float> w;
    transformed(corner, nc, pose, w);
    if (first) cm->build(w.data(), nc, 4);
    else cm->add_points(w.data(), nc, 4, true);
  };
  if (m->live() == 0) {
    std::vector<float> w;
    transformed(ground, n, x, w);
    m->build(w.data(), n, 4);
    corner_update(x, true);
    for (int e = 0; e < 7; e++) out_pose[e] = x[e];
    return;
  }
  std::vector<float> vox((size_t)std::max(n, 1) * 4);
  int nv = 0;
  std::vector<float> g4((size_t)n * 4);
  for (int i = 0; i < n; i++) {  // PointXYZ: only x, y, z are averaged
    g4[i * 4 + 0] = ground[i * 4 + 0]; g4[i * 4 + 1] = ground[i * 4 + 1]; g4[i * 4 + 2] = ground[i * 4 + 2];
    g4[i * 4 + 3] = 0;
  }
  oracle_voxel_grid(g4.data(), n, 0.8f, 1, vox.data(), &nv);
  const double x0[7] = {x[0], x[1], x[2], x[3], x[4], x[5], x[6]};
  Problem P;
  P.huber_a = 0.1;
  for (int i = 0; i < nv; i++) {
    double rec[9];
    if (associate(*m, 1, &vox[(size_t)i * 4], x, rec)) add_block(P, 2, rec);
  }
  summary[0] = (int)P.blocks.size();
  SolveSummary s = ceres_solve(P, x, 10);
  summary[1] = s.iterations;
  summary[2] = s.termination;
  const bool conv = s.termination == 1;
  if (conv) {  // transformUpdate: q_wmap_wodom = q_w_curr q_wodom^-1; t_wmap_wodom = t_w_curr - q_wmap_wodom t_wodom
    Q4<double> qinv{-qo[0], -qo[1], -qo[2], qo[3]};
    Q4<double> nq = qmul(Q4<double>{x[0], x[1], x[2], x[3]}, qinv);
    qm[0] = nq.x; qm[1] = nq.y; qm[2] = nq.z; qm[3] = nq.w;
    double r[3];
    qrot(qm, to, r);
    for (int k = 0; k < 3; k++) tm[k] = x[4 + k] - r[k];
  }
  std::vector<float> w;
  transformed(vox.data(), nv, conv ? x : x0, w);
  m->add_points(w.data(), nv, 4, true);
  corner_update(conv ? x : x0, false);
  for (int e = 0; e < 7; e++) out_pose[e] = x[e];
}

// One laserMapping optimization (laserMapping.cpp:620-875): corner / surf maps, downsampled
// current corner / surf stacks (sensor frame, stride 4), pose x (in/out, = parameters), two
// outer passes of association + Ceres(4 it).  stats[4] = corners, surfs of pass 0 / 1.
void oracle_laser_mapping(void* hc, void* hs, const float* corner, int nc, const float* surf, int ns, double* x,
                          int* stats) {
  IkdMap* mc = static_cast<IkdMap*>(hc);
  IkdMap* ms = static_cast<IkdMap*>(hs);
  for (int outer = 0; outer < 2; outer++) {
    Problem P;
    P.huber_a = 0.1;
    int cn = 0, sn = 0;
    for (int i = 0; i < nc; i++) {
      double rec[9];
      if (associate(*mc, 0, corner + (size_t)i * 4, x, rec)) { add_block(P, 0, rec); cn++; }
    }
    for (int i = 0; i < ns; i++) {
      double rec[9];
      if (associate(*ms, 1, surf + (size_t)i * 4, x, rec)) { add_block(P, 2, rec); sn++; }
    }
    stats[outer * 2] = cn;
    stats[outer * 2 + 1] = sn;
    ceres_solve(P, x, 4);
  }
}

}  // extern "C"

// ------------------------------------------------------------------ laserMapping cube map
// The A-LOAM local map of laserMapping::process: 21 x 21 x 11 cubes of
// 50 m (laserMapping.cpp:70-99) holding the corner / surf points in map frame.  One frame
// (:319-1002, without publishing; the duplicated surf insert :950-981 dropped, SURVEY.md §8(c)
// repair 2): transformAssociateToMap (:138-142), re-centring shifts (:330-565), the local map of
// the <= 5 x 5 x 3 valid cubes in i, j, k loop order (:566-602), VoxelGrid of the current corner /
// surf clouds (:608-616), the optimization when the map holds > 10 corner and > 50 surf points
// (:620-857, oracle_laser_mapping), transformUpdate (:145-149, Eigen's Quaternion::inverse),
// insertion of the voxelized clouds at the optimized pose (:880-949) and a VoxelGrid of every
// valid cube (:984-1002).
namespace oracle {
struct CubeMap {
  static constexpr int W = 21, H = 21, D = 11, NC = W * H * D;
  int cenW = 10, cenH = 10, cenD = 5;
  float line_res = 0.4f, plane_res = 0.8f;
  std::vector<std::vector<P4>> corner, surf;
  CubeMap() : corner(NC), surf(NC) {}
};
}  // namespace oracle

extern "C" {

void* oracle_lmap_create(float line_res, float plane_res) {
  auto* m = new oracle::CubeMap();
  m->line_res = line_res;
  m->plane_res = plane_res;
  return m;
}
void oracle_lmap_destroy(void* h) { delete static_cast<oracle::CubeMap*>(h); }

// cube counts (corner, surf) in cube index order
void oracle_lmap_counts(void* h, int* cc, int* sc) {
  auto* m = static_cast<oracle::CubeMap*>(h);
  for (int i = 0; i < oracle::CubeMap::NC; i++) { cc[i] = (int)m->corner[i].size(); sc[i] = (int)m->surf[i].size(); }
}
// all points of one cloud (0 corner, 1 surf) in cube index order; returns the count
int oracle_lmap_points(void* h, int which, float* out) {
  auto* m = static_cast<oracle::CubeMap*>(h);
  auto& arr = which ? m->surf : m->corner;
  int n = 0;
  for (auto& v : arr)
    for (auto& p : v) {
      if (out) { out[4 * n] = p.x; out[4 * n + 1] = p.y; out[4 * n + 2] = p.z; out[4 * n + 3] = p.i; }
      n++;
    }
  return n;
}

// stats[8] = corner / surf local-map sizes, corner / surf stack sizes, optimization stats of
// oracle_laser_mapping (-1 when the map is too small to optimize); out_pose = q_w_curr, t_w_curr.
void oracle_lmap_step(void* h, const float* corner_last, int nc, const float* surf_last, int ns, const double* odom,
                      double* state, double* out_pose, int* stats) {
  using oracle::CubeMap;
  using oracle::P4;
  auto* m = static_cast<CubeMap*>(h);
  const int W = CubeMap::W, H = CubeMap::H, D = CubeMap::D;
  const double* qo = odom;
  const double* to = odom + 4;
  double* qm = state;
  double* tm = state + 4;
  // transformAssociateToMap
  oracle::Q4<double> qw = oracle::qmul(oracle::Q4<double>{qm[0], qm[1], qm[2], qm[3]}, oracle::Q4<double>{qo[0], qo[1], qo[2], qo[3]});
  double x[7] = {qw.x, qw.y, qw.z, qw.w, 0, 0, 0};
  {
    double tr[3];
    oracle::qrot(qm, to, tr);
    for (int k = 0; k < 3; k++) x[4 + k] = tr[k] + tm[k];
  }
  // re-centring (the pointer rotations of :340-565; the cube that wraps around is cleared)
  auto cube_of = [](double v, int cen) {
    int c = int((v + 25.0) / 50.0) + cen;
    if (v + 25.0 < 0) c--;
    return c;
  };
  int cI = cube_of(x[4], m->cenW), cJ = cube_of(x[5], m->cenH), cK = cube_of(x[6], m->cenD);
  auto at = [&](int i, int j, int k) { return i + W * j + W * H * k; };
  auto rot = [&](int a0, int step, int cnt) {  // a[a0 + step (cnt-1)] <- ... <- a[a0], a[a0] <- old last, cleared
    for (auto* arr : {&m->corner, &m->surf}) {
      std::vector<P4> last = std::move((*arr)[a0 + step * (cnt - 1)]);
      for (int t = cnt - 1; t >= 1; t--) (*arr)[a0 + step * t] = std::move((*arr)[a0 + step * (t - 1)]);
      last.clear();
      (*arr)[a0] = std::move(last);
    }
  };
  while (cI < 3) {
    for (int j = 0; j < H; j++)
      for (int k = 0; k < D; k++) rot(at(0, j, k), 1, W);
    cI++; m->cenW++;
  }
  while (cI >= W - 3) {
    for (int j = 0; j < H; j++)
      for (int k = 0; k < D; k++) rot(at(W - 1, j, k), -1, W);
    cI--; m->cenW--;
  }
  while (cJ < 3) {
    for (int i = 0; i < W; i++)
      for (int k = 0; k < D; k++) rot(at(i, 0, k), W, H);
    cJ++; m->cenH++;
  }
  while (cJ >= H - 3) {
    for (int i = 0; i < W; i++)
      for (int k = 0; k < D; k++) rot(at(i, H - 1, k), -W, H);
    cJ--; m->cenH--;
  }
  while (cK < 3) {
    for (int i = 0; i < W; i++)
      for (int j = 0; j < H; j++) rot(at(i, j, 0), W * H, D);
    cK++; m->cenD++;
  }
  while (cK >= D - 3) {
    for (int i = 0; i < W; i++)
      for (int j = 0; j < H; j++) rot(at(i, j, D - 1), -W * H, D);
    cK--; m->cenD--;
  }
  // valid cubes and the local map
  std::vector<int> valid;
  for (int i = cI - 2; i <= cI + 2; i++)
    for (int j = cJ - 2; j <= cJ + 2; j++)
      for (int k = cK - 1; k <= cK + 1; k++)
        if (i >= 0 && i < W && j >= 0 && j < H && k >= 0 && k < D) valid.push_back(at(i, j, k));
  std::vector<float> cmap, smap;
  for (int v : valid) {
    for (auto& p : m->corner[v]) cmap.insert(cmap.end(), {p.x, p.y, p.z, p.i});
    for (auto& p : m->surf[v]) smap.insert(smap.end(), {p.x, p.y, p.z, p.i});
  }
  const int ncm = (int)cmap.size() / 4, nsm = (int)smap.size() / 4;
  // current clouds, voxelized
  std::vector<float> cst((size_t)std::max(nc, 1) * 4), sst((size_t)std::max(ns, 1) * 4);
  int ncs = 0, nss = 0;
  oracle_voxel_grid(corner_last, nc, m->line_res, 1, cst.data(), &ncs);
  oracle_voxel_grid(surf_last, ns, m->plane_res, 1, sst.data(), &nss);
  stats[0] = ncm; stats[1] = nsm; stats[2] = ncs; stats[3] = nss;
  stats[4] = stats[5] = stats[6] = stats[7] = -1;
  if (ncm > 10 && nsm > 50) {
    oracle::IkdMap mc, ms;
    mc.build(cmap.data(), ncm, 4);
    ms.build(smap.data(), nsm, 4);
    oracle_laser_mapping(&mc, &ms, cst.data(), ncs, sst.data(), nss, x, stats + 4);
  }
  // transformUpdate: q_wmap_wodom = q_w_curr * q_wodom_curr.inverse(); t_wmap_wodom = t_w_curr - q_wmap_wodom * t_wodom_curr
  {
    const double n2 = (qo[0] * qo[0] + qo[2] * qo[2]) + (qo[1] * qo[1] + qo[3] * qo[3]);  // Eigen SSE2 squaredNorm
    const oracle::Q4<double> qinv{-qo[0] / n2, -qo[1] / n2, -qo[2] / n2, qo[3] / n2};
    const oracle::Q4<double> nq = oracle::qmul(oracle::Q4<double>{x[0], x[1], x[2], x[3]}, qinv);
    qm[0] = nq.x; qm[1] = nq.y; qm[2] = nq.z; qm[3] = nq.w;
    double r[3];
    oracle::qrot(qm, to, r);
    for (int k = 0; k < 3; k++) tm[k] = x[4 + k] - r[k];
  }
  // insertion (pointAssociateToMap at the optimized pose)
  auto insert = [&](const std::vector<float>& stack, int n, std::vector<std::vector<P4>>& arr) {
    for (int i = 0; i < n; i++) {
      float w[3];
      oracle::to_world(x, &stack[(size_t)i * 4], w);
      const int ci = cube_of(w[0], m->cenW), cj = cube_of(w[1], m->cenH), ck = cube_of(w[2], m->cenD);
      if (ci >= 0 && ci < W && cj >= 0 && cj < H && ck >= 0 && ck < D) arr[at(ci, cj, ck)].push_back(P4{w[0], w[1], w[2], stack[(size_t)i * 4 + 3]});
    }
  };
  insert(cst, ncs, m->corner);
  insert(sst, nss, m->surf);
  // VoxelGrid of the valid cubes
  for (int v : valid) {
    for (int t = 0; t < 2; t++) {
      auto& cube = t == 0 ? m->corner[v] : m->surf[v];
      const int n = (int)cube.size();
      std::vector<P4> o((size_t)std::max(n, 1));
      int no = 0;
      oracle_voxel_grid(reinterpret_cast<const float*>(cube.data()), n, t == 0 ? m->line_res : m->plane_res, 1,
                        reinterpret_cast<float*>(o.data()), &no);
      o.resize(no);
      cube = std::move(o);
    }
  }
  for (int e = 0; e < 7; e++) out_pose[e] = x[e];
}

}  // extern "C"

// ------------------------------------------------------------------ loop-closure ICP
// feature_tracker::loopClosureThread's USE_ICP block (src/intensity_feature_tracker.cpp:217-366)
// with its helpers tranformCurrentScanToMap (:167-172) and getSubmapOfhistory (:174-193):
//   current = keyframe cloud_track transformed by T_cur (pcl::transformPointCloud with a Matrix4d:
//   per point ((T00 x + T01 y) + T02 z) + T03 in double, stored as float; intensity copied),
//   submap = the history keyframes' clouds transformed by their poses, concatenated in order;
//   removeNaNFromPointCloud (non-finite x, y or z dropped), CropBox [-crop, crop]^3 inclusive
//   (USE_CROP), VoxelGrid(vf_scan_res) (USE_DOWNSAMPLE), and when both clouds hold > 10 points
//   pcl::IterativeClosestPoint (PCL 1.10, absent here: restated from its published algorithm):
//     setMaxCorrespondenceDistance(100), setMaximumIterations(100), setTransformationEpsilon(1e-6),
//     setEuclideanFitnessEpsilon(1e-6), RANSAC iterations 0 (:219-223).
//   Each iteration: CorrespondenceEstimation (1-NN of every source point in the target, squared
//   float distance <= max^2; ties by target index), < 3 correspondences -> NO_CORRESPONDENCES;
//   TransformationEstimationSVD (umeyama without scaling) — the rotation maximising
//   trace(R^T Sigma) is taken from Horn's 4x4 quaternion eigenproblem in double (cyclic Jacobi):
//   the same minimiser as Eigen's JacobiSVD route, parity against PCL's float SVD unpinned; the
//   float transformation_ is applied to the source (((m00 x + m01 y) + m02 z) + m03 in float),
//   final = transformation_ * final (float 4x4, k = 0..3 left to right); then
//   DefaultConvergenceCriteria (max iterations -> ITERATIONS, translation^2 <= eps and
//   cos(angle) >= 1 - eps -> TRANSFORM, |dMSE| < 1e-12 -> ABS_MSE, |dMSE| / MSE_prev < fitness eps
//   -> REL_MSE; max_iterations_similar_transforms 0).  getFitnessScore: the original source under
//   `final`, mean 1-NN squared distance.  accepted = converged && fitness <= icp_fitness_score
//   (:314); T_cur2map_gt = double(final) * T_cur (:316-321).
// Sums over points (MSE, means, cross-covariance, fitness) use one fixed order shared with the
// device: 1024 strided partial sums in double, then a halving tree.
namespace oracle {

constexpr int kIcpRed = 1024;

template <int V, class F>
static void icp_sum(int n, F f, double out[V]) {
  std::vector<double> acc((size_t)kIcpRed * V, 0.0);
  for (int t = 0; t < kIcpRed; t++)
    for (int i = t; i < n; i += kIcpRed) {
      double v[V];
      if (f(i, v))
        for (int k = 0; k < V; k++) acc[(size_t)t * V + k] += v[k];
    }
  for (int s = kIcpRed / 2; s > 0; s >>= 1)
    for (int t = 0; t < s; t++)
      for (int k = 0; k < V; k++) acc[(size_t)t * V + k] += acc[(size_t)(t + s) * V + k];
  for (int k = 0; k < V; k++) out[k] = acc[k];
}

// cyclic Jacobi of a symmetric 4x4 (A is destroyed; V = eigenvectors in columns)
static void jacobi4(double A[4][4], double V[4][4]) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) V[i][j] = i == j ? 1.0 : 0.0;
  double tot = 0;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) tot += A[i][j] * A[i][j];
  for (int sweep = 0; sweep < 32; sweep++) {
    double off = 0;
    for (int p = 0; p < 4; p++)
      for (int q = p + 1; q < 4; q++) off += A[p][q] * A[p][q];
    if (!(off > 1e-36 * tot)) break;
    for (int p = 0; p < 4; p++)
      for (int q = p + 1; q < 4; q++) {
        const double apq = A[p][q];
        if (apq == 0.0) continue;
        const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
        double t = 1.0 / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        if (theta < 0) t = -t;
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 4; k++) {
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = c * akp - s * akq;
          A[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 4; k++) {
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = c * apk - s * aqk;
          A[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 4; k++) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
}

// umeyama(src, tgt, false) from the demeaned cross-covariance S[a][b] = mean (s_a - ms_a)(t_b - mt_b)
static void horn_rt(const double S[3][3], const double ms[3], const double mt[3], double R[3][3], double t[3]) {
  const double Sxx = S[0][0], Sxy = S[0][1], Sxz = S[0][2], Syx = S[1][0], Syy = S[1][1], Syz = S[1][2], Szx = S[2][0],
               Szy = S[2][1], Szz = S[2][2];
  double N[4][4] = {{(Sxx + Syy) + Szz, Syz - Szy, Szx - Sxz, Sxy - Syx},
                    {Syz - Szy, (Sxx - Syy) - Szz, Sxy + Syx, Szx + Sxz},
                    {Szx - Sxz, Sxy + Syx, (Syy - Sxx) - Szz, Syz + Szy},
                    {Sxy - Syx, Szx + Sxz, Syz + Szy, (Szz - Sxx) - Syy}};
  double V[4][4];
  jacobi4(N, V);
  int k = 0;
  for (int j = 1; j < 4; j++)
    if (N[j][j] > N[k][k]) k = j;
  double w = V[0][k], x = V[1][k], y = V[2][k], z = V[3][k];
  const double nn = std::sqrt(((w * w + x * x) + y * y) + z * z);
  w /= nn; x /= nn; y /= nn; z /= nn;
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;  // Eigen's toRotationMatrix
  const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y,
               tyz = tz * y, tzz = tz * z;
  R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz; R[0][2] = txz + twy;
  R[1][0] = txy + twz; R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
  R[2][0] = txz - twy; R[2][1] = tyz + twx; R[2][2] = 1 - (txx + tyy);
  for (int a = 0; a < 3; a++) t[a] = mt[a] - ((R[a][0] * ms[0] + R[a][1] * ms[1]) + R[a][2] * ms[2]);
}

static inline P4 tf_f(const float* T, const P4& p) {
  return P4{((T[0] * p.x + T[1] * p.y) + T[2] * p.z) + T[3], ((T[4] * p.x + T[5] * p.y) + T[6] * p.z) + T[7],
            ((T[8] * p.x + T[9] * p.y) + T[10] * p.z) + T[11], p.i};
}
static inline P4 tf_d(const double* T, const P4& p) {
  const double x = p.x, y = p.y, z = p.z;
  return P4{(float)(((T[0] * x + T[1] * y) + T[2] * z) + T[3]), (float)(((T[4] * x + T[5] * y) + T[6] * z) + T[7]),
            (float)(((T[8] * x + T[9] * y) + T[10] * z) + T[11]), p.i};
}

struct IcpCfg {
  int use_crop;
  float crop_size;
  int use_downsample;
  float voxel_size;
  float max_corr_dist;
  int max_iterations;
  double trans_eps, fitness_eps, fitness_threshold;
};

static void icp_prepare(const IcpCfg& cfg, std::vector<P4>& c) {
  std::vector<P4> o;
  o.reserve(c.size());
  const float lo = -cfg.crop_size, hi = cfg.crop_size;
  for (const P4& p : c) {
    if (!std::isfinite(p.x) || !std::isfinite(p.y) || !std::isfinite(p.z)) continue;
    if (cfg.use_crop && (p.x < lo || p.y < lo || p.z < lo || p.x > hi || p.y > hi || p.z > hi)) continue;
    o.push_back(p);
  }
  if (cfg.use_downsample && !o.empty()) {
    std::vector<P4> v(o.size());
    int nv = 0;
    oracle_voxel_grid(reinterpret_cast<const float*>(o.data()), (int)o.size(), cfg.voxel_size, 1,
                      reinterpret_cast<float*>(v.data()), &nv);
    v.resize(nv);
    o.swap(v);
  }
  c.swap(o);
}

}  // namespace oracle

extern "C" {

// cfg_f[4] = crop_size, voxel_size, max_corr_dist, (unused); cfg_i[4] = use_crop, use_downsample,
// max_iterations, (unused); cfg_d[3] = transformation eps, euclidean fitness eps, icp_fitness_score.
// cur: n_cur points (x, y, z, i); hist: the history clouds concatenated, hist_counts[n_hist];
// T_cur[16], T_hist[n_hist][16] row-major.  Outputs T_icp[16] (the float final transformation),
// T_cur2map[16], fitness[1], info[8] = accepted (1 / 0; -1 submap empty, -2 <= 10 points),
// converged, convergence state (0 not converged, 1 iterations, 2 transform, 3 abs MSE,
// 4 rel MSE, 5 no correspondences), iterations, source points, target points, last
// correspondences, 0.
void oracle_loop_icp(const float* cfg_f, const int* cfg_i, const double* cfg_d, const float* cur, int n_cur,
                     const double* T_cur, const float* hist, const int* hist_counts, int n_hist, const double* T_hist,
                     double* T_icp, double* T_cur2map, double* fitness, int* info) {
  using namespace oracle;
  IcpCfg cfg{cfg_i[0], cfg_f[0], cfg_i[1], cfg_f[1], cfg_f[2], cfg_i[2], cfg_d[0], cfg_d[1], cfg_d[2]};
  for (int k = 0; k < 8; k++) info[k] = 0;
  for (int k = 0; k < 16; k++) { T_icp[k] = (k % 5 == 0) ? 1.0 : 0.0; T_cur2map[k] = T_cur[k]; }
  *fitness = DBL_MAX;
  std::vector<P4> src, tgt;
  const P4* cp = reinterpret_cast<const P4*>(cur);
  for (int i = 0; i < n_cur; i++) src.push_back(tf_d(T_cur, cp[i]));
  const P4* hp = reinterpret_cast<const P4*>(hist);
  for (int h = 0, off = 0; h < n_hist; off += hist_counts[h], h++)
    for (int i = 0; i < hist_counts[h]; i++) tgt.push_back(tf_d(T_hist + 16 * h, hp[off + i]));
  if (tgt.empty()) { info[0] = -1; return; }
  icp_prepare(cfg, src);
  icp_prepare(cfg, tgt);
  const int ns = (int)src.size(), nt = (int)tgt.size();
  info[4] = ns;
  info[5] = nt;
  if (ns <= 10 || nt <= 10) { info[0] = -2; return; }
  KnnTree tree;
  {
    std::vector<MapPoint> mp(nt);
    for (int i = 0; i < nt; i++) mp[i] = MapPoint{tgt[i].x, tgt[i].y, tgt[i].z, i};
    tree.build(mp);
  }
  std::vector<int> nn(ns);
  std::vector<float> nd(ns);
  auto nearest = [&](const std::vector<P4>& q, float maxd2) {
    std::vector<KnnTree::Best> best;
    for (int i = 0; i < ns; i++) {
      best.clear();
      const float qq[3] = {q[i].x, q[i].y, q[i].z};
      tree.search(0, qq, 1, maxd2, best);
      nn[i] = best.empty() ? -1 : best[0].id;
      nd[i] = best.empty() ? 0.f : best[0].d;
    }
  };
  const float md2 = cfg.max_corr_dist * cfg.max_corr_dist;
  float F[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  std::vector<P4> cur_src = src;
  double prev_mse = DBL_MAX;
  int it = 0, state = 0;
  const double rot_thr = 1.0 - cfg.trans_eps, trans_thr = cfg.trans_eps, mse_abs = 1e-12, mse_rel = cfg.fitness_eps;
  while (true) {
    nearest(cur_src, md2);
    double s1[8];
    icp_sum<8>(ns, [&](int i, double* v) {
      if (nn[i] < 0) return false;
      const P4& t = tgt[nn[i]];
      v[0] = 1; v[1] = nd[i];
      v[2] = cur_src[i].x; v[3] = cur_src[i].y; v[4] = cur_src[i].z;
      v[5] = t.x; v[6] = t.y; v[7] = t.z;
      return true;
    }, s1);
    const int cnt = (int)s1[0];
    info[6] = cnt;
    if (cnt < 3) { state = 5; break; }
    const double ms[3] = {s1[2] / s1[0], s1[3] / s1[0], s1[4] / s1[0]}, mt[3] = {s1[5] / s1[0], s1[6] / s1[0], s1[7] / s1[0]};
    double s2[9];
    icp_sum<9>(ns, [&](int i, double* v) {
      if (nn[i] < 0) return false;
      const P4& t = tgt[nn[i]];
      const double a[3] = {cur_src[i].x - ms[0], cur_src[i].y - ms[1], cur_src[i].z - ms[2]};
      const double b[3] = {t.x - mt[0], t.y - mt[1], t.z - mt[2]};
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) v[3 * r + c] = a[r] * b[c];
      return true;
    }, s2);
    double S[3][3], R[3][3], tr[3];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) S[r][c] = s2[3 * r + c] / s1[0];
    horn_rt(S, ms, mt, R, tr);
    float T[16] = {(float)R[0][0], (float)R[0][1], (float)R[0][2], (float)tr[0], (float)R[1][0], (float)R[1][1],
                   (float)R[1][2], (float)tr[1], (float)R[2][0], (float)R[2][1], (float)R[2][2], (float)tr[2],
                   0.f, 0.f, 0.f, 1.f};
    for (int i = 0; i < ns; i++) cur_src[i] = tf_f(T, cur_src[i]);
    float G[16];
    for (int r = 0; r < 4; r++)
      for (int c = 0; c < 4; c++)
        G[4 * r + c] = ((T[4 * r] * F[c] + T[4 * r + 1] * F[4 + c]) + T[4 * r + 2] * F[8 + c]) + T[4 * r + 3] * F[12 + c];
    std::memcpy(F, G, sizeof(F));
    ++it;
    // DefaultConvergenceCriteria::hasConverged
    if (it >= cfg.max_iterations) { state = 1; break; }
    const double cos_angle = 0.5 * ((((double)T[0] + (double)T[5]) + (double)T[10]) - 1.0);
    const double tsq = ((double)T[3] * (double)T[3] + (double)T[7] * (double)T[7]) + (double)T[11] * (double)T[11];
    if (cos_angle >= rot_thr && tsq <= trans_thr) { state = 2; break; }
    const double mse = s1[1] / s1[0];
    if (std::fabs(mse - prev_mse) < mse_abs) { state = 3; break; }
    if (std::fabs(mse - prev_mse) / prev_mse < mse_rel) { state = 4; break; }
    prev_mse = mse;
  }
  info[1] = (state >= 1 && state <= 4) ? 1 : 0;
  info[2] = state;
  info[3] = it;
  for (int k = 0; k < 16; k++) T_icp[k] = F[k];
  // getFitnessScore: the original source under final
  std::vector<P4> fsrc(ns);
  for (int i = 0; i < ns; i++) fsrc[i] = tf_f(F, src[i]);
  nearest(fsrc, INFINITY);
  double s3[2];
  icp_sum<2>(ns, [&](int i, double* v) {
    if (nn[i] < 0) return false;
    v[0] = 1; v[1] = nd[i];
    return true;
  }, s3);
  *fitness = s3[0] > 0 ? s3[1] / s3[0] : DBL_MAX;
  info[0] = (info[1] && *fitness <= cfg.fitness_threshold) ? 1 : 0;
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++)
      T_cur2map[4 * r + c] = ((T_icp[4 * r] * T_cur[c] + T_icp[4 * r + 1] * T_cur[4 + c]) + T_icp[4 * r + 2] * T_cur[8 + c]) +
                             T_icp[4 * r + 3] * T_cur[12 + c];
}

}  // extern "C"
