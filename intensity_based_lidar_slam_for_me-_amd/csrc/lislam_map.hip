// lislam scan-to-map stages on gfx950 (a19-a21 of SURVEY.md §8(a)): a device-resident point map
// with the semantics of the vendored ikd-Tree (src/ikd-Tree/ikd_Tree.cpp), exact k-NN, the 5-NN
// line / plane fits of laserMapping / mapOptimization, the PCL VoxelGrid of whole clouds, and the
// multi-workgroup Ceres-semantics pose solve.
//
// Map layout in HBM.  The ikd-Tree is a pointer-chasing balanced kd-tree; its results (which
// points a box search returns, which k points are nearest) do not depend on its layout, so the
// map is stored the way a wide GPU reads best:
//   pts   float4 [n]  (x, y, z, id bits), sorted by hash-grid cell (CSR), one 16-B load per point
//   hkey  u64 [hcap]  open-addressing table of occupied cells (21-bit biased ix, iy, iz)
//   hval  int2 [hcap] (begin, count) of the cell's points in pts
// Build = cell keys -> radix sort (rocPRIM via hipCUB) -> gather -> run-length cells into the
// table.  Add_Points rewrites the point array (live points + entering inputs) and rebuilds the
// table (one sort of the map per call).
//
// Search (k_knn).  Sixteen lanes per query (4 queries per wavefront).  The lanes walk the cells of
// the 3x3x3 block around the query's cell, then of ever larger shells; each lane keeps a sorted
// k-best list in registers, the group merges the lists with xor-shuffle lexicographic minima of
// (float squared distance, id).  A shell walk stops when k points are closer than the distance
// from the query to the faces of the walked block (every unvisited point is farther: the cell
// index floor(p / cell) is monotone in p) or when the block covers max_dist.  The result is the
// exact (distance, id)-ordered k-NN, i.e. ikd's Nearest_Search with ties broken by id.
#include <hip/hip_runtime.h>


#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lislam_prims.hpp"
#include "lislam_ctx.hpp"
#include "lislam_device.hpp"
#include "lislam_lm.hpp"
#include "lislam_lm_wave.hpp"

namespace lislam {
namespace mapk {

constexpr uint64_t kEmptyKey = ~0ull;
constexpr int kMaxShell = 24;   // beyond this the search scans the whole map (exact either way)
constexpr float kInf = __builtin_huge_valf();

__host__ __device__ __forceinline__ uint64_t pack_cell(int ix, int iy, int iz) {
  return ((uint64_t)(uint32_t)((ix + (1 << 20)) & 0x1fffff) << 42) |
         ((uint64_t)(uint32_t)((iy + (1 << 20)) & 0x1fffff) << 21) | (uint64_t)(uint32_t)((iz + (1 << 20)) & 0x1fffff);
}
__device__ __forceinline__ uint32_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return (uint32_t)k;
}
__device__ __forceinline__ int cell_of(float v, float inv) { return (int)floorf(v * inv); }

// ikd_Tree.cpp:2224-2235, left-to-right float sum (no contraction: -ffp-contract=off)
__device__ __forceinline__ float calc_dist(float ax, float ay, float az, float bx, float by, float bz) {
  return (ax - bx) * (ax - bx) + (ay - by) * (ay - by) + (az - bz) * (az - bz);
}

struct MapView {
  const float4* pts;
  const uint64_t* hkey;
  const int2* hval;
  uint32_t hmask;
  float cell, inv_cell;
  int n;
  int scan_shell;  // after this shell a query scans the whole map: the shells' cell probes would cost more
  float near2;     // first pass of the 3x3x3 block: the cells within this squared distance (< 0: all 27)
};

// The 3x3x3 block's first pass probes only the cells whose box is within LISLAM_KNN_NEAR metres of
// the query (default half a cell: the query's own cell and the 7 or fewer nearest); a second pass
// takes the block's other cells that could still beat the k-th best.  A negative value probes the
// whole block in one pass.  Either way the k-best is exact (same (distance, id) order).  Read at
// every launch (the parity tests run each setting in one process).
inline float knn_near2(float cell) {
  const char* e = getenv("LISLAM_KNN_NEAR");
  const float near = e && *e ? (float)atof(e) : 0.5f * cell;
  return near < 0 ? -1.f : near * near;
}

// first shell s whose cells walked so far (27 + sum_{j=2..s} 24 j^2 + 2) reach n / 4 point loads
inline int scan_shell_for(int64_t n) {
  int64_t cum = 27;
  int s = 1;
  while (s < kMaxShell && cum * 4 < n) {
    s++;
    cum += 24 * (int64_t)s * s + 2;
  }
  return std::max(s, 2);
}

__device__ __forceinline__ int2 cell_lookup(const MapView& m, uint64_t key) {
  uint32_t h = mix64(key) & m.hmask;
  while (true) {
    const uint64_t k = m.hkey[h];
    if (k == key) return m.hval[h];
    if (k == kEmptyKey) return make_int2(0, 0);
    h = (h + 1) & m.hmask;
  }
}

// ------------------------------------------------------------------ build
__global__ void k_cell_keys(const float4* pts, int n, float inv, uint64_t* keys, int* idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = pts[i];
  keys[i] = pack_cell(cell_of(p.x, inv), cell_of(p.y, inv), cell_of(p.z, inv));
  idx[i] = i;
}

__global__ void k_gather(const float4* src, const int* perm, int n, float4* dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[perm[i]];
}

__global__ __launch_bounds__(256) void k_count_runs(const uint64_t* keys, int n, int* count) {
  __shared__ int wsum[4];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool start = i < n && (i == 0 || keys[i] != keys[i - 1]);
  const uint64_t b = __ballot(start);
  if (lane_id() == 0) wsum[threadIdx.x >> 6] = __popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) {  // one atomic per workgroup
    const int t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (t) atomicAdd(count, t);
  }
}

__global__ void k_insert_runs(const uint64_t* keys, int n, uint64_t* hkey, int2* hval, uint32_t mask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (i > 0 && keys[i] == keys[i - 1])) return;
  const uint64_t key = keys[i];
  int e = i + 1;
  while (e < n && keys[e] == key) e++;
  uint32_t h = mix64(key) & mask;
  while (true) {
    const unsigned long long prev = atomicCAS((unsigned long long*)&hkey[h], (unsigned long long)kEmptyKey,
                                              (unsigned long long)key);
    if (prev == kEmptyKey) break;
    h = (h + 1) & mask;
  }
  hval[h] = make_int2(i, e - i);
}

// points (stride floats) -> float4 (x, y, z, id = id0 + i)
__global__ void k_pack_points(const float* src, int n, int stride, int id0, float4* dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* p = src + (size_t)i * stride;
  dst[i] = make_float4(p[0], p[1], p[2], __int_as_float(id0 + i));
}

// ------------------------------------------------------------------ k-NN
template <int K>
struct KBest {
  float d[K];
  int id[K];
  int ix[K];
};

__device__ __forceinline__ bool lex_less(float d1, int i1, float d2, int i2) {
  return d1 < d2 || (d1 == d2 && i1 < i2);
}

template <int K>
__device__ __forceinline__ void kb_clear(KBest<K>& b) {
#pragma unroll
  for (int j = 0; j < K; j++) { b.d[j] = kInf; b.id[j] = 0x7fffffff; b.ix[j] = -1; }
}

template <int K>
__device__ __forceinline__ void kb_insert(KBest<K>& b, float d, int id, int ix) {
  if (!lex_less(d, id, b.d[K - 1], b.id[K - 1])) return;
  bool placed = false;
#pragma unroll
  for (int j = K - 1; j >= 0; j--) {
    if (!placed) {
      if (j > 0 && lex_less(d, id, b.d[j - 1], b.id[j - 1])) {
        b.d[j] = b.d[j - 1]; b.id[j] = b.id[j - 1]; b.ix[j] = b.ix[j - 1];
      } else {
        b.d[j] = d; b.id[j] = id; b.ix[j] = ix;
        placed = true;
      }
    }
  }
}

// Merge the k-best lists of the G lanes of each group (a wave, or a 16-lane row): afterwards every lane of the group
// returns the merged list in `out`; the group leader keeps it in b, the others are cleared.
template <int K, int G>
__device__ __forceinline__ void group_merge(KBest<K>& b, KBest<K>& out) {
#pragma unroll
  for (int r = 0; r < K; r++) {
    float md = b.d[0];
    int mi = b.id[0];
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
      const float od = __shfl_xor(md, o, G);
      const int oi = __shfl_xor(mi, o, G);
      if (lex_less(od, oi, md, mi)) { md = od; mi = oi; }
    }
    const bool own = b.d[0] == md && b.id[0] == mi && md != kInf;
    int ox = own ? b.ix[0] : 0;
#pragma unroll
    for (int o = 1; o < G; o <<= 1) ox += __shfl_xor(ox, o, G);
    out.d[r] = md; out.id[r] = mi; out.ix[r] = md == kInf ? -1 : ox;
    if (own) {
#pragma unroll
      for (int j = 0; j < K - 1; j++) { b.d[j] = b.d[j + 1]; b.id[j] = b.id[j + 1]; b.ix[j] = b.ix[j + 1]; }
      b.d[K - 1] = kInf; b.id[K - 1] = 0x7fffffff; b.ix[K - 1] = -1;
    }
  }
  if ((threadIdx.x & (G - 1)) == 0) b = out;
  else kb_clear(b);
}

// pointAssociateToMap (laserMapping.cpp:138-147) / mapOptimization.cpp:385: q * p + t in
// double, stored as float.
__device__ __forceinline__ float4 to_world(const double* x, float px, float py, float pz) {
  const DQ q{x[0], x[1], x[2], x[3]};
  const D3 w = qrot(q, D3{(double)px, (double)py, (double)pz});
  return make_float4((float)(w.x + x[4]), (float)(w.y + x[5]), (float)(w.z + x[6]), 0.f);
}

// distance from q to the faces of the block of cells [c - s, c + s] (per axis), minus the
// rounding of the face positions; 0 if negative
__device__ __forceinline__ double block_gap(double q, int c, int s, double cell) {
  const double lo = (double)(c - s) * cell, hi = (double)(c + s + 1) * cell;
  const double tol = 1e-6 * (fabs(q) + fabs(lo) + fabs(hi)) + 1e-9;
  return fmax(0.0, fmin(q - lo, hi - q) - tol);
}

// Cell (dx, dy, dz) number j of pass s: s == 1 the whole 3x3x3 block, s > 1 the 24 s^2 + 2
// cells at Chebyshev distance s (two z faces, then the square rings of the z layers between).
__device__ __forceinline__ void shell_cell(int s, int j, int& dx, int& dy, int& dz) {
  if (s == 1) {
    dz = j / 9 - 1;
    dy = (j / 3) % 3 - 1;
    dx = j % 3 - 1;
    return;
  }
  const int side = 2 * s + 1, face = side * side;
  if (j < 2 * face) {
    dz = j < face ? -s : s;
    const int r = j % face;
    dx = r % side - s;
    dy = r / side - s;
    return;
  }
  const int jj = j - 2 * face, ring = 8 * s;
  dz = jj / ring - (s - 1);
  const int r = jj % ring, e = r / (2 * s), o = r % (2 * s);
  if (e == 0) { dx = -s + o; dy = -s; }
  else if (e == 1) { dx = s; dy = -s + o; }
  else if (e == 2) { dx = s - o; dy = s; }
  else { dx = -s; dy = s - o; }
}

// lower bound of the squared distance from q to any point stored in cell (ix, iy, iz): the box
// [i c, (i+1) c] widened by the rounding of floor(p / c), squared in double, shrunk by 1e-6
__device__ __forceinline__ double cell_lb2(const float4& q, int ix, int iy, int iz, float cell) {
  const double c = cell;
  const double qs[3] = {q.x, q.y, q.z};
  const int is[3] = {ix, iy, iz};
  double s2 = 0;
  for (int a = 0; a < 3; a++) {
    const double lo = (double)is[a] * c, hi = lo + c;
    const double tol = 1e-6 * (fabs(qs[a]) + fabs(lo) + c) + 1e-9;
    const double g = fmax(0.0, fmax((lo - tol) - qs[a], qs[a] - (hi + tol)));
    s2 += g * g;
  }
  return s2 * (1.0 - 1e-6);
}

// mg.d[k - 1] without a dynamic register index
template <int K>
__device__ __forceinline__ float kth_of(const KBest<K>& mg, int k) {
  float v = kInf;
#pragma unroll
  for (int r = 0; r < K; r++) v = r == k - 1 ? mg.d[r] : v;
  return v;
}

// Block b of a grid of nblk is dealt to XCD b % 8; give each XCD one contiguous range of
// (spatially ordered) queries so the cells it walks stay in its own L2.  Bijective for any nblk.
__device__ __forceinline__ int xcd_block(int b, int nblk) {
  const int q = nblk >> 3, r = nblk & 7, x = b & 7;
  return x * q + min(x, r) + (b >> 3);
}

// One pass over `total` cells (the 3x3x3 block for s == 1, else the shell at radius s): lanes
// probe one cell each (skipping cells whose box cannot beat `bound`, and those within `skip` — a
// pass over them already ran; skip < 0: none; s == 1 with bound = inf: every cell, no box test),
// then the points of the probed cells are dealt evenly over the G lanes (exclusive prefix of the
// counts + a log2(G)-step binary search per point), four loads in flight per lane.  G lanes per
// query: a wave (64) or a 16-lane row (four queries per wave; every group-wide step is a row op).
template <int K, int G>
__device__ __forceinline__ void knn_pass(const MapView& m, const float4& q, int cx, int cy, int cz, int s, float skip,
                                         float bound, float max_d2, KBest<K>& b) {
  const int lane = threadIdx.x & (G - 1);
  const int total = s == 1 ? 27 : 24 * s * s + 2;
  const bool all = s == 1 && bound == kInf && skip < 0;
  for (int j0 = 0; j0 < total; j0 += G) {
    const int j = j0 + lane;
    int cnt = 0, beg = 0;
    if (j < total) {
      int dx, dy, dz;
      shell_cell(s, j, dx, dy, dz);
      bool probe = all;
      if (!all) {
        const double lb = cell_lb2(q, cx + dx, cy + dy, cz + dz, m.cell);
        probe = lb <= (double)bound && !(skip >= 0 && lb <= (double)skip);
      }
      if (probe) {
        const int2 r = cell_lookup(m, pack_cell(cx + dx, cy + dy, cz + dz));
        beg = r.x;
        cnt = r.y;
      }
    }
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
      const int v = __shfl_up(incl, o, G);
      if (lane >= o) incl += v;
    }
    const int T = __shfl(incl, G - 1, G);
    const int excl = incl - cnt;
    for (int t0 = 0; t0 < T; t0 += 4 * G) {
      int pi[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int t = t0 + u * G + lane;
        int lo = 0;
#pragma unroll
        for (int st = G / 2; st > 0; st >>= 1) {
          const int e = __shfl(excl, lo + st, G);
          if (e <= t) lo += st;
        }
        const int bb = __shfl(beg, lo, G), ee = __shfl(excl, lo, G);
        pi[u] = t < T ? bb + (t - ee) : -1;
      }
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) v[u] = pi[u] >= 0 ? m.pts[pi[u]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (pi[u] < 0) continue;
        const float d = calc_dist(q.x, q.y, q.z, v[u].x, v[u].y, v[u].z);
        if (d <= max_d2) kb_insert(b, d, __float_as_int(v[u].w), pi[u]);
      }
    }
  }
}

// queries: n points of `stride` floats (optionally counted on the device: *qcount); pose
// (device, nullable): queries are sensor-frame points mapped by pointAssociateToMap first.
template <int K, int G>
__global__ __launch_bounds__(256) void k_knn(MapView m, const float* queries, int stride, const int* qcount, int nq,
                                             const double* pose, int k, float max_d2, float4* out_pts, float* out_d2,
                                             int* out_found) {
  const int qi = xcd_block(blockIdx.x, gridDim.x) * (256 / G) + (int)(threadIdx.x / G);
  const int lane = threadIdx.x & (G - 1);
  const int n = qcount ? min(*qcount, nq) : nq;
  if (qi >= n) return;  // whole groups leave
  const float* qp = queries + (size_t)qi * stride;
  float4 q = make_float4(qp[0], qp[1], qp[2], 0.f);
  if (pose) q = to_world(pose, q.x, q.y, q.z);
  const int cx = cell_of(q.x, m.inv_cell), cy = cell_of(q.y, m.inv_cell), cz = cell_of(q.z, m.inv_cell);
  KBest<K> b, mg;
  kb_clear(b);
  kb_clear(mg);
  const double maxd = sqrt((double)max_d2);
  for (int s = 1;; s++) {
    // a cell is probed only if its (conservative) box distance can beat the current k-th best
    if (s == 1 && m.near2 >= 0) {
      // the block's near cells first; then its other cells that can still beat the k-th best
      // (cells within near2 are in exactly one of the two passes: the same test decides both)
      const float b1 = fminf(max_d2, m.near2);
      knn_pass<K, G>(m, q, cx, cy, cz, 1, -1.f, b1, max_d2, b);
      group_merge<K, G>(b, mg);
      const float b2 = fminf(max_d2, kth_of(mg, k));
      if (max_d2 > m.near2 && b2 > m.near2) {
        knn_pass<K, G>(m, q, cx, cy, cz, 1, m.near2, b2, max_d2, b);
        group_merge<K, G>(b, mg);
      }
    } else {
      const float bound = fminf(max_d2, s == 1 ? kInf : kth_of(mg, k));
      knn_pass<K, G>(m, q, cx, cy, cz, s, -1.f, bound, max_d2, b);
      group_merge<K, G>(b, mg);
    }
    const float kth = kth_of(mg, k);
    const double gap = fmin(block_gap(q.x, cx, s, m.cell), fmin(block_gap(q.y, cy, s, m.cell), block_gap(q.z, cz, s, m.cell)));
    if (gap >= maxd * (1.0 + 1e-6)) break;                                  // every point within max_dist seen
    if (kth != kInf && (double)kth < gap * gap * (1.0 - 1e-6)) break;  // none closer outside
    if (s >= m.scan_shell) {                                                // far from the map: scan it all
      kb_clear(b);
      for (int p = lane; p < m.n; p += G) {
        const float4 v = m.pts[p];
        const float d = calc_dist(q.x, q.y, q.z, v.x, v.y, v.z);
        if (d <= max_d2) kb_insert(b, d, __float_as_int(v.w), p);
      }
      group_merge<K, G>(b, mg);
      break;
    }
  }
  int found = 0;
#pragma unroll
  for (int r = 0; r < K; r++) found += (r < k && mg.d[r] != kInf);
#pragma unroll
  for (int r = 0; r < K; r++) {
    if (r >= k || lane != r) continue;
    const bool ok = mg.d[r] != kInf;
    if (out_pts) out_pts[(size_t)qi * k + r] = ok ? m.pts[mg.ix[r]] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (out_d2) out_d2[(size_t)qi * k + r] = mg.d[r];
  }
  if (out_found && lane == 0) out_found[qi] = found;
}

// ------------------------------------------------------------------ fits (fp64, one thread per query)
// Eigen::ColPivHouseholderQR<Matrix<double,5,3>>::compute + solve(-1): column-pivoted
// Householder QR with norm downdating, rank from the threshold, R^-1 Q^T b, un-permuted.
__device__ __forceinline__ void colpiv_qr_solve_5x3(double (&A)[5][3], double* x) {
  // Every loop has a constant trip count and every data-dependent index (the pivot column, the
  // rank) is a predicate over unrolled indices, so A and the work arrays stay in registers (a
  // dynamic index puts them in LDS or scratch); the arithmetic and its order are Eigen's.
  constexpr int R = 5, C = 3;
  double upd[3], dir[3], tau[3];
  int trans[3];
  double maxn = 0;
#pragma unroll
  for (int j = 0; j < C; j++) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < R; i++) s += A[i][j] * A[i][j];
    upd[j] = dir[j] = sqrt(s);
    maxn = fmax(maxn, upd[j]);
  }
  const double eps = 2.220446049250313e-16;
  const double thr = (maxn * eps) * (maxn * eps) / R;
  const double downdate = sqrt(eps);
  int nonzero = C;
#pragma unroll
  for (int k = 0; k < C; k++) {
    int big = k;
    double ub = upd[k];
#pragma unroll
    for (int j = k + 1; j < C; j++)
      if (upd[j] > ub) { big = j; ub = upd[j]; }
    const double bsq = ub * ub;
    if (nonzero == C && bsq < thr * (R - k)) nonzero = k;
    trans[k] = big;
#pragma unroll
    for (int j = k + 1; j < C; j++) {
      if (j == big) {
#pragma unroll
        for (int i = 0; i < R; i++) { const double t = A[i][k]; A[i][k] = A[i][j]; A[i][j] = t; }
        double t = upd[k]; upd[k] = upd[j]; upd[j] = t;
        t = dir[k]; dir[k] = dir[j]; dir[j] = t;
      }
    }
    const double c0 = A[k][k];
    double tail = 0;
#pragma unroll
    for (int i = k + 1; i < R; i++) tail += A[i][k] * A[i][k];
    double beta;
    if (tail <= 2.2250738585072014e-308) {
      tau[k] = 0;
      beta = c0;
#pragma unroll
      for (int i = k + 1; i < R; i++) A[i][k] = 0;
    } else {
      beta = sqrt(c0 * c0 + tail);
      if (c0 >= 0) beta = -beta;
#pragma unroll
      for (int i = k + 1; i < R; i++) A[i][k] = A[i][k] / (c0 - beta);
      tau[k] = (beta - c0) / beta;
    }
    A[k][k] = beta;
#pragma unroll
    for (int j = k + 1; j < C; j++) {
      if (tau[k] == 0) continue;
      double t = A[k][j];
#pragma unroll
      for (int i = k + 1; i < R; i++) t += A[i][k] * A[i][j];
      A[k][j] -= tau[k] * t;
#pragma unroll
      for (int i = k + 1; i < R; i++) A[i][j] -= tau[k] * A[i][k] * t;
    }
#pragma unroll
    for (int j = k + 1; j < C; j++) {
      if (upd[j] == 0) continue;
      double t = fabs(A[k][j]) / upd[j];
      t = (1 + t) * (1 - t);
      t = t < 0 ? 0 : t;
      const double t2 = t * (upd[j] / dir[j]) * (upd[j] / dir[j]);
      if (t2 <= downdate) {
        double s = 0;
#pragma unroll
        for (int i = k + 1; i < R; i++) s += A[i][j] * A[i][j];
        dir[j] = upd[j] = sqrt(s);
      } else {
        upd[j] *= sqrt(t);
      }
    }
  }
  // perm: the transpositions applied in order (perm[k] <-> perm[trans[k]])
  int perm[3] = {0, 1, 2};
#pragma unroll
  for (int k = 0; k < C; k++) {
#pragma unroll
    for (int j = k + 1; j < C; j++)
      if (j == trans[k]) { const int t = perm[k]; perm[k] = perm[j]; perm[j] = t; }
  }
  double c[5] = {-1, -1, -1, -1, -1};
#pragma unroll
  for (int k = 0; k < C; k++) {
    if (k >= nonzero || tau[k] == 0) continue;
    double t = c[k];
#pragma unroll
    for (int i = k + 1; i < R; i++) t += A[i][k] * c[i];
    c[k] -= tau[k] * t;
#pragma unroll
    for (int i = k + 1; i < R; i++) c[i] -= tau[k] * A[i][k] * t;
  }
#pragma unroll
  for (int i = C - 1; i >= 0; i--) {
    if (i >= nonzero) continue;
    c[i] /= A[i][i];
#pragma unroll
    for (int r = 0; r < i; r++) c[r] -= A[r][i] * c[i];
  }
#pragma unroll
  for (int i = 0; i < C; i++) {
    const double v = i < nonzero ? c[i] : 0.0;
#pragma unroll
    for (int j = 0; j < C; j++)
      if (perm[i] == j) x[j] = v;
  }
}

// laserMapping.cpp:756-788, mapOptimization.cpp:398-420
__device__ __forceinline__ bool plane_fit(const float4* nb, double* n, double* d) {
  double A[5][3];
  for (int j = 0; j < 5; j++) { A[j][0] = nb[j].x; A[j][1] = nb[j].y; A[j][2] = nb[j].z; }
  colpiv_qr_solve_5x3(A, n);
  const double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
  *d = 1 / nn;
  if (nn > 0) { n[0] /= nn; n[1] /= nn; n[2] /= nn; }
  for (int j = 0; j < 5; j++)
    if (fabs(n[0] * nb[j].x + n[1] * nb[j].y + n[2] * nb[j].z + *d) > 0.2) return false;
  return true;
}

// symmetric 3x3 eigen-decomposition, cyclic Jacobi; ascending eigenvalues, V[:, k] vectors.  Loops
// unrolled and the final ordering a compare-swap network on (eigenvalue, column) pairs, so nothing
// is indexed by data (the arrays stay in registers).
__device__ __forceinline__ void sym_eig3(double (&a)[3][3], double* w, double (&V)[3][3]) {
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) V[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 32; sweep++) {
    const double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    if (off == 0.0) break;
#pragma unroll
    for (int p = 0; p < 2; p++)
#pragma unroll
      for (int q = p + 1; q < 3; q++) {
        if (a[p][q] == 0.0) continue;
        const double theta = (a[q][q] - a[p][p]) / (2.0 * a[p][q]);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
  // ascending order: the index sort of the round-4 code (ord[i] <-> ord[j] when a[ord[j]][ord[j]] <
  // a[ord[i]][ord[i]], i < j) applied to the (eigenvalue, column) pairs themselves
  double d[3] = {a[0][0], a[1][1], a[2][2]};
  double col[3][3];
#pragma unroll
  for (int k = 0; k < 3; k++)
#pragma unroll
    for (int i = 0; i < 3; i++) col[k][i] = V[i][k];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = i + 1; j < 3; j++)
      if (d[j] < d[i]) {
        const double t = d[i]; d[i] = d[j]; d[j] = t;
#pragma unroll
        for (int r = 0; r < 3; r++) { const double u = col[i][r]; col[i][r] = col[j][r]; col[j][r] = u; }
      }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    w[k] = d[k];
#pragma unroll
    for (int i = 0; i < 3; i++) V[i][k] = col[k][i];
  }
}

// laserMapping.cpp:681-723
__device__ __forceinline__ bool line_fit(const float4* nb, double* pa, double* pb) {
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

// One thread per query: the 5 neighbours from k_knn -> residual-block record + kind.
__global__ void k_fit(int match, const float* queries, int stride, const int* qcount, int nq, const float4* nb,
                      const float* d2, const int* found, double* rec, int* kind) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = qcount ? min(*qcount, nq) : nq;
  if (i >= n) return;
  double r[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  int kd = -1;
  if (found[i] == 5 && d2[(size_t)i * 5 + 4] < 1.0f) {  // pointSearchSqDis[4] < 1.0
    const float* p = queries + (size_t)i * stride;
    r[0] = p[0]; r[1] = p[1]; r[2] = p[2];
    float4 v[5];
    for (int j = 0; j < 5; j++) v[j] = nb[(size_t)i * 5 + j];
    if (match == 0) {
      if (line_fit(v, r + 3, r + 6)) kd = 0;
    } else {
      double nn[3], d;
      if (plane_fit(v, nn, &d)) {
        r[3] = nn[0]; r[4] = nn[1]; r[5] = nn[2]; r[6] = d;
        kd = 2;
      }
    }
  }
  for (int e = 0; e < 9; e++) rec[(size_t)i * 9 + e] = r[e];
  kind[i] = kd;
}

// ------------------------------------------------------------------ Add_Points with downsampling
// Sequential semantics of ikd_Tree.cpp:594-640 per box B (inputs in order n1..nj, stored points
// S0): after the first input B holds exactly one point, and input n_i replaces the holder m iff
// dist(n_i, mid) <= dist(m, mid) (a stored point wins only with a strictly smaller distance).
// So B ends with the lexicographic minimum over [S0 (first strict minimum, ascending id), n1..nj]
// of (dist, later-wins): the inputs' winner is (min dist, max index); it enters iff its distance
// is <= that of S0's best; every other stored point of B leaves (all of them if the input wins).
struct DsArgs {
  MapView m;
  const float4* in;  // [nin] inputs (x, y, z, id bits)
  int nin;
  float L;
  uint64_t* bkey;   // [bcap]
  unsigned long long* bwin;  // [bcap] (dist bits << 32) | ~index
  uint32_t bmask;
  int* boxes;       // [nin] claimed slots
  int* nbox;
  uint8_t* dead;    // [map n]
  uint8_t* enter;   // [nin]
};

__device__ __forceinline__ void ds_box(float L, const float4& p, float* bmin, float* bmax, float* mid) {
  const float c[3] = {p.x, p.y, p.z};
  for (int k = 0; k < 3; k++) {
    bmin[k] = floorf(c[k] / L) * L;
    bmax[k] = bmin[k] + L;
    mid[k] = (float)(bmin[k] + (bmax[k] - bmin[k]) / 2.0);
  }
}

__global__ void k_ds_claim(DsArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.nin) return;
  const float4 p = a.in[i];
  float bmin[3], bmax[3], mid[3];
  ds_box(a.L, p, bmin, bmax, mid);
  const uint64_t key = pack_cell((int)floorf(p.x / a.L), (int)floorf(p.y / a.L), (int)floorf(p.z / a.L));
  const float d = calc_dist(p.x, p.y, p.z, mid[0], mid[1], mid[2]);
  uint32_t h = mix64(key) & a.bmask;
  while (true) {
    const unsigned long long prev = atomicCAS((unsigned long long*)&a.bkey[h], (unsigned long long)kEmptyKey,
                                              (unsigned long long)key);
    if (prev == kEmptyKey) { a.boxes[atomicAdd(a.nbox, 1)] = (int)h; break; }
    if (prev == key) break;
    h = (h + 1) & a.bmask;
  }
  atomicMin(&a.bwin[h], ((unsigned long long)__float_as_uint(d) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)i));
}

__global__ void k_ds_resolve(DsArgs a) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= *a.nbox) return;
  const unsigned long long wv = a.bwin[a.boxes[t]];
  const int w = (int)(0xffffffffu - (uint32_t)(wv & 0xffffffffu));
  const float dw = __uint_as_float((uint32_t)(wv >> 32));
  const float4 pw = a.in[w];
  float bmin[3], bmax[3], mid[3];
  ds_box(a.L, pw, bmin, bmax, mid);
  const MapView& m = a.m;
  // Search_by_range: cells [cell(bmin), cell(bmax)] hold every point with bmin <= p < bmax
  // (floor(p / cell) is monotone in p)
  const int x0 = cell_of(bmin[0], m.inv_cell), x1 = cell_of(bmax[0], m.inv_cell);
  const int y0 = cell_of(bmin[1], m.inv_cell), y1 = cell_of(bmax[1], m.inv_cell);
  const int z0 = cell_of(bmin[2], m.inv_cell), z1 = cell_of(bmax[2], m.inv_cell);
  int ns = 0, best = -1, best_id = 0x7fffffff;
  float bd = kInf;
  for (int pass = 0; pass < 2; pass++) {
    for (int ix = x0; ix <= x1; ix++)
      for (int iy = y0; iy <= y1; iy++)
        for (int iz = z0; iz <= z1; iz++) {
          if (m.n == 0) continue;
          const int2 r = cell_lookup(m, pack_cell(ix, iy, iz));
          for (int p = r.x; p < r.x + r.y; p++) {
            const float4 v = m.pts[p];
            if (!(bmin[0] <= v.x && bmax[0] > v.x && bmin[1] <= v.y && bmax[1] > v.y && bmin[2] <= v.z && bmax[2] > v.z))
              continue;
            if (pass == 0) {
              ns++;
              const float d = calc_dist(v.x, v.y, v.z, mid[0], mid[1], mid[2]);
              const int id = __float_as_int(v.w);
              if (d < bd || (d == bd && id < best_id)) { bd = d; best = p; best_id = id; }
            } else {
              const bool input_wins = dw <= bd;
              if (input_wins || (ns > 1 && p != best)) a.dead[p] = 1;
            }
          }
        }
    if (ns == 0) break;
  }
  if (ns == 0 || dw <= bd) a.enter[w] = 1;
}

__global__ void k_flags_inv(const uint8_t* dead, int n, uint8_t* live) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) live[i] = dead[i] ? 0 : 1;
}

// ------------------------------------------------------------------ PCL VoxelGrid of a whole cloud
// pcl::VoxelGrid<PointT>::applyFilter (PCL 1.10): bounds, ijk = floor(p / leaf) - min_b, index
// i + j*div0 + k*div0*div1, (index, point) pairs sorted by index (stable: points of a voxel in
// input order), one centroid of all four fields per voxel in index order.  A leaf too small for
// 32-bit indices returns the input (PCL warns and copies).
struct VgArgs {
  const float4* in;
  int n;
  float inv;
  float* bounds;     // [6] min xyz, max xyz (device)
  uint32_t* keys;    // [n]
  int* idx;          // [n]
  int* overflow;     // [1]
};

__device__ __forceinline__ unsigned ord_f(float f) {  // order-preserving float -> uint
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f(unsigned u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }

__global__ __launch_bounds__(1024) void k_vg_bounds(VgArgs a) {
  __shared__ unsigned smn[3][16], smx[3][16];
  unsigned mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
  for (int i = threadIdx.x; i < a.n; i += blockDim.x) {
    const float4 p = a.in[i];
    const unsigned c[3] = {ord_f(p.x), ord_f(p.y), ord_f(p.z)};
    for (int k = 0; k < 3; k++) { mn[k] = min(mn[k], c[k]); mx[k] = max(mx[k], c[k]); }
  }
  for (int o = 32; o > 0; o >>= 1)
    for (int k = 0; k < 3; k++) { mn[k] = min(mn[k], (unsigned)__shfl_xor((int)mn[k], o)); mx[k] = max(mx[k], (unsigned)__shfl_xor((int)mx[k], o)); }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 3; k++) { smn[k][w] = mn[k]; smx[k][w] = mx[k]; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) / 64;
    for (int k = 0; k < 3; k++) {
      unsigned a0 = smn[k][0], a1 = smx[k][0];
      for (int j = 1; j < nw; j++) { a0 = min(a0, smn[k][j]); a1 = max(a1, smx[k][j]); }
      a.bounds[k] = unord_f(a0);
      a.bounds[3 + k] = unord_f(a1);
    }
  }
}

__global__ void k_vg_keys(VgArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const float inv = a.inv;
  const float mn[3] = {a.bounds[0], a.bounds[1], a.bounds[2]}, mx[3] = {a.bounds[3], a.bounds[4], a.bounds[5]};
  const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1, dy = (int64_t)((mx[1] - mn[1]) * inv) + 1,
                dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
  if (dx * dy * dz > (int64_t)0x7fffffff) {
    if (i == 0) *a.overflow = 1;
    return;
  }
  if (i >= a.n) return;
  int min_b[3], div_b[3];
  for (int k = 0; k < 3; k++) {
    min_b[k] = (int)floorf(mn[k] * inv);
    div_b[k] = (int)floorf(mx[k] * inv) - min_b[k] + 1;
  }
  const int mul1 = div_b[0], mul2 = div_b[0] * div_b[1];
  const float4 p = a.in[i];
  const int i0 = (int)(floorf(p.x * inv) - (float)min_b[0]);
  const int i1 = (int)(floorf(p.y * inv) - (float)min_b[1]);
  const int i2 = (int)(floorf(p.z * inv) - (float)min_b[2]);
  a.keys[i] = (uint32_t)(i0 + i1 * mul1 + i2 * mul2);
  a.idx[i] = i;
}

__global__ void k_vg_runs(const uint32_t* skeys, int n, const int* overflow, int* flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flag[i] = (*overflow == 0) && (i == 0 || skeys[i] != skeys[i - 1]) ? 1 : 0;
}

__global__ void k_vg_centroids(const float4* in, const uint32_t* skeys, const int* sidx, const int* pos, const int* flag,
                               int n, const int* overflow, float4* out, int* n_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (*overflow) {  // leaf too small: output = input
    if (i < n) out[i] = in[i];
    if (i == 0) *n_out = n;
    return;
  }
  if (i == 0) *n_out = n > 0 ? pos[n - 1] + flag[n - 1] : 0;
  if (i >= n || !flag[i]) return;
  // the run's points are summed one after another in sorted (input) order; the loads of 16
  // points are issued ahead of their adds so a long run (e.g. the dropout points of a scan)
  // costs one memory latency per 16 points
  const uint32_t key = skeys[i];
  float4 c = in[sidx[i]];
  int e = i + 1;
  constexpr int U = 16;
  int cntn = 1;
  bool more = true;
  while (more) {
    int ix[U];
#pragma unroll
    for (int u = 0; u < U; u++) ix[u] = (e + u < n && skeys[e + u] == key) ? sidx[e + u] : -1;
    float4 p[U];
#pragma unroll
    for (int u = 0; u < U; u++) p[u] = ix[u] >= 0 ? in[ix[u]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (ix[u] >= 0) {
        c.x += p[u].x; c.y += p[u].y; c.z += p[u].z; c.w += p[u].w;
        cntn++;
      }
    }
    more = ix[U - 1] >= 0;
    e += U;
  }
  const float cnt = (float)cntn;
  c.x /= cnt; c.y /= cnt; c.z /= cnt; c.w /= cnt;
  out[pos[i]] = c;
}

// ------------------------------------------------------------------ multi-workgroup pose solve
constexpr int kEvalThreads = 256;
constexpr int kMaxParts = 256;
constexpr int kPart = kAcc + 2;  // acc + edge / plane block counts

struct LmDev {
  EngLM s;  // the step state (lislam_lm_wave.hpp), staged through LDS by the launch that steps
  double x0[7], xe[7];
  int flag, phase, nedge, nplane;
};

// ctl (nullable): k_lm_solve's arrival count, generation and give-up words, zeroed here
__global__ void k_lm_init(LmDev* st, const double* x0, unsigned* ctl) {
  if (threadIdx.x != 0) return;
  if (ctl) { ctl[0] = 0u; ctl[1] = 0u; ctl[2] = 0u; }
  for (int e = 0; e < 7; e++) { st->x0[e] = x0[e]; st->xe[e] = x0[e]; }
  st->flag = 1;
  st->phase = 0;
  st->nedge = st->nplane = 0;
  st->s.it = 0;
  st->s.term = 1;
}

// Agent-scope (sc1) accesses of the solve state and the partials: inside one launch of k_lm_solve
// another workgroup (on another XCD, behind another L2) reads what a workgroup wrote, so these bypass
// the non-coherent caches instead of fencing the whole L2 (the chain engine's hand-offs,
// lislam_odometry.hip).  The stores are drained (s_waitcnt vmcnt(0)) before the count or the
// generation word that publishes them.
typedef __attribute__((address_space(1))) unsigned long long gmu64;
typedef __attribute__((address_space(1))) unsigned gmu32;
__device__ __forceinline__ double ld_ag(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((gmu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_ag(double* p, double v) {
  __hip_atomic_store((gmu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ld_ag(const unsigned* p) {
  return __hip_atomic_load((gmu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag(unsigned* p, unsigned v) {
  __hip_atomic_store((gmu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_ag(const int* p) { return (int)ld_ag((const unsigned*)p); }
__device__ __forceinline__ void st_ag(int* p, int v) { st_ag((unsigned*)p, (unsigned)v); }
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Partial blk (of nblk: the records blk * kEvalThreads + threadIdx.x, strided by nblk * kEvalThreads)
// of the evaluation at xe (acc + block counts), stored agent-scope (ag) or plainly.
__device__ __forceinline__ void lm_eval_partial(const double* rec, const int* kind, int nn, const double* xe, int blk,
                                                int nblk, double* partial, bool ag) {
  __shared__ double red[kEvalThreads / 16][kPart];
  double acc[kPart];
#pragma unroll
  for (int e = 0; e < kPart; e++) acc[e] = 0;
  const DQ q{xe[0], xe[1], xe[2], xe[3]};
  const D3 t{xe[4], xe[5], xe[6]};
  for (int i = blk * kEvalThreads + threadIdx.x; i < nn; i += nblk * kEvalThreads) {
    const int kd = kind[i];
    if (kd < 0) continue;
    block_accum(kd, rec + (size_t)i * 9, q, t, acc);
    acc[kAcc + (kd == 0 ? 0 : 1)] += 1.0;
  }
  const int lane = threadIdx.x & 63, row = threadIdx.x >> 4;
#pragma unroll
  for (int e = 0; e < kPart; e++) {
    const double v = row_sum(acc[e]);
    if ((lane & 15) == 0) red[row][e] = v;
  }
  __syncthreads();
  if (threadIdx.x < kPart) {
    double v = 0;
    for (int w = 0; w < kEvalThreads / 16; w++) v += red[w][threadIdx.x];
    double* o = partial + (size_t)blk * kPart + threadIdx.x;
    if (ag) st_ag(o, v);
    else *o = v;
  }
}

__global__ __launch_bounds__(kEvalThreads) void k_lm_eval(const double* rec, const int* kind, const int* ncount, int n,
                                                          LmDev* st, double* partial) {
  if (!st->flag) return;
  lm_eval_partial(rec, kind, ncount ? min(*ncount, n) : n, st->xe, blockIdx.x, gridDim.x, partial, false);
}

// The G partials summed in a fixed two-level order, then the trust-region step on wave 0
// (lislam_lm_wave.hpp, the chain engine's step: a short fp64 chain, the state through LDS); every
// thread of the workgroup calls it.  Lane group g (of kSumGroups) sums parts g, g + kSumGroups, ... of
// column e with every load issued before the first add (a serial chain of L2 round trips cost more
// than the evaluation), then thread e sums the groups in order.  The state is read and written
// agent-scope.  x_out / summary (k_lm_finish's outputs) are written when the solve ends.
__device__ __forceinline__ void lm_sum_step(const double* partial, int G, LmDev* st, int max_it, double* x_out,
                                            int* summary) {
  constexpr int kSumGroups = kEvalThreads / 32;
  __shared__ double gsum[kSumGroups][kPart];
  __shared__ double acc[kPart];
  {
    const int e = threadIdx.x & 31, g = threadIdx.x >> 5;
    if (e < kPart) {
      constexpr int kLoads = kMaxParts / kSumGroups;
      double v[kLoads];
#pragma unroll
      for (int j = 0; j < kLoads; j++) {
        const int w = g + j * kSumGroups;
        v[j] = w < G ? ld_ag(partial + (size_t)w * kPart + e) : 0.0;
      }
      double s = 0;
#pragma unroll
      for (int j = 0; j < kLoads; j++) s += v[j];
      gsum[g][e] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x < kPart) {
    double v = 0;
#pragma unroll
    for (int g = 0; g < kSumGroups; g++) v += gsum[g][threadIdx.x];
    acc[threadIdx.x] = v;
  }
  __syncthreads();
  if (threadIdx.x >= 64) return;  // wave 0 takes the step (every lane alike)
  const int lane = threadIdx.x;
  __shared__ EngLM sl;
  constexpr int kWords = (int)(sizeof(EngLM) / 4);
  for (int i = lane; i < kWords; i += 64)
    reinterpret_cast<unsigned*>(&sl)[i] = ld_ag(reinterpret_cast<const unsigned*>(&st->s) + i);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  LdsLM& s = *(LdsLM*)&sl;
  const int phase = ld_ag(&st->phase);
  int nedge = ld_ag(&st->nedge), nplane = ld_ag(&st->nplane);
  double a[kAcc];
#pragma unroll
  for (int e = 0; e < kAcc; e++) a[e] = acc[e];
  bool cont;
  if (phase == 0) {
    nedge = (int)acc[kAcc];
    nplane = (int)acc[kAcc + 1];
    double x0[7];
#pragma unroll
    for (int e = 0; e < 7; e++) x0[e] = ld_ag(&st->x0[e]);
    if (nedge + nplane == 0) {  // no residual blocks: Ceres leaves the parameters untouched
#pragma unroll
      for (int e = 0; e < 7; e++) s.x[e] = x0[e];
      s.it = 0;
      s.term = 1;
      cont = false;
    } else {
      cont = eng_step(s, x0, a, true, max_it);
    }
  } else {
    cont = eng_step(s, nullptr, a, false, max_it);
  }
  if (cont) eng_step_post(s);  // the candidate's parameter tolerance and 1 / model cost change
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (int i = lane; i < kWords; i += 64)
    st_ag(reinterpret_cast<unsigned*>(&st->s) + i, reinterpret_cast<const unsigned*>(&sl)[i]);
  if (lane != 0) return;
  st_ag(&st->nedge, nedge);
  st_ag(&st->nplane, nplane);
  st_ag(&st->phase, phase + 1);
  st_ag(&st->flag, (int)cont);
  if (cont)
    for (int e = 0; e < 7; e++) st_ag(&st->xe[e], sl.xc[e]);
  if (!cont || phase + 1 > max_it) {  // the solve's end (or its last evaluation)
    if (x_out)
      for (int e = 0; e < 7; e++) x_out[e] = sl.x[e];
    if (summary) { summary[0] = sl.it; summary[1] = sl.term; summary[2] = nedge; summary[3] = nplane; }
  }
}

// One evaluation of ceres::Solve with its trust-region step per launch (the default: solve_device
// launches it max_it + 1 times; a launch after the solve has ended returns at once):
// every workgroup sums its strided share of the records and counts itself in; the last one sums the
// partials and takes the step.
__global__ __launch_bounds__(kEvalThreads) void k_lm_evalstep(const double* rec, const int* kind, const int* ncount, int n,
                                                              LmDev* st, double* partial, unsigned* arrive, int max_it,
                                                              double* x_out, int* summary) {
  if (!st->flag) return;
  lm_eval_partial(rec, kind, ncount ? min(*ncount, n) : n, st->xe, blockIdx.x, gridDim.x, partial, true);
  __shared__ int last;
  drain_vm();  // this workgroup's partial before its arrival
  __syncthreads();
  if (threadIdx.x == 0) last = __hip_atomic_fetch_add((gmu32*)arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) *arrive = 0u;  // the next evaluation's count (its launch follows this one on the stream)
  lm_sum_step(partial, gridDim.x, st, max_it, x_out, summary);
}

// ceres::Solve in one launch (LISLAM_MAP_SOLVE=persistent): the workgroups run every evaluation (at most max_it + 1),
// one grid-wide hand-off apart.  Each workgroup stores its partial, drains and counts itself in
// (ctl[0], monotonic over the launch); the last arrival of evaluation e sums and steps
// (lm_sum_step), drains and publishes generation e + 1 (ctl[1]); the others wait for it on one lane
// with s_sleep, then read the new state.  Every wait is bounded (wait_ticks of the 100 MHz clock):
// a workgroup that gives up sets ctl[2] and leaves, every waiting workgroup sees it and leaves, and
// k_lm_rescue (next on the stream) finishes the solve from the last completed step — the same
// partials and the same sum order, so the same bits.  (The workgroups need not be resident
// together: a late one only delays the hand-off.)
__global__ __launch_bounds__(kEvalThreads) void k_lm_solve(const double* rec, const int* kind, const int* ncount, int n,
                                                           LmDev* st, double* partial, unsigned* ctl, int max_it,
                                                           double* x_out, int* summary, unsigned long long wait_ticks) {
  const int nn = ncount ? min(*ncount, n) : n;
  const unsigned G = gridDim.x;
  __shared__ int s_go, s_last;
  __shared__ double s_xe[7];
  for (int e = 0; e <= max_it; e++) {
    if (threadIdx.x == 0) s_go = ld_ag(&st->flag) != 0 && ld_ag(ctl + 2) == 0u;
    if (threadIdx.x < 7) s_xe[threadIdx.x] = ld_ag(&st->xe[threadIdx.x]);
    __syncthreads();
    if (!s_go) return;
    lm_eval_partial(rec, kind, nn, s_xe, blockIdx.x, G, partial, true);
    drain_vm();  // this workgroup's partial before its arrival
    __syncthreads();
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add((gmu32*)ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(e + 1) * G - 1u;
    __syncthreads();
    if (s_last) {
      lm_sum_step(partial, G, st, max_it, x_out, summary);
      drain_vm();  // the new state before its generation
      __syncthreads();
      if (threadIdx.x == 0) st_ag(ctl + 1, (unsigned)(e + 1));
    } else {
      if (threadIdx.x == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        while (ld_ag(ctl + 1) < (unsigned)(e + 1)) {
          if (ld_ag(ctl + 2) != 0u) { ok = 0; break; }
          if (__builtin_amdgcn_s_memrealtime() - t0 > wait_ticks) {
            st_ag(ctl + 2, 1u);
            ok = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        s_go = ok;
      }
      __syncthreads();
      if (!s_go) return;
    }
  }
}

// After k_lm_solve: nothing unless it gave up (ctl[2]); then one workgroup finishes the solve from
// the last completed step, computing every partial as its workgroup would have (same records, same
// order) and the same sum and step.
__global__ __launch_bounds__(kEvalThreads) void k_lm_rescue(const double* rec, const int* kind, const int* ncount, int n,
                                                            LmDev* st, double* partial, const unsigned* ctl, int parts,
                                                            int max_it, double* x_out, int* summary) {
  if (ctl[2] == 0u) return;
  const int nn = ncount ? min(*ncount, n) : n;
  __shared__ int s_go;
  __shared__ double s_xe[7];
  for (;;) {
    if (threadIdx.x == 0) s_go = ld_ag(&st->flag) != 0 && ld_ag(&st->phase) <= max_it;
    if (threadIdx.x < 7) s_xe[threadIdx.x] = ld_ag(&st->xe[threadIdx.x]);
    __syncthreads();
    if (!s_go) return;
    for (int w = 0; w < parts; w++) {
      lm_eval_partial(rec, kind, nn, s_xe, w, parts, partial, true);
      __syncthreads();
    }
    drain_vm();
    __syncthreads();
    lm_sum_step(partial, parts, st, max_it, x_out, summary);
    drain_vm();
    __syncthreads();
  }
}

// x_out = solved pose; summary = iterations, termination, edge blocks, plane blocks
__global__ void k_lm_finish(const LmDev* st, double* x_out, int* summary) {
  if (threadIdx.x != 0) return;
  for (int e = 0; e < 7; e++) x_out[e] = st->s.x[e];
  if (summary) { summary[0] = st->s.it; summary[1] = st->s.term; summary[2] = st->nedge; summary[3] = st->nplane; }
}

// mapOptimization.cpp:730-746: transformAssociateToMap (mode 0) / transformUpdate on
// CONVERGENCE + keyframe pose selection (mode 1).  st7 = q_wmap_wodom, t_wmap_wodom; odom =
// q_wodom_curr, t_wodom_curr; x = q_w_curr, t_w_curr.
__global__ void k_mapopt_pose(int mode, double* st7, const double* odom, double* x, const LmDev* lm, double* key_pose) {
  if (threadIdx.x != 0) return;
  const DQ qm{st7[0], st7[1], st7[2], st7[3]};
  const DQ qo{odom[0], odom[1], odom[2], odom[3]};
  const D3 to{odom[4], odom[5], odom[6]};
  if (mode == 0) {
    const DQ qw = qmul(qm, qo);
    const D3 tw = qrot(qm, to) + D3{st7[4], st7[5], st7[6]};
    x[0] = qw.x; x[1] = qw.y; x[2] = qw.z; x[3] = qw.w; x[4] = tw.x; x[5] = tw.y; x[6] = tw.z;
    return;
  }
  const bool conv = lm->s.term == 1;
  const double* xs = lm->s.x;
  if (conv) {
    const DQ nq = qmul(DQ{xs[0], xs[1], xs[2], xs[3]}, DQ{-odom[0], -odom[1], -odom[2], odom[3]});
    st7[0] = nq.x; st7[1] = nq.y; st7[2] = nq.z; st7[3] = nq.w;
    const D3 r = qrot(nq, to);
    st7[4] = xs[4] - r.x; st7[5] = xs[5] - r.y; st7[6] = xs[6] - r.z;
  }
  for (int e = 0; e < 7; e++) key_pose[e] = conv ? xs[e] : x[e];
  for (int e = 0; e < 7; e++) x[e] = xs[e];
}

// world points of a cloud at a device pose: pcl::transformPointCloud(cloud, T(q, t))
__global__ void k_transform(const float* src, int stride, const int* ncount, int n, const double* pose, float* dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int nn = ncount ? min(*ncount, n) : n;
  if (i >= nn) return;
  const float* p = src + (size_t)i * stride;
  const float4 w = to_world(pose, p[0], p[1], p[2]);
  dst[(size_t)i * 4 + 0] = w.x; dst[(size_t)i * 4 + 1] = w.y; dst[(size_t)i * 4 + 2] = w.z; dst[(size_t)i * 4 + 3] = 0.f;
}

}  // namespace mapk
}  // namespace lislam

// ================================================================== host side
using namespace lislam;
using namespace lislam::mapk;

namespace {

int mfail(lislam_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define MCHK(ctx, x)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) return mfail(ctx, LISLAM_ERR_DEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

#define MRC(x)                    \
  do {                            \
    int rc_ = (x);                \
    if (rc_ != LISLAM_OK) return rc_; \
  } while (0)

inline int blocks(int64_t n, int t = 256) { return (int)std::max<int64_t>(1, (n + t - 1) / t); }

// Growable device buffer.
struct DBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DBuf() { if (p) (void)hipFree(p); }
  hipError_t reserve(size_t b) {
    if (b <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    const size_t nb = std::max<size_t>(b, 256) + b / 4;
    hipError_t e = hipMalloc(&p, nb);
    if (e == hipSuccess) bytes = nb;
    return e;
  }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};

uint32_t pow2_at_least(uint64_t v) {
  uint32_t c = 1024;
  while (c < v) c <<= 1;
  return c;
}

}  // namespace

struct LoopState;  // lislam_loop_icp's target map and buffers (end of file)

// Scratch shared by the stateless entry points of a context (voxel grid, solve, association).
struct MapScratch {
  DBuf sort_tmp, keys32a, keys32b, idxa, idxb, flag, pos, vin, vout, bounds, counters;
  DBuf lm, partial, rec, kind, x, nb, d2, found, q, vox, qc, qs;
  LoopState* loop = nullptr;
};

struct lislam_map {
  lislam_ctx* ctx = nullptr;
  float ds = 0.2f, cell = 0.2f;
  int64_t n = 0;
  int next_id = 0;
  DBuf pts, tmp, keys, keys2, idx, idx2, sort_tmp, hkey, hval, counter, dead, live, enter, newp, bkey, bwin, boxes, sel;
  uint32_t hcap = 0;
  MapScratch sc;
  MapView view() const {
    MapView v;
    v.pts = pts.as<float4>();
    v.hkey = hkey.as<uint64_t>();
    v.hval = hval.as<int2>();
    v.hmask = hcap ? hcap - 1 : 0;
    v.cell = cell;
    v.inv_cell = 1.0f / cell;
    v.n = (int)n;
    v.scan_shell = mapk::scan_shell_for(n);
    v.near2 = mapk::knn_near2(cell);
    return v;
  }
};

namespace {

hipStream_t stream_of(lislam_ctx* c) { return c->stream; }

// Stable radix sort of (u64 / u32 key, int) pairs (lislam_prims.hpp); ki / vi are clobbered.
int sort_pairs_u64(lislam_ctx* c, DBuf& tmp, uint64_t* ki, uint64_t* ko, int* vi, int* vo, int n) {
  MCHK(c, tmp.reserve(prims::sort_temp_bytes(n)));
  MCHK(c, prims::sort_pairs<uint64_t>(tmp.p, ki, ko, vi, vo, n, 64, stream_of(c)));
  return LISLAM_OK;
}
int sort_pairs_u32(lislam_ctx* c, DBuf& tmp, uint32_t* ki, uint32_t* ko, int* vi, int* vo, int n) {
  MCHK(c, tmp.reserve(prims::sort_temp_bytes(n)));
  MCHK(c, prims::sort_pairs<uint32_t>(tmp.p, ki, ko, vi, vo, n, 32, stream_of(c)));
  return LISLAM_OK;
}

// Rebuild the cell index of the n points in m->tmp (unsorted) into m->pts.
int rebuild(lislam_map* m, int64_t n) {
  lislam_ctx* c = m->ctx;
  hipStream_t st = stream_of(c);
  m->n = n;
  MCHK(c, m->pts.reserve(std::max<int64_t>(n, 1) * sizeof(float4)));
  if (n == 0) { m->hcap = 0; return LISLAM_OK; }
  MCHK(c, m->keys.reserve(n * 8));
  MCHK(c, m->keys2.reserve(n * 8));
  MCHK(c, m->idx.reserve(n * 4));
  MCHK(c, m->idx2.reserve(n * 4));
  MCHK(c, m->counter.reserve(16));
  const float inv = 1.0f / m->cell;
  TimedScope ts(c, kT_rebuild);
  hipLaunchKernelGGL(k_cell_keys, dim3(blocks(n)), dim3(256), 0, st, m->tmp.as<float4>(), (int)n, inv,
                     m->keys.as<uint64_t>(), m->idx.as<int>());
  MRC(sort_pairs_u64(c, m->sort_tmp, m->keys.as<uint64_t>(), m->keys2.as<uint64_t>(), m->idx.as<int>(), m->idx2.as<int>(),
                     (int)n));
  hipLaunchKernelGGL(k_gather, dim3(blocks(n)), dim3(256), 0, st, m->tmp.as<float4>(), m->idx2.as<int>(), (int)n,
                     m->pts.as<float4>());
  MCHK(c, hipMemsetAsync(m->counter.p, 0, sizeof(int), st));
  hipLaunchKernelGGL(k_count_runs, dim3(blocks(n)), dim3(256), 0, st, m->keys2.as<uint64_t>(), (int)n, m->counter.as<int>());
  int ncell = 0;
  MCHK(c, hipMemcpyAsync(&ncell, m->counter.p, sizeof(int), hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  m->hcap = pow2_at_least((uint64_t)ncell * 2);
  MCHK(c, m->hkey.reserve((size_t)m->hcap * 8));
  MCHK(c, m->hval.reserve((size_t)m->hcap * 8));
  MCHK(c, hipMemsetAsync(m->hkey.p, 0xff, (size_t)m->hcap * 8, st));
  hipLaunchKernelGGL(k_insert_runs, dim3(blocks(n)), dim3(256), 0, st, m->keys2.as<uint64_t>(), (int)n,
                     m->hkey.as<uint64_t>(), m->hval.as<int2>(), m->hcap - 1);
  MCHK(c, hipGetLastError());
  return LISLAM_OK;
}

// points (host or device, stride floats) -> device float4 with ids id0.. in dst[off..]
int upload_points(lislam_map* m, const float* pts, int64_t n, int stride, int id0, DBuf& dst, int64_t off) {
  lislam_ctx* c = m->ctx;
  hipStream_t st = stream_of(c);
  if (n == 0) return LISLAM_OK;
  MCHK(c, m->sc.vin.reserve((size_t)n * stride * 4));
  MCHK(c, hipMemcpyAsync(m->sc.vin.p, pts, (size_t)n * stride * 4, hipMemcpyDefault, st));
  hipLaunchKernelGGL(k_pack_points, dim3(blocks(n)), dim3(256), 0, st, m->sc.vin.as<float>(), (int)n, stride, id0,
                     dst.as<float4>() + off);
  MCHK(c, hipGetLastError());
  return LISLAM_OK;
}

// Add n points already packed (float4 with ids) in m->newp.
int add_packed(lislam_map* m, int64_t nin, bool downsample, int64_t* n_added) {
  lislam_ctx* c = m->ctx;
  hipStream_t st = stream_of(c);
  const int64_t n0 = m->n;
  if (!downsample) {
    MCHK(c, m->tmp.reserve((n0 + nin) * sizeof(float4)));
    if (n0) MCHK(c, hipMemcpyAsync(m->tmp.p, m->pts.p, n0 * sizeof(float4), hipMemcpyDeviceToDevice, st));
    MCHK(c, hipMemcpyAsync(m->tmp.as<float4>() + n0, m->newp.p, nin * sizeof(float4), hipMemcpyDeviceToDevice, st));
    if (n_added) *n_added = nin;
    return rebuild(m, n0 + nin);
  }
  const uint32_t bcap = pow2_at_least((uint64_t)nin * 2);
  MCHK(c, m->bkey.reserve((size_t)bcap * 8));
  MCHK(c, m->bwin.reserve((size_t)bcap * 8));
  MCHK(c, m->boxes.reserve(nin * 4));
  MCHK(c, m->dead.reserve(std::max<int64_t>(n0, 1)));
  MCHK(c, m->enter.reserve(nin));
  MCHK(c, m->counter.reserve(16));
  MCHK(c, hipMemsetAsync(m->bkey.p, 0xff, (size_t)bcap * 8, st));
  MCHK(c, hipMemsetAsync(m->bwin.p, 0xff, (size_t)bcap * 8, st));
  MCHK(c, hipMemsetAsync(m->dead.p, 0, std::max<int64_t>(n0, 1), st));
  MCHK(c, hipMemsetAsync(m->enter.p, 0, nin, st));
  MCHK(c, hipMemsetAsync(m->counter.p, 0, 16, st));
  DsArgs a;
  a.m = m->view();
  a.in = m->newp.as<float4>();
  a.nin = (int)nin;
  a.L = m->ds;
  a.bkey = m->bkey.as<uint64_t>();
  a.bwin = m->bwin.as<unsigned long long>();
  a.bmask = bcap - 1;
  a.boxes = m->boxes.as<int>();
  a.nbox = m->counter.as<int>();
  a.dead = m->dead.as<uint8_t>();
  a.enter = m->enter.as<uint8_t>();
  {
    TimedScope ts(c, kT_downsample);
    hipLaunchKernelGGL(k_ds_claim, dim3(blocks(nin)), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_ds_resolve, dim3(blocks(nin)), dim3(256), 0, st, a);
  }
  // survivors (stable) + entering inputs (input order) -> tmp
  MCHK(c, m->tmp.reserve((n0 + nin) * sizeof(float4)));
  MCHK(c, m->live.reserve(std::max<int64_t>(n0, 1)));
  int* nsel = m->counter.as<int>() + 1;
  int* nsel2 = m->counter.as<int>() + 2;
  if (n0) hipLaunchKernelGGL(k_flags_inv, dim3(blocks(n0)), dim3(256), 0, st, m->dead.as<uint8_t>(), (int)n0, m->live.as<uint8_t>());
  MCHK(c, m->sort_tmp.reserve(std::max(prims::select_temp_bytes((int)n0), prims::select_temp_bytes((int)nin))));
  MCHK(c, prims::select_flagged(m->sort_tmp.p, m->pts.as<float4>(), m->live.as<uint8_t>(), m->tmp.as<float4>(), nsel,
                                (int)n0, st));
  int h[2] = {0, 0};
  MCHK(c, hipMemcpyAsync(&h[0], nsel, sizeof(int), hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  MCHK(c, prims::select_flagged(m->sort_tmp.p, m->newp.as<float4>(), m->enter.as<uint8_t>(), m->tmp.as<float4>() + h[0],
                                nsel2, (int)nin, st));
  MCHK(c, hipMemcpyAsync(&h[1], nsel2, sizeof(int), hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  if (n_added) *n_added = h[1];
  return rebuild(m, (int64_t)h[0] + h[1]);
}

// k-NN of n queries (device buffer, stride floats, optional device count / pose).  Lanes per query:
// LISLAM_KNN_LANES = 64 (a wave, the default) or 16 (a 16-lane row: four queries per wave), read at
// every launch.  Four queries per wave measured slower on config 5 (k_knn 0.213 vs 0.195 ms per
// step, profiles/r05_map_ab.txt): the search is issue-bound, not latency-bound per wave.
int knn_lanes() {
  const char* e = getenv("LISLAM_KNN_LANES");
  return e && atoi(e) == 16 ? 16 : 64;
}
int knn_device(lislam_map* m, const float* q, int stride, const int* qcount, int n, const double* pose, int k, float max_d2,
               float4* out_pts, float* out_d2, int* out_found) {
  lislam_ctx* c = m->ctx;
  if (n <= 0) return LISLAM_OK;
  const int G = knn_lanes();
  const int nb = blocks((int64_t)n * G);  // G lanes per query, 256-thread workgroups
  MapView v = m->view();
  TimedScope ts(c, kT_knn);
  if (G == 16) {
    if (k <= 5)
      hipLaunchKernelGGL((k_knn<5, 16>), dim3(nb), dim3(256), 0, stream_of(c), v, q, stride, qcount, n, pose, k, max_d2,
                         out_pts, out_d2, out_found);
    else
      hipLaunchKernelGGL((k_knn<8, 16>), dim3(nb), dim3(256), 0, stream_of(c), v, q, stride, qcount, n, pose, k, max_d2,
                         out_pts, out_d2, out_found);
  } else {
    if (k <= 5)
      hipLaunchKernelGGL((k_knn<5, 64>), dim3(nb), dim3(256), 0, stream_of(c), v, q, stride, qcount, n, pose, k, max_d2,
                         out_pts, out_d2, out_found);
    else
      hipLaunchKernelGGL((k_knn<8, 64>), dim3(nb), dim3(256), 0, stream_of(c), v, q, stride, qcount, n, pose, k, max_d2,
                         out_pts, out_d2, out_found);
  }
  MCHK(c, hipGetLastError());
  return LISLAM_OK;
}

// association of n device queries at a device pose into device rec / kind
int associate_device(lislam_map* m, int match, const float* q, int stride, const int* qcount, int n, const double* pose,
                     double* rec, int* kind) {
  lislam_ctx* c = m->ctx;
  if (n <= 0) return LISLAM_OK;
  MCHK(c, m->sc.nb.reserve((size_t)n * 5 * sizeof(float4)));
  MCHK(c, m->sc.d2.reserve((size_t)n * 5 * 4));
  MCHK(c, m->sc.found.reserve((size_t)n * 4));
  if (m->n == 0) {
    MCHK(c, hipMemsetAsync(m->sc.found.p, 0, (size_t)n * 4, stream_of(c)));
  } else {
    MRC(knn_device(m, q, stride, qcount, n, pose, 5, 1.0f, m->sc.nb.as<float4>(), m->sc.d2.as<float>(),
                   m->sc.found.as<int>()));
  }
  {
    TimedScope ts(c, kT_fit);
    hipLaunchKernelGGL(k_fit, dim3(blocks(n)), dim3(256), 0, stream_of(c), match, q, stride, qcount, n,
                       m->sc.nb.as<float4>(), m->sc.d2.as<float>(), m->sc.found.as<int>(), rec, kind);
  }
  MCHK(c, hipGetLastError());
  return LISLAM_OK;
}

// The solve's schedule: one k_lm_evalstep launch per evaluation (default), or LISLAM_MAP_SOLVE=persistent:
// k_lm_solve, every evaluation in one launch.  The two measure the same on config 5 (a grid-wide
// hand-off costs what a kernel boundary does: 2.59k / 2.63k vs 2.64k / 2.70k registrations/s,
// profiles/r05_map_ab.txt), so the default needs no co-residency at all.
// (Both knobs are read at every solve: the parity tests run each setting in one process.)
bool map_solve_launches() {
  const char* e = getenv("LISLAM_MAP_SOLVE");
  return !(e && strcmp(e, "persistent") == 0);
}
// Bound of k_lm_solve's hand-off waits (100 MHz ticks): LISLAM_MAP_SOLVE_WAIT_US, default 2 s.
unsigned long long map_solve_wait_ticks() {
  const char* e = getenv("LISLAM_MAP_SOLVE_WAIT_US");
  const double us = e && *e ? atof(e) : 2e6;
  return (unsigned long long)(us * 100.0);
}

// ceres::Solve over n device records; result stays in the LmDev (device).
// (x_out / summary: k_lm_finish's outputs, written by the evaluation that ends the solve, when given)
int solve_device(lislam_ctx* c, MapScratch& sc, const double* rec, const int* kind, const int* ncount, int n,
                 const double* x0_dev, int max_it, double* x_out, int* summary) {
  hipStream_t st = stream_of(c);
  MCHK(c, sc.lm.reserve(sizeof(LmDev)));
  MCHK(c, sc.partial.reserve((size_t)kMaxParts * kPart * 8 + 64));
  LmDev* lm = sc.lm.as<LmDev>();
  unsigned* ctl = reinterpret_cast<unsigned*>(sc.partial.as<char>() + (size_t)kMaxParts * kPart * 8);
  const int parts = std::min(kMaxParts, blocks(std::max(n, 1), kEvalThreads));
  hipLaunchKernelGGL(k_lm_init, dim3(1), dim3(64), 0, st, lm, x0_dev, ctl);
  if (map_solve_launches()) {  // one launch per evaluation
    for (int e = 0; e <= max_it; e++) {  // the initial evaluation + at most one per iteration
      TimedScope ts(c, kT_lm_solve);
      hipLaunchKernelGGL(k_lm_evalstep, dim3(parts), dim3(kEvalThreads), 0, st, rec, kind, ncount, n, lm,
                         sc.partial.as<double>(), ctl, max_it, x_out, summary);
    }
  } else {
    TimedScope ts(c, kT_lm_solve);
    hipLaunchKernelGGL(k_lm_solve, dim3(parts), dim3(kEvalThreads), 0, st, rec, kind, ncount, n, lm,
                       sc.partial.as<double>(), ctl, max_it, x_out, summary, map_solve_wait_ticks());
    hipLaunchKernelGGL(k_lm_rescue, dim3(1), dim3(kEvalThreads), 0, st, rec, kind, ncount, n, lm, sc.partial.as<double>(),
                       ctl, parts, max_it, x_out, summary);
  }
  MCHK(c, hipGetLastError());
  return LISLAM_OK;
}

// PCL VoxelGrid of n device float4 points into out (device); n_out device count.
int voxel_grid_device(lislam_ctx* c, MapScratch& sc, const float4* in, int n, float leaf, float4* out, int* n_out) {
  hipStream_t st = stream_of(c);
  if (n == 0) {
    MCHK(c, hipMemsetAsync(n_out, 0, sizeof(int), st));
    return LISLAM_OK;
  }
  MCHK(c, sc.bounds.reserve(64));
  MCHK(c, sc.keys32a.reserve((size_t)n * 4));
  MCHK(c, sc.keys32b.reserve((size_t)n * 4));
  MCHK(c, sc.idxa.reserve((size_t)n * 4));
  MCHK(c, sc.idxb.reserve((size_t)n * 4));
  MCHK(c, sc.flag.reserve((size_t)n * 4));
  MCHK(c, sc.pos.reserve((size_t)n * 4));
  VgArgs a;
  a.in = in;
  a.n = n;
  a.inv = 1.0f / leaf;
  a.bounds = sc.bounds.as<float>();
  a.overflow = sc.bounds.as<int>() + 8;
  a.keys = sc.keys32a.as<uint32_t>();
  a.idx = sc.idxa.as<int>();
  MCHK(c, hipMemsetAsync(a.overflow, 0, sizeof(int), st));
  hipLaunchKernelGGL(k_vg_bounds, dim3(1), dim3(1024), 0, st, a);
  hipLaunchKernelGGL(k_vg_keys, dim3(blocks(n)), dim3(256), 0, st, a);
  MRC(sort_pairs_u32(c, sc.sort_tmp, sc.keys32a.as<uint32_t>(), sc.keys32b.as<uint32_t>(), sc.idxa.as<int>(),
                     sc.idxb.as<int>(), n));
  hipLaunchKernelGGL(k_vg_runs, dim3(blocks(n)), dim3(256), 0, st, sc.keys32b.as<uint32_t>(), n, a.overflow, sc.flag.as<int>());
  MCHK(c, sc.sort_tmp.reserve(prims::exclusive_sum_temp_bytes(n)));
  MCHK(c, prims::exclusive_sum(sc.sort_tmp.p, sc.flag.as<int>(), sc.pos.as<int>(), n, st));
  hipLaunchKernelGGL(k_vg_centroids, dim3(blocks(n)), dim3(256), 0, st, in, sc.keys32b.as<uint32_t>(), sc.idxb.as<int>(),
                     sc.pos.as<int>(), sc.flag.as<int>(), n, a.overflow, out, n_out);
  MCHK(c, hipGetLastError());
  return LISLAM_OK;
}

// host-or-device input of n points (stride floats) -> device float4 buffer (intensity = 0 when stride 3)
int stage_points(lislam_ctx* c, MapScratch& sc, DBuf& dst, const float* pts, int n, int stride) {
  hipStream_t st = stream_of(c);
  MCHK(c, dst.reserve((size_t)std::max(n, 1) * sizeof(float4)));
  if (n == 0) return LISLAM_OK;
  if (stride == 4) {
    MCHK(c, hipMemcpyAsync(dst.p, pts, (size_t)n * 16, hipMemcpyDefault, st));
    return LISLAM_OK;
  }
  MCHK(c, sc.vin.reserve((size_t)n * stride * 4));
  MCHK(c, hipMemcpyAsync(sc.vin.p, pts, (size_t)n * stride * 4, hipMemcpyDefault, st));
  hipLaunchKernelGGL(k_pack_points, dim3(blocks(n)), dim3(256), 0, st, sc.vin.as<float>(), n, stride, 0, dst.as<float4>());
  MCHK(c, hipGetLastError());
  return LISLAM_OK;
}

MapScratch& ctx_scratch(lislam_ctx* c) {
  if (!c->map_scratch) c->map_scratch = new MapScratch();
  return *static_cast<MapScratch*>(c->map_scratch);
}

bool valid_stride(int s) { return s >= 3; }

}  // namespace


extern "C" {

int lislam_map_create(lislam_ctx* c, const lislam_map_config* cfg, lislam_map** out) {
  if (!c || !cfg || !out) return LISLAM_ERR_ARG;
  *out = nullptr;
  if (!(cfg->downsample_size > 0) || cfg->cell_size < 0) return mfail(c, LISLAM_ERR_ARG, "lislam_map_create: bad sizes");
  hipSetDevice(c->device);
  lislam_map* m = new lislam_map();
  m->ctx = c;
  m->ds = cfg->downsample_size;
  m->cell = cfg->cell_size > 0 ? cfg->cell_size : cfg->downsample_size;
  *out = m;
  return LISLAM_OK;
}

int lislam_map_set_timing(lislam_ctx* c, int32_t enable) {
  if (!c) return LISLAM_ERR_ARG;
  c->mtimer.on = enable != 0;
  return LISLAM_OK;
}

int lislam_map_kernel_times(lislam_ctx* c, float* ms, int32_t* launches) {
  if (!c || !ms) return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  MCHK(c, hipStreamSynchronize(c->stream));
  for (int k = 0; k < kT_count; k++) { ms[k] = 0; if (launches) launches[k] = 0; }
  for (auto& r : c->mtimer.rec) {
    float t = 0;
    MCHK(c, hipEventElapsedTime(&t, r.second.first, r.second.second));
    lislam::timeline_print(c->device, "ctx", c, r.first, r.second.first, r.second.second);
    ms[r.first] += t;
    if (launches) launches[r.first]++;
    c->mtimer.pool.push_back(r.second.first);
    c->mtimer.pool.push_back(r.second.second);
  }
  c->mtimer.rec.clear();
  return LISLAM_OK;
}

int lislam_map_destroy(lislam_map* m) {
  if (!m) return LISLAM_OK;
  hipSetDevice(m->ctx->device);
  (void)hipStreamSynchronize(m->ctx->stream);
  delete m;
  return LISLAM_OK;
}

int lislam_map_build(lislam_map* m, const float* pts, int64_t n, int32_t stride) {
  if (!m || n < 0 || (n > 0 && !pts) || !valid_stride(stride) || n > 0x7fffffff) return LISLAM_ERR_ARG;
  hipSetDevice(m->ctx->device);
  MCHK(m->ctx, m->tmp.reserve((size_t)std::max<int64_t>(n, 1) * sizeof(float4)));
  MRC(upload_points(m, pts, n, stride, 0, m->tmp, 0));
  m->next_id = (int)n;
  MRC(rebuild(m, n));
  MCHK(m->ctx, hipStreamSynchronize(m->ctx->stream));
  return LISLAM_OK;
}

int lislam_map_add_points(lislam_map* m, const float* pts, int64_t n, int32_t stride, int32_t downsample_on,
                          int64_t* n_added) {
  if (!m || n < 0 || (n > 0 && !pts) || !valid_stride(stride)) return LISLAM_ERR_ARG;
  if (m->n + n > 0x7fffffff || (int64_t)m->next_id + n > 0x7fffffff) return mfail(m->ctx, LISLAM_ERR_CAPACITY, "map too large");
  hipSetDevice(m->ctx->device);
  if (n_added) *n_added = 0;
  if (n == 0) return LISLAM_OK;
  MCHK(m->ctx, m->newp.reserve((size_t)n * sizeof(float4)));
  MRC(upload_points(m, pts, n, stride, m->next_id, m->newp, 0));
  m->next_id += (int)n;
  MRC(add_packed(m, n, downsample_on != 0, n_added));
  MCHK(m->ctx, hipStreamSynchronize(m->ctx->stream));
  return LISLAM_OK;
}

int lislam_map_size(lislam_map* m, int64_t* n) {
  if (!m || !n) return LISLAM_ERR_ARG;
  *n = m->n;
  return LISLAM_OK;
}

int lislam_map_points(lislam_map* m, float* out, int64_t cap, int64_t* n) {
  if (!m || !n) return LISLAM_ERR_ARG;
  *n = m->n;
  if (m->n == 0) return LISLAM_OK;
  if (!out || cap < m->n) return mfail(m->ctx, LISLAM_ERR_CAPACITY, "lislam_map_points: capacity %lld < %lld",
                                       (long long)cap, (long long)m->n);
  hipSetDevice(m->ctx->device);
  MCHK(m->ctx, hipMemcpyAsync(out, m->pts.p, m->n * sizeof(float4), hipMemcpyDefault, m->ctx->stream));
  MCHK(m->ctx, hipStreamSynchronize(m->ctx->stream));
  return LISLAM_OK;
}

int lislam_map_nearest_search(lislam_map* m, const float* queries, int32_t n, int32_t stride, int32_t k,
                              float max_dist, float* out_pts, float* out_d2, int32_t* out_found) {
  if (!m || n < 0 || (n > 0 && !queries) || !valid_stride(stride) || k < 1 || k > 8) return LISLAM_ERR_ARG;
  if (n == 0) return LISLAM_OK;
  lislam_ctx* c = m->ctx;
  hipSetDevice(c->device);
  MapScratch& sc = m->sc;
  hipStream_t st = stream_of(c);
  MCHK(c, sc.q.reserve((size_t)n * stride * 4));
  MCHK(c, hipMemcpyAsync(sc.q.p, queries, (size_t)n * stride * 4, hipMemcpyDefault, st));
  MCHK(c, sc.nb.reserve((size_t)n * k * sizeof(float4)));
  MCHK(c, sc.d2.reserve((size_t)n * k * 4));
  MCHK(c, sc.found.reserve((size_t)n * 4));
  const float md2 = max_dist > 0 ? max_dist * max_dist : kInf;
  if (m->n == 0) {
    MCHK(c, hipMemsetAsync(sc.nb.p, 0, (size_t)n * k * sizeof(float4), st));
    std::vector<float> inf((size_t)n * k, kInf);
    MCHK(c, hipMemcpyAsync(sc.d2.p, inf.data(), inf.size() * 4, hipMemcpyHostToDevice, st));
    MCHK(c, hipMemsetAsync(sc.found.p, 0, (size_t)n * 4, st));
    MCHK(c, hipStreamSynchronize(st));
  } else {
    MRC(knn_device(m, sc.q.as<float>(), stride, nullptr, n, nullptr, k, md2, sc.nb.as<float4>(), sc.d2.as<float>(),
                   sc.found.as<int>()));
  }
  if (out_pts) MCHK(c, hipMemcpyAsync(out_pts, sc.nb.p, (size_t)n * k * sizeof(float4), hipMemcpyDefault, st));
  if (out_d2) MCHK(c, hipMemcpyAsync(out_d2, sc.d2.p, (size_t)n * k * 4, hipMemcpyDefault, st));
  if (out_found) MCHK(c, hipMemcpyAsync(out_found, sc.found.p, (size_t)n * 4, hipMemcpyDefault, st));
  MCHK(c, hipStreamSynchronize(st));
  return LISLAM_OK;
}

int lislam_map_associate(lislam_map* m, int32_t kind, const float* pts, int32_t n, int32_t stride, const double* x,
                         double* out_rec, int32_t* out_kind) {
  if (!m || n < 0 || (n > 0 && !pts) || !valid_stride(stride) || !x || (kind != 0 && kind != 1)) return LISLAM_ERR_ARG;
  if (n == 0) return LISLAM_OK;
  lislam_ctx* c = m->ctx;
  hipSetDevice(c->device);
  MapScratch& sc = m->sc;
  hipStream_t st = stream_of(c);
  MCHK(c, sc.q.reserve((size_t)n * stride * 4));
  MCHK(c, hipMemcpyAsync(sc.q.p, pts, (size_t)n * stride * 4, hipMemcpyDefault, st));
  MCHK(c, sc.x.reserve(64));
  MCHK(c, hipMemcpyAsync(sc.x.p, x, 56, hipMemcpyDefault, st));
  MCHK(c, sc.rec.reserve((size_t)n * 72));
  MCHK(c, sc.kind.reserve((size_t)n * 4));
  MRC(associate_device(m, kind, sc.q.as<float>(), stride, nullptr, n, sc.x.as<double>(), sc.rec.as<double>(),
                       sc.kind.as<int>()));
  if (out_rec) MCHK(c, hipMemcpyAsync(out_rec, sc.rec.p, (size_t)n * 72, hipMemcpyDefault, st));
  if (out_kind) MCHK(c, hipMemcpyAsync(out_kind, sc.kind.p, (size_t)n * 4, hipMemcpyDefault, st));
  MCHK(c, hipStreamSynchronize(st));
  return LISLAM_OK;
}

int lislam_normal_equations(lislam_ctx* c, const double* rec, const int32_t* kind, int32_t n, const double* x,
                            double* out28) {
  if (!c || n < 0 || (n > 0 && (!rec || !kind)) || !x || !out28) return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  MapScratch& sc = ctx_scratch(c);
  hipStream_t st = stream_of(c);
  MCHK(c, sc.rec.reserve((size_t)std::max(n, 1) * 72));
  MCHK(c, sc.kind.reserve((size_t)std::max(n, 1) * 4));
  MCHK(c, sc.lm.reserve(sizeof(LmDev)));
  MCHK(c, sc.partial.reserve((size_t)kMaxParts * kPart * 8));
  MCHK(c, sc.x.reserve(64));
  if (n) {
    MCHK(c, hipMemcpyAsync(sc.rec.p, rec, (size_t)n * 72, hipMemcpyDefault, st));
    MCHK(c, hipMemcpyAsync(sc.kind.p, kind, (size_t)n * 4, hipMemcpyDefault, st));
  }
  MCHK(c, hipMemcpyAsync(sc.x.p, x, 56, hipMemcpyDefault, st));
  LmDev* lm = sc.lm.as<LmDev>();
  hipLaunchKernelGGL(k_lm_init, dim3(1), dim3(64), 0, st, lm, sc.x.as<double>(), (unsigned*)nullptr);
  const int parts = std::min(kMaxParts, blocks(std::max(n, 1), kEvalThreads));
  hipLaunchKernelGGL(k_lm_eval, dim3(parts), dim3(kEvalThreads), 0, st, sc.rec.as<double>(), sc.kind.as<int>(), nullptr,
                     n, lm, sc.partial.as<double>());
  std::vector<double> part((size_t)parts * kPart);
  MCHK(c, hipMemcpyAsync(part.data(), sc.partial.p, part.size() * 8, hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  for (int e = 0; e < kAcc; e++) {
    double v = 0;
    for (int p = 0; p < parts; p++) v += part[(size_t)p * kPart + e];
    out28[e] = v;
  }
  return LISLAM_OK;
}

int lislam_pose_solve(lislam_ctx* c, const double* rec, const int32_t* kind, int32_t n, double* x, int32_t max_iterations,
                      int32_t* summary) {
  if (!c || n < 0 || (n > 0 && (!rec || !kind)) || !x || max_iterations < 0) return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  MapScratch& sc = ctx_scratch(c);
  hipStream_t st = stream_of(c);
  MCHK(c, sc.rec.reserve((size_t)std::max(n, 1) * 72));
  MCHK(c, sc.kind.reserve((size_t)std::max(n, 1) * 4));
  MCHK(c, sc.x.reserve(128));
  if (n) {
    MCHK(c, hipMemcpyAsync(sc.rec.p, rec, (size_t)n * 72, hipMemcpyDefault, st));
    MCHK(c, hipMemcpyAsync(sc.kind.p, kind, (size_t)n * 4, hipMemcpyDefault, st));
  }
  MCHK(c, hipMemcpyAsync(sc.x.p, x, 56, hipMemcpyDefault, st));
  int* dsum = reinterpret_cast<int*>(sc.x.as<double>() + 8);
  MRC(solve_device(c, sc, sc.rec.as<double>(), sc.kind.as<int>(), nullptr, n, sc.x.as<double>(), max_iterations,
                   sc.x.as<double>(), dsum));
  int hs[4];
  MCHK(c, hipMemcpyAsync(x, sc.x.p, 56, hipMemcpyDefault, st));
  MCHK(c, hipMemcpyAsync(hs, dsum, 16, hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  if (summary) for (int e = 0; e < 4; e++) summary[e] = hs[e];
  return LISLAM_OK;
}

int lislam_voxel_grid(lislam_ctx* c, const float* pts, int32_t n, float leaf, float* out, int32_t* n_out) {
  if (!c || n < 0 || (n > 0 && (!pts || !out)) || !n_out || !(leaf > 0)) return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  MapScratch& sc = ctx_scratch(c);
  hipStream_t st = stream_of(c);
  MRC(stage_points(c, sc, sc.q, pts, n, 4));
  MCHK(c, sc.vout.reserve((size_t)std::max(n, 1) * 16));
  MCHK(c, sc.counters.reserve(64));
  MRC(voxel_grid_device(c, sc, sc.q.as<float4>(), n, leaf, sc.vout.as<float4>(), sc.counters.as<int>()));
  int no = 0;
  MCHK(c, hipMemcpyAsync(&no, sc.counters.p, 4, hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  if (no) MCHK(c, hipMemcpyAsync(out, sc.vout.p, (size_t)no * 16, hipMemcpyDefault, st));
  MCHK(c, hipStreamSynchronize(st));
  *n_out = no;
  return LISLAM_OK;
}

int lislam_mapopt_step(lislam_map* m, const float* ground, int32_t n, const double* odom, double* state,
                       double* out_pose, int32_t* summary) {
  return lislam_mapopt_step_corner(m, nullptr, ground, n, nullptr, 0, odom, state, out_pose, summary);
}

// pc_corner into the corner ikd-Tree at the keyframe pose (device pose): Build on the ground map's
// first keyframe (mapOptimization.cpp:193-195), Add_Points(downsample) on every later one
// (:477-479) — also when the first keyframe's corner cloud was empty and the tree still is.
static int corner_map_update(lislam_map* cm, const float* corner, int nc, const double* pose, bool first) {
  lislam_ctx* c = cm->ctx;
  hipStream_t st = stream_of(c);
  MapScratch& sc = cm->sc;
  MRC(stage_points(c, sc, sc.vout, corner, nc, 4));
  MCHK(c, sc.vin.reserve((size_t)std::max(nc, 1) * 16));
  hipLaunchKernelGGL(k_transform, dim3(blocks(nc)), dim3(256), 0, st, sc.vout.as<float>(), 4, (const int*)nullptr, nc,
                     pose, sc.vin.as<float>());
  if (first) {
    MCHK(c, cm->tmp.reserve((size_t)std::max(nc, 1) * 16));
    hipLaunchKernelGGL(k_pack_points, dim3(blocks(nc)), dim3(256), 0, st, sc.vin.as<float>(), nc, 4, 0, cm->tmp.as<float4>());
    cm->next_id = nc;
    MRC(rebuild(cm, nc));
  } else {
    MCHK(c, cm->newp.reserve((size_t)std::max(nc, 1) * 16));
    hipLaunchKernelGGL(k_pack_points, dim3(blocks(nc)), dim3(256), 0, st, sc.vin.as<float>(), nc, 4, cm->next_id,
                       cm->newp.as<float4>());
    cm->next_id += nc;
    MRC(add_packed(cm, nc, true, nullptr));
  }
  MCHK(c, hipGetLastError());
  return LISLAM_OK;
}

int lislam_mapopt_step_corner(lislam_map* m, lislam_map* cm, const float* ground, int32_t n, const float* corner,
                              int32_t nc, const double* odom, double* state, double* out_pose, int32_t* summary) {
  if (!m || n < 0 || (n > 0 && !ground) || !odom || !state || nc < 0 || (nc > 0 && !corner) ||
      (cm && (cm->ctx != m->ctx || cm == m)))
    return LISLAM_ERR_ARG;
  lislam_ctx* c = m->ctx;
  hipSetDevice(c->device);
  MapScratch& sc = m->sc;
  hipStream_t st = stream_of(c);
  // device pose block: [0,7) state, [8,15) odom, [16,23) x, [24,31) keyframe pose
  MCHK(c, sc.x.reserve(40 * 8));
  double* dp = sc.x.as<double>();
  MCHK(c, hipMemcpyAsync(dp, state, 56, hipMemcpyDefault, st));
  MCHK(c, hipMemcpyAsync(dp + 8, odom, 56, hipMemcpyDefault, st));
  hipLaunchKernelGGL(k_mapopt_pose, dim3(1), dim3(64), 0, st, 0, dp, dp + 8, dp + 16, (const LmDev*)nullptr, dp + 24);
  int32_t summ[3] = {0, 0, -1};
  MRC(stage_points(c, sc, sc.vout, ground, n, 4));  // sensor-frame ground cloud (float4)
  if (m->n == 0) {  // first keyframe: Build with the transformed raw cloud (mapOptimization.cpp:185-192)
    MCHK(c, m->tmp.reserve((size_t)std::max(n, 1) * 16));
    MCHK(c, sc.vin.reserve((size_t)std::max(n, 1) * 16));
    hipLaunchKernelGGL(k_transform, dim3(blocks(n)), dim3(256), 0, st, sc.vout.as<float>(), 4, (const int*)nullptr, n,
                       dp + 16, sc.vin.as<float>());
    hipLaunchKernelGGL(k_pack_points, dim3(blocks(n)), dim3(256), 0, st, sc.vin.as<float>(), n, 4, 0, m->tmp.as<float4>());
    m->next_id = n;
    MRC(rebuild(m, n));
    if (cm && nc > 0) MRC(corner_map_update(cm, corner, nc, dp + 16, true));
    MCHK(c, hipMemcpyAsync(out_pose, dp + 16, 56, hipMemcpyDefault, st));
  } else {
    // VoxelGrid(0.8) (:368-370) of the xyz cloud (PointXYZ: intensity lane zeroed)
    MCHK(c, sc.flag.reserve((size_t)std::max(n, 1) * 4));
    MCHK(c, sc.counters.reserve(64));
    MCHK(c, sc.vin.reserve((size_t)std::max(n, 1) * 16));
    MCHK(c, hipMemcpy2DAsync(sc.vin.p, 16, sc.vout.p, 16, 12, n, hipMemcpyDeviceToDevice, st));
    MCHK(c, hipMemset2DAsync(sc.vin.as<char>() + 12, 16, 0, 4, n, st));
    DBuf& voxbuf = sc.vox;
    MCHK(c, voxbuf.reserve((size_t)std::max(n, 1) * 16));
    int* nvox = sc.counters.as<int>();
    MRC(voxel_grid_device(c, sc, sc.vin.as<float4>(), n, 0.8f, voxbuf.as<float4>(), nvox));
    MCHK(c, sc.rec.reserve((size_t)std::max(n, 1) * 72));
    MCHK(c, sc.kind.reserve((size_t)std::max(n, 1) * 4));
    MRC(associate_device(m, 1, voxbuf.as<float>(), 4, nvox, n, dp + 16, sc.rec.as<double>(), sc.kind.as<int>()));
    MRC(solve_device(c, sc, sc.rec.as<double>(), sc.kind.as<int>(), nvox, n, dp + 16, 10, nullptr, nullptr));
    LmDev* lm = sc.lm.as<LmDev>();
    hipLaunchKernelGGL(k_mapopt_pose, dim3(1), dim3(64), 0, st, 1, dp, dp + 8, dp + 16, lm, dp + 24);
    int* dsum = reinterpret_cast<int*>(dp + 32);
    hipLaunchKernelGGL(k_lm_finish, dim3(1), dim3(64), 0, st, lm, dp + 16, dsum);
    // Add_Points(downsample) of the voxelized cloud at the keyframe pose (:467-475)
    MCHK(c, m->newp.reserve((size_t)std::max(n, 1) * 16));
    hipLaunchKernelGGL(k_transform, dim3(blocks(n)), dim3(256), 0, st, voxbuf.as<float>(), 4, nvox, n, dp + 24,
                       sc.vin.as<float>());
    int hn = 0;
    int hs[4];
    MCHK(c, hipMemcpyAsync(&hn, nvox, 4, hipMemcpyDeviceToHost, st));
    MCHK(c, hipMemcpyAsync(hs, dsum, 16, hipMemcpyDeviceToHost, st));
    MCHK(c, hipStreamSynchronize(st));
    summ[0] = hs[3];
    summ[1] = hs[0];
    summ[2] = hs[1];
    hipLaunchKernelGGL(k_pack_points, dim3(blocks(hn)), dim3(256), 0, st, sc.vin.as<float>(), hn, 4, m->next_id,
                       m->newp.as<float4>());
    m->next_id += hn;
    MRC(add_packed(m, hn, true, nullptr));
    if (cm && nc > 0) MRC(corner_map_update(cm, corner, nc, dp + 24, false));  // the same keyframe pose as the ground cloud
    MCHK(c, hipMemcpyAsync(out_pose, dp + 16, 56, hipMemcpyDefault, st));
    MCHK(c, hipMemcpyAsync(state, dp, 56, hipMemcpyDefault, st));
  }
  MCHK(c, hipStreamSynchronize(st));
  if (summary) for (int e = 0; e < 3; e++) summary[e] = summ[e];
  return LISLAM_OK;
}

int lislam_laser_mapping(lislam_map* mc, lislam_map* ms, const float* corner, int32_t nc, const float* surf, int32_t ns,
                         double* x, int32_t* stats) {
  if (!mc || !ms || mc->ctx != ms->ctx || nc < 0 || ns < 0 || (nc && !corner) || (ns && !surf) || !x)
    return LISLAM_ERR_ARG;
  lislam_ctx* c = mc->ctx;
  hipSetDevice(c->device);
  MapScratch& sc = mc->sc;
  hipStream_t st = stream_of(c);
  const int n = nc + ns;
  MCHK(c, sc.x.reserve(40 * 8));
  double* dp = sc.x.as<double>();
  MCHK(c, hipMemcpyAsync(dp, x, 56, hipMemcpyDefault, st));
  DBuf& qc = sc.qc;
  DBuf& qs = sc.qs;
  MRC(stage_points(c, sc, qc, corner, nc, 4));
  MRC(stage_points(c, sc, qs, surf, ns, 4));
  MCHK(c, sc.rec.reserve((size_t)std::max(n, 1) * 72));
  MCHK(c, sc.kind.reserve((size_t)std::max(n, 1) * 4));
  int hs[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  int* dsum = reinterpret_cast<int*>(dp + 32);
  for (int outer = 0; outer < 2; outer++) {
    MRC(associate_device(mc, 0, qc.as<float>(), 4, nullptr, nc, dp, sc.rec.as<double>(), sc.kind.as<int>()));
    MRC(associate_device(ms, 1, qs.as<float>(), 4, nullptr, ns, dp, sc.rec.as<double>() + (size_t)nc * 9,
                         sc.kind.as<int>() + nc));
    MRC(solve_device(c, sc, sc.rec.as<double>(), sc.kind.as<int>(), nullptr, n, dp, 4, dp, dsum + outer * 4));
  }
  MCHK(c, hipMemcpyAsync(x, dp, 56, hipMemcpyDefault, st));
  MCHK(c, hipMemcpyAsync(hs, dsum, 32, hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  if (stats)
    for (int o = 0; o < 2; o++) { stats[o * 2] = hs[o][2]; stats[o * 2 + 1] = hs[o][3]; }
  return LISLAM_OK;
}

}  // extern "C"

// ===================================================================== laserMapping cube map
// The A-LOAM local map of laserMapping::process (laserMapping.cpp:70-99,
// 319-1002) kept on the device.  Semantics: oracle/oracle_map.cpp oracle_lmap_step.
//   pool     per cloud (corner, surf): points float4 (x, y, z, intensity) sorted by cube index,
//            with the cube index of each point and the CSR offsets of the 4851 cubes
//   shift    re-centring moves cube (i, j, k) to (i + si, j + sj, k + sk) and clears the cubes
//            that wrap around: a translation of every index — order-preserving — plus a drop
//   local    the valid cubes (i, j, k loop order) concatenated into the maps the optimization
//            searches (lislam_map_build + lislam_laser_mapping)
//   update   the voxelized current clouds at the optimized pose join their cubes after the old
//            points, and every valid cube is voxelized: one stable radix sort of
//            (cube << 32 | voxel index) keys over old + new points — non-valid (and too-fine)
//            cubes key by position, so each point is its own voxel and passes unchanged
namespace lislam {
namespace cubek {

constexpr int kW = 21, kH = 21, kD = 11, kNC = kW * kH * kD;

struct CubeSeg {  // per valid cube: VoxelGrid parameters of its points (old + new)
  unsigned mn[3], mx[3];  // ord_f-encoded bounds
  int min_b[3], mul1, mul2, overflow;
};

__device__ __forceinline__ int cube_of(double v, int cen) {
  int c = int((v + 25.0) / 50.0) + cen;
  if (v + 25.0 < 0) c--;
  return c;
}

// re-centring: the kept flag and the translated cube index of every pool point
__global__ void k_cm_shift(const int* cube, int n, int si, int sj, int sk, int* keep, int* ncube) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = cube[i];
  const int ci = c % kW + si, cj = (c / kW) % kH + sj, ck = c / (kW * kH) + sk;
  const bool ok = ci >= 0 && ci < kW && cj >= 0 && cj < kH && ck >= 0 && ck < kD;
  keep[i] = ok;
  ncube[i] = ok ? ci + kW * cj + kW * kH * ck : -1;
}

// CSR offsets of the cubes over a pool sorted by cube (off[kNC] = n)
__global__ void k_cm_offsets(const int* cube, int n, int* off) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > kNC) return;
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cube[mid] < c) lo = mid + 1; else hi = mid;
  }
  off[c] = lo;
}

// local map: workgroup v copies valid cube v (loop order) to its place in the concatenation
__global__ __launch_bounds__(256) void k_cm_gather(const int* valid, int nvalid, const int* off, const float4* pts,
                                                   float4* out, int* n_out) {
  const int v = blockIdx.x;
  int pre = 0;
  for (int u = 0; u < v; u++) pre += off[valid[u] + 1] - off[valid[u]];
  const int c = valid[v], b = off[c], cnt = off[c + 1] - b;
  for (int k = threadIdx.x; k < cnt; k += blockDim.x) out[pre + k] = pts[b + k];
  if (v == nvalid - 1 && threadIdx.x == 0) *n_out = pre + cnt;
}

// new points: pointAssociateToMap at the pose x (laserMapping.cpp:152-161) and their cube
__global__ void k_cm_newpts(const float4* in, const int* n_in, const double* x, int cenW, int cenH, int cenD,
                            float4* out, int* cube) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *n_in) return;
  const float4 p = in[i];
  const float4 w = mapk::to_world(x, p.x, p.y, p.z);
  const int ci = cube_of(w.x, cenW), cj = cube_of(w.y, cenH), ck = cube_of(w.z, cenD);
  const bool ok = ci >= 0 && ci < kW && cj >= 0 && cj < kH && ck >= 0 && ck < kD;
  out[i] = make_float4(w.x, w.y, w.z, p.w);
  cube[i] = ok ? ci + kW * cj + kW * kH * ck : -1;
}

// bounds and VoxelGrid parameters of valid cube v: its old pool points and its new points
__global__ __launch_bounds__(256) void k_cm_bounds(const int* valid, const int* off, const float4* pts, const float4* newp,
                                                   const int* ncube, const int* n_new, float inv, CubeSeg* seg) {
  __shared__ unsigned smn[3][4], smx[3][4];
  const int v = blockIdx.x, c = valid[v];
  unsigned mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
  auto add = [&](float4 p) {
    const unsigned q[3] = {mapk::ord_f(p.x), mapk::ord_f(p.y), mapk::ord_f(p.z)};
    for (int k = 0; k < 3; k++) { mn[k] = min(mn[k], q[k]); mx[k] = max(mx[k], q[k]); }
  };
  for (int i = off[c] + threadIdx.x; i < off[c + 1]; i += blockDim.x) add(pts[i]);
  for (int i = threadIdx.x; i < *n_new; i += blockDim.x)
    if (ncube[i] == c) add(newp[i]);
  for (int o = 32; o > 0; o >>= 1)
    for (int k = 0; k < 3; k++) {
      mn[k] = min(mn[k], (unsigned)__shfl_xor((int)mn[k], o));
      mx[k] = max(mx[k], (unsigned)__shfl_xor((int)mx[k], o));
    }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 3; k++) { smn[k][w] = mn[k]; smx[k][w] = mx[k]; }
  __syncthreads();
  if (threadIdx.x != 0) return;
  CubeSeg s;
  float fmn[3], fmx[3];
  for (int k = 0; k < 3; k++) {
    unsigned a0 = smn[k][0], a1 = smx[k][0];
    for (int j = 1; j < 4; j++) { a0 = min(a0, smn[k][j]); a1 = max(a1, smx[k][j]); }
    s.mn[k] = a0; s.mx[k] = a1;
    fmn[k] = mapk::unord_f(a0); fmx[k] = mapk::unord_f(a1);
  }
  // pcl::VoxelGrid::applyFilter (as k_vg_keys): 32-bit index space or the input unchanged
  const int64_t dx = (int64_t)((fmx[0] - fmn[0]) * inv) + 1, dy = (int64_t)((fmx[1] - fmn[1]) * inv) + 1,
                dz = (int64_t)((fmx[2] - fmn[2]) * inv) + 1;
  s.overflow = dx * dy * dz > (int64_t)0x7fffffff;
  int div_b[3];
  for (int k = 0; k < 3; k++) {
    s.min_b[k] = (int)floorf(fmn[k] * inv);
    div_b[k] = (int)floorf(fmx[k] * inv) - s.min_b[k] + 1;
  }
  s.mul1 = div_b[0];
  s.mul2 = div_b[0] * div_b[1];
  seg[v] = s;
}

// keys over the concatenation [pool (n_pool), new points]: cube << 32 | voxel index in a
// valid cube, | concatenation index otherwise; dropped new points sort last
__global__ void k_cm_keys(const float4* pts, const int* cube, int n_pool, const float4* newp, const int* ncube,
                          const int* n_new, const int* vrank, const CubeSeg* seg, float inv, uint64_t* keys, int* idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int m = n_pool + *n_new;
  if (i >= m) return;
  const bool old = i < n_pool;
  const int c = old ? cube[i] : ncube[i - n_pool];
  idx[i] = i;
  if (c < 0) { keys[i] = ~0ull; return; }
  const int v = vrank[c];
  uint32_t low = (uint32_t)i;
  if (v >= 0 && !seg[v].overflow) {
    const float4 p = old ? pts[i] : newp[i - n_pool];
    const CubeSeg& s = seg[v];
    const int i0 = (int)(floorf(p.x * inv) - (float)s.min_b[0]);
    const int i1 = (int)(floorf(p.y * inv) - (float)s.min_b[1]);
    const int i2 = (int)(floorf(p.z * inv) - (float)s.min_b[2]);
    low = (uint32_t)(i0 + i1 * s.mul1 + i2 * s.mul2);
  }
  keys[i] = ((uint64_t)(uint32_t)c << 32) | low;
}

__global__ void k_cm_runs(const uint64_t* skeys, const int* n_pool_new, int n_pool, int* flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_pool + *n_pool_new) return;
  flag[i] = skeys[i] != ~0ull && (i == 0 || skeys[i] != skeys[i - 1]) ? 1 : 0;
}

// centroids of the runs (sums in concatenation order), cube index from the key
__global__ void k_cm_centroids(const float4* pts, int n_pool, const float4* newp, const int* n_new, const uint64_t* skeys,
                               const int* sidx, const int* pos, const int* flag, float4* out, int* ocube, int* n_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int m = n_pool + *n_new;
  if (i == 0) *n_out = m > 0 ? pos[m - 1] + flag[m - 1] : 0;
  if (i >= m || !flag[i]) return;
  auto at = [&](int j) { const int s = sidx[j]; return s < n_pool ? pts[s] : newp[s - n_pool]; };
  float4 c = at(i);
  int e = i + 1;
  for (; e < m && skeys[e] == skeys[i]; e++) {
    const float4 p = at(e);
    c.x += p.x; c.y += p.y; c.z += p.z; c.w += p.w;
  }
  const float cnt = (float)(e - i);
  c.x /= cnt; c.y /= cnt; c.z /= cnt; c.w /= cnt;
  out[pos[i]] = c;
  ocube[pos[i]] = (int)(skeys[i] >> 32);
}

__global__ void k_cm_vrank(int* vrank) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < kNC) vrank[c] = -1;
}
__global__ void k_cm_vrank_set(const int* valid, int nvalid, int* vrank) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < nvalid) vrank[valid[v]] = v;
}

}  // namespace cubek
}  // namespace lislam

namespace {
// host restatements of the Eigen double quaternion operations (lislam_device.hpp term grouping)
void h_qmul(const double* a, const double* b, double* r) {
  r[0] = (a[3] * b[0] + a[1] * b[2]) + (-(a[2] * b[1] - a[0] * b[3]));
  r[1] = (a[3] * b[1] + a[1] * b[3]) + (a[2] * b[0] - a[0] * b[2]);
  r[2] = (a[3] * b[2] - a[1] * b[0]) + (a[2] * b[3] + a[0] * b[1]);
  r[3] = (a[3] * b[3] - a[1] * b[1]) + (-(a[2] * b[2] + a[0] * b[0]));
}
void h_qrot(const double* q, const double* v, double* o) {
  double u[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
  for (int k = 0; k < 3; k++) u[k] = u[k] + u[k];
  const double c[3] = {q[1] * u[2] - q[2] * u[1], q[2] * u[0] - q[0] * u[2], q[0] * u[1] - q[1] * u[0]};
  for (int k = 0; k < 3; k++) o[k] = (v[k] + q[3] * u[k]) + c[k];
}
int h_cube_of(double v, int cen) {
  int c = int((v + 25.0) / 50.0) + cen;
  if (v + 25.0 < 0) c--;
  return c;
}
}  // namespace

struct lislam_lmap {
  lislam_ctx* ctx = nullptr;
  float res[2] = {0.4f, 0.8f};  // line (corner), plane (surf) resolutions
  int cen[3] = {10, 10, 5};
  int64_t n[2] = {0, 0};
  DBuf pts[2], cube[2], off[2], tmp_pts, tmp_cube, keep, local[2], counts, valid, vrank, seg, newp, ncube, keys, keys2,
      idx, idx2, flag, pos, sort_tmp, x, stack[2];
  lislam_map* maps[2] = {nullptr, nullptr};
  MapScratch sc;
};

namespace {

using namespace lislam::cubek;

// offsets of pool w after its points / cubes changed (n on the host)
int cm_offsets(lislam_lmap* L, int w) {
  lislam_ctx* c = L->ctx;
  MCHK(c, L->off[w].reserve((kNC + 1) * sizeof(int)));
  hipLaunchKernelGGL(k_cm_offsets, dim3(blocks(kNC + 1)), dim3(256), 0, stream_of(c), L->cube[w].as<int>(), (int)L->n[w],
                     L->off[w].as<int>());
  MCHK(c, hipGetLastError());
  return LISLAM_OK;
}

// re-centring of pool w by (si, sj, sk)
int cm_shift(lislam_lmap* L, int w, int si, int sj, int sk) {
  lislam_ctx* c = L->ctx;
  hipStream_t st = stream_of(c);
  const int n = (int)L->n[w];
  if (n == 0) return LISLAM_OK;
  MCHK(c, L->keep.reserve((size_t)n * 4));
  MCHK(c, L->tmp_cube.reserve((size_t)n * 4));
  MCHK(c, L->tmp_pts.reserve((size_t)n * 16));
  MCHK(c, L->counts.reserve(64));
  hipLaunchKernelGGL(k_cm_shift, dim3(blocks(n)), dim3(256), 0, st, L->cube[w].as<int>(), n, si, sj, sk,
                     L->keep.as<int>(), L->tmp_cube.as<int>());
  MCHK(c, L->sort_tmp.reserve(prims::select_temp_bytes(n)));
  MCHK(c, prims::select_flagged(L->sort_tmp.p, L->pts[w].as<float4>(), L->keep.as<int>(), L->tmp_pts.as<float4>(),
                                L->counts.as<int>(), n, st));
  MCHK(c, prims::select_flagged(L->sort_tmp.p, L->tmp_cube.as<int>(), L->keep.as<int>(), L->cube[w].as<int>(),
                                L->counts.as<int>() + 1, n, st));
  int kept = 0;
  MCHK(c, hipMemcpyAsync(&kept, L->counts.p, 4, hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  MCHK(c, hipMemcpyAsync(L->pts[w].p, L->tmp_pts.p, (size_t)kept * 16, hipMemcpyDeviceToDevice, st));
  L->n[w] = kept;
  return cm_offsets(L, w);
}

// insertion of the (device, count on the device) stack of cloud w at the pose on the device, then
// the VoxelGrid of every valid cube
int cm_update(lislam_lmap* L, int w, const float4* stack, const int* n_stack, int n_stack_host, int nvalid) {
  lislam_ctx* c = L->ctx;
  hipStream_t st = stream_of(c);
  const int np = (int)L->n[w], nn = n_stack_host, m = np + nn;
  const float inv = 1.0f / L->res[w];
  MCHK(c, L->newp.reserve((size_t)std::max(nn, 1) * 16));
  MCHK(c, L->ncube.reserve((size_t)std::max(nn, 1) * 4));
  if (nn > 0)
    hipLaunchKernelGGL(k_cm_newpts, dim3(blocks(nn)), dim3(256), 0, st, stack, n_stack, L->x.as<double>(), L->cen[0],
                       L->cen[1], L->cen[2], L->newp.as<float4>(), L->ncube.as<int>());
  if (m == 0) return LISLAM_OK;
  MCHK(c, L->seg.reserve((size_t)std::max(nvalid, 1) * sizeof(CubeSeg)));
  if (nvalid > 0)
    hipLaunchKernelGGL(k_cm_bounds, dim3(nvalid), dim3(256), 0, st, L->valid.as<int>(), L->off[w].as<int>(),
                       L->pts[w].as<float4>(), L->newp.as<float4>(), L->ncube.as<int>(), n_stack, inv, L->seg.as<CubeSeg>());
  MCHK(c, L->keys.reserve((size_t)m * 8));
  MCHK(c, L->keys2.reserve((size_t)m * 8));
  MCHK(c, L->idx.reserve((size_t)m * 4));
  MCHK(c, L->idx2.reserve((size_t)m * 4));
  MCHK(c, L->flag.reserve((size_t)m * 4));
  MCHK(c, L->pos.reserve((size_t)m * 4));
  hipLaunchKernelGGL(k_cm_keys, dim3(blocks(m)), dim3(256), 0, st, L->pts[w].as<float4>(), L->cube[w].as<int>(), np,
                     L->newp.as<float4>(), L->ncube.as<int>(), n_stack, L->vrank.as<int>(), L->seg.as<CubeSeg>(), inv,
                     L->keys.as<uint64_t>(), L->idx.as<int>());
  MRC(sort_pairs_u64(c, L->sort_tmp, L->keys.as<uint64_t>(), L->keys2.as<uint64_t>(), L->idx.as<int>(),
                     L->idx2.as<int>(), m));
  hipLaunchKernelGGL(k_cm_runs, dim3(blocks(m)), dim3(256), 0, st, L->keys2.as<uint64_t>(), n_stack, np, L->flag.as<int>());
  MCHK(c, L->sort_tmp.reserve(prims::exclusive_sum_temp_bytes(m)));
  MCHK(c, prims::exclusive_sum(L->sort_tmp.p, L->flag.as<int>(), L->pos.as<int>(), m, st));
  MCHK(c, L->tmp_pts.reserve((size_t)m * 16));
  MCHK(c, L->tmp_cube.reserve((size_t)m * 4));
  MCHK(c, L->counts.reserve(64));
  hipLaunchKernelGGL(k_cm_centroids, dim3(blocks(m)), dim3(256), 0, st, L->pts[w].as<float4>(), np, L->newp.as<float4>(),
                     n_stack, L->keys2.as<uint64_t>(), L->idx2.as<int>(), L->pos.as<int>(), L->flag.as<int>(),
                     L->tmp_pts.as<float4>(), L->tmp_cube.as<int>(), L->counts.as<int>() + 2);
  MCHK(c, hipGetLastError());
  int nout = 0;
  MCHK(c, hipMemcpyAsync(&nout, L->counts.as<int>() + 2, 4, hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  MCHK(c, L->pts[w].reserve((size_t)std::max(nout, 1) * 16));
  MCHK(c, L->cube[w].reserve((size_t)std::max(nout, 1) * 4));
  MCHK(c, hipMemcpyAsync(L->pts[w].p, L->tmp_pts.p, (size_t)nout * 16, hipMemcpyDeviceToDevice, st));
  MCHK(c, hipMemcpyAsync(L->cube[w].p, L->tmp_cube.p, (size_t)nout * 4, hipMemcpyDeviceToDevice, st));
  L->n[w] = nout;
  return cm_offsets(L, w);
}

}  // namespace

extern "C" {

int lislam_lmap_create(lislam_ctx* c, float line_res, float plane_res, lislam_lmap** out) {
  if (!c || !out || !(line_res > 0) || !(plane_res > 0)) return LISLAM_ERR_ARG;
  *out = nullptr;
  hipSetDevice(c->device);
  lislam_lmap* L = new lislam_lmap();
  L->ctx = c;
  L->res[0] = line_res;
  L->res[1] = plane_res;
  const lislam_map_config mc{0.4f, 0.0f};
  int rc = LISLAM_OK;
  for (int w = 0; w < 2 && !rc; w++) {
    rc = lislam_map_create(c, &mc, &L->maps[w]);
    if (!rc && L->off[w].reserve((kNC + 1) * sizeof(int)) != hipSuccess) rc = LISLAM_ERR_DEVICE;
    if (!rc && hipMemsetAsync(L->off[w].p, 0, (kNC + 1) * sizeof(int), c->stream) != hipSuccess) rc = LISLAM_ERR_DEVICE;
  }
  if (!rc && (L->vrank.reserve(kNC * sizeof(int)) != hipSuccess || L->valid.reserve(128 * sizeof(int)) != hipSuccess ||
              L->x.reserve(64) != hipSuccess))
    rc = LISLAM_ERR_DEVICE;
  if (rc) {
    for (auto* m : L->maps) lislam_map_destroy(m);
    delete L;
    return mfail(c, LISLAM_ERR_DEVICE, "lislam_lmap_create failed");
  }
  *out = L;
  return LISLAM_OK;
}

int lislam_lmap_destroy(lislam_lmap* L) {
  if (!L) return LISLAM_OK;
  hipSetDevice(L->ctx->device);
  (void)hipStreamSynchronize(L->ctx->stream);
  for (auto* m : L->maps) lislam_map_destroy(m);
  delete L;
  return LISLAM_OK;
}

int lislam_lmap_counts(lislam_lmap* L, int32_t* corner_counts, int32_t* surf_counts) {
  if (!L) return LISLAM_ERR_ARG;
  lislam_ctx* c = L->ctx;
  hipSetDevice(c->device);
  int32_t* dst[2] = {corner_counts, surf_counts};
  for (int w = 0; w < 2; w++) {
    if (!dst[w]) continue;
    std::vector<int> off(kNC + 1);
    MCHK(c, hipMemcpyAsync(off.data(), L->off[w].p, off.size() * 4, hipMemcpyDeviceToHost, c->stream));
    MCHK(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < kNC; k++) dst[w][k] = off[k + 1] - off[k];
  }
  return LISLAM_OK;
}

int lislam_lmap_points(lislam_lmap* L, int32_t which, float* out, int64_t cap, int64_t* n) {
  if (!L || which < 0 || which > 1 || !n) return LISLAM_ERR_ARG;
  lislam_ctx* c = L->ctx;
  hipSetDevice(c->device);
  *n = L->n[which];
  if (!out) return LISLAM_OK;
  if (L->n[which] > cap) return mfail(c, LISLAM_ERR_CAPACITY, "lislam_lmap_points: %lld points, cap %lld",
                                      (long long)L->n[which], (long long)cap);
  if (L->n[which]) MCHK(c, hipMemcpyAsync(out, L->pts[which].p, (size_t)L->n[which] * 16, hipMemcpyDefault, c->stream));
  MCHK(c, hipStreamSynchronize(c->stream));
  return LISLAM_OK;
}

int lislam_lmap_step(lislam_lmap* L, const float* corner_last, int32_t nc, const float* surf_last, int32_t ns,
                     const double* odom, double* state, double* out_pose, int32_t* stats) {
  if (!L || nc < 0 || ns < 0 || (nc && !corner_last) || (ns && !surf_last) || !odom || !state) return LISLAM_ERR_ARG;
  lislam_ctx* c = L->ctx;
  hipSetDevice(c->device);
  hipStream_t st = stream_of(c);
  const double* qo = odom;
  const double* to = odom + 4;
  double* qm = state;
  double* tm = state + 4;
  // transformAssociateToMap (laserMapping.cpp:138-142)
  double x[7];
  h_qmul(qm, qo, x);
  {
    double tr[3];
    h_qrot(qm, to, tr);
    for (int k = 0; k < 3; k++) x[4 + k] = tr[k] + tm[k];
  }
  // re-centring (:330-565): the total translation of the cube indices
  int cc[3] = {h_cube_of(x[4], L->cen[0]), h_cube_of(x[5], L->cen[1]), h_cube_of(x[6], L->cen[2])};
  const int dims[3] = {kW, kH, kD};
  int sh[3] = {0, 0, 0};
  for (int a = 0; a < 3; a++) {
    while (cc[a] < 3) { cc[a]++; L->cen[a]++; sh[a]++; }
    while (cc[a] >= dims[a] - 3) { cc[a]--; L->cen[a]--; sh[a]--; }
  }
  if (sh[0] || sh[1] || sh[2])
    for (int w = 0; w < 2; w++) MRC(cm_shift(L, w, sh[0], sh[1], sh[2]));
  // valid cubes in the reference's loop order (:566-588)
  std::vector<int> valid;
  for (int i = cc[0] - 2; i <= cc[0] + 2; i++)
    for (int j = cc[1] - 2; j <= cc[1] + 2; j++)
      for (int k = cc[2] - 1; k <= cc[2] + 1; k++)
        if (i >= 0 && i < kW && j >= 0 && j < kH && k >= 0 && k < kD) valid.push_back(i + kW * j + kW * kH * k);
  const int nvalid = (int)valid.size();
  MCHK(c, hipMemcpyAsync(L->valid.p, valid.data(), (size_t)nvalid * 4, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_cm_vrank, dim3(blocks(kNC)), dim3(256), 0, st, L->vrank.as<int>());
  hipLaunchKernelGGL(k_cm_vrank_set, dim3(1), dim3(128), 0, st, L->valid.as<int>(), nvalid, L->vrank.as<int>());
  // local maps (:590-602)
  MCHK(c, L->counts.reserve(64));
  int* dcnt = L->counts.as<int>() + 8;  // [8, 10) local map sizes, [10, 12) stack sizes
  MCHK(c, hipMemsetAsync(dcnt, 0, 16, st));
  for (int w = 0; w < 2; w++) {
    MCHK(c, L->local[w].reserve((size_t)std::max<int64_t>(L->n[w], 1) * 16));
    if (nvalid > 0 && L->n[w] > 0)
      hipLaunchKernelGGL(k_cm_gather, dim3(nvalid), dim3(256), 0, st, L->valid.as<int>(), nvalid, L->off[w].as<int>(),
                         L->pts[w].as<float4>(), L->local[w].as<float4>(), dcnt + w);
  }
  // the current clouds, voxelized (:608-616)
  const float* last[2] = {corner_last, surf_last};
  const int nlast[2] = {nc, ns};
  for (int w = 0; w < 2; w++) {
    DBuf& q = w == 0 ? L->sc.qc : L->sc.qs;
    MRC(stage_points(c, L->sc, q, last[w], nlast[w], 4));
    MCHK(c, L->stack[w].reserve((size_t)std::max(nlast[w], 1) * 16));
    MRC(voxel_grid_device(c, L->sc, q.as<float4>(), nlast[w], L->res[w], L->stack[w].as<float4>(), dcnt + 2 + w));
  }
  int h4[4] = {0, 0, 0, 0};
  MCHK(c, hipMemcpyAsync(h4, dcnt, 16, hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  const int ncm = h4[0], nsm = h4[1], ncs = h4[2], nss = h4[3];
  if (stats) {
    stats[0] = ncm; stats[1] = nsm; stats[2] = ncs; stats[3] = nss;
    stats[4] = stats[5] = stats[6] = stats[7] = -1;
  }
  // the optimization (:620-857) when the map is large enough
  if (ncm > 10 && nsm > 50) {
    MRC(lislam_map_build(L->maps[0], L->local[0].as<float>(), ncm, 4));
    MRC(lislam_map_build(L->maps[1], L->local[1].as<float>(), nsm, 4));
    int s4[4];
    MRC(lislam_laser_mapping(L->maps[0], L->maps[1], L->stack[0].as<float>(), ncs, L->stack[1].as<float>(), nss, x, s4));
    if (stats) for (int k = 0; k < 4; k++) stats[4 + k] = s4[k];
  }
  // transformUpdate (:145-149) with Eigen's Quaternion::inverse (conjugate / squaredNorm)
  {
    const double n2 = (qo[0] * qo[0] + qo[2] * qo[2]) + (qo[1] * qo[1] + qo[3] * qo[3]);
    const double qinv[4] = {-qo[0] / n2, -qo[1] / n2, -qo[2] / n2, qo[3] / n2};
    double nq[4];
    h_qmul(x, qinv, nq);
    for (int k = 0; k < 4; k++) qm[k] = nq[k];
    double r[3];
    h_qrot(qm, to, r);
    for (int k = 0; k < 3; k++) tm[k] = x[4 + k] - r[k];
  }
  // insertion at the optimized pose and the VoxelGrid of the valid cubes (:880-1002)
  MCHK(c, hipMemcpyAsync(L->x.p, x, 56, hipMemcpyHostToDevice, st));
  MRC(cm_update(L, 0, L->stack[0].as<float4>(), dcnt + 2, ncs, nvalid));
  MRC(cm_update(L, 1, L->stack[1].as<float4>(), dcnt + 3, nss, nvalid));
  if (out_pose) for (int e = 0; e < 7; e++) out_pose[e] = x[e];
  return LISLAM_OK;
}

}  // extern "C"

// ================================================================== loop-closure ICP
// feature_tracker::loopClosureThread's USE_ICP block (src/intensity_feature_tracker.cpp:217-366)
// with tranformCurrentScanToMap (:167-172) and getSubmapOfhistory (:174-193), device resident:
//   k_lc_tf_d      transformPointCloud with the Matrix4d keyframe poses (double, stored as float)
//   k_lc_flags     removeNaNFromPointCloud + CropBox, compacted with hipCUB Select::Flagged
//   VoxelGrid      voxel_grid_device (PCL VoxelGrid semantics, as a21)
//   target map     the hash-grid k-NN map of a19-a21 (exact 1-NN, ties by target index)
//   per iteration  k_knn (1-NN of every source point) -> k_lc_step (one 1024-thread workgroup:
//                  correspondence MSE, means, demeaned cross-covariance in a fixed strided +
//                  halving-tree double order, Horn's quaternion eigenproblem by cyclic Jacobi,
//                  final = T * final, DefaultConvergenceCriteria) -> k_lc_apply (source *= T).
//   The host launches the iterations in chunks and reads one flag per chunk; once converged the
//   k-NN query count on the device drops to 0 and every later launch of the chunk exits at once.
//   getFitnessScore: the original source under `final`, 1-NN, mean squared distance.
// The restatement (oracle/oracle_map.cpp oracle_loop_icp) performs the same floating-point
// operations in the same order: results are bit-identical.
namespace lislam {
namespace loopk {

using mapk::MapView;

constexpr int kRed = 1024;

struct Mat34d {
  double m[12];
};

struct IcpParams {
  int max_iter;
  double rot_thr, trans_thr, mse_abs, mse_rel;
};

struct IcpDev {
  float T[16];  // transformation_ of the last iteration
  float F[16];  // final_transformation_
  double prev_mse, fitness;
  int iter, state, done, run, nq, ncorr;
};

__global__ void k_lc_tf_d(const float4* in, int n, Mat34d T, float4* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  const double x = p.x, y = p.y, z = p.z;
  const double* m = T.m;
  out[i] = make_float4((float)(((m[0] * x + m[1] * y) + m[2] * z) + m[3]), (float)(((m[4] * x + m[5] * y) + m[6] * z) + m[7]),
                       (float)(((m[8] * x + m[9] * y) + m[10] * z) + m[11]), p.w);
}

__global__ void k_lc_flags(const float4* in, int n, int use_crop, float lo, float hi, uint8_t* flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  bool keep = isfinite(p.x) && isfinite(p.y) && isfinite(p.z);
  if (keep && use_crop) keep = !(p.x < lo || p.y < lo || p.z < lo || p.x > hi || p.y > hi || p.z > hi);
  flag[i] = keep ? 1 : 0;
}

// target points for the k-NN map: w = index (the map's tie-break id)
__global__ void k_lc_ids(const float4* in, int n, float4* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  out[i] = make_float4(p.x, p.y, p.z, __int_as_float(i));
}

__device__ void jacobi4(double A[4][4], double V[4][4]) {
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
        double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
        if (theta < 0) t = -t;
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
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

// umeyama(src, tgt, false) through Horn's 4x4 quaternion matrix of S[a][b] = mean s'_a t'_b
__device__ void horn_rt(const double S[3][3], const double ms[3], const double mt[3], double R[3][3], double t[3]) {
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
  const double nn = sqrt(((w * w + x * x) + y * y) + z * z);
  w /= nn; x /= nn; y /= nn; z /= nn;
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y,
               tyz = tz * y, tzz = tz * z;
  R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz; R[0][2] = txz + twy;
  R[1][0] = txy + twz; R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
  R[2][0] = txz - twy; R[2][1] = tyz + twx; R[2][2] = 1 - (txx + tyy);
  for (int a = 0; a < 3; a++) t[a] = mt[a] - ((R[a][0] * ms[0] + R[a][1] * ms[1]) + R[a][2] * ms[2]);
}

// in-place halving tree over red[V][kRed] (every thread of the 1024-thread block calls it)
template <int V>
__device__ __forceinline__ void tree_sum(double (*red)[kRed]) {
  const int t = threadIdx.x;
  for (int s = kRed / 2; s > 0; s >>= 1) {
    if (t < s)
#pragma unroll
      for (int k = 0; k < V; k++) red[k][t] += red[k][t + s];
    __syncthreads();
  }
}

__global__ __launch_bounds__(kRed) void k_lc_step(IcpDev* st, const float4* src, const float4* nb, const float* d2,
                                                  const int* found, int n, IcpParams P) {
  __shared__ double red[9][kRed];
  const int t = threadIdx.x;
  if (st->done) {
    if (t == 0) st->run = 0;
    return;
  }
  {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = t; i < n; i += kRed) {
      if (found[i] <= 0) continue;
      const float4 s = src[i], q = nb[i];
      a[0] += 1.0; a[1] += (double)d2[i];
      a[2] += (double)s.x; a[3] += (double)s.y; a[4] += (double)s.z;
      a[5] += (double)q.x; a[6] += (double)q.y; a[7] += (double)q.z;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) red[k][t] = a[k];
  }
  __syncthreads();
  tree_sum<8>(red);
  const double cnt = red[0][0], sd2 = red[1][0];
  if (cnt < 3.0) {
    if (t == 0) {
      st->ncorr = (int)cnt;
      st->state = 5;
      st->done = 1;
      st->run = 0;
      st->nq = 0;
    }
    return;
  }
  const double ms[3] = {red[2][0] / cnt, red[3][0] / cnt, red[4][0] / cnt};
  const double mt[3] = {red[5][0] / cnt, red[6][0] / cnt, red[7][0] / cnt};
  __syncthreads();  // everyone has read the pass-1 sums
  {
    double a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = t; i < n; i += kRed) {
      if (found[i] <= 0) continue;
      const float4 s = src[i], q = nb[i];
      const double u[3] = {s.x - ms[0], s.y - ms[1], s.z - ms[2]};
      const double v[3] = {q.x - mt[0], q.y - mt[1], q.z - mt[2]};
#pragma unroll
      for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) a[3 * r + c] += u[r] * v[c];
    }
#pragma unroll
    for (int k = 0; k < 9; k++) red[k][t] = a[k];
  }
  __syncthreads();
  tree_sum<9>(red);
  if (t != 0) return;
  double S[3][3], R[3][3], tr[3];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) S[r][c] = red[3 * r + c][0] / cnt;
  horn_rt(S, ms, mt, R, tr);
  float T[16] = {(float)R[0][0], (float)R[0][1], (float)R[0][2], (float)tr[0], (float)R[1][0], (float)R[1][1],
                 (float)R[1][2], (float)tr[1], (float)R[2][0], (float)R[2][1], (float)R[2][2], (float)tr[2],
                 0.f, 0.f, 0.f, 1.f};
  float F[16], G[16];
  for (int k = 0; k < 16; k++) F[k] = st->F[k];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++)
      G[4 * r + c] = ((T[4 * r] * F[c] + T[4 * r + 1] * F[4 + c]) + T[4 * r + 2] * F[8 + c]) + T[4 * r + 3] * F[12 + c];
  for (int k = 0; k < 16; k++) { st->T[k] = T[k]; st->F[k] = G[k]; }
  const int it = st->iter + 1;
  st->iter = it;
  st->ncorr = (int)cnt;
  st->run = 1;
  int state = 0;
  const double mse = sd2 / cnt, prev = st->prev_mse;
  const double cos_angle = 0.5 * ((((double)T[0] + (double)T[5]) + (double)T[10]) - 1.0);
  const double tsq = ((double)T[3] * (double)T[3] + (double)T[7] * (double)T[7]) + (double)T[11] * (double)T[11];
  if (it >= P.max_iter) state = 1;
  else if (cos_angle >= P.rot_thr && tsq <= P.trans_thr) state = 2;
  else if (fabs(mse - prev) < P.mse_abs) state = 3;
  else if (fabs(mse - prev) / prev < P.mse_rel) state = 4;
  st->prev_mse = mse;
  if (state) {
    st->state = state;
    st->done = 1;
    st->nq = 0;
  }
}

// source *= T of this iteration (skipped when k_lc_step did not run)
__global__ void k_lc_apply(const IcpDev* st, float4* src, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !st->run) return;
  const float* T = st->T;
  const float4 p = src[i];
  src[i] = make_float4(((T[0] * p.x + T[1] * p.y) + T[2] * p.z) + T[3], ((T[4] * p.x + T[5] * p.y) + T[6] * p.z) + T[7],
                       ((T[8] * p.x + T[9] * p.y) + T[10] * p.z) + T[11], p.w);
}

// getFitnessScore's transformPointCloud(*input_, final_transformation_)
__global__ void k_lc_final_tf(const IcpDev* st, const float4* src, int n, float4* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* T = st->F;
  const float4 p = src[i];
  out[i] = make_float4(((T[0] * p.x + T[1] * p.y) + T[2] * p.z) + T[3], ((T[4] * p.x + T[5] * p.y) + T[6] * p.z) + T[7],
                       ((T[8] * p.x + T[9] * p.y) + T[10] * p.z) + T[11], p.w);
}

__global__ __launch_bounds__(kRed) void k_lc_fitness(IcpDev* st, const float* d2, const int* found, int n) {
  __shared__ double red[2][kRed];
  const int t = threadIdx.x;
  double a0 = 0, a1 = 0;
  for (int i = t; i < n; i += kRed) {
    if (found[i] <= 0) continue;
    a0 += 1.0;
    a1 += (double)d2[i];
  }
  red[0][t] = a0;
  red[1][t] = a1;
  __syncthreads();
  tree_sum<2>(red);
  if (t == 0) st->fitness = red[0][0] > 0 ? red[1][0] / red[0][0] : DBL_MAX;
}

}  // namespace loopk
}  // namespace lislam

using namespace lislam::loopk;

struct LoopState {
  lislam_map map;
  DBuf raw, tf, flag, sel, cnt, src, src0, tgt, nb, d2, found, st, tmp, ftf;
  IcpDev* host = nullptr;  // pinned
  LoopState() { (void)hipHostMalloc((void**)&host, sizeof(IcpDev)); }
  ~LoopState() { if (host) (void)hipHostFree(host); }
};

void lislam_free_map_scratch(void* p) {
  auto* s = static_cast<MapScratch*>(p);
  delete s->loop;
  delete s;
}

namespace {

// transform n staged points (device raw) by T (row-major 4x4 double) into tf[off..]
void lc_transform(lislam_ctx* c, const float4* raw, int n, const double* T, float4* out) {
  if (n <= 0) return;
  Mat34d m;
  for (int k = 0; k < 12; k++) m.m[k] = T[k];
  hipLaunchKernelGGL(k_lc_tf_d, dim3(blocks(n)), dim3(256), 0, stream_of(c), raw, n, m, out);
}

// removeNaN + CropBox + VoxelGrid of the n device points in ls.tf (in place through ls.sel) ->
// dst; returns the count (host)
int lc_prepare(lislam_ctx* c, LoopState& ls, int n, const lislam_icp_config* cfg, DBuf& dst, int* n_out) {
  hipStream_t st = stream_of(c);
  MapScratch& sc = ctx_scratch(c);
  *n_out = 0;
  MCHK(c, dst.reserve((size_t)std::max(n, 1) * sizeof(float4)));
  if (n == 0) return LISLAM_OK;
  MCHK(c, ls.flag.reserve((size_t)n));
  MCHK(c, ls.sel.reserve((size_t)n * sizeof(float4)));
  MCHK(c, ls.cnt.reserve(16));
  hipLaunchKernelGGL(k_lc_flags, dim3(blocks(n)), dim3(256), 0, st, ls.tf.as<float4>(), n, cfg->use_crop ? 1 : 0,
                     -cfg->crop_size, cfg->crop_size, ls.flag.as<uint8_t>());
  MCHK(c, ls.tmp.reserve(prims::select_temp_bytes(n)));
  MCHK(c, prims::select_flagged(ls.tmp.p, ls.tf.as<float4>(), ls.flag.as<uint8_t>(), ls.sel.as<float4>(), ls.cnt.as<int>(), n,
                                st));
  int m = 0;
  MCHK(c, hipMemcpyAsync(&m, ls.cnt.p, sizeof(int), hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  if (!cfg->use_downsample || m == 0) {
    if (m) MCHK(c, hipMemcpyAsync(dst.p, ls.sel.p, (size_t)m * sizeof(float4), hipMemcpyDeviceToDevice, st));
    *n_out = m;
    return LISLAM_OK;
  }
  MRC(voxel_grid_device(c, sc, ls.sel.as<float4>(), m, cfg->voxel_size, dst.as<float4>(), ls.cnt.as<int>() + 1));
  MCHK(c, hipMemcpyAsync(n_out, ls.cnt.as<int>() + 1, sizeof(int), hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  return LISLAM_OK;
}

}  // namespace

extern "C" {

int lislam_loop_icp(lislam_ctx* c, const lislam_icp_config* cfg, const float* cur, int32_t n_cur, const double* T_cur,
                    const float* hist, const int32_t* hist_counts, int32_t n_hist, const double* T_hist, double* T_icp,
                    double* T_cur2map, double* fitness, int32_t* info) {
  if (!c || !cfg || n_cur < 0 || (n_cur > 0 && !cur) || !T_cur || n_hist < 0 || (n_hist > 0 && (!hist_counts || !T_hist)))
    return LISLAM_ERR_ARG;
  if (cfg->use_downsample && !(cfg->voxel_size > 0)) return mfail(c, LISLAM_ERR_ARG, "lislam_loop_icp: voxel_size <= 0");
  int64_t n_h = 0;
  for (int h = 0; h < n_hist; h++) {
    if (hist_counts[h] < 0) return LISLAM_ERR_ARG;
    n_h += hist_counts[h];
  }
  if (n_h > 0 && !hist) return LISLAM_ERR_ARG;
  if (n_h > 0x3fffffff || n_cur > 0x3fffffff) return mfail(c, LISLAM_ERR_CAPACITY, "lislam_loop_icp: clouds too large");
  hipSetDevice(c->device);
  hipStream_t st = stream_of(c);
  MapScratch& sc = ctx_scratch(c);
  if (!sc.loop) {
    sc.loop = new LoopState();
    sc.loop->map.ctx = c;
  }
  LoopState& ls = *sc.loop;
  if (!ls.host) return mfail(c, LISLAM_ERR_DEVICE, "lislam_loop_icp: pinned allocation failed");
  int32_t inf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  double Ti[16], Tc[16], fit = DBL_MAX;
  for (int k = 0; k < 16; k++) { Ti[k] = (k % 5 == 0) ? 1.0 : 0.0; Tc[k] = T_cur[k]; }
  auto finish = [&]() {
    if (T_icp) std::memcpy(T_icp, Ti, sizeof(Ti));
    if (T_cur2map) std::memcpy(T_cur2map, Tc, sizeof(Tc));
    if (fitness) *fitness = fit;
    if (info) std::memcpy(info, inf, sizeof(inf));
    return LISLAM_OK;
  };
  // stage + transform: the current keyframe, then the history keyframes in order
  const int64_t ntot = std::max<int64_t>(n_cur, n_h);
  MCHK(c, ls.raw.reserve((size_t)std::max<int64_t>(ntot, 1) * sizeof(float4)));
  MCHK(c, ls.tf.reserve((size_t)std::max<int64_t>(ntot, 1) * sizeof(float4)));
  if (n_h == 0) {
    inf[0] = -1;
    return finish();
  }
  int ns = 0, nt = 0;
  if (n_cur) MCHK(c, hipMemcpyAsync(ls.raw.p, cur, (size_t)n_cur * 16, hipMemcpyDefault, st));
  lc_transform(c, ls.raw.as<float4>(), n_cur, T_cur, ls.tf.as<float4>());
  MRC(lc_prepare(c, ls, n_cur, cfg, ls.src0, &ns));
  MCHK(c, hipMemcpyAsync(ls.raw.p, hist, (size_t)n_h * 16, hipMemcpyDefault, st));
  for (int h = 0, off = 0; h < n_hist; off += hist_counts[h], h++)
    lc_transform(c, ls.raw.as<float4>() + off, hist_counts[h], T_hist + 16 * h, ls.tf.as<float4>() + off);
  MRC(lc_prepare(c, ls, (int)n_h, cfg, ls.tgt, &nt));
  inf[4] = ns;
  inf[5] = nt;
  if (ns <= 10 || nt <= 10) {
    inf[0] = -2;
    return finish();
  }
  // target map (ids = target index)
  lislam_map& m = ls.map;
  m.cell = std::max(1.0f, cfg->use_downsample ? 2.0f * cfg->voxel_size : 1.0f);
  m.ds = m.cell;
  MCHK(c, m.tmp.reserve((size_t)nt * sizeof(float4)));
  hipLaunchKernelGGL(k_lc_ids, dim3(blocks(nt)), dim3(256), 0, st, ls.tgt.as<float4>(), nt, m.tmp.as<float4>());
  MRC(rebuild(&m, nt));
  // ICP state
  MCHK(c, ls.src.reserve((size_t)ns * sizeof(float4)));
  MCHK(c, ls.ftf.reserve((size_t)ns * sizeof(float4)));
  MCHK(c, ls.nb.reserve((size_t)ns * sizeof(float4)));
  MCHK(c, ls.d2.reserve((size_t)ns * 4));
  MCHK(c, ls.found.reserve((size_t)ns * 4));
  MCHK(c, ls.st.reserve(sizeof(IcpDev)));
  MCHK(c, hipMemcpyAsync(ls.src.p, ls.src0.p, (size_t)ns * sizeof(float4), hipMemcpyDeviceToDevice, st));
  IcpDev* h = ls.host;
  std::memset(h, 0, sizeof(IcpDev));
  for (int k = 0; k < 16; k++) h->T[k] = h->F[k] = (k % 5 == 0) ? 1.f : 0.f;
  h->prev_mse = DBL_MAX;
  h->nq = ns;
  IcpDev* d = ls.st.as<IcpDev>();
  MCHK(c, hipMemcpyAsync(d, h, sizeof(IcpDev), hipMemcpyHostToDevice, st));
  IcpParams P;
  P.max_iter = cfg->max_iterations;
  P.rot_thr = 1.0 - cfg->transformation_epsilon;
  P.trans_thr = cfg->transformation_epsilon;
  P.mse_abs = 1e-12;
  P.mse_rel = cfg->euclidean_fitness_epsilon;
  const float md2 = cfg->max_correspondence_distance * cfg->max_correspondence_distance;
  const int cap = std::max(cfg->max_iterations, 1);
  constexpr int kChunk = 6;
  for (int it0 = 0; it0 < cap; it0 += kChunk) {
    for (int j = 0; j < kChunk && it0 + j < cap; j++) {
      MRC(knn_device(&m, ls.src.as<float>(), 4, &d->nq, ns, nullptr, 1, md2, ls.nb.as<float4>(), ls.d2.as<float>(),
                     ls.found.as<int>()));
      {
        TimedScope ts(c, kT_icp_step);
        hipLaunchKernelGGL(k_lc_step, dim3(1), dim3(kRed), 0, st, d, ls.src.as<float4>(), ls.nb.as<float4>(),
                           ls.d2.as<float>(), ls.found.as<int>(), ns, P);
      }
      TimedScope ts(c, kT_icp_apply);
      hipLaunchKernelGGL(k_lc_apply, dim3(blocks(ns)), dim3(256), 0, st, d, ls.src.as<float4>(), ns);
    }
    MCHK(c, hipMemcpyAsync(h, d, sizeof(IcpDev), hipMemcpyDeviceToHost, st));
    MCHK(c, hipStreamSynchronize(st));
    if (h->done) break;
  }
  if (!h->done) return mfail(c, LISLAM_ERR_STATE, "lislam_loop_icp: iteration loop did not terminate");
  // fitness
  hipLaunchKernelGGL(k_lc_final_tf, dim3(blocks(ns)), dim3(256), 0, st, d, ls.src0.as<float4>(), ns, ls.ftf.as<float4>());
  MRC(knn_device(&m, ls.ftf.as<float>(), 4, nullptr, ns, nullptr, 1, mapk::kInf, ls.nb.as<float4>(), ls.d2.as<float>(),
                 ls.found.as<int>()));
  hipLaunchKernelGGL(k_lc_fitness, dim3(1), dim3(kRed), 0, st, d, ls.d2.as<float>(), ls.found.as<int>(), ns);
  MCHK(c, hipGetLastError());
  MCHK(c, hipMemcpyAsync(h, d, sizeof(IcpDev), hipMemcpyDeviceToHost, st));
  MCHK(c, hipStreamSynchronize(st));
  fit = h->fitness;
  inf[1] = (h->state >= 1 && h->state <= 4) ? 1 : 0;
  inf[2] = h->state;
  inf[3] = h->iter;
  inf[6] = h->ncorr;
  inf[0] = (inf[1] && fit <= cfg->fitness_threshold) ? 1 : 0;
  for (int k = 0; k < 16; k++) Ti[k] = h->F[k];
  for (int r = 0; r < 4; r++)
    for (int col = 0; col < 4; col++)
      Tc[4 * r + col] = ((Ti[4 * r] * T_cur[col] + Ti[4 * r + 1] * T_cur[4 + col]) + Ti[4 * r + 2] * T_cur[8 + col]) +
                        Ti[4 * r + 3] * T_cur[12 + col];
  return finish();
}

}  // extern "C"

// ================================================================== odometry fusion
// odomHandler's callback (src/odom_handler_node.cpp:44-132): per synchronized pair both poses
// become 4x4 (Quaterniond::toRotationMatrix, :65-67, :83-85); the first pair sets prev and
// odom_cur = intensity (:88-95); afterwards odom_cur *= prev.inverse() * cur of the A-LOAM pose
// when the intensity tracker skipped the frame ("/odom_skip", intensity_feature_tracker.cpp:
// 722-730, 861-866), else of the intensity pose (:98-107); prev = cur; published as
// Quaterniond(rot_cur), t_cur (:113-128).  A sequential chain of ~250 flops per pair: one lane
// walks the n pairs of a call, the state stays on the device between calls.  Rigid inverse
// [R^T, -R^T t]; 4x4 products sum k = 0..3 left to right (oracle/oracle_fuse.cpp, same order).
namespace lislam {
namespace fusek {

__device__ void to_mat(const double* p, double* M) {
  const double x = p[0], y = p[1], z = p[2], w = p[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x, tyy = ty * y,
               tyz = tz * y, tzz = tz * z;
  const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
                       txz - twy, tyz + twx, 1 - (txx + tyy)};
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) M[4 * r + c] = R[3 * r + c];
    M[4 * r + 3] = p[4 + r];
  }
  M[12] = M[13] = M[14] = 0;
  M[15] = 1;
}

__device__ void inv_rigid(const double* M, double* I) {
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) I[4 * r + c] = M[4 * c + r];
    I[4 * r + 3] = -((M[r] * M[3] + M[4 + r] * M[7]) + M[8 + r] * M[11]);
  }
  I[12] = I[13] = I[14] = 0;
  I[15] = 1;
}

__device__ void mul(const double* A, const double* B, double* C) {
  double T[16];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++)
      T[4 * r + c] = ((A[4 * r] * B[c] + A[4 * r + 1] * B[4 + c]) + A[4 * r + 2] * B[8 + c]) + A[4 * r + 3] * B[12 + c];
  for (int k = 0; k < 16; k++) C[k] = T[k];
}

// Quaterniond(Matrix3d) (Eigen: trace branch / largest diagonal) + translation
__device__ void to_pose(const double* M, double* out) {
  double q[4];
  double t = (M[0] + M[5]) + M[10];
  if (t > 0) {
    t = sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (M[9] - M[6]) * t;
    q[1] = (M[2] - M[8]) * t;
    q[2] = (M[4] - M[1]) * t;
  } else {
    int i = 0;
    if (M[5] > M[0]) i = 1;
    if (M[10] > M[5 * i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = sqrt(((M[5 * i] - M[5 * j]) - M[5 * k]) + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (M[4 * k + j] - M[4 * j + k]) * t;
    q[j] = (M[4 * j + i] + M[4 * i + j]) * t;
    q[k] = (M[4 * k + i] + M[4 * i + k]) * t;
  }
  for (int e = 0; e < 4; e++) out[e] = q[e];
  out[4] = M[3];
  out[5] = M[7];
  out[6] = M[11];
}

// state[49] = prev A-LOAM, prev intensity, odom_cur (4x4 each), initialised flag
__global__ void k_fuse(double* state, const double* aloam, const double* intensity, const int* skip, int n, double* fused) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double pa[16], pi[16], cur[16];
  for (int k = 0; k < 16; k++) { pa[k] = state[k]; pi[k] = state[16 + k]; cur[k] = state[32 + k]; }
  bool init = state[48] != 0;
  for (int f = 0; f < n; f++) {
    double A[16], I[16];
    to_mat(aloam + 7 * f, A);
    to_mat(intensity + 7 * f, I);
    if (!init) {
      for (int k = 0; k < 16; k++) { pa[k] = A[k]; pi[k] = I[k]; cur[k] = I[k]; }
      init = true;
    } else {
      double inv[16], d[16];
      if (skip[f]) {
        inv_rigid(pa, inv);
        mul(inv, A, d);
      } else {
        inv_rigid(pi, inv);
        mul(inv, I, d);
      }
      mul(cur, d, cur);
      for (int k = 0; k < 16; k++) { pa[k] = A[k]; pi[k] = I[k]; }
    }
    to_pose(cur, fused + 7 * f);
  }
  for (int k = 0; k < 16; k++) { state[k] = pa[k]; state[16 + k] = pi[k]; state[32 + k] = cur[k]; }
  state[48] = init ? 1.0 : 0.0;
}

}  // namespace fusek
}  // namespace lislam

struct lislam_odom_fuser {
  lislam_ctx* ctx = nullptr;
  DBuf state, io;
};

extern "C" {

int lislam_odom_fuser_create(lislam_ctx* c, lislam_odom_fuser** out) {
  if (!c || !out) return LISLAM_ERR_ARG;
  *out = nullptr;
  hipSetDevice(c->device);
  auto* f = new lislam_odom_fuser();
  f->ctx = c;
  if (f->state.reserve(49 * 8) != hipSuccess || hipMemsetAsync(f->state.p, 0, 49 * 8, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess) {
    delete f;
    return mfail(c, LISLAM_ERR_DEVICE, "lislam_odom_fuser_create: allocation failed");
  }
  *out = f;
  return LISLAM_OK;
}

int lislam_odom_fuser_destroy(lislam_odom_fuser* f) {
  if (!f) return LISLAM_OK;
  hipSetDevice(f->ctx->device);
  (void)hipStreamSynchronize(f->ctx->stream);
  delete f;
  return LISLAM_OK;
}

int lislam_odom_fuse(lislam_odom_fuser* f, const double* aloam, const double* intensity, const int32_t* skip, int32_t n,
                     double* fused) {
  if (!f || n < 0 || (n > 0 && (!aloam || !intensity || !skip || !fused))) return LISLAM_ERR_ARG;
  if (n == 0) return LISLAM_OK;
  lislam_ctx* c = f->ctx;
  hipSetDevice(c->device);
  hipStream_t st = c->stream;
  const size_t pb = (size_t)n * 7 * 8;
  MCHK(c, f->io.reserve(3 * pb + (size_t)n * 4));
  char* base = f->io.as<char>();
  double* da = reinterpret_cast<double*>(base);
  double* di = reinterpret_cast<double*>(base + pb);
  double* dout = reinterpret_cast<double*>(base + 2 * pb);
  int* ds = reinterpret_cast<int*>(base + 3 * pb);
  MCHK(c, hipMemcpyAsync(da, aloam, pb, hipMemcpyDefault, st));
  MCHK(c, hipMemcpyAsync(di, intensity, pb, hipMemcpyDefault, st));
  MCHK(c, hipMemcpyAsync(ds, skip, (size_t)n * 4, hipMemcpyDefault, st));
  {
    TimedScope ts(c, kT_fuse);
    hipLaunchKernelGGL(lislam::fusek::k_fuse, dim3(1), dim3(64), 0, st, f->state.as<double>(), da, di, ds, n, dout);
  }
  MCHK(c, hipGetLastError());
  MCHK(c, hipMemcpyAsync(fused, dout, pb, hipMemcpyDefault, st));
  MCHK(c, hipStreamSynchronize(st));
  return LISLAM_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------ primitives check
// Host-array entry points of the map path's primitives (lislam_prims.hpp) for the GPU tests
// (tests/test_gpu_prims.py): each copies in, runs the primitive on the default stream, copies out.
extern "C" {

int lislam_debug_sort_pairs(const void* keys, const int32_t* vals, int32_t n, int32_t key_bits, void* keys_out,
                            int32_t* vals_out) {
  if (n < 0 || (key_bits != 32 && key_bits != 64)) return LISLAM_ERR_ARG;
  const size_t kb = (size_t)std::max(n, 1) * (key_bits / 8), vb = (size_t)std::max(n, 1) * 4;
  void *ki = nullptr, *ko = nullptr, *vi = nullptr, *vo = nullptr, *tmp = nullptr;
  int rc = LISLAM_ERR_DEVICE;
  if (hipMalloc(&ki, kb) == hipSuccess && hipMalloc(&ko, kb) == hipSuccess && hipMalloc(&vi, vb) == hipSuccess &&
      hipMalloc(&vo, vb) == hipSuccess && hipMalloc(&tmp, prims::sort_temp_bytes(n)) == hipSuccess &&
      hipMemcpy(ki, keys, kb, hipMemcpyHostToDevice) == hipSuccess &&
      hipMemcpy(vi, vals, vb, hipMemcpyHostToDevice) == hipSuccess) {
    const hipError_t e = key_bits == 64
        ? prims::sort_pairs<uint64_t>(tmp, (uint64_t*)ki, (uint64_t*)ko, (int*)vi, (int*)vo, n, 64, nullptr)
        : prims::sort_pairs<uint32_t>(tmp, (uint32_t*)ki, (uint32_t*)ko, (int*)vi, (int*)vo, n, 32, nullptr);
    if (e == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
        hipMemcpy(keys_out, ko, (size_t)n * (key_bits / 8), hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(vals_out, vo, (size_t)n * 4, hipMemcpyDeviceToHost) == hipSuccess)
      rc = LISLAM_OK;
  }
  for (void* p : {ki, ko, vi, vo, tmp}) if (p) (void)hipFree(p);
  return rc;
}

int lislam_debug_select_scan(const uint8_t* flags, const int32_t* vals, int32_t n, int32_t* selected, int32_t* count,
                             int32_t* exclusive) {
  if (n < 0) return LISLAM_ERR_ARG;
  const size_t nb = (size_t)std::max(n, 1);
  void *f = nullptr, *v = nullptr, *o = nullptr, *x = nullptr, *cnt = nullptr, *tmp = nullptr;
  int rc = LISLAM_ERR_DEVICE;
  if (hipMalloc(&f, nb) == hipSuccess && hipMalloc(&v, nb * 4) == hipSuccess && hipMalloc(&o, nb * 4) == hipSuccess &&
      hipMalloc(&x, nb * 4) == hipSuccess && hipMalloc(&cnt, 16) == hipSuccess &&
      hipMalloc(&tmp, std::max(prims::select_temp_bytes(n), prims::exclusive_sum_temp_bytes(n))) == hipSuccess &&
      hipMemcpy(f, flags, nb, hipMemcpyHostToDevice) == hipSuccess &&
      hipMemcpy(v, vals, nb * 4, hipMemcpyHostToDevice) == hipSuccess) {
    hipError_t e = prims::select_flagged(tmp, (const int*)v, (const uint8_t*)f, (int*)o, (int*)cnt, n, nullptr);
    if (e == hipSuccess) e = prims::exclusive_sum(tmp, (const int*)v, (int*)x, n, nullptr);
    int c = 0;
    if (e == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
        hipMemcpy(&c, cnt, 4, hipMemcpyDeviceToHost) == hipSuccess && c >= 0 && c <= n &&
        hipMemcpy(selected, o, (size_t)c * 4, hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(exclusive, x, (size_t)n * 4, hipMemcpyDeviceToHost) == hipSuccess) {
      *count = c;
      rc = LISLAM_OK;
    }
  }
  for (void* p : {f, v, o, x, cnt, tmp}) if (p) (void)hipFree(p);
  return rc;
}

}  // extern "C"
