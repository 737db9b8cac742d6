// lislam scan-to-scan odometry on gfx950 (a12..a18 of SURVEY.md §8(a)), forced geometric mode.
//
// Work decomposition.  A batch of S scans is split into chains; chain c is a fresh laserOdometry
// node over scans [c*L, min(c*L + L, S-1)] (laserOdometry.cpp:382-389) that carries
// para_q/para_t from pair to pair as the initial guess (:130-135) and accumulates the pose
// (:716-717).  The serial dependency is only along a chain, so every pair of every chain at the
// same position r ("round") runs together, as two phases per outer pass (:417):
//   k_odom_assoc  one thread per query of every chain: TransformToStart (:147-172), exact 1-NN
//                 in the previous less-sharp / less-flat cloud (KdTreeFLANN :452/:574) and the
//                 scan-line searches (:467-520, :589-646), both pruned by chunk / super-chunk
//                 AABBs of the target cloud (k_target_index) without changing any result: the
//                 float lower bound of a box never exceeds the float distance of a point inside
//                 it (monotone rounding), and boxes are skipped only when that bound is >= the
//                 current best (ties keep the reference's visit order).
//   k_odom_lm     one workgroup per chain: ceres::Solve(DENSE_QR, max 4 it) restated as a device
//                 trust-region Levenberg-Marquardt (Ceres 1.14 defaults); every evaluation is one
//                 fp64 pass over the residual blocks producing cost, J^T J and J^T r of the
//                 Huber-corrected LidarEdgeFactor / LidarPlaneFactor, reduced across the
//                 workgroup; thread 0 runs the 6x6 step logic.
#include <hip/hip_runtime.h>

#include "lislam_device.hpp"
#include "lislam_factors.hpp"
#include "lislam_internal.hpp"

namespace lislam {

constexpr int kAssocThreads = 256;
constexpr int kLmThreads = 512;
constexpr int kLmWaves = kLmThreads / 64;
constexpr double kDistSq = 25.0;   // DISTANCE_SQ_THRESHOLD (laserOdometry.cpp:89)
constexpr double kNearby = 2.5;    // NEARBY_SCAN (:90)

// ------------------------------------------------------------------ target index
// Per feature cloud (less-sharp / less-flat of every scan), one 1024-thread workgroup:
//   1. chunk / super-chunk AABBs + scan-line label ranges in the cloud's own order;
//   2. a z-order (Morton) permutation on a cubic grid over the cloud's AABB, sorted as
//      (code, index) keys by a bitonic sort in LDS (global scratch beyond kSortCap keys), and the
//      chunk / super-chunk AABBs of the permuted cloud, which are spatially compact.
constexpr int kIdxThreads = 1024;
constexpr int kSortCap = 16384;  // keys sorted in LDS (128 KiB)

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every third bit
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

__device__ __forceinline__ void stg4(float4* p, float4 v) {
  f4v w = {v.x, v.y, v.z, v.w};
  *(gf4v_mut*)p = w;
}

__device__ __forceinline__ void chunk_boxes(const float4* pts, int n, bool label_from_w, float4* chunk, float4* super) {
  const int nch = (n + kChunk - 1) / kChunk;
  for (int c = threadIdx.x; c < nch; c += kIdxThreads) {
    float4 lo = make_float4(3.4e38f, 3.4e38f, 3.4e38f, 1e9f), hi = make_float4(-3.4e38f, -3.4e38f, -3.4e38f, -1e9f);
    for (int j = c * kChunk; j < min(n, c * kChunk + kChunk); j++) {
      const float4 p = ldg(pts + j);
      const float l = label_from_w ? (float)int(p.w) : 0.f;
      lo.x = fminf(lo.x, p.x); lo.y = fminf(lo.y, p.y); lo.z = fminf(lo.z, p.z); lo.w = fminf(lo.w, l);
      hi.x = fmaxf(hi.x, p.x); hi.y = fmaxf(hi.y, p.y); hi.z = fmaxf(hi.z, p.z); hi.w = fmaxf(hi.w, l);
    }
    stg4(chunk + 2 * c, lo);
    stg4(chunk + 2 * c + 1, hi);
  }
  __syncthreads();
  const int nsu = (nch + kChunk - 1) / kChunk;
  for (int c = threadIdx.x; c < nsu; c += kIdxThreads) {
    float4 lo = make_float4(3.4e38f, 3.4e38f, 3.4e38f, 1e9f), hi = make_float4(-3.4e38f, -3.4e38f, -3.4e38f, -1e9f);
    for (int k = c * kChunk; k < min(nch, c * kChunk + kChunk); k++) {
      const float4 l = ldg(chunk + 2 * k), h = ldg(chunk + 2 * k + 1);
      lo.x = fminf(lo.x, l.x); lo.y = fminf(lo.y, l.y); lo.z = fminf(lo.z, l.z); lo.w = fminf(lo.w, l.w);
      hi.x = fmaxf(hi.x, h.x); hi.y = fmaxf(hi.y, h.y); hi.z = fmaxf(hi.z, h.z); hi.w = fmaxf(hi.w, h.w);
    }
    stg4(super + 2 * c, lo);
    stg4(super + 2 * c + 1, hi);
  }
  __syncthreads();
}

template <typename KeyPtr>
__device__ __forceinline__ void block_bitonic(KeyPtr keys, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += kIdxThreads) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t x = keys[i], y = keys[ixj];
          if ((x > y) == ((i & k) == 0)) { keys[i] = y; keys[ixj] = x; }
        }
      }
      __syncthreads();
    }
  }
}

typedef __attribute__((address_space(1))) uint64_t gu64;

// which_map: blockIdx.x -> (scan, cloud) for the launch (0 less-sharp, 1 less-flat, 2 sharp, 3 flat)
__global__ __launch_bounds__(kIdxThreads) void k_target_index(OdomArgs a, int per_scan, int w0, int w1, int w2, int lds_keys) {
  extern __shared__ __attribute__((aligned(16))) uint64_t skeys[];
  __shared__ float red[6][kIdxThreads / 64];
  const int s = blockIdx.x / per_scan, wi = blockIdx.x % per_scan;
  const int which = wi == 0 ? w0 : wi == 1 ? w1 : w2;
  const bool query = which >= 2;
  const TargetIndex& ix = (which & 1) ? a.idx_lf : a.idx_ls;
  const float4* pts = reinterpret_cast<const float4*>(
      which == 0 ? a.less_sharp + (size_t)s * a.cap_less_sharp : which == 1 ? a.less_flat + (size_t)s * a.N
      : which == 2 ? a.sharp + (size_t)s * a.cap_sharp : a.flat + (size_t)s * a.cap_flat);
  const int n = a.n_feat[s * 4 + (which == 0 ? 1 : which == 1 ? 3 : which == 2 ? 0 : 2)];
  if (!query) chunk_boxes(pts, n, true, ix.chunk + (size_t)s * ix.nchunk * 2, ix.super + (size_t)s * ix.nsuper * 2);
  if (n == 0) return;
  // cloud AABB
  float mn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, mx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
  for (int j = threadIdx.x; j < n; j += kIdxThreads) {
    const float4 p = ldg(pts + j);
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  for (int d = 0; d < 3; d++)
    for (int o = 32; o > 0; o >>= 1) {
      mn[d] = fminf(mn[d], __shfl_xor(mn[d], o));
      mx[d] = fmaxf(mx[d], __shfl_xor(mx[d], o));
    }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0)
    for (int d = 0; d < 3; d++) { red[d][wave] = mn[d]; red[3 + d][wave] = mx[d]; }
  __syncthreads();
  for (int d = 0; d < 3; d++) {
    mn[d] = red[d][0]; mx[d] = red[3 + d][0];
    for (int w = 1; w < kIdxThreads / 64; w++) { mn[d] = fminf(mn[d], red[d][w]); mx[d] = fmaxf(mx[d], red[3 + d][w]); }
  }
  const float ext = fmaxf(fmaxf(mx[0] - mn[0], mx[1] - mn[1]), fmaxf(mx[2] - mn[2], 1e-6f));
  const float inv = 1023.0f / ext;  // cubic cells
  int P = 64;
  while (P < n) P <<= 1;
  const bool in_lds = P <= lds_keys;
  gu64* gkeys = (gu64*)(ix.keys + (size_t)s * 2 * ix.cap);
  for (int j = threadIdx.x; j < P; j += kIdxThreads) {
    uint64_t key = ~0ull;
    if (j < n) {
      const float4 p = ldg(pts + j);
      const uint32_t qx = (uint32_t)fminf(fmaxf((p.x - mn[0]) * inv, 0.f), 1023.f);
      const uint32_t qy = (uint32_t)fminf(fmaxf((p.y - mn[1]) * inv, 0.f), 1023.f);
      const uint32_t qz = (uint32_t)fminf(fmaxf((p.z - mn[2]) * inv, 0.f), 1023.f);
      const uint32_t code = spread10(qx) | (spread10(qy) << 1) | (spread10(qz) << 2);
      key = ((uint64_t)code << 32) | (uint32_t)j;
    }
    if (in_lds) skeys[j] = key;
    else gkeys[j] = key;
  }
  __syncthreads();
  if (in_lds) block_bitonic(skeys, P);
  else block_bitonic(gkeys, P);
  if (query) {  // association threads take their queries in this order (spatially coherent waves)
    int* perm = which == 2 ? a.qperm_sharp + (size_t)s * a.cap_sharp : a.qperm_flat + (size_t)s * a.cap_flat;
    for (int j = threadIdx.x; j < n; j += kIdxThreads) perm[j] = (int)(uint32_t)(in_lds ? skeys[j] : gkeys[j]);
    return;
  }
  float4* sorted = ix.sorted + (size_t)s * ix.cap;
  for (int j = threadIdx.x; j < n; j += kIdxThreads) {
    const uint32_t o = (uint32_t)(in_lds ? skeys[j] : gkeys[j]);
    const float4 p = ldg(pts + o);
    stg4(sorted + j, make_float4(p.x, p.y, p.z, __int_as_float((int)o)));
  }
  __syncthreads();
  chunk_boxes(sorted, n, false, ix.nn_chunk + (size_t)s * ix.nchunk * 2, ix.nn_super + (size_t)s * ix.nsuper * 2);
}

// ------------------------------------------------------------------ association helpers
__device__ __forceinline__ P4 transform_to_start(const P4& pi, const double* x) {
  const DQ q{x[0], x[1], x[2], x[3]};
  const D3 u = qrot(q, D3{(double)pi.x, (double)pi.y, (double)pi.z}) + D3{1.0 * x[4], 1.0 * x[5], 1.0 * x[6]};
  return P4{(float)u.x, (float)u.y, (float)u.z, pi.i};
}

// FLANN L2_Simple: diff = q - p accumulated in float (== the line-search distance of :478)
__device__ __forceinline__ float d2f(const P4& q, const P4& p) {
  const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
  return dx * dx + dy * dy + dz * dz;
}

// float lower bound of d2f(q, p) over every p in the box (monotone rounding => never above)
__device__ __forceinline__ float box_lb(const float4& lo, const float4& hi, const P4& q) {
  const float dx = fmaxf(fmaxf(lo.x - q.x, q.x - hi.x), 0.f);
  const float dy = fmaxf(fmaxf(lo.y - q.y, q.y - hi.y), 0.f);
  const float dz = fmaxf(fmaxf(lo.z - q.z, q.z - hi.z), 0.f);
  return dx * dx + dy * dy + dz * dz;
}

// The 16 points of chunk c, loaded with independent loads (clamped to the cloud) so that a whole
// chunk is in flight at once; the caller masks indices >= n.
__device__ __forceinline__ void load_chunk(const P4* tgt, int c, int n, P4 (&p)[kChunk]) {
#pragma unroll
  for (int k = 0; k < kChunk; k++) p[k] = ld4(tgt + min(c * kChunk + k, n - 1));
}

// Chunk / super-chunk metadata, either staged in LDS (kLds) or read from global memory; the
// address space is a template parameter so every access compiles to ds_read / global_load.
template <bool kLds>
struct MetaT {
  const float4* chunk_p;
  const float4* super_p;
  __device__ __forceinline__ float4 chunk(int i) const {
    if constexpr (kLds) return lds4(chunk_p + i);
    else return ldg(chunk_p + i);
  }
  __device__ __forceinline__ float4 super(int i) const {
    if constexpr (kLds) return lds4(super_p + i);
    else return ldg(super_p + i);
  }
};

// 1-NN candidates of chunk c of the Morton-ordered cloud: lexicographic (distance, original index).
__device__ __forceinline__ void nn_chunk(const P4* sorted, int c, int n, const P4& q, float& best, int& bi) {
  P4 p[kChunk];
  load_chunk(sorted, c, n, p);
#pragma unroll
  for (int k = 0; k < kChunk; k++) {
    if (c * kChunk + k < n) {
      const int j = __float_as_int(p[k].i);
      const float d = d2f(q, p[k]);
      if (d < best || (d == best && j < bi)) { best = d; bi = j; }
    }
  }
}

template <class M>
__device__ __forceinline__ void nn_super(const P4* sorted, int n, const M& m, int u, const P4& q, float& best, int& bi) {
  const int nch = (n + kChunk - 1) / kChunk;
  for (int c = u * kChunk; c < min(nch, u * kChunk + kChunk); c++) {
    if (box_lb(m.chunk(2 * c), m.chunk(2 * c + 1), q) > best) continue;
    nn_chunk(sorted, c, n, q, best, bi);
  }
}

// Exact 1-NN restricted to d < 25 (the reference discards farther neighbours, :455/:577) over the
// Morton-ordered copy: the super-chunk nearest the query first (a tight bound), then every other
// super-chunk / chunk whose box bound does not exceed the best distance.  Returns the
// lexicographically smallest (float distance, original index), or -1.
template <class M>
__device__ __forceinline__ int nn_search(const P4* sorted, int n, const M& m, const P4& q) {
  float best = 25.0f;
  int bi = -1;
  const int nsu = ((n + kChunk - 1) / kChunk + kChunk - 1) / kChunk;
  int u0 = -1;
  float lb0 = 3.4e38f;
  for (int u = 0; u < nsu; u++) {
    const float lb = box_lb(m.super(2 * u), m.super(2 * u + 1), q);
    if (lb < lb0) { lb0 = lb; u0 = u; }
  }
  if (u0 < 0 || lb0 > best) return -1;
  nn_super(sorted, n, m, u0, q, best, bi);
  for (int u = 0; u < nsu; u++) {
    if (u == u0 || box_lb(m.super(2 * u), m.super(2 * u + 1), q) > best) continue;
    nn_super(sorted, n, m, u, q, best, bi);
  }
  return bi;
}

__device__ __forceinline__ double line_d2(const P4& p, const P4& sel) {  // laserOdometry.cpp:478-483
  return (double)((p.x - sel.x) * (p.x - sel.x) + (p.y - sel.y) * (p.y - sel.y) + (p.z - sel.z) * (p.z - sel.z));
}

// Corner second point (laserOdometry.cpp:464-520): min over scanID in (cid, cid+2.5] going up,
// then [cid-2.5, cid) going down; strict '<', 'continue' / 'break' on int(intensity).  A chunk is
// skipped from its metadata only when that cannot change the outcome; otherwise its 16 points
// are loaded at once and walked in the reference's order.
template <class M>
__device__ __forceinline__ int corner_second(const P4* L, int n, const M& m, int closest, int cid, const P4& sel) {
  double best = kDistSq;
  int mi = -1;
  const double hiL = cid + kNearby, loL = cid - kNearby;
  bool stop = false;
  for (int c = (closest + 1) / kChunk; !stop && c * kChunk < n; c++) {  // up
    const int j0 = max(closest + 1, c * kChunk);
    if (j0 == c * kChunk) {
      const float4 lo = m.chunk(2 * c), hi = m.chunk(2 * c + 1);
      if ((double)(int)lo.w > hiL) break;                    // its first point breaks
      if (!((double)(int)hi.w > hiL)) {                      // no break inside
        if ((int)hi.w <= cid) continue;                      // every point 'continue's
        if ((double)box_lb(lo, hi, sel) >= best) continue;   // none can be closer
      }
    }
    P4 p[kChunk];
    load_chunk(L, c, n, p);
#pragma unroll
    for (int k = 0; k < kChunk; k++) {
      const int j = c * kChunk + k;
      if (stop || j < j0 || j >= n) continue;
      const int pid = int(p[k].i);
      if (pid <= cid) continue;
      if ((double)pid > hiL) { stop = true; continue; }
      const double d = line_d2(p[k], sel);
      if (d < best) { best = d; mi = j; }
    }
  }
  stop = false;
  for (int c = (closest - 1) / kChunk; !stop && closest >= 1 && c >= 0; c--) {  // down
    const int j0 = min(closest - 1, min(n, c * kChunk + kChunk) - 1);
    if (j0 == min(n, c * kChunk + kChunk) - 1) {
      const float4 lo = m.chunk(2 * c), hi = m.chunk(2 * c + 1);
      if ((double)(int)hi.w < loL) break;
      if (!((double)(int)lo.w < loL)) {
        if ((int)lo.w >= cid) continue;
        if ((double)box_lb(lo, hi, sel) >= best) continue;
      }
    }
    P4 p[kChunk];
    load_chunk(L, c, n, p);
#pragma unroll
    for (int k = kChunk - 1; k >= 0; k--) {
      const int j = c * kChunk + k;
      if (stop || j > j0) continue;
      const int pid = int(p[k].i);
      if (pid >= cid) continue;
      if ((double)pid < loL) { stop = true; continue; }
      const double d = line_d2(p[k], sel);
      if (d < best) { best = d; mi = j; }
    }
  }
  return mi;
}

// Surf second / third points (laserOdometry.cpp:586-646).
template <class M>
__device__ __forceinline__ void surf_second_third(const P4* L, int n, const M& m, int closest, int cid, const P4& sel, int* m2,
                                  int* m3) {
  double b2 = kDistSq, b3 = kDistSq;
  int i2 = -1, i3 = -1;
  const double hiL = cid + kNearby, loL = cid - kNearby;
  bool stop = false;
  for (int c = (closest + 1) / kChunk; !stop && c * kChunk < n; c++) {  // up
    const int j0 = max(closest + 1, c * kChunk);
    if (j0 == c * kChunk) {
      const float4 lo = m.chunk(2 * c), hi = m.chunk(2 * c + 1);
      if ((double)(int)lo.w > hiL) break;
      if (!((double)(int)hi.w > hiL)) {
        const double lb = box_lb(lo, hi, sel);
        const bool need2 = (int)lo.w <= cid && lb < b2;
        const bool need3 = (int)hi.w > cid && lb < b3;
        if (!need2 && !need3) continue;
      }
    }
    P4 p[kChunk];
    load_chunk(L, c, n, p);
#pragma unroll
    for (int k = 0; k < kChunk; k++) {
      const int j = c * kChunk + k;
      if (stop || j < j0 || j >= n) continue;
      const int pid = int(p[k].i);
      if ((double)pid > hiL) { stop = true; continue; }
      const double d = line_d2(p[k], sel);
      if (pid <= cid && d < b2) { b2 = d; i2 = j; }
      else if (pid > cid && d < b3) { b3 = d; i3 = j; }
    }
  }
  stop = false;
  for (int c = (closest - 1) / kChunk; !stop && closest >= 1 && c >= 0; c--) {  // down
    const int j0 = min(closest - 1, min(n, c * kChunk + kChunk) - 1);
    if (j0 == min(n, c * kChunk + kChunk) - 1) {
      const float4 lo = m.chunk(2 * c), hi = m.chunk(2 * c + 1);
      if ((double)(int)hi.w < loL) break;
      if (!((double)(int)lo.w < loL)) {
        const double lb = box_lb(lo, hi, sel);
        const bool need2 = (int)hi.w >= cid && lb < b2;
        const bool need3 = (int)lo.w < cid && lb < b3;
        if (!need2 && !need3) continue;
      }
    }
    P4 p[kChunk];
    load_chunk(L, c, n, p);
#pragma unroll
    for (int k = kChunk - 1; k >= 0; k--) {
      const int j = c * kChunk + k;
      if (stop || j > j0) continue;
      const int pid = int(p[k].i);
      if ((double)pid < loL) { stop = true; continue; }
      const double d = line_d2(p[k], sel);
      if (pid >= cid && d < b2) { b2 = d; i2 = j; }
      else if (pid < cid && d < b3) { b3 = d; i3 = j; }
    }
  }
  *m2 = i2;
  *m3 = i3;
}

__device__ __forceinline__ bool pair_of(const OdomArgs& a, int c, int r, int* k) {
  const int k0 = c * a.chain_len;
  const int k1 = min(k0 + a.chain_len, a.S - 1);
  *k = k0 + r + 1;
  return *k <= k1;
}

// ------------------------------------------------------------------ phase 1: association
// Grid: x = corner blocks (cap_sharp / 256) then surf blocks (cap_flat / 256), y = chain.  A
// block handles one query kind, so it stages only its target cloud's metadata in LDS.
constexpr int kMetaCap = 768;  // chunks per structure staged in LDS; larger clouds read global memory

struct AssocShared {
  float4 chunk[2 * kMetaCap];                // scan-line order
  float4 super[2 * (kMetaCap / kChunk)];
  float4 nn_chunk[2 * kMetaCap];             // Morton order
  float4 nn_super[2 * (kMetaCap / kChunk)];
};

template <bool kCorner, class M>
__device__ __forceinline__ void assoc_query(const OdomArgs& a, int c, int k, int q, const M& lm, const M& nm, const P4* L,
                            const P4* sorted, int nL, bool* found_out) {
  double x[7];
  const double* st = a.state + (size_t)c * 16;
  for (int e = 0; e < 7; e++) x[e] = st[e];
  double* blk = a.blk + (size_t)c * (a.cap_sharp + a.cap_flat) * 9;
  int* kind = a.blk_kind + (size_t)c * (a.cap_sharp + a.cap_flat);
  const P4 cur = kCorner ? ld4(a.sharp + (size_t)k * a.cap_sharp + q) : ld4(a.flat + (size_t)k * a.cap_flat + q);
  const P4 sel = transform_to_start(cur, x);
  const int closest = (a.dbg & 1) ? -1 : nn_search(sorted, nL, nm, sel);
  const int slot = kCorner ? q : a.cap_sharp + q;
  double* rec = blk + (size_t)slot * 9;
  bool found = false;
  if (closest >= 0 && !(a.dbg & 2)) {
    const P4 pa = ld4(L + closest);
    const int cid = int(pa.i);
    if (kCorner) {  // LidarEdgeFactor(curr, a, b)
      const int m2 = corner_second(L, nL, lm, closest, cid, sel);
      if (m2 >= 0) {
        const P4 pb = ld4(L + m2);
        rec[0] = cur.x; rec[1] = cur.y; rec[2] = cur.z; rec[3] = pa.x; rec[4] = pa.y; rec[5] = pa.z;
        rec[6] = pb.x; rec[7] = pb.y; rec[8] = pb.z;
        found = true;
      }
    } else {        // LidarPlaneFactor(curr, j, l, m)
      int m2, m3;
      surf_second_third(L, nL, lm, closest, cid, sel, &m2, &m3);
      if (m2 >= 0 && m3 >= 0) {
        const P4 pl = ld4(L + m2), pm = ld4(L + m3);
        const D3 j{pa.x, pa.y, pa.z};
        const D3 nrm = plane_normal(j, D3{pl.x, pl.y, pl.z}, D3{pm.x, pm.y, pm.z});
        rec[0] = cur.x; rec[1] = cur.y; rec[2] = cur.z; rec[3] = j.x; rec[4] = j.y; rec[5] = j.z;
        rec[6] = nrm.x; rec[7] = nrm.y; rec[8] = nrm.z;
        found = true;
      }
    }
  }
  kind[slot] = found ? (kCorner ? 0 : 1) : -1;
  *found_out = found;
}

__global__ __launch_bounds__(kAssocThreads) void k_odom_assoc(OdomArgs a, int r) {
  __shared__ AssocShared sh;
  const int c = blockIdx.y;
  int k;
  if (!pair_of(a, c, r, &k)) return;
  const int cb = (a.cap_sharp + kAssocThreads - 1) / kAssocThreads;
  const bool corner = (int)blockIdx.x < cb;
  const int t = (corner ? blockIdx.x : blockIdx.x - cb) * kAssocThreads + threadIdx.x;
  const int nq = a.n_feat[k * 4 + (corner ? 0 : 2)];
  if ((t - (int)threadIdx.x) >= nq) return;  // whole block past the queries
  const int q = t < nq ? (corner ? a.qperm_sharp[(size_t)k * a.cap_sharp + t] : a.qperm_flat[(size_t)k * a.cap_flat + t]) : nq;
  const TargetIndex& ix = corner ? a.idx_ls : a.idx_lf;
  const P4* L = corner ? a.less_sharp + (size_t)(k - 1) * a.cap_less_sharp : a.less_flat + (size_t)(k - 1) * a.N;
  const P4* sorted = reinterpret_cast<const P4*>(ix.sorted + (size_t)(k - 1) * ix.cap);
  const int nL = a.n_feat[(k - 1) * 4 + (corner ? 1 : 3)];
  const int nch = (nL + kChunk - 1) / kChunk, nsu = (nch + kChunk - 1) / kChunk;
  const size_t mo = (size_t)(k - 1) * ix.nchunk * 2, so = (size_t)(k - 1) * ix.nsuper * 2;
  const MetaT<false> glm{ix.chunk + mo, ix.super + so}, gnm{ix.nn_chunk + mo, ix.nn_super + so};
  const bool staged = nch <= kMetaCap;
  if (staged) {
    for (int e = threadIdx.x; e < 2 * nch; e += kAssocThreads) { sh.chunk[e] = glm.chunk(e); sh.nn_chunk[e] = gnm.chunk(e); }
    for (int e = threadIdx.x; e < 2 * nsu; e += kAssocThreads) { sh.super[e] = glm.super(e); sh.nn_super[e] = gnm.super(e); }
  }
  __syncthreads();
  bool found = false;
  if (t < nq) {
    if (staged) {
      const MetaT<true> lm{sh.chunk, sh.super}, nm{sh.nn_chunk, sh.nn_super};
      if (corner) assoc_query<true>(a, c, k, q, lm, nm, L, sorted, nL, &found);
      else assoc_query<false>(a, c, k, q, lm, nm, L, sorted, nL, &found);
    } else {
      if (corner) assoc_query<true>(a, c, k, q, glm, gnm, L, sorted, nL, &found);
      else assoc_query<false>(a, c, k, q, glm, gnm, L, sorted, nL, &found);
    }
  }
  // corner_correspondence / plane_correspondence (:562/:685), one atomic per wave
  const uint64_t mf = __ballot(found);
  if ((threadIdx.x & 63) == 0 && mf) atomicAdd(&a.counters[c * 2 + (corner ? 0 : 1)], __popcll(mf));
}

// ------------------------------------------------------------------ phase 2: LM solve
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

struct LmShared {
  double red[kLmWaves][28];
  double x[7];
  double acc[28];
  int flag;
};

// One evaluation at sh.x: cost, J^T J (upper, row-major), J^T r -> sh.acc
__device__ __forceinline__ void evaluate(LmShared& sh, const double* blk, const int* kind, int ns, int cap_sharp, int nf) {
  double acc[28];
#pragma unroll
  for (int e = 0; e < 28; e++) acc[e] = 0;
  const DQ q{sh.x[0], sh.x[1], sh.x[2], sh.x[3]};
  const D3 t{sh.x[4], sh.x[5], sh.x[6]};
  const double ha = 0.1;  // HuberLoss(0.1), laserOdometry.cpp:424
  const int total = ns + nf;
  for (int i = threadIdx.x; i < total; i += kLmThreads) {
    const int idx = i < ns ? i : cap_sharp + (i - ns);
    const int kd = kind[idx];
    if (kd < 0) continue;
    const double* r9 = blk + (size_t)idx * 9;
    const D3 c{r9[0], r9[1], r9[2]};
    if (kd == 0) {
      double res[3], J[3][6];
      edge_factor(q, t, c, D3{r9[3], r9[4], r9[5]}, D3{r9[6], r9[7], r9[8]}, res, J);
      const double sc = huber_scale(ha, res[0] * res[0] + res[1] * res[1] + res[2] * res[2], &acc[0]);
      for (int k = 0; k < 3; k++) {
        double Js[6];
        for (int cc = 0; cc < 6; cc++) Js[cc] = J[k][cc] * sc;
        accum_row(acc, Js, res[k] * sc);
      }
    } else {
      double res, J[6];
      plane_factor(q, t, c, D3{r9[3], r9[4], r9[5]}, D3{r9[6], r9[7], r9[8]}, &res, J);
      const double sc = huber_scale(ha, res * res, &acc[0]);
      for (int cc = 0; cc < 6; cc++) J[cc] *= sc;
      accum_row(acc, J, res * sc);
    }
  }
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
    for (int w = 0; w < kLmWaves; w++) v += sh.red[w][threadIdx.x];
    sh.acc[threadIdx.x] = v;
  }
  __syncthreads();
}

struct LM {
  double x[7], xc[7];
  double cost;
  double A[36], g[6];
  double scale[6], diag[6];
  double radius, dfac;
  bool reuse;
  int it, invalid, term;
};

__device__ __forceinline__ void unpack(const double* acc, double* cost, double* A, double* g) {
  *cost = acc[0];
  int e = 1;
  for (int i = 0; i < 6; i++)
    for (int j = i; j < 6; j++) { A[i * 6 + j] = acc[e]; A[j * 6 + i] = acc[e]; e++; }
  for (int i = 0; i < 6; i++) g[i] = acc[22 + i];
}

__device__ __forceinline__ void quat_plus(const double* x, const double* d, double* xp) {
  const double nd = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd > 0.0) {
    const double sdd = sin(nd) / nd;
    const DQ r = qmul(DQ{sdd * d[0], sdd * d[1], sdd * d[2], cos(nd)}, DQ{x[0], x[1], x[2], x[3]});
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
// system [J S; sqrt(diag/radius)] y = [r; 0]).
__device__ __forceinline__ bool lm_solve(const LM& s, double* y) {
  double M[36], b[6], L[36];
  for (int i = 0; i < 6; i++) {
    for (int j = 0; j < 6; j++) { M[i * 6 + j] = s.scale[i] * s.A[i * 6 + j] * s.scale[j]; L[i * 6 + j] = 0; }
    M[i * 6 + i] += s.diag[i] / s.radius;
    b[i] = s.scale[i] * s.g[i];
  }
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

// Next candidate into s.xc (TrustRegionMinimizer + LevenbergMarquardtStrategy); false = stop.
__device__ __forceinline__ bool lm_propose(LM& s, int max_it, double* mcc_out) {
  while (s.it < max_it) {
    s.it++;
    if (!s.reuse)
      for (int c = 0; c < 6; c++) s.diag[c] = fmin(fmax(s.scale[c] * s.scale[c] * s.A[c * 6 + c], 1e-6), 1e32);
    double y[6] = {0, 0, 0, 0, 0, 0};
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
    if (!ok || !(mcc > 0.0)) {  // invalid step: rejected-step radius update, solve again
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
  s.term = 0;  // NO_CONVERGENCE: max_num_iterations
  return false;
}

__global__ __launch_bounds__(kLmThreads) void k_odom_lm(OdomArgs a, int r, int outer) {
  __shared__ LmShared sh;
  const int c = blockIdx.x;
  int k;
  if (!pair_of(a, c, r, &k)) return;
  double* st = a.state + (size_t)c * 16;
  const int ns = a.n_feat[k * 4 + 0], nf = a.n_feat[k * 4 + 2];
  const double* blk = a.blk + (size_t)c * (a.cap_sharp + a.cap_flat) * 9;
  const int* kind = a.blk_kind + (size_t)c * (a.cap_sharp + a.cap_flat);
  const int nc = a.counters[c * 2 + 0], np = a.counters[c * 2 + 1];
  LM s;
  double mcc = 0;
  bool go = (nc + np) > 0;  // no residual blocks: Ceres leaves the parameters untouched
  if (go) {
    if (threadIdx.x == 0)
      for (int e = 0; e < 7; e++) sh.x[e] = st[e];
    __syncthreads();
    evaluate(sh, blk, kind, ns, a.cap_sharp, nf);
    if (threadIdx.x == 0) {
      for (int e = 0; e < 7; e++) s.x[e] = sh.x[e];
      unpack(sh.acc, &s.cost, s.A, s.g);
      for (int cc = 0; cc < 6; cc++) s.scale[cc] = 1.0 / (1.0 + sqrt(s.A[cc * 6 + cc]));  // jacobi scaling
      s.radius = 1e4; s.dfac = 2.0; s.reuse = false;
      s.it = 0; s.invalid = 0; s.term = 0;
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
    evaluate(sh, blk, kind, ns, a.cap_sharp, nf);  // cost + J^T J + J^T r at the candidate
    if (threadIdx.x == 0) {
      double ccost, cA[36], cg[6];
      unpack(sh.acc, &ccost, cA, cg);
      if (!isfinite(ccost)) ccost = 1.7976931348623157e308;
      bool cont = true;
      double xn = 0, sn = 0;
      for (int e = 0; e < 7; e++) { xn += s.x[e] * s.x[e]; sn += (s.x[e] - s.xc[e]) * (s.x[e] - s.xc[e]); }
      xn = sqrt(xn); sn = sqrt(sn);
      if (sn <= 1e-8 * (xn + 1e-8)) { s.term = 1; cont = false; }                      // parameter_tolerance
      else if (fabs(s.cost - ccost) <= 1e-6 * s.cost) { s.term = 1; cont = false; }   // function_tolerance
      else {
        const double rel = (s.cost - ccost) / mcc;
        if (rel > 1e-3) {  // min_relative_decrease: accept
          for (int e = 0; e < 7; e++) s.x[e] = s.xc[e];
          s.cost = ccost;
          for (int e = 0; e < 36; e++) s.A[e] = cA[e];
          for (int e = 0; e < 6; e++) s.g[e] = cg[e];
          const double t3 = 2.0 * rel - 1.0;
          s.radius = fmin(1e16, s.radius / fmax(1.0 / 3.0, 1.0 - t3 * t3 * t3));
          s.dfac = 2.0;
          s.reuse = false;
          if (grad_max_norm(s.x, s.g) <= 1e-10) { s.term = 1; cont = false; }       // gradient_tolerance
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
  if (threadIdx.x != 0) return;
  int* so = a.stats + (size_t)k * 8;
  so[outer * 2 + 0] = nc;
  so[outer * 2 + 1] = np;
  so[4 + outer] = (nc + np) > 0 ? s.it : 0;
  so[6 + outer] = (nc + np) > 0 ? s.term : 1;
  if ((nc + np) > 0)
    for (int e = 0; e < 7; e++) st[e] = s.x[e];
  a.counters[c * 2 + 0] = 0;
  a.counters[c * 2 + 1] = 0;
  if (outer == 1) {
    // t_w_curr = t_w_curr + q_w_curr * t_last_curr; q_w_curr = q_w_curr * q_last_curr
    DQ qw{st[7], st[8], st[9], st[10]};
    D3 tw{st[11], st[12], st[13]};
    tw = tw + qrot(qw, D3{st[4], st[5], st[6]});
    qw = qmul(qw, DQ{st[0], st[1], st[2], st[3]});
    st[7] = qw.x; st[8] = qw.y; st[9] = qw.z; st[10] = qw.w; st[11] = tw.x; st[12] = tw.y; st[13] = tw.z;
    double* op = a.para + (size_t)k * 7;
    double* ow = a.pose + (size_t)k * 7;
    for (int e = 0; e < 7; e++) { op[e] = st[e]; ow[e] = st[7 + e]; }
  }
}

__global__ void k_odom_init(OdomArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.n_chains) return;
  double* st = a.state + (size_t)c * 16;
  if (a.init_state) {
    for (int e = 0; e < 14; e++) st[e] = a.init_state[(size_t)c * 14 + e];
  } else {
    const double id[14] = {0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0};
    for (int e = 0; e < 14; e++) st[e] = id[e];
  }
  a.counters[c * 2 + 0] = 0;
  a.counters[c * 2 + 1] = 0;
  if (c == 0 && !a.init_state) {  // scan 0 of the batch: first frame, initialization only
    for (int e = 0; e < 7; e++) { a.para[e] = st[e]; a.pose[e] = st[7 + e]; }
    for (int e = 0; e < 8; e++) a.stats[e] = 0;
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

void launch_target_index(const OdomArgs& a, int n_scans, hipStream_t st) {
  static bool attr = false;
  if (!attr) {  // > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute((const void*)k_target_index, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kSortCap * sizeof(uint64_t));
    attr = true;
  }
  // less-flat clouds: 128 KiB of LDS keys; less-sharp + query clouds: 64 KiB (two workgroups per CU)
  hipLaunchKernelGGL(k_target_index, dim3(n_scans), dim3(kIdxThreads), kSortCap * sizeof(uint64_t), st, a, 1, 1, 1, 1,
                     kSortCap);
  hipLaunchKernelGGL(k_target_index, dim3(3 * n_scans), dim3(kIdxThreads), (kSortCap / 2) * sizeof(uint64_t), st, a,
                     3, 0, 2, 3, kSortCap / 2);
}

void launch_odometry(const OdomArgs& a, hipStream_t st, std::vector<hipEvent_t>* ev, hipEvent_t (*get_event)(void*),
                     void* owner) {
  if (a.n_chains <= 0) return;
  auto mark = [&]() {
    if (ev) {
      hipEvent_t e = get_event(owner);
      (void)hipEventRecord(e, st);
      ev->push_back(e);
    }
  };
  mark();
  hipLaunchKernelGGL(k_odom_init, dim3((a.n_chains + 63) / 64), dim3(64), 0, st, a);
  const int qblocks = (a.cap_sharp + kAssocThreads - 1) / kAssocThreads + (a.cap_flat + kAssocThreads - 1) / kAssocThreads;
  const int rounds = min(a.chain_len, a.S - 1);
  mark();
  for (int r = 0; r < rounds; r++) {
    for (int outer = 0; outer < 2; outer++) {
      hipLaunchKernelGGL(k_odom_assoc, dim3(qblocks, a.n_chains), dim3(kAssocThreads), 0, st, a, r);
      mark();
      hipLaunchKernelGGL(k_odom_lm, dim3(a.n_chains), dim3(kLmThreads), 0, st, a, r, outer);
      mark();
    }
  }
}

}  // namespace lislam
