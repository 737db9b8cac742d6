// lislam scan-to-scan odometry on gfx950 (a12..a18 of SURVEY.md §8(a)), forced geometric mode.
//
// Work decomposition.  A batch of S scans is split into chains; chain c is a fresh laserOdometry
// node over scans [c*L, min(c*L + L, S-1)] (laserOdometry.cpp:382-389) that carries
// para_q/para_t from pair to pair as the initial guess (:130-135) and accumulates the pose
// (:716-717).  The serial dependency is only along a chain, so every pair of every chain at the
// same position r ("round") runs together, as two phases per outer pass (:417):
//   association   per query: TransformToStart (:147-172), exact 1-NN in the previous less-sharp /
//                 less-flat cloud (KdTreeFLANN :452/:574) and the scan-line searches (:467-520,
//                 :589-646), both pruned by chunk / super-chunk AABBs of the target cloud
//                 (k_target_index) without changing any result: the float lower bound of a box
//                 never exceeds the float distance of a point inside it (monotone rounding), and
//                 boxes are skipped only when that bound is >= the current best (ties keep the
//                 reference's visit order).
//   solve         per chain: ceres::Solve(DENSE_QR, max 4 it) restated as a device trust-region
//                 Levenberg-Marquardt (Ceres 1.14 defaults); every evaluation is one fp64 pass
//                 over the residual blocks producing cost, J^T J and J^T r of the Huber-corrected
//                 LidarEdgeFactor / LidarPlaneFactor, reduced across the workgroup.
// Two schedules run them: the persistent chain engine (k_odom_chain, few long chains: every pass
// of every chain in one launch) and per-round launches (k_odom_assoc16 + k_odom_lm2, many short
// chains).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "lislam_device.hpp"
#include "lislam_factors.hpp"
#include "lislam_internal.hpp"
#include "lislam_lm.hpp"
#include "lislam_lm_wave.hpp"

namespace lislam {

// a value every lane holds alike (LDS broadcasts), as a scalar: branches on it stay uniform
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

constexpr double kDistSq = 25.0;   // DISTANCE_SQ_THRESHOLD (laserOdometry.cpp:89)
constexpr double kNearby = 2.5;    // NEARBY_SCAN (:90)

// ------------------------------------------------------------------ target index
// Per feature cloud (less-sharp / less-flat of every scan), one workgroup of kW waves:
//   1. chunk / super-chunk AABBs + scan-line label ranges in the cloud's own order;
//   2. a z-order (Morton) permutation on a cubic grid over the cloud's AABB — (code, index) keys
//      sorted by a workgroup bitonic network held in registers (16 keys per lane, index
//      i = 1024 w + 64 t + lane): stages j < 64 in-lane DPP / swizzle exchanges, j < 1024 slot
//      swaps, j >= 1024 through LDS in two halves; clouds beyond 1024 kW keys sort in global
//      scratch — and the chunk / super-chunk AABBs of the permuted cloud, which are spatially
//      compact.  The permutation only steers the search's pruning: every association result is
//      independent of it (exact distances, ties by original index).

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
  for (int c = threadIdx.x; c < nch; c += blockDim.x) {
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
  for (int c = threadIdx.x; c < nsu; c += blockDim.x) {
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

typedef __attribute__((address_space(1))) uint64_t gu64;

// Bitonic sort of P keys in global scratch (clouds larger than a workgroup's registers hold).
__device__ __forceinline__ void global_bitonic(gu64* keys, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
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

// Workgroup bitonic sort of the first P = 64 kK nw keys (nw active waves, a power of two; kK keys
// per lane, a multiple of 8); the other waves only join the barriers.  xch: kW * 8 * 64 keys of LDS.
template <int kW, int kK>
__device__ __forceinline__ void wg_bitonic(uint64_t (&key)[kK], int P, uint64_t* xch) {
  constexpr int kPer = 64 * kK;  // keys per wave
  const int w = threadIdx.x >> 6, lane = lane_id();
  const bool active = w * kPer < P;
  const int base = w * kPer;
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j >= kPer; j >>= 1) {  // partner wave w ^ (j / kPer), same slot and lane
      const int pw = w ^ (j / kPer);
      const bool up = (base & k) == 0, lower = (w & (j / kPer)) == 0;
#pragma unroll
      for (int h = 0; h < kK / 8; h++) {
        if (active)
#pragma unroll
          for (int t = 0; t < 8; t++) xch[(w * 8 + t) * 64 + lane] = key[h * 8 + t];
        __syncthreads();
        if (active)
#pragma unroll
          for (int t = 0; t < 8; t++) {
            const uint64_t x = key[h * 8 + t], y = xch[(pw * 8 + t) * 64 + lane];
            key[h * 8 + t] = (lower == up) ? (x < y ? x : y) : (x < y ? y : x);
          }
        __syncthreads();
      }
    }
    if (active) reg_bitonic_level<kK>(key, k, min(k >> 1, kPer / 2), base);
  }
}

// which: 0 less-sharp, 1 less-flat (targets), 2 sharp, 3 flat (queries: permutation only);
// blockIdx.x -> (scan, w0 / w1 / w2 of the launch).  kW waves of kK keys per lane (64 kK kW keys in
// registers).
#ifndef LISLAM_TI_WPE32
#define LISLAM_TI_WPE32 4  // waves per SIMD the 32-keys-per-lane build is compiled for (4: 128 VGPRs)
#endif
// (the body of workgroup `bid` of a launch; xch / red: the workgroup's LDS, kW * 8 * 64 / 6 * kW)
template <int kW, int kK>
__device__ __forceinline__ void target_index_body(const OdomArgs& a, int bid, int per_scan, int w0, int w1, int w2,
                                                  uint64_t* xch, float (*red)[kW]) {
  constexpr int kKeysPerLane = kK, kPer = 64 * kK;
  const int s = bid / per_scan, wi = bid % per_scan;
  const int which = wi == 0 ? w0 : wi == 1 ? w1 : w2;
  const bool query = which >= 2;
  const TargetIndex& ix = (which & 1) ? a.idx_lf : a.idx_ls;
  const float4* pts = reinterpret_cast<const float4*>(
      which == 0 ? a.less_sharp + (size_t)s * a.cap_less_sharp : which == 1 ? a.less_flat + (size_t)s * a.N
      : which == 2 ? a.sharp + (size_t)s * a.cap_sharp : a.flat + (size_t)s * a.cap_flat);
  const int n = a.n_feat[s * 4 + (which == 0 ? 1 : which == 1 ? 3 : which == 2 ? 0 : 2)];
  if (!query) chunk_boxes(pts, n, true, ix.chunk + (size_t)s * ix.nchunk * 2, ix.super + (size_t)s * ix.nsuper * 2);
  if (n == 0) return;
  // cloud AABB: from the super-chunk boxes just written (targets), from the points (queries)
  float mn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, mx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
  if (!query) {
    const float4* sb = ix.super + (size_t)s * ix.nsuper * 2;
    const int nsu = ((n + kChunk - 1) / kChunk + kChunk - 1) / kChunk;
    for (int u = threadIdx.x; u < nsu; u += 64 * kW) {
      const float4 l = ldg(sb + 2 * u), h = ldg(sb + 2 * u + 1);
      mn[0] = fminf(mn[0], l.x); mn[1] = fminf(mn[1], l.y); mn[2] = fminf(mn[2], l.z);
      mx[0] = fmaxf(mx[0], h.x); mx[1] = fmaxf(mx[1], h.y); mx[2] = fmaxf(mx[2], h.z);
    }
  } else {
    for (int j = threadIdx.x; j < n; j += 64 * kW) {
      const float4 p = ldg(pts + j);
      mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
      mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
    }
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
    for (int w = 1; w < kW; w++) { mn[d] = fminf(mn[d], red[d][w]); mx[d] = fmaxf(mx[d], red[3 + d][w]); }
  }
  const float ext = fmaxf(fmaxf(mx[0] - mn[0], mx[1] - mn[1]), fmaxf(mx[2] - mn[2], 1e-6f));
  const float inv = 1023.0f / ext;  // cubic cells
  auto key_of = [&](int j) -> uint64_t {
    if (j >= n) return ~0ull;
    const float4 p = ldg(pts + j);
    const uint32_t qx = (uint32_t)fminf(fmaxf((p.x - mn[0]) * inv, 0.f), 1023.f);
    const uint32_t qy = (uint32_t)fminf(fmaxf((p.y - mn[1]) * inv, 0.f), 1023.f);
    const uint32_t qz = (uint32_t)fminf(fmaxf((p.z - mn[2]) * inv, 0.f), 1023.f);
    const uint32_t code = spread10(qx) | (spread10(qy) << 1) | (spread10(qz) << 2);
    return ((uint64_t)code << 32) | (uint32_t)j;
  };
  int P = 1024;
  while (P < n) P <<= 1;
  uint64_t key[kKeysPerLane];
  const bool in_regs = P <= kPer * kW;
  gu64* gkeys = (gu64*)(ix.keys + (size_t)s * 2 * ix.cap);
  if (in_regs) {
#pragma unroll
    for (int t = 0; t < kKeysPerLane; t++) key[t] = key_of(wave * kPer + t * 64 + lane);
    wg_bitonic<kW, kK>(key, P, xch);
  } else {
    for (int j = threadIdx.x; j < P; j += 64 * kW) gkeys[j] = key_of(j);
    __syncthreads();
    global_bitonic(gkeys, P);
  }
  // sorted position i -> original index
  auto emit = [&](auto&& f) {
    if (in_regs) {
#pragma unroll
      for (int t = 0; t < kKeysPerLane; t++) {
        const int i = wave * kPer + t * 64 + lane;
        if (i < n) f(i, (int)(uint32_t)key[t]);
      }
    } else {
      for (int i = threadIdx.x; i < n; i += 64 * kW) f(i, (int)(uint32_t)gkeys[i]);
    }
  };
  if (query) {  // association waves take their queries in this order (spatially coherent workgroups)
    float4* qp = which == 2 ? a.qpts_sharp + (size_t)s * a.cap_sharp : a.qpts_flat + (size_t)s * a.cap_flat;
    emit([&](int i, int o) {
      const float4 p = ldg(pts + o);
      stg4(qp + i, make_float4(p.x, p.y, p.z, __int_as_float(o)));
    });
    return;
  }
  float4* sorted = ix.sorted + (size_t)s * ix.cap;
  if (!in_regs) {
    emit([&](int i, int o) {
      const float4 p = ldg(pts + o);
      stg4(sorted + i, make_float4(p.x, p.y, p.z, __int_as_float(o)));
    });
    __syncthreads();
    chunk_boxes(sorted, n, false, ix.nn_chunk + (size_t)s * ix.nchunk * 2, ix.nn_super + (size_t)s * ix.nsuper * 2);
    return;
  }
  // Registers: sorted position i = 64 kK wave + 64 t + lane, so a chunk (16 positions) is a 16-lane
  // row of one slot and a super-chunk (256) is the four slots t = 4 v .. 4 v + 3 of one wave:
  // both boxes are reduced from the gathered points without reading the sorted copy back.
  float4* nch_out = ix.nn_chunk + (size_t)s * ix.nchunk * 2;
  float4* nsu_out = ix.nn_super + (size_t)s * ix.nsuper * 2;
  auto rmin = [](float v) {
    v = fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xf, 0xf, true)));
    v = fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xf, 0xf, true)));
    v = fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xf, 0xf, true)));
    return fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xf, 0xf, true)));
  };
  float slo[3] = {3.4e38f, 3.4e38f, 3.4e38f}, shi[3] = {-3.4e38f, -3.4e38f, -3.4e38f};  // super box (row leaders)
#pragma unroll
  for (int t = 0; t < kKeysPerLane; t++) {
    const int i = wave * kPer + t * 64 + lane;
    float4 p = make_float4(3.4e38f, 3.4e38f, 3.4e38f, 0.f);
    float q[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    if (i < n) {
      const int o = (int)(uint32_t)key[t];
      p = ldg(pts + o);
      stg4(sorted + i, make_float4(p.x, p.y, p.z, __int_as_float(o)));
      q[0] = p.x; q[1] = p.y; q[2] = p.z;
    }
    const float lo0 = rmin(p.x), lo1 = rmin(p.y), lo2 = rmin(p.z);
    const float hi0 = -rmin(-q[0]), hi1 = -rmin(-q[1]), hi2 = -rmin(-q[2]);
    const int c = i >> 4;  // chunk of this row
    if ((lane & 15) == 0 && i < n) {
      stg4(nch_out + 2 * c, make_float4(lo0, lo1, lo2, 0.f));
      stg4(nch_out + 2 * c + 1, make_float4(hi0, hi1, hi2, 0.f));
    }
    slo[0] = fminf(slo[0], lo0); slo[1] = fminf(slo[1], lo1); slo[2] = fminf(slo[2], lo2);
    shi[0] = fmaxf(shi[0], hi0); shi[1] = fmaxf(shi[1], hi1); shi[2] = fmaxf(shi[2], hi2);
    if ((t & 3) == 3) {  // super-chunk (wave * 4 + t / 4): combine the four row leaders 0, 16, 32, 48
      float r[6] = {slo[0], slo[1], slo[2], -shi[0], -shi[1], -shi[2]};
#pragma unroll
      for (int e = 0; e < 6; e++) {
        float v = r[e];
        v = fminf(v, __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (16 << 10) | 0x1f)));  // lane ^ 16
        v = fminf(v, __shfl_xor(v, 32));
        r[e] = v;
      }
      const int u = (wave * kPer + (t - 3) * 64) >> 8;
      if (lane == 0 && u * kSuper < n) {
        stg4(nsu_out + 2 * u, make_float4(r[0], r[1], r[2], 0.f));
        stg4(nsu_out + 2 * u + 1, make_float4(-r[3], -r[4], -r[5], 0.f));
      }
      slo[0] = slo[1] = slo[2] = 3.4e38f;
      shi[0] = shi[1] = shi[2] = -3.4e38f;
    }
  }
}

template <int kW, int kK>
__global__ __launch_bounds__(64 * kW, kK >= 32 ? LISLAM_TI_WPE32 : 4) void k_target_index(OdomArgs a, int per_scan, int w0, int w1, int w2) {
  __shared__ uint64_t xch[kW * 8 * 64];
  __shared__ float red[6][kW];
  target_index_body<kW, kK>(a, blockIdx.x, per_scan, w0, w1, w2, xch, red);
}

// Both target-index launches of a batch in one (round 6): workgroups [0, n_scans) index the
// less-flat clouds (32 keys per lane), the rest the less-sharp and query clouds (16 keys per lane),
// one LDS allocation shared by both.  One dependent launch fewer per extraction.
__global__ __launch_bounds__(512, LISLAM_TI_WPE32) void k_target_index_all(OdomArgs a, int n_scans) {
  __shared__ uint64_t xch[8 * 8 * 64];
  __shared__ float red[6][8];
  if ((int)blockIdx.x < n_scans)
    target_index_body<8, 32>(a, blockIdx.x, 1, 1, 1, 1, xch, red);
  else
    target_index_body<8, 16>(a, blockIdx.x - n_scans, 3, 0, 2, 3, xch, red);
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


// ------------------------------------------------------------------ phase 1: association
// One wavefront per query.  Every step of a search is one round trip in which the 64 lanes
// look at 64 candidates at once: super-chunk / chunk bounds, or four 16-point chunks (lane
// groups g = lane / 16).  Results are combined by wave-wide lexicographic minima, so the visit
// order of the reference is only needed as a tie-break key:
//   1-NN         (distance, original index)                 == FLANN's nearest, ties lowest index
//   line search  (distance, walk rank) with rank = j - closest going up, n + closest - j going
//                down == the first strict '<' improvement along the reference's walk (:467-520,
//                :589-646); a chunk is skipped only if its float bound is > the current best.
#ifdef LISLAM_PHASE_PROF  // developer statistics of the searches (scripts/phase_prof.py)
__device__ unsigned long long g_assoc_stats[16];
#ifdef LISLAM_ASSOC_COUNT  // search statistics (global atomics: they distort the timing)
#define ASTAT(i) do { if (lane_id() == 0) atomicAdd(&g_assoc_stats[i], 1ull); } while (0)
#else
#define ASTAT(i)
#endif
extern "C" int lislam_debug_assoc_stats(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_assoc_stats), sizeof(g_assoc_stats)) != hipSuccess) return -2;
  static const unsigned long long zero[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_assoc_stats), zero, sizeof(zero)) == hipSuccess ? 0 : -2;
}
#else
#define ASTAT(i)
#endif
constexpr int kNone = 0x7fffffff;
constexpr int kBatch = 8;  // chunks evaluated per round trip: 4 lane groups x 2 slots

__device__ __forceinline__ int rdlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// (distance, key) pairs packed as one 64-bit integer, distance bits high: distances are
// non-negative floats, whose bit patterns order like their values, so the lexicographic minimum
// of the pairs is the integer minimum (one 64-bit compare instead of three 32-bit ones).
typedef unsigned long long dkey;
__device__ __forceinline__ dkey dk(float d, int key) {
  return ((dkey)__float_as_uint(d) << 32) | (uint32_t)key;
}
__device__ __forceinline__ float dk_d(dkey v) { return __uint_as_float((uint32_t)(v >> 32)); }
__device__ __forceinline__ int dk_key(dkey v) { return (int)(uint32_t)v; }
__device__ __forceinline__ dkey dmin(dkey a, dkey b) { return b < a ? b : a; }
#define kIdent dk(3.4e38f, kNone)  // identity of the minima (no candidate)

// Wave-wide minimum of the pairs (lislam_device.hpp: the minimum distance, then the smallest key
// among the lanes holding it).
__device__ __forceinline__ dkey wave_min(dkey v) { return wave_min_u64(v); }
__device__ __forceinline__ void wave_min2(dkey& va, dkey& vb) {
  const uint32_t ha = (uint32_t)(va >> 32), la = (uint32_t)va, hb = (uint32_t)(vb >> 32), lb = (uint32_t)vb;
  uint32_t ma = ha, mb = hb;
  wave_umin2(ma, mb);
  const uint64_t ta = __ballot(ha == ma), tb = __ballot(hb == mb);
  uint32_t ka, kb;
  if (__popcll(ta) == 1 && __popcll(tb) == 1) {
    ka = (uint32_t)rdlane((int)la, (int)__builtin_ctzll(ta));
    kb = (uint32_t)rdlane((int)lb, (int)__builtin_ctzll(tb));
  } else {
    ka = ha == ma ? la : 0xffffffffu;
    kb = hb == mb ? lb : 0xffffffffu;
    wave_umin2(ka, kb);
  }
  va = ((dkey)ma << 32) | ka;
  vb = ((dkey)mb << 32) | kb;
}

__device__ __forceinline__ int mbcnt(uint64_t m) {  // set bits of m below this lane
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// One batch: the first kBatch pending lanes of m0, then of m1 (lane order), numbered 0..7;
// lane group g = lane / 16 takes items g (slot 0) and 4 + g (slot 1).  Item lanes push
// (value << 1 | list) to lane `item` with ds_permute and every lane pulls its two items with
// ds_bpermute: four crossbar operations instead of a scalar read-lane loop per item.
struct Picked {
  int v[2];       // item values of slots 0 / 1, -1 past the end of the batch
  int list[2];    // which mask the item came from
  bool took0, took1;  // this lane's m0 / m1 entry is in the batch
};
__device__ __forceinline__ Picked pick(uint64_t m0, int v0, uint64_t m1, int v1) {
  const int lane = lane_id();
  const int n0 = min(__popcll(m0), kBatch), ntot = min(n0 + __popcll(m1), kBatch);
  const int r0 = mbcnt(m0), r1 = n0 + mbcnt(m1);
  Picked p;
  p.took0 = ((m0 >> lane) & 1ull) && r0 < kBatch;
  p.took1 = ((m1 >> lane) & 1ull) && r1 < kBatch;
  // lanes outside the batch all push to lane 63, which is never read
  const int q0 = __builtin_amdgcn_ds_permute((p.took0 ? r0 : 63) << 2, v0 << 1);
  const int q1 = __builtin_amdgcn_ds_permute((p.took1 ? r1 : 63) << 2, (v1 << 1) | 1);
  const int items = lane < n0 ? q0 : q1;
  const int g = lane >> 4;
#pragma unroll
  for (int t = 0; t < 2; t++) {
    const int e = g + 4 * t;
    const int it = __builtin_amdgcn_ds_bpermute(e << 2, items);
    p.v[t] = e < ntot ? (it >> 1) : -1;
    p.list[t] = it & 1;
  }
  return p;
}
__device__ __forceinline__ int sel4(int g, int v0, int v1, int v2, int v3) {
  return g == 0 ? v0 : g == 1 ? v1 : g == 2 ? v2 : v3;
}

// Evaluate up to eight 16-point chunks of the Morton-ordered cloud against q.
// ch[t]: this lane group's chunk in slot t (-1 = none).
__device__ __forceinline__ void nn_eval(const P4* sorted, int n, const int (&ch)[2], const P4& q, dkey& best) {
  const int lane = lane_id();
  P4 p[2];
  bool ok[2];
#pragma unroll
  for (int t = 0; t < 2; t++) {
    const int c = ch[t];
    const int j = c * kChunk + (lane & 15);
    ok[t] = c >= 0 && j < n;
    p[t] = ld4(sorted + (ok[t] ? j : 0));  // unpredicated load (point 0 always exists)
  }
  dkey v = kIdent;
#pragma unroll
  for (int t = 0; t < 2; t++) {  // selects, not branches: no exec-mask traffic in the round
    const float dd = d2f(q, p[t]);
    const dkey kk = dk(dd, __float_as_int(p[t].i));
    v = (ok[t] && dd < 25.f && kk < v) ? kk : v;
  }
  best = dmin(best, wave_min(v));
}

// Exact 1-NN with d < 25 (the reference drops farther neighbours, :455/:577) over the
// Morton-ordered copy: the 256 points of the super-chunk with the smallest bound first, then the
// chunk bounds of every other super-chunk whose bound is not above the best (eight super-chunks
// per round trip), then those chunks (eight per round trip).  Returns the original index of the
// lexicographically smallest (distance, index), or -1.
__device__ __forceinline__ int nn_wave(const P4* sorted, int n, const float4* chm, const float4* sum, const P4& q,
                                       dkey seed = kIdent) {
  const int lane = lane_id();
  if (n <= 0) return -1;
  const int nch = (n + kChunk - 1) / kChunk, nsu = (nch + kChunk - 1) / kChunk;
  dkey ub = kIdent;
  float lb0 = 3.4e38f;  // this lane's bound in the first window of super-chunks
  for (int u = lane; u < nsu; u += 64) {
    const float lb = box_lb(ldg(sum + 2 * u), ldg(sum + 2 * u + 1), q);
    if (u < 64) lb0 = lb;
    ub = dmin(ub, dk(lb, u));
  }
  ub = wave_min(ub);
  if (!(dk_d(ub) < 25.f)) return -1;  // every point is at least 25 away
  const int u0 = dk_key(ub);
  ASTAT(0);
  // The next four super-chunks by bound in the first window (< 25): lane group g fetches the 16
  // chunk bounds of the g-th one in the same round trip as u0's points, so the common case needs
  // no separate super-chunk round.  Visiting extra bounds never changes the result.
  int spec = -1;           // this lane group's speculative super-chunk
  bool spec_lane = false;  // this lane's super-chunk (window 0) was fetched speculatively
  {  // (ranking by bound beat taking u0's Morton neighbours u0 -+1, -+2 in an A/B: 4.15 vs 4.18 ms)
    // A heuristic order only (any choice is exact), so 32-bit keys: the bound's bits with the
    // lane in the low 6 (ties within 64 ulps by lane), one 32-bit wave minimum per pick.
    uint32_t v = (lane < nsu && lane != u0 && lb0 < 25.f) ? ((__float_as_uint(lb0) & ~63u) | (uint32_t)lane) : 0xffffffffu;
#pragma unroll
    for (int g = 0; g < 4; g++) {
      const uint32_t m = wave_umin(v);
      const int sg = m != 0xffffffffu ? (int)(m & 63u) : -1;
      if ((lane >> 4) == g) spec = sg;
      if (sg >= 0 && lane == sg) { v = 0xffffffffu; spec_lane = true; }
    }
  }
  int c[2] = {spec >= 0 ? spec * kChunk + (lane & 15) : -1, -1};
  bool cpend[2] = {c[0] >= 0 && c[0] < nch, false};
  float4 slo = make_float4(0.f, 0.f, 0.f, 0.f), shi = slo;
  if (cpend[0]) { slo = ldg(chm + 2 * c[0]); shi = ldg(chm + 2 * c[0] + 1); }
  dkey best = dmin(dk(25.f, kNone), seed);  // seed: a known point (d < 25) only tightens the pruning
  {  // the nearest super-chunk, all 256 points in one round trip
    dkey v = kIdent;
    P4 p[4];
#pragma unroll
    for (int t = 0; t < 4; t++) p[t] = ld4(sorted + min(u0 * kChunk * kChunk + lane + 64 * t, n - 1));
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int j = u0 * kChunk * kChunk + lane + 64 * t;
      const float dd = d2f(q, p[t]);
      if (j < n && dd < 25.f) v = dmin(v, dk(dd, __float_as_int(p[t].i)));
    }
    best = dmin(best, wave_min(v));
  }
  // evaluate the pending chunks (cc, clb, cp) eight per round trip while their bound can beat best
  auto chunk_rounds = [&](int (&cc)[2], float (&clb)[2], bool (&cp)[2]) {
    for (;;) {
      const float bd2 = dk_d(best);
      const uint64_t m0 = __ballot(cp[0] && !(clb[0] > bd2));
      const uint64_t m1 = __ballot(cp[1] && !(clb[1] > bd2));
      if (!m0 && !m1) break;
      ASTAT(2);
      const Picked pk = pick(m0, cc[0], m1, cc[1]);
      if (pk.took0) cp[0] = false;
      if (pk.took1) cp[1] = false;
      nn_eval(sorted, n, pk.v, q, best);
    }
  };
  if (__ballot(cpend[0])) {
    ASTAT(3);
    float clb[2] = {cpend[0] ? box_lb(slo, shi, q) : 3.4e38f, 3.4e38f};
    chunk_rounds(c, clb, cpend);
  }
  for (int ub = 0; ub < nsu; ub += 64) {
    const int u = ub + lane;
    float slb = ub == 0 ? lb0 : 3.4e38f;
    if (ub > 0 && u < nsu) slb = box_lb(ldg(sum + 2 * u), ldg(sum + 2 * u + 1), q);
    bool spend = u < nsu && u != u0 && !(ub == 0 && spec_lane);
    for (;;) {
      const float bd = dk_d(best);
      const uint64_t um = __ballot(spend && !(slb > bd));
      if (!um) break;
      ASTAT(1);
      const Picked su = pick(um, u, 0ull, 0);
      if (su.took0) spend = false;
      // the 16 chunk bounds of each of those super-chunks: lane group g, slots 0 / 1
      float clb[2];
      float4 lo[2], hi[2];
#pragma unroll
      for (int t = 0; t < 2; t++) {
        const int sg = su.v[t];
        c[t] = sg >= 0 ? sg * kChunk + (lane & 15) : -1;
        cpend[t] = c[t] >= 0 && c[t] < nch;
        if (cpend[t]) { lo[t] = ldg(chm + 2 * c[t]); hi[t] = ldg(chm + 2 * c[t] + 1); }
      }
#pragma unroll
      for (int t = 0; t < 2; t++) clb[t] = cpend[t] ? box_lb(lo[t], hi[t], q) : 3.4e38f;
      chunk_rounds(c, clb, cpend);
    }
  }
  const int bi = dk_key(best);
  return bi == kNone ? -1 : bi;
}

// Scan-line searches in the target cloud (scan-line order) around `closest` (label cid).
// kCorner: the corner's second point (:467-520), best in (b2, k2).
// else:    the surf's second (same side of the line, :600-612 / :628-640) and third points.
struct LineSearch {
  const P4* L;
  const float4* chm;  // chunk bounds (scan-line order), w = label min / max
  int n, nch, closest, cid;
  P4 sel;
  dkey b2, b3;  // running bests (distance, walk-rank key); (25, kNone) = none
};

// Evaluate up to eight chunks (dir: 1 up / 0 down) against the running bests.  brk[t]: the
// lane group met the walk's 'break' inside its slot-t chunk.
// ch[t] / upd[t]: this lane group's chunk and direction in slot t (-1 = none).
template <bool kCorner>
__device__ __forceinline__ void ls_eval(LineSearch& s, const int (&ch)[2], const bool (&upd)[2],
                                        uint64_t* brk_mask = nullptr) {
  const int lane = lane_id(), l16 = lane & 15;
  P4 p[2];
  bool valid[2], up[2];
  int j[2];
#pragma unroll
  for (int t = 0; t < 2; t++) {
    const int c = ch[t];
    up[t] = upd[t];
    j[t] = c * kChunk + l16;
    valid[t] = c >= 0 && j[t] < s.n && (up[t] ? j[t] > s.closest : j[t] < s.closest);
    p[t] = ld4(s.L + (valid[t] ? j[t] : s.closest));  // unpredicated load
  }
  dkey v2 = kIdent, v3 = kIdent;
#pragma unroll
  for (int t = 0; t < 2; t++) {  // selects, not branches: no exec-mask traffic in the round
    const int pid = int(p[t].i);
    const bool brk = valid[t] && (up[t] ? pid > s.cid + 2 : pid < s.cid - 2);  // the walk's 'break'
    const uint64_t bm = __ballot(brk);
    if (brk_mask) brk_mask[t] = bm;
    const uint32_t gm = (uint32_t)((bm >> (lane & 48)) & 0xffffull);
    const int first_brk = gm ? (int)__builtin_ctz(gm) : 16, last_brk = gm ? 31 - (int)__builtin_clz(gm) : -1;
    const bool v = valid[t] && (up[t] ? l16 < first_brk : l16 > last_brk);
    const float d = d2f(s.sel, p[t]);
    const dkey kk = dk(d, up[t] ? j[t] - s.closest : s.n + s.closest - j[t]);
    const bool near = v && d < 25.f;
    const bool other = up[t] ? pid > s.cid : pid < s.cid;  // another scan line
    if (kCorner) {
      v2 = (near && other && kk < v2) ? kk : v2;
    } else {
      v2 = (near && !other && kk < v2) ? kk : v2;
      v3 = (near && other && kk < v3) ? kk : v3;
    }
  }
  if (kCorner) {
    s.b2 = dmin(s.b2, wave_min(v2));
  } else {
    wave_min2(v2, v3);
    s.b2 = dmin(s.b2, v2);
    s.b3 = dmin(s.b3, v3);
  }
}

// Does an up / down chunk with bounds (lo, hi) and bound lb still need a visit?
template <bool kCorner>
__device__ __forceinline__ bool ls_need(const LineSearch& s, bool up, const float4& lo, const float4& hi, float lb) {
  const int lmin = (int)lo.w, lmax = (int)hi.w;
  if (kCorner) return (up ? lmax > s.cid : lmin < s.cid) && !(lb > dk_d(s.b2));
  const bool n2 = (up ? lmin <= s.cid : lmax >= s.cid) && !(lb > dk_d(s.b2));
  const bool n3 = (up ? lmax > s.cid : lmin < s.cid) && !(lb > dk_d(s.b3));
  return n2 || n3;
}

template <bool kCorner>
__device__ __forceinline__ void line_search(LineSearch& s) {
  const int lane = lane_id();
  const int hc = s.closest / kChunk;
  // Round trip 1: the home chunk in both directions and its two neighbours, together with the
  // bounds of the next 64 chunks each way (window 0).
  int w = 0;
  int cu = hc + 2 + lane, cd = hc - 2 - lane;
  float4 ulo = make_float4(0, 0, 0, 0), uhi = ulo, dlo = ulo, dhi = ulo;
  bool uin = cu < s.nch, din = cd >= 0;
  if (uin) { ulo = ldg(s.chm + 2 * cu); uhi = ldg(s.chm + 2 * cu + 1); }
  if (din) { dlo = ldg(s.chm + 2 * cd); dhi = ldg(s.chm + 2 * cd + 1); }
  bool up_open, dn_open;  // no 'break' met yet in that direction
  {
    // lane groups: home up, home down, hc + 1 up, hc - 1 down
    const int g = lane >> 4;
    const int ch[2] = {sel4(g, hc, hc, hc + 1 < s.nch ? hc + 1 : -1, hc - 1), -1};
    const bool dir[2] = {(g & 1) == 0, true};
    uint64_t bm[2];
    LineSearch s0 = s;
    ls_eval<kCorner>(s0, ch, dir, bm);
    const bool home_up_brk = bm[0] & 0xffffull, home_dn_brk = (bm[0] >> 16) & 0xffffull;
    if (!home_up_brk && !home_dn_brk) {
      s = s0;
    } else {  // rare: the home chunk broke a walk; redo without the neighbour beyond it
      const int ch2[2] = {(g == 2 && home_up_brk) || (g == 3 && home_dn_brk) ? -1 : ch[0], -1};
      ls_eval<kCorner>(s, ch2, dir);
    }
    up_open = !home_up_brk && !((bm[0] >> 32) & 0xffffull);
    dn_open = !home_dn_brk && !((bm[0] >> 48) & 0xffffull);
  }
  for (;;) {
    uin = uin && up_open;
    din = din && dn_open;
    if (!__ballot(uin) && !__ballot(din)) break;
    ASTAT(4);
    // the first chunk holding a label past the nearby range is where that walk breaks
    const uint64_t ufl = __ballot(uin && (int)uhi.w > s.cid + 2);
    const uint64_t dfl = __ballot(din && (int)dlo.w < s.cid - 2);
    const int ulast = ufl ? (int)__builtin_ctzll(ufl) : 63, dlast = dfl ? (int)__builtin_ctzll(dfl) : 63;
    bool upend = uin && lane <= ulast, dpend = din && lane <= dlast;
    const float ulb = upend ? box_lb(ulo, uhi, s.sel) : 3.4e38f;
    const float dlb = dpend ? box_lb(dlo, dhi, s.sel) : 3.4e38f;
    if (w == 0) {
      // first batch: around the up and the down chunk with the smallest bound among those that
      // can still improve a best (chunks i-1 .. i+2 of each), which sets tight bests at once
      // (a heuristic start: 32-bit keys, the bound's bits with the lane in the low 6)
      uint32_t mu = upend && ls_need<kCorner>(s, true, ulo, uhi, ulb) ? ((__float_as_uint(ulb) & ~63u) | (uint32_t)lane) : 0xffffffffu;
      uint32_t md = dpend && ls_need<kCorner>(s, false, dlo, dhi, dlb) ? ((__float_as_uint(dlb) & ~63u) | (uint32_t)lane) : 0xffffffffu;
      wave_umin2(mu, md);
      const int iu = mu != 0xffffffffu ? (int)(mu & 63u) : kNone, id = md != 0xffffffffu ? (int)(md & 63u) : kNone;
      // lane group g: up chunk iu - 1 + g (slot 0), down chunk id - 1 + g (slot 1)
      const int g = lane >> 4;
      const int lu = (iu != kNone ? iu : 0) - 1 + g, ld = (id != kNone ? id : 0) - 1 + g;
      const int pu = __builtin_amdgcn_ds_bpermute((lu & 63) << 2, (int)upend);
      const int pd = __builtin_amdgcn_ds_bpermute((ld & 63) << 2, (int)dpend);
      const bool okl = iu != kNone && lu >= 0 && lu <= ulast && pu;
      const bool okd = id != kNone && ld >= 0 && ld <= dlast && pd;
      const int ch[2] = {okl ? hc + 2 + lu : -1, okd ? hc - 2 - ld : -1};
      const bool dir[2] = {true, false};
      if (iu != kNone || id != kNone) {
        ASTAT(5);
        if (iu != kNone && lane >= iu - 1 && lane <= iu + 2) upend = false;
        if (id != kNone && lane >= id - 1 && lane <= id + 2) dpend = false;
        ls_eval<kCorner>(s, ch, dir);
      }
    }
    for (;;) {
      const uint64_t um = __ballot(upend && ls_need<kCorner>(s, true, ulo, uhi, ulb));
      const uint64_t dm = __ballot(dpend && ls_need<kCorner>(s, false, dlo, dhi, dlb));
      if (!um && !dm) break;
      ASTAT(kCorner ? 6 : 7);
      const Picked pk = pick(um, cu, dm, cd);
      if (pk.took0) upend = false;
      if (pk.took1) dpend = false;
      const bool dir[2] = {pk.list[0] == 0, pk.list[1] == 0};
      ls_eval<kCorner>(s, pk.v, dir);
    }
    // next window only where the walk did not break inside this one
    w++;
    up_open = up_open && !ufl;
    dn_open = dn_open && !dfl;
    cu += 64;
    cd -= 64;
    uin = cu < s.nch;
    din = cd >= 0;
    if (uin && up_open) { ulo = ldg(s.chm + 2 * cu); uhi = ldg(s.chm + 2 * cu + 1); }
    if (din && dn_open) { dlo = ldg(s.chm + 2 * cd); dhi = ldg(s.chm + 2 * cd + 1); }
  }
}

__device__ __forceinline__ int rank_to_index(const LineSearch& s, int key) {
  return key < s.n ? s.closest + key : s.closest - (key - s.n);
}

__device__ __forceinline__ bool pair_of(const OdomArgs& a, int c, int r, int* k) {
  const int k0 = c * a.chain_len;
  const int k1 = min(k0 + a.chain_len, a.S - 1);
  *k = k0 + r + 1;
  return *k <= k1;
}

// ------------------------------------------------------------------ 16-lane association
// The same exact searches as the engine's (nn_wave / line_search) with one query per 16-lane row,
// four queries per wave:
// a round trip looks at one 16-point chunk per query (lane r = lane & 15 takes point r of it),
// and the lexicographic minima are row reductions by DPP inside the row.  The four rows advance
// in lockstep; a row with nothing left to do contributes the identity, so every lane is active at
// every reduction.  Results are the same by construction: 1-NN = lexicographic min (distance,
// original index) over the points with d < 25, chunks skipped only when their float bound is
// above the row's best distance; line searches = the first strict improvement along the
// reference's walk (distance, walk rank), over chunks up to the one where the walk breaks.
template <int kCtrl>
__device__ __forceinline__ dkey dpp_dkey(dkey v) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), kCtrl, 0xf, 0xf, true);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, kCtrl, 0xf, 0xf, true);
  return ((dkey)hi << 32) | lo;
}
// minimum over the 16 lanes of the row (quad xor 1, xor 2, half-row mirror, row mirror)
__device__ __forceinline__ dkey row_min(dkey v) {
  v = dmin(v, dpp_dkey<0xB1>(v));
  v = dmin(v, dpp_dkey<0x4E>(v));
  v = dmin(v, dpp_dkey<0x141>(v));
  v = dmin(v, dpp_dkey<0x140>(v));
  return v;
}
__device__ __forceinline__ uint32_t row_bits(uint64_t m) { return (uint32_t)(m >> (lane_id() & 48)) & 0xffffu; }

// The 16-lane searches take up to K chunks per round trip (lane r loads point r of each): the
// row's pending chunks whose bound can still beat its best, the first K of them in chunk order.
// Which pending chunks a round takes never changes a minimum (every chunk whose bound is not
// above the best is evaluated before a search ends); K only trades loads per lane for round trips.
#ifndef LISLAM_NN16_K
#define LISLAM_NN16_K 4
#endif
#ifndef LISLAM_LS16_K
#define LISLAM_LS16_K 4
#endif
constexpr int kNn16K = LISLAM_NN16_K, kLs16K = LISLAM_LS16_K;

// The K lowest set bits of m (16-bit, the row's), lowest first; -1 past the last.
template <int K>
__device__ __forceinline__ void first_bits(uint32_t m, int (&pc)[K]) {
#pragma unroll
  for (int t = 0; t < K; t++) {
    pc[t] = m ? (int)__builtin_ctz(m) : -1;
    m &= m - 1u;
  }
}

// Every chunk of super-chunk u (u < 0: the row takes no part) whose bound is not above the row's
// best, K per round trip.
__device__ __forceinline__ void nn16_super(const P4* sorted, int n, int nch, const float4* chm, int u, const P4& q,
                                           dkey& best) {
  constexpr int K = kNn16K;
  const int lr = lane_id() & 15;
  const int c = u * kChunk + lr;
  bool cp = u >= 0 && c < nch;
  float clb = 3.4e38f;
  if (cp) clb = box_lb(ldg(chm + 2 * c), ldg(chm + 2 * c + 1), q);
  for (;;) {
    const uint32_t m = row_bits(__ballot(cp && !(clb > dk_d(best))));
    if (!__ballot(m != 0u)) break;
    int pc[K];
    first_bits<K>(m, pc);
    bool took = false;
#pragma unroll
    for (int t = 0; t < K; t++) took = took || pc[t] == lr;
    if (took) cp = false;
    P4 p[K];
#pragma unroll
    for (int t = 0; t < K; t++) {
      const int j = (u * kChunk + pc[t]) * kChunk + lr;
      p[t] = ld4(sorted + (pc[t] >= 0 && j < n ? j : 0));
    }
    dkey v = kIdent;
#pragma unroll
    for (int t = 0; t < K; t++) {
      const int j = (u * kChunk + pc[t]) * kChunk + lr;
      const float d = d2f(q, p[t]);
      if (pc[t] >= 0 && j < n && d < 25.f) v = dmin(v, dk(d, __float_as_int(p[t].i)));
    }
    best = dmin(best, row_min(v));
  }
}

// Exact 1-NN (d < 25) of the row's query in the Morton-ordered copy; -1 = none.  seed: a known
// point (d < 25) that only tightens the pruning.
__device__ __forceinline__ int nn16(const P4* sorted, int n, const float4* chm, const float4* sum, const P4& q,
                                    bool act, dkey seed = kIdent) {
  const int lr = lane_id() & 15;
  const int nch = (n + kChunk - 1) / kChunk, nsu = act && n > 0 ? (nch + kChunk - 1) / kChunk : 0;
  dkey ub = kIdent;
  float slb[4];  // window 0: this lane's super-chunks lr + 16 kk, kept for the visits below
  const int kmax = (int)wave_umax((uint32_t)((nsu + 15) >> 4));
#pragma unroll
  for (int kk = 0; kk < 4; kk++) slb[kk] = 3.4e38f;
  for (int k0 = 0; k0 < kmax; k0 += 4) {  // four super-chunk bounds per lane per round trip
    float4 lo[4], hi[4];
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
      const int u = lr + 16 * (k0 + kk);
      if (u < nsu) { lo[kk] = ldg(sum + 2 * u); hi[kk] = ldg(sum + 2 * u + 1); }
    }
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
      const int u = lr + 16 * (k0 + kk);
      if (u < nsu) {
        const float lb = box_lb(lo[kk], hi[kk], q);
        ub = dmin(ub, dk(lb, u));
        if (k0 == 0) slb[kk] = lb;
      }
    }
  }
  ub = row_min(ub);
  const bool go = nsu > 0 && dk_d(ub) < 25.f;
  const int u0 = go ? dk_key(ub) : -1;
  dkey best = dmin(dk(25.f, kNone), seed);
  nn16_super(sorted, n, nch, chm, u0, q, best);
  // the other super-chunks, 64 per window (four per lane), in bound order while <= best
  const int wmax = (int)wave_umax((uint32_t)(go ? (nsu + 63) >> 6 : 0));
  for (int win = 0; win < wmax; win++) {
    bool sp[4];
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
      const int u = win * 64 + kk * 16 + lr;
      sp[kk] = go && u < nsu && u != u0;
      if (win > 0) slb[kk] = sp[kk] ? box_lb(ldg(sum + 2 * u), ldg(sum + 2 * u + 1), q) : 3.4e38f;
    }
    for (;;) {
      dkey m = kIdent;
#pragma unroll
      for (int kk = 0; kk < 4; kk++)
        if (sp[kk] && !(slb[kk] > dk_d(best))) m = dmin(m, dk(slb[kk], win * 64 + kk * 16 + lr));
      m = row_min(m);
      const bool want = m != kIdent;
      if (!__ballot(want)) break;
      const int uu = want ? dk_key(m) : -1;
#pragma unroll
      for (int kk = 0; kk < 4; kk++)
        if (want && uu == win * 64 + kk * 16 + lr) sp[kk] = false;
      nn16_super(sorted, n, nch, chm, uu, q, best);
    }
  }
  const int bi = dk_key(best);
  return bi == kNone ? -1 : bi;
}

// Does a chunk with label range [lmin, lmax] and bound lb still need a visit?
__device__ __forceinline__ bool ls16_need(bool corner, bool up, int lmin, int lmax, int cid, float lb, float b2,
                                          float b3) {
  if (corner) return (up ? lmax > cid : lmin < cid) && !(lb > b2);
  const bool n2 = (up ? lmin <= cid : lmax >= cid) && !(lb > b2);
  const bool n3 = (up ? lmax > cid : lmin < cid) && !(lb > b3);
  return n2 || n3;
}

// The scan-line searches of the row (corner: b2; surf: b2, b3) around `closest` in the target
// cloud L (scan-line order, labels non-decreasing), windows of 16 chunks up and down; every round
// trip takes up to K pending chunks, nearest the home chunk first, split between the directions.
__device__ __forceinline__ void ls16(const P4* L, const float4* chm, int n, int closest, int cid, const P4& sel,
                                     bool corner, bool act, dkey& b2, dkey& b3) {
  constexpr int K = kLs16K;
  const int lr = lane_id() & 15;
  const int nch = (n + kChunk - 1) / kChunk;
  const int hc = act ? closest / kChunk : 0;
  bool up_open = act, dn_open = act;
  for (int win = 0;; win++) {
    const int cu = hc + 16 * win + lr, cd = hc - 16 * win - lr;
    const bool uin = up_open && cu < nch, din = dn_open && cd >= 0;
    if (!__ballot(uin || din)) break;
    float4 ulo = make_float4(0.f, 0.f, 0.f, 0.f), uhi = ulo, dlo = ulo, dhi = ulo;
    if (uin) { ulo = ldg(chm + 2 * cu); uhi = ldg(chm + 2 * cu + 1); }
    if (din) { dlo = ldg(chm + 2 * cd); dhi = ldg(chm + 2 * cd + 1); }
    // the first chunk holding a label past the nearby range is where that walk breaks
    const uint32_t ufl = row_bits(__ballot(uin && (int)uhi.w > cid + 2));
    const uint32_t dfl = row_bits(__ballot(din && (int)dlo.w < cid - 2));
    const int ulast = ufl ? (int)__builtin_ctz(ufl) : 15, dlast = dfl ? (int)__builtin_ctz(dfl) : 15;
    bool upend = uin && lr <= ulast, dpend = din && lr <= dlast;
    const float ulb = upend ? box_lb(ulo, uhi, sel) : 3.4e38f, dlb = dpend ? box_lb(dlo, dhi, sel) : 3.4e38f;
    for (;;) {
      const float bd2 = dk_d(b2), bd3 = dk_d(b3);
      const bool nu = upend && ls16_need(corner, true, (int)ulo.w, (int)uhi.w, cid, ulb, bd2, bd3);
      const bool nd = dpend && ls16_need(corner, false, (int)dlo.w, (int)dhi.w, cid, dlb, bd2, bd3);
      uint32_t mu = row_bits(__ballot(nu)), md = row_bits(__ballot(nd));
      if (!__ballot((mu | md) != 0u)) break;
      // ku from the up walk, the rest from the down walk (half each unless one side has fewer)
      const int ku = min(__builtin_popcount(mu), max(K / 2, K - __builtin_popcount(md)));
      int pk[K];
      bool pup[K];
#pragma unroll
      for (int t = 0; t < K; t++) {
        const bool up = t < ku;
        const uint32_t mm = up ? mu : md;
        pk[t] = mm ? (int)__builtin_ctz(mm) : -1;
        if (up) mu &= mu - 1u;
        else md &= md - 1u;
        pup[t] = up;
      }
#pragma unroll
      for (int t = 0; t < K; t++) {
        if (pk[t] == lr && pup[t]) upend = false;
        if (pk[t] == lr && !pup[t]) dpend = false;
      }
      P4 p[K];
      int jj[K];
#pragma unroll
      for (int t = 0; t < K; t++) {
        const int c = pup[t] ? hc + 16 * win + pk[t] : hc - 16 * win - pk[t];
        jj[t] = c * kChunk + lr;
        const bool valid = pk[t] >= 0 && jj[t] >= 0 && jj[t] < n && (pup[t] ? jj[t] > closest : jj[t] < closest);
        if (!valid) jj[t] = -1;
        p[t] = ld4(L + (valid ? jj[t] : 0));
      }
      dkey v2 = kIdent, v3 = kIdent;
#pragma unroll
      for (int t = 0; t < K; t++) {
        const bool up = pup[t];
        const int j = jj[t];
        const int pid = int(p[t].i);
        bool v = j >= 0;
        // the walk's break inside this chunk: up, the first point past cid + 2; down, the last below cid - 2
        const uint32_t bm = row_bits(__ballot(v && (up ? pid > cid + 2 : pid < cid - 2)));
        if (bm) v = v && (up ? lr < (int)__builtin_ctz(bm) : lr > 31 - (int)__builtin_clz(bm));
        const float d = d2f(sel, p[t]);
        const int rk = up ? j - closest : n + closest - j;
        if (v && d < 25.f) {
          if (corner) {
            if (up ? pid > cid : pid < cid) v2 = dmin(v2, dk(d, rk));
          } else {
            if (up ? pid <= cid : pid >= cid) v2 = dmin(v2, dk(d, rk));
            else v3 = dmin(v3, dk(d, rk));
          }
        }
      }
      b2 = dmin(b2, row_min(v2));
      b3 = dmin(b3, row_min(v3));
    }
    up_open = up_open && !ufl;
    dn_open = dn_open && !dfl;
  }
}

template <int kW>
__global__ __launch_bounds__(64 * kW) void k_odom_assoc16(OdomArgs a, int r, int qblocks) {
  int c, qb;
  if (a.cn >= 8) {
    const int b = blockIdx.x, x = b & 7, rr = b >> 3;
    c = 8 * (rr / qblocks) + x;
    qb = rr % qblocks;
  } else {
    c = blockIdx.x / qblocks;
    qb = blockIdx.x % qblocks;
  }
  if (c >= a.cn) return;
  c += a.c0;
  int k;
  if (!pair_of(a, c, r, &k)) return;
  if (a.gate && !a.gate[k]) return;  // not optimized: no association (laserOdometry.cpp:417)
  const int lane = lane_id(), lr = lane & 15;
  const int w = (qb * kW + (int)(threadIdx.x >> 6)) * 4 + (lane >> 4);  // this row's query
  const int ns = a.n_feat[k * 4 + 0], nf = a.n_feat[k * 4 + 2];
  if (__ballot(w < ns + nf) == 0ull) return;  // whole waves leave; nothing below synchronizes the workgroup
  const bool has = w < ns + nf;
  const bool corner = w < ns;
  const int t = corner ? w : w - ns;
  const P4 qp = has ? ld4(corner ? reinterpret_cast<const P4*>(a.qpts_sharp) + (size_t)k * a.cap_sharp + t
                                 : reinterpret_cast<const P4*>(a.qpts_flat) + (size_t)k * a.cap_flat + t)
                    : P4{0.f, 0.f, 0.f, 0.f};
  const int q = __float_as_int(qp.i);
  const TargetIndex& ix = corner ? a.idx_ls : a.idx_lf;
  const P4* L = corner ? a.less_sharp + (size_t)(k - 1) * a.cap_less_sharp : a.less_flat + (size_t)(k - 1) * a.N;
  const P4* sorted = reinterpret_cast<const P4*>(ix.sorted + (size_t)(k - 1) * ix.cap);
  const int nL = a.n_feat[(k - 1) * 4 + (corner ? 1 : 3)];
  const size_t mo = (size_t)(k - 1) * ix.nchunk * 2, so = (size_t)(k - 1) * ix.nsuper * 2;
  double x[7];
  const double* st = a.state + (size_t)c * 16;
  for (int e = 0; e < 7; e++) x[e] = st[e];
  const P4 cur{qp.x, qp.y, qp.z, 0.f};
  const P4 sel = transform_to_start(cur, x);
  const int closest = nn16(sorted, nL, ix.nn_chunk + mo, ix.nn_super + so, sel, has);
  const bool act = has && closest >= 0;
  const P4 pa = ld4(L + (act ? closest : 0));
  const int cid = act ? int(pa.i) : 0;
  dkey b2 = dk(25.f, kNone), b3 = dk(25.f, kNone);
  ls16(L, ix.chunk + mo, nL, act ? closest : 0, cid, sel, corner, act, b2, b3);
  auto idx_of = [&](dkey b) { const int kk = dk_key(b); return kk < nL ? closest + kk : closest - (kk - nL); };
  bool found = false;
  double v = 0.0;  // this lane's record entry (lanes 0..8 of the row)
  if (act && corner && dk_key(b2) != kNone) {  // LidarEdgeFactor(curr, a, b)
    const P4 pb = ld4(L + idx_of(b2));
    const float e9[9] = {cur.x, cur.y, cur.z, pa.x, pa.y, pa.z, pb.x, pb.y, pb.z};
    for (int e = 0; e < 9; e++) if (lr == e) v = e9[e];
    found = true;
  } else if (act && !corner && dk_key(b2) != kNone && dk_key(b3) != kNone) {  // LidarPlaneFactor(curr, j, l, m)
    const P4 pl = ld4(L + idx_of(b2)), pm = ld4(L + idx_of(b3));
    const D3 j{pa.x, pa.y, pa.z};
    const D3 nrm = plane_normal(j, D3{pl.x, pl.y, pl.z}, D3{pm.x, pm.y, pm.z});
    const double e9[9] = {cur.x, cur.y, cur.z, j.x, j.y, j.z, nrm.x, nrm.y, nrm.z};
    for (int e = 0; e < 9; e++) if (lr == e) v = e9[e];
    found = true;
  }
  if (!has) return;
  const int slot = corner ? q : a.cap_sharp + q;
  double* rec = a.blk + ((size_t)c * (a.cap_sharp + a.cap_flat) + slot) * 9;
  if (found && lr < 9) rec[lr] = v;
  if (lr == 0) a.blk_kind[(size_t)c * (a.cap_sharp + a.cap_flat) + slot] = found ? (corner ? 0 : 1) : -1;
}

// ------------------------------------------------------------------ phase 2: LM solve
#ifdef LISLAM_PHASE_PROF
__device__ unsigned long long g_lm_phase[8];
extern "C" int lislam_debug_lm_phases(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lm_phase), sizeof(g_lm_phase)) != hipSuccess) return -2;
  static const unsigned long long zero[8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_lm_phase), zero, sizeof(zero)) == hipSuccess ? 0 : -2;
}
#define LM_PHASE(i)                                                     \
  do {                                                                  \
    if (threadIdx.x == 0) {                                             \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime(); \
      atomicAdd(&g_lm_phase[i], now_ - t_ph);                           \
      t_ph = now_;                                                      \
    }                                                                   \
  } while (0)
#else
#define LM_PHASE(i)
#endif
// ---- the per-round solve, the chain's residual blocks held in LDS across its evaluations
// One workgroup per chain reads the block records once, into LDS, compacted to the bits the records carry: the
// query point and the first matched point are floats in every record (laserOdometry.cpp:554-556,
// :677-681 take them from float clouds), the third triple is the edge's second point (float) or
// the plane's unit normal (double).  Blocks past kLmLds (only when cap_sharp + cap_flat exceeds
// it, H > 64 lines) are evaluated from the global records.  The reduction sums 16-lane rows by
// DPP, then each wave sums one accumulator entry over the 64 row partials.
#ifndef LISLAM_LM2_THREADS
#define LISLAM_LM2_THREADS 512
#endif
constexpr int kLm2Threads = LISLAM_LM2_THREADS;
constexpr int kLm2Waves = kLm2Threads / 64;
#ifndef LISLAM_LM_LDS
#define LISLAM_LM_LDS 2816
#endif
constexpr int kLmLds = LISLAM_LM_LDS;

struct Lm2Shared {
  float c[3][kLmLds];    // query point
  float p[3][kLmLds];    // edge point a / plane point j
  double d[3][kLmLds];   // edge point b / plane normal
  int8_t kind[kLmLds];
  double red[kLm2Waves * 4][kAcc];
  double x[7];
  double acc[kAcc];
  int cnt[kLm2Waves][2];
  int nc, np, flag;
};

__device__ __forceinline__ void block_accum3(int kd, const D3& c, const D3& p1, const D3& p2, const DQ& q, const D3& t,
                                             double* acc) {
  const double ha = 0.1;  // HuberLoss(0.1)
  const D3 p = qrot(q, c);
  const D3 lp = p + t;
  if (kd == 0) {
    // edge_factor, one residual row at a time (its Jacobian row is 6 live doubles, not 18), and
    // the six divisions by |a - b| as products with its reciprocal
    const D3 nu = cross(lp - p1, lp - p2);
    const D3 de = p1 - p2;
    const double inv = 1.0 / sqrt(de.x * de.x + de.y * de.y + de.z * de.z);  // one division, six products
    const double r0 = nu.x * inv, r1 = nu.y * inv, r2 = nu.z * inv;
    const double sc = huber_scale(ha, r0 * r0 + r1 * r1 + r2 * r2, &acc[0]);
    const D3 d{(p2.x - p1.x) * inv, (p2.y - p1.y) * inv, (p2.z - p1.z) * inv};
    const double P[3][3] = {{0, 2 * p.z, -2 * p.y}, {-2 * p.z, 0, 2 * p.x}, {2 * p.y, -2 * p.x, 0}};  // -2[p]x
#pragma unroll 1
    for (int k = 0; k < 3; k++) {
      const double m0 = k == 0 ? 0.0 : k == 1 ? d.z : -d.y;
      const double m1 = k == 0 ? -d.z : k == 1 ? 0.0 : d.x;
      const double m2 = k == 0 ? d.y : k == 1 ? -d.x : 0.0;
      const double rk = k == 0 ? r0 : k == 1 ? r1 : r2;
      double Js[6];
#pragma unroll
      for (int cc = 0; cc < 3; cc++) Js[cc] = (m0 * P[0][cc] + m1 * P[1][cc] + m2 * P[2][cc]) * sc;
      Js[3] = m0 * sc; Js[4] = m1 * sc; Js[5] = m2 * sc;
      accum_row(acc, Js, rk * sc);
    }
  } else {
    // plane_factor (p2 = the constructor's unit normal)
    const double res = dot(lp - p1, p2);
    const D3 pn = cross(p, p2);
    double J[6] = {2 * pn.x, 2 * pn.y, 2 * pn.z, p2.x, p2.y, p2.z};
    const double sc = huber_scale(ha, res * res, &acc[0]);
#pragma unroll
    for (int cc = 0; cc < 6; cc++) J[cc] *= sc;
    accum_row(acc, J, res * sc);
  }
}

__device__ __forceinline__ void evaluate2(Lm2Shared& sh, const double* blk, const int* kind, int ns, int cap_sharp,
                                          int nf) {
  double acc[kAcc];
#pragma unroll
  for (int e = 0; e < kAcc; e++) acc[e] = 0;
  const DQ q{sh.x[0], sh.x[1], sh.x[2], sh.x[3]};
  const D3 t{sh.x[4], sh.x[5], sh.x[6]};
  const int total = ns + nf;
  for (int i = threadIdx.x; i < total; i += kLm2Threads) {
    int kd;
    D3 c, p1, p2;
    if (i < kLmLds) {
      kd = sh.kind[i];
      c = D3{sh.c[0][i], sh.c[1][i], sh.c[2][i]};
      p1 = D3{sh.p[0][i], sh.p[1][i], sh.p[2][i]};
      p2 = D3{sh.d[0][i], sh.d[1][i], sh.d[2][i]};
    } else {  // beyond the LDS cache
      const int idx = i < ns ? i : cap_sharp + (i - ns);
      kd = kind[idx];
      const double* rb = blk + (size_t)idx * 9;
      c = D3{rb[0], rb[1], rb[2]};
      p1 = D3{rb[3], rb[4], rb[5]};
      p2 = D3{rb[6], rb[7], rb[8]};
    }
    if (kd >= 0) block_accum3(kd, c, p1, p2, q, t, acc);
  }
  const int lane = threadIdx.x & 63, row = threadIdx.x >> 4;
#pragma unroll
  for (int e = 0; e < kAcc; e++) {
    const double v = row_sum(acc[e]);
    if ((lane & 15) == 0) sh.red[row][e] = v;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6;
  for (int e = w; e < kAcc; e += kLm2Waves) {  // wave w: entries w, w + kLm2Waves, ...
    double v = lane < kLm2Waves * 4 ? sh.red[lane][e] : 0.0;
    v = row_sum(v);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane == 0) sh.acc[e] = v;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kLm2Threads) void k_odom_lm2(OdomArgs a, int r, int outer) {
  __shared__ Lm2Shared sh;
  __shared__ LM lm;
#ifdef LISLAM_PHASE_PROF
  unsigned long long t_ph = __builtin_amdgcn_s_memrealtime();
#endif
  const int c = a.c0 + blockIdx.x;
  int k;
  if (!pair_of(a, c, r, &k)) return;
  double* st = a.state + (size_t)c * 16;
  const int ns = a.n_feat[k * 4 + 0], nf = a.n_feat[k * 4 + 2];
  const double* blk = a.blk + (size_t)c * (a.cap_sharp + a.cap_flat) * 9;
  const int* kind = a.blk_kind + (size_t)c * (a.cap_sharp + a.cap_flat);
  const bool gated_off = a.gate && !a.gate[k];  // use_aloam false: no solve, the pose still accumulates
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  {
    // the records into LDS, and the correspondence counts (:562/:685)
    int c0 = 0, c1 = 0;
    const int total = gated_off ? 0 : ns + nf;
    for (int i = threadIdx.x; i < total; i += kLm2Threads) {
      const int idx = i < ns ? i : a.cap_sharp + (i - ns);
      const int kd = kind[idx];
      c0 += kd == 0;
      c1 += kd == 1;
      if (i < kLmLds) {
        sh.kind[i] = (int8_t)kd;
        if (kd >= 0) {
          const double* rb = blk + (size_t)idx * 9;
          double v[9];
#pragma unroll
          for (int e = 0; e < 9; e++) v[e] = rb[e];
#pragma unroll
          for (int e = 0; e < 3; e++) {
            sh.c[e][i] = (float)v[e];
            sh.p[e][i] = (float)v[3 + e];
            sh.d[e][i] = v[6 + e];
          }
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      c0 += __shfl_xor(c0, o);
      c1 += __shfl_xor(c1, o);
    }
    if (lane == 0) { sh.cnt[w][0] = c0; sh.cnt[w][1] = c1; }
    if (threadIdx.x == 0)
      for (int e = 0; e < 7; e++) sh.x[e] = st[e];
    __syncthreads();
    if (threadIdx.x == 0) {
      int a0 = 0, a1 = 0;
      for (int v = 0; v < kLm2Waves; v++) { a0 += sh.cnt[v][0]; a1 += sh.cnt[v][1]; }
      sh.nc = a0;
      sh.np = a1;
    }
    __syncthreads();
  }
  const int nc = sh.nc, np = sh.np;
  LM_PHASE(3);
  bool go = (nc + np) > 0;  // no residual blocks: Ceres leaves the parameters untouched
  if (go) {
    evaluate2(sh, blk, kind, ns, a.cap_sharp, nf);
    LM_PHASE(0);
    if (threadIdx.x == 0) {
      const bool cont = lm_start(lm, sh.x, sh.acc, a.max_iterations);
      sh.flag = cont;
      if (cont)
        for (int e = 0; e < 7; e++) sh.x[e] = lm.xc[e];
    }
    __syncthreads();
    go = uni(sh.flag);
  }
  LM_PHASE(2);
  while (go) {
    evaluate2(sh, blk, kind, ns, a.cap_sharp, nf);  // cost + J^T J + J^T r at the candidate
    LM_PHASE(1);
#ifdef LISLAM_PHASE_PROF
    if (threadIdx.x == 0) atomicAdd(&g_lm_phase[5], 1ull);
#endif
    if (threadIdx.x == 0) {
      const bool cont = lm_next(lm, sh.acc, a.max_iterations);
      sh.flag = cont;
      if (cont)
        for (int e = 0; e < 7; e++) sh.x[e] = lm.xc[e];
    }
    __syncthreads();
    LM_PHASE(2);
    go = sh.flag;
  }
  if (threadIdx.x != 0) return;
  int* so = a.stats + (size_t)k * 8;
  so[outer * 2 + 0] = nc;
  so[outer * 2 + 1] = np;
  so[4 + outer] = (nc + np) > 0 ? lm.it : 0;
  so[6 + outer] = (nc + np) > 0 ? lm.term : 1;
  if ((nc + np) > 0)
    for (int e = 0; e < 7; e++) st[e] = lm.x[e];
  if (outer == 1) {
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

// d(q * c)/dq of Eigen's _transformVector p = c + w uv + u x uv, uv = 2 (u x c), u = (x, y, z):
// columns x, y, z, w of the raw quaternion block (the polynomial ceres::Jet differentiates).
__device__ __forceinline__ void drot_dq(const DQ& q, const D3& c, double (*P)[4]) {
  const D3 u{q.x, q.y, q.z};
  const D3 uv = 2.0 * cross(u, c);
  const D3 e[3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  for (int i = 0; i < 3; i++) {
    const D3 duv = 2.0 * cross(e[i], c);
    const D3 d = q.w * duv + cross(e[i], uv) + cross(u, duv);
    P[0][i] = d.x; P[1][i] = d.y; P[2][i] = d.z;
  }
  P[0][3] = uv.x; P[1][3] = uv.y; P[2][3] = uv.z;
}

// One thread per residual block.  r(lp) with lp = q * c (+ t): J_q = dr/dlp . dlp/dq, J_t = dr/dlp.
// The functors' identity.slerp(s = 1, q) is +-q (lidarFeaturePointsFunction.hpp:165,262), which
// rotates exactly like q and has the same raw derivative (the sign squares out).
__global__ __launch_bounds__(256) void k_eval_factors_raw(RawFactorArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const DQ q{a.x[0], a.x[1], a.x[2], a.x[3]};
  const D3 t{a.x[4], a.x[5], a.x[6]};
  const double* p = a.pts + (size_t)i * 12;
  const D3 c{p[0], p[1], p[2]};
  const int kd = a.kind[i];
  if (kd == 5 || kd == 6) {  // DISTORTION 1: the slerp-interpolated functors, by dual numbers
    const double qa[4] = {q.x, q.y, q.z, q.w}, ta[3] = {t.x, t.y, t.z};
    DJet rj[3];
    const int R = kd == 5 ? 3 : 1;
    if (kd == 5) edge_factor_s(qa, ta, p, rj);
    else plane_factor_s(qa, ta, p, rj);
    for (int k = 0; k < 3; k++) {
      if (a.res) a.res[(size_t)i * 3 + k] = k < R ? rj[k].a : 0.0;
      if (a.jq)
        for (int cc = 0; cc < 4; cc++) a.jq[((size_t)i * 3 + k) * 4 + cc] = k < R ? rj[k].v[cc] : 0.0;
      if (a.jt)
        for (int cc = 0; cc < 3; cc++) a.jt[((size_t)i * 3 + k) * 3 + cc] = k < R ? rj[k].v[4 + cc] : 0.0;
    }
    return;
  }
  double r[3] = {0, 0, 0}, G[3][3] = {{0}};  // G = dr/dlp (rows = residuals)
  int R = 1;
  if (kd == 0) {
    double J[3][6];
    edge_factor(q, t, c, D3{p[3], p[4], p[5]}, D3{p[6], p[7], p[8]}, r, J);
    for (int k = 0; k < 3; k++) for (int cc = 0; cc < 3; cc++) G[k][cc] = J[k][3 + cc];
    R = 3;
  } else if (kd == 1) {
    const D3 n = plane_normal(D3{p[3], p[4], p[5]}, D3{p[6], p[7], p[8]}, D3{p[9], p[10], p[11]});
    double J[6];
    plane_factor(q, t, c, D3{p[3], p[4], p[5]}, n, r, J);
    G[0][0] = n.x; G[0][1] = n.y; G[0][2] = n.z;
  } else if (kd == 2 || kd == 4) {
    const D3 n{p[3], p[4], p[5]};
    const D3 pr = qrot(q, c);
    r[0] = dot(n, kd == 2 ? pr + t : pr) + p[6];
    G[0][0] = n.x; G[0][1] = n.y; G[0][2] = n.z;
  } else {
    double J[3][6];
    p2p_factor(q, t, c, D3{p[3], p[4], p[5]}, r, J);
    for (int k = 0; k < 3; k++) G[k][k] = 1.0;
    R = 3;
  }
  double P[3][4];
  drot_dq(q, c, P);
  for (int k = 0; k < 3; k++) {
    if (a.res) a.res[(size_t)i * 3 + k] = k < R ? r[k] : 0.0;
    if (a.jq)
      for (int cc = 0; cc < 4; cc++)
        a.jq[((size_t)i * 3 + k) * 4 + cc] = k < R ? G[k][0] * P[0][cc] + G[k][1] * P[1][cc] + G[k][2] * P[2][cc] : 0.0;
    if (a.jt)
      for (int cc = 0; cc < 3; cc++) a.jt[((size_t)i * 3 + k) * 3 + cc] = (k < R && kd != 4) ? G[k][cc] : 0.0;
  }
}

// Developer profile of the engine (null in production): per ticket kProfSlots u64 = s_memrealtime
// (100 MHz) at claim, inputs ready, records loaded (solve), done; summed evaluation and step ticks and
// the evaluation count (solve), 11 step 0's share sum; items: 10 the end of the item's last query.  lislam_debug_engine_prof(n) arms it (n tickets; 0 disarms),
// lislam_debug_engine_prof_read copies it out.
constexpr int kProfSlots = 16;
__device__ unsigned long long* g_eng_prof = nullptr;
__device__ unsigned g_eng_prof_n = 0;  // tickets the buffer holds (writes past it are dropped)
static unsigned long long* s_eng_prof = nullptr;
static int s_eng_prof_n = 0;
extern "C" int lislam_debug_engine_prof(int n_tickets) {
  if (s_eng_prof) { (void)hipFree(s_eng_prof); s_eng_prof = nullptr; }
  s_eng_prof_n = 0;
  unsigned long long* d = nullptr;
  if (n_tickets > 0) {
    if (hipMalloc((void**)&d, sizeof(unsigned long long) * kProfSlots * n_tickets) != hipSuccess) return -2;
    if (hipMemset(d, 0, sizeof(unsigned long long) * kProfSlots * n_tickets) != hipSuccess) return -2;
    s_eng_prof = d;
    s_eng_prof_n = n_tickets;
  }
  const unsigned n = (unsigned)s_eng_prof_n;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_eng_prof_n), &n, sizeof(n)) != hipSuccess) return -2;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_eng_prof), &d, sizeof(d)) == hipSuccess ? 0 : -2;
}
extern "C" int lislam_debug_engine_prof_read(unsigned long long* out, int n_tickets) {
  if (!s_eng_prof || n_tickets > s_eng_prof_n) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return hipMemcpy(out, s_eng_prof, sizeof(unsigned long long) * kProfSlots * n_tickets, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
// LISLAM_ENG_PROF = 0 compiles the engine's developer timestamps out (rt_now() = 0, eng_prof a no-op).
#ifndef LISLAM_ENG_PROF
#define LISLAM_ENG_PROF 0  // developer builds: -DLISLAM_ENG_PROF=1 (scripts/engine_prof.py); the stamps cost ~4 %
#endif
__device__ __forceinline__ void eng_prof(unsigned tk, int slot, unsigned long long v, bool add = false) {
#if LISLAM_ENG_PROF
  unsigned long long* p = g_eng_prof;
  if (!p || tk >= g_eng_prof_n) return;
  if (add) p[(size_t)tk * kProfSlots + slot] += v;
  else if (slot == 10) atomicMax(p + (size_t)tk * kProfSlots + slot, v);  // the item's last own query
  else p[(size_t)tk * kProfSlots + slot] = v;
#endif
}
__device__ __forceinline__ unsigned long long rt_now() {
#if LISLAM_ENG_PROF
  return __builtin_amdgcn_s_memrealtime();
#else
  return 0ull;
#endif
}
// per-query record of one pair (developer): [outer][query] = {1-NN ticks, line-search ticks, closest, kind}
__device__ int* g_eng_qlog = nullptr;
__device__ int g_eng_qlog_pair = -1;
extern "C" int lislam_debug_engine_qlog(int* dev_buf, int pair) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_eng_qlog), &dev_buf, sizeof(dev_buf)) != hipSuccess) return -2;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_eng_qlog_pair), &pair, sizeof(pair)) == hipSuccess ? 0 : -2;
}

// ================================================================== the chain engine
// The whole odometry schedule of a few long chains (the reference's continuous para_q / para_t
// carry, laserOdometry.cpp:130-135,716-717) as ONE persistent launch.  The schedule is a ticket
// queue: for every round r and outer pass o (:417), and every chain c, I association items (32
// queries each: 8 waves x four 16-lane rows, the searches of k_odom_assoc16) then one solve item
// (the Ceres-semantics LM of k_odom_lm2, on one workgroup).  A workgroup takes the next ticket
// with one atomic add and waits, polling one word, until the ticket's inputs exist:
//   association (c, r, o)  needs the solve before it (lm_gen[c] >= 2 r + o): x = para_q / para_t;
//   solve (c, r, o)        needs its I association items (assoc_done[c][2 r + o] == I).
// Every dependency of a ticket is a lower ticket, taken earlier by a running workgroup, so the
// queue drains whatever the residency (one resident workgroup runs it all, serially): there is
// no grid barrier to deadlock.  Every spin is bounded (2 s) and raises the abort word, which every
// waiting workgroup also polls, so the grid always drains.
// Hand-offs (MI355X_MICROARCH.md, visibility): the payloads (records, x) are stored write-through
// (relaxed agent-scope atomic stores = global_store sc1), every storing wave drains vmcnt, ONE
// lane signals with an agent-scope atomic; the consumer polls relaxed, then every load of the
// payload is an agent-scope (sc1) load.
// The solve evaluates each block in the form J^T J = G^T M G, J^T r = G^T v with G = [-2 [p]x, I]
// (p = R c, the local parameterization of EigenQuaternionParameterization): M = w (|u|^2 I - u u^T)
// and v = w (u x r) for LidarEdgeFactor (r = (lp - a) x u, u = (a - b) / |a - b|, the functor's
// (lp - a) x (lp - b) / |a - b| rearranged), M = w n n^T and v = w r n for LidarPlaneFactor
// (r = (lp - j) . n); w = the Huber corrector's rho'.  28 sums per thread: cost, M, T = [p]x M,
// U = T [p]x, v, p x v; H = [[-4 U, 2 T], [2 T^T, M]], g = [2 p x v, v].
#ifndef LISLAM_ENG_THREADS
#define LISLAM_ENG_THREADS 512  // 256 VGPRs: the fp64 evaluation's 28 sums + block state spill at 128
#endif
constexpr int kEngThreads = LISLAM_ENG_THREADS;
constexpr int kEngWaves = kEngThreads / 64;
// Queries per association item: one per wave (64 lanes), EngCtl::Q = the item workgroup's waves —
// kEngWaves in the single-launch engine (items share its workgroup size), up to kMaxItemWaves in the
// split engine's items kernel (LISLAM_ENGINE_ITEM_WAVES).
#ifndef LISLAM_MAX_ITEM_WAVES
#define LISLAM_MAX_ITEM_WAVES 16
#endif
constexpr int kMaxItemWaves = LISLAM_MAX_ITEM_WAVES;
// A block record: 64 B = four 16-B quads, written by the association wave of its query (lanes 0..3,
// write-through) and read by the solve with 16-B loads:
//   q0 c.x c.y c.z a.x (float) | q1 a.y a.z (float) kind (int) - | q2 u.x u.y (double) | q3 u.z (double) -
// (c the query point, a the first matched point, u the edge direction / plane normal).
constexpr int kRecBytes = 64;
constexpr int kRecWords = kRecBytes / 8;
constexpr int kAuxSc1 = 16;  // buffer instruction cache policy: sc1 (write-through stores, L1-bypassing loads)
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc make_rsrc(const void* base, unsigned bytes) {  // base wave-uniform
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1d(double* p, double v) { st_sc1((uint64_t*)p, (uint64_t)__double_as_longlong(v)); }
__device__ __forceinline__ double ld_sc1d(const double* p) { return __longlong_as_double((long long)ld_sc1((const uint64_t*)p)); }
__device__ __forceinline__ unsigned ld_rlx(unsigned* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(unsigned* p, unsigned v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned add_rlx(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double uniform_d(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// control words: [0] ticket, [1] abort (this launch), [2] error, [3] sticky abort (set with [1], never
// cleared by a launch: lislam_batch_odometry_status reads and clears it), [4, 4 + C) lm_gen, then
// assoc_done[C][2 R]
constexpr int kMaxShareItems = 256;  // 16 threads x 8 loads per item row: 32 rows per round x 8
struct EngCtl {
  unsigned* w;
  int C, R, I;
  unsigned long long wait_ticks;  // bound of every device wait (s_memrealtime ticks, 100 MHz)
  unsigned backoff;               // eng_wait's longest sleep between polls (x 64 cycles)
  int prefetch;  // waiting association tickets warm this XCD's L2 with their pair's target structures
  int roles;     // solve-role tickets ahead of the items in this launch's queue (C, or 0: roles in their own launch)
  int budget;    // association items per (pass, chain) at most: what the resident workgroups can hold at
                 // once, and at most kMaxShareItems (the solve sums the shares in one round of loads)
  unsigned gen;  // this launch's number: with the pass, the tag of a complete item row (eng_tag)
  int P;         // rows per chain of eng_part (engine_part_rows)
  int Q;         // the association item workgroup's waves
  int qpw;       // queries per wave: 1..3 (64-lane searches, one after another) or 4 (one per 16-lane row)
  __host__ __device__ int qpi() const { return Q * qpw; }  // queries per item
  __device__ unsigned* ticket() const { return w; }
  __device__ unsigned* abort_w() const { return w + 1; }
  __device__ unsigned* lm_gen(int c) const { return w + 4 + c; }
  __device__ unsigned* assoc_done(int c, int ro) const { return w + 4 + C + (size_t)c * 2 * R + ro; }
  __device__ unsigned* role_ticket() const { return w + 4 + C + (size_t)2 * R * C; }
  __device__ unsigned* role_arrive() const { return w + 5 + C + (size_t)2 * R * C; }
  // the device's solve roles per XCD (k_odom_roles), or null: roles taken without regard to XCD
  unsigned* xbusy = nullptr;
  int rgrid = 0;  // k_odom_roles' grid
};
// Word 31 of an item's eng_part row once its records and share of pass ro are written.
__device__ __forceinline__ uint64_t eng_tag(const EngCtl& ctl, int ro) {
  return ((uint64_t)ctl.gen << 32) | (uint64_t)(unsigned)(ro + 1);
}

// Association items of pair k that hold queries (the rest of the ctl.I items are skipped).
__device__ __forceinline__ int eng_live_items(const OdomArgs& a, const EngCtl& ctl, int k) {
  if (a.gate && !a.gate[k]) return 0;
  return uni(min((a.n_feat[k * 4 + 0] + a.n_feat[k * 4 + 2] + ctl.qpi() - 1) / ctl.qpi(), ctl.budget));
}

// A pass's association: ieff items of qpi() queries; when the pair holds more queries than that
// (the items are capped by EngCtl::budget, what the resident workgroups hold), the items take the
// novf overflow queries in further rounds (eng_item_run).
struct PassShape {
  int ieff, novf;
};
__device__ __forceinline__ PassShape pass_shape(const OdomArgs& a, const EngCtl& ctl, int k) {
  PassShape ps;
  ps.ieff = eng_live_items(a, ctl, k);
  const int nq = a.n_feat[k * 4 + 0] + a.n_feat[k * 4 + 2];
  ps.novf = ps.ieff > 0 ? uni(max(0, nq - ctl.qpi() * ps.ieff)) : 0;
  return ps;
}
__device__ __forceinline__ double* part_row(const OdomArgs& a, const EngCtl& ctl, int c, int row) {
  return a.eng_part + ((size_t)c * ctl.P + row) * 32;
}

// Developer trace of the engine (null in production): per workgroup {ticket, stage, LM passes,
// time}, stored system-scope into host-pinned memory so the host can read it while the kernel runs.
__device__ unsigned* g_eng_trace = nullptr;
__device__ unsigned g_eng_trace_n = 0;  // workgroups the buffer holds
extern "C" int lislam_debug_engine_trace(int n_wgs, unsigned** host_out) {
  static unsigned* h = nullptr;
  static int cap = 0;
  if (n_wgs <= 0) {
    unsigned* z = nullptr;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_eng_trace), &z, sizeof(z)) == hipSuccess ? 0 : -2;
  }
  if (n_wgs > cap) {
    if (h) (void)hipHostFree(h);
    if (hipHostMalloc((void**)&h, sizeof(unsigned) * 256 * n_wgs, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return -2;
    cap = n_wgs;
  }
  for (int i = 0; i < 256 * n_wgs; i++) h[i] = 0xffffffffu;
  unsigned* d = nullptr;
  if (hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess) return -2;
  const unsigned n = (unsigned)n_wgs;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_eng_trace_n), &n, sizeof(n)) != hipSuccess) return -2;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_eng_trace), &d, sizeof(d)) != hipSuccess) return -2;
  *host_out = h;
  return 0;
}
__device__ __forceinline__ void eng_trace(int slot, unsigned v) {
  unsigned* t = g_eng_trace;
  if (t && blockIdx.x < g_eng_trace_n) __hip_atomic_store(t + (blockIdx.x * 16 + slot) * 16, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // a 64-B line each
}

// One lane: wait until *p >= target; false = aborted (the bound, 2 s by default, or another
// workgroup's abort).  An expired bound raises this launch's abort word and the sticky one.
// Arguments by value: a struct passed by reference would live in scratch, and values loaded from
// scratch count as divergent, which would put the ticket loop's barriers in divergent control flow.
// code: which wait (EngCtl word 2 when its bound expires): 1 an item for the previous pass's items,
// 2 an item for x, 3 a solve role for its pass's items.
// Developer builds (LISLAM_ENG_PROF=1) count every wait's polls per wait code (g_eng_polls[code],
// g_eng_polls[8 + code] the waits): each poll is two agent-scope loads (the word, the abort word),
// the traffic attribution of DESIGN.md §5 (lislam_debug_engine_polls reads and clears them).
__device__ unsigned long long g_eng_polls[16];
extern "C" int lislam_debug_engine_polls(unsigned long long* out16) {
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_eng_polls), sizeof(g_eng_polls)) != hipSuccess) return -2;
  static const unsigned long long zero[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_eng_polls), zero, sizeof(zero)) == hipSuccess ? 0 : -2;
}
__device__ __forceinline__ void eng_count_polls(unsigned code, unsigned long long polls) {
#if LISLAM_ENG_PROF
  __hip_atomic_fetch_add(&g_eng_polls[code & 7], polls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_add(&g_eng_polls[8 + (code & 7)], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}
// backoff: the sleep between polls doubles from 64 cycles up to `backoff` x 64 (1 = a fixed 64).
__device__ __noinline__ bool eng_wait(unsigned* p, unsigned target, unsigned* abort_w, unsigned long long bound,
                                      unsigned code, unsigned backoff) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long polls = 0;
  unsigned nap = 1;
  bool ok;
  for (;;) {
    polls++;
    if (ld_rlx(p) >= target) { ok = true; break; }
    if (ld_rlx(abort_w)) { ok = false; break; }
    if (__builtin_amdgcn_s_memrealtime() - t0 > bound) {  // 100 MHz clock
      st_rlx(abort_w + 1, code);  // the error word
      st_rlx(abort_w, 1u);
      st_rlx(abort_w + 2, 1u);  // sticky (EngCtl word 3)
      ok = false;
      break;
    }
    for (unsigned i = 0; i < nap; i++) __builtin_amdgcn_s_sleep(1);
    nap = nap * 2 > backoff ? backoff : nap * 2;
  }
  eng_count_polls(code, polls);
  return ok;
}

struct EngShared {
  double red[kEngWaves * 4][32];  // kAcc sums (+ 2 counts) per 16-lane row
  double xw[kMaxItemWaves][8];     // each wave's copy of its item's x (the item's queries read it here)
  P4 prew[kMaxItemWaves][4][4];    // each wave's ItemPre of its first query per row: qp, the seeds' points
  int prei[kMaxItemWaves][4][4];   // ... and the seeds' indices
  double acc[kAcc];
  double x[7];
  double cx[7], cpw[7];  // solve role: the chain's x (para_q / para_t) and pose between passes
  int cnt[kEngWaves][2];
  unsigned ticket;
  int flag, flag0, nc, np, pref;
  unsigned sink;
};

// Word e of x (para_q, para_t) a ticket of (c, r, o) starts from: the chain's initial state for
// its first pass, else the last solve's (write-through) result.
__device__ __forceinline__ double eng_x_word(const OdomArgs& a, int c, int r, int o, int e) {
  if (r == 0 && o == 0) return a.init_state ? a.init_state[(size_t)c * 14 + e] : (e == 3 ? 1.0 : 0.0);
  return ld_sc1d(a.state + (size_t)c * 16 + e);
}


// One block's 28 sums (see the engine comment) at p = R c, lp = p + t (R, t uniform): emit(e, v)
// receives each block's contribution v to sum e once (a fresh sum's accumulate, fma(a, b, 0) ==
// a * b).  Edge blocks: M (rank 2) and each row of T emitted as soon as it exists, to keep few
// doubles live.  Plane blocks are rank 1: with a = p x n, M = w n n^T, T = [p]x M = w a n^T,
// U = T [p]x = -w a a^T, v = w r n, p x v = w r a (39 multiplies instead of ~90).
template <class Emit>
__device__ __forceinline__ void eng_block_emit(int kd, const D3& c, const D3& pa, const D3& u, const double* R, const D3& t,
                                               Emit&& emit) {
  const D3 p{fma(R[0], c.x, fma(R[1], c.y, R[2] * c.z)), fma(R[3], c.x, fma(R[4], c.y, R[5] * c.z)),
             fma(R[6], c.x, fma(R[7], c.y, R[8] * c.z))};
  const D3 e{(p.x + t.x) - pa.x, (p.y + t.y) - pa.y, (p.z + t.z) - pa.z};
  double r0 = 0, r1 = 0, r2 = 0, rp = 0, s2;
  if (kd == 0) {
    r0 = fma(e.y, u.z, -e.z * u.y); r1 = fma(e.z, u.x, -e.x * u.z); r2 = fma(e.x, u.y, -e.y * u.x);
    s2 = fma(r0, r0, fma(r1, r1, r2 * r2));
  } else {
    rp = fma(e.x, u.x, fma(e.y, u.y, e.z * u.z));
    s2 = rp * rp;
  }
  double w = 1.0;
  if (s2 > 0.01) {  // HuberLoss(0.1): rho = 2 a sqrt(s) - a^2, rho' = a / sqrt(s)
    const double rr = sqrt(s2);
    emit(0, 0.5 * (0.2 * rr - 0.01));
    w = fmax(2.2250738585072014e-308, 0.1 / rr);
  } else {
    emit(0, 0.5 * s2);
  }
  const double wx = w * u.x, wy = w * u.y, wz = w * u.z;
  if (kd != 0) {
    const D3 av{fma(p.y, u.z, -p.z * u.y), fma(p.z, u.x, -p.x * u.z), fma(p.x, u.y, -p.y * u.x)};
    const double ax = w * av.x, ay = w * av.y, az = w * av.z;
    emit(1, wx * u.x); emit(2, wx * u.y); emit(3, wx * u.z);
    emit(4, wy * u.y); emit(5, wy * u.z); emit(6, wz * u.z);
    emit(7, ax * u.x); emit(8, ax * u.y); emit(9, ax * u.z);
    emit(10, ay * u.x); emit(11, ay * u.y); emit(12, ay * u.z);
    emit(13, az * u.x); emit(14, az * u.y); emit(15, az * u.z);
    emit(16, -ax * av.x); emit(17, -ax * av.y); emit(18, -ax * av.z);
    emit(19, -ay * av.y); emit(20, -ay * av.z); emit(21, -az * av.z);
    emit(22, rp * wx); emit(23, rp * wy); emit(24, rp * wz);
    emit(25, rp * ax); emit(26, rp * ay); emit(27, rp * az);
    return;
  }
  double m00, m01, m02, m11, m12, m22, v0, v1, v2;
  {
    const double wuu = w * fma(u.x, u.x, fma(u.y, u.y, u.z * u.z));
    m00 = fma(-wx, u.x, wuu); m01 = -wx * u.y; m02 = -wx * u.z;
    m11 = fma(-wy, u.y, wuu); m12 = -wy * u.z; m22 = fma(-wz, u.z, wuu);
    // v = w (u x r)
    v0 = w * fma(u.y, r2, -u.z * r1); v1 = w * fma(u.z, r0, -u.x * r2); v2 = w * fma(u.x, r1, -u.y * r0);
  }
  emit(1, m00); emit(2, m01); emit(3, m02); emit(4, m11); emit(5, m12); emit(6, m22);
  emit(22, v0); emit(23, v1); emit(24, v2);
  emit(25, fma(p.y, v2, -p.z * v1)); emit(26, fma(p.z, v0, -p.x * v2)); emit(27, fma(p.x, v1, -p.y * v0));
  // T = [p]x M row by row; U = T [p]x (symmetric): U[i][0] = T[i][1] pz - T[i][2] py,
  // U[i][1] = T[i][2] px - T[i][0] pz, U[i][2] = T[i][0] py - T[i][1] px
  {
    const double t0 = fma(-p.z, m01, p.y * m02), t1 = fma(-p.z, m11, p.y * m12), t2 = fma(-p.z, m12, p.y * m22);
    emit(7, t0); emit(8, t1); emit(9, t2);
    emit(16, fma(t1, p.z, -t2 * p.y));
    emit(17, fma(t2, p.x, -t0 * p.z));
    emit(18, fma(t0, p.y, -t1 * p.x));
  }
  {
    const double t0 = fma(p.z, m00, -p.x * m02), t1 = fma(p.z, m01, -p.x * m12), t2 = fma(p.z, m02, -p.x * m22);
    emit(10, t0); emit(11, t1); emit(12, t2);
    emit(19, fma(t2, p.x, -t0 * p.z));
    emit(20, fma(t0, p.y, -t1 * p.x));
  }
  {
    const double t0 = fma(-p.y, m00, p.x * m01), t1 = fma(-p.y, m01, p.x * m11), t2 = fma(-p.y, m02, p.x * m12);
    emit(13, t0); emit(14, t1); emit(15, t2);
    emit(21, fma(t0, p.y, -t1 * p.x));
  }
}
// The 28 sums of one block into a fresh s (zeros).
__device__ __forceinline__ void eng_block(int kd, const D3& c, const D3& pa, const D3& u, const double* R, const D3& t,
                                          double (&s)[kAcc]) {
  eng_block_emit(kd, c, pa, u, R, t, [&](int e, double v) { s[e] += v; });
}

// What an association item loads before its pass's x exists (all waves, while the lead waits):
// the wave's query point and, in the second outer pass, the first pass's matches of that query
// (closest / second / third, written by the pass-0 items) and their points.
struct ItemPre {
  P4 qp;
  int wi[3];
  P4 wp[3];
};
__device__ __forceinline__ ItemPre eng_item_pre(const OdomArgs& a, int k, int w, const int* warm, int outer) {
  ItemPre pre;
  const int ns = a.n_feat[k * 4 + 0], nf = a.n_feat[k * 4 + 2];
  const bool has = w < ns + nf;
  const bool corner = w < ns;
  const int t = corner ? w : w - ns;
  pre.qp = has ? ld4(corner ? reinterpret_cast<const P4*>(a.qpts_sharp) + (size_t)k * a.cap_sharp + t
                            : reinterpret_cast<const P4*>(a.qpts_flat) + (size_t)k * a.cap_flat + t)
               : P4{0.f, 0.f, 0.f, 0.f};
  const P4* L = corner ? a.less_sharp + (size_t)(k - 1) * a.cap_less_sharp : a.less_flat + (size_t)(k - 1) * a.N;
  const int nL = a.n_feat[(k - 1) * 4 + (corner ? 1 : 3)];
#pragma unroll
  for (int e = 0; e < 3; e++)
    pre.wi[e] = (has && outer == 1)
                    ? (int)__hip_atomic_load((gu32*)(warm + (size_t)w * 4 + e), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    : -1;
#pragma unroll
  for (int e = 0; e < 3; e++) pre.wp[e] = ld4(L + (pre.wi[e] >= 0 && pre.wi[e] < nL ? pre.wi[e] : 0));
  return pre;
}

// R (row-major rotation matrix of x's quaternion: qrot of the unit vectors) and t, in scalar
// registers (every lane holds them alike).
// (Eigen's Quaternion::toRotationMatrix: 22 flops, not three vector rotations; the evaluation only
// needs R to rounding, the association's TransformToStart keeps the reference's q * v.)
__device__ __forceinline__ void eng_rt_x(const double* xs, double (&R)[9], D3& t) {
  const double x = uniform_d(xs[0]), y = uniform_d(xs[1]), z = uniform_d(xs[2]), w = uniform_d(xs[3]);
  const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
  R[3] = txy + twz; R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1.0 - (txx + tyy);
  t = D3{uniform_d(xs[4]), uniform_d(xs[5]), uniform_d(xs[6])};
}
__device__ __forceinline__ void eng_rt(const EngShared& sh, double (&R)[9], D3& t) { eng_rt_x(sh.x, R, t); }

// One association item, one query per wave (the 64-lane searches nn_wave / line_search: every round
// trip looks at 64 candidates): query item * Q + wave of pair k, at the pass's x (each wave's
// own copy).  Faster than four 16-lane rows per wave when one chain's ~2000 queries are all the
// GPU runs (latency bound: 16.5 vs 34.9 us per round as separate launches).  The record goes out
// write-through; the wave's share of the solve's first evaluation (its block's 28 sums at x and
// the corner / plane counts) goes to sh.red[wave].
__device__ __forceinline__ void eng_query(const OdomArgs& a, EngShared& sh, int k, int w, Rsrc rec, int* warm, int outer,
                                          unsigned tk, const P4* pw, const int* pi, const double* x, double* row) {
  const unsigned long long tq0 = threadIdx.x == 0 ? rt_now() : 0ull;
  const int lane = lane_id();
  const int ns = a.n_feat[k * 4 + 0];
  const bool corner = w < ns;
  const P4 qp = pw[0];
  const TargetIndex& ix = corner ? a.idx_ls : a.idx_lf;
  const P4* L = corner ? a.less_sharp + (size_t)(k - 1) * a.cap_less_sharp : a.less_flat + (size_t)(k - 1) * a.N;
  const P4* sorted = reinterpret_cast<const P4*>(ix.sorted + (size_t)(k - 1) * ix.cap);
  const int nL = a.n_feat[(k - 1) * 4 + (corner ? 1 : 3)];
  const size_t mo = (size_t)(k - 1) * ix.nchunk * 2, so = (size_t)(k - 1) * ix.nsuper * 2;
  const P4 cur{qp.x, qp.y, qp.z, 0.f};
  const P4 sel = transform_to_start(cur, x);
  // Second outer pass: the first pass's closest / second / third points (pi / pw[1..3], loaded
  // before x existed into the wave's LDS slot) seed the searches (the pose moved little).  A seed is
  // one of the candidates of the minimum it seeds, so every result is unchanged; only the pruning
  // starts tighter.  The seeds (and x) are read from LDS where they are used, not held in
  // registers across the 1-NN search.
  dkey seed = kIdent;
#pragma unroll
  for (int e = 0; e < 3; e++) {
    const int wi = pi[e];
    const float d = d2f(sel, pw[1 + e]);
    if (wi >= 0 && wi < nL && d < 25.f) seed = dmin(seed, dk(d, wi));
  }
  const bool qlog = g_eng_qlog && g_eng_qlog_pair == k;
  const unsigned long long tq1 = (threadIdx.x == 0 || qlog) ? rt_now() : 0ull;
  const int closest = nn_wave(sorted, nL, ix.nn_chunk + mo, ix.nn_super + so, sel, seed);
  asm volatile("" ::: "memory");  // re-read the LDS seeds below rather than keep them live
  const unsigned long long tq2 = (threadIdx.x == 0 || qlog) ? rt_now() : 0ull;
  int kind = -1;
  D3 u{0.0, 0.0, 0.0};
  P4 pa{0.f, 0.f, 0.f, 0.f};
  int i2 = -1, i3 = -1;
  if (closest >= 0) {
    pa = ld4(L + closest);
    const int cid = int(pa.i);
    dkey s2 = dk(25.f, kNone), s3 = dk(25.f, kNone);
#pragma unroll
    for (int e = 0; e < 3; e++) {  // seeds of the walks (:467-520 / :589-646) under this closest
      const int j = pi[e];
      if (j < 0 || j >= nL || j == closest) continue;
      const P4 wpe = pw[1 + e];
      const int lab = int(wpe.i);
      const bool up = j > closest;
      if (up ? lab > cid + 2 : lab < cid - 2) continue;  // past the walk's break
      const float d = d2f(sel, wpe);
      if (!(d < 25.f)) continue;
      const dkey kd2 = dk(d, up ? j - closest : nL + closest - j);
      const bool other = up ? lab > cid : lab < cid;  // another scan line
      if (corner) {
        if (other) s2 = dmin(s2, kd2);
      } else {
        if (other) s3 = dmin(s3, kd2);
        else s2 = dmin(s2, kd2);
      }
    }
    LineSearch ls{L, ix.chunk + mo, nL, (nL + kChunk - 1) / kChunk, closest, cid, sel, s2, s3};
    if (corner) {  // LidarEdgeFactor(curr, a, b)
      line_search<true>(ls);
      if (dk_key(ls.b2) != kNone) {
        i2 = rank_to_index(ls, dk_key(ls.b2));
        const P4 pb = ld4(L + i2);
        const D3 de{(double)pa.x - (double)pb.x, (double)pa.y - (double)pb.y, (double)pa.z - (double)pb.z};
        const double inv = 1.0 / sqrt(de.x * de.x + de.y * de.y + de.z * de.z);
        u = D3{de.x * inv, de.y * inv, de.z * inv};
        kind = 0;
      }
    } else {        // LidarPlaneFactor(curr, j, l, m)
      line_search<false>(ls);
      if (dk_key(ls.b2) != kNone) i2 = rank_to_index(ls, dk_key(ls.b2));
      if (dk_key(ls.b3) != kNone) i3 = rank_to_index(ls, dk_key(ls.b3));
      if (i2 >= 0 && i3 >= 0) {
        const P4 pl = ld4(L + i2), pm = ld4(L + i3);
        u = plane_normal(D3{pa.x, pa.y, pa.z}, D3{pl.x, pl.y, pl.z}, D3{pm.x, pm.y, pm.z});
        kind = 1;
      }
    }
  }
  if (qlog && lane == 0) {
    int* ql = g_eng_qlog + ((size_t)outer * (a.cap_sharp + a.cap_flat) + w) * 4;
    ql[0] = (int)(tq2 - tq1);
    ql[1] = (int)(rt_now() - tq2);
    ql[2] = closest;
    ql[3] = kind + (corner ? 10 : 20);
  }
  if (threadIdx.x == 0) {
    const unsigned long long tq3 = rt_now();
    eng_prof(tk, 4, tq1 - tq0);  // transform, seeds
    eng_prof(tk, 5, tq2 - tq1);  // 1-NN
    eng_prof(tk, 6, tq3 - tq2);  // line searches + record
  }
  if (outer == 0 && lane < 3)  // seeds of the second pass (write-through: another workgroup reads them)
    __hip_atomic_store((gu32*)(warm + (size_t)w * 4 + lane), (unsigned)(lane == 0 ? closest : lane == 1 ? i2 : i3),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the record: four 16-B write-through stores (lanes 0..3) -- layout of rec_unpack.  All four even
  // without a correspondence (zeros): the evaluation weighs an absent block by 0, and 0 x a stale
  // non-finite word from an earlier use of the buffer would be NaN (a read-before-write)
  if (lane < 4) {
    v4u q;
    if (lane == 0) q = v4u{__float_as_uint(cur.x), __float_as_uint(cur.y), __float_as_uint(cur.z), __float_as_uint(pa.x)};
    else if (lane == 1) q = v4u{__float_as_uint(pa.y), __float_as_uint(pa.z), (unsigned)kind, 0u};
    else if (lane == 2) {
      const uint64_t ux = (uint64_t)__double_as_longlong(u.x), uy = (uint64_t)__double_as_longlong(u.y);
      q = v4u{(unsigned)ux, (unsigned)(ux >> 32), (unsigned)uy, (unsigned)(uy >> 32)};
    } else {
      const uint64_t uz = (uint64_t)__double_as_longlong(u.z);
      q = v4u{(unsigned)uz, (unsigned)(uz >> 32), 0u, 0u};
    }
    __builtin_amdgcn_raw_buffer_store_b128(q, rec, w * kRecBytes + lane * 16, 0, kAuxSc1);
  }
  // the share of the first evaluation, added to the wave's row sh.red[wave] (kind is wave-uniform;
  // every lane computes, lane 0 adds; a wave's LDS accesses stay in order)
  if (kind >= 0 && lane == 0) {  // one lane: each sum straight into the row (few doubles live)
    double R[9];
    D3 t;
    eng_rt_x(x, R, t);
    eng_block_emit(kind, D3{cur.x, cur.y, cur.z}, D3{pa.x, pa.y, pa.z}, u, R, t, [&](int e, double v) { row[e] += v; });
    row[28 + kind] += 1.0;
  }
}

// One association query per 16-lane row, four per wave (EngCtl::qpw = 4): the searches of the
// per-round schedule (nn16 / ls16: a round trip looks at 16 candidates per query) with eng_query's
// seeds, record, second-pass seeds and share.  A quarter of eng_query's waves per pass, so a pass's
// queries fit the resident item waves in one round and leave the SIMDs room for whatever runs
// beside the engine.  has: this row holds a query (w < the pair's queries).
__device__ __forceinline__ void eng_query16(const OdomArgs& a, int k, int w, bool has, Rsrc rec, int* warm, int outer,
                                            unsigned tk, const ItemPre& pre, const double* x, double* row) {
  const unsigned long long tq0 = threadIdx.x == 0 ? rt_now() : 0ull;
  const int lane = lane_id(), lr = lane & 15;
  const int ns = a.n_feat[k * 4 + 0];
  const bool corner = w < ns;
  const TargetIndex& ix = corner ? a.idx_ls : a.idx_lf;
  const P4* L = corner ? a.less_sharp + (size_t)(k - 1) * a.cap_less_sharp : a.less_flat + (size_t)(k - 1) * a.N;
  const P4* sorted = reinterpret_cast<const P4*>(ix.sorted + (size_t)(k - 1) * ix.cap);
  const int nL = a.n_feat[(k - 1) * 4 + (corner ? 1 : 3)];
  const size_t mo = (size_t)(k - 1) * ix.nchunk * 2, so = (size_t)(k - 1) * ix.nsuper * 2;
  const P4 cur{pre.qp.x, pre.qp.y, pre.qp.z, 0.f};
  const P4 sel = transform_to_start(cur, x);
  const int (&wi)[3] = pre.wi;
  const P4 (&wp)[3] = pre.wp;
  dkey seed = kIdent;  // the first pass's matches (second pass): candidates of the minimum they seed
#pragma unroll
  for (int e = 0; e < 3; e++) {
    const float d = d2f(sel, wp[e]);
    if (wi[e] >= 0 && wi[e] < nL && d < 25.f) seed = dmin(seed, dk(d, wi[e]));
  }
  const unsigned long long tq1 = threadIdx.x == 0 ? rt_now() : 0ull;
  const int closest = nn16(sorted, nL, ix.nn_chunk + mo, ix.nn_super + so, sel, has, seed);
  const unsigned long long tq2 = threadIdx.x == 0 ? rt_now() : 0ull;
  const bool act = has && closest >= 0;
  P4 pa = ld4(L + (act ? closest : 0));
  if (!act) pa = P4{0.f, 0.f, 0.f, 0.f};  // the record's defined zeros (no correspondence)
  const int cid = act ? int(pa.i) : 0;
  dkey b2 = dk(25.f, kNone), b3 = dk(25.f, kNone);
  if (act) {
#pragma unroll
    for (int e = 0; e < 3; e++) {  // seeds of the walks under this closest (as eng_query)
      const int j = wi[e];
      if (j < 0 || j >= nL || j == closest) continue;
      const int lab = int(wp[e].i);
      const bool up = j > closest;
      if (up ? lab > cid + 2 : lab < cid - 2) continue;
      const float d = d2f(sel, wp[e]);
      if (!(d < 25.f)) continue;
      const dkey kd2 = dk(d, up ? j - closest : nL + closest - j);
      const bool other = up ? lab > cid : lab < cid;
      if (corner) {
        if (other) b2 = dmin(b2, kd2);
      } else {
        if (other) b3 = dmin(b3, kd2);
        else b2 = dmin(b2, kd2);
      }
    }
  }
  ls16(L, ix.chunk + mo, nL, act ? closest : 0, cid, sel, corner, act, b2, b3);
  auto idx_of = [&](dkey b) { const int kk = dk_key(b); return kk < nL ? closest + kk : closest - (kk - nL); };
  int kind = -1, i2 = -1, i3 = -1;
  D3 u{0.0, 0.0, 0.0};
  if (act && dk_key(b2) != kNone) i2 = idx_of(b2);
  if (act && !corner && dk_key(b3) != kNone) i3 = idx_of(b3);
  if (act && corner && i2 >= 0) {  // LidarEdgeFactor(curr, a, b)
    const P4 pb = ld4(L + i2);
    const D3 de{(double)pa.x - (double)pb.x, (double)pa.y - (double)pb.y, (double)pa.z - (double)pb.z};
    const double inv = 1.0 / sqrt(de.x * de.x + de.y * de.y + de.z * de.z);
    u = D3{de.x * inv, de.y * inv, de.z * inv};
    kind = 0;
  } else if (act && !corner && i2 >= 0 && i3 >= 0) {  // LidarPlaneFactor(curr, j, l, m)
    const P4 pl = ld4(L + i2), pm = ld4(L + i3);
    u = plane_normal(D3{pa.x, pa.y, pa.z}, D3{pl.x, pl.y, pl.z}, D3{pm.x, pm.y, pm.z});
    kind = 1;
  }
  if (threadIdx.x == 0) {  // the wave's four queries together (developer profile)
    const unsigned long long tq3 = rt_now();
    eng_prof(tk, 4, tq1 - tq0);
    eng_prof(tk, 5, tq2 - tq1);
    eng_prof(tk, 6, tq3 - tq2);
  }
  if (has && outer == 0 && lr < 3)  // seeds of the second pass (write-through: another workgroup reads them)
    __hip_atomic_store((gu32*)(warm + (size_t)w * 4 + lr), (unsigned)(lr == 0 ? closest : lr == 1 ? i2 : i3),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the record (rec_unpack's layout): lanes 0..3 of the row, 16 B each, all four always (eng_query)
  if (has && lr < 4) {
    v4u q;
    if (lr == 0) q = v4u{__float_as_uint(cur.x), __float_as_uint(cur.y), __float_as_uint(cur.z), __float_as_uint(pa.x)};
    else if (lr == 1) q = v4u{__float_as_uint(pa.y), __float_as_uint(pa.z), (unsigned)kind, 0u};
    else if (lr == 2) {
      const uint64_t ux = (uint64_t)__double_as_longlong(u.x), uy = (uint64_t)__double_as_longlong(u.y);
      q = v4u{(unsigned)ux, (unsigned)(ux >> 32), (unsigned)uy, (unsigned)(uy >> 32)};
    } else {
      const uint64_t uz = (uint64_t)__double_as_longlong(u.z);
      q = v4u{(unsigned)uz, (unsigned)(uz >> 32), 0u, 0u};
    }
    __builtin_amdgcn_raw_buffer_store_b128(q, rec, w * kRecBytes + lr * 16, 0, kAuxSc1);
  }
  // the rows' shares of the first evaluation: every lane of a row computes its row's block, and lane
  // 0 adds the four rows' sums (rows 0 + 1, 2 + 3, then the two) to the wave's row of sh.red
  double sb[kAcc];
#pragma unroll
  for (int e = 0; e < kAcc; e++) sb[e] = 0.0;
  if (kind >= 0) {
    double R[9];
    D3 t;
    eng_rt_x(x, R, t);
    eng_block(kind, D3{cur.x, cur.y, cur.z}, D3{pa.x, pa.y, pa.z}, u, R, t, sb);
  }
  const uint64_t mc = __ballot(lr == 0 && kind == 0), mp = __ballot(lr == 0 && kind == 1);
  auto rd = [](double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(unsigned)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)(unsigned)hi << 32) | (unsigned)lo));
  };
  double tot[kAcc];
#pragma unroll
  for (int e = 0; e < kAcc; e++) tot[e] = (rd(sb[e], 0) + rd(sb[e], 16)) + (rd(sb[e], 32) + rd(sb[e], 48));
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < kAcc; e++) row[e] += tot[e];
    row[28] += (double)__builtin_popcountll(mc);
    row[29] += (double)__builtin_popcountll(mp);
  }
}

// A bounds check of the engine's own index arithmetic (the rows it publishes, the records it
// writes): a violation raises this launch's abort (and the sticky word) with `code` in the error
// word instead of faulting, so the host re-runs the launch on the per-round schedule and the code
// says which check fired.  Wave-uniform operands only.
__device__ __forceinline__ bool eng_check(const EngCtl& ctl, bool ok, unsigned code) {
  if (ok) return true;
  if (lane_id() == 0) {
    st_rlx(ctl.w + 2, code);
    st_rlx(ctl.abort_w(), 1u);
    st_rlx(ctl.w + 3, 1u);
  }
  return false;
}

// One association item: wave wv of item `item` takes queries (item + m ieff) qpi + wv qpw + s,
// s < qpw (four 16-lane rows at once when qpw = 4, else one 64-lane query after another), m = 0,
// 1, ...: one round while the pair's queries fit ieff items (the common case), more when the pair
// holds more queries than the engine keeps items in flight (EngCtl::budget), so that no item waits
// for a workgroup to come free.  The wave's share of the first evaluation (its blocks' 28 sums at
// x, and the corner / plane counts) goes to sh.red[wave].
template <int kQpw>
__device__ __forceinline__ void eng_item_run(const OdomArgs& a, const EngCtl& ctl, EngShared& sh, int k, int item,
                                             const PassShape& ps, Rsrc rec, int* warm, int outer, unsigned tk) {
  const int ql = (int)(threadIdx.x >> 6);
  const int row = kQpw == 4 ? lane_id() >> 4 : 0;
  const int ieff = ps.ieff;
  const int nq = a.n_feat[k * 4 + 0] + a.n_feat[k * 4 + 2];
  if (lane_id() < 30) sh.red[ql][lane_id()] = 0.0;
  // the pass's x stays in the wave's LDS copy: read where a query needs it (its transform, its
  // share), not held in 14 VGPRs across the searches
  const double* x = sh.xw[ql];
  for (int m = 0;; m++) {
    const int w0 = (item + m * ieff) * ctl.Q * kQpw + ql * kQpw;  // the wave's first query
    if (w0 >= nq) break;  // wave-uniform
    if constexpr (kQpw == 4) {
      const int w = w0 + row;
      ItemPre pre;
      if (m > 0) {
        pre = eng_item_pre(a, k, w, warm, outer);
      } else {  // loaded before x existed, parked in this wave's LDS slots
        pre.qp = sh.prew[ql][row][0];
#pragma unroll
        for (int e = 0; e < 3; e++) { pre.wp[e] = sh.prew[ql][row][1 + e]; pre.wi[e] = sh.prei[ql][row][e]; }
      }
      eng_query16(a, k, w, w < nq, rec, warm, outer, tk, pre, x, sh.red[ql]);
    } else {
      for (int s = 0; s < kQpw; s++) {  // the wave's queries one after another (slot s: parked by row s)
        const int w = w0 + s;
        if (w >= nq) break;  // wave-uniform
        if (m > 0) {  // an overflow query: its loads parked in the slot now (a wave's LDS accesses stay in order)
          const ItemPre pre = eng_item_pre(a, k, w, warm, outer);
          if (lane_id() == 0) {
            sh.prew[ql][s][0] = pre.qp;
#pragma unroll
            for (int e = 0; e < 3; e++) { sh.prew[ql][s][1 + e] = pre.wp[e]; sh.prei[ql][s][e] = pre.wi[e]; }
          }
        }
        eng_query(a, sh, k, w, rec, warm, outer, tk, sh.prew[ql][s], sh.prei[ql][s], x, sh.red[ql]);
      }
    }
  }
  if (lane_id() == 0) eng_prof(tk, 10, rt_now());
}

// The 28 sums of every thread -> sh.acc in lislam_lm.hpp's layout (cost, H upper, g).  Inside each
// 16-lane row a reduce-scatter: xor 1 / xor 2 (quad_perm) halve the values each lane carries
// (lane i of an 8-lane group keeps part(i), part(7 - i) == part(i)), the half- and full-row mirrors
// then pair lanes holding the same part; lanes 0..3 of each row write their 7 sums to LDS.
// sum index e of eng_block -> index in lislam_lm.hpp's acc (H upper row-major over (theta 0..2,
// t 0..2), then g) and its scale: cost; M -> H_tt; T -> H_theta,t = 2 T; U -> H_theta,theta = -4 U;
// v -> g_t; p x v -> g_theta = 2 p x v
__device__ __forceinline__ int acc_index(int e, double* scale) {
  *scale = e == 0 ? 1.0 : e <= 6 ? 1.0 : e <= 15 ? 2.0 : e <= 21 ? -4.0 : e <= 24 ? 1.0 : 2.0;
  // H upper index (lislam_lm.hpp: 1 + pu(i, j)) of the (i, j) each group of sums fills; arithmetic,
  // not a table in memory (a divergent load on the reduction's critical path)
  auto pu1 = [](int i, int j) { return 1 + i * 6 - i * (i - 1) / 2 + (j - i); };
  auto upper = [](int q, int& i, int& j) {  // q-th entry of a 3x3 upper triangle, row-major
    i = q < 3 ? 0 : q < 5 ? 1 : 2;
    j = i + q - (i == 0 ? 0 : i == 1 ? 3 : 5);
  };
  int i, j;
  if (e == 0) return 0;
  if (e <= 6) { upper(e - 1, i, j); return pu1(3 + i, 3 + j); }  // M -> H_tt
  if (e <= 15) return pu1((e - 7) / 3, 3 + (e - 7) % 3);           // T -> H_theta,t
  if (e <= 21) { upper(e - 16, i, j); return pu1(i, j); }          // U -> H_theta,theta
  return e <= 24 ? e + 3 : e - 3;                                   // v -> g_t, p x v -> g_theta
}

// Sum of a double over the four 16-lane rows of the wave (every lane gets its column's sum):
// v_permlane16_swap / v_permlane32_swap pair rows (0,1)(2,3), then halves, without LDS.
__device__ __forceinline__ double rows_sum(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  auto lo16 = __builtin_amdgcn_permlane16_swap((uint32_t)u, (uint32_t)u, false, false);
  auto hi16 = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  v = __longlong_as_double((long long)(((uint64_t)hi16[0] << 32) | lo16[0])) +
      __longlong_as_double((long long)(((uint64_t)hi16[1] << 32) | lo16[1]));
  const uint64_t w = (uint64_t)__double_as_longlong(v);
  auto lo32 = __builtin_amdgcn_permlane32_swap((uint32_t)w, (uint32_t)w, false, false);
  auto hi32 = __builtin_amdgcn_permlane32_swap((uint32_t)(w >> 32), (uint32_t)(w >> 32), false, false);
  return __longlong_as_double((long long)(((uint64_t)hi32[0] << 32) | lo32[0])) +
         __longlong_as_double((long long)(((uint64_t)hi32[1] << 32) | lo32[1]));
}

// Inside each 16-lane row: o[7] = the row's sums 14 (part & 1) + 7 (part >> 1) + [0, 7).
__device__ __forceinline__ int row_reduce_scatter28(const double (&s)[kAcc], double (&o)[7]) {
  const int lane = lane_id(), i8 = lane & 7;
  const int part = (i8 & 4) ? (~i8 & 3) : (i8 & 3);
  const bool h1 = part & 1, h2 = (part >> 1) & 1;
  double h[14];
#pragma unroll
  for (int q = 0; q < 14; q++) {
    const double snd = h1 ? s[q] : s[q + 14];
    const double kp = h1 ? s[q + 14] : s[q];
    h[q] = kp + dpp_d<0xB1>(snd);
  }
#pragma unroll
  for (int q = 0; q < 7; q++) {
    const double snd = h2 ? h[q] : h[q + 7];
    const double kp = h2 ? h[q + 7] : h[q];
    o[q] = kp + dpp_d<0x4E>(snd);
  }
#pragma unroll
  for (int q = 0; q < 7; q++) o[q] += dpp_d<0x141>(o[q]);
#pragma unroll
  for (int q = 0; q < 7; q++) o[q] += dpp_d<0x140>(o[q]);
  return part;
}

__device__ __forceinline__ int part_base(int part) { return 14 * (part & 1) + 7 * (part >> 1); }

// ---- the evaluation: blocks in the evaluating waves' registers, typed slots
// Waves 1.. of the solve hold the pass's residual blocks in registers, loaded once per pass, in
// slots of a fixed kind: thread tp's edge slots are corner queries tp + kEvalThreads s, its plane
// slots surf queries ns + tp + kEvalThreads s.  The block formulas are branch-free (the Huber
// weight by selects; a missing correspondence weighs 0), so the slots' dependent chains
// interleave.  Queries beyond the slots (H > 64 lines) are read from the records at each
// evaluation.
constexpr int kEvalThreads = kEngThreads - 64;
constexpr int kEdgeSlots = 2;   // 896 >= 12 * 64 corner queries
constexpr int kPlaneSlots = 4;  // 1792 >= 24 * 64 surf queries

struct BlkReg {
  float c[3], a[3];  // query point, first matched point a (edge) / j (plane)
  double u[3];       // edge: u = (a - b) / |a - b|; plane: unit normal
  int kd;            // 0 edge, 1 plane, -1 none
};

__device__ __forceinline__ void rec_unpack(const v4u& q0, const v4u& q1, const v4u& q2, const v4u& q3, BlkReg& b) {
  b.c[0] = __uint_as_float(q0.x); b.c[1] = __uint_as_float(q0.y); b.c[2] = __uint_as_float(q0.z);
  b.a[0] = __uint_as_float(q0.w); b.a[1] = __uint_as_float(q1.x); b.a[2] = __uint_as_float(q1.y);
  b.kd = (int)q1.z;
  b.u[0] = __longlong_as_double((long long)(((uint64_t)q2.y << 32) | q2.x));
  b.u[1] = __longlong_as_double((long long)(((uint64_t)q2.w << 32) | q2.z));
  b.u[2] = __longlong_as_double((long long)(((uint64_t)q3.y << 32) | q3.x));
}
// Record w (ok) or a copy of record 0 marked absent: unconditional 16-B loads, no branches.
__device__ __forceinline__ void rec_load(Rsrc rec, int w, bool ok, BlkReg& b) {
  const int off = (ok ? w : 0) * kRecBytes;
  const v4u q0 = __builtin_amdgcn_raw_buffer_load_b128(rec, off, 0, kAuxSc1);
  const v4u q1 = __builtin_amdgcn_raw_buffer_load_b128(rec, off + 16, 0, kAuxSc1);
  const v4u q2 = __builtin_amdgcn_raw_buffer_load_b128(rec, off + 32, 0, kAuxSc1);
  const v4u q3 = __builtin_amdgcn_raw_buffer_load_b128(rec, off + 48, 0, kAuxSc1);
  rec_unpack(q0, q1, q2, q3, b);
  if (!ok) b.kd = -1;
}

// HuberLoss(0.1) of s2 = |r|^2: the cost term 0.5 rho and the corrector weight rho' (rho = 2 a
// sqrt(s) - a^2, rho' = a / sqrt(s) above a^2), both 0 for an absent block; selects, no branches.
__device__ __forceinline__ void huber_sel(double s2, bool live, double& w, double& cterm) {
  const bool big = s2 > 0.01;
  const double rs = rsqrt_d(big ? s2 : 1.0);
  cterm = live ? (big ? 0.5 * fma(0.2 * s2, rs, -0.01) : 0.5 * s2) : 0.0;
  w = live ? (big ? fmax(2.2250738585072014e-308, 0.1 * rs) : 1.0) : 0.0;
}

__device__ __forceinline__ D3 rot_rc(const double* R, const float* c) {
  const double cx = c[0], cy = c[1], cz = c[2];
  return D3{fma(R[0], cx, fma(R[1], cy, R[2] * cz)), fma(R[3], cx, fma(R[4], cy, R[5] * cz)),
            fma(R[6], cx, fma(R[7], cy, R[8] * cz))};
}

// LidarEdgeFactor block (eng_block's edge form, branch-free).
__device__ __forceinline__ void eng_edge_sel(const BlkReg& b, const double* R, const D3& t, double (&s)[kAcc]) {
  const D3 p = rot_rc(R, b.c);
  const D3 u{b.u[0], b.u[1], b.u[2]};
  const D3 e{(p.x + t.x) - (double)b.a[0], (p.y + t.y) - (double)b.a[1], (p.z + t.z) - (double)b.a[2]};
  const double r0 = fma(e.y, u.z, -e.z * u.y), r1 = fma(e.z, u.x, -e.x * u.z), r2 = fma(e.x, u.y, -e.y * u.x);
  double w, ct;
  huber_sel(fma(r0, r0, fma(r1, r1, r2 * r2)), b.kd >= 0, w, ct);
  s[0] += ct;
  const double wx = w * u.x, wy = w * u.y, wz = w * u.z;
  const double wuu = w * fma(u.x, u.x, fma(u.y, u.y, u.z * u.z));
  const double m00 = fma(-wx, u.x, wuu), m01 = -wx * u.y, m02 = -wx * u.z;
  const double m11 = fma(-wy, u.y, wuu), m12 = -wy * u.z, m22 = fma(-wz, u.z, wuu);
  const double v0 = w * fma(u.y, r2, -u.z * r1), v1 = w * fma(u.z, r0, -u.x * r2), v2 = w * fma(u.x, r1, -u.y * r0);
  s[1] += m00; s[2] += m01; s[3] += m02; s[4] += m11; s[5] += m12; s[6] += m22;
  s[22] += v0; s[23] += v1; s[24] += v2;
  s[25] += fma(p.y, v2, -p.z * v1); s[26] += fma(p.z, v0, -p.x * v2); s[27] += fma(p.x, v1, -p.y * v0);
  {
    const double t0 = fma(-p.z, m01, p.y * m02), t1 = fma(-p.z, m11, p.y * m12), t2 = fma(-p.z, m12, p.y * m22);
    s[7] += t0; s[8] += t1; s[9] += t2;
    s[16] += fma(t1, p.z, -t2 * p.y);
    s[17] += fma(t2, p.x, -t0 * p.z);
    s[18] += fma(t0, p.y, -t1 * p.x);
  }
  {
    const double t0 = fma(p.z, m00, -p.x * m02), t1 = fma(p.z, m01, -p.x * m12), t2 = fma(p.z, m02, -p.x * m22);
    s[10] += t0; s[11] += t1; s[12] += t2;
    s[19] += fma(t2, p.x, -t0 * p.z);
    s[20] += fma(t0, p.y, -t1 * p.x);
  }
  {
    const double t0 = fma(-p.y, m00, p.x * m01), t1 = fma(-p.y, m01, p.x * m11), t2 = fma(-p.y, m02, p.x * m12);
    s[13] += t0; s[14] += t1; s[15] += t2;
    s[21] += fma(t0, p.y, -t1 * p.x);
  }
}

// LidarPlaneFactor block (eng_block's plane form, branch-free).
__device__ __forceinline__ void eng_plane_sel(const BlkReg& b, const double* R, const D3& t, double (&s)[kAcc]) {
  const D3 p = rot_rc(R, b.c);
  const D3 u{b.u[0], b.u[1], b.u[2]};
  const D3 e{(p.x + t.x) - (double)b.a[0], (p.y + t.y) - (double)b.a[1], (p.z + t.z) - (double)b.a[2]};
  const double rp = fma(e.x, u.x, fma(e.y, u.y, e.z * u.z));
  double w, ct;
  huber_sel(rp * rp, b.kd >= 0, w, ct);
  s[0] += ct;
  const double wx = w * u.x, wy = w * u.y, wz = w * u.z;
  const D3 av{fma(p.y, u.z, -p.z * u.y), fma(p.z, u.x, -p.x * u.z), fma(p.x, u.y, -p.y * u.x)};
  const double ax = w * av.x, ay = w * av.y, az = w * av.z;
  s[1] = fma(wx, u.x, s[1]); s[2] = fma(wx, u.y, s[2]); s[3] = fma(wx, u.z, s[3]);
  s[4] = fma(wy, u.y, s[4]); s[5] = fma(wy, u.z, s[5]); s[6] = fma(wz, u.z, s[6]);
  s[7] = fma(ax, u.x, s[7]); s[8] = fma(ax, u.y, s[8]); s[9] = fma(ax, u.z, s[9]);
  s[10] = fma(ay, u.x, s[10]); s[11] = fma(ay, u.y, s[11]); s[12] = fma(ay, u.z, s[12]);
  s[13] = fma(az, u.x, s[13]); s[14] = fma(az, u.y, s[14]); s[15] = fma(az, u.z, s[15]);
  s[16] = fma(-ax, av.x, s[16]); s[17] = fma(-ax, av.y, s[17]); s[18] = fma(-ax, av.z, s[18]);
  s[19] = fma(-ay, av.y, s[19]); s[20] = fma(-ay, av.z, s[20]); s[21] = fma(-az, av.z, s[21]);
  s[22] = fma(rp, wx, s[22]); s[23] = fma(rp, wy, s[23]); s[24] = fma(rp, wz, s[24]);
  s[25] = fma(rp, ax, s[25]); s[26] = fma(rp, ay, s[26]); s[27] = fma(rp, az, s[27]);
}

struct EvalSlots {
  BlkReg e[kEdgeSlots], p[kPlaneSlots];
  bool tail;  // wave-uniform: a lane of this wave holds a block in edge slot 1 or plane slot 3
};

__device__ __forceinline__ void eval_slots_load(Rsrc rec, int ns, int nf, int tp, EvalSlots& S) {
#pragma unroll
  for (int k = 0; k < kEdgeSlots; k++) {
    const int w = tp + k * kEvalThreads;
    rec_load(rec, w, w < ns, S.e[k]);
  }
#pragma unroll
  for (int k = 0; k < kPlaneSlots; k++) {
    const int q = tp + k * kEvalThreads;
    rec_load(rec, ns + q, q < nf, S.p[k]);
  }
  S.tail = __ballot(tp + kEvalThreads < ns || tp + 3 * kEvalThreads < nf) != 0ull;
}

// One evaluation at sh.x by the evaluating waves; each wave's 28 sums go to its row sh.red[wave]
// (lanes 0..3 write 7 each: the reduce-scatter of row_reduce_scatter28, then rows_sum).
__device__ __forceinline__ void eng_eval_slots(EngShared& sh, const EvalSlots& S, Rsrc rec, int ns, int nf, int tp) {
  double s[kAcc];
#pragma unroll
  for (int e = 0; e < kAcc; e++) s[e] = 0.0;
  double R[9];
  D3 t;
  eng_rt(sh, R, t);
  eng_edge_sel(S.e[0], R, t, s);
  eng_plane_sel(S.p[0], R, t, s);
  eng_plane_sel(S.p[1], R, t, s);
  eng_plane_sel(S.p[2], R, t, s);
  if (S.tail) {
    eng_edge_sel(S.e[1], R, t, s);
    eng_plane_sel(S.p[3], R, t, s);
  }
  // beyond the slots (H > 64 lines): from the records
  for (int w = tp + kEdgeSlots * kEvalThreads; w < ns; w += kEvalThreads) {
    BlkReg b;
    rec_load(rec, w, true, b);
    eng_edge_sel(b, R, t, s);
  }
  for (int q = tp + kPlaneSlots * kEvalThreads; q < nf; q += kEvalThreads) {
    BlkReg b;
    rec_load(rec, ns + q, true, b);
    eng_plane_sel(b, R, t, s);
  }
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  double o[7];
  const int part = row_reduce_scatter28(s, o);
#pragma unroll
  for (int q = 0; q < 7; q++) o[q] = rows_sum(o[q]);  // the wave's sums of part(lane)
  if (lane < 4) {
    const int base = part_base(part);
#pragma unroll
    for (int q = 0; q < 7; q++) sh.red[wv][base + q] = o[q];
  }
}

// Wave 0, after the evaluating waves' rows are in: acc (lislam_lm.hpp layout) in every lane.
__device__ __forceinline__ void eng_gather_rows(EngShared& sh, double (&acc)[kAcc]) {
  const int lane = lane_id();
  if (lane < kAcc) {
    double r[kEngWaves - 1];
#pragma unroll
    for (int w = 1; w < kEngWaves; w++) r[w - 1] = sh.red[w][lane];
    // pairwise tree over the rows (independent adds, not a serial chain)
#pragma unroll
    for (int h = 1; h < kEngWaves - 1; h <<= 1)
#pragma unroll
      for (int w = 0; w + h < kEngWaves - 1; w += 2 * h) r[w] += r[w + h];
    double sc;
    const int ai = acc_index(lane, &sc);
    sh.acc[ai] = sc * r[0];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int e = 0; e < kAcc; e++) acc[e] = sh.acc[e];
}


// ---- the solve role: one workgroup per chain, for the whole chain
// Pass ro = 2 r + o of chain c (pair k): gather its association items' records and shares of the
// first evaluation, then the LM loop (wave 0 steps, waves 1.. evaluate; 1 + 2 barriers per
// iteration), then publish x (para_q / para_t, write-through) and lm_gen[c] = ro + 1.  The chain's
// x and pose stay in LDS.
//
// The solve's gather: wait for every item of the pass (the assoc_done count), then load every
// item's share row at once (summed in a fixed tree) and, while wave 0 takes step 0 from the shares,
// the records into the evaluating waves' slots.
constexpr int kShareQuads = 15;  // doubles 0..29 of an item's row: 28 sums + 2 counts

__device__ __forceinline__ bool eng_solve_pass(const OdomArgs& a, const EngCtl& ctl, EngShared& sh, EngLM& lm,
                                               int c, int k, int ro, const PassShape& ps, Rsrc rec, bool wave0, unsigned tk) {
  const int ns = a.n_feat[k * 4 + 0], nf = a.n_feat[k * 4 + 2];
  const int lane = lane_id();
  const int tp = (int)threadIdx.x - 64;
  const int ieff = ps.ieff;
  EvalSlots S;
  const int q = threadIdx.x & 15, g = threadIdx.x >> 4;  // share quad q of rows g, g + 32, ..., g + 224
  double d0[8], d1[8];
  {  // the items' rows (the records follow while wave 0 takes step 0: it needs only the shares)
    const Rsrc parts = make_rsrc(part_row(a, ctl, c, 0), (unsigned)(ctl.P * 256));
    v4u v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int it = g + 32 * j;
      v[j] = __builtin_amdgcn_raw_buffer_load_b128(parts, (it < ieff ? it : 0) * 256 + q * 16, 0, kAuxSc1);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const bool ok = g + 32 * j < ieff && q < kShareQuads;
      d0[j] = ok ? __longlong_as_double((long long)(((uint64_t)v[j].y << 32) | v[j].x)) : 0.0;
      d1[j] = ok ? __longlong_as_double((long long)(((uint64_t)v[j].w << 32) | v[j].z)) : 0.0;
    }
  }
  {  // the rows' shares: pairwise tree over rows g + 32 j, then (wave 0) over the 32 sums
#pragma unroll
    for (int h = 1; h < 8; h <<= 1)
#pragma unroll
      for (int j = 0; j + h < 8; j += 2 * h) { d0[j] += d0[j + h]; d1[j] += d1[j + h]; }
    if (q < kShareQuads) { sh.red[g][2 * q] = d0[0]; sh.red[g][2 * q + 1] = d1[0]; }
  }
  __syncthreads();
  LdsLM& s = *(LdsLM*)&lm;
  // Two loops, one per role, each with the same barriers (1 + 2 per LM iteration): the slots exist
  // only in the evaluating waves' loop and the step's working set only in wave 0's, so neither is
  // live across the other (the branch is wave-uniform; s_barrier counts waves).
  if (wave0) {
    const unsigned long long tf0 = rt_now();
    if (lane < 30) {  // the 32 rows of shares: pairwise tree
      double r[32];
#pragma unroll
      for (int w = 0; w < 32; w++) r[w] = sh.red[w][lane];
#pragma unroll
      for (int h = 1; h < 32; h <<= 1)
#pragma unroll
        for (int w = 0; w + h < 32; w += 2 * h) r[w] += r[w + h];
      if (lane < kAcc) {
        double sc;
        const int ai = acc_index(lane, &sc);
        sh.acc[ai] = sc * r[0];
      } else {
        sh.cnt[0][lane - kAcc] = (int)r[0];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const unsigned long long tfa = rt_now();  // the shares summed
    const int nc = uni(sh.cnt[0][0]), np = uni(sh.cnt[0][1]);
    bool cont = false;
    if (nc + np > 0) {  // no residual blocks: Ceres leaves the parameters untouched
      double acc[kAcc], x0[7];
#pragma unroll
      for (int e = 0; e < kAcc; e++) acc[e] = sh.acc[e];
#pragma unroll
      for (int e = 0; e < 7; e++) { x0[e] = sh.cx[e]; sh.x[e] = x0[e]; }
      cont = eng_step(s, x0, acc, true, a.max_iterations);  // step 0 while the records land
      if (cont)
#pragma unroll
        for (int e = 0; e < 7; e++) sh.x[e] = s.xc[e];
    }
    if (lane == 0) { sh.flag = cont; sh.nc = nc; sh.np = np; }
    const unsigned long long tf1 = rt_now();
    __syncthreads();
    if (lane == 0) {
      eng_prof(tk, 0, tf1 - tf0);          // step 0 (wave 0)
      eng_prof(tk, 11, tfa - tf0);         // ... of which the shares' sum
      eng_prof(tk, 7, rt_now() - tf0);     // step 0 and the blocks' load (to the first barrier)
      eng_prof(tk, 2, tf0);                // shares summed
    }
    bool more = uni(sh.flag) != 0;
    while (more) {
      const unsigned long long t0 = rt_now();
      eng_step_post(s);  // while the candidate is evaluated
      __syncthreads();
      double acc[kAcc];
      eng_gather_rows(sh, acc);
      const unsigned long long t2 = rt_now();
      const bool c2 = eng_step(s, nullptr, acc, false, a.max_iterations);
      if (c2)
#pragma unroll
        for (int e = 0; e < 7; e++) sh.x[e] = s.xc[e];
      if (lane == 0) {
        sh.flag = c2;
        eng_prof(tk, 4, t2 - t0, true);  // evaluation (wave 0's view: barrier to barrier) + the rows' sums
        eng_prof(tk, 5, rt_now() - t2, true);  // step
        eng_prof(tk, 6, 1ull, true);
      }
      __syncthreads();
      more = uni(sh.flag) != 0;
    }
  } else {
    // the records not loaded yet, while wave 0 takes step 0
    if (ieff > 0) eval_slots_load(rec, ns, nf, tp, S);
    __syncthreads();
    bool more = uni(sh.flag) != 0;
    while (more) {
      eng_eval_slots(sh, S, rec, ns, nf, tp);  // cost + J^T J + J^T r at the candidate
      __syncthreads();
      __syncthreads();  // wave 0's step
      more = uni(sh.flag) != 0;
    }
  }
  return true;
}

// The solve role of chain c (ticket c): every pass of the chain, in order.  false = aborted.
__device__ __forceinline__ bool eng_solve_role(const OdomArgs& a, const EngCtl& ctl, EngShared& sh, EngLM& lm, int c,
                                               bool wave0, unsigned tk) {
  const int lane = lane_id();
  const size_t rec_stride = (size_t)(a.cap_sharp + a.cap_flat) * 9;  // doubles per chain (a.blk)
  const Rsrc rec = make_rsrc(a.blk + (size_t)c * rec_stride, (unsigned)((a.cap_sharp + a.cap_flat) * kRecBytes));
  double* st = a.state + (size_t)c * 16;
  if (wave0 && lane < 7) {  // the chain's x (para) and pose at its first scan
    sh.cx[lane] = a.init_state ? a.init_state[(size_t)c * 14 + lane] : (lane == 3 ? 1.0 : 0.0);
    sh.cpw[lane] = a.init_state ? a.init_state[(size_t)c * 14 + 7 + lane] : (lane == 3 ? 1.0 : 0.0);
  }
  if (wave0 && lane == 0 && c == 0 && !a.init_state) {  // scan 0 of the batch: first frame
    for (int e = 0; e < 7; e++) { a.para[e] = e == 3 ? 1.0 : 0.0; a.pose[e] = e == 3 ? 1.0 : 0.0; }
    for (int e = 0; e < 8; e++) a.stats[e] = 0;
  }
  for (int ro = 0; ro < 2 * ctl.R; ro++) {
    const int r = ro >> 1, o = ro & 1;
    int k;
    if (!pair_of(a, c, r, &k)) break;  // uniform: this chain is shorter
    const PassShape ps = pass_shape(a, ctl, k);
    const int ieff = ps.ieff;
    const unsigned ptk = (unsigned)(ro * ctl.C * (ctl.I + 1)) + tk;  // profile slot of the pass (developer builds)
    if (wave0 && lane == 0) {
      eng_prof(ptk, 1, rt_now());
      sh.flag0 = ieff > 0 ? eng_wait(ctl.assoc_done(c, ro), (unsigned)ieff, ctl.abort_w(), ctl.wait_ticks, 3u, ctl.backoff) : 1;
      eng_prof(ptk, 1, rt_now());
    }
    __syncthreads();
    if (!uni(sh.flag0)) return false;
    if (!eng_solve_pass(a, ctl, sh, lm, c, k, ro, ps, rec, wave0, ptk)) return false;
    if (wave0 && lane == 0) {
      const int nc = sh.nc, np = sh.np;
      int* so = a.stats + (size_t)k * 8;
      so[o * 2 + 0] = nc;
      so[o * 2 + 1] = np;
      so[4 + o] = (nc + np) > 0 ? lm.it : 0;
      so[6 + o] = (nc + np) > 0 ? lm.term : 1;
      double xs[7];
#pragma unroll
      for (int e = 0; e < 7; e++) xs[e] = (nc + np) > 0 ? lm.x[e] : sh.cx[e];  // unchanged without blocks
#pragma unroll
      for (int e = 0; e < 7; e++) st_sc1d(st + e, xs[e]);  // the next pass's items start from it
      drain_stores();
      st_rlx(ctl.lm_gen(c), (unsigned)(ro + 1));
#pragma unroll
      for (int e = 0; e < 7; e++) sh.cx[e] = xs[e];
      if (o == 1) {
        // t_w_curr = t_w_curr + q_w_curr * t_last_curr; q_w_curr = q_w_curr * q_last_curr (:716-717)
        DQ qw{sh.cpw[0], sh.cpw[1], sh.cpw[2], sh.cpw[3]};
        D3 tw{sh.cpw[4], sh.cpw[5], sh.cpw[6]};
        tw = tw + qrot(qw, D3{xs[4], xs[5], xs[6]});
        qw = qmul(qw, DQ{xs[0], xs[1], xs[2], xs[3]});
        const double pw[7] = {qw.x, qw.y, qw.z, qw.w, tw.x, tw.y, tw.z};
        double* op = a.para + (size_t)k * 7;
        double* ow = a.pose + (size_t)k * 7;
        for (int e = 0; e < 7; e++) { op[e] = xs[e]; ow[e] = pw[e]; sh.cpw[e] = pw[e]; }
      }
      eng_trace(1, 5u);
      eng_prof(ptk, 3, rt_now());
    }
    __syncthreads();
  }
  if (wave0 && lane < 7) { st[lane] = sh.cx[lane]; st[7 + lane] = sh.cpw[lane]; }  // the chain's final state
  return true;
}


// Touch (one dword per 128-B line, plain loads: they allocate in this XCD's L2) every structure the
// association of pair k reads: the Morton copies, the chunk / super-chunk boxes and the clouds of
// scan k-1's less-sharp and less-flat sets.  Waves 1.. of a workgroup whose ticket must wait.  The
// workgroups of one XCD (dispatched round-robin over the 8 XCDs) split the lines between them:
// workgroup b touches lines congruent to (b / 8) mod 32.
__device__ __forceinline__ void eng_prefetch(const OdomArgs& a, EngShared& sh, int k, int t0, int nt) {
  unsigned acc = 0;
  const size_t part = (blockIdx.x >> 3) & 31;
  auto touch = [&](const void* base, size_t bytes) {
    const __attribute__((address_space(1))) unsigned* p = (const __attribute__((address_space(1))) unsigned*)base;
    const size_t lines = (bytes + 127) / 128;
    for (size_t l = part + (size_t)t0 * 32; l < lines; l += (size_t)nt * 32) acc ^= p[l * 32];
  };
  for (int which = 0; which < 2; which++) {
    const TargetIndex& ix = which ? a.idx_lf : a.idx_ls;
    const int nL = a.n_feat[(k - 1) * 4 + (which ? 3 : 1)];
    const int nch = (nL + kChunk - 1) / kChunk, nsu = (nch + kChunk - 1) / kChunk;
    const P4* L = which ? a.less_flat + (size_t)(k - 1) * a.N : a.less_sharp + (size_t)(k - 1) * a.cap_less_sharp;
    touch(ix.nn_super + (size_t)(k - 1) * ix.nsuper * 2, (size_t)nsu * 32);
    touch(ix.nn_chunk + (size_t)(k - 1) * ix.nchunk * 2, (size_t)nch * 32);
    touch(ix.chunk + (size_t)(k - 1) * ix.nchunk * 2, (size_t)nch * 32);
    touch(ix.sorted + (size_t)(k - 1) * ix.cap, (size_t)nL * 16);
    touch(L, (size_t)nL * 16);
  }
  if (acc == 0x9e3779b9u) sh.sink = acc;  // keeps the loads
}

// Tickets: [0, C) the chains' solve roles, then the association items in (pass, chain, item)
// order.  Item ticket t -> pass ro, chain c, item; pidx = its slot in the developer profile
// (ro * C * (I + 1) + c * (I + 1) + item; the solve of a pass at item = I).
struct ItemTicket {
  int ro, c, item;
};
__device__ __forceinline__ ItemTicket item_ticket(const EngCtl& ctl, unsigned t) {
  const unsigned tt = t - (unsigned)ctl.roles, per_ro = (unsigned)ctl.C * ctl.I;
  const int ro = (int)(tt / per_ro), rem = (int)(tt % per_ro);
  return ItemTicket{ro, rem / ctl.I, rem % ctl.I};
}

// An association ticket whose pass's x does not exist yet: its waves 1.. prefetch meanwhile.
__device__ __forceinline__ int eng_wants_prefetch(const OdomArgs& a, const EngCtl& ctl, unsigned t, unsigned total) {
  if (!ctl.prefetch || t < (unsigned)ctl.roles || t >= total) return 0;
  const ItemTicket it = item_ticket(ctl, t);
  if (it.ro == 0) return 0;
  int k;
  if (!pair_of(a, it.c, it.ro >> 1, &k) || it.item >= eng_live_items(a, ctl, k)) return 0;
  return ld_rlx(ctl.lm_gen(it.c)) < (unsigned)it.ro ? 1 : 0;
}

// One association item ticket (pass ro, chain c, item): wait for the pass's x, run the item's
// queries, publish its records and share.  false = aborted.
template <int kQpw>
__device__ __forceinline__ bool eng_item_ticket(const OdomArgs& a, const EngCtl& ctl, EngShared& sh, bool wave0, bool lead,
                                                const ItemTicket& it) {
  bool ok = true;
  const int ro = uni(it.ro), c = uni(it.c), item = uni(it.item);
  const int r = ro >> 1, o = ro & 1;
  const unsigned ptk = (unsigned)(ro * ctl.C * (ctl.I + 1) + c * (ctl.I + 1) + item);
  if (wave0 && lead) eng_prof(ptk, 0, rt_now());
  int k;
  bool live = pair_of(a, c, r, &k);
  // items holding queries of pair k: ceil((sharp + flat) / Q), none for a gated-off scan
  PassShape ps{0, 0};
  if (live) ps = pass_shape(a, ctl, k);
  const int ieff = ps.ieff;
  if (item >= ieff) live = false;  // an empty item: nothing to wait for or signal
  const size_t rec_stride = (size_t)(a.cap_sharp + a.cap_flat) * 9;  // doubles per chain (a.blk)
  const Rsrc rec = make_rsrc(a.blk + (size_t)c * rec_stride, (unsigned)((a.cap_sharp + a.cap_flat) * kRecBytes));
  int* warm = a.warm + (size_t)c * (a.cap_sharp + a.cap_flat) * 4;
  // An item of the second outer pass first waits for the first pass's items (its seeds), long
  // done in the common case; then every wave loads what needs no x while the lead waits for x.
  if (wave0) {
    if (lead) {
      sh.flag0 = (live && o == 1) ? eng_wait(ctl.assoc_done(c, ro - 1), (unsigned)ieff, ctl.abort_w(), ctl.wait_ticks, 1u, ctl.backoff) : true;
    }
  }
  __syncthreads();
  ok = uni(sh.flag0) != 0;
  if (ok && live) {  // each wave parks its first query's loads in its LDS slots
    // lane group `row` (16 lanes) loads the wave's query row: its 16-lane row (qpw 4) or its row-th
    // query in turn (qpw 2, 3)
    const int wv = (int)(threadIdx.x >> 6), row = kQpw > 1 ? min(lane_id() >> 4, kQpw - 1) : 0, l = lane_id() & 15;
    const ItemPre pre = eng_item_pre(a, k, (item * ctl.Q + wv) * kQpw + row, warm, o);
    P4 v = pre.qp;  // selects, not a lane-indexed array (which would live in scratch)
    int wi = pre.wi[0];
    if (l == 1) { v = pre.wp[0]; wi = pre.wi[1]; }
    if (l == 2) { v = pre.wp[1]; wi = pre.wi[2]; }
    if (l == 3) v = pre.wp[2];
    if (l < 4 && lane_id() < 16 * kQpw) sh.prew[wv][row][l] = v;
    if (l < 3 && lane_id() < 16 * kQpw) sh.prei[wv][row][l] = wi;
  }
  if (!wave0 && ok && live && uni(sh.pref)) eng_prefetch(a, sh, k, threadIdx.x - 64, (int)blockDim.x - 64);
  if (wave0) {
    if (lead) {
      if (ok && live) {
        eng_prof(ptk, 2, rt_now());  // the item's lead starts its wait for x
        ok = eng_wait(ctl.lm_gen(c), (unsigned)ro, ctl.abort_w(), ctl.wait_ticks, 2u, ctl.backoff);
        eng_trace(1, ok ? 2u : 99u);
        eng_prof(ptk, 1, rt_now());
      }
      sh.flag = ok;
    }
  }
  __syncthreads();
  ok = uni(sh.flag) != 0;  // false: aborted, leave (the host reads the abort word)
  if (ok && live) {
    {  // each wave its own copy of x (its lanes 0..6 load it): no barrier
      const int l = lane_id();
      if (l < 7) sh.xw[threadIdx.x >> 6][l] = eng_x_word(a, c, r, o, l);
    }
    eng_item_run<kQpw>(a, ctl, sh, k, item, ps, rec, warm, o, ptk);
    drain_stores();  // this wave's record (and seed) stores
    __syncthreads();
    if (wave0) {
      const unsigned long long tp0 = lead ? rt_now() : 0ull;
      if (lane_id() < 30) {  // the item's share: the sum of its waves' shares
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < ctl.Q; w++) v += sh.red[w][lane_id()];
        st_sc1d(part_row(a, ctl, c, item) + lane_id(), v);
      }
      drain_stores();
      if (lead) {
        eng_prof(ptk, 7, rt_now() - tp0);
        st_sc1(reinterpret_cast<uint64_t*>(part_row(a, ctl, c, item)) + 31, eng_tag(ctl, ro));  // row complete
        add_rlx(ctl.assoc_done(c, ro), 1u);
        eng_trace(1, 4u);
        eng_prof(ptk, 3, rt_now());
      }
    }
  }
  return ok;
}

// Control flow around the workgroup barriers.  Every branch tests a wave-uniform scalar: LDS
// broadcasts go through readfirstlane, and single-lane work (ticket, waits, signals) sits in
// `if (wave0) { if (lane == 0) ... }` — the divergent part closed inside a uniform branch.  The
// loop takes its next ticket at the bottom and tests it at the top.  (A `for (;;)` opening with
// `if (threadIdx.x == 0)` let the compiler rotate the divergent block into the latch, so wave 0's
// other lanes reached the next barrier ahead of lane 0 and the waves' barrier counts diverged.)
// The first C tickets are the solve roles: they are claimed before any item, by running workgroups,
// so every item a role waits for is claimed by a running workgroup too; the queue drains on any
// grid of at least C + 1 workgroups (launch_odometry_chain enforces it).
__global__ __launch_bounds__(kEngThreads) void k_odom_chain(OdomArgs a, EngCtl ctl) {
  __shared__ EngShared sh;
  __shared__ EngLM lm;
#ifdef LISLAM_ENG_ZERO_LDS  // developer: start from zeroed LDS (a read-before-write hunt)
  for (int i = threadIdx.x; i < (int)(sizeof(EngShared) / 4); i += blockDim.x) reinterpret_cast<unsigned*>(&sh)[i] = 0u;
  for (int i = threadIdx.x; i < (int)(sizeof(EngLM) / 4); i += blockDim.x) reinterpret_cast<unsigned*>(&lm)[i] = 0u;
  __syncthreads();
#endif
  const unsigned per_ro = (unsigned)ctl.C * ctl.I;
  const unsigned total = (unsigned)ctl.roles + per_ro * 2u * ctl.R;
  const bool wave0 = uni((int)(threadIdx.x >> 6)) == 0;
  const bool lead = lane_id() == 0;
  if (wave0) {
    if (lead) {
      const unsigned t = add_rlx(ctl.ticket(), 1u);
      sh.ticket = t;
      sh.pref = eng_wants_prefetch(a, ctl, t, total);
      eng_trace(0, t);
    }
  }
  __syncthreads();
  unsigned tk = (unsigned)uni((int)sh.ticket);
  while (tk < total) {
    bool ok = true;
    if (tk < (unsigned)ctl.roles) {
      const int c = uni((int)tk);
      ok = eng_solve_role(a, ctl, sh, lm, c, wave0, (unsigned)(c * (ctl.I + 1) + ctl.I));
    } else {
      ok = eng_item_ticket<1>(a, ctl, sh, wave0, lead, item_ticket(ctl, tk));
    }
    if (wave0) {
      if (lead) {
        const unsigned t = add_rlx(ctl.ticket(), 1u);
        sh.ticket = t;
        sh.pref = eng_wants_prefetch(a, ctl, t, total);
        eng_trace(0, t);
      }
    }
    __syncthreads();
    tk = ok ? (unsigned)uni((int)sh.ticket) : total;
  }
}

// ---- the engine as two launches (the production schedule): the chains' solve roles, one
// workgroup per chain (256 VGPRs: the evaluation's register slots and the step), and the
// association items (at most 128 VGPRs, a small LDS footprint), on two CU-masked streams: the
// roles on one reserved CU per XCD, the items on the others.  An item workgroup then leaves half
// of its CU's registers and most of its LDS to whatever else runs (the next batch's extraction,
// the ORB front end), and the roles always find a CU (launch_odometry_chain).

// The grid is one workgroup per role CU (at least C): a workgroup takes the next chain from a ticket
// when it starts, so the chains go to whichever role CUs are free (another engine may hold some:
// LISLAM_ENGINE_DEPTH), and the workgroups left over exit at once.
__device__ __forceinline__ unsigned xcc_id() {
  return __builtin_amdgcn_s_getreg((4 - 1) << 11 | 0 << 6 | 20) & 15u;  // HW_REG_XCC_ID[3:0]
}

// Developer builds (-DLISLAM_ENG_STAMPS=1, scripts/engines_concurrent.py): per launch (gen % 64)
// s_memrealtime of the role's start and end, its XCD, the first and last item workgroup's start, the
// item workgroups that ran, and the last item's end.
#ifndef LISLAM_ENG_STAMPS
#define LISLAM_ENG_STAMPS 0
#endif
#if LISLAM_ENG_STAMPS
__device__ unsigned long long g_eng_stamps[64][12];
__device__ __forceinline__ void eng_stamp_max(int k, const EngCtl& ctl, unsigned long long v) {
  __hip_atomic_fetch_max(&g_eng_stamps[ctl.gen % 64][k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void eng_stamp_min(int k, const EngCtl& ctl, unsigned long long v) {
  __hip_atomic_fetch_min(&g_eng_stamps[ctl.gen % 64][k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
extern "C" int lislam_debug_engine_stamps(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_eng_stamps), sizeof(g_eng_stamps)) != hipSuccess) return 1;
  static unsigned long long init[64][12];
  for (auto& r : init) { for (auto& v : r) v = 0; r[3] = r[10] = ~0ull; }
  return hipMemcpyToSymbol(HIP_SYMBOL(g_eng_stamps), init, sizeof(init)) == hipSuccess ? 0 : 1;
}
#endif

// The launch's control words to zero, all but word 3 (the sticky abort): one workgroup on the roles
// stream ahead of both kernels (two runtime memsets were two dispatches).
__global__ __launch_bounds__(256) void k_eng_zero(EngCtl ctl, int words) {
#if LISLAM_ENG_STAMPS
  if (threadIdx.x == 0) {
    eng_stamp_max(7, ctl, __builtin_amdgcn_s_memrealtime());
    eng_stamp_max(8, ctl, xcc_id() + 1);
  }
#endif
  for (int i = threadIdx.x; i < words; i += 256)
    if (i != 3) ctl.w[i] = 0u;
}

__global__ __launch_bounds__(kEngThreads) void k_odom_roles(OdomArgs a, EngCtl ctl) {
  __shared__ EngShared sh;
  __shared__ EngLM lm;
  __shared__ unsigned held_x;
#ifdef LISLAM_ENG_ZERO_LDS  // developer: start from zeroed LDS (a read-before-write hunt)
  for (int i = threadIdx.x; i < (int)(sizeof(EngShared) / 4); i += blockDim.x) reinterpret_cast<unsigned*>(&sh)[i] = 0u;
  for (int i = threadIdx.x; i < (int)(sizeof(EngLM) / 4); i += blockDim.x) reinterpret_cast<unsigned*>(&lm)[i] = 0u;
  __syncthreads();
#endif
  const bool wave0 = uni((int)(threadIdx.x >> 6)) == 0;
#if LISLAM_ENG_STAMPS
  if (wave0 && lane_id() == 0) {  // every roles workgroup's start: the first and the last
    eng_stamp_max(9, ctl, __builtin_amdgcn_s_memrealtime());
    eng_stamp_min(10, ctl, __builtin_amdgcn_s_memrealtime());
  }
#endif
  if (wave0 && lane_id() == 0) {
    if (!ctl.xbusy) {
      sh.ticket = add_rlx(ctl.role_ticket(), 1u);
    } else {
      // One role per XCD while a free one exists (each XCD holds two role CUs): the workgroups of the
      // next launch that land on this XCD — those that exit at once, or the control words' memset —
      // then find its other role CU free instead of queueing behind this chain.  A workgroup takes
      // the chain only if its XCD held no role; the last to arrive takes it if none of them could.
      const unsigned x = xcc_id();
      unsigned* xb = ctl.xbusy + x;
      unsigned t = ~0u;
      const bool mine = add_rlx(xb, 1u) == 0u;  // this XCD held no role: the count stays ours
      if (mine) t = add_rlx(ctl.role_ticket(), 1u);
      else (void)add_rlx(xb, ~0u);
      __threadfence();  // the claim is settled before the arrival is counted
      if (t >= (unsigned)ctl.C && add_rlx(ctl.role_arrive(), 1u) == (unsigned)ctl.rgrid - 1u) {
        t = add_rlx(ctl.role_ticket(), 1u);  // the last arrival: every other claim is settled
        if (t < (unsigned)ctl.C && !mine) (void)add_rlx(xb, 1u);
      } else if (t < (unsigned)ctl.C) {
        (void)add_rlx(ctl.role_arrive(), 1u);
      }
      if (t >= (unsigned)ctl.C && mine) (void)add_rlx(xb, ~0u);
      sh.ticket = t;
      held_x = t < (unsigned)ctl.C ? x : ~0u;
    }
  }
  __syncthreads();
  const int c = uni((int)min(sh.ticket, (unsigned)ctl.C));
  if (c >= ctl.C) return;
#if LISLAM_ENG_STAMPS
  if (wave0 && lane_id() == 0) {
    eng_stamp_max(0, ctl, __builtin_amdgcn_s_memrealtime());
    eng_stamp_max(2, ctl, xcc_id() + 1);
  }
#endif
  (void)eng_solve_role(a, ctl, sh, lm, c, wave0, (unsigned)(c * (ctl.I + 1) + ctl.I));
#if LISLAM_ENG_STAMPS
  if (wave0 && lane_id() == 0) eng_stamp_max(1, ctl, __builtin_amdgcn_s_memrealtime());
#endif
  if (ctl.xbusy && wave0 && lane_id() == 0) {
    __threadfence();
    (void)add_rlx(ctl.xbusy + held_x, ~0u);
  }
}

#ifndef LISLAM_ITEM_WPE
#define LISLAM_ITEM_WPE 4  // waves per SIMD the items are compiled for: 4 = 128 VGPRs
#endif
template <int kQpw>
__device__ __forceinline__ void eng_items_body(const OdomArgs& a, const EngCtl& ctl) {
  __shared__ EngShared sh;
  const unsigned total = (unsigned)ctl.C * ctl.I * 2u * ctl.R;
  const bool wave0 = uni((int)(threadIdx.x >> 6)) == 0;
  const bool lead = lane_id() == 0;
#if LISLAM_ENG_STAMPS
  if (wave0 && lead) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    eng_stamp_min(3, ctl, t);
    eng_stamp_max(4, ctl, t);
    __hip_atomic_fetch_add(&g_eng_stamps[ctl.gen % 64][5], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#endif
  if (wave0) {
    if (lead) {
      const unsigned t = add_rlx(ctl.ticket(), 1u);
      sh.ticket = t;
      sh.pref = eng_wants_prefetch(a, ctl, t, total);
    }
  }
  __syncthreads();
  unsigned tk = (unsigned)uni((int)sh.ticket);
  while (tk < total) {
    const bool ok = eng_item_ticket<kQpw>(a, ctl, sh, wave0, lead, item_ticket(ctl, tk));
    if (wave0) {
      if (lead) {
        const unsigned t = add_rlx(ctl.ticket(), 1u);
        sh.ticket = t;
        sh.pref = eng_wants_prefetch(a, ctl, t, total);
      }
    }
    __syncthreads();
    tk = ok ? (unsigned)uni((int)sh.ticket) : total;
  }
#if LISLAM_ENG_STAMPS
  if (wave0 && lead) eng_stamp_max(6, ctl, __builtin_amdgcn_s_memrealtime());
#endif
}
template <int kQpw>
__global__ __launch_bounds__(64 * kMaxItemWaves, LISLAM_ITEM_WPE) void k_odom_items(OdomArgs a, EngCtl ctl) {
  eng_items_body<kQpw>(a, ctl);
}
// One engine at a time (the latency shape: qpw 1, depth 1, 12-wave items): the same items compiled
// for 3 waves per SIMD (168 VGPRs: no spills, where the 128-VGPR build spills 36 VGPRs and ~180
// SGPRs).  With several engines in flight the 128-VGPR build stays: two item workgroups per CU beat
// spill-free ones (profiles/r05_shape_ab.txt, r05wpe); one engine gains 2-3 % (single sequence 10.40k /
// 10.43k vs 10.20k / 10.10k, r05solo).  LISLAM_ENGINE_SOLO_ITEMS=0: the 128-VGPR build (A/B).
constexpr int kSoloItemWaves = 12;
__global__ __launch_bounds__(64 * kSoloItemWaves, 3) void k_odom_items_solo(OdomArgs a, EngCtl ctl) {
  eng_items_body<1>(a, ctl);
}

static int item_waves(int qpw, int depth);
// eng_wait's longest sleep between polls in units of 64 cycles: 1 (a fixed 64) with one engine in
// flight, whose wake-up latency is the chain's; 8 with several, whose waiting items would otherwise
// poll 1.5x as often (profiles/r06b_backoff_ab.txt).  LISLAM_ENGINE_BACKOFF overrides (1..64).
static unsigned engine_backoff(int depth) {
  static const int env = getenv("LISLAM_ENGINE_BACKOFF") ? std::max(1, std::min(64, atoi(getenv("LISLAM_ENGINE_BACKOFF")))) : 0;
  return env ? (unsigned)env : depth <= 1 ? 1u : 8u;
}
// Items per (pass, chain) of the split engine at qpw queries per wave and `depth` engines in flight
// (the developer profile's ticket layout).
extern "C" int lislam_debug_engine_items(int cap_queries, int qpw, int depth) {
  const int qpi = item_waves(qpw, depth) * qpw;
  return (cap_queries + qpi - 1) / qpi;
}
// A number per engine launch (the item rows' tags tell this launch's passes from an earlier one's).
static unsigned next_engine_gen() {
  static std::atomic<unsigned> gen{0};
  return ++gen;
}

int engine_items(int cap_queries) { return (cap_queries + kEngWaves - 1) / kEngWaves; }  // rows: Q >= kEngWaves

// Waves per item workgroup of the split engine: LISLAM_ENGINE_ITEM_WAVES (up to kMaxItemWaves, and
// at least kEngWaves queries per item: the share rows are sized for that); by default 12 for one
// engine at a time at one query per wave (248 x 12 waves hold a pass's ~2,100 queries in one
// round: no overflow round, 25.0 vs 26.9 ms per chain), else 8 (qpw 1..3: two engines' items fit
// a CU's 16 wave slots at 128 VGPRs) / 4 (qpw 4).
static int item_waves(int qpw, int depth) {
  const int def = qpw == 4 ? 4 : (qpw == 1 && depth == 1) ? 12 : 8;
  const char* e = getenv("LISLAM_ENGINE_ITEM_WAVES");
  const int q = e ? atoi(e) : def;
  return q * qpw >= kEngWaves && q <= kMaxItemWaves ? q : def;
}
int engine_part_rows(int cap_queries) { return max(engine_items(cap_queries), kMaxShareItems); }

bool use_chain_engine(const OdomArgs& a, int mode) {
  if (mode == 0 || a.n_chains < 1 || !a.eng_ctl) return false;
  if (mode == 2) return true;
  return a.n_chains <= 4;  // few long chains (the continuous chain, a rank's shard); many short: rounds
}

// Workgroups of k_odom_chain resident at once on `dev` (CUs x occupancy), per device.
static int engine_resident(int dev) {
  static int cache[64] = {0};
  if (dev >= 0 && dev < 64 && cache[dev]) return cache[dev];
  int cus = 0, per_cu = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_odom_chain, kEngThreads, 0);
  const int r = max(1, cus * max(per_cu, 1));
  if (dev >= 0 && dev < 64) cache[dev] = r;
  return r;
}

int launch_odometry_chain(const OdomArgs& a, hipStream_t st) {
  if (a.n_chains <= 0) return 0;
  EngCtl ctl;
  ctl.gen = next_engine_gen();
  ctl.P = engine_part_rows(a.cap_sharp + a.cap_flat);
  ctl.w = a.eng_ctl;
  ctl.C = a.n_chains;
  ctl.R = min(a.chain_len, a.S - 1);
  ctl.Q = kEngWaves;  // items run in the engine's own workgroups
  ctl.I = engine_items(a.cap_sharp + a.cap_flat);
  ctl.prefetch = 1;
  ctl.roles = ctl.C;
  ctl.qpw = 1;
  // every device wait is bounded (2 s); LISLAM_ENGINE_WAIT_US shortens it (tests: a forced abort)
  const char* wb = getenv("LISLAM_ENGINE_WAIT_US");
  ctl.wait_ticks = wb ? (unsigned long long)std::max(1L, atol(wb)) * 100ull : 200000000ull;
  ctl.backoff = engine_backoff(a.eng_depth);
  // Items per (pass, chain): the workgroups resident at once, less the chains' solve roles and one
  // spare, shared by the chains.  More queries than
  // that are dealt as second queries to the items' waves (eng_item_run).  LISLAM_ENGINE_BUDGET
  // overrides (tests).
  int dev = 0;
  (void)hipGetDevice(&dev);
  const int resident = engine_resident(dev);
  const char* bud = getenv("LISLAM_ENGINE_BUDGET");
  ctl.budget = min(kMaxShareItems, bud ? max(1, atoi(bud)) : max(1, (resident - ctl.C - 1) / ctl.C));
  // zero the control words of this launch, all but word 3 (the sticky abort)
  const size_t words = ((size_t)4 + ctl.C + (size_t)2 * ctl.R * ctl.C + 3) / 4 * 4;  // + assoc_done
  (void)hipMemsetAsync(a.eng_ctl, 0, 3 * sizeof(unsigned), st);
  (void)hipMemsetAsync(a.eng_ctl + 4, 0, (words - 4) * sizeof(unsigned), st);
  // LISLAM_ENGINE_WGS caps the grid (tests: one workgroup drains the whole queue)
  const char* cap_env = getenv("LISLAM_ENGINE_WGS");
  const int cap = cap_env ? atoi(cap_env) : 0;
  int grid = ctl.C * (ctl.I + 1);
  if (cap > 0) grid = min(grid, max(cap, ctl.C + 1));  // the roles and one item worker at least
  hipLaunchKernelGGL(k_odom_chain, dim3(grid), dim3(kEngThreads), 0, st, a, ctl);
  return grid;
}

// The engine as two launches (k_odom_roles / k_odom_items) on a pair of CU-masked streams
// (make_engine_streams); false = unavailable on this device (the caller runs the single-launch
// engine instead).  A mask bit i selects a CU of XCD i % 8 (gfx942 / gfx950, measured:
// scripts/micro/cumask.hip; a mask with no bit of some XCD leaves that XCD unmasked), the roles one
// CU in every XCD, the items every other CU, so an item workgroup never takes the CU a solve role
// needs whole (256 VGPRs x 8 waves).  (Unmasked priority streams were measured to starve the role
// of a whole CU under the pipelined extraction, r04i, and are not offered.)
// Every CU-masked stream is a hardware queue of its own, and past about 20 of them in one process
// every launch slows (r05c56: the isolated chain 34.7 -> 47-50 ms).  The library's masked streams
// are registered here, so the count is known (lislam_device_queue_count, bench.py's config) and kept
// low by construction: a context holds one (its stream, which its ORB front end shares), the
// engine's kMaxDepth pairs and the per-round schedule's group streams belong to the device.
namespace {
std::mutex g_masked_mu;
std::vector<std::pair<hipStream_t, int>> g_masked;  // (stream, device)
bool masked_stream(int dev, hipStream_t* s, int words, const uint32_t* mask) {
  if (hipExtStreamCreateWithCUMask(s, words, mask) != hipSuccess) return false;
  std::lock_guard<std::mutex> lk(g_masked_mu);
  g_masked.emplace_back(*s, dev);
  return true;
}
}  // namespace

void destroy_stream(hipStream_t s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> lk(g_masked_mu);
    for (size_t i = 0; i < g_masked.size(); i++)
      if (g_masked[i].first == s) { g_masked.erase(g_masked.begin() + i); break; }
  }
  (void)hipStreamDestroy(s);
}

int masked_queue_count(int dev) {
  std::lock_guard<std::mutex> lk(g_masked_mu);
  int n = 0;
  for (const auto& e : g_masked) n += e.second == dev;
  return n;
}

// XCDs of the device (hipDeviceAttributeNumberOfXccs: 8 on an MI355X in SPX mode, 1 per device in
// CPX mode); a CU mask bit i selects a CU of XCD i % xccs (measured on gfx942 / gfx950 in SPX:
// scripts/micro/cumask.hip).  0 = unknown.
static int device_xccs(int dev) {
  int x = 0;
  if (hipDeviceGetAttribute(&x, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess) {
    (void)hipGetLastError();
    x = 0;
  }
  return x;
}

// The CU masks.  Bit i selects a CU of XCD i % nx, and the bit groups [k nx, k nx + nx) walk the
// XCDs' shader engines: group k is a CU of SE k % 4 in every XCD (gfx950, measured:
// scripts/micro/cumask2.hip).  A workgroup is dealt to a shader engine before a CU is chosen, so a
// CU free in another SE does not help it.
//   roles: groups 0 and 4, two CUs of SE 0 in every XCD.  With one role per XCD (k_odom_roles) the
//     next launch's roles workgroups that land on a role's XCD — those that exit at once, or the
//     control-word zeroing — find the other CU free instead of queueing behind that whole chain (one
//     role CU per XCD: 75-80 vs 40 ms whenever it happened, scripts/engines_concurrent.py).
//     LISLAM_ROLE_CUS=1 keeps group 0 only.
//   items: every other CU; LISLAM_ITEMS_SE0=0 leaves SE 0 out (its six free CUs get as many item
//     workgroups dealt as the other SEs' eight).
//   work (extraction, ORB, per-round odometry): shader engines 1-3.  Work dealt evenly over the SEs
//     runs at the pace of the SE with the fewest CUs, so SE 0's six left-over CUs added next to
//     eight-CU SEs would be worth no more than none, and they are the items' alone instead: the
//     driver-shape headline 23.3-23.4k vs 20.3-20.6k scans/s with the work streams on SE 0 too
//     (profiles/r06_semask_ab.txt).  LISLAM_WORK_SE0=1 shares SE 0.
static int role_cus_per_xcd() {
  static const int r = getenv("LISLAM_ROLE_CUS") && atoi(getenv("LISLAM_ROLE_CUS")) == 1 ? 1 : 2;
  return r;
}
static bool role_bit(int i, int nx) { return i / nx == 0 || (role_cus_per_xcd() == 2 && i / nx == 4); }
// Slot s's items: SE 0's six item CUs hold two workgroups each, as many as four engines deal them
// (96 items / 32 SEs = 3 per SE each), so the pairs of slots 4 and 5 leave SE 0 out: a fifth engine
// deals its 96 items to SEs 1-3 (4 per SE, 16 with the other four's 12 = their 8 CUs x 2), where
// with SE 0 it found 12 slots for 15 and part of its items waited for an engine to end
// (scripts/engines_concurrent.py: 61 vs 41 ms).  LISLAM_ITEMS_SE0=0: no slot's items on SE 0;
// =2: every slot's.
static bool item_bit(int i, int nx, int slot) {
  static const int se0 = getenv("LISLAM_ITEMS_SE0") ? atoi(getenv("LISLAM_ITEMS_SE0")) : 1;
  const bool with_se0 = se0 == 2 || (se0 == 1 && slot < 4);
  return !role_bit(i, nx) && (with_se0 || (i / nx) % 4 != 0);
}
static int g_item_cus[64];  // CUs of the items mask per device (make_engine_streams)

static bool make_engine_streams(int dev, int slot, hipStream_t* roles, hipStream_t* items) {
  hipDeviceProp_t prop{};
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
  const bool multi_xcd = std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 || std::strncmp(prop.gcnArchName, "gfx942", 6) == 0;
  const int cus = prop.multiProcessorCount, nx = device_xccs(dev);
  if (!multi_xcd || nx < 1 || cus < 8 * nx || cus % nx) return false;
  const int words = (cus + 31) / 32;
  std::vector<uint32_t> mr(words, 0u), mi(words, 0u);
  int n_items = 0;
  for (int i = 0; i < cus; i++) {
    if (role_bit(i, nx)) mr[i / 32] |= 1u << (i % 32);
    else if (item_bit(i, nx, slot)) { mi[i / 32] |= 1u << (i % 32); n_items++; }
  }
  if (slot == 0 && dev >= 0 && dev < 64) g_item_cus[dev] = n_items;
  if (!masked_stream(dev, roles, words, mr.data())) return false;
  if (!masked_stream(dev, items, words, mi.data())) {
    destroy_stream(*roles);
    *roles = nullptr;
    return false;
  }
  return true;
}

// A stream for the library's other kernels (extraction, ORB, per-round odometry): shader engines 1-3
// (above), never the solve roles' CUs, so a role launched beside the next batch's extraction finds a
// whole CU free instead of waiting for the extraction's waves on it to drain — they would refill each
// freed slot first.  Plain non-blocking stream where CU masks do not apply.
bool work_stream(int dev, hipStream_t* s) {
  hipDeviceProp_t prop{};
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess) {
    const bool multi_xcd = std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 || std::strncmp(prop.gcnArchName, "gfx942", 6) == 0;
    const int cus = prop.multiProcessorCount, nx = device_xccs(dev);
    if (multi_xcd && nx >= 1 && cus >= 8 * nx && cus % nx == 0) {
      const int words = (cus + 31) / 32;
      std::vector<uint32_t> m(words, 0u);
      // LISLAM_WORK_XCDS=n (developer: traffic attribution) keeps the stream on the first n XCDs
      const char* xe = getenv("LISLAM_WORK_XCDS");
      const int nxu = xe ? std::max(1, std::min(nx, atoi(xe))) : nx;
      // shader engine 0 (the role CUs' SE) is left to the engines; LISLAM_WORK_SE0=1 (A/B) shares it
      static const bool se0 = getenv("LISLAM_WORK_SE0") && atoi(getenv("LISLAM_WORK_SE0")) == 1;
      for (int i = 0; i < cus; i++)
        if (!role_bit(i, nx) && i % nx < nxu && (se0 || (i / nx) % 4 != 0)) m[i / 32] |= 1u << (i % 32);
      if (masked_stream(dev, s, words, m.data())) return true;
    }
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking) == hipSuccess;
}

// One engine at a time per device (contexts included): each split launch waits for the previous
// one, so two pipelined batches' chains do not split the CUs the extraction beside them needs.  The
// wait on the previous engine and the re-record of the event are one critical section (the mutex),
// so two host threads launching on different contexts cannot both pass the gate.
// Slot s of the ring also owns a pair of engine streams, shared by every batch of the device: the
// launches of all contexts run on kMaxDepth stream pairs, not one pair per batch, so five or six
// pipelined contexts do not push the process past the device's hardware queues (past ~20 masked
// queues every launch slowed: the isolated chain 34.7 -> 47-50 ms with six contexts, r05c56).
// Launch n takes slot n % kMaxDepth (its stream pair) and waits for the event of launch n - depth,
// whatever slot that one used: with contexts of different depths on one device, a depth-1 launch
// still waits for the launch just before it (a per-depth ring would wait for the last launch that
// used its slot instead).
struct EngineGate {
  static constexpr int kMaxDepth = kMaxEngineDepth;  // pairs are made per slot used
  std::mutex mu;
  hipEvent_t ev[kMaxDepth] = {};
  hipStream_t roles[kMaxDepth] = {}, items[kMaxDepth] = {};
  unsigned long long launches = 0;
  int avail = -1;  // -1 not probed, 0 no CU masks on this device, 1 ready
  static constexpr int kRoundGroups = 4;
  hipStream_t round[kRoundGroups] = {};  // the per-round schedule's group streams (round_stream)
  // the dispatcher (submit_odometry_chain_split): its thread (a pointer: a static std::thread still
  // joinable at process exit would terminate), queue, and the slots' last launches
  std::thread* th = nullptr;
  unsigned* xbusy = nullptr;  // solve roles running per XCD (k_odom_roles), made with the streams
  bool stop = false;
  std::deque<EngineRequest*> q;
  std::condition_variable cv_req, cv_launched;
  hipEvent_t slot_ev[kMaxDepth] = {};
  bool slot_used[kMaxDepth] = {};
};
static EngineGate* engine_gate(int dev) {
  static EngineGate gates[64];
  return dev >= 0 && dev < 64 ? &gates[dev] : nullptr;
}

// g->mu held.  Slot 0's pair is made on the first probe (it tells whether CU masks work here); the
// other slots' pairs when a launch first takes them, so a device holds 2 x (the deepest depth used)
// engine queues.
static bool probe_engine_streams(EngineGate* g, int dev) {
  if (g->avail < 0) {
    g->avail = make_engine_streams(dev, 0, &g->roles[0], &g->items[0]) ? 1 : 0;
    if (g->avail == 1 && !g->xbusy) {
      if (hipMalloc(&g->xbusy, 16 * sizeof(unsigned)) != hipSuccess || hipMemset(g->xbusy, 0, 16 * sizeof(unsigned)) != hipSuccess) {
        (void)hipGetLastError();
        if (g->xbusy) (void)hipFree(g->xbusy);
        g->xbusy = nullptr;
      }
    }
  }
  return g->avail == 1;
}

bool engine_streams_available(int dev) {
  EngineGate* g = engine_gate(dev);
  if (!g) return false;
  std::lock_guard<std::mutex> lk(g->mu);
  return probe_engine_streams(g, dev);
}

hipStream_t round_stream(int dev, int grp) {
  EngineGate* g = engine_gate(dev);
  if (!g || grp < 1 || grp >= EngineGate::kRoundGroups) return nullptr;
  std::lock_guard<std::mutex> lk(g->mu);
  if (!g->round[grp] && !work_stream(dev, &g->round[grp])) g->round[grp] = nullptr;
  return g->round[grp];
}

// The device's engine streams, round streams and slot events are released with its last context
// (a stream left to the process's exit is torn down after the runtime, which a profiler's exit
// path trips over).
void release_engine_streams(int dev) {
  EngineGate* g = engine_gate(dev);
  if (!g) return;
  {  // the dispatcher first: it launches what is still queued, then exits
    std::unique_lock<std::mutex> lk(g->mu);
    g->stop = true;
    g->cv_req.notify_all();
  }
  if (g->th) {
    g->th->join();
    delete g->th;
    g->th = nullptr;
  }
  std::lock_guard<std::mutex> lk(g->mu);
  g->stop = false;
  for (int s = 0; s < EngineGate::kMaxDepth; s++) {
    if (g->slot_ev[s]) (void)hipEventDestroy(g->slot_ev[s]);
    g->slot_ev[s] = nullptr;
    g->slot_used[s] = false;
  }
  for (int s = 0; s < EngineGate::kMaxDepth; s++) {
    if (g->items[s]) { (void)hipStreamSynchronize(g->items[s]); destroy_stream(g->items[s]); }
    if (g->roles[s]) { (void)hipStreamSynchronize(g->roles[s]); destroy_stream(g->roles[s]); }
    if (g->ev[s]) (void)hipEventDestroy(g->ev[s]);
    g->items[s] = g->roles[s] = nullptr;
    g->ev[s] = nullptr;
  }
  for (int r = 1; r < EngineGate::kRoundGroups; r++) {
    if (g->round[r]) { (void)hipStreamSynchronize(g->round[r]); destroy_stream(g->round[r]); }
    g->round[r] = nullptr;
  }
  if (g->xbusy) (void)hipFree(g->xbusy);
  g->xbusy = nullptr;
  g->launches = 0;
  g->avail = -1;
}

// Item workgroups of one build (qpw 1..4, or 0: the solo build) that fit one CU, per device build
// (hipOccupancyMaxActiveBlocksPerMultiprocessor: registers, LDS, waves), cached.
static int item_occupancy(int qpw, int threads) {
  static int cache[5][17] = {};
  const int w = std::min(16, std::max(1, threads / 64));
  int& r = cache[qpw][w];
  if (r) return r;
  int n = 0;
  hipError_t e = hipErrorInvalidValue;
  switch (qpw) {
    case 0: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_odom_items_solo, threads, 0); break;
    case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_odom_items<1>, threads, 0); break;
    case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_odom_items<2>, threads, 0); break;
    case 3: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_odom_items<3>, threads, 0); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_odom_items<4>, threads, 0); break;
  }
  if (e != hipSuccess || n < 1) {
    (void)hipGetLastError();
    n = 1;
  }
  return r = n;
}

// The launch parameters of one split engine launch (EngCtl, grid, item build).
struct SplitPlan {
  EngCtl ctl;
  int grid = 0, depth = 1, roles_grid = 8;
  bool solo = false;
  size_t words = 0;
};
static SplitPlan split_plan(const OdomArgs& a, int dev) {
  SplitPlan p;
  EngCtl& ctl = p.ctl;
  ctl.gen = 0;  // numbered when queued on the device (split_enqueue)
  ctl.P = engine_part_rows(a.cap_sharp + a.cap_flat);
  ctl.w = a.eng_ctl;
  ctl.C = a.n_chains;
  ctl.R = min(a.chain_len, a.S - 1);
  ctl.qpw = a.eng_qpw >= 1 && a.eng_qpw <= 4 ? a.eng_qpw : 1;  // lislam_set_engine_shape
  ctl.Q = item_waves(ctl.qpw, std::max(1, a.eng_depth));
  ctl.I = (a.cap_sharp + a.cap_flat + ctl.qpi() - 1) / ctl.qpi();
  // waiting items warm their XCD's L2 with the pair's target structures: with one engine in flight
  // (with several, each warming all eight L2s for its own pair evicts the others': 18.9k vs 17.9k
  // scans/s over three alternating runs at the throughput shape, profiles/r05_shape_ab.txt)
  ctl.prefetch = getenv("LISLAM_ENGINE_PREFETCH") ? atoi(getenv("LISLAM_ENGINE_PREFETCH")) : (a.eng_depth <= 1 ? 1 : 0);
  ctl.roles = 0;
  const char* wb = getenv("LISLAM_ENGINE_WAIT_US");
  ctl.wait_ticks = wb ? (unsigned long long)std::max(1L, atol(wb)) * 100ull : 200000000ull;
  ctl.backoff = engine_backoff(a.eng_depth);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  p.depth = std::min(EngineGate::kMaxDepth, std::max(1, a.eng_depth));
  static const bool solo_ok = !(getenv("LISLAM_ENGINE_SOLO_ITEMS") && atoi(getenv("LISLAM_ENGINE_SOLO_ITEMS")) == 0);
  p.solo = solo_ok && p.depth == 1 && ctl.qpw == 1 && ctl.Q <= kSoloItemWaves;
  // Co-residency, checked at launch rather than assumed: the item workgroups one engine may hold at
  // once = the item CUs (all but one per XCD) x the workgroups of this item build that fit a CU
  // (hipOccupancyMaxActiveBlocksPerMultiprocessor), shared by the `depth` engines in flight.  The
  // grid and the items per (pass, chain) never exceed it, so a pass's items are all resident.
  const int per_cu = item_occupancy(p.solo ? 0 : ctl.qpw, 64 * ctl.Q);
  const int xccs = std::max(1, device_xccs(dev));
  const int item_cus = std::max(1, dev >= 0 && dev < 64 && g_item_cus[dev] ? g_item_cus[dev] : cus - role_cus_per_xcd() * xccs);
  const int resident = std::max(1, item_cus * per_cu / p.depth);
  const char* cap_env = getenv("LISLAM_ENGINE_WGS");
  const int cap = cap_env ? atoi(cap_env) : std::min(item_cus, resident);
  p.grid = ctl.C * ctl.I;
  if (cap > 0) p.grid = min(p.grid, max(cap, 1));
  const char* bud = getenv("LISLAM_ENGINE_BUDGET");
  ctl.budget = min(kMaxShareItems, bud ? max(1, atoi(bud)) : max(1, p.grid / ctl.C));
  p.words = ((size_t)6 + ctl.C + (size_t)2 * ctl.R * ctl.C + 3) / 4 * 4;  // + assoc_done, role ticket, arrivals
  p.roles_grid = std::max(ctl.C, xccs);
  ctl.rgrid = p.roles_grid;
  // one role per XCD for single-chain launches (k_odom_roles); LISLAM_ROLE_GATE=0: any XCD
  static const bool xgate = !(getenv("LISLAM_ROLE_GATE") && atoi(getenv("LISLAM_ROLE_GATE")) == 0);
  EngineGate* g = engine_gate(dev);
  ctl.xbusy = xgate && ctl.C == 1 && role_cus_per_xcd() >= 2 && g ? g->xbusy : nullptr;
  return p;
}

// Queue one launch on a slot's stream pair: the roles stream waits for `ready` and (if given) for
// `prev`, the items stream forks from it; `mine` is recorded at the end (the slot's busy mark).
static void split_enqueue(const OdomArgs& a, SplitPlan& p, hipStream_t roles, hipStream_t items, hipEvent_t ready,
                          hipEvent_t prev, hipEvent_t mine, hipEvent_t fork, hipEvent_t join_r, hipEvent_t join_i,
                          hipEvent_t t0, hipEvent_t t1, unsigned* h_abort, hipEvent_t done) {
  EngCtl& ctl = p.ctl;
  ctl.gen = next_engine_gen();
  (void)hipStreamWaitEvent(roles, ready, 0);
  if (prev) (void)hipStreamWaitEvent(roles, prev, 0);
  if (t0) (void)hipEventRecord(t0, roles);
  // zero the control words of this launch, all but word 3 (the sticky abort)
  hipLaunchKernelGGL(k_eng_zero, dim3(1), dim3(256), 0, roles, ctl, (int)p.words);
  (void)hipEventRecord(fork, roles);
  (void)hipStreamWaitEvent(items, fork, 0);
  hipLaunchKernelGGL(k_odom_roles, dim3(p.roles_grid), dim3(kEngThreads), 0, roles, a, ctl);
  if (p.solo) hipLaunchKernelGGL(k_odom_items_solo, dim3(p.grid), dim3(64 * ctl.Q), 0, items, a, ctl);
  else switch (ctl.qpw) {
    case 4: hipLaunchKernelGGL(k_odom_items<4>, dim3(p.grid), dim3(64 * ctl.Q), 0, items, a, ctl); break;
    case 3: hipLaunchKernelGGL(k_odom_items<3>, dim3(p.grid), dim3(64 * ctl.Q), 0, items, a, ctl); break;
    case 2: hipLaunchKernelGGL(k_odom_items<2>, dim3(p.grid), dim3(64 * ctl.Q), 0, items, a, ctl); break;
    default: hipLaunchKernelGGL(k_odom_items<1>, dim3(p.grid), dim3(64 * ctl.Q), 0, items, a, ctl); break;
  }
  (void)hipEventRecord(join_r, roles);
  (void)hipEventRecord(join_i, items);
  (void)hipStreamWaitEvent(items, join_r, 0);  // the device's engine ends when both kernels do
  if (t1) (void)hipEventRecord(t1, items);
  // the launch's error and sticky abort words to the host, and its end, before the slot's next
  // launch can queue behind it
  if (h_abort) (void)hipMemcpyAsync(h_abort, a.eng_ctl + 2, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, items);
  if (done) (void)hipEventRecord(done, items);
  (void)hipEventRecord(mine, items);
}

// g->mu held: slot s's stream pair, made when first used; false = it cannot be made
static bool slot_streams(EngineGate* g, int dev, int s) {
  return g->roles[s] || make_engine_streams(dev, s, &g->roles[s], &g->items[s]);
}

int launch_odometry_chain_split(const OdomArgs& a, hipEvent_t ready, hipEvent_t fork, hipEvent_t join_r,
                                hipEvent_t join_i, hipEvent_t t0, hipEvent_t t1, unsigned* h_abort, hipEvent_t done) {
  if (a.n_chains <= 0) return 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  SplitPlan p = split_plan(a, dev);
  const int depth = p.depth;
  EngineGate* gate = engine_gate(dev);
  if (!gate) return 0;
  std::unique_lock<std::mutex> lock(gate->mu);
  // the streams may have been released (the device's last context went away) since the caller
  // probed them: probe again under the lock
  if (!probe_engine_streams(gate, dev)) return 0;
  const unsigned long long n = gate->launches++;
  // slot n % depth: the launch it waits for (n - depth) used the same slot, so a slot's pair holds
  // one engine at a time
  int slot = (int)(n % depth);
  if (!slot_streams(gate, dev, slot)) slot = 0;
  for (hipEvent_t& e : gate->ev)
    if (!e) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  // launch n - depth (its event is re-recorded only by launch n - depth + kMaxDepth > n)
  hipEvent_t prev = n >= (unsigned long long)depth ? gate->ev[(n - depth) % EngineGate::kMaxDepth] : nullptr;
  // and the dispatcher's launches (contexts of another depth on this device): a gated engine sizes
  // its grid for `depth` engines, so it starts once theirs have ended
  for (int s = 0; s < EngineGate::kMaxDepth; s++)
    if (gate->slot_used[s]) (void)hipStreamWaitEvent(gate->roles[slot], gate->slot_ev[s], 0);
  split_enqueue(a, p, gate->roles[slot], gate->items[slot], ready, prev, gate->ev[n % EngineGate::kMaxDepth], fork,
                join_r, join_i, t0, t1, h_abort, done);
  return p.grid;
}

// ---- the engine dispatcher: one host thread per device, started by the first submit and joined by
// release_engine_streams.  Requests are launched in submission order among those whose `ready`
// event has completed, each on a slot whose last launch has ended (slot_ev), while fewer than the
// request's depth engines are in flight.  It polls every 20 us while something waits.
bool engine_dispatch_enabled() {
  static const bool on = !(getenv("LISLAM_ENGINE_DISPATCH") && atoi(getenv("LISLAM_ENGINE_DISPATCH")) == 0);
  return on;
}

static void dispatcher_loop(EngineGate* g, int dev) {
  (void)hipSetDevice(dev);
  std::unique_lock<std::mutex> lk(g->mu);
  for (;;) {
    if (g->q.empty()) {
      if (g->stop) break;
      g->cv_req.wait(lk);
      continue;
    }
    EngineRequest* r = nullptr;
    size_t at = 0;
    for (size_t i = 0; i < g->q.size(); i++)
      if (hipEventQuery(g->q[i]->ready) == hipSuccess) { r = g->q[i]; at = i; break; }
    if (r) {
      SplitPlan& p = *static_cast<SplitPlan*>(r->plan);
      // a gated launch in flight (a depth-1 context on this device) holds the CUs its grid was
      // sized for: nothing is dispatched beside it
      bool gated = false;
      for (hipEvent_t e : g->ev) gated = gated || (e && hipEventQuery(e) != hipSuccess);
      int busy = gated ? EngineGate::kMaxDepth : 0, free_slot = -1;
      for (int s = 0; s < EngineGate::kMaxDepth; s++) {
        const bool running = g->slot_used[s] && hipEventQuery(g->slot_ev[s]) != hipSuccess;
        busy += running;
        if (!running && free_slot < 0 && s < p.depth) free_slot = s;
      }
      if (busy < p.depth && free_slot >= 0 && slot_streams(g, dev, free_slot)) {
        if (!g->slot_ev[free_slot]) (void)hipEventCreateWithFlags(&g->slot_ev[free_slot], hipEventDisableTiming);
        split_enqueue(r->a, p, g->roles[free_slot], g->items[free_slot], r->ready, nullptr, g->slot_ev[free_slot],
                      r->fork, r->join_r, r->join_i, r->t0, r->t1, r->h_abort, r->done);
        g->slot_used[free_slot] = true;
#if LISLAM_ENG_STAMPS
        fprintf(stderr, "dispatch gen %u slot %d at %.3f ms (queued %zu, busy %d)\n", p.ctl.gen, free_slot,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(),
                g->q.size(), busy);
#endif
        g->q.erase(g->q.begin() + (long)at);
        delete static_cast<SplitPlan*>(r->plan);
        r->plan = nullptr;
        r->state.store(2);
        g->cv_launched.notify_all();
        continue;
      }
    }
    (void)hipGetLastError();  // hipEventQuery's not-ready status
    lk.unlock();
    std::this_thread::sleep_for(std::chrono::microseconds(20));
    lk.lock();
  }
}

// At process exit (contexts never destroyed): the dispatchers launch what is queued and stop
// before the runtime is torn down.
static void stop_dispatchers() {
  for (int d = 0; d < 64; d++) {
    EngineGate* g = engine_gate(d);
    {
      std::lock_guard<std::mutex> lk(g->mu);
      if (!g->th) continue;
      g->stop = true;
      g->cv_req.notify_all();
    }
    g->th->join();
    delete g->th;
    g->th = nullptr;
  }
}

int submit_odometry_chain_split(EngineRequest* r) {
  if (r->a.n_chains <= 0) return 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  EngineGate* g = engine_gate(dev);
  if (!g) return 0;
  std::lock_guard<std::mutex> lk(g->mu);
  if (!probe_engine_streams(g, dev)) return 0;
  if (!g->th) {
    static std::once_flag once;
    std::call_once(once, [] { std::atexit(stop_dispatchers); });
    g->stop = false;
    g->th = new std::thread(dispatcher_loop, g, dev);
  }
  r->plan = new SplitPlan(split_plan(r->a, dev));
  r->state.store(1);
  g->q.push_back(r);
  g->cv_req.notify_one();
  return 1;
}

void wait_engine_launched(EngineRequest* r) {
  if (r->state.load() != 1) return;
  int dev = 0;
  (void)hipGetDevice(&dev);
  EngineGate* g = engine_gate(dev);
  std::unique_lock<std::mutex> lk(g->mu);
  g->cv_launched.wait(lk, [&] { return r->state.load() != 1; });
}

void launch_factors_raw(const RawFactorArgs& a, hipStream_t st) {
  if (a.n > 0) hipLaunchKernelGGL(k_eval_factors_raw, dim3((a.n + 255) / 256), dim3(256), 0, st, a);
}

void launch_factors(const FactorArgs& a, hipStream_t st) {
  if (a.n > 0) hipLaunchKernelGGL(k_eval_factors, dim3((a.n + 255) / 256), dim3(256), 0, st, a);
}

void launch_target_index(const OdomArgs& a, int n_scans, hipStream_t st) {
  // less-flat clouds: 8 waves of 32 keys per lane (16384 keys in registers); less-sharp + query
  // clouds: 8 waves of 16 (8192 keys).  Workgroups of 512 threads at <= 128 VGPRs and 32 KiB of LDS
  // run beside the chain engine's item workgroups (2 waves per SIMD at 128 VGPRs).
  // One launch (k_target_index_all); LISLAM_TI_SPLIT=1: the two launches (A/B).
  static const bool split = getenv("LISLAM_TI_SPLIT") && atoi(getenv("LISLAM_TI_SPLIT")) == 1;
  if (!split) {
    hipLaunchKernelGGL(k_target_index_all, dim3(4 * n_scans), dim3(512), 0, st, a, n_scans);
    return;
  }
  hipLaunchKernelGGL((k_target_index<8, 32>), dim3(n_scans), dim3(512), 0, st, a, 1, 1, 1, 1);
  hipLaunchKernelGGL((k_target_index<8, 16>), dim3(3 * n_scans), dim3(512), 0, st, a, 3, 0, 2, 3);
}

void launch_odometry(const OdomArgs& a0, const hipStream_t* streams, int ngroups, hipEvent_t fork,
                     const hipEvent_t* join, std::vector<OdoTimed>* ev, hipEvent_t (*get_event)(void*),
                     void* owner) {
  if (a0.n_chains <= 0) return;
  const hipStream_t st = streams[0];
  hipLaunchKernelGGL(k_odom_init, dim3((a0.n_chains + 63) / 64), dim3(64), 0, st, a0);
  const int G = max(1, min(ngroups, a0.n_chains));
  if (G > 1) {
    (void)hipEventRecord(fork, st);
    for (int g = 1; g < G; g++) (void)hipStreamWaitEvent(streams[g], fork, 0);
  }
  const int qblocks16 = (a0.cap_sharp + a0.cap_flat + 8 - 1) / 8;  // 2 waves x 4 rows
  const int rounds = min(a0.chain_len, a0.S - 1);
  auto timed = [&](int kernel, hipStream_t s, auto&& launch) {
    hipEvent_t b = nullptr, e = nullptr;
    if (ev) { b = get_event(owner); (void)hipEventRecord(b, s); }
    launch();
    if (ev) { e = get_event(owner); (void)hipEventRecord(e, s); ev->push_back({kernel, b, e}); }
  };
  // round-major issue order: every group's round r is queued before any group's round r + 1
  for (int r = 0; r < rounds; r++) {
    for (int outer = 0; outer < 2; outer++) {
      for (int g = 0; g < G; g++) {
        OdomArgs a = a0;
        a.c0 = (int)((long)a0.n_chains * g / G);
        a.cn = (int)((long)a0.n_chains * (g + 1) / G) - a.c0;
        const hipStream_t s = streams[g];
        const int cb = a.cn >= 8 ? (a.cn + 7) / 8 * 8 : a.cn;
        timed(4, s, [&] {
          hipLaunchKernelGGL(k_odom_assoc16<2>, dim3(qblocks16 * cb), dim3(128), 0, s, a, r, qblocks16);
        });
        timed(5, s, [&] {
          hipLaunchKernelGGL(k_odom_lm2, dim3(a.cn), dim3(kLm2Threads), 0, s, a, r, outer);
        });
      }
    }
  }
  if (G > 1) {
    for (int g = 1; g < G; g++) {
      (void)hipEventRecord(join[g], streams[g]);
      (void)hipStreamWaitEvent(st, join[g], 0);
    }
  }
}

}  // namespace lislam
