// Device-side helpers shared by the lislam HIP kernels (gfx950 / CDNA4, wave64).
//
// FP semantics: every translation unit is built with -ffp-contract=off so that each a*b+c in
// the reference's float/double expressions rounds twice, exactly as the reference build
// (x86-64 SSE2, no -march, CMakeLists.txt:6) does.  Float atan/atan2 are the correctly rounded
// float of the double function (DESIGN.md "FP semantics"); float division and sqrt are IEEE.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lislam {

constexpr double kPi = 3.14159265358979323846;  // M_PI

struct __attribute__((aligned(16))) P4 {
  float x, y, z, i;
};

__device__ __forceinline__ float atan2_f(float y, float x) {
  return (float)atan2((double)y, (double)x);
}
__device__ __forceinline__ float atan_f(float v) { return (float)atan((double)v); }

// Explicit address spaces: a generic pointer would make hipcc emit flat_* accesses, which count on
// both vmcnt and lgkmcnt and serialize every wait.
typedef float f4v __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) f4v gf4v;
typedef __attribute__((address_space(1))) f4v gf4v_mut;
typedef const __attribute__((address_space(3))) f4v sf4v;

__device__ __forceinline__ float4 ldg(const void* p) {  // global memory only
  const f4v v = *(gf4v*)p;
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 lds4(const void* p) {  // LDS only
  const f4v v = *(sf4v*)p;
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ P4 ld4(const P4* p) {  // global memory only
  const f4v v = *(gf4v*)p;
  return P4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void st4(P4* p, const P4& v) {  // global memory only
  f4v w = {v.x, v.y, v.z, v.i};
  *(gf4v_mut*)p = w;
}

// scanRegistration.cpp:290-331: scan line of a point from its elevation; -1 = dropped.
__device__ __forceinline__ int scan_id_of(float angle, int n_scans) {
  int id;
  if (n_scans == 16) {
    id = int((angle + 15) / 2 + 0.5);
  } else if (n_scans == 32) {
    id = int((angle + 92.0 / 3.0) * 3.0 / 4.0);
  } else if (n_scans == 64) {
    id = int((angle + 22.5) * 1.41 + 0.5) - 1;
  } else {
    id = int((angle + 22.5) * 2.83 + 0.5) - 1;
  }
  return (id > n_scans - 1 || id < 0) ? -1 : id;
}

__device__ __forceinline__ float elevation_deg(const P4& p) {
  // atan(z / sqrt(x*x + y*y)) * 180 / M_PI with float atan/sqrt (scanRegistration.cpp:285)
  return (float)((double)(atan_f(p.z / sqrtf(p.x * p.x + p.y * p.y)) * 180) / kPi);
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Order this wave's earlier LDS writes before its later LDS reads (lanes exchanging data through
// LDS inside one wave, no workgroup barrier).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- wave reductions (DPP)
// Wave-wide unsigned minimum / maximum, returned uniform: DPP within each 16-lane row (quad xor 1,
// xor 2, half-row mirror, row mirror; each folds into one v_min/max_u32_dpp), then row_bcast:15 /
// row_bcast:31 carry the row results up to lane 63.  Every lane of the wave must be active.
#define LISLAM_WAVE_RED(op, v)                                                                          \
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, true));  /* quad_perm [1,0,3,2] */ \
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, true));  /* quad_perm [2,3,0,1] */ \
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, true)); /* row_half_mirror */     \
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, true)); /* row_mirror */          \
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xa, 0xf, false)); /* bcast15 */  \
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xc, 0xf, false)); /* bcast31 */
__device__ __forceinline__ uint32_t wave_umin(uint32_t v) {
  LISLAM_WAVE_RED(min, v)
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t wave_umax(uint32_t v) {
  LISLAM_WAVE_RED(max, v)
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
#undef LISLAM_WAVE_RED
// Two independent minima interleaved step by step (each step's DPP read waits on the previous
// step's write; the other reduction fills those wait states).
__device__ __forceinline__ void wave_umin2(uint32_t& a, uint32_t& b) {
#define LISLAM_UMIN2_STEP(ctrl)                                                   \
  a = min(a, (uint32_t)__builtin_amdgcn_mov_dpp((int)a, ctrl, 0xf, 0xf, true)); \
  b = min(b, (uint32_t)__builtin_amdgcn_mov_dpp((int)b, ctrl, 0xf, 0xf, true));
  LISLAM_UMIN2_STEP(0xB1)
  LISLAM_UMIN2_STEP(0x4E)
  LISLAM_UMIN2_STEP(0x141)
  LISLAM_UMIN2_STEP(0x140)
#undef LISLAM_UMIN2_STEP
  a = min(a, (uint32_t)__builtin_amdgcn_update_dpp((int)a, (int)a, 0x142, 0xa, 0xf, false));
  b = min(b, (uint32_t)__builtin_amdgcn_update_dpp((int)b, (int)b, 0x142, 0xa, 0xf, false));
  a = min(a, (uint32_t)__builtin_amdgcn_update_dpp((int)a, (int)a, 0x143, 0xc, 0xf, false));
  b = min(b, (uint32_t)__builtin_amdgcn_update_dpp((int)b, (int)b, 0x143, 0xc, 0xf, false));
  a = (uint32_t)__builtin_amdgcn_readlane((int)a, 63);
  b = (uint32_t)__builtin_amdgcn_readlane((int)b, 63);
}
// 64-bit minimum: the minimum high word, then the minimum low word among the lanes holding it
// (one lane in the common case: read directly).
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
  const uint32_t m = wave_umin(hi);
  const uint64_t tie = __ballot(hi == m);
  const uint32_t l = __popcll(tie) == 1 ? (uint32_t)__builtin_amdgcn_readlane((int)lo, (int)__builtin_ctzll(tie))
                                        : wave_umin(hi == m ? lo : 0xffffffffu);
  return ((uint64_t)m << 32) | l;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) { return ~wave_min_u64(~v); }

// ---------------------------------------------------------------- register bitonic sort
// Keys of one wave in registers: index i = base + 64 t + lane (slot t < kS, base = the wave's
// offset in a workgroup-wide sort, a multiple of 64 kS).  One stage of the bitonic network
// compare-exchanges i with i ^ j in direction ((i & k) == 0).
template <int kS, int kJJ>  // partner i ^ (64 kJJ): slot t ^ kJJ of the same lane
__device__ __forceinline__ void bx_slots(uint64_t (&key)[kS], int k, int base) {
  if constexpr (kJJ < kS) {
#pragma unroll
    for (int t = 0; t < kS; t++) {
      if (t & kJJ) continue;
      const int u = t | kJJ;
      const bool up = ((base | (t * 64)) & k) == 0;
      const uint64_t x = key[t], y = key[u];
      const bool sw = (x > y) == up;
      key[t] = sw ? y : x;
      key[u] = sw ? x : y;
    }
  }
}
template <int kJ>
__device__ __forceinline__ uint32_t xor_lane32(uint32_t v) {
  if constexpr (kJ == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, true);  // quad_perm [1,0,3,2]
  else if constexpr (kJ == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, true);  // [2,3,0,1]
  else if constexpr (kJ < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (kJ << 10) | 0x1f);  // xor mask
  else return (uint32_t)__builtin_amdgcn_ds_bpermute((lane_id() ^ 32) << 2, (int)v);
}
template <int kS, int kJ>  // partner i ^ kJ: lane ^ kJ, same slot
__device__ __forceinline__ void bx_lanes(uint64_t (&key)[kS], int k, int base) {
  const int lane = lane_id();
  const bool lower = (lane & kJ) == 0;
#pragma unroll
  for (int t = 0; t < kS; t++) {
    const uint64_t x = key[t];
    const uint64_t y = ((uint64_t)xor_lane32<kJ>((uint32_t)(x >> 32)) << 32) | xor_lane32<kJ>((uint32_t)x);
    const bool up = ((base | (t * 64) | lane) & k) == 0;
    key[t] = (lower == up) ? (x < y ? x : y) : (x < y ? y : x);
    if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // four slots' exchanges in flight (registers)
  }
}
// Every stage j < 64 kS of level k (the in-wave part of the network).
template <int kS>
__device__ __forceinline__ void reg_bitonic_level(uint64_t (&key)[kS], int k, int jmax, int base) {
  for (int j = jmax; j > 0; j >>= 1) {
    switch (j) {
      case 1: bx_lanes<kS, 1>(key, k, base); break;
      case 2: bx_lanes<kS, 2>(key, k, base); break;
      case 4: bx_lanes<kS, 4>(key, k, base); break;
      case 8: bx_lanes<kS, 8>(key, k, base); break;
      case 16: bx_lanes<kS, 16>(key, k, base); break;
      case 32: bx_lanes<kS, 32>(key, k, base); break;
      case 64: bx_slots<kS, 1>(key, k, base); break;
      case 128: bx_slots<kS, 2>(key, k, base); break;
      case 256: bx_slots<kS, 4>(key, k, base); break;
      case 512: bx_slots<kS, 8>(key, k, base); break;
      default: bx_slots<kS, 16>(key, k, base); break;
    }
  }
}
// Ascending bitonic sort of the 64 kS keys of one wave (every slot: a runtime slot bound doubled
// the registers the exchanges hold).
template <int kS>
__device__ __forceinline__ void reg_bitonic(uint64_t (&key)[kS]) {
  constexpr int P = 64 * kS;
  for (int k = 2; k <= P; k <<= 1) reg_bitonic_level<kS>(key, k, k >> 1, 0);
}

// ---------------------------------------------------------------- double 3-vectors / quats
struct D3 {
  double x, y, z;
};
__device__ __forceinline__ D3 operator+(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ D3 operator-(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ D3 operator*(double s, D3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ D3 cross(D3 a, D3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

struct DQ {
  double x, y, z, w;
};

// Eigen's Quaternion * Vector3 (_transformVector): uv = 2 (q.vec x v); v + w uv + q.vec x uv.
__device__ __forceinline__ D3 qrot(const DQ& q, D3 v) {
  D3 qv{q.x, q.y, q.z};
  D3 uv = cross(qv, v);
  uv = uv + uv;
  D3 wuv{q.w * uv.x, q.w * uv.y, q.w * uv.z};
  return (v + wuv) + cross(qv, uv);
}

// Quaternion product in the term grouping of Eigen 3.3's SSE2 quat_product<double>.
__device__ __forceinline__ DQ qmul(const DQ& a, const DQ& b) {
  DQ r;
  r.x = (a.w * b.x + a.y * b.z) + (-(a.z * b.y - a.x * b.w));
  r.y = (a.w * b.y + a.y * b.w) + (a.z * b.x - a.x * b.z);
  r.z = (a.w * b.z - a.y * b.x) + (a.z * b.w + a.x * b.y);
  r.w = (a.w * b.w - a.y * b.y) + (-(a.z * b.z + a.x * b.x));
  return r;
}

}  // namespace lislam
