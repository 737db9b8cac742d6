// lislam ground-plane extraction on gfx950: ImageHandler::groundPlaneExtraction
// (src/image_handler.h_ouster:41-100), the RANSAC ground cloud mapOptimization merges with the
// less-flat cloud (src/mapOptimization.cpp:136,148) — SURVEY.md §8(f) row 3.
//
// Semantics are those of oracle/oracle_ground.cpp (PCL 1.10 single-thread SACSegmentation,
// SACMODEL_PLANE, RANSAC, threshold 0.01, optimized coefficients; then the n.z > cos 15 deg test
// and the 0.03 m height band in double).  For a batch of S organized scans resident in HBM:
//   k_ground_screen   1 WG per scan: ordered compaction of the points with z in [-2, -0.45]
//                     (:49-54, index order) into a candidate list.
//   k_ground_ransac   1 WG per scan:
//                     - one lane replays PCL's sampling — the mt19937(12345) >> 1 draw sequence is
//                       the same for every call, so it is a host-precomputed table, and the
//                       partial Fisher-Yates of drawIndexSample runs on an LDS hash map of the
//                       touched positions — and builds up to max_iterations + 1 = 51 plane
//                       hypotheses (they do not depend on the inlier counts);
//                     - the workgroup counts the inliers of every hypothesis, 16 hypotheses per
//                       pass over the candidates (register counters);
//                     - one lane replays RandomSampleConsensus::computeModel's adaptive-k loop on
//                       the counts (the same best model and iteration count as the sequential loop);
//                     - the refit's float sums run in PCL's sequential inlier order: the workgroup
//                       stages each inlier's 9 products in LDS (candidate order), one lane per
//                       accumulator adds them in order; then pcl::eigen33 on one lane.
//   k_ground_extract  1 WG per scan: ordered compaction of the points within 0.03 m of the plane
//                     with z < 0 (:79-89), in double.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <random>
#include <vector>

#include "lislam_batch.hpp"
#include "lislam_ctx.hpp"
#include "lislam_device.hpp"

namespace lislam {
namespace ground {

constexpr int kThreads = 1024;          // screen / extract
constexpr int kRansacThreads = 1024;
constexpr int kMaxHyp = 51;             // max_iterations (50) + 1
constexpr int kMaxSampleChecks = 1000;  // SampleConsensusModel::max_sample_checks_
constexpr int kTable = kMaxHyp * kMaxSampleChecks * 3;  // every draw computeModel can make
constexpr int kHash = 4096;             // LDS slots of the shuffled-position map (<= 2048 used)
constexpr int kTabLds = 1024;           // draws staged in LDS (a call needs ~160 without retries)
// setDistanceThreshold(0.01): a float distance d satisfies d < 0.01 (double) exactly when
// d < 0x1.47ae16p-7f, the float after (float)0.01 (which is below 0.01)
constexpr float kThrF = 0.010000000707805157f;

struct Args {
  const float4* pts;  // [S][N] x, y, z, intensity
  int S, N;
  float4* cand;       // [S][N] screened candidates (x, y, z, 0)
  int* ncand;         // [S]
  float4* out;        // [S][N] ground cloud (x, y, z, 1)
  int* nout;          // [S]
  float* plane;       // [S][4]
  int* info;          // [S][4] status, iterations, best inliers, refit inliers
  const uint32_t* tab;  // [kTable] mt19937(12345) outputs >> 1
};

// Block-wide exclusive prefix of a flag (ballot + per-wave counts); *tot = the block's count.
__device__ __forceinline__ int block_rank(int* wsum, bool flag, int* tot) {
  const uint64_t b = __ballot(flag);
  const int lane = lane_id(), w = threadIdx.x >> 6;
  if (lane == 0) wsum[w] = __popcll(b);
  __syncthreads();
  int before = 0, all = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); k++) {
    const int v = wsum[k];
    if (k < w) before += v;
    all += v;
  }
  __syncthreads();
  *tot = all;
  return before + __popcll(b & lanemask_lt());
}

__global__ __launch_bounds__(kThreads) void k_ground_screen(Args a) {
  __shared__ int wsum[kThreads / 64];
  const int s = blockIdx.x;
  const float4* P = a.pts + (size_t)s * a.N;
  float4* C = a.cand + (size_t)s * a.N;
  int m = 0;
  for (int b0 = 0; b0 < a.N; b0 += kThreads) {
    const int i = b0 + threadIdx.x;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    bool keep = false;
    if (i < a.N) {
      p = ldg(P + i);
      keep = (double)p.z >= -2.0 && (double)p.z <= -0.45;
    }
    int tot;
    const int r = block_rank(wsum, keep, &tot);
    if (keep) *(gf4v_mut*)(C + m + r) = f4v{p.x, p.y, p.z, 0.f};
    m += tot;
  }
  if (threadIdx.x == 0) a.ncand[s] = m;
}

// ---- plane arithmetic, in the oracle's (PCL / Eigen 3.3 SSE) operation order
__device__ __forceinline__ float sum4(float e0, float e1, float e2, float e3) { return (e0 + e2) + (e1 + e3); }
__device__ __forceinline__ float sum3(float e0, float e1, float e2) { return e0 + (e1 + e2); }

__device__ __forceinline__ bool sample_good(float4 p0, float4 p1, float4 p2) {
  const float d0 = (p1.x - p0.x) / (p2.x - p0.x), d1 = (p1.y - p0.y) / (p2.y - p0.y), d2 = (p1.z - p0.z) / (p2.z - p0.z);
  return (d0 != d1) || (d2 != d1);
}

__device__ __forceinline__ float4 plane_from_3(float4 p0, float4 p1, float4 p2) {
  const float a0 = p1.x - p0.x, a1 = p1.y - p0.y, a2 = p1.z - p0.z;
  const float b0 = p2.x - p0.x, b1 = p2.y - p0.y, b2 = p2.z - p0.z;
  float c[4] = {a1 * b2 - a2 * b1, a2 * b0 - a0 * b2, a0 * b1 - a1 * b0, 0.f};
  const float z = sum4(c[0] * c[0], c[1] * c[1], c[2] * c[2], c[3] * c[3]);
  if (z > 0.f) {
    const float sq = sqrtf(z);
    for (int k = 0; k < 4; k++) c[k] /= sq;
  }
  c[3] = -1.f * sum4(c[0] * p0.x, c[1] * p0.y, c[2] * p0.z, c[3] * 1.f);
  return make_float4(c[0], c[1], c[2], c[3]);
}

__device__ __forceinline__ float plane_dist(float4 c, float4 p) {
  return fabsf(sum4(c.x * p.x, c.y * p.y, c.z * p.z, c.w * 1.f));
}

__device__ __forceinline__ float f_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
__device__ __forceinline__ float f_cos(float v) { return (float)cos((double)v); }
__device__ __forceinline__ float f_sin(float v) { return (float)sin((double)v); }

__device__ void compute_roots2(float b, float c, float* r) {
  r[0] = 0.f;
  float d = (float)((double)(b * b) - 4.0 * (double)c);
  if (d < 0.0) d = 0.f;
  const float sd = sqrtf(d);
  r[2] = 0.5f * (b + sd);
  r[1] = 0.5f * (b - sd);
}

__device__ void compute_roots(const float* m, float* r) {
  const float m00 = m[0], m01 = m[1], m02 = m[2], m11 = m[4], m12 = m[5], m22 = m[8];
  const float c0 = m00 * m11 * m22 + 2.f * m01 * m02 * m12 - m00 * m12 * m12 - m11 * m02 * m02 - m22 * m01 * m01;
  const float c1 = m00 * m11 - m01 * m01 + m00 * m22 - m02 * m02 + m11 * m22 - m12 * m12;
  const float c2 = m00 + m11 + m22;
  if (fabsf(c0) < 1.1920928955078125e-07f) {  // FLT_EPSILON
    compute_roots2(c2, c1, r);
    return;
  }
  const float s_inv3 = (float)(1.0 / 3.0);
  const float s_sqrt3 = sqrtf(3.0f);
  const float c2_over_3 = c2 * s_inv3;
  float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
  if (a_over_3 > 0.f) a_over_3 = 0.f;
  const float half_b = 0.5f * (c0 + c2_over_3 * (2.f * c2_over_3 * c2_over_3 - c1));
  float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
  if (q > 0.f) q = 0.f;
  const float rho = sqrtf(-a_over_3);
  const float theta = f_atan2(sqrtf(-q), half_b) * s_inv3;
  const float ct = f_cos(theta), st = f_sin(theta);
  r[0] = c2_over_3 + 2.f * rho * ct;
  r[1] = c2_over_3 - rho * (ct + s_sqrt3 * st);
  r[2] = c2_over_3 - rho * (ct - s_sqrt3 * st);
  float t;
  if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
  if (r[1] >= r[2]) {
    t = r[1]; r[1] = r[2]; r[2] = t;
    if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
  }
  if (r[0] <= 0.f) compute_roots2(c2, c1, r);
}

__device__ void eigen33_min(const float* mat, float* ev) {
  float scale = 0.f;
  for (int k = 0; k < 9; k++) scale = fmaxf(scale, fabsf(mat[k]));
  if (scale <= 1.17549435e-38f) scale = 1.f;  // FLT_MIN
  float m[9];
  for (int k = 0; k < 9; k++) m[k] = mat[k] / scale;
  float r[3];
  compute_roots(m, r);
  m[0] -= r[0];
  m[4] -= r[0];
  m[8] -= r[0];
  float v[3][3];
  const int pi[3] = {0, 0, 1}, pj[3] = {1, 2, 2};
  float l[3];
  for (int c = 0; c < 3; c++) {
    const float* x = m + 3 * pi[c];
    const float* y = m + 3 * pj[c];
    v[c][0] = x[1] * y[2] - x[2] * y[1];
    v[c][1] = x[2] * y[0] - x[0] * y[2];
    v[c][2] = x[0] * y[1] - x[1] * y[0];
    l[c] = sum3(v[c][0] * v[c][0], v[c][1] * v[c][1], v[c][2] * v[c][2]);
  }
  const int c = (l[0] >= l[1] && l[0] >= l[2]) ? 0 : (l[1] >= l[0] && l[1] >= l[2]) ? 1 : 2;
  const float sq = sqrtf(l[c]);
  for (int k = 0; k < 3; k++) ev[k] = v[c][k] / sq;
}

struct RansacShared {
  int hkey[kHash];   // position + 1, 0 = empty
  int hval[kHash];
  float4 hyp[kMaxHyp];
  int cnt[kMaxHyp];
  int nhyp, fail_at, used;
  int best, iters, status;
  float4 model;
  float prod[kRansacThreads][9];  // per-inlier products x x, x y, x z, y y, y z, z z, x, y, z (in order)
  float acc[9];
  int ninl;
  int wsum[kRansacThreads / 64];
  uint32_t tab[kTabLds];
};

// value of shuffled_indices_[pos] (identity unless touched)
__device__ __forceinline__ int sh_get(RansacShared& sh, int pos) {
  uint32_t h = ((uint32_t)pos * 2654435761u) & (kHash - 1);
  for (;;) {
    const int k = sh.hkey[h];
    if (k == 0) return pos;
    if (k == pos + 1) return sh.hval[h];
    h = (h + 1) & (kHash - 1);
  }
}
__device__ __forceinline__ bool sh_set(RansacShared& sh, int pos, int val) {
  uint32_t h = ((uint32_t)pos * 2654435761u) & (kHash - 1);
  for (;;) {
    const int k = sh.hkey[h];
    if (k == 0) {
      if (++sh.used > kHash / 2) return false;
      sh.hkey[h] = pos + 1;
      sh.hval[h] = val;
      return true;
    }
    if (k == pos + 1) { sh.hval[h] = val; return true; }
    h = (h + 1) & (kHash - 1);
  }
}

#ifdef LISLAM_PHASE_PROF
__device__ unsigned long long g_ground_phase[8];
extern "C" int lislam_debug_ground_phases(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ground_phase), sizeof(g_ground_phase)) != hipSuccess) return -2;
  static const unsigned long long zero[8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_ground_phase), zero, sizeof(zero)) == hipSuccess ? 0 : -2;
}
#define G_PHASE(i)                                                   \
  do {                                                               \
    __syncthreads();                                                 \
    if (threadIdx.x == 0) {                                          \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime(); \
      atomicAdd(&g_ground_phase[i], now_ - t_ph);                    \
      t_ph = now_;                                                   \
    }                                                                \
  } while (0)
#else
#define G_PHASE(i)
#endif
__global__ __launch_bounds__(kRansacThreads) void k_ground_ransac(Args a) {
  __shared__ RansacShared sh;
#ifdef LISLAM_PHASE_PROF
  unsigned long long t_ph = __builtin_amdgcn_s_memrealtime();
#endif
  const int s = blockIdx.x, tid = threadIdx.x, lane = lane_id();
  const int n = a.ncand[s];
  const float4* C = a.cand + (size_t)s * a.N;
  int* info = a.info + (size_t)s * 4;
  float* plane = a.plane + (size_t)s * 4;
  if (n < 3) {  // getSamples: too few points; the model stays empty
    if (tid < 4) { info[tid] = tid == 0 ? -1 : 0; plane[tid] = 0.f; }
    return;
  }
  for (int k = tid; k < kHash; k += kRansacThreads) sh.hkey[k] = 0;
  for (int k = tid; k < kTabLds; k += kRansacThreads) sh.tab[k] = a.tab[k];
  __syncthreads();
  // 1. the hypotheses (SampleConsensusModel::getSamples + computeModelCoefficients), one lane;
  //    shuffled_indices_[0..2] live in registers, the other touched positions in the LDS map
  if (tid == 0) {
    sh.used = 0;
    int draw = 0, h = 0, fail_at = -1;
    int head[3] = {0, 1, 2};
    bool overflow = false;
    for (; h < kMaxHyp && !overflow; h++) {
      bool got = false;
      for (int chk = 0; chk < kMaxSampleChecks && !got && !overflow; chk++) {
#pragma unroll
        for (int i = 0; i < 3; i++) {
          const uint32_t r = draw < kTabLds ? sh.tab[draw] : a.tab[draw];
          draw++;
          const int j = i + (int)(r % (uint32_t)(n - i));
          const int vi = head[i];
          if (j < 3) {
            head[i] = head[j];
            head[j] = vi;
          } else {
            head[i] = sh_get(sh, j);
            overflow |= !sh_set(sh, j, vi);
          }
        }
        got = sample_good(ldg(C + head[0]), ldg(C + head[1]), ldg(C + head[2]));
      }
      if (!got) { fail_at = h; break; }
      sh.hyp[h] = plane_from_3(ldg(C + head[0]), ldg(C + head[1]), ldg(C + head[2]));
    }
    sh.nhyp = h;
    sh.fail_at = overflow ? -2 : fail_at;
  }
  __syncthreads();
  G_PHASE(0);
  const int H = sh.nhyp;
  if (sh.fail_at == -2) {  // more touched positions than the LDS map holds (pathological input)
    if (tid < 4) { info[tid] = tid == 0 ? -3 : 0; plane[tid] = 0.f; }
    return;
  }
  // 2. inlier counts of every hypothesis (countWithinDistance), one pass over the candidates
  for (int h = tid; h < kMaxHyp; h += kRansacThreads) sh.cnt[h] = 0;
  __syncthreads();
  constexpr int kGroup = 16;  // hypotheses counted per pass over the candidates (register counters)
  for (int h0 = 0; h0 < H; h0 += kGroup) {
    int cnt[kGroup];
#pragma unroll
    for (int h = 0; h < kGroup; h++) cnt[h] = 0;
    for (int i = tid; i < n; i += kRansacThreads) {
      const float4 p = ldg(C + i);
#pragma unroll
      for (int h = 0; h < kGroup; h++) {
        if (h0 + h < H) {
          const float4 hy = lds4(&sh.hyp[h0 + h]);
          cnt[h] += plane_dist(hy, p) < kThrF;
        }
      }
    }
#pragma unroll
    for (int h = 0; h < kGroup; h++) {
      if (h0 + h < H) {  // uniform
        int v = cnt[h];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) atomicAdd(&sh.cnt[h0 + h], v);
      }
    }
  }
  __syncthreads();
  G_PHASE(1);
  // 3. RandomSampleConsensus::computeModel's loop on the counts, one lane
  if (tid == 0) {
    int it = 0, best = -0x7fffffff, bh = -1;
    double k = 1.0;
    const double logp = log(1.0 - 0.99), inv_n = 1.0 / (double)n;
    while (it < k) {
      if (it >= H) break;  // getSamples found no good sample (fail_at == it)
      const int c = sh.cnt[it];
      if (c > best) {
        best = c;
        bh = it;
        const double w = (double)best * inv_n;
        double pno = 1.0 - pow(w, 3.0);
        pno = fmax(2.220446049250313e-16, pno);
        pno = fmin(1.0 - 2.220446049250313e-16, pno);
        k = logp / log(pno);
      }
      ++it;
      if (it > kMaxHyp - 1) break;
    }
    sh.iters = it;
    sh.best = best;
    sh.status = bh >= 0 ? 1 : -2;
    if (bh >= 0) sh.model = sh.hyp[bh];
  }
  __syncthreads();
  if (sh.status < 0) {
    if (tid < 4) { info[tid] = tid == 0 ? -2 : tid == 1 ? sh.iters : 0; plane[tid] = 0.f; }
    return;
  }
  // 4. selectWithinDistance + computeMeanAndCovarianceMatrix in inlier order
  {
    // every round: the workgroup tests 1024 candidates, writes the 9 products of each inlier to
    // LDS in candidate order (one rounding each, as the sequential loop), then lane e < 9 of
    // wave 0 adds column e in order
    const float4 M = sh.model;
    float acc = 0.f;
    int ni = 0;
    for (int b0 = 0; b0 < n; b0 += kRansacThreads) {
      const int i = b0 + tid;
      float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < n) p = ldg(C + i);
      const bool inl = i < n && plane_dist(M, p) < kThrF;
      int tot;
      const int r = block_rank(sh.wsum, inl, &tot);
      if (inl) {
        float* o = sh.prod[r];
        o[0] = p.x * p.x; o[1] = p.x * p.y; o[2] = p.x * p.z;
        o[3] = p.y * p.y; o[4] = p.y * p.z; o[5] = p.z * p.z;
        o[6] = p.x; o[7] = p.y; o[8] = p.z;
      }
      __syncthreads();
      if (tid < 9) {
        int k = 0;
        for (; k + 8 <= tot; k += 8) {
          float v[8];
#pragma unroll
          for (int t = 0; t < 8; t++) v[t] = sh.prod[k + t][tid];
#pragma unroll
          for (int t = 0; t < 8; t++) acc += v[t];
        }
        for (; k < tot; k++) acc += sh.prod[k][tid];
      }
      ni += tot;
      __syncthreads();
    }
    if (tid < 9) sh.acc[tid] = acc;
    if (tid == 0) sh.ninl = ni;
  }
  __syncthreads();
  G_PHASE(2);
  if (tid == 0) {
    float4 coef = sh.model;
    const int ni = sh.ninl;
    if (ni > 3) {  // optimizeModelCoefficients (more than the 3-point sample)
      float acc[9];
      for (int e = 0; e < 9; e++) acc[e] = sh.acc[e] / (float)ni;
      float cov[9];
      cov[0] = acc[0] - acc[6] * acc[6];
      cov[1] = acc[1] - acc[6] * acc[7];
      cov[2] = acc[2] - acc[6] * acc[8];
      cov[4] = acc[3] - acc[7] * acc[7];
      cov[5] = acc[4] - acc[7] * acc[8];
      cov[8] = acc[5] - acc[8] * acc[8];
      cov[3] = cov[1];
      cov[6] = cov[2];
      cov[7] = cov[5];
      float ev[3];
      eigen33_min(cov, ev);
      coef = make_float4(ev[0], ev[1], ev[2], 0.f);
      coef.w = -1.f * sum4(coef.x * acc[6], coef.y * acc[7], coef.z * acc[8], coef.w * 1.f);
    }
    plane[0] = coef.x; plane[1] = coef.y; plane[2] = coef.z; plane[3] = coef.w;
    const float nz = sum3(coef.x * 0.f, coef.y * 0.f, coef.z * 1.f);
    info[0] = ((double)nz > cos(15 * kPi / 180)) ? 1 : 0;
    info[1] = sh.iters;
    info[2] = sh.best;
    info[3] = ni;
  }
  G_PHASE(3);
}

__global__ __launch_bounds__(kThreads) void k_ground_extract(Args a) {
  __shared__ int wsum[kThreads / 64];
  const int s = blockIdx.x;
  const int* info = a.info + (size_t)s * 4;
  if (info[0] != 1) {
    if (threadIdx.x == 0) a.nout[s] = 0;
    return;
  }
  const float* pl = a.plane + (size_t)s * 4;
  const double A = pl[0], B = pl[1], Cc = pl[2], D = pl[3];
  const double nrm = sqrt(A * A + B * B + Cc * Cc);
  const float4* P = a.pts + (size_t)s * a.N;
  float4* O = a.out + (size_t)s * a.N;
  int m = 0;
  for (int b0 = 0; b0 < a.N; b0 += kThreads) {
    const int i = b0 + threadIdx.x;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    bool keep = false;
    if (i < a.N) {
      p = ldg(P + i);
      const double X = p.x, Y = p.y, Z = p.z;
      const double height = fabs(A * X + B * Y + Cc * Z + D) / nrm;
      keep = height <= 0.03 && p.z < -0.0f;
    }
    int tot;
    const int r = block_rank(wsum, keep, &tot);
    if (keep) *(gf4v_mut*)(O + m + r) = f4v{p.x, p.y, p.z, 1.f};
    m += tot;
  }
  if (threadIdx.x == 0) a.nout[s] = m;
}

// ------------------------------------------------------------------ host side
struct Engine {
  int S = 0, N = 0;
  float4* cand = nullptr;
  int* ncand = nullptr;
  float4* out = nullptr;
  int* nout = nullptr;
  float* plane = nullptr;
  int* info = nullptr;
  uint32_t* tab = nullptr;
  ~Engine() {
    for (void* p : {(void*)cand, (void*)ncand, (void*)out, (void*)nout, (void*)plane, (void*)info, (void*)tab})
      if (p) (void)hipFree(p);
  }
};

}  // namespace ground
}  // namespace lislam

using lislam::ground::Engine;

void lislam_free_ground(void* p) { delete static_cast<Engine*>(p); }

static int gfail(lislam_ctx* c, int code, const char* msg) {
  if (c) c->err = msg;
  return code;
}

// Ground outputs of one scan of a batch (lislam_batch_download).
int lislam_ground_batch_output(lislam_batch* b, int what, int scan, const void** src, int* cnt, size_t* esz) {
  const Engine* e = static_cast<const Engine*>(b->ground);
  if (!e || scan >= e->S) return LISLAM_ERR_STATE;
  switch (what) {
    case LISLAM_OUT_GROUND:
      if (hipMemcpy(cnt, e->nout + scan, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return LISLAM_ERR_DEVICE;
      *src = e->out + (size_t)scan * e->N;
      *esz = 16;
      return LISLAM_OK;
    case LISLAM_OUT_GROUND_PLANE: *src = e->plane + (size_t)scan * 4; *cnt = 4; *esz = 4; return LISLAM_OK;
    case LISLAM_OUT_GROUND_INFO: *src = e->info + (size_t)scan * 4; *cnt = 4; *esz = 4; return LISLAM_OK;
    default: return LISLAM_ERR_ARG;
  }
}

extern "C" int lislam_batch_ground(lislam_batch* b, int32_t n_scans) {
  if (!b || n_scans < 1 || n_scans > b->max_scans) return LISLAM_ERR_ARG;
  lislam_ctx* c = b->ctx;
  hipSetDevice(c->device);
  Engine* e = static_cast<Engine*>(b->ground);
  if (!e) {
    e = new Engine();
    e->S = b->max_scans;
    e->N = b->N;
    const size_t SN = (size_t)e->S * e->N;
    bool ok = hipMalloc(&e->cand, SN * sizeof(float4)) == hipSuccess && hipMalloc(&e->out, SN * sizeof(float4)) == hipSuccess &&
              hipMalloc(&e->ncand, e->S * sizeof(int)) == hipSuccess && hipMalloc(&e->nout, e->S * sizeof(int)) == hipSuccess &&
              hipMalloc(&e->plane, e->S * 4 * sizeof(float)) == hipSuccess &&
              hipMalloc(&e->info, e->S * 4 * sizeof(int)) == hipSuccess &&
              hipMalloc(&e->tab, lislam::ground::kTable * sizeof(uint32_t)) == hipSuccess;
    if (ok) {  // boost::uniform_int<>(0, INT_MAX) over boost::mt19937(12345): every draw of computeModel
      std::vector<uint32_t> h(lislam::ground::kTable);
      std::mt19937 g(12345u);
      for (auto& v : h) v = (uint32_t)g() >> 1;
      ok = hipMemcpy(e->tab, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice) == hipSuccess;
    }
    if (!ok) {
      delete e;
      return gfail(c, LISLAM_ERR_DEVICE, "lislam_batch_ground: device allocation failed");
    }
    b->ground = e;
  }
  lislam::ground::Args a{};
  a.pts = reinterpret_cast<const float4*>(b->fa.pts);
  a.S = n_scans;
  a.N = b->N;
  a.cand = e->cand; a.ncand = e->ncand; a.out = e->out; a.nout = e->nout;
  a.plane = e->plane; a.info = e->info; a.tab = e->tab;
  hipStream_t st = c->stream;
  {
    TimedScope t(c, kT_ground_screen);
    hipLaunchKernelGGL(lislam::ground::k_ground_screen, dim3(n_scans), dim3(lislam::ground::kThreads), 0, st, a);
  }
  {
    TimedScope t(c, kT_ground_ransac);
    hipLaunchKernelGGL(lislam::ground::k_ground_ransac, dim3(n_scans), dim3(lislam::ground::kRansacThreads), 0, st, a);
  }
  {
    TimedScope t(c, kT_ground_extract);
    hipLaunchKernelGGL(lislam::ground::k_ground_extract, dim3(n_scans), dim3(lislam::ground::kThreads), 0, st, a);
  }
  if (hipGetLastError() != hipSuccess) return gfail(c, LISLAM_ERR_DEVICE, "lislam_batch_ground: launch failed");
  return LISLAM_OK;
}
