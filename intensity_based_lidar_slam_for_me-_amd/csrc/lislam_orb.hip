// lislam ORB intensity front end on gfx950 (a8-a11 of SURVEY.md §8(a)): per-scan ORB detect +
// describe on the intensity image, cloud-track lookup, Hamming cross-check matching of
// consecutive scans, match selection and the front_end_residual pose solve
// (src/intensity_feature_tracker.cpp:597-941, src/lidarFeaturePointsFunction.hpp:21-58).
//
// Layout in HBM (per scan): the 8-level pyramid as OpenCV lays it out level by level — each level
// its own (h + 46) x (w + 46) byte image with a 23-pixel reflect-101 border — once unblurred
// (FAST, Harris, intensity centroid) and once with the blurred interior (descriptors sample the
// blurred interior and the unblurred border, as OpenCV's in-place GaussianBlur of the level ROI
// leaves them); FAST scores per level pixel; keypoints as float x, y, size, angle, response,
// octave; descriptors 32 B; cloud points float4.
//
// Kernels (the semantics are those of oracle/oracle_orb.cpp, which restates OpenCV 4.x):
//   k_orb_pyramid   1 WG per scan (images whose levels 0 + 1 fit LDS, e.g. 64 x 1024): the level
//                   chain in LDS — levels 1..7 by the bit-exact fixed-point INTER_LINEAR_EXACT
//                   resize of the previous level — and each level's ROI rows (border columns
//                   included) written once
//   k_orb_level     (larger images) per level, in order, 1 thread per 4 padded pixels: the same
//                   resize; border pixels evaluate their reflect-101 source directly
//   k_orb_blur      (larger images) 1 WG per band of 8 padded rows, staged in LDS: 7x7 sigma-2
//                   separable float Gaussian (row sums then the symmetric column sum, the
//                   FilterEngine order) on the ROI, border copy
//   k_orb_fastnms   1 WG per band of LISLAM_FAST_BAND level rows, reflect-staged in LDS: cheap test
//                   of every pixel of the band into one candidate list, FAST-9/16 segment test +
//                   cornerScore<16> of the list into an LDS score tile, then 3x3 non-max
//                   suppression, mask, border; after k_orb_pyramid also the band's blurred rows
//                   (packed float pairs) and the level's border rows
//   k_orb_select    1 WG per (scan, level): ordered compaction (a contiguous pixel segment per
//                   thread), retainBest(2n) on the FAST score (256-bin histogram), Harris responses
//                   (a wavefront per 4 candidates, all their loads in flight), retainBest(n) on
//                   them (radix select of the n-th largest; bin searches by a wave suffix scan),
//                   intensity-centroid angle (a wavefront per 4 keypoints); detection order is
//                   kept (OpenCV's set, canonical order)
//   k_orb_finish    1 WG per scan: levels concatenated, coordinates scaled to level 0,
//                   cloud-track lookup + |x| < 0.01 filter (extractPointsAndFilterZeroValue)
//   k_orb_desc      32 lanes per keypoint: the keypoint's 37 x 37 blurred patch staged in LDS,
//                   steered rBRIEF-256 bytes from it
//   k_orb_xdist_mfma per (pair, 256 trains): Hamming distances on the int8 matrix cores over
//                   0/1-expanded descriptors, batchDistance's cross-check (atomicMin)
//   k_orb_match     1 WG per scan pair: stable counting selection of the first ceil(frac M)
//                   matches, good-frame test, front_end_residual records
//   k_orb_lm        1 WG per scan pair: Ceres-semantics LM (20 iterations) of those records
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include "lislam_batch.hpp"
#include "lislam_ctx.hpp"
#include "lislam_device.hpp"
#include "lislam_lm.hpp"

namespace lislam {
namespace orbk {

constexpr int kB = 23;  // pyramid border: max(edgeThreshold 1, max(22, 4)) + 1
constexpr int kL = 8;   // nlevels
constexpr int kHalf = 15;
constexpr int kFastT = 20;
#ifndef LISLAM_SEL_THREADS
#define LISLAM_SEL_THREADS 512
#endif
constexpr int kSelThreads = LISLAM_SEL_THREADS;  // k_orb_select workgroup
constexpr int kPairThreads = 512;  // k_orb_match: 8 waves, so a workgroup finds room beside the chain engines
constexpr int kLmThreads = 256;
constexpr int kNoMatch = 0x7f7f7f7f;
#ifndef LISLAM_FAST_BAND
#define LISLAM_FAST_BAND 4
#endif
constexpr int kFastBand = LISLAM_FAST_BAND;  // ROI rows per k_orb_fastnms workgroup
constexpr int kBlurBand = 8;   // padded rows per k_orb_blur workgroup
constexpr int kRoiBand = 16;   // ROI rows per k_orb_roiblur workgroup  // best[] sentinel (memset 0x7f): above any (distance << 16 | train)

constexpr int kNPatch = 749;  // pixels of the ICAngles circular patch (half size 15; checked on the host)
constexpr int kPatchIters = (kNPatch + 63) / 64;
__constant__ short2 c_patch[1024];  // (du, dv) of every pixel of the ICAngles patch (host-filled)

// the rBRIEF pattern as bytes biased by 13 (every coordinate is in [-13, 13]): a descriptor byte's 8
// point pairs are 32 consecutive bytes, 8 dwords per lane.  (Unsigned on purpose: a sign-extended
// byte converted to float was compiled as an unsigned conversion.)
constexpr int kPatternInt[256 * 4] = {
#include "lislam_orb_pattern.inc"
};
struct PatternU8 {
  uint8_t v[256 * 4];
};
constexpr PatternU8 pattern_u8() {
  PatternU8 p{};
  for (int i = 0; i < 256 * 4; i++) p.v[i] = (uint8_t)(kPatternInt[i] + 13);
  return p;
}
__constant__ __attribute__((aligned(16))) PatternU8 c_pattern = pattern_u8();

struct Geom {
  int W, H;
  int npatch;            // pixels of the circular intensity-centroid patch (c_patch)
  int w[kL], h[kL], stride[kL];
  int off[kL];      // byte offset of padded level l in a scan's pyramid
  int pix[kL + 1];  // prefix of w*h (flattened level pixels)
  int pad[kL + 1];  // prefix of padded sizes
  int bytes;        // per scan
  float scale[kL];
  int nper[kL];     // nfeaturesPerLevel
  int lcap[kL];     // keypoint capacity per level
  int lofs[kL + 1]; // prefix of lcap
  int cap;          // per scan keypoints (sum lcap)
  float gk[7];      // Gaussian taps
  int umax[kHalf + 2];
  int fband[kL + 1];  // prefix of FAST bands (kFastBand ROI rows) per level
  int bband[kL + 1];  // prefix of blur bands (kBlurBand padded rows) per level
  int rband[kL + 1];  // prefix of ROI blur bands (kRoiBand ROI rows) per level
};

struct Tabs {  // resize coefficients of level l from level l-1 (l >= 1), per axis
  const int* xo; const uint16_t* xc; const int* yo; const uint16_t* yc;
  const int* lim;  // [kL][4] xmin, xmax, ymin, ymax
  int xs, ys;      // row strides of the x / y tables
};

struct Args {
  Geom g;
  Tabs t;
  int S;
  const uint8_t* img;     // [S][H*W]
  const float4* track;    // [S][H*W]
  uint8_t* pyr;           // [S][bytes]
  uint8_t* blur;          // [S][bytes]
  const uint8_t* mpyr;    // [bytes] mask pyramid or null
  uint8_t* nms;           // [S][pix[kL]] FAST score of a keypoint (non-max, mask, border), else 0
  int* cand;              // [S][pix[kL]] candidate pixel indices
  float* cresp;           // [S][pix[kL]]
  float* lkp;             // [S][cap][6] per-level staging (level l at lofs[l])
  int* lcnt;              // [S][kL]
  float* kp;              // [S][cap][6] x, y, size, angle, response, octave
  float4* p3d;            // [S][cap]
  uint8_t* desc;          // [S][cap][32]
  int* nkp;               // [S]
  int* overflow;          // [1]
  const int* smap;        // scan of each grid scan index (null: identity from the slot base)
  const int* scount;      // device count of grid scan indices in use (null: all); the rest exit
};

__device__ __forceinline__ int reflect101(int p, int len) {
  if ((unsigned)p < (unsigned)len) return p;
  if (len == 1) return 0;
  do {
    if (p < 0) p = -p;
    else p = 2 * len - p - 2;
  } while ((unsigned)p >= (unsigned)len);
  return p;
}

// pixel (r, c) of level l (r, c relative to the ROI origin; may reach into the border)
__device__ __forceinline__ uint8_t& px(uint8_t* base, const Geom& g, int l, int r, int c) {
  return base[g.off[l] + (r + kB) * g.stride[l] + (c + kB)];
}
__device__ __forceinline__ uint8_t pxc(const uint8_t* base, const Geom& g, int l, int r, int c) {
  return base[g.off[l] + (r + kB) * g.stride[l] + (c + kB)];
}

// ------------------------------------------------------------------ pyramid
__device__ __forceinline__ uint32_t hval(const uint8_t* base, const Geom& g, const Tabs& t, int l, int row, int x) {
  const int* lim = t.lim + l * 4;
  if (x < lim[0]) return (uint32_t)pxc(base, g, l - 1, row, 0) << 8;
  if (x < lim[1]) {
    const int o = t.xo[l * t.xs + x];
    const uint32_t c1 = t.xc[l * t.xs + x];
    return (256u - c1) * pxc(base, g, l - 1, row, o) + c1 * pxc(base, g, l - 1, row, o + 1);
  }
  return (uint32_t)pxc(base, g, l - 1, row, t.xo[l * t.xs + g.w[l] - 1]) << 8;
}

// Level l of the pyramid (one thread per kLevelPx consecutive padded pixels of a row — rows are
// 16-byte aligned — levels launched in order): a border pixel takes the value of its reflect-101
// image (mode 0) or 0 (mode 1, the mask pyramid); a ROI pixel is level 0's image or the
// INTER_LINEAR_EXACT resize of level l-1 (mask: threshold 254 to 0).
#ifndef LISLAM_LEVEL_PX
#define LISLAM_LEVEL_PX 4
#endif
constexpr int kLevelPx = LISLAM_LEVEL_PX;
__global__ __launch_bounds__(256) void k_orb_level(Args a, int l, int mode) {
  const Geom& g = a.g;
  const int s = a.smap ? a.smap[blockIdx.y] : blockIdx.y;
  const int w = g.w[l], h = g.h[l], pw = g.stride[l];
  const int i0 = (blockIdx.x * blockDim.x + threadIdx.x) * kLevelPx;
  if (i0 >= pw * (h + 2 * kB)) return;
  uint8_t* base = mode ? const_cast<uint8_t*>(a.mpyr) : a.pyr + (size_t)s * g.bytes;
  const int r = i0 / pw - kB, c0 = i0 % pw - kB;
  const bool roi_r = r >= 0 && r < h;
  const int y = reflect101(r, h);
  const uint8_t* img = a.img + (size_t)s * g.W * g.H + (size_t)y * g.W;
  // row terms of the vertical interpolation (levels >= 1)
  int ya = 0, yb = 0;
  uint32_t cy = 0;
  bool yclamp = false;
  if (l > 0) {
    const int* lim = a.t.lim + l * 4;
    yclamp = y < lim[2] || y >= lim[3];
    if (yclamp) {
      ya = y < lim[2] ? 0 : g.h[l - 1] - 1;
    } else {
      ya = a.t.yo[l * a.t.ys + y];
      yb = ya + 1;
      cy = a.t.yc[l * a.t.ys + y];
    }
  }
  uint32_t word[(kLevelPx + 3) / 4] = {};
#pragma unroll
  for (int k = 0; k < kLevelPx; k++) {
    const int c = c0 + k;
    const bool roi = roi_r && c >= 0 && c < w;
    uint32_t v = 0;
    if (roi || !mode) {
      const int x = reflect101(c, w);
      if (l == 0) {
        v = img[x];
      } else {
        if (yclamp) {
          v = min(255u, (hval(base, g, a.t, l, ya, x) + 128u) >> 8);
        } else {
          const uint32_t rr = hval(base, g, a.t, l, ya, x) * (256u - cy) + hval(base, g, a.t, l, yb, x) * cy;
          v = min(255u, (rr + 32768u) >> 16);
        }
        if (mode && v <= 254) v = 0;  // threshold(254, THRESH_TOZERO)
      }
    }
    word[k >> 2] |= v << (8 * (k & 3));
  }
  uint8_t* dst = base + g.off[l] + i0;
  typedef uint32_t u2v __attribute__((ext_vector_type(2)));
  if constexpr (kLevelPx == 8)
    *(__attribute__((address_space(1))) u2v*)dst = u2v{word[0], word[kLevelPx / 8]};
  else if constexpr (kLevelPx == 4)
    *(__attribute__((address_space(1))) uint32_t*)dst = word[0];
  else if constexpr (kLevelPx == 2)
    *(__attribute__((address_space(1))) uint16_t*)dst = (uint16_t)word[0];
  else
    *(__attribute__((address_space(1))) uint8_t*)dst = (uint8_t)word[0];
}

// The pyramid of a scan in one workgroup (80 KiB of LDS: level 0 in 64, then two buffers of 48 and
// 32): level l-1's ROI stays in LDS while level l is resized from it (level 1, which overwrites
// level 0, through its ROI rows in HBM); each level's ROI rows go to HBM from LDS with dword
// stores (a dword never spans rows: strides are 16-byte multiples).  Same pixels as k_orb_level:
// ROI pixels are level 0's image or the INTER_LINEAR_EXACT fixed-point resize (hval) of level l-1,
// border columns their reflect-101 ROI pixel.  A thread owns a column of the level (its horizontal
// taps in registers) and walks the rows four at a time; the row taps (levels >= 1 have <= 64 rows)
// sit one per lane and are read with readlane.  The border rows and the blurred copy are written
// by k_orb_fastnms' bands, which stage the rows they need anyway.
#ifdef LISLAM_PHASE_PROF
// k_orb_pyramid phase split (profiling builds): slot 0 the image load, 8 p + l phase p (1 resize,
// 2 padded copy, 3 blur) of level l, summed over workgroups in s_memrealtime ticks (100 MHz)
__device__ unsigned long long g_pyr_phase[32];
extern "C" int lislam_debug_pyr_phases(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pyr_phase), sizeof(g_pyr_phase)) != hipSuccess) return -2;
  static const unsigned long long zero[32] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_pyr_phase), zero, sizeof(zero)) == hipSuccess ? 0 : -2;
}
#define PYR_PHASE(i)                                                          \
  do {                                                                        \
    __syncthreads();                                                          \
    if (threadIdx.x == 0) {                                                   \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();      \
      atomicAdd(&g_pyr_phase[i], now_ - t_ph);                                \
      t_ph = now_;                                                            \
    }                                                                         \
  } while (0)
#else
#define PYR_PHASE(i)
#endif
constexpr int kPyrThreads = 1024;
// LDS: level 0 in [0, 64 KiB); levels >= 1 ping-pong between [0, 48 KiB) (odd levels) and
// [48 KiB, 80 KiB) (even levels).  <= 80 KiB per workgroup runs beside the chain engine's items.
constexpr int kPyrLds0 = 64 * 1024, kPyrOdd = 48 * 1024, kPyrEven = 32 * 1024;
constexpr int kPyrLds = kPyrOdd + kPyrEven;
__host__ __device__ __forceinline__ int pyr_split(const Geom& g) { return (g.w[0] * g.h[0] + 15) & ~15; }
__global__ __launch_bounds__(kPyrThreads) void k_orb_pyramid(Args a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kPyrLds];
#ifdef LISLAM_PHASE_PROF
  unsigned long long t_ph = __builtin_amdgcn_s_memrealtime();
#endif
  const Geom& g = a.g;
  const int s = a.smap ? a.smap[blockIdx.x] : blockIdx.x;
  const int lane = threadIdx.x & 63;
  uint8_t* const base = a.pyr + (size_t)s * g.bytes;
  {
    const uint32_t* img = reinterpret_cast<const uint32_t*>(a.img + (size_t)s * g.W * g.H);
    uint32_t* e32 = reinterpret_cast<uint32_t*>(lds);
    const int nd = g.W * g.H / 4;
    for (int d = threadIdx.x; d < nd; d += kPyrThreads) e32[d] = __builtin_nontemporal_load(img + d);
  }
  __syncthreads();
  PYR_PHASE(0);
  for (int l = 0; l < kL; l++) {
    const int w = g.w[l], h = g.h[l];
    uint8_t* const cur = (l & 1) || l == 0 ? lds : lds + kPyrOdd;
    if (l > 0) {
      const uint8_t* const prev = l == 1 || !(l & 1) ? lds : lds + kPyrOdd;
      const int wp = g.w[l - 1], hl = g.h[l - 1] - 1;
      const int* lim = a.t.lim + l * 4;
      const int lx0 = lim[0], lx1 = lim[1], ly0 = lim[2], ly1 = lim[3];
      // row taps of this level, lane y: byte offsets of source rows ya, yb and the weight cy; a
      // row outside [ly0, ly1) clamps to row 0 / hl with cy = 0, where the two-row formula is the
      // one-row one: (256 ha + 32768) >> 16 = (ha + 128) >> 8
      int ra_l = 0, rb_l = 0, cy_l = 0;
      if (lane < h) {
        if (lane >= ly0 && lane < ly1) {
          const int ya = a.t.yo[l * a.t.ys + lane];
          ra_l = ya * wp;
          rb_l = ra_l + wp;
          cy_l = (int)a.t.yc[l * a.t.ys + lane];
        } else {
          ra_l = rb_l = (lane < ly0 ? 0 : hl) * wp;
        }
      }
      const int xlast = a.t.xo[l * a.t.xs + w - 1];
      // level 1 overwrites level 0's LDS, so it goes to its ROI rows in HBM first and comes back
      // after the barrier; later levels are written to the other LDS buffer directly
      uint8_t* const roi1 = base + g.off[1] + kB * g.stride[1] + kB;
      for (int x = threadIdx.x; x < w; x += kPyrThreads) {
        int o0 = 0, o1 = 0;
        uint32_t w0 = 256u, w1 = 0u;  // hval = w0 * pr[o0] + w1 * pr[o1]
        if (x >= lx0 && x < lx1) {
          o0 = a.t.xo[l * a.t.xs + x];
          o1 = o0 + 1;
          w1 = a.t.xc[l * a.t.xs + x];
          w0 = 256u - w1;
        } else if (x >= lx1) {
          o0 = o1 = xlast;
        }
        // four rows per step, their eight source bytes' loads in flight together
        for (int y0 = 0; y0 < h; y0 += 4) {
          uint32_t v[4];
#pragma unroll
          for (int u = 0; u < 4; u++) {
            const int y = min(y0 + u, h - 1);
            const uint8_t* pa = prev + __builtin_amdgcn_readlane(ra_l, y);
            const uint8_t* pb = prev + __builtin_amdgcn_readlane(rb_l, y);
            const uint32_t cy = (uint32_t)__builtin_amdgcn_readlane(cy_l, y);
            const uint32_t ha = w0 * pa[o0] + w1 * pa[o1], hb = w0 * pb[o0] + w1 * pb[o1];
            v[u] = min(255u, (ha * (256u - cy) + hb * cy + 32768u) >> 16);
          }
#pragma unroll
          for (int u = 0; u < 4; u++) {
            if (y0 + u >= h) break;
            if (l == 1)
              roi1[(size_t)(y0 + u) * g.stride[1] + x] = (uint8_t)v[u];
            else
              cur[(y0 + u) * w + x] = (uint8_t)v[u];
          }
        }
      }
      if (l == 1) {
        __threadfence_block();
        __syncthreads();  // level 0 is read and level 1 is in HBM: bring it into LDS
        for (int i = threadIdx.x; i < w * h; i += kPyrThreads) {
          const int y = i / w, x = i - y * w;
          cur[i] = roi1[(size_t)y * g.stride[1] + x];
        }
      }
      __syncthreads();  // level l complete; the next level writes the buffer read above
      PYR_PHASE(8 + l);
    }
    // the ROI rows of the padded level (border columns included): ndr dword columns x P row
    // phases (P = threads / ndr), a thread's column and its reflections fixed per level.  A dword
    // of 4 ROI columns is the two aligned LDS dwords around it shifted (alignbyte); a border dword
    // gathers its 4 reflected bytes.  The border rows and the blurred copy are k_orb_fastnms' (its
    // bands stage these rows anyway).
    const int ndr = g.stride[l] / 4;
    uint32_t* dst = reinterpret_cast<uint32_t*>(base + g.off[l]);
    {
      const int P = kPyrThreads / ndr, dc = (int)threadIdx.x % ndr, ph = (int)threadIdx.x / ndr;
      if (ph < P) {
        int cx[4];
#pragma unroll
        for (int k = 0; k < 4; k++) cx[k] = reflect101(4 * dc + k - kB, w);
        const bool inner = 4 * dc - kB >= 0 && 4 * dc + 3 - kB < w;
        for (int r = ph; r < h; r += P) {
          uint32_t v;
          if (inner) {
            const int A = r * w + 4 * dc - kB;
            const uint32_t* d = reinterpret_cast<const uint32_t*>(cur + (A & ~3));
            v = __builtin_amdgcn_alignbyte(d[1], d[0], (uint32_t)(A & 3));
          } else {
            const uint8_t* src = cur + r * w;
            v = (uint32_t)src[cx[0]] | (uint32_t)src[cx[1]] << 8 | (uint32_t)src[cx[2]] << 16 | (uint32_t)src[cx[3]] << 24;
          }
          dst[(r + kB) * ndr + dc] = v;
        }
      }
    }
    PYR_PHASE(16 + l);
  }
}

// Stage `rows` (<= kMaxRows) rows of nd dwords (source rows 4-byte aligned, sstride bytes apart)
// into LDS rows of nd dwords: every load of a thread is issued before its first store.
template <int kMaxRows>
__device__ __forceinline__ void stage_rows(uint32_t* dst, const uint8_t* src, int sstride, int rows, int nd) {
  for (int j0 = 0; j0 < nd; j0 += 3 * 256) {
    uint32_t v[kMaxRows][3];
#pragma unroll
    for (int r = 0; r < kMaxRows; r++)
#pragma unroll
      for (int u = 0; u < 3; u++) {
        const int d = j0 + u * 256 + (int)threadIdx.x;
        if (r < rows && d < nd)
          v[r][u] = *(const __attribute__((address_space(1))) uint32_t*)(src + (size_t)r * sstride + 4 * d);
      }
#pragma unroll
    for (int r = 0; r < kMaxRows; r++)
#pragma unroll
      for (int u = 0; u < 3; u++) {
        const int d = j0 + u * 256 + (int)threadIdx.x;
        if (r < rows && d < nd) dst[r * nd + d] = v[r][u];
      }
  }
}

// GaussianBlur(level ROI, 7x7, 2, 2, BORDER_REFLECT_101): row sums then symmetric column sum.
// One workgroup per band of kBlurBand padded rows of a level: the band's rows +-3 staged in LDS
// (row-coalesced dword loads), then one thread per 4 columns keeps the band's row sums in
// registers (3 LDS dwords per staged row); border rows / columns are copies.
__global__ __launch_bounds__(256) void k_orb_blur(Args a) {
  extern __shared__ uint8_t btile[];  // (kBlurBand + 6) x stride[l]
  const Geom& g = a.g;
  const int s = a.smap ? a.smap[blockIdx.y] : blockIdx.y;
  int l = 0;
  while ((int)blockIdx.x >= g.bband[l + 1]) l++;
  const int w = g.w[l], h = g.h[l], pw = g.stride[l];
  const int p0 = ((int)blockIdx.x - g.bband[l]) * kBlurBand;  // first padded row of the band
  const int nr = min(kBlurBand, h + 2 * kB - p0);
  const uint8_t* src = a.pyr + (size_t)s * g.bytes + g.off[l];
  uint8_t* dst = a.blur + (size_t)s * g.bytes + g.off[l];
  // staged rows: padded rows p0 - 3 .. p0 + nr + 2, clamped to the level's buffer
  const int t0 = max(0, p0 - 3), t1 = min(h + 2 * kB, p0 + nr + 3);
  stage_rows<kBlurBand + 6>(reinterpret_cast<uint32_t*>(btile + (t0 - (p0 - 3)) * pw), src + (size_t)t0 * pw, pw,
                            t1 - t0, pw >> 2);
  __syncthreads();
  // one thread per 4 columns: each staged row's 10 source bytes come from 3 LDS dwords
  const uint32_t* t32 = reinterpret_cast<const uint32_t*>(btile);
  const int pw4 = pw >> 2;
  for (int c4 = 4 * (int)threadIdx.x; c4 < pw; c4 += 4 * (int)blockDim.x) {
    bool roi_c[4];
    bool any_roi = false;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int cr = c4 + j - kB;  // ROI column
      roi_c[j] = cr >= 0 && cr < w;
      any_roi |= roi_c[j];
    }
    float rs[kBlurBand + 6][4];
    if (any_roi) {  // then c4 >= kB - 3, so the dword at c4 - 4 is inside the row
#pragma unroll
      for (int k = 0; k < kBlurBand + 6; k++) {
        const int pr = p0 - 3 + k;
#pragma unroll
        for (int j = 0; j < 4; j++) rs[k][j] = 0.f;
        if (pr >= kB - 3 && pr < h + kB + 3 && k < nr + 6) {  // rows some ROI output of the band reads
          const uint32_t* rw = t32 + k * pw4 + (c4 >> 2) - 1;
          const uint32_t d0 = rw[0], d1 = rw[1], d2 = rw[2];
          float b[12];
#pragma unroll
          for (int e = 0; e < 4; e++) {
            b[e] = (float)((d0 >> (8 * e)) & 255u);
            b[4 + e] = (float)((d1 >> (8 * e)) & 255u);
            b[8 + e] = (float)((d2 >> (8 * e)) & 255u);
          }
#pragma unroll
          for (int j = 0; j < 4; j++) {  // column c4 + j: bytes c4 + j - 3 .. c4 + j + 3 = b[j + 1 .. j + 7]
            float v = g.gk[0] * b[j + 1];
#pragma unroll
            for (int t = 1; t < 7; t++) v += g.gk[t] * b[j + 1 + t];
            rs[k][j] = v;
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kBlurBand; k++) {
      if (k >= nr) break;
      const int pr = p0 + k, r = pr - kB;
      uint32_t o = t32[(k + 3) * pw4 + (c4 >> 2)];
      if (r >= 0 && r < h) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if (!roi_c[j]) continue;
          float v = g.gk[3] * rs[k + 3][j];
#pragma unroll
          for (int t = 1; t <= 3; t++) v += g.gk[3 + t] * (rs[k + 3 + t][j] + rs[k + 3 - t][j]);
          const uint32_t ob = (uint32_t)min(255, max(0, (int)rintf(v)));
          o = (o & ~(255u << (8 * j))) | (ob << (8 * j));
        }
      }
      *(__attribute__((address_space(1))) uint32_t*)(dst + (size_t)pr * pw + c4) = o;
    }
  }
}

// ------------------------------------------------------------------ FAST
__constant__ int c_fast[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                                  {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

__device__ int corner_score(const int* d, int threshold) {
  int a0 = threshold;
  for (int k = 0; k < 16; k += 2) {
    int a = min(d[k + 1], d[k + 2]);
    a = min(a, d[k + 3]);
    if (a <= a0) continue;
    a = min(a, d[k + 4]);
    a = min(a, d[k + 5]);
    a = min(a, d[k + 6]);
    a = min(a, d[k + 7]);
    a = min(a, d[k + 8]);
    a0 = max(a0, min(a, d[k]));
    a0 = max(a0, min(a, d[k + 9]));
  }
  int b0 = -a0;
  for (int k = 0; k < 16; k += 2) {
    int b = max(d[k + 1], d[k + 2]);
    b = max(b, d[k + 3]);
    b = max(b, d[k + 4]);
    b = max(b, d[k + 5]);
    if (b >= b0) continue;
    b = max(b, d[k + 6]);
    b = max(b, d[k + 7]);
    b = max(b, d[k + 8]);
    b0 = min(b0, max(b, d[k]));
    b0 = min(b0, max(b, d[k + 9]));
  }
  return -b0 - 1;
}

// Is there a run of 9 set bits in the circular 16-bit mask m (FAST's "count > 8" over the
// 25-step doubled walk)?
__device__ __forceinline__ bool has_run9(uint32_t m) {
  m |= m << 16;
  uint32_t r = m & (m >> 1);  // runs of 2 starting at each bit
  r &= r >> 2;                // 4
  r &= r >> 4;                // 8
  r &= m >> 8;                // 9
  return (r & 0xffffu) != 0;
}

// FAST-9/16 segment test + cornerScore<16> of the pixel at p (an LDS tile with row stride ts).
// The opposite-pair pre-tests of OpenCV only reject pixels that have no 9-run either, so the
// test is the run check of both masks.
__device__ __forceinline__ int fast_full(const uint8_t* p, int ts) {
  const int v = p[0];
  int x[16];
#pragma unroll
  for (int k = 0; k < 16; k++) x[k] = p[c_fast[k][1] * ts + c_fast[k][0]];
  uint32_t dark = 0, bright = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    dark |= (uint32_t)(x[k] < v - kFastT) << k;
    bright |= (uint32_t)(x[k] > v + kFastT) << k;
  }
  if (!has_run9(dark) && !has_run9(bright)) return 0;
  int dd[25];
#pragma unroll
  for (int k = 0; k < 25; k++) dd[k] = v - x[k & 15];
  return corner_score(dd, kFastT);
}

// LDS of a k_orb_fastnms workgroup for a level of padded row stride ps and width w: the image tile
// ((kFastBand + 8) padded rows), the score tile ((kFastBand + 2) rows of w + 2 bytes,
// dword-padded) and the candidate list (u16 score-tile positions: (kFastBand + 2) (w + 2) <= 65536,
// host-checked)
__host__ __device__ __forceinline__ int fast_score_bytes(int w) { return ((kFastBand + 2) * (w + 2) + 3) & ~3; }
__host__ __device__ __forceinline__ size_t fast_lds_bytes(int ps, int w) {
  return (size_t)(kFastBand + 8) * ps + fast_score_bytes(w) + (size_t)2 * (kFastBand + 2) * (w + 2);
}

// Stage tile rows t = 0 .. rows-1 = level rows r0 - halo + t, reflect-101 (so only the ROI rows of
// the padded level are read), whole padded rows of nd dwords; every load before the first store.
template <int kMaxRows>
__device__ __forceinline__ void stage_rows_reflect(uint32_t* dst, const uint8_t* lvl, int ps, int r0, int halo, int h,
                                                   int rows, int nd) {
  for (int j0 = 0; j0 < nd; j0 += 2 * 256) {
    uint32_t v[kMaxRows][2];
#pragma unroll
    for (int r = 0; r < kMaxRows; r++) {
      const uint8_t* src = lvl + (size_t)(reflect101(r0 - halo + r, h) + kB) * ps;
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const int d = j0 + u * 256 + (int)threadIdx.x;
        if (r < rows && d < nd) v[r][u] = *(const __attribute__((address_space(1))) uint32_t*)(src + 4 * d);
      }
    }
#pragma unroll
    for (int r = 0; r < kMaxRows; r++)
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const int d = j0 + u * 256 + (int)threadIdx.x;
        if (r < rows && d < nd) dst[r * nd + d] = v[r][u];
      }
  }
}

// FAST keypoints of a band of kFastBand ROI rows of a level: the band's rows +-4 staged in LDS
// (whole padded rows), FAST scores of the band +-1 (border pixels 0) into a second LDS tile, then
// 3x3 non-max suppression of FAST_t, the pixel mask (runByPixelsMask) and the image border
// (edgeThreshold 1): nms = the FAST score of a keypoint, else 0.  The scores take two passes over
// the whole band, one barrier apart: every pixel takes the cheap necessary test (an opposite pair
// on each axis has a pixel beyond the threshold on the same side) and the survivors are compacted
// into one LDS list (wave ballot + one LDS atomic per wave), then the full segment test and
// cornerScore run on the list with every lane busy.  The list's order is the atomics' order; each
// entry writes only its own score, so the result does not depend on it.
__global__ __launch_bounds__(256) void k_orb_fastnms(Args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t ftile[];
  __shared__ int lcnt;
  const Geom& g = a.g;
  const int s = a.smap ? a.smap[blockIdx.y] : blockIdx.y;
  int l = 0;
  while ((int)blockIdx.x >= g.fband[l + 1]) l++;
  const int w = g.w[l], h = g.h[l];
  const int r0 = ((int)blockIdx.x - g.fband[l]) * kFastBand;
  const int nr = min(kFastBand, h - r0);
  // image tile: rows r0-4 .. r0+nr+3, whole padded rows (tile column = padded column)
  const int ts = g.stride[l], nd = ts >> 2;
  constexpr int kC0 = kB;  // tile column of level column 0
  uint8_t* img = ftile;
  uint8_t* sct = ftile + (kFastBand + 8) * ts;  // scores: rows r0-1 .., columns -1 .. w
  const int ss = w + 2;
  uint16_t* list = reinterpret_cast<uint16_t*>(sct + fast_score_bytes(w));
  uint8_t* const lvl = a.pyr + (size_t)s * g.bytes + g.off[l];
  stage_rows_reflect<kFastBand + 8>(reinterpret_cast<uint32_t*>(img), lvl, ts, r0, 4, h, nr + 8, nd);
  {
    uint32_t* z = reinterpret_cast<uint32_t*>(sct);
    for (int i = threadIdx.x; i < fast_score_bytes(w) / 4; i += blockDim.x) z[i] = 0u;
  }
  if (threadIdx.x == 0) lcnt = 0;
  __syncthreads();
  // 1. cheap test of the score rows r0-1 .. r0+nr inside the FAST area (3 <= r < h-3, 3 <= c < w-3)
  const int lane = threadIdx.x & 63;
  const int rlo = max(0, 4 - r0), rhi = min(nr + 2, h - 2 - r0);
  for (int rr = rlo; rr < rhi; rr++) {
    const uint8_t* prow = img + (rr + 3) * ts + kC0;
    for (int c0 = 3; c0 < w - 3; c0 += blockDim.x) {
      const int c = c0 + (int)threadIdx.x;
      bool cand = false;
      if (c < w - 3) {
        const uint8_t* p = prow + c;
        const int v = p[0];
        auto tab = [&](int x) { const int dd = x - v; return dd < -kFastT ? 1 : dd > kFastT ? 2 : 0; };
        cand = ((tab(p[3 * ts]) | tab(p[-3 * ts])) & (tab(p[3]) | tab(p[-3]))) != 0;
      }
      const uint64_t m = __ballot(cand);
      if (m) {
        int at = 0;
        if (lane == 0) at = atomicAdd(&lcnt, __popcll(m));
        at = __shfl(at, 0);
        if (cand) list[at + __popcll(m & lanemask_lt())] = (uint16_t)(rr * ss + c + 1);
      }
    }
  }
  __syncthreads();
  // 2. full test + score of the candidates (row = position / ss: exact in float, the quotient's
  //    fractional part is >= 0.5 / ss away from an integer and the product errs by < 2^-8 / ss)
  const int n = lcnt;
  const float iss = 1.f / (float)ss;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int idx = list[i];
    const int rr = (int)(((float)idx + 0.5f) * iss);
    const int c = idx - rr * ss - 1;
    sct[idx] = (uint8_t)fast_full(img + (rr + 3) * ts + c + kC0, ts);
  }
  __syncthreads();
  uint8_t* out = a.nms + (size_t)s * g.pix[kL] + g.pix[l];
  for (int rr = 0; rr < nr; rr++) {
    const int r = r0 + rr;
    for (int c = threadIdx.x; c < w; c += blockDim.x) {
      const uint8_t* q = sct + (rr + 1) * ss + (c + 1);
      const int v = q[0];
      bool keep = false;
      if (v && r >= 3 && r < h - 3) {
        keep = v > q[1] && v > q[-1] && v > q[-ss - 1] && v > q[-ss] && v > q[-ss + 1] && v > q[ss - 1] &&
               v > q[ss] && v > q[ss + 1];
        if (keep && a.mpyr && pxc(a.mpyr, g, l, r, c) == 0) keep = false;
        if (keep && !(c >= 1 && c < w - 1 && r >= 1 && r < h - 1)) keep = false;
      }
      out[r * w + c] = keep ? (uint8_t)v : 0;
    }
  }
}

// After k_orb_pyramid (which writes only the ROI rows): one workgroup per band of kRoiBand ROI
// rows of a level writes the band's rows of the blurred copy — GaussianBlur(7x7, sigma 2,
// BORDER_REFLECT_101) of the ROI from the band's rows +-3 staged in LDS (reflect-101 ROI rows, whole
// padded rows), per dword column a sliding window of 7 row sums in float pairs (columns j, j + 1:
// the packed multiplies and adds round like the scalar ones, in the same order: row taps 0..6,
// then the symmetric column sum), bytes outside the ROI copied — and the first / last band the
// level's border rows (reflect-101 copies of ROI rows) of both padded pyramids.
__global__ __launch_bounds__(256) void k_orb_roiblur(Args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t rtile[];  // (kRoiBand + 6) padded rows
  const Geom& g = a.g;
  const int s = a.smap ? a.smap[blockIdx.y] : blockIdx.y;
  int l = 0;
  while ((int)blockIdx.x >= g.rband[l + 1]) l++;
  const int w = g.w[l], h = g.h[l];
  const int r0 = ((int)blockIdx.x - g.rband[l]) * kRoiBand;
  const int nr = min(kRoiBand, h - r0);
  const int nd = g.stride[l] >> 2;
  uint8_t* const lvl = a.pyr + (size_t)s * g.bytes + g.off[l];
  stage_rows_reflect<kRoiBand + 6>(reinterpret_cast<uint32_t*>(rtile), lvl, g.stride[l], r0, 3, h, nr + 6, nd);
  __syncthreads();
  uint32_t* const bl = a.blur ? reinterpret_cast<uint32_t*>(a.blur + (size_t)s * g.bytes + g.off[l]) : nullptr;
  const uint32_t* const t32 = reinterpret_cast<const uint32_t*>(rtile);
  typedef float f2 __attribute__((ext_vector_type(2)));
  for (int dc = threadIdx.x; bl && dc < nd; dc += blockDim.x) {
    const bool roi_dw = 4 * dc + 3 >= kB && 4 * dc < kB + w;
    if (!roi_dw) {
      for (int k = 0; k < nr; k++) bl[(r0 + k + kB) * nd + dc] = t32[(k + 3) * nd + dc];
      continue;
    }
    auto rowsum = [&](int t, f2* out2) {  // tile row t, padded columns 4 dc - 3 .. 4 dc + 6
      const uint32_t d0 = t32[t * nd + dc - 1], d1 = t32[t * nd + dc], d2 = t32[t * nd + dc + 1];
      float b[10];
      b[0] = (float)((d0 >> 8) & 255u);
      b[1] = (float)((d0 >> 16) & 255u);
      b[2] = (float)(d0 >> 24);
#pragma unroll
      for (int e = 0; e < 4; e++) b[3 + e] = (float)((d1 >> (8 * e)) & 255u);
#pragma unroll
      for (int e = 0; e < 3; e++) b[7 + e] = (float)((d2 >> (8 * e)) & 255u);
#pragma unroll
      for (int jp = 0; jp < 2; jp++) {
        f2 v = g.gk[0] * f2{b[2 * jp], b[2 * jp + 1]};
#pragma unroll
        for (int t2 = 1; t2 < 7; t2++) v += g.gk[t2] * f2{b[2 * jp + t2], b[2 * jp + 1 + t2]};
        out2[jp] = v;
      }
    };
    f2 rs[7][2];
#pragma unroll
    for (int k = 0; k < 6; k++) rowsum(k, rs[k + 1]);
    for (int k = 0; k < nr; k++) {  // ROI row r0 + k = tile row k + 3, from tile rows k .. k + 6
#pragma unroll
      for (int q = 0; q < 6; q++)
#pragma unroll
        for (int jp = 0; jp < 2; jp++) rs[q][jp] = rs[q + 1][jp];
      rowsum(k + 6, rs[6]);
      float cv[4];
#pragma unroll
      for (int jp = 0; jp < 2; jp++) {
        f2 v = g.gk[3] * rs[3][jp];
#pragma unroll
        for (int t2 = 1; t2 <= 3; t2++) v += g.gk[3 + t2] * (rs[3 + t2][jp] + rs[3 - t2][jp]);
        cv[2 * jp] = v.x;
        cv[2 * jp + 1] = v.y;
      }
      const uint32_t raw = t32[(k + 3) * nd + dc];
      uint32_t o = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int cr = 4 * dc + j - kB;
        const uint32_t ob = (cr >= 0 && cr < w) ? (uint32_t)min(255, max(0, (int)rintf(cv[j]))) : (raw >> (8 * j)) & 255u;
        o |= ob << (8 * j);
      }
      bl[(r0 + k + kB) * nd + dc] = o;
    }
  }
  // border rows (first / last band): padded row rr = ROI row reflect101(rr - kB), both copies
  const bool top = r0 == 0, bottom = r0 + nr == h;
  if (top || bottom) {
    uint32_t* const py = reinterpret_cast<uint32_t*>(lvl);
    for (int half = 0; half < 2; half++) {
      if (!(half ? bottom : top)) continue;
      for (int it = threadIdx.x; it < kB * nd; it += blockDim.x) {
        const int q = it / nd, dc = it - q * nd;
        const int rr = half ? kB + h + q : q;
        const uint32_t v = py[(reflect101(rr - kB, h) + kB) * nd + dc];
        py[rr * nd + dc] = v;
        if (bl) bl[rr * nd + dc] = v;
      }
    }
  }
}

// ------------------------------------------------------------------ selection (1 WG per scan, level)
// The counter hand-off of several workgroups to the last of them (in-launch fold of a dependent
// launch): every wave drains its stores, lane 0 releases them at agent scope once per workgroup
// (buffer_wbl2: the other XCDs' L2s) and adds to the counter; the workgroup whose add returns
// total - 1 resets the counter for the next launch, acquires once (this CU's L1) and reads the
// others' bytes with plain loads after the barrier.  Returns that verdict, uniform over the
// workgroup.  (A __threadfence() per thread instead costs every wave a write-back and an
// invalidate: the folds measured 2-3x slower than the launches they replaced.)
__device__ __forceinline__ bool wg_arrive_last(int* cnt, int total, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const bool last = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1;
    if (last) {
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag;
}

struct SelShared {
  int wsum[kSelThreads / 64];
  int hist[256];
  int total;
  uint32_t prefix;  // radix-select prefix
  int want;
};

// Ordered compaction helper: block-wide exclusive prefix of flag; returns the rank, *tot the sum.
__device__ __forceinline__ int block_rank(SelShared& sh, bool flag, int* tot) {
  const uint64_t b = __ballot(flag);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int inwave = __popcll(b & lanemask_lt());
  if (lane == 0) sh.wsum[w] = __popcll(b);
  __syncthreads();
  int before = 0, all = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); k++) {
    const int v = sh.wsum[k];
    if (k < w) before += v;
    all += v;
  }
  __syncthreads();
  *tot = all;
  return before + inwave;
}

__device__ __forceinline__ uint32_t ord_key(float f) {  // larger float -> larger key
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// cv::fastAtan2 (degrees)
__device__ float fast_atan2(float y, float x) {
  const float k = (float)(180 / kPi);
  const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k, p5 = 0.1555786518463281f * k,
              p7 = -0.04432655554792128f * k;
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + (float)2.220446049250313e-16);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + (float)2.220446049250313e-16);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// Wave 0 of the block: the largest bin b of the 256-bin histogram whose suffix sum
// S(b) = sum_{b' >= b} hist[b'] reaches want (the first bin of a walk from 255 down where the
// running count reaches it), and rem = want - S(b + 1); b = -1 if the total is below want.
// Lane l holds bins 4l .. 4l + 3; suffix sums by a wave scan.
__device__ __forceinline__ void top_bin(const int* hist, int want, int* b_out, int* rem_out) {
  const int lane = threadIdx.x & 63;
  int h[4];
#pragma unroll
  for (int u = 0; u < 4; u++) h[u] = hist[4 * lane + u];
  const int tl = h[0] + h[1] + h[2] + h[3];
  int suf = tl;  // sum over lanes >= this lane
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_down(suf, o, 64);
    if (lane + o < 64) suf += t;
  }
  int above = suf - tl;  // S(4 lane + 4)
  int found = -1, rem = 0;
#pragma unroll
  for (int u = 3; u >= 0; u--) {
    const int sb = above + h[u];
    if (found < 0 && sb >= want) { found = 4 * lane + u; rem = want - above; }
    above = sb;
  }
  const uint64_t m = __ballot(found >= 0);
  if (!m) { *b_out = -1; *rem_out = want; return; }
  const int L = 63 - __builtin_clzll(m);
  *b_out = __shfl(found, L, 64);
  *rem_out = __shfl(rem, L, 64);
}

// n-th largest key among cnt keys (radix select, 4 x 8 bits); all threads get it
__device__ uint32_t nth_largest(SelShared& sh, const float* resp, int cnt, int n) {
  uint32_t prefix = 0;
  int want = n;
  for (int pass = 3; pass >= 0; pass--) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) sh.hist[b] = 0;
    __syncthreads();
    const uint32_t hmask = pass == 3 ? 0u : (0xffffffffu << ((pass + 1) * 8));
    for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
      const uint32_t k = ord_key(resp[i]);
      if ((k & hmask) == prefix) atomicAdd(&sh.hist[(k >> (pass * 8)) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      int b, rem;
      top_bin(sh.hist, want, &b, &rem);
      if (threadIdx.x == 0) {
        sh.prefix = prefix | ((uint32_t)max(b, 0) << (pass * 8));
        sh.want = rem;
      }
    }
    __syncthreads();
    prefix = sh.prefix;
    want = sh.want;
  }
  return prefix;
}

// every lane of each 16-lane row gets the row's sum (DPP: pairs, quads, half rows, rows)
__device__ __forceinline__ int row_sum16(int v) {
  v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, false);  // row_half_mirror
  v += __builtin_amdgcn_mov_dpp(v, 0x140, 0xf, 0xf, false);  // row_mirror
  return v;
}
// the wave's sum (uniform): row sums + the four rows read as scalars
__device__ __forceinline__ int wave_sum(int v) {
  v = row_sum16(v);
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}

// block-wide exclusive prefix of an int per thread; *tot = the sum
__device__ __forceinline__ int block_excl(SelShared& sh, int v, int* tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) sh.wsum[w] = incl;
  __syncthreads();
  int before = 0, all = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); k++) {
    const int x = sh.wsum[k];
    if (k < w) before += x;
    all += x;
  }
  __syncthreads();
  *tot = all;
  return before + incl - v;
}

#ifdef LISLAM_PHASE_PROF
__device__ unsigned long long g_sel_phase[8];
extern "C" int lislam_debug_sel_phases(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sel_phase), sizeof(g_sel_phase)) != hipSuccess) return -2;
  static const unsigned long long zero[8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_sel_phase), zero, sizeof(zero)) == hipSuccess ? 0 : -2;
}
#define SEL_PHASE(i)                                                          \
  do {                                                                        \
    __syncthreads();                                                          \
    if (threadIdx.x == 0) {                                                   \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();      \
      atomicAdd(&g_sel_phase[i], now_ - t_ph);                                \
      t_ph = now_;                                                            \
    }                                                                         \
  } while (0)
#else
#define SEL_PHASE(i)
#endif
constexpr int kPatchDw = 2 * 279;  // LDS dwords per wave: 2 angle patches (31 x 9) >= 4 Harris patches (9 x 4)
__device__ __forceinline__ void orb_select_body(const Args& a, int gi, int l) {
  __shared__ SelShared sh;
  __shared__ uint32_t sh_patch[(kSelThreads / 64) * kPatchDw];
#ifdef LISLAM_PHASE_PROF
  unsigned long long t_ph = __builtin_amdgcn_s_memrealtime();
#endif
  const Geom& g = a.g;
  const int s = a.smap ? a.smap[gi] : gi;
  const int w = g.w[l], h = g.h[l];
  const uint8_t* base = a.pyr + (size_t)s * g.bytes;
  const uint8_t* kf = a.nms + (size_t)s * g.pix[kL] + g.pix[l];
  const uint8_t* sc = kf;  // a keypoint's nms value is its FAST score
  int* cand = a.cand + (size_t)s * g.pix[kL] + g.pix[l];
  float* resp = a.cresp + (size_t)s * g.pix[kL] + g.pix[l];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // 1. FAST keypoints in row-major order: each thread compacts one contiguous pixel segment,
  //    read as the aligned dwords that cover it (bit 7 of each byte of nz = a nonzero score)
  const int npx = w * h, seg = (npx + blockDim.x - 1) / blockDim.x;
  const int p0 = min(npx, (int)threadIdx.x * seg), p1 = min(npx, p0 + seg);
  const uintptr_t b0 = (uintptr_t)kf + p0, b1 = (uintptr_t)kf + p1;
  auto nz_of = [&](uintptr_t a) {
    const uint32_t v = *(const __attribute__((address_space(1))) uint32_t*)(a);
    uint32_t nz = (((v & 0x7f7f7f7fu) + 0x7f7f7f7fu) | v) & 0x80808080u;
    if (b0 > a) nz &= 0xffffffffu << (8 * (int)(b0 - a));        // bytes before the segment
    if (b1 - a < 4) nz &= 0xffffffffu >> (8 * (4 - (int)(b1 - a)));  // bytes after it
    return nz;
  };
  int mine = 0;
  for (uintptr_t a = b0 & ~(uintptr_t)3; a < b1; a += 4) mine += __popc(nz_of(a));
  int n;
  int at = block_excl(sh, mine, &n);
  for (uintptr_t a = b0 & ~(uintptr_t)3; a < b1; a += 4) {
    uint32_t nz = nz_of(a);
    while (nz) {
      cand[at++] = (int)((intptr_t)a - (intptr_t)kf) + (__builtin_ctz(nz) >> 3);
      nz &= nz - 1;
    }
  }
  __syncthreads();
  SEL_PHASE(0);
  // 2. retainBest(2 n_l) on the FAST score: keep every score >= the (2 n_l)-th largest
  const int n2 = 2 * g.nper[l];
  if (n > n2) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) sh.hist[b] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&sh.hist[sc[cand[i]]], 1);
    __syncthreads();
    if (threadIdx.x < 64) {
      int b, rem;
      top_bin(sh.hist, n2, &b, &rem);
      if (threadIdx.x == 0) sh.total = n2 > 0 ? max(b, 0) : 256;
    }
    __syncthreads();
    const int thr = sh.total;
    int m = 0;
    for (int b0 = 0; b0 < n; b0 += blockDim.x) {
      const int i = b0 + threadIdx.x;
      const int ci = i < n ? cand[i] : 0;
      const bool keep = i < n && sc[ci] >= thr;
      int tot;
      const int rank = block_rank(sh, keep, &tot);
      if (keep) cand[m + rank] = ci;
      m += tot;
    }
    n = m;
  }
  __syncthreads();
  SEL_PHASE(1);
  // 3. Harris responses: one wavefront per 4 candidates, 16 lanes per candidate over the 7x7 block
  //    pixels (the integer sums are order-free, so the float formula sees OpenCV's exact a, b, c)
  // The 9 x 16-byte patches (rows y0-4 .. y0+4 from the dword holding column x0-4) of 4
  // candidates per wave iteration are staged in LDS by 144 dword loads, then each 16-lane row
  // reads the neighbourhoods of its candidate's 49 block pixels from LDS.
  //    Software pipelined like the angles below: the next iteration's patch dwords are loaded into
  //    registers while this iteration's sums read LDS.
  constexpr int kPerWave = 4;
  constexpr int kHStg = (kPerWave * 36 + 63) / 64;
  const int stride_l = g.stride[l];
  const uint8_t* lvl = base + g.off[l];
  uint32_t hbuf[kHStg];
  auto hfetch = [&](int i0f) {
#pragma unroll
    for (int k = 0; k < kHStg; k++) {
      const int item = lane + 64 * k;
      if (item < kPerWave * 36) {
        const int u = item / 36, rr = (item % 36) >> 2, dw = item & 3;
        const int ci = cand[min(i0f + u, n - 1)];
        const int x0 = ci % w, y0 = ci / w;
        hbuf[k] = *(const __attribute__((address_space(1))) uint32_t*)(lvl + (y0 - 4 + rr + kB) * stride_l +
                                                                          ((x0 - 4 + kB) & ~3) + 4 * dw);
      }
    }
  };
  if (wv * kPerWave < n) hfetch(wv * kPerWave);
  for (int i0 = wv * kPerWave; i0 < n; i0 += nw * kPerWave) {
    uint32_t* hp = sh_patch + wv * kPatchDw;
#pragma unroll
    for (int k = 0; k < kHStg; k++) {
      const int item = lane + 64 * k;
      if (item < kPerWave * 36) hp[item] = hbuf[k];
    }
    if (i0 + nw * kPerWave < n) hfetch(i0 + nw * kPerWave);
    wave_lds_sync();
    // lane row u = lane >> 4 takes candidate i0 + u; its 16 lanes cover the 49 block pixels
    // (pixel t, t + 16, t + 32, t + 48) and the integer sums close with one row sum each
    const uint8_t* hb = reinterpret_cast<const uint8_t*>(hp);
    const int u = lane >> 4, t16 = lane & 15, i = i0 + u;
    int A = 0, B = 0, C = 0;
    if (i < n) {
      const int x0 = cand[i] % w;
      const uint8_t* P = hb + u * 144 + ((x0 - 4 + kB) & 3);  // P[r * 16 + c]: row y0-4+r, column x0-4+c
      auto at = [&](int r, int c) { return (int)P[r * 16 + c]; };
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int px = t16 + 16 * k;
        if (px < 49) {
          const int ar = px / 7, bc = px % 7;  // position (y0-3+ar, x0-3+bc) = patch (ar+1, bc+1)
          const int Ix = (at(ar + 1, bc + 2) - at(ar + 1, bc)) * 2 + (at(ar, bc + 2) - at(ar, bc)) +
                         (at(ar + 2, bc + 2) - at(ar + 2, bc));
          const int Iy = (at(ar + 2, bc + 1) - at(ar, bc + 1)) * 2 + (at(ar + 2, bc) - at(ar, bc)) +
                         (at(ar + 2, bc + 2) - at(ar, bc + 2));
          A += Ix * Ix; B += Iy * Iy; C += Ix * Iy;
        }
      }
    }
    wave_lds_sync();  // the patch is rewritten by the next iteration
    A = row_sum16(A); B = row_sum16(B); C = row_sum16(C);
    if (t16 == 0 && i < n) {
      const float scale = 1.f / ((1 << 2) * 7 * 255.f);
      const float sq = scale * scale * scale * scale;
      resp[i] = ((float)A * B - (float)C * C - 0.04f * ((float)A + B) * ((float)A + B)) * sq;
    }
  }
  __syncthreads();
  SEL_PHASE(2);
  // 4. retainBest(n_l) on the Harris response
  const int n1 = g.nper[l];
  if (n > n1) {
    const uint32_t thr = n1 > 0 ? nth_largest(sh, resp, n, n1) : 0xffffffffu;
    int m = 0;
    for (int b0 = 0; b0 < n; b0 += blockDim.x) {
      const int i = b0 + threadIdx.x;
      const bool keep = i < n && n1 > 0 && ord_key(resp[i]) >= thr;
      const int ci = i < n ? cand[i] : 0;
      const float rv = i < n ? resp[i] : 0.f;
      __syncthreads();
      int tot;
      const int rank = block_rank(sh, keep, &tot);
      if (keep) { cand[m + rank] = ci; resp[m + rank] = rv; }
      m += tot;
    }
    n = m;
  }
  __syncthreads();
  SEL_PHASE(3);
  if (n > g.lcap[l]) {
    if (threadIdx.x == 0) atomicOr(a.overflow, 1);
    n = g.lcap[l];
  }
  // 5. intensity-centroid angle: one wavefront per 4 keypoints over the circular patch (integer
  //    moments, order-free), fastAtan2 on lane 0; per-level staging
  float* out = a.lkp + ((size_t)s * g.cap + g.lofs[l]) * 6;
  // The 31 x 36-byte patches (rows y-15 .. y+15 from the dword holding column x-15) of 2
  // keypoints per wave iteration are staged in LDS by 558 dword loads; lane t then reads the
  // circle pixels t, t + 64, ... of each from LDS.
  constexpr int kAngPerWave = 2;
  // this lane's circle pixels t = 64 k + lane, once per workgroup: LDS offset | (du + 16) << 16 |
  // (dv + 16) << 24 (du = dv = 0 past the end)
  uint32_t cpx[kPatchIters];
#pragma unroll
  for (int k = 0; k < kPatchIters; k++) {
    const int t = k * 64 + lane;
    const short2 d = c_patch[t < kNPatch ? t : 0];
    cpx[k] = t < kNPatch ? (uint32_t)((d.y + 15) * 36 + d.x + 15) | (uint32_t)(d.x + 16) << 16 | (uint32_t)(d.y + 16) << 24
                         : (16u << 16) | (16u << 24);
  }
  // software pipelined: the next iteration's patch dwords are loaded into registers while this
  // iteration's moments are summed from LDS
  constexpr int kStg = (kAngPerWave * 279 + 63) / 64;
  uint32_t rbuf[kStg];
  int xs[kAngPerWave], ys[kAngPerWave];
  auto fetch = [&](int i0f) {
#pragma unroll
    for (int u = 0; u < kAngPerWave; u++) {
      const int ci = cand[min(i0f + u, n - 1)];
      xs[u] = ci % w; ys[u] = ci / w;
    }
#pragma unroll
    for (int k = 0; k < kStg; k++) {
      const int item = lane + 64 * k;
      if (item < kAngPerWave * 279) {
        const int u = item / 279, rr = (item % 279) / 9, dw = (item % 279) % 9;
        int x = xs[0], y = ys[0];
#pragma unroll
        for (int v = 1; v < kAngPerWave; v++)
          if (u == v) { x = xs[v]; y = ys[v]; }
        rbuf[k] = *(const __attribute__((address_space(1))) uint32_t*)(lvl + (y - 15 + rr + kB) * stride_l +
                                                                          ((x - 15 + kB) & ~3) + 4 * dw);
      }
    }
  };
  if (wv * kAngPerWave < n) fetch(wv * kAngPerWave);
  for (int i0 = wv * kAngPerWave; i0 < n; i0 += nw * kAngPerWave) {
    uint32_t* hp = sh_patch + wv * kPatchDw;
#pragma unroll
    for (int k = 0; k < kStg; k++) {
      const int item = lane + 64 * k;
      if (item < kAngPerWave * 279) hp[item] = rbuf[k];
    }
    int cx[kAngPerWave], cy[kAngPerWave];
#pragma unroll
    for (int u = 0; u < kAngPerWave; u++) { cx[u] = xs[u]; cy[u] = ys[u]; }
    if (i0 + nw * kAngPerWave < n) fetch(i0 + nw * kAngPerWave);
    wave_lds_sync();
    const uint8_t* hb = reinterpret_cast<const uint8_t*>(hp);
    int m01[kAngPerWave], m10[kAngPerWave];
#pragma unroll
    for (int u = 0; u < kAngPerWave; u++) {
      const uint8_t* P = hb + u * 279 * 4 + ((cx[u] - 15 + kB) & 3);  // P[r * 36 + c]: row y-15+r, column x-15+c
      m01[u] = m10[u] = 0;
#pragma unroll
      for (int k = 0; k < kPatchIters; k++) {
        const int v = (int)P[cpx[k] & 0xffffu];
        m10[u] += ((int)((cpx[k] >> 16) & 0xffu) - 16) * v;
        m01[u] += ((int)(cpx[k] >> 24) - 16) * v;
      }
    }
    wave_lds_sync();  // the patch is rewritten by the next iteration
#pragma unroll
    for (int u = 0; u < kAngPerWave; u++) { m01[u] = wave_sum(m01[u]); m10[u] = wave_sum(m10[u]); }
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < kAngPerWave; u++) {
        const int i = i0 + u;
        if (i >= n) break;
        float* o = out + (size_t)i * 6;
        o[0] = (float)cx[u]; o[1] = (float)cy[u]; o[2] = 31 * g.scale[l];
        o[3] = fast_atan2((float)m01[u], (float)m10[u]);
        o[4] = resp[i];
        o[5] = (float)l;
      }
    }
  }
  SEL_PHASE(4);
  if (threadIdx.x == 0) a.lcnt[s * kL + l] = n;
}

// Level-major blocks: consecutive blocks (dealt round-robin to the XCDs) are different scans of one
// level, so the heavy level-0 workgroups spread over every XCD.  One scan per grid scan index.
__global__ __launch_bounds__(kSelThreads, 4) void k_orb_select(Args a) {
  const int S = gridDim.x / kL;
  orb_select_body(a, blockIdx.x % S, blockIdx.x / S);
}

// The scans of a device list (a.smap, *a.scount entries): the grid's scan indices stride over the
// entries, so the launch is a few slots wide (placing a workgroup per possible entry, thousands that
// exit at once, took milliseconds beside the chain engines).
__global__ __launch_bounds__(kSelThreads, 4) void k_orb_select_list(Args a) {
  const int S = gridDim.x / kL;
  const int l = blockIdx.x / S, cnt = *a.scount;
  for (int i = blockIdx.x % S; i < cnt; i += S) {
    orb_select_body(a, i, l);
    __syncthreads();
  }
}

// levels in order, level-0 coordinates, cloud-track lookup and zero filter (a9)
__device__ __forceinline__ void orb_finish_body(const Args& a, int gi) {
  __shared__ SelShared sh;
  const Geom& g = a.g;
  const int s = a.smap ? a.smap[gi] : gi;
  int n = 0;
  for (int l = 0; l < kL; l++) {
    const int cnt = a.lcnt[s * kL + l];
    const float* in = a.lkp + ((size_t)s * g.cap + g.lofs[l]) * 6;
    for (int b0 = 0; b0 < cnt; b0 += blockDim.x) {
      const int i = b0 + threadIdx.x;
      bool keep = false;
      float o[6];
      float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < cnt) {
        for (int e = 0; e < 6; e++) o[e] = in[(size_t)i * 6 + e];
        o[0] *= g.scale[l];
        o[1] *= g.scale[l];
        const int col = (int)rintf(o[0]), row = (int)rintf(o[1]);
        p = a.track[(size_t)s * g.W * g.H + row * g.W + col];
        keep = !(fabsf(p.x) < 0.01f);
      }
      int tot;
      const int rank = block_rank(sh, keep, &tot);
      if (keep) {
        float* d = a.kp + ((size_t)s * g.cap + n + rank) * 6;
        for (int e = 0; e < 6; e++) d[e] = o[e];
        a.p3d[(size_t)s * g.cap + n + rank] = make_float4(p.x, p.y, p.z, 0.f);
      }
      n += tot;
    }
  }
  if (threadIdx.x == 0) a.nkp[s] = n;
}

__global__ __launch_bounds__(256) void k_orb_finish(Args a) {
  const int cnt = a.scount ? *a.scount : (int)gridDim.x;
  for (int gi = blockIdx.x; gi < cnt; gi += gridDim.x) {
    orb_finish_body(a, gi);
    __syncthreads();
  }
}

// steered rBRIEF: 32 lanes per keypoint, one descriptor byte each.  A workgroup takes chunks of
// kDescChunk keypoints (grid-strided): one lane per keypoint first computes its rotation (the
// double-precision cos / sin, once per keypoint instead of once per wavefront) and patch address
// into LDS tables, then each half-wave slot runs every 8th keypoint of the chunk.  The pattern's
// points lie in [-13, 13]^2, so rotated and rounded they stay within kDescR = 18 of the keypoint:
// its 37 x 37 blurred patch is staged in the slot's LDS by its 32 lanes (10 aligned dwords per row;
// the next keypoint's loads are in flight while this one's 512 tests read LDS).  A slot is written
// and read by one wavefront only.
constexpr int kDescR = 18;
constexpr int kDescRow = 40;  // staged bytes per patch row: 37 + the dword misalignment (<= 3)
constexpr int kDescDw = (2 * kDescR + 1) * (kDescRow / 4);  // 370 dwords per patch
constexpr int kDescChunk = 64;
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// kSlots = blockDim.x / 32; chunks c0, c0 + cstep, ... of the scan's keypoints
template <int kSlots>
__device__ __forceinline__ void orb_desc_body(const Args& a, int gi, int c0, int cstep) {
  __shared__ uint32_t patch[kSlots][kDescDw];
  __shared__ float kcs[kDescChunk][2];  // cos, sin of the keypoint's angle
  __shared__ int kpos[kDescChunk][2];   // patch byte offset in the scan's blurred pyramid, stride | shift << 16
  const Geom& g = a.g;
  const int s = a.smap ? a.smap[gi] : gi;
  const int byte = threadIdx.x & 31, slot = threadIdx.x >> 5;
  const int nk = a.nkp[s];
  const uint8_t* base = a.blur + (size_t)s * g.bytes;
  const uint8_t* P = reinterpret_cast<const uint8_t*>(patch[slot]);
  const uint32_t* pat = reinterpret_cast<const uint32_t*>(c_pattern.v) + byte * 8;  // x1 y1 x2 y2 of bits 0..7, + 13
  for (int k0 = c0 * kDescChunk; k0 < nk; k0 += cstep * kDescChunk) {
    __syncthreads();  // the previous chunk's tables are no longer read
    if (threadIdx.x < kDescChunk && k0 + (int)threadIdx.x < nk) {
      const float* kp = a.kp + ((size_t)s * g.cap + k0 + threadIdx.x) * 6;
      const int l = (int)kp[5];
      const float scale = 1.f / g.scale[l];
      const float ang = kp[3] * (float)(kPi / 180.f);
      kcs[threadIdx.x][0] = (float)cos((double)ang);
      kcs[threadIdx.x][1] = (float)sin((double)ang);
      const int cy = (int)rintf(kp[1] * scale), cx = (int)rintf(kp[0] * scale);
      // padded rows cy - 18 .. cy + 18, padded columns pc0 .. pc0 + 39 (pc0 = cx - 18 + kB rounded
      // down to a dword; the row has >= 44 bytes right of cx, kB = 23 > 18 above and below)
      const int pc = cx - kDescR + kB, pc0 = pc & ~3;
      kpos[threadIdx.x][0] = g.off[l] + (cy - kDescR + kB) * g.stride[l] + pc0;
      kpos[threadIdx.x][1] = g.stride[l] | (pc - pc0) << 16;
    }
    __syncthreads();
    const int n = min(kDescChunk, nk - k0);
    uint32_t v[(kDescDw + 31) / 32];
    auto load = [&](int j) {
      const uint8_t* src = base + kpos[j][0];
      const int ps = kpos[j][1] & 0xffff;
#pragma unroll
      for (int i = 0; i < (kDescDw + 31) / 32; i++) {
        const int e = byte + 32 * i, row = e / 10, d = e - 10 * row;
        if (e < kDescDw) v[i] = *(const __attribute__((address_space(1))) uint32_t*)(src + row * ps + 4 * d);
      }
    };
    if (slot < n) load(slot);
    for (int j = slot; j < n; j += kSlots) {
      wave_lds_sync();  // the previous keypoint's tests have read the slot
#pragma unroll
      for (int i = 0; i < (kDescDw + 31) / 32; i++) {
        const int e = byte + 32 * i;
        if (e < kDescDw) patch[slot][e] = v[i];
      }
      wave_lds_sync();
      if (j + kSlots < n) load(j + kSlots);
      const float ca = kcs[j][0], sa = kcs[j][1];
      const uint8_t* c0 = P + kDescR * kDescRow + kDescR + (kpos[j][1] >> 16);  // the keypoint's byte
      int bits = 0;
#pragma unroll
      for (int bit = 0; bit < 8; bit++) {
        const uint32_t pw = pat[bit];
        int t[2];
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const float qx = (float)((pw >> (16 * e)) & 255u) - 13.f, qy = (float)((pw >> (16 * e + 8)) & 255u) - 13.f;
          const float x = qx * ca - qy * sa, y = qx * sa + qy * ca;
          t[e] = c0[(int)rintf(y) * kDescRow + (int)rintf(x)];
        }
        bits |= (t[0] < t[1]) << bit;
      }
      a.desc[((size_t)s * g.cap + k0 + j) * 32 + byte] = (uint8_t)bits;
    }
  }
}

__global__ __launch_bounds__(256) void k_orb_desc(Args a) {
  const int cnt = a.scount ? *a.scount : (int)gridDim.y;
  for (int gi = blockIdx.y; gi < cnt; gi += gridDim.y) orb_desc_body<8>(a, gi, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------ matching (a10) + records
struct PairArgs {
  int npairs;
  const int* pslot;   // [npairs] buffer slot of pair pr (null: pr)
  const int* qscan;   // [npairs] cur scan (query)
  const int* tscan;   // [npairs] prev scan (train)
  const uint8_t* qdesc; const uint8_t* tdesc;  // descriptor arrays ([scan][cap][32])
  const float4* qp3d; const float4* tp3d;
  const int* qn; const int* tn;                // keypoint counts per scan
  int qcap, tcap;                              // descriptor / point strides per scan
  int bstride;                                 // per-pair stride of the buffers below (>= qcap)
  double frac;                                 // 0.3 / 0.2
  int* mscratch;      // [npairs][qcap] packed (dist << 16 | train)
  int* mout;          // [npairs][qcap][3] all matches (query, train, distance) in query order, or null
  double* rec;        // [npairs][qcap][9]
  int* kind;          // [npairs][qcap]
  int* stats;         // [npairs][8]: ok, -, nq, matches, good, iterations, termination, nt
  double* T;          // [npairs][7]
  const int* pcount;  // device count of pairs in use (null: npairs); the grid's other pairs exit
  int* arrive;        // [npairs] k_orb_pairs: train-block workgroups of the slot arrived (0 between launches)
};

__device__ __forceinline__ int hamming32(const uint32_t* a, const uint32_t* b) {
  int d = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d += __popc(a[i] ^ b[i]);
  return d;
}

// batchDistance cross-check, distance part: train i -> its nearest query (first minimum); each
// query keeps the nearest train among those that chose it (first minimum) = atomicMin of the
// packed (distance << 16 | train) (best[] preset to 0x7f7f7f7f).
// The same result on the matrix cores: Hamming(q, t) = |q| + |t| - 2 <q, t> with the 256
// descriptor bits as 0/1 int8 vectors and <q, t> from v_mfma_i32_16x16x64_i8 (four k-steps of 64
// bits; A and B fragments use one and the same lane -> k map, so the dot product does not depend
// on the hardware's k order).  A workgroup = kXmWaves waves x 16 trains; each 256-query tile is expanded
// to 0/1 bytes in LDS once and read by all the waves.  By the C/D layout lane l owns train column
// l & 15 and query rows 4 (l >> 4) .. +3 of every 16-query tile, so its running first minimum
// follows query order; the four lanes of a column merge by (distance, query) at the end.
constexpr int kXmWaves = 8;                 // waves per workgroup (8: room beside the chain engines)
constexpr int kXmTrains = 16 * kXmWaves;    // trains per workgroup (16 per wave)
constexpr int kXmQTile = 256;   // queries expanded per LDS tile
constexpr int kXmRow = 272;     // LDS bytes per expanded query (256 + 16: rows start on distinct banks)
using i32x4 = __attribute__((ext_vector_type(4))) int;

__device__ __forceinline__ uint32_t spread4(uint32_t n) { return (n * 0x00204081u) & 0x01010101u; }
__device__ __forceinline__ i32x4 expand16(uint32_t b) {  // 16 bits -> 16 bytes of 0 / 1
  i32x4 v;
  v.x = (int)spread4(b & 15u);
  v.y = (int)spread4((b >> 4) & 15u);
  v.z = (int)spread4((b >> 8) & 15u);
  v.w = (int)spread4((b >> 12) & 15u);
  return v;
}

__device__ __forceinline__ void orb_xdist_mfma_body(const PairArgs& p, int pi) {
  __shared__ i32x4 qx[kXmQTile * kXmRow / 16];
  __shared__ int qpop[kXmQTile];
  const int pr = p.pslot ? p.pslot[pi] : pi;
  const int qs = p.qscan[pi], ts = p.tscan[pi];
  const int nq = p.qn[qs], nt = p.tn[ts];
  const int t0 = blockIdx.y * kXmTrains;
  if (t0 >= nt) return;
  const uint32_t* Q = reinterpret_cast<const uint32_t*>(p.qdesc + (size_t)qs * p.qcap * 32);
  const uint32_t* T = reinterpret_cast<const uint32_t*>(p.tdesc + (size_t)ts * p.tcap * 32);
  int* best = p.mscratch + (size_t)pr * p.bstride;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, h = lane >> 4, col = lane & 15;
  const int ti = t0 + wv * 16 + col;  // this lane's train
  // B fragments: bits 64 s + 16 h .. +15 of train ti for k-step s
  i32x4 bfr[4];
  int tpop = 0;
  {
    uint32_t td[8];
#pragma unroll
    for (int e = 0; e < 8; e++) td[e] = ti < nt ? T[(size_t)ti * 8 + e] : 0u;
#pragma unroll
    for (int e = 0; e < 8; e++) tpop += __popc(td[e]);
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const uint32_t w = td[2 * s + (h >> 1)];
      bfr[s] = expand16((h & 1) ? (w >> 16) : (w & 0xffffu));
    }
  }
  int bd = 0x7fffffff, bj = -1;
  for (int q0 = 0; q0 < nq; q0 += kXmQTile) {
    const int tn = min(kXmQTile, nq - q0);
    __syncthreads();  // the previous tile is no longer read
    for (int it = threadIdx.x; it < kXmQTile * 16; it += 64 * kXmWaves) {
      const int q = it >> 4, c = it & 15;
      const uint32_t w = q < tn ? Q[(size_t)(q0 + q) * 8 + (c >> 1)] : 0u;
      qx[(q * kXmRow + c * 16) / 16] = expand16((c & 1) ? (w >> 16) : (w & 0xffffu));
    }
    if (threadIdx.x < kXmQTile) {
      const int q = threadIdx.x;
      int pc = 0;
      if (q < tn)
#pragma unroll
        for (int e = 0; e < 8; e++) pc += __popc(Q[(size_t)(q0 + q) * 8 + e]);
      qpop[q] = pc;
    }
    __syncthreads();
    for (int r0 = 0; r0 < tn; r0 += 16) {
      i32x4 acc = {0, 0, 0, 0};
      const int rowb = ((r0 + col) * kXmRow + h * 16) / 16;
#pragma unroll
      for (int s = 0; s < 4; s++) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(qx[rowb + s * 4], bfr[s], acc, 0, 0, 0);
#pragma unroll
      for (int reg = 0; reg < 4; reg++) {
        const int j = r0 + 4 * h + reg;
        if (j < tn) {
          const int d = qpop[j] + tpop - 2 * acc[reg];
          if (d < bd) { bd = d; bj = q0 + j; }
        }
      }
    }
  }
  // merge the four lanes of each column: first minimum in query order
#pragma unroll
  for (int o = 16; o <= 32; o <<= 1) {
    const int od = __shfl_xor(bd, o), oj = __shfl_xor(bj, o);
    if (od < bd || (od == bd && oj >= 0 && (bj < 0 || oj < bj))) { bd = od; bj = oj; }
  }
  if (h == 0 && ti < nt && bj >= 0) atomicMin(&best[bj], (bd << 16) | ti);
}

// the grid's pair indices stride over the pairs in use (*p.pcount of them when given)
__global__ __launch_bounds__(64 * kXmWaves) void k_orb_xdist_mfma(PairArgs p) {
  const int cnt = p.pcount ? *p.pcount : (int)gridDim.x;
  for (int pi = blockIdx.x; pi < cnt; pi += gridDim.x) {
    orb_xdist_mfma_body(p, pi);
    __syncthreads();
  }
}

// Selection part: std::sort by distance (stable, query order), the first ceil(frac M), the
// good-frame test and the front_end_residual records.
__device__ __forceinline__ void orb_match_body(const PairArgs& p, int pi) {
  __shared__ SelShared sh;
  __shared__ int hist[257];
  __shared__ int sM, sG;
  const int pr = p.pslot ? p.pslot[pi] : pi;
  const int qs = p.qscan[pi], ts = p.tscan[pi];
  const int nq = p.qn[qs], nt = p.tn[ts];
  int* best = p.mscratch + (size_t)pr * p.bstride;
  __syncthreads();
  // std::sort by distance (stable, query order) + the first ceil(frac M)
  for (int b = threadIdx.x; b < 257; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  for (int j = threadIdx.x; j < nq; j += blockDim.x)
    if (best[j] != kNoMatch) atomicAdd(&hist[best[j] >> 16], 1);
  __syncthreads();
  if (threadIdx.x < 64) {
    // wave 0: lane i holds bins 5i .. 5i+4; M = all matches, G = ceil(frac M) (the first G with
    // G >= M frac, in double), d* = the first bin whose inclusive prefix reaches G
    const int lane = threadIdx.x;
    int hb[5], loc = 0;
#pragma unroll
    for (int e = 0; e < 5; e++) {
      const int b = 5 * lane + e;
      hb[e] = b < 257 ? hist[b] : 0;
      loc += hb[e];
    }
    int inc = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    const int M = __shfl(inc, 63);
    const int G = (int)ceil((double)M * p.frac);
    int cum = inc - loc, hit = -1, before = 0;
#pragma unroll
    for (int e = 0; e < 5; e++) {
      if (hit < 0 && G > 0 && cum + hb[e] >= G) { hit = 5 * lane + e; before = cum; }
      cum += hb[e];
    }
    const uint64_t m = __ballot(hit >= 0);
    if (lane == 0) {
      sM = M;
      sG = G;
      sh.total = 257;
      sh.want = G;
    }
    if (m && lane == __ffsll((long long)m) - 1) {
      sh.total = hit;
      sh.want = G - before;  // matches of distance d* to take, in query order
    }
  }
  __syncthreads();
  const int M = sM, G = sG, dstar = sh.total, take = sh.want;
  int n = 0, neq = 0, nm = 0;
  for (int b0 = 0; b0 < nq; b0 += blockDim.x) {
    const int j = b0 + threadIdx.x;
    const int v = j < nq ? best[j] : kNoMatch;
    const int d = v >> 16;
    if (p.mout) {
      int tm;
      const int rm = block_rank(sh, v != kNoMatch, &tm);
      if (v != kNoMatch) {
        int* o = p.mout + ((size_t)pr * p.bstride + nm + rm) * 3;
        o[0] = j; o[1] = v & 0xffff; o[2] = d;
      }
      nm += tm;
    }
    const bool eq = v != kNoMatch && d == dstar;
    int te;
    const int req = block_rank(sh, eq, &te);
    const bool keep = v != kNoMatch && (d < dstar || (eq && neq + req < take));
    neq += te;
    int tot;
    const int rank = block_rank(sh, keep, &tot);
    if (keep) {
      const int i = v & 0xffff;
      const float4 a = p.qp3d[(size_t)qs * p.qcap + j], b = p.tp3d[(size_t)ts * p.tcap + i];
      double* r = p.rec + ((size_t)pr * p.bstride + n + rank) * 9;
      r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = b.x; r[4] = b.y; r[5] = b.z; r[6] = r[7] = r[8] = 0;
      p.kind[(size_t)pr * p.bstride + n + rank] = 3;
    }
    n += tot;
  }
  // every read of this pair's best[] row is done: back to the "no match" sentinel for the next
  // launch that uses the slot (k_orb_xdist_mfma writes entries < nq only; the rest stay sentinel
  // from the allocation), so no fill launch precedes the distances
  __syncthreads();
  for (int j = threadIdx.x; j < nq; j += blockDim.x) best[j] = kNoMatch;
  if (threadIdx.x == 0) {
    int* st = p.stats + pr * 8;
    st[0] = (nt != nq && G >= 4 && G != M) ? 1 : 0;
    st[1] = 0;
    st[2] = nq;
    st[3] = M;
    st[4] = G;
    st[5] = 0;
    st[6] = -1;
    st[7] = nt;
  }
}

// the grid's pair indices stride over the pairs in use (*p.pcount of them when given)
__global__ __launch_bounds__(kPairThreads, 8) void k_orb_match(PairArgs p) {
  const int cnt = p.pcount ? *p.pcount : (int)gridDim.x;
  for (int pi = blockIdx.x; pi < cnt; pi += gridDim.x) {
    orb_match_body(p, pi);
    __syncthreads();
  }
}

// front_end_residual solve per pair (p2p_calculateRandT): identity start, 20 iterations
struct LmSh {
  double red[kLmThreads / 16][kAcc];
  double x[7];
  double acc[kAcc];
  int flag;
};

__device__ void pair_eval(LmSh& sh, const double* rec, int n) {
  double acc[kAcc];
#pragma unroll
  for (int e = 0; e < kAcc; e++) acc[e] = 0;
  const DQ q{sh.x[0], sh.x[1], sh.x[2], sh.x[3]};
  const D3 t{sh.x[4], sh.x[5], sh.x[6]};
  for (int i = threadIdx.x; i < n; i += kLmThreads) block_accum(3, rec + (size_t)i * 9, q, t, acc);
  const int lane = threadIdx.x & 63, row = threadIdx.x >> 4;
#pragma unroll
  for (int e = 0; e < kAcc; e++) {
    const double v = row_sum(acc[e]);
    if ((lane & 15) == 0) sh.red[row][e] = v;
  }
  __syncthreads();
  if (threadIdx.x < kAcc) {
    double v = 0;
    for (int w = 0; w < kLmThreads / 16; w++) v += sh.red[w][threadIdx.x];
    sh.acc[threadIdx.x] = v;
  }
  __syncthreads();
}

// Batch outputs: scan 0 is the first frame (stats -1, its keypoint count), scan k > 0 pair
// (k-1, k) with its re-detection flag.
struct OutArgs {
  int* outS; double* outT;
  const int* stats; const double* T; const int* redet; const int* nkp0;
  int n_scans;
};

__device__ __forceinline__ void orb_out_at(const OutArgs& a, int k) {
  int* outS = a.outS;
  double* outT = a.outT;
  const int* stats = a.stats;
  const double* T = a.T;
  const int* redet = a.redet;
  const int* nkp0 = a.nkp0;
  int* o = outS + (size_t)k * 8;
  double* t = outT + (size_t)k * 7;
  if (k == 0) {
    for (int e = 0; e < 8; e++) o[e] = e == 0 ? -1 : e == 2 ? nkp0[0] : 0;
    for (int e = 0; e < 7; e++) t[e] = e == 3 ? 1.0 : 0.0;
    return;
  }
  for (int e = 0; e < 8; e++) o[e] = stats[(size_t)(k - 1) * 8 + e];
  if (redet[k - 1]) o[1] = 1;
  for (int e = 0; e < 7; e++) t[e] = T[(size_t)(k - 1) * 7 + e];
}

__global__ __launch_bounds__(256) void k_orb_out(OutArgs a) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k < a.n_scans) orb_out_at(a, k);
}

// ---- the re-detection rule of detectfeatures decided on the device (lislam_batch_intensity_odometry)
// Pair k (query scan k, train scan k-1, buffer slot k-1) first tries frame k's n-feature set against
// the set frame k-1 ended with; when that fails, both frames re-detect with 2n features and frame k
// keeps the 2n set (intensity_feature_tracker.cpp:631-687).  cur2[k] = frame k holds the 2n set;
// pset[k] = the set (0: n, 1: 2n of frame k-1) pair k's current first attempt used; ok1[k] = that
// attempt succeeded (its stats word).  One decision pass replays the sequential rule over the
// attempts made so far and lists the pairs whose attempt used the wrong previous set (to redo,
// grouped by the set they need) and the frames whose 2n set is missing; the final pass (mode 2)
// lists the re-detecting pairs' 2n-against-2n matches instead, or reports "not converged".
struct CascadeArgs {
  int n;
  const int* stats;   // [n - 1][8] pair buffer stats (slot k - 1 = pair k)
  int8_t* pset;       // [n]
  int8_t* cur2;       // [n]
  int8_t* have2;      // [n] frame's 2n set detected
  int* e2list;        // [n] frames to detect with 2n features
  int* e2cnt;         // [1]
  int* plist;         // [2][3][n] pairs to (re)attempt against the n / 2n previous set; final: [0]
                      // (each [3][n]: query scans | train scans | slots, stride n)
  int* pcnt;          // [2]
  int* redet;         // [n - 1] pair k re-detected (k_orb_out)
  int* status;        // [2] converged, decision passes
};
constexpr int kCascadeMax = 8192;

// (256 threads: the last k_orb_lm workgroup of a launch, or k_orb_tail)
__device__ __forceinline__ void orb_decide_body(const CascadeArgs& cs, int mode) {
  __shared__ int8_t ok1[kCascadeMax], ps[kCascadeMax], c2[kCascadeMax], h2[kCascadeMax];
  const int n = cs.n;
  for (int k = threadIdx.x; k < n; k += 256) {
    ok1[k] = k >= 1 ? (int8_t)(cs.stats[(size_t)(k - 1) * 8] == 1) : (int8_t)1;
    ps[k] = mode == 0 ? (int8_t)0 : cs.pset[k];
    c2[k] = mode == 0 ? (int8_t)0 : cs.cur2[k];
    h2[k] = mode == 0 ? (int8_t)0 : cs.have2[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int prev = 0;  // frame 0 keeps its n set
    for (int k = 1; k < n; k++) {
      if (ps[k] == prev) c2[k] = (int8_t)!ok1[k];
      prev = c2[k];
    }
    int cnt[2] = {0, 0}, ne = 0;
    bool dirty = false;
    for (int k = 1; k < n; k++) {
      const int g = c2[k - 1];
      if (ps[k] == g) continue;
      dirty = true;
      if (mode == 2) break;
      int* L = cs.plist + (size_t)g * 3 * n;
      L[cnt[g]] = k; L[n + cnt[g]] = k - 1; L[2 * n + cnt[g]] = k - 1;
      cnt[g]++;
      if (g == 1 && !h2[k - 1]) { h2[k - 1] = 1; cs.e2list[ne++] = k - 1; }
      ps[k] = (int8_t)g;
    }
    if (mode == 2) {
      if (!dirty) {  // converged: the re-detecting pairs, 2n against 2n (frac 0.2)
        int* L = cs.plist;
        for (int k = 1; k < n; k++) {
          const int r = c2[k];
          cs.redet[k - 1] = r;
          if (!r) continue;
          if (!h2[k - 1]) { h2[k - 1] = 1; cs.e2list[ne++] = k - 1; }
          if (!h2[k]) { h2[k] = 1; cs.e2list[ne++] = k; }
          L[cnt[0]] = k; L[n + cnt[0]] = k - 1; L[2 * n + cnt[0]] = k - 1;
          cnt[0]++;
        }
      }
      cs.status[0] = dirty ? 0 : 1;
    }
    cs.pcnt[0] = cnt[0];
    cs.pcnt[1] = cnt[1];
    *cs.e2cnt = ne;
    cs.status[1] = mode == 0 ? 1 : cs.status[1] + 1;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < n; k += 256) {
    cs.pset[k] = ps[k];
    cs.cur2[k] = c2[k];
    cs.have2[k] = h2[k];
  }
}


// What the last k_orb_lm workgroup of a launch runs once every pair's solve is done (kind 0:
// nothing; 1: the cascade decision of `mode`; 2: the batch outputs): the launch that would follow
// the solve on the stream, folded into it.
struct LmTail {
  int kind = 0, mode = 0;
  int* arrive = nullptr;  // one counter (0 between launches)
  CascadeArgs cs{};
  OutArgs out{};
};

// the kind-1 / kind-2 launch on its own (a launch with no pairs)
__global__ __launch_bounds__(256) void k_orb_tail(LmTail tl) {
  if (tl.kind == 1) orb_decide_body(tl.cs, tl.mode);
  if (tl.kind == 2)
    for (int k = threadIdx.x; k < tl.out.n_scans; k += 256) orb_out_at(tl.out, k);
}

__device__ __forceinline__ void orb_lm_body(const PairArgs& p, int max_it, int pi) {
  __shared__ LmSh sh;
  const int pr = p.pslot ? p.pslot[pi] : pi;
  int* st = p.stats + pr * 8;
  double* T = p.T + pr * 7;
  const bool good = st[0] == 1;
  const int n = st[4];
  const double* rec = p.rec + (size_t)pr * p.bstride * 9;
  if (!good) {
    if (threadIdx.x == 0) {
      const double I[7] = {0, 0, 0, 1, 0, 0, 0};
      for (int e = 0; e < 7; e++) T[e] = I[e];
    }
    return;
  }
  __shared__ LM lm;  // in registers only inside thread 0's step
  if (threadIdx.x == 0) {
    const double I[7] = {0, 0, 0, 1, 0, 0, 0};
    for (int e = 0; e < 7; e++) sh.x[e] = I[e];
  }
  __syncthreads();
  pair_eval(sh, rec, n);
  if (threadIdx.x == 0) {
    const bool cont = lm_start(lm, sh.x, sh.acc, max_it);
    sh.flag = cont;
    if (cont)
      for (int e = 0; e < 7; e++) sh.x[e] = lm.xc[e];
  }
  __syncthreads();
  bool go = sh.flag;
  while (go) {
    pair_eval(sh, rec, n);
    if (threadIdx.x == 0) {
      const bool cont = lm_next(lm, sh.acc, max_it);
      sh.flag = cont;
      if (cont)
        for (int e = 0; e < 7; e++) sh.x[e] = lm.xc[e];
    }
    __syncthreads();
    go = sh.flag;
  }
  if (threadIdx.x == 0) {
    for (int e = 0; e < 7; e++) T[e] = lm.x[e];
    st[5] = lm.it;
    st[6] = lm.term;
  }
}

__global__ __launch_bounds__(kLmThreads) void k_orb_lm(PairArgs p, int max_it, LmTail tl) {
  static_assert(kLmThreads == 256, "the tail bodies are written for 256 threads");
  const int cnt = p.pcount ? *p.pcount : (int)gridDim.x;
  for (int pi = blockIdx.x; pi < cnt; pi += gridDim.x) {
    orb_lm_body(p, max_it, pi);
    __syncthreads();
  }
  if (tl.kind == 0) return;
  // the last workgroup to arrive (told by the value its add returns) runs the tail once every
  // workgroup's stats and poses are visible
  __shared__ int s_last;
  if (!wg_arrive_last(tl.arrive, (int)gridDim.x, &s_last)) return;  // every pair's stats and pose
  if (tl.kind == 1) orb_decide_body(tl.cs, tl.mode);
  if (tl.kind == 2)
    for (int k = threadIdx.x; k < tl.out.n_scans; k += 256) orb_out_at(tl.out, k);
}

// A pair's distances and selection in one launch (the two kernels above, unchanged): the last of a
// pair's train-block workgroups to arrive — an agent-scope counter per buffer slot, told by the
// value its add returns — runs the selection over the pair's best[] row once every block's
// atomicMin is visible, and puts the counter back to 0 for the next launch.  One dependent launch
// fewer per attempt, each of which waits for room beside the chain engines.  (The solve stays a
// launch of its own: its 256-VGPR thread-0 step would cap the distance blocks at one workgroup per
// CU.)
__global__ __launch_bounds__(64 * kXmWaves) void k_orb_pairs(PairArgs p) {
  static_assert(64 * kXmWaves == kPairThreads, "k_orb_pairs workgroup");
  __shared__ int s_last;
  const int cnt = p.pcount ? *p.pcount : (int)gridDim.x;
  for (int pi = blockIdx.x; pi < cnt; pi += gridDim.x) {
    orb_xdist_mfma_body(p, pi);
    const int pr = p.pslot ? p.pslot[pi] : pi;
    if (wg_arrive_last(p.arrive + pr, (int)gridDim.y, &s_last))  // every block's atomicMin
      orb_match_body(p, pi);
    __syncthreads();
  }
}

}  // namespace orbk
}  // namespace lislam

// ================================================================== host side
using namespace lislam;
using namespace lislam::orbk;

namespace {

int ofail(lislam_ctx* c, int code, const char* fmt, ...) {
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

#define OCHK(ctx, x)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) return ofail(ctx, LISLAM_ERR_DEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)
#define ORC(x)                        \
  do {                                \
    int rc_ = (x);                    \
    if (rc_ != LISLAM_OK) return rc_; \
  } while (0)

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

int cv_round(float v) { return (int)std::nearbyint(v); }

// nfeaturesPerLevel of computeKeyPoints (orb.cpp)
void features_per_level(int nfeatures, int* n) {
  const float factor = (float)(1.0 / (double)1.2f);
  float nd = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)kL));
  int sum = 0;
  for (int l = 0; l < kL - 1; l++) {
    n[l] = cv_round(nd);
    sum += n[l];
    nd *= factor;
  }
  n[kL - 1] = std::max(nfeatures - sum, 0);
}

}  // namespace

// One ORB engine: geometry, resize tables, mask pyramid, per-scan buffers for up to max_scans
// scans of one image size and feature budget.
struct OrbEngine {
  lislam_ctx* ctx = nullptr;
  int H = 0, W = 0, max_scans = 0, nfeatures = 0;
  Geom g{};
  std::vector<void*> allocs;
  int *xo = nullptr, *yo = nullptr, *lim = nullptr;
  uint16_t *xc = nullptr, *yc = nullptr;
  int xs = 0, ys = 0;
  uint8_t* mpyr = nullptr;
  uint8_t *pyr = nullptr, *blur = nullptr, *nms = nullptr, *desc = nullptr;
  int *cand = nullptr, *lcnt = nullptr, *nkp = nullptr, *overflow = nullptr, *smap = nullptr;
  float *cresp = nullptr, *lkp = nullptr, *kp = nullptr;
  float4* p3d = nullptr;
  ~OrbEngine() {
    for (void* p : allocs) (void)hipFree(p);
  }
  template <typename T>
  int alloc(T** p, size_t count) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
    if (e != hipSuccess) return ofail(ctx, LISLAM_ERR_DEVICE, "hipMalloc(%zu): %s", count * sizeof(T), hipGetErrorString(e));
    allocs.push_back(q);
    *p = static_cast<T*>(q);
    return LISLAM_OK;
  }
  Args args(const uint8_t* img, const float4* track) const {
    Args a{};
    a.g = g;
    a.t.xo = xo; a.t.xc = xc; a.t.yo = yo; a.t.yc = yc; a.t.lim = lim; a.t.xs = xs; a.t.ys = ys;
    a.S = max_scans;
    a.img = img; a.track = track;
    a.pyr = pyr; a.blur = blur; a.mpyr = mpyr; a.nms = nms; a.cand = cand; a.cresp = cresp;
    a.lkp = lkp; a.lcnt = lcnt; a.kp = kp; a.p3d = p3d; a.desc = desc; a.nkp = nkp; a.overflow = overflow;
    a.smap = nullptr;
    return a;
  }
};

namespace {

int engine_init(OrbEngine* e, lislam_ctx* c, int H, int W, int max_scans, int nfeatures, const uint8_t* mask) {
  e->ctx = c; e->H = H; e->W = W; e->max_scans = max_scans; e->nfeatures = nfeatures;
  Geom& g = e->g;
  g.W = W; g.H = H;
  int off = 0;
  g.pix[0] = 0;
  g.pad[0] = 0;
  features_per_level(nfeatures, g.nper);
  g.lofs[0] = 0;
  for (int l = 0; l < kL; l++) {
    const float scale = (float)std::pow((double)1.2f, (double)l);
    const float inv = 1.0f / scale;
    g.scale[l] = scale;
    g.w[l] = cv_round((float)W * inv);
    g.h[l] = cv_round((float)H * inv);
    if (g.w[l] < 1 || g.h[l] < 1) return ofail(c, LISLAM_ERR_ARG, "image %dx%d too small for 8 ORB levels", W, H);
    g.stride[l] = (g.w[l] + 2 * kB + 15) & ~15;  // 16-byte aligned rows (staged as dwords)
    g.off[l] = off;
    off += g.stride[l] * (g.h[l] + 2 * kB);
    g.pix[l + 1] = g.pix[l] + g.w[l] * g.h[l];
    g.pad[l + 1] = g.pad[l] + g.stride[l] * (g.h[l] + 2 * kB);
    g.lcap[l] = 2 * g.nper[l] + 64;
    g.lofs[l + 1] = g.lofs[l] + g.lcap[l];
  }
  if ((kFastBand + 2) * (g.w[0] + 2) > 65536)  // k_orb_fastnms' u16 candidate list
    return ofail(c, LISLAM_ERR_ARG, "image width %d too large for the FAST band", W);
  g.fband[0] = 0;
  g.bband[0] = 0;
  g.rband[0] = 0;
  for (int l = 0; l < kL; l++) {
    g.fband[l + 1] = g.fband[l] + (g.h[l] + kFastBand - 1) / kFastBand;
    g.bband[l + 1] = g.bband[l] + (g.h[l] + 2 * kB + kBlurBand - 1) / kBlurBand;
    g.rband[l + 1] = g.rband[l] + (g.h[l] + kRoiBand - 1) / kRoiBand;
  }
  g.bytes = (off + 255) & ~255;
  g.cap = g.lofs[kL];
  // Gaussian taps (getGaussianKernel(7, 2, CV_32F))
  double sum = 0;
  for (int i = 0; i < 7; i++) {
    const double x = i - 3.0;
    g.gk[i] = (float)std::exp(-0.5 / 4.0 * x * x);
    sum += g.gk[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 7; i++) g.gk[i] = (float)(g.gk[i] * sum);
  // umax of the circular patch
  {
    int* umax = g.umax;
    const int vmax = (int)std::floor(kHalf * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(kHalf * std::sqrt(2.f) / 2);
    for (int v = 0; v <= vmax; ++v) umax[v] = (int)std::nearbyint(std::sqrt((double)kHalf * kHalf - v * v));
    for (int v = kHalf, v0 = 0; v >= vmin; --v) {
      while (umax[v0] == umax[v0 + 1]) ++v0;
      umax[v] = v0;
      ++v0;
    }
    std::vector<short2> patch;  // the circular patch of ICAngles: rows -15..15, |u| <= umax[|v|]
    for (int v = -kHalf; v <= kHalf; v++)
      for (int u = -umax[std::abs(v)]; u <= umax[std::abs(v)]; u++) patch.push_back(make_short2((short)u, (short)v));
    g.npatch = (int)patch.size();
    if (g.npatch != kNPatch) return ofail(c, LISLAM_ERR_STATE, "ICAngles patch has %d pixels", g.npatch);
    OCHK(c, hipMemcpyToSymbolAsync(HIP_SYMBOL(c_patch), patch.data(), patch.size() * sizeof(short2), 0,
                                   hipMemcpyHostToDevice, c->stream));
  }
  // resize tables (INTER_LINEAR_EXACT of level l from level l-1)
  e->xs = g.w[0];
  e->ys = g.h[0];
  std::vector<int> hxo((size_t)kL * e->xs, 0), hyo((size_t)kL * e->ys, 0), hlim(kL * 4, 0);
  std::vector<uint16_t> hxc((size_t)kL * e->xs, 0), hyc((size_t)kL * e->ys, 0);
  for (int l = 1; l < kL; l++) {
    for (int axis = 0; axis < 2; axis++) {
      const int src = axis == 0 ? g.w[l - 1] : g.h[l - 1], dst = axis == 0 ? g.w[l] : g.h[l];
      int* o = axis == 0 ? &hxo[(size_t)l * e->xs] : &hyo[(size_t)l * e->ys];
      uint16_t* cc = axis == 0 ? &hxc[(size_t)l * e->xs] : &hyc[(size_t)l * e->ys];
      int mn = 0, mx = dst;
      const double inv_scale = (double)dst / src;
      const double scale = 1.0 / inv_scale;
      for (int v = 0; v < dst; v++) {
        const double fval = scale * ((double)v + 0.5) - 0.5;
        const int ival = (int)std::floor(fval);
        if (ival >= 0 && src > 1) {
          if (ival < src - 1) {
            o[v] = ival;
            cc[v] = (uint16_t)std::nearbyint((fval - (double)ival) * 256.0);
          } else {
            o[v] = src - 1;
            mx = std::min(mx, v);
          }
        } else {
          mn = std::max(mn, v + 1);
        }
      }
      hlim[l * 4 + axis * 2] = mn;
      hlim[l * 4 + axis * 2 + 1] = mx;
    }
  }
  hipStream_t st = c->stream;
  ORC(e->alloc(&e->xo, hxo.size()));
  ORC(e->alloc(&e->yo, hyo.size()));
  ORC(e->alloc(&e->xc, hxc.size()));
  ORC(e->alloc(&e->yc, hyc.size()));
  ORC(e->alloc(&e->lim, hlim.size()));
  OCHK(c, hipMemcpyAsync(e->xo, hxo.data(), hxo.size() * 4, hipMemcpyHostToDevice, st));
  OCHK(c, hipMemcpyAsync(e->yo, hyo.data(), hyo.size() * 4, hipMemcpyHostToDevice, st));
  OCHK(c, hipMemcpyAsync(e->xc, hxc.data(), hxc.size() * 2, hipMemcpyHostToDevice, st));
  OCHK(c, hipMemcpyAsync(e->yc, hyc.data(), hyc.size() * 2, hipMemcpyHostToDevice, st));
  OCHK(c, hipMemcpyAsync(e->lim, hlim.data(), hlim.size() * 4, hipMemcpyHostToDevice, st));
  const size_t S = max_scans;
  ORC(e->alloc(&e->pyr, S * g.bytes));
  ORC(e->alloc(&e->blur, S * g.bytes));
  ORC(e->alloc(&e->nms, S * g.pix[kL] + 16));  // + 16: k_orb_select reads whole aligned dwords
  ORC(e->alloc(&e->cand, S * g.pix[kL]));
  ORC(e->alloc(&e->cresp, S * g.pix[kL]));
  ORC(e->alloc(&e->lkp, S * g.cap * 6));
  ORC(e->alloc(&e->lcnt, S * kL));
  ORC(e->alloc(&e->kp, S * g.cap * 6));
  ORC(e->alloc(&e->p3d, S * g.cap));
  ORC(e->alloc(&e->desc, S * g.cap * 32));
  ORC(e->alloc(&e->nkp, S));
  ORC(e->alloc(&e->overflow, 1));
  ORC(e->alloc(&e->smap, S));
  OCHK(c, hipMemsetAsync(e->overflow, 0, 4, st));
  if (mask) {  // mask pyramid, once
    uint8_t* dmask = nullptr;
    ORC(e->alloc(&dmask, (size_t)H * W));
    ORC(e->alloc(&e->mpyr, g.bytes));
    OCHK(c, hipMemcpyAsync(dmask, mask, (size_t)H * W, hipMemcpyDefault, st));
    Args a = e->args(dmask, nullptr);
    for (int l = 0; l < kL; l++)
      hipLaunchKernelGGL(k_orb_level, dim3(cdiv(g.stride[l] * (g.h[l] + 2 * kB), 256 * kLevelPx), 1), dim3(256), 0, st,
                         a, l, 1);
    OCHK(c, hipGetLastError());
  }
  return LISLAM_OK;
}

}  // namespace

namespace {

Args args_slot(const OrbEngine* e, const uint8_t* img, const float4* track, int slot) {
  Args a = e->args(img, track);
  const Geom& g = e->g;
  const size_t s = slot;
  a.img = img ? img + s * g.W * g.H : nullptr;
  a.track = track ? track + s * g.W * g.H : nullptr;
  a.pyr = e->pyr + s * g.bytes;
  a.blur = e->blur + s * g.bytes;
  a.nms = e->nms + s * g.pix[kL];
  a.cand = e->cand + s * g.pix[kL];
  a.cresp = e->cresp + s * g.pix[kL];
  a.lkp = e->lkp + s * g.cap * 6;
  a.lcnt = e->lcnt + s * kL;
  a.kp = e->kp + s * g.cap * 6;
  a.p3d = e->p3d + s * g.cap;
  a.desc = e->desc + s * g.cap * 32;
  a.nkp = e->nkp + s;
  return a;
}

// a8 + a9 for scans [slot0, slot0 + n) of the engine (device images / tracks indexed by scan),
// or for the scans of `list` (host, n entries) when given
int engine_detect_slots(OrbEngine* e, const uint8_t* d_img, const float4* d_track, int slot0, int n,
                        const int* list = nullptr) {
  lislam_ctx* c = e->ctx;
  hipStream_t st = c->stream;
  if (n <= 0) return LISLAM_OK;
  Args a = list ? e->args(d_img, d_track) : args_slot(e, d_img, d_track, slot0);
  a.S = n;
  if (list) {
    OCHK(c, hipMemcpyAsync(e->smap, list, (size_t)n * 4, hipMemcpyHostToDevice, st));
    a.smap = e->smap;
  }
  const Geom& g = e->g;
  const bool fused = g.W % 4 == 0 && g.h[1] <= 64 && g.stride[0] / 4 <= kPyrThreads && pyr_split(g) <= kPyrLds0 &&
                     g.w[1] * g.h[1] <= kPyrOdd && g.w[2] * g.h[2] <= kPyrEven;
  {
    TimedScope t(c, kT_orb_pyramid);
    // one workgroup per scan when level 0 fits 64 KiB of LDS (64 x 1024; the border rows and the
    // blurred copy follow from k_orb_roiblur); larger images run the level-by-level kernel and
    // k_orb_blur
    if (fused) {
      hipLaunchKernelGGL(k_orb_pyramid, dim3(n), dim3(kPyrThreads), 0, st, a);
    } else {
      for (int l = 0; l < kL; l++)
        hipLaunchKernelGGL(k_orb_level, dim3(cdiv(g.stride[l] * (g.h[l] + 2 * kB), 256 * kLevelPx), n), dim3(256), 0,
                           st, a, l, 0);
    }
  }
  {
    TimedScope t(c, kT_orb_fast);
    const size_t lds = fast_lds_bytes(g.stride[0], g.w[0]);
    hipLaunchKernelGGL(k_orb_fastnms, dim3(g.fband[kL], n), dim3(256), lds, st, a);
  }
  if (fused) {  // the border rows of both pyramids and the blurred copy's rows
    TimedScope t(c, kT_orb_roiblur);
    hipLaunchKernelGGL(k_orb_roiblur, dim3(g.rband[kL], n), dim3(256), (size_t)(kRoiBand + 6) * g.stride[0], st, a);
  }
  { TimedScope t(c, kT_orb_select); hipLaunchKernelGGL(k_orb_select, dim3(n * kL), dim3(kSelThreads), 0, st, a); }
  { TimedScope t(c, kT_orb_finish); hipLaunchKernelGGL(k_orb_finish, dim3(n), dim3(256), 0, st, a); }
  if (!fused) {
    TimedScope t(c, kT_orb_blur);
    hipLaunchKernelGGL(k_orb_blur, dim3(g.bband[kL], n), dim3(256), (size_t)(kBlurBand + 6) * g.stride[0], st, a);
  }
  { TimedScope t(c, kT_orb_desc); hipLaunchKernelGGL(k_orb_desc, dim3(cdiv(g.cap, kDescChunk), n), dim3(256), 0, st, a); }
  OCHK(c, hipGetLastError());
  return LISLAM_OK;
}

// a8 + a9 of engine e (2n features) for the scans of a device list (dlist, *dcount of them, at most
// nmax), reading the pyramid, FAST / NMS scores and blurred pyramid that engine src (n features)
// built for the same scans: those depend only on the image and the mask, not on the feature
// budget, so a re-detection is retainBest + Harris / angles (k_orb_select), the level
// concatenation (k_orb_finish) and the descriptors (k_orb_desc).
constexpr int kListSlots = 16;  // grid slots of a device-list launch (scans or pairs in use: a few)

int engine_select_from(OrbEngine* e, const OrbEngine* src, const uint8_t* d_img, const float4* d_track,
                       const int* dlist, const int* dcount, int nmax) {
  lislam_ctx* c = e->ctx;
  hipStream_t st = c->stream;
  if (nmax <= 0) return LISLAM_OK;
  Args a = e->args(d_img, d_track);
  a.S = nmax;
  a.smap = dlist;
  a.scount = dcount;
  a.pyr = src->pyr;
  a.blur = src->blur;
  a.nms = src->nms;
  const Geom& g = e->g;
  // kListSlots grid scan indices stride over the list: the count is only known on the device
  const int ns = std::min(nmax, kListSlots);
  { TimedScope t(c, kT_orb_select); hipLaunchKernelGGL(k_orb_select_list, dim3(ns * kL), dim3(kSelThreads), 0, st, a); }
  { TimedScope t(c, kT_orb_finish); hipLaunchKernelGGL(k_orb_finish, dim3(ns), dim3(256), 0, st, a); }
  { TimedScope t(c, kT_orb_desc); hipLaunchKernelGGL(k_orb_desc, dim3(cdiv(g.cap, kDescChunk), ns), dim3(256), 0, st, a); }
  OCHK(c, hipGetLastError());
  return LISLAM_OK;
}

// Device buffers of up to `maxp` scan pairs with queries of up to qcap keypoints.
struct PairBufs {
  lislam_ctx* ctx = nullptr;
  int maxp = 0, qcap = 0;
  std::vector<void*> allocs;
  int *args = nullptr;  // [3][maxp] staged per launch: query scans, train scans, slots
  int *mscratch = nullptr, *mout = nullptr, *kind = nullptr, *stats = nullptr, *redet = nullptr, *arrive = nullptr;
  int* tail_arrive = nullptr;  // k_orb_lm's workgroup counter for its tail (0 between launches)
  double *rec = nullptr, *T = nullptr;
  ~PairBufs() {
    for (void* p : allocs) (void)hipFree(p);
  }
  template <typename T_>
  int alloc(T_** p, size_t count) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T_));
    if (e != hipSuccess) return ofail(ctx, LISLAM_ERR_DEVICE, "hipMalloc(%zu): %s", count * sizeof(T_), hipGetErrorString(e));
    allocs.push_back(q);
    *p = static_cast<T_*>(q);
    return LISLAM_OK;
  }
  int init(lislam_ctx* c, int maxp_, int qcap_, bool raw) {
    ctx = c; maxp = maxp_; qcap = qcap_;
    ORC(alloc(&args, (size_t)3 * maxp));
    ORC(alloc(&redet, maxp));
    ORC(alloc(&mscratch, (size_t)maxp * qcap));
    // the best[] rows start at the "no match" sentinel; k_orb_match puts back each row it consumed
    if (hipMemset(mscratch, 0x7f, (size_t)maxp * qcap * sizeof(int)) != hipSuccess)
      return ofail(ctx, LISLAM_ERR_DEVICE, "hipMemset of the match rows failed");
    ORC(alloc(&arrive, maxp + 1));  // k_orb_pairs' arrival counters and k_orb_lm's, 0 between launches
    tail_arrive = arrive + maxp;
    if (hipMemset(arrive, 0, (size_t)(maxp + 1) * sizeof(int)) != hipSuccess)
      return ofail(ctx, LISLAM_ERR_DEVICE, "hipMemset of the pair arrival counters failed");
    if (raw) ORC(alloc(&mout, (size_t)maxp * qcap * 3));
    ORC(alloc(&kind, (size_t)maxp * qcap));
    ORC(alloc(&stats, (size_t)maxp * 8));
    ORC(alloc(&rec, (size_t)maxp * qcap * 9));
    ORC(alloc(&T, (size_t)maxp * 7));
    return LISLAM_OK;
  }
};

// Match pairs (query scan qs[i] of engine qe, train scan ts[i] of te), select frac, test, and
// (lm) solve; pair i writes buffer slot slots[i] (null: p0 + i).
// dlist / dcount: the lists are already on the device (dlist = [3][n] query scans | train scans |
// slots, dcount = how many are in use; n is the grid's upper bound and the lists' stride), decided
// by an earlier kernel.
// tail (with lm): what the stream runs next — the cascade decision or the batch outputs — run by
// the solve launch's last workgroup instead of a launch of its own.
int run_pairs(lislam_ctx* c, const OrbEngine* qe, const OrbEngine* te, const int* qs, const int* ts, int n, double frac,
              PairBufs& pb, int p0, bool lm, const int* slots = nullptr, const int* dlist = nullptr,
              const int* dcount = nullptr, const LmTail* tail = nullptr) {
  hipStream_t st = c->stream;
  LmTail tl;
  if (tail) {
    tl = *tail;
    tl.arrive = pb.tail_arrive;
  }
  if (n <= 0) {
    if (tl.kind) hipLaunchKernelGGL(k_orb_tail, dim3(1), dim3(256), 0, st, tl);
    OCHK(c, hipGetLastError());
    return LISLAM_OK;
  }
  if (qe->g.cap > pb.qcap || (!slots && !dlist && p0 + n > pb.maxp) || n > pb.maxp)
    return ofail(c, LISLAM_ERR_CAPACITY, "pair buffers too small");
  PairArgs p;
  p.npairs = n;
  p.pcount = dcount;
  if (dlist) {
    p.qscan = dlist; p.tscan = dlist + n; p.pslot = dlist + 2 * n;
  } else {
    // one upload of the launch's lists: query scans | train scans | slots (stream-ordered after
    // the previous launch's kernels, which read the same staging area)
    std::vector<int> host((size_t)3 * n);
    std::copy(qs, qs + n, host.begin());
    std::copy(ts, ts + n, host.begin() + n);
    if (slots) std::copy(slots, slots + n, host.begin() + 2 * n);
    OCHK(c, hipMemcpyAsync(pb.args, host.data(), (size_t)(slots ? 3 : 2) * n * 4, hipMemcpyHostToDevice, st));
    p.pslot = slots ? pb.args + 2 * n : nullptr;
    p.qscan = pb.args; p.tscan = pb.args + n;
  }
  p.qdesc = qe->desc; p.tdesc = te->desc;
  p.qp3d = qe->p3d; p.tp3d = te->p3d;
  p.qn = qe->nkp; p.tn = te->nkp;
  p.qcap = qe->g.cap; p.tcap = te->g.cap;
  p.bstride = pb.qcap;
  p.frac = frac;
  const int b0 = (slots || dlist) ? 0 : p0;  // buffer base (slots index from buffer 0)
  const int gp = dlist ? std::min(n, kListSlots) : n;  // grid pair slots (device lists: strided)
  p.mscratch = pb.mscratch + (size_t)b0 * pb.qcap;
  p.mout = pb.mout ? pb.mout + (size_t)b0 * pb.qcap * 3 : nullptr;
  p.rec = pb.rec + (size_t)b0 * pb.qcap * 9;
  p.kind = pb.kind + (size_t)b0 * pb.qcap;
  p.stats = pb.stats + b0 * 8;
  p.T = pb.T + b0 * 7;
  p.arrive = pb.arrive + b0;
  {
    // one launch (k_orb_pairs); LISLAM_ORB_PAIR_SPLIT=1: the distance and selection kernels one
    // after the other (A/B)
    static const bool split = getenv("LISLAM_ORB_PAIR_SPLIT") && atoi(getenv("LISLAM_ORB_PAIR_SPLIT")) == 1;
    TimedScope t(c, kT_orb_match);
    if (!split) {
      hipLaunchKernelGGL(k_orb_pairs, dim3(gp, cdiv(te->g.cap, kXmTrains)), dim3(64 * kXmWaves), 0, st, p);
    } else {
      hipLaunchKernelGGL(k_orb_xdist_mfma, dim3(gp, cdiv(te->g.cap, kXmTrains)), dim3(64 * kXmWaves), 0, st, p);
      hipLaunchKernelGGL(k_orb_match, dim3(gp), dim3(kPairThreads), 0, st, p);
    }
  }
  if (lm) {
    TimedScope t(c, kT_orb_lm);
    hipLaunchKernelGGL(k_orb_lm, dim3(gp), dim3(kLmThreads), 0, st, p, 20, tl);
  } else if (tl.kind) {
    hipLaunchKernelGGL(k_orb_tail, dim3(1), dim3(256), 0, st, tl);
  }
  OCHK(c, hipGetLastError());
  return LISLAM_OK;
}

}  // namespace

// ---------------------------------------------------------------- batch intensity odometry
struct OrbBatch {
  lislam_ctx* ctx = nullptr;
  int nfeatures = 0;
  bool has_mask = false;
  OrbEngine* e1 = nullptr;
  OrbEngine* e2 = nullptr;  // 2 * nfeatures, re-detection
  PairBufs pb;
  std::vector<void*> allocs;
  double* outT = nullptr;   // [S][7]
  int* outS = nullptr;      // [S][8]
  // The batch front end runs on the context stream: the split chain engine queues nothing there, so
  // the ORB kernels still overlap the chain, and a context holds one hardware queue, not two (past
  // ~20 CU-masked queues per process every launch slows; six pipelined contexts used to hold twelve
  // here).  LISLAM_ORB_SIDE_STREAM=1: a stream of the batch's own, ordered only after the a1 images.
  hipStream_t side = nullptr;
  hipStream_t st(const lislam_ctx* c) const { return side ? side : c->stream; }
  hipEvent_t done = nullptr;
  // the device-decided re-detection cascade (k_orb_decide): state, lists, and its verdict copied
  // to pinned host memory; `pending` until a reader of the outputs has checked it
  CascadeArgs cs{};
  int* h_status = nullptr;   // pinned [2]
  hipEvent_t settled = nullptr;
  bool pending = false;
  int pending_n = 0;
  int info[2] = {-1, 0};     // lislam_batch_orb_cascade_info
  ~OrbBatch() {
    if (side) (void)hipStreamSynchronize(side);
    if (side) destroy_stream(side);
    if (done) (void)hipEventDestroy(done);
    if (settled) (void)hipEventDestroy(settled);
    if (h_status) (void)hipHostFree(h_status);
    delete e1;
    delete e2;
    for (void* p : allocs) (void)hipFree(p);
  }
};

void lislam_free_orb(void* p) { delete static_cast<OrbBatch*>(p); }

namespace {

int orb_batch_get(lislam_batch* b, int nfeatures, const uint8_t* mask, OrbBatch** out) {
  lislam_ctx* c = b->ctx;
  OrbBatch* ob = static_cast<OrbBatch*>(b->orb);
  if (ob && (ob->nfeatures != nfeatures || ob->has_mask != (mask != nullptr))) {
    (void)hipStreamSynchronize(c->stream);
    delete ob;
    ob = nullptr;
    b->orb = nullptr;
  }
  if (!ob) {
    ob = new OrbBatch();
    b->orb = ob;
    ob->ctx = c;
    ob->nfeatures = nfeatures;
    ob->has_mask = mask != nullptr;
    ob->e1 = new OrbEngine();
    ob->e2 = new OrbEngine();
    static const bool own_side = getenv("LISLAM_ORB_SIDE_STREAM") && atoi(getenv("LISLAM_ORB_SIDE_STREAM")) == 1;
    if (own_side && !work_stream(c->device, &ob->side)) return ofail(c, LISLAM_ERR_DEVICE, "ORB stream");
    OCHK(c, hipEventCreateWithFlags(&ob->done, hipEventDisableTiming));
    // the engines' tables and mask pyramids are uploaded / built on the side stream, where the
    // front end that reads them runs
    struct StreamSwap {
      lislam_ctx* c;
      hipStream_t keep;
      ~StreamSwap() { c->stream = keep; }
    } swap{c, c->stream};
    c->stream = ob->st(c);
    ORC(engine_init(ob->e1, c, b->H, b->W, b->max_scans, nfeatures, mask));
    ORC(engine_init(ob->e2, c, b->H, b->W, b->max_scans, 2 * nfeatures, mask));
    ORC(ob->pb.init(c, b->max_scans, std::max(ob->e1->g.cap, ob->e2->g.cap), false));
    void* q = nullptr;
    OCHK(c, hipMalloc(&q, (size_t)b->max_scans * 7 * 8));
    ob->allocs.push_back(q);
    ob->outT = static_cast<double*>(q);
    OCHK(c, hipMalloc(&q, (size_t)b->max_scans * 8 * 4));
    ob->allocs.push_back(q);
    ob->outS = static_cast<int*>(q);
    const size_t S = (size_t)b->max_scans;
    CascadeArgs& cs = ob->cs;
    OCHK(c, hipMalloc(&q, S * 3 + 64));
    ob->allocs.push_back(q);
    cs.pset = static_cast<int8_t*>(q); cs.cur2 = cs.pset + S; cs.have2 = cs.pset + 2 * S;
    OCHK(c, hipMalloc(&q, (S * 8 + 8) * 4));
    ob->allocs.push_back(q);
    int* qi = static_cast<int*>(q);
    cs.e2list = qi; cs.plist = qi + S; cs.redet = qi + 7 * S; cs.e2cnt = qi + 8 * S; cs.pcnt = qi + 8 * S + 2;
    cs.status = qi + 8 * S + 4;
    OCHK(c, hipHostMalloc((void**)&ob->h_status, 2 * sizeof(int), hipHostMallocDefault));
    OCHK(c, hipEventCreateWithFlags(&ob->settled, hipEventDisableTiming));
  }
  *out = ob;
  return LISLAM_OK;
}

}  // namespace


namespace {

// Body of lislam_batch_intensity_odometry; runs with c->stream switched to the batch's ORB stream
// (OrbBatch::st: the context stream unless LISLAM_ORB_SIDE_STREAM=1).
int batch_intensity_odometry(lislam_batch* b, OrbBatch* ob, int n_scans) {
  lislam_ctx* c = b->ctx;
  hipStream_t st = c->stream;
  const uint8_t* img = b->fa.img_int;
  const float4* trk = reinterpret_cast<const float4*>(b->fa.track);
  ORC(engine_detect_slots(ob->e1, img, trk, 0, n_scans));
  const int np = n_scans - 1;
  std::vector<int> qs(std::max(np, 1)), ts(std::max(np, 1));
  for (int k = 1; k < n_scans; k++) { qs[k - 1] = k; ts[k - 1] = k - 1; }
  ORC(run_pairs(c, ob->e1, ob->e1, qs.data(), ts.data(), np, 0.3, ob->pb, 0, true));
  std::vector<int> hs((size_t)std::max(np, 1) * 8);
  if (np > 0) OCHK(c, hipMemcpyAsync(hs.data(), ob->pb.stats, (size_t)np * 8 * 4, hipMemcpyDeviceToHost, st));
  OCHK(c, hipStreamSynchronize(st));
  // The sequential rule of detectfeatures: pair k re-detects both frames (2 * nfeatures, 20 %)
  // when its first attempt fails, and frame k then keeps the 2n set, against which pair k+1's
  // first attempt is made.  Resolved as a fixed point in batched rounds: cur2[k] follows from the
  // first attempt of pair k made against the right previous set (pset[k] == cur2[k-1]); pairs whose
  // attempt used the wrong set are redone together; finally every re-detecting pair is matched
  // 2n-against-2n in one batch.
  std::vector<int> pset(n_scans, 0), cur2(n_scans, 0), ok1(n_scans, 1);
  std::vector<char> have2(n_scans, 0);
  for (int k = 1; k < n_scans; k++) ok1[k] = hs[(size_t)(k - 1) * 8] == 1;
  auto detect2 = [&](std::vector<int> need) -> int {  // 2n detection of scans not done yet
    std::vector<int> todo;
    for (int sc : need)
      if (!have2[sc]) { have2[sc] = 1; todo.push_back(sc); }
    std::sort(todo.begin(), todo.end());
    todo.erase(std::unique(todo.begin(), todo.end()), todo.end());
    if (!todo.empty()) ORC(engine_detect_slots(ob->e2, img, trk, 0, (int)todo.size(), todo.data()));
    return LISLAM_OK;
  };
  for (int round = 0; round < n_scans; round++) {
    for (int k = 1; k < n_scans; k++) cur2[k] = (pset[k] == cur2[k - 1]) ? !ok1[k] : cur2[k];
    std::vector<int> dirty[2];
    for (int k = 1; k < n_scans; k++)
      if (pset[k] != cur2[k - 1]) dirty[cur2[k - 1]].push_back(k);
    if (dirty[0].empty() && dirty[1].empty()) break;
    std::vector<int> need;
    for (int k : dirty[1]) need.push_back(k - 1);
    ORC(detect2(need));
    for (int g2 = 0; g2 < 2; g2++) {
      const std::vector<int>& d = dirty[g2];
      if (d.empty()) continue;
      std::vector<int> q, t, sl;
      for (int k : d) { q.push_back(k); t.push_back(k - 1); sl.push_back(k - 1); pset[k] = g2; }
      ORC(run_pairs(c, ob->e1, g2 ? ob->e2 : ob->e1, q.data(), t.data(), (int)d.size(), 0.3, ob->pb, 0, true, sl.data()));
    }
    OCHK(c, hipMemcpyAsync(hs.data(), ob->pb.stats, (size_t)np * 8 * 4, hipMemcpyDeviceToHost, st));
    OCHK(c, hipStreamSynchronize(st));
    for (int g2 = 0; g2 < 2; g2++)
      for (int k : dirty[g2]) ok1[k] = hs[(size_t)(k - 1) * 8] == 1;
  }
  std::vector<int> redet, flag(std::max(np, 1), 0);
  for (int k = 1; k < n_scans; k++)
    if (cur2[k]) { redet.push_back(k); flag[k - 1] = 1; }
  if (!redet.empty()) {
    std::vector<int> need, q, t, sl;
    for (int k : redet) { need.push_back(k - 1); need.push_back(k); q.push_back(k); t.push_back(k - 1); sl.push_back(k - 1); }
    ORC(detect2(need));
    ORC(run_pairs(c, ob->e2, ob->e2, q.data(), t.data(), (int)redet.size(), 0.2, ob->pb, 0, true, sl.data()));
  }
  // outputs: scan 0 = first frame; scan k = pair (k-1, k), whose final attempt sits in slot k-1
  OCHK(c, hipMemcpyAsync(ob->pb.redet, flag.data(), (size_t)std::max(np, 1) * 4, hipMemcpyHostToDevice, st));
  const OutArgs oa{ob->outS, ob->outT, ob->pb.stats, ob->pb.T, ob->pb.redet, ob->e1->nkp, n_scans};
  hipLaunchKernelGGL(k_orb_out, dim3(cdiv(n_scans, 256)), dim3(256), 0, st, oa);
  OCHK(c, hipGetLastError());
  OCHK(c, hipStreamSynchronize(st));
  return LISLAM_OK;
}

// The same cascade with every decision on the device: no host synchronization.  The first
// attempts of all pairs, then `rounds` passes of (re-detections the last decision listed, the
// re-attempts, decision), then the final 2n-against-2n matches.  After the first attempts every
// pair to redo follows a failed pair, so pass 0 only re-attempts against 2n sets; later passes
// (a re-attempt that failed again, flipping the next pair's previous set) need both groups.  One
// pass resolves the bench sequence (its re-detections are isolated); a sequence whose re-attempts
// flip further ends "not converged", and orb_settle redoes the batch with host rounds
// (batch_intensity_odometry) before anything reads it.  LISLAM_ORB_ROUNDS sets the passes
// (default 1).
int cascade_rounds() {
  const char* e = getenv("LISLAM_ORB_ROUNDS");
  const int r = e ? atoi(e) : 1;
  return r < 1 ? 1 : r > 64 ? 64 : r;
}

int batch_intensity_odometry_dev(lislam_batch* b, OrbBatch* ob, int n_scans) {
  lislam_ctx* c = b->ctx;
  hipStream_t st = c->stream;
  const uint8_t* img = b->fa.img_int;
  const float4* trk = reinterpret_cast<const float4*>(b->fa.track);
  ORC(engine_detect_slots(ob->e1, img, trk, 0, n_scans));
  const int np = n_scans - 1;
  std::vector<int> qs(np), ts(np);
  for (int k = 1; k < n_scans; k++) { qs[k - 1] = k; ts[k - 1] = k - 1; }
  CascadeArgs cs = ob->cs;
  cs.n = n_scans;
  cs.stats = ob->pb.stats;
  // each decision (k_orb_decide) and the outputs (k_orb_out) run in the last workgroup of the
  // solve launch before them (LmTail)
  LmTail tl;
  tl.kind = 1;
  tl.mode = 0;
  tl.cs = cs;
  ORC(run_pairs(c, ob->e1, ob->e1, qs.data(), ts.data(), np, 0.3, ob->pb, 0, true, nullptr, nullptr, nullptr, &tl));
  const int rounds = cascade_rounds();
  for (int r = 0; r < rounds; r++) {
    ORC(engine_select_from(ob->e2, ob->e1, img, trk, cs.e2list, cs.e2cnt, n_scans));
    tl.mode = r + 1 < rounds ? 1 : 2;
    for (int g2 = r == 0 ? 1 : 0; g2 < 2; g2++)
      ORC(run_pairs(c, ob->e1, g2 ? ob->e2 : ob->e1, nullptr, nullptr, n_scans, 0.3, ob->pb, 0, true, nullptr,
                    cs.plist + (size_t)g2 * 3 * n_scans, cs.pcnt + g2, g2 == 1 ? &tl : nullptr));
  }
  ORC(engine_select_from(ob->e2, ob->e1, img, trk, cs.e2list, cs.e2cnt, n_scans));
  tl.kind = 2;
  tl.out = OutArgs{ob->outS, ob->outT, ob->pb.stats, ob->pb.T, cs.redet, ob->e1->nkp, n_scans};
  ORC(run_pairs(c, ob->e2, ob->e2, nullptr, nullptr, n_scans, 0.2, ob->pb, 0, true, nullptr, cs.plist, cs.pcnt, &tl));
  OCHK(c, hipGetLastError());
  OCHK(c, hipMemcpyAsync(ob->h_status, cs.status, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
  OCHK(c, hipEventRecord(ob->settled, st));
  ob->pending = true;
  ob->pending_n = n_scans;
  return LISLAM_OK;
}

}  // namespace

// Before the outputs of a device-decided cascade are read, and before lislam_batch_extract
// overwrites the images it read: wait for its verdict (the reader synchronizes anyway) and, if it
// did not converge in LISLAM_ORB_ROUNDS passes, redo the batch with host rounds from the same
// images (the redo finishes before this returns).
int orb_settle(lislam_batch* b) {
  OrbBatch* ob = static_cast<OrbBatch*>(b->orb);
  if (!ob || !ob->pending) return LISLAM_OK;
  lislam_ctx* c = b->ctx;
  OCHK(c, hipEventSynchronize(ob->settled));
  ob->pending = false;
  ob->info[0] = ob->h_status[0];
  ob->info[1] = ob->h_status[1];
  if (ob->h_status[0] == 1) return LISLAM_OK;
  const hipStream_t main_stream = c->stream;
  const hipStream_t side = ob->st(c);
  if (side != main_stream) OCHK(c, hipStreamWaitEvent(side, b->ev_images, 0));
  c->stream = side;
  const int rc = batch_intensity_odometry(b, ob, ob->pending_n);
  c->stream = main_stream;
  return rc;
}

extern "C" {

// The ORB front end of every scan pair.  It is queued on the context stream, after the last
// lislam_batch_extract (with LISLAM_ORB_SIDE_STREAM=1 on a stream of the batch's own, ordered only
// after that extract's images); the split chain engine the caller may already have queued runs on
// the device's engine streams, so the two overlap.  On return the context stream is ordered after
// all of its work.
int lislam_batch_intensity_odometry(lislam_batch* b, int32_t n_scans, int32_t nfeatures, const uint8_t* mask) {
  if (!b || n_scans < 1 || n_scans > b->max_scans || nfeatures < 1 || nfeatures > 16384) return LISLAM_ERR_ARG;
  lislam_ctx* c = b->ctx;
  if (!b->fa.img_int || !b->fa.track)
    return ofail(c, LISLAM_ERR_STATE, "lislam_batch_intensity_odometry needs want_images (the a1 images)");
  if (b->extracted < n_scans) return ofail(c, LISLAM_ERR_STATE, "extract %d scans before intensity odometry", n_scans);
  hipSetDevice(c->device);
  OrbBatch* ob = nullptr;
  ORC(orb_batch_get(b, nfeatures, mask, &ob));
  const hipStream_t main_stream = c->stream;
  const hipStream_t side = ob->st(c);
  if (side != main_stream) OCHK(c, hipStreamWaitEvent(side, b->ev_images, 0));
  c->stream = side;
  ob->pending = false;  // a newer batch replaces results nobody read
  ob->info[0] = -1;
  ob->info[1] = 0;
  const int rc = (n_scans < 2 || n_scans > kCascadeMax) ? batch_intensity_odometry(b, ob, n_scans)
                                                                               : batch_intensity_odometry_dev(b, ob, n_scans);
  c->stream = main_stream;
  if (side != main_stream) {
    OCHK(c, hipEventRecord(ob->done, side));
    OCHK(c, hipStreamWaitEvent(main_stream, ob->done, 0));
  }
  return rc;
}

}  // extern "C"

// ---------------------------------------------------------------- single frame drop-in
struct lislam_intensity_tracker {
  lislam_ctx* ctx = nullptr;
  int H = 0, W = 0, nfeatures = 0;
  OrbEngine e1, e2;
  PairBufs pb;
  uint8_t* img = nullptr;   // [2][H*W]
  float4* trk = nullptr;    // [2][H*W]
  int cur = 0;
  bool have_prev = false, prev2 = false;
};

extern "C" {

int lislam_intensity_tracker_create(lislam_ctx* c, int32_t H, int32_t W, int32_t nfeatures, const uint8_t* mask,
                                    lislam_intensity_tracker** out) {
  if (!c || !out || H < 8 || W < 8 || nfeatures < 1 || nfeatures > 16384) return LISLAM_ERR_ARG;
  *out = nullptr;
  hipSetDevice(c->device);
  lislam_intensity_tracker* t = new lislam_intensity_tracker();
  t->ctx = c; t->H = H; t->W = W; t->nfeatures = nfeatures;
  int rc = engine_init(&t->e1, c, H, W, 2, nfeatures, mask);
  if (!rc) rc = engine_init(&t->e2, c, H, W, 2, 2 * nfeatures, mask);
  if (!rc) rc = t->pb.init(c, 1, std::max(t->e1.g.cap, t->e2.g.cap), false);
  if (!rc) rc = t->e1.alloc(&t->img, (size_t)2 * H * W);
  if (!rc) rc = t->e1.alloc(&t->trk, (size_t)2 * H * W);
  if (rc) { delete t; return rc; }
  *out = t;
  return LISLAM_OK;
}

int lislam_intensity_tracker_destroy(lislam_intensity_tracker* t) {
  if (!t) return LISLAM_OK;
  hipSetDevice(t->ctx->device);
  (void)hipStreamSynchronize(t->ctx->stream);
  delete t;
  return LISLAM_OK;
}

int lislam_intensity_tracker_step(lislam_intensity_tracker* t, const uint8_t* image, const float* cloud_track,
                                  double* T_out, int32_t* stats_out) {
  if (!t || !image || !cloud_track) return LISLAM_ERR_ARG;
  lislam_ctx* c = t->ctx;
  hipSetDevice(c->device);
  hipStream_t st = c->stream;
  const size_t N = (size_t)t->H * t->W;
  const int cs = t->cur, ps = 1 - t->cur;
  OCHK(c, hipMemcpyAsync(t->img + cs * N, image, N, hipMemcpyDefault, st));
  OCHK(c, hipMemcpyAsync(t->trk + cs * N, cloud_track, N * 16, hipMemcpyDefault, st));
  ORC(engine_detect_slots(&t->e1, t->img, t->trk, cs, 1));
  int h8[8] = {-1, 0, 0, 0, 0, 0, 0, 0};
  double T[7] = {0, 0, 0, 1, 0, 0, 0};
  bool cur2 = false;
  if (!t->have_prev) {
    OCHK(c, hipMemcpyAsync(&h8[2], t->e1.nkp + cs, 4, hipMemcpyDeviceToHost, st));
    OCHK(c, hipStreamSynchronize(st));
  } else {
    ORC(run_pairs(c, &t->e1, t->prev2 ? &t->e2 : &t->e1, &cs, &ps, 1, 0.3, t->pb, 0, true));
    OCHK(c, hipMemcpyAsync(h8, t->pb.stats, 32, hipMemcpyDeviceToHost, st));
    OCHK(c, hipStreamSynchronize(st));
    if (h8[0] != 1) {  // re-detect both frames with 2 * nfeatures (intensity_feature_tracker.cpp:652-687)
      ORC(engine_detect_slots(&t->e2, t->img, t->trk, cs, 1));
      if (!t->prev2) ORC(engine_detect_slots(&t->e2, t->img, t->trk, ps, 1));
      ORC(run_pairs(c, &t->e2, &t->e2, &cs, &ps, 1, 0.2, t->pb, 0, true));
      OCHK(c, hipMemcpyAsync(h8, t->pb.stats, 32, hipMemcpyDeviceToHost, st));
      OCHK(c, hipStreamSynchronize(st));
      h8[1] = 1;
      cur2 = true;
    }
    OCHK(c, hipMemcpyAsync(T, t->pb.T, 56, hipMemcpyDeviceToHost, st));
    OCHK(c, hipStreamSynchronize(st));
  }
  t->have_prev = true;
  t->prev2 = cur2;
  t->cur = ps;
  if (T_out) std::memcpy(T_out, T, 56);
  if (stats_out) std::memcpy(stats_out, h8, 32);
  return LISLAM_OK;
}

// ---------------------------------------------------------------- building blocks
int lislam_orb_detect(lislam_ctx* c, const uint8_t* image, const float* cloud_track, const uint8_t* mask, int32_t H,
                      int32_t W, int32_t nfeatures, float* kp, uint8_t* desc, float* p3d, int32_t cap, int32_t* n) {
  if (!c || !image || !cloud_track || !n || H < 8 || W < 8 || nfeatures < 1 || nfeatures > 16384) return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  hipStream_t st = c->stream;
  OrbEngine e;
  ORC(engine_init(&e, c, H, W, 1, nfeatures, mask));
  uint8_t* dimg = nullptr;
  float4* dtrk = nullptr;
  ORC(e.alloc(&dimg, (size_t)H * W));
  ORC(e.alloc(&dtrk, (size_t)H * W));
  OCHK(c, hipMemcpyAsync(dimg, image, (size_t)H * W, hipMemcpyDefault, st));
  OCHK(c, hipMemcpyAsync(dtrk, cloud_track, (size_t)H * W * 16, hipMemcpyDefault, st));
  ORC(engine_detect_slots(&e, dimg, dtrk, 0, 1));
  int cnt = 0, ovf = 0;
  OCHK(c, hipMemcpyAsync(&cnt, e.nkp, 4, hipMemcpyDeviceToHost, st));
  OCHK(c, hipMemcpyAsync(&ovf, e.overflow, 4, hipMemcpyDeviceToHost, st));
  OCHK(c, hipStreamSynchronize(st));
  *n = cnt;
  if (ovf) return ofail(c, LISLAM_ERR_CAPACITY, "ORB level keypoint capacity exceeded");
  if (cnt > cap) return ofail(c, LISLAM_ERR_CAPACITY, "lislam_orb_detect: %d keypoints > cap %d", cnt, cap);
  if (kp) OCHK(c, hipMemcpyAsync(kp, e.kp, (size_t)cnt * 24, hipMemcpyDefault, st));
  if (desc) OCHK(c, hipMemcpyAsync(desc, e.desc, (size_t)cnt * 32, hipMemcpyDefault, st));
  if (p3d) OCHK(c, hipMemcpyAsync(p3d, e.p3d, (size_t)cnt * 16, hipMemcpyDefault, st));
  OCHK(c, hipStreamSynchronize(st));
  return LISLAM_OK;
}

int lislam_orb_match(lislam_ctx* c, const uint8_t* qdesc, int32_t nq, const uint8_t* tdesc, int32_t nt, int32_t* matches,
                     int32_t* n_matches) {
  if (!c || nq < 0 || nt < 0 || nq > 65535 || nt > 65535 || !n_matches || (nq && !qdesc) || (nt && !tdesc))
    return LISLAM_ERR_ARG;
  hipSetDevice(c->device);
  hipStream_t st = c->stream;
  // a minimal engine-shaped view: descriptors with cap = max(nq, nt, 1) per "scan"
  OrbEngine e;
  e.ctx = c;
  const int cap = std::max(std::max(nq, nt), 1);
  e.g.cap = cap;
  ORC(e.alloc(&e.desc, (size_t)2 * cap * 32));
  ORC(e.alloc(&e.p3d, (size_t)2 * cap));
  ORC(e.alloc(&e.nkp, 2));
  const int cnts[2] = {nq, nt};
  OCHK(c, hipMemcpyAsync(e.nkp, cnts, 8, hipMemcpyHostToDevice, st));
  OCHK(c, hipMemsetAsync(e.p3d, 0, (size_t)2 * cap * 16, st));
  if (nq) OCHK(c, hipMemcpyAsync(e.desc, qdesc, (size_t)nq * 32, hipMemcpyDefault, st));
  if (nt) OCHK(c, hipMemcpyAsync(e.desc + (size_t)cap * 32, tdesc, (size_t)nt * 32, hipMemcpyDefault, st));
  PairBufs pb;
  ORC(pb.init(c, 1, cap, true));
  const int q = 0, t = 1;
  ORC(run_pairs(c, &e, &e, &q, &t, 1, 0.3, pb, 0, false));
  int h8[8];
  OCHK(c, hipMemcpyAsync(h8, pb.stats, 32, hipMemcpyDeviceToHost, st));
  OCHK(c, hipStreamSynchronize(st));
  *n_matches = h8[3];
  if (matches && h8[3]) OCHK(c, hipMemcpyAsync(matches, pb.mout, (size_t)h8[3] * 12, hipMemcpyDefault, st));
  OCHK(c, hipStreamSynchronize(st));
  return LISLAM_OK;
}

}  // extern "C"

// Outputs of lislam_batch_intensity_odometry for lislam_batch_download.
extern "C" int lislam_batch_orb_cascade_info(lislam_batch* b, int32_t* info) {
  if (!b || !info) return LISLAM_ERR_ARG;
  OrbBatch* ob = static_cast<OrbBatch*>(b->orb);
  if (!ob) return LISLAM_ERR_STATE;
  ORC(orb_settle(b));
  info[0] = ob->info[0];
  info[1] = ob->info[1];
  return LISLAM_OK;
}

int lislam_orb_batch_output(lislam_batch* b, int what, int scan, const void** src, int* cnt, size_t* esz) {
  OrbBatch* ob = static_cast<OrbBatch*>(b->orb);
  if (!ob) return LISLAM_ERR_STATE;
  ORC(orb_settle(b));
  const Geom& g = ob->e1->g;
  switch (what) {
    case LISLAM_OUT_ORB_T: *src = ob->outT + (size_t)scan * 7; *cnt = 7; *esz = 8; return LISLAM_OK;
    case LISLAM_OUT_ORB_STATS: *src = ob->outS + (size_t)scan * 8; *cnt = 8; *esz = 4; return LISLAM_OK;
    case LISLAM_OUT_ORB_KEYPOINTS:
    case LISLAM_OUT_ORB_POINTS:
    case LISLAM_OUT_ORB_DESCRIPTORS: {
      int n = 0;
      hipStream_t st = b->ctx->stream;
      if (hipMemcpyAsync(&n, ob->e1->nkp + scan, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        return LISLAM_ERR_DEVICE;
      *cnt = n;
      if (what == LISLAM_OUT_ORB_KEYPOINTS) { *src = ob->e1->kp + (size_t)scan * g.cap * 6; *esz = 24; }
      else if (what == LISLAM_OUT_ORB_POINTS) { *src = ob->e1->p3d + (size_t)scan * g.cap; *esz = 16; }
      else { *src = ob->e1->desc + (size_t)scan * g.cap * 32; *esz = 32; }
      return LISLAM_OK;
    }
  }
  return LISLAM_ERR_ARG;
}
