// lislam feature front end on gfx950: ImageHandler::cloud_handler + scanRegistration's
// laserCloudHandler (a1..a7 of SURVEY.md §8(a)) for a batch of S organized scans resident in HBM.
//
//   k_front_count / k_front_scan / k_front_scatter ("k_scan_front" in the timers): one wave per
//                  1024-point range streams the ring-ordered xyzI buffer with 16-B coalesced
//                  loads, twice:
//                    count:   range/intensity images + cloud_track (image_handler.h_ouster:112-139),
//                             close-point filter (scanRegistration.cpp:152-186), per-range scan
//                             line histogram (:285-331) and the first index where halfPassed flips
//                             (:336-353) — the loop's only sequential state is a monotone flag, so
//                             it reduces to "first index where";
//                    scan:    per scan, line offsets, per-range write bases, the scan's flip index;
//                    scatter: ori/relTime/intensity (:334-371) and the stable counting sort by
//                             scanID (= the per-line push_back + concatenation, :373-394) using
//                             64-lane ballot peer masks for in-wave ranks.
//   k_scan_lines   one wave per (scan, line): curvature (:397-412), per-segment bitonic sort of
//                  (curvature, index) keys in LDS (:445), the sharp / flat greedy walks with
//                  ±5 neighbour suppression as ballot scans (:450-568), the less-flat collection
//                  (:570-577) and a PCL-semantics VoxelGrid(0.2) of the line (:579-589).
//   k_scan_compact one wave per (scan, line): concatenates the per-line outputs in line order
//                  (offsets = wave sums of the earlier lines' counts).
#include <hip/hip_runtime.h>

#include "../../include/lislam.h"
#include "lislam_device.hpp"
#include "lislam_internal.hpp"

namespace lislam {

// ------------------------------------------------------------------------------- front kernels
// The scan is cut into ranges of kRange consecutive ring-order points, one wavefront per range
// (4 per workgroup, S x ceil(R/4) workgroups: ~4.8k for a 300-scan batch, so every CU streams).
constexpr int kRange = 1024;
constexpr int kFrontWaves = 4;

__device__ __forceinline__ bool keep_point(const P4& p, float thr2) {
  return !(p.x * p.x + p.y * p.y + p.z * p.z < thr2);
}

// ori before halfPassed (scanRegistration.cpp:339-347)
__device__ __forceinline__ float ori_not_passed(float ori, float startOri) {
  if ((double)ori < (double)startOri - kPi / 2)
    ori = (float)((double)ori + 2 * kPi);
  else if ((double)ori > (double)startOri + kPi * 3 / 2)
    ori = (float)((double)ori - 2 * kPi);
  return ori;
}
// ori after halfPassed (scanRegistration.cpp:357-365)
__device__ __forceinline__ float ori_passed(float ori, float endOri) {
  ori = (float)((double)ori + 2 * kPi);
  if ((double)ori < (double)endOri - kPi * 3 / 2)
    ori = (float)((double)ori + 2 * kPi);
  else if ((double)ori > (double)endOri + kPi / 2)
    ori = (float)((double)ori - 2 * kPi);
  return ori;
}

// startOri / endOri of the scan from its first and last kept points (scanRegistration.cpp:247-262).
// Every wave finds them itself (one or two cached 1 KiB reads in practice), so the count pass
// needs no cross-wave step.
__device__ __forceinline__ bool scan_oris(const P4* pts, int N, float thr2, float& so, float& eo) {
  const int lane = lane_id();
  int first = -1, last = -1;
  for (int b = 0; b < N && first < 0; b += 64) {
    const int i = b + lane;
    const uint64_t m = __ballot(i < N && keep_point(ld4(pts + i), thr2));
    if (m) first = b + (int)__builtin_ctzll(m);
  }
  if (first < 0) return false;
  for (int b = N - 1; b >= 0 && last < 0; b -= 64) {
    const int i = b - lane;
    const uint64_t m = __ballot(i >= 0 && keep_point(ld4(pts + i), thr2));
    if (m) last = b - (int)__builtin_ctzll(m);
  }
  const P4 p0 = ld4(pts + first), p1 = ld4(pts + last);
  so = -atan2_f(p0.y, p0.x);
  eo = (float)((double)(-atan2_f(p1.y, p1.x)) + 2 * kPi);
  if ((double)(eo - so) > 3 * kPi)
    eo = (float)((double)eo - 2 * kPi);
  else if ((double)(eo - so) < kPi)
    eo = (float)((double)eo + 2 * kPi);
  return true;
}

// Lanes holding the same scan line as this lane (7 ballots over the bits of sid < 128).
__device__ __forceinline__ uint64_t line_peers(int sid) {
  uint64_t peers = __ballot(sid >= 0);
  for (int bit = 0; bit < 7; bit++) {
    const uint64_t m = __ballot((sid >> bit) & 1);
    peers &= ((sid >> bit) & 1) ? m : ~m;
  }
  return peers;
}

// Pass 1 (one wave per range): range / intensity images + cloud_track (image_handler.h_ouster:
// 112-139), the close-point filter (scanRegistration.cpp:152-186), the per-range scan-line
// histogram (:285-331) and the first index of the range where halfPassed would flip (:336-353):
// the loop's only sequential state is a monotone flag, so it reduces to "first index where".
__global__ __launch_bounds__(64 * kFrontWaves) void k_front_count(FeatureArgs a) {
  __shared__ int hist[kFrontWaves][kMaxLines];
  const int RB = (a.fr_R + kFrontWaves - 1) / kFrontWaves;
  const int s = blockIdx.x / RB, wave = threadIdx.x >> 6, lane = lane_id();
  const int r = (blockIdx.x % RB) * kFrontWaves + wave;
  if (r >= a.fr_R) return;
  const int N = a.N, H = a.H;
  const P4* pts = a.pts + (size_t)s * N;
  const float thr2 = a.min_range * a.min_range;
  int* h = hist[wave];
  for (int l = lane; l < H; l += 64) h[l] = 0;
  float startOri = 0.f, endOri = 0.f;
  const bool any = scan_oris(pts, N, thr2, startOri, endOri);
  if (r == 0 && lane == 0) {
    a.fr_ori[2 * s] = startOri;
    a.fr_ori[2 * s + 1] = endOri;
  }
  uint8_t* img_r = a.img_range ? a.img_range + (size_t)s * N : nullptr;
  uint8_t* img_i = a.img_int ? a.img_int + (size_t)s * N : nullptr;
  P4* track = a.track ? a.track + (size_t)s * N : nullptr;
  int flip = N;
  const int i0 = r * kRange, i1 = min(N, i0 + kRange);
  for (int b = i0; b < i1; b += 64) {
    const int i = b + lane;
    int sid = -1;
    if (i < i1) {
      const P4 p = ld4(pts + i);
      const float d2 = p.x * p.x + p.y * p.y + p.z * p.z;
      const float range = sqrtf(d2);
      const float inten = fminf(p.i, 255.0f);
      if (img_r) img_r[i] = (uint8_t)fminf(range * 20, 255.0f);
      if (img_i) img_i[i] = (uint8_t)inten;
      if (track) st4(track + i, (double)range >= 0.1 ? P4{p.x, p.y, p.z, inten} : P4{0.f, 0.f, 0.f, 0.f});
      if (!(d2 < thr2) && any) {
        sid = scan_id_of(elevation_deg(p), H);
        if (sid >= 0 && flip == N) {
          const float ori = ori_not_passed(-atan2_f(p.y, p.x), startOri);
          if ((double)(ori - startOri) > kPi) flip = i;
        }
      }
    }
    const uint64_t peers = line_peers(sid);
    if (sid >= 0 && __popcll(peers & lanemask_lt()) == 0) h[sid] += __popcll(peers);  // one leader per line
    __builtin_amdgcn_wave_barrier();
  }
  flip = (int)wave_umin((uint32_t)flip);
  int* dst = a.fr_hist + ((size_t)s * a.fr_R + r) * H;
  for (int l = lane; l < H; l += 64) dst[l] = h[l];
  if (lane == 0) a.fr_flip[(size_t)s * a.fr_R + r] = flip;
}

// Per scan: line totals -> line offsets (scanStartInd = off + 5, scanEndInd = off + len - 6,
// :384-394), each range's per-line write base (in place of its histogram), and the scan's flip
// index (minimum over the ranges).
__global__ __launch_bounds__(kMaxLines) void k_front_scan(FeatureArgs a) {
  __shared__ int tot[kMaxLines];
  __shared__ uint32_t wflip[kMaxLines / 64];
  const int s = blockIdx.x, l = threadIdx.x, H = a.H, R = a.fr_R;
  int* hist = a.fr_hist + (size_t)s * R * H;
  int t = 0;
  if (l < H)
    for (int r = 0; r < R; r++) t += hist[(size_t)r * H + l];
  tot[l] = t;
  uint32_t f = 0xffffffffu;
  for (int r = l; r < R; r += kMaxLines) f = min(f, (uint32_t)a.fr_flip[(size_t)s * R + r]);
  f = wave_umin(f);
  if (lane_id() == 0) wflip[l >> 6] = f;
  __syncthreads();
  if (l < H) {
    int off = 0;
    for (int k = 0; k < l; k++) off += tot[k];
    a.line_off[(size_t)s * (H + 1) + l] = off;
    if (l == H - 1) {
      a.line_off[(size_t)s * (H + 1) + H] = off + t;
      a.n_cloud[s] = off + t;
    }
    for (int r = 0; r < R; r++) {
      const int c = hist[(size_t)r * H + l];
      hist[(size_t)r * H + l] = off;
      off += c;
    }
  }
  if (l == 0) a.fr_flip[(size_t)s * R] = (int)min(wflip[0], wflip[1]);  // range 0 slot = scan flip
}

// Pass 2 (one wave per range): ori / relTime / intensity = scanID + 0.1 relTime (:334-371) and the
// stable scatter by scan line (= the per-line push_back + concatenation, :373-394): in-wave ranks
// from ballot peer masks, the running per-line base of the range in LDS.
__global__ __launch_bounds__(64 * kFrontWaves) void k_front_scatter(FeatureArgs a) {
  __shared__ int base[kFrontWaves][kMaxLines];
  const int RB = (a.fr_R + kFrontWaves - 1) / kFrontWaves;
  const int s = blockIdx.x / RB, wave = threadIdx.x >> 6, lane = lane_id();
  const int r = (blockIdx.x % RB) * kFrontWaves + wave;
  if (r >= a.fr_R) return;
  const int N = a.N, H = a.H;
  if (a.n_cloud[s] == 0) return;
  const P4* pts = a.pts + (size_t)s * N;
  const float thr2 = a.min_range * a.min_range;
  int* bs = base[wave];
  const int* src = a.fr_hist + ((size_t)s * a.fr_R + r) * H;
  for (int l = lane; l < H; l += 64) bs[l] = src[l];
  const float startOri = a.fr_ori[2 * s], endOri = a.fr_ori[2 * s + 1];
  const int flip = a.fr_flip[(size_t)s * a.fr_R];
  P4* cloud = a.cloud + (size_t)s * N;
  const uint64_t lt = lanemask_lt();
  __builtin_amdgcn_wave_barrier();
  const int i0 = r * kRange, i1 = min(N, i0 + kRange);
  for (int b = i0; b < i1; b += 64) {
    const int i = b + lane;
    P4 p{0.f, 0.f, 0.f, 0.f};
    int sid = -1;
    if (i < i1) {
      p = ld4(pts + i);
      if (keep_point(p, thr2)) sid = scan_id_of(elevation_deg(p), H);
    }
    if (sid >= 0) {
      float ori = -atan2_f(p.y, p.x);
      ori = (i <= flip) ? ori_not_passed(ori, startOri) : ori_passed(ori, endOri);
      const float relTime = (ori - startOri) / (endOri - startOri);
      p.i = (float)((double)sid + 0.1 * (double)relTime);
    }
    const uint64_t peers = line_peers(sid);
    if (sid >= 0) {
      const int rank = __popcll(peers & lt);
      st4(cloud + bs[sid] + rank, p);
      __builtin_amdgcn_wave_barrier();
      if (rank == 0) bs[sid] += __popcll(peers);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------------------- line kernel
// Optional per-phase cycle accounting (built only with -DLISLAM_PHASE_PROF, scripts/phase_prof.py).
#ifdef LISLAM_PHASE_PROF
__device__ unsigned long long g_phase_cycles[16];
__device__ unsigned long long* g_line_log;  // k_scan_lines per-wave timeline (lislam_debug_line_log)
// Each phase's cycles accumulate in the wave's registers; the wave adds them to the global counters
// once, when the line is done (PHASE_FLUSH), so the profiler's atomics do not sit inside the phases
// they measure (round 6: adding them at every phase boundary made the first vector-memory wait
// after them absorb their L2 contention).
#define PHASE_BEGIN                                 \
  uint64_t t_ph = __builtin_readcyclecounter();     \
  uint64_t ph_acc[16];                              \
  _Pragma("unroll") for (int i_ = 0; i_ < 16; i_++) ph_acc[i_] = 0
#define PHASE(i)                                                     \
  do {                                                               \
    const uint64_t now_ = __builtin_readcyclecounter();              \
    ph_acc[i] += now_ - t_ph;                                        \
    t_ph = now_;                                                     \
  } while (0)
#define PHASE_COUNT(i) \
  do {                   \
    if (lane_id() == 0) atomicAdd(&g_phase_cycles[i], 1ull); \
  } while (0)
#define PHASE_FLUSH                                                              \
  do {                                                                           \
    if (lane_id() == 0)                                                          \
      _Pragma("unroll") for (int i_ = 0; i_ < 16; i_++) if (ph_acc[i_])          \
        atomicAdd(&g_phase_cycles[i_], ph_acc[i_]);                              \
  } while (0)
#else
#define PHASE_BEGIN
#define PHASE(i)
#define PHASE_COUNT(i)
#define PHASE_FLUSH
#endif
// LDS capacities of the fast path; longer lines run the same code on global scratch.
constexpr int kLineCap = 2048;

// Line kernel workgroups are one wave.  With the line in LDS, a wave's LDS accesses complete in
// issue order, so ordering them only needs the LDS counter drained and a compiler barrier (no
// s_barrier, and no wait on the wave's outstanding global stores); the long-line path keeps its
// state in global scratch and uses a full workgroup barrier.
template <bool kLds>
__device__ __forceinline__ void wave_sync() {
  if (kLds) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// Bitonic sort (ascending) of P (power of two, >= 64) 64-bit keys by one wave.  Each stage loads
// all of a lane's pairs before it compares and stores any, so a stage costs one LDS round trip
// (kMaxT = P/128 bound of the fast path); the long-line path keeps the simple loop.
template <int kMaxT, typename KeyPtr>
__device__ __forceinline__ void bitonic_sort(KeyPtr keys, int P) {
  const int lane = lane_id();
  const int npairs = P >> 1;
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (kMaxT > 0) {
        uint64_t A[kMaxT > 0 ? kMaxT : 1], B[kMaxT > 0 ? kMaxT : 1];
        int I[kMaxT > 0 ? kMaxT : 1];
#pragma unroll
        for (int t = 0; t < kMaxT; t++) {
          const int q = lane + 64 * t;
          I[t] = -1;
          if (q < npairs) {
            const int i = ((q & ~(j - 1)) << 1) | (q & (j - 1));
            I[t] = i;
            A[t] = keys[i];
            B[t] = keys[i | j];
          }
        }
#pragma unroll
        for (int t = 0; t < kMaxT; t++) {
          const int i = I[t];
          if (i >= 0) {
            const bool up = (i & k) == 0;
            if ((A[t] > B[t]) == up) { keys[i] = B[t]; keys[i | j] = A[t]; }
          }
        }
      } else {
        for (int q = lane; q < npairs; q += 64) {
          const int i = ((q & ~(j - 1)) << 1) | (q & (j - 1));
          const uint64_t x = keys[i], y = keys[i | j];
          const bool up = (i & k) == 0;
          if ((x > y) == up) { keys[i] = y; keys[i | j] = x; }
        }
      }
      wave_sync<(kMaxT > 0)>();
    }
  }
}

__device__ __forceinline__ uint64_t first_lane(uint64_t m) { return (uint64_t)__builtin_ctzll(m); }

// ------------------------------------------------------------------ libstdc++ std::sort tie order
// PCL VoxelGrid sorts (voxel, point) pairs with std::sort comparing the voxel only
// (scanRegistration.cpp:583-586 -> pcl::VoxelGrid::applyFilter), so the order of a voxel's points
// — the order its centroid is summed in — is whatever libstdc++'s introsort leaves.  These
// functions reproduce that order on one wave (checked against std::sort itself by
// tests/cpp/introsort_emu.cpp, which restates the same formulation on the host):
//   std::__introsort_loop: ranges of more than 16 elements are split by
//     __unguarded_partition_pivot (median of first + 1, mid, last - 1 moved to first, then the
//     two-pointer walk); below depth 2 floor(log2 n) a range is heap-sorted instead;
//   the walk is computed with prefix counts: the m-th element >= pivot from the left, L[m], swaps
//     with the m-th element <= pivot from the right, R[m], while L[m] < R[m]; the cut is
//     min(L[m*], R[m* - 1]) for the first m* where that fails;
//   std::__final_insertion_sort never reorders equal keys, so the final order is a stable sort
//     by key of the array the loop leaves (the caller's bitonic sort of (key, position)).
// a: the elements (LDS or global), ordered by kof(element) (an unsigned key; the element's other
// bits are its payload); lidx / ridx: scratch of at least n / 2 + 1 entries each.  Ranges of the
// partition stack live one per lane.
template <bool kLds, typename ElemPtr, typename KeyOf, typename IdxPtr>
__device__ __forceinline__ int introsort_partition(ElemPtr a, KeyOf kof, int f, int l, IdxPtr lidx, IdxPtr ridx) {
  const int lane = lane_id();
  const int mid = f + (l - f) / 2;
  // std::__move_median_to_first(f, f + 1, mid, l - 1)
  const auto ea = a[f + 1], eb = a[mid], ec = a[l - 1], e0 = a[f];
  const auto ka = kof(ea), kb = kof(eb), kc = kof(ec);
  int pick;
  if (ka < kb) pick = kb < kc ? mid : (ka < kc ? l - 1 : f + 1);
  else pick = ka < kc ? f + 1 : (kb < kc ? l - 1 : mid);
  const auto ep = pick == f + 1 ? ea : pick == mid ? eb : ec;
  const auto p = kof(ep);
  wave_sync<kLds>();  // every lane has read before lane 0 swaps
  if (lane == 0) { a[f] = ep; a[pick] = e0; }
  wave_sync<kLds>();
  const int lo = f + 1, hi = l - 1;
  const int cap = ((hi - lo + 1) >> 1) + 1;  // L[m] < R[m] pairs use 2m distinct positions
  int total_le = 0;
  for (int b = lo; b <= hi; b += 64) {
    const int i = b + lane;
    total_le += __popcll(__ballot(i <= hi && !(p < kof(a[i]))));
  }
  int ge_before = 0, le_seen = 0, mstar = 0, next_ge = -1;
  const uint64_t lt = lanemask_lt();
  for (int b = lo; b <= hi; b += 64) {
    const int i = b + lane;
    const bool valid = i <= hi;
    const auto k = valid ? kof(a[i]) : p;
    const bool ge = valid && !(k < p), le = valid && !(p < k);
    const uint64_t mge = __ballot(ge), mle = __ballot(le);
    const int rank = ge_before + __popcll(mge & lt);                        // L rank of i
    const int after = total_le - (le_seen + __popcll(mle & lt) + (int)le);  // <= elements after i = R rank
    const bool cond = ge && after >= rank + 1;                               // L[rank] < R[rank]
    const uint64_t mc = __ballot(cond);
    if (cond) lidx[rank] = i;
    if (le && after < cap) ridx[after] = i;
    if (next_ge < 0) {
      const uint64_t nc = mge & ~mc;  // the first >= element left unmatched is L[m*]
      if (nc) next_ge = b + (int)first_lane(nc);
    }
    mstar += __popcll(mc);
    ge_before += __popcll(mge);
    le_seen += __popcll(mle);
  }
  wave_sync<kLds>();
  for (int r = lane; r < mstar; r += 64) {
    const int x = lidx[r], y = ridx[r];
    const auto ex = a[x], ey = a[y];
    a[x] = ey;
    a[y] = ex;
  }
  int cut = mstar > 0 ? (int)ridx[mstar - 1] : l;
  if (next_ge >= 0 && next_ge < cut) cut = next_ge;
  wave_sync<kLds>();
  return cut;
}

// std::__heap_select + std::__sort_heap of [first, first + len) (the introsort depth fallback);
// serial on lane 0.
template <typename ElemPtr, typename KeyOf>
__device__ __forceinline__ void heap_sort_serial(ElemPtr a, KeyOf kof, int first, int len) {
  auto adjust = [&](int hole, int n, auto v) {  // std::__adjust_heap + std::__push_heap
    const int top = hole;
    int child = hole;
    while (child < (n - 1) / 2) {
      child = 2 * (child + 1);
      if (kof(a[first + child]) < kof(a[first + child - 1])) child--;
      a[first + hole] = a[first + child];
      hole = child;
    }
    if ((n & 1) == 0 && child == (n - 2) / 2) {
      child = 2 * (child + 1);
      a[first + hole] = a[first + child - 1];
      hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && kof(a[first + parent]) < kof(v)) {
      a[first + hole] = a[first + parent];
      hole = parent;
      parent = (hole - 1) / 2;
    }
    a[first + hole] = v;
  };
  if (len >= 2)
    for (int parent = (len - 2) / 2;; parent--) {
      adjust(parent, len, a[first + parent]);
      if (parent == 0) break;
    }
  for (int last = len; last > 1;) {
    --last;
    const auto v = a[first + last];
    a[first + last] = a[first];
    adjust(0, last, v);
  }
}

template <bool kLds, typename ElemPtr, typename KeyOf, typename IdxPtr>
__device__ __forceinline__ void introsort_order(ElemPtr a, KeyOf kof, int n, IdxPtr lidx, IdxPtr ridx) {
  if (n <= 16) return;
  const int lane = lane_id();
  int sf = 0, sl = 0, sd = 0, sp = 0;  // lane sp holds stack entry sp
  int f = 0, l = n, d = 2 * (31 - __builtin_clz((unsigned)n));
  for (;;) {
    while (l - f > 16) {
      if (d == 0) {
        if (lane == 0) heap_sort_serial(a, kof, f, l - f);
        wave_sync<kLds>();
        break;
      }
      d--;
      const int cut = introsort_partition<kLds>(a, kof, f, l, lidx, ridx);
      if (lane == sp) { sf = cut; sl = l; sd = d; }
      sp++;
      l = cut;
    }
    if (sp == 0) break;
    sp--;
    f = __builtin_amdgcn_readlane(sf, sp);
    l = __builtin_amdgcn_readlane(sl, sp);
    d = __builtin_amdgcn_readlane(sd, sp);
  }
}

// ---- the same order with the line in LDS (the register path): ranges of up to 64 elements run
// their whole subtree in registers (one element per lane; the partition's swaps are lane
// permutes), larger ranges read their elements once into registers per partition.

// std::__unguarded_partition_pivot of lanes [f, l) of e (one element per lane).
template <typename KeyOf>
__device__ __forceinline__ int partition_reg(uint32_t& e, KeyOf kof, int f, int l) {
  const int lane = lane_id();
  const int mid = f + (l - f) / 2;
  const uint32_t ea = (uint32_t)__builtin_amdgcn_readlane((int)e, f + 1);
  const uint32_t eb = (uint32_t)__builtin_amdgcn_readlane((int)e, mid);
  const uint32_t ec = (uint32_t)__builtin_amdgcn_readlane((int)e, l - 1);
  const uint32_t e0 = (uint32_t)__builtin_amdgcn_readlane((int)e, f);
  const uint32_t ka = kof(ea), kb = kof(eb), kc = kof(ec);
  int pick;
  if (ka < kb) pick = kb < kc ? mid : (ka < kc ? l - 1 : f + 1);
  else pick = ka < kc ? f + 1 : (kb < kc ? l - 1 : mid);
  const uint32_t ep = pick == f + 1 ? ea : pick == mid ? eb : ec;
  if (lane == f) e = ep;
  else if (lane == pick) e = e0;
  const uint32_t p = kof(ep), k = kof(e);
  const bool in = lane > f && lane < l;
  const bool ge = in && !(k < p), le = in && !(p < k);
  const uint64_t mge = __ballot(ge), mle = __ballot(le), lt = lanemask_lt();
  const int rank = __popcll(mge & lt);
  const int after = __popcll(mle) - __popcll(mle & lt) - (int)le;
  const bool cond = ge && after >= rank + 1;
  const uint64_t mc = __ballot(cond);
  const int mstar = __popcll(mc);
  const bool isR = le && after < mstar;  // L[m] < R[m]: the swapped L and R lanes are disjoint
  // slot m <- the lane of R[m] / of L[m] (lanes outside the swap push to slot 63, never read)
  const int toR = __builtin_amdgcn_ds_permute((isR ? after : 63) << 2, lane);
  const int toL = __builtin_amdgcn_ds_permute((cond ? rank : 63) << 2, lane);
  const int slot = cond ? rank : (isR ? after : 0);
  const int pR = __builtin_amdgcn_ds_bpermute(slot << 2, toR), pL = __builtin_amdgcn_ds_bpermute(slot << 2, toL);
  const int partner = cond ? pR : (isR ? pL : lane);
  e = (uint32_t)__builtin_amdgcn_ds_bpermute(partner << 2, (int)e);
  int cut = l;
  if (mstar > 0) cut = (int)first_lane(__ballot(le && after == mstar - 1));
  const uint64_t nc = mge & ~mc;  // L[m*]
  if (nc) cut = min(cut, (int)first_lane(nc));
  return cut;
}

// std::__heap_select + std::__sort_heap of lanes [f, l) of e (uniform serial steps).
template <typename KeyOf>
__device__ __forceinline__ void heap_sort_reg(uint32_t& e, KeyOf kof, int f, int l) {
  auto get = [&](int i) { return (uint32_t)__builtin_amdgcn_readlane((int)e, f + i); };
  const int lane = lane_id();
  auto set = [&](int i, uint32_t v) { e = lane == f + i ? v : e; };
  auto adjust = [&](int hole, int n, uint32_t v) {
    const int top = hole;
    int child = hole;
    while (child < (n - 1) / 2) {
      child = 2 * (child + 1);
      if (kof(get(child)) < kof(get(child - 1))) child--;
      set(hole, get(child));
      hole = child;
    }
    if ((n & 1) == 0 && child == (n - 2) / 2) {
      child = 2 * (child + 1);
      set(hole, get(child - 1));
      hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && kof(get(parent)) < kof(v)) {
      set(hole, get(parent));
      hole = parent;
      parent = (hole - 1) / 2;
    }
    set(hole, v);
  };
  const int len = l - f;
  for (int parent = (len - 2) / 2;; parent--) {
    adjust(parent, len, get(parent));
    if (parent == 0) break;
  }
  for (int last = len; last > 1;) {
    --last;
    const uint32_t v = get(last);
    set(last, get(0));
    adjust(0, last, v);
  }
}

// The introsort subtree of a[F, F + n), n <= 64, with depth limit D, in registers.
template <typename KeyOf>
__device__ __forceinline__ void introsort_small(uint32_t* a, KeyOf kof, int F, int n, int D) {
  const int lane = lane_id();
  uint32_t e = lane < n ? a[F + lane] : 0u;
  int sf = 0, sl = 0, sd = 0, sp = 0;
  int f = 0, l = n, d = D;
  for (;;) {
    while (l - f > 16) {
      if (d == 0) {
        PHASE_COUNT(13);
        heap_sort_reg(e, kof, f, l);
        break;
      }
      d--;
      PHASE_COUNT(14);
      const int cut = partition_reg(e, kof, f, l);
      if (lane == sp) { sf = cut; sl = l; sd = d; }
      sp++;
      l = cut;
    }
    if (sp == 0) break;
    sp--;
    f = __builtin_amdgcn_readlane(sf, sp);
    l = __builtin_amdgcn_readlane(sl, sp);
    d = __builtin_amdgcn_readlane(sd, sp);
  }
  if (lane < n) a[F + lane] = e;
}

// A partition of a range of more than 64 elements of the LDS array (two counting passes over the
// range, then the swaps).
template <int kC, typename KeyOf>
__device__ __forceinline__ int partition_lds(uint32_t* a, KeyOf kof, int f, int l, uint16_t* lidx, uint16_t* ridx) {
  const int lane = lane_id();
  const int mid = f + (l - f) / 2;
  const uint32_t ea = a[f + 1], eb = a[mid], ec = a[l - 1], e0 = a[f];
  const uint32_t ka = kof(ea), kb = kof(eb), kc = kof(ec);
  int pick;
  if (ka < kb) pick = kb < kc ? mid : (ka < kc ? l - 1 : f + 1);
  else pick = ka < kc ? f + 1 : (kb < kc ? l - 1 : mid);
  const uint32_t ep = pick == f + 1 ? ea : pick == mid ? eb : ec;
  const uint32_t p = kof(ep);
  const int lo = f + 1, hi = l - 1;
  // the median swap (a[f] <-> a[pick]) as the reads below see it; the swap itself is written
  // after the counting passes
  auto key_at = [&](int i) { return i == pick ? kof(e0) : kof(a[i]); };
  int total_le = 0;
  for (int b = lo; b <= hi; b += 64) {
    const int i = b + lane;
    total_le += __popcll(__ballot(i <= hi && !(p < key_at(i))));
  }
  const int cap = ((hi - lo + 1) >> 1) + 1;
  int ge_before = 0, le_seen = 0, mstar = 0, next_ge = -1;
  const uint64_t lt = lanemask_lt();
  for (int b = lo; b <= hi; b += 64) {
    const int i = b + lane;
    const bool valid = i <= hi;
    const uint32_t k = valid ? key_at(i) : p;
    const bool ge = valid && !(k < p), le = valid && !(p < k);
    const uint64_t mge = __ballot(ge), mle = __ballot(le);
    const int rank = ge_before + __popcll(mge & lt);
    const int after = total_le - (le_seen + __popcll(mle & lt) + (int)le);
    const bool cond = ge && after >= rank + 1;
    const uint64_t mc = __ballot(cond);
    if (cond) lidx[rank] = (uint16_t)i;
    if (le && after < cap) ridx[after] = (uint16_t)i;
    if (next_ge < 0) {
      const uint64_t nc = mge & ~mc;
      if (nc) next_ge = b + (int)first_lane(nc);
    }
    mstar += __popcll(mc);
    ge_before += __popcll(mge);
    le_seen += __popcll(mle);
  }
  if (lane == 0) { a[f] = ep; a[pick] = e0; }
  wave_sync<true>();
  for (int r = lane; r < mstar; r += 64) {
    const int x = lidx[r], y = ridx[r];
    const uint32_t ex = a[x], ey = a[y];
    a[x] = ey;
    a[y] = ex;
  }
  int cut = mstar > 0 ? (int)ridx[mstar - 1] : l;
  if (next_ge >= 0 && next_ge < cut) cut = next_ge;
  wave_sync<true>();
  return cut;
}

// introsort_order for an LDS array of at most 64 kC elements (the register path's line).
template <int kC, typename KeyOf>
__device__ __forceinline__ void introsort_order_lds(uint32_t* a, KeyOf kof, int n, uint16_t* lidx, uint16_t* ridx) {
  if (n <= 16) return;
  const int lane = lane_id();
  int sf = 0, sl = 0, sd = 0, sp = 0;
  int f = 0, l = n, d = 2 * (31 - __builtin_clz((unsigned)n));
  for (;;) {
    while (l - f > 16) {
      if (l - f <= 64) {
        introsort_small(a, kof, f, l - f, d);
        wave_sync<true>();
        break;
      }
      if (d == 0) {
        PHASE_COUNT(13);
        if (lane == 0) heap_sort_serial(a, kof, f, l - f);
        wave_sync<true>();
        break;
      }
      d--;
      PHASE_COUNT(15);
      const int cut = partition_lds<kC>(a, kof, f, l, lidx, ridx);
      if (lane == sp) { sf = cut; sl = l; sd = d; }
      sp++;
      l = cut;
    }
    if (sp == 0) break;
    sp--;
    f = __builtin_amdgcn_readlane(sf, sp);
    l = __builtin_amdgcn_readlane(sl, sp);
    d = __builtin_amdgcn_readlane(sd, sp);
  }
}

// std::sort's final positions after its introsort loop (std::__final_insertion_sort, see the
// VoxelGrid below): element el[j] ends at j minus the greater keys among the 15 positions before
// it plus the smaller keys among the 15 after it.  pos[el[j]] <- that position (pos is distinct
// from el; the elements are 0 .. n-1).
template <bool kLds, typename ElemPtr, typename KeyOf, typename PosPtr>
__device__ __forceinline__ void final_positions(ElemPtr el, KeyOf kof, int n, PosPtr pos) {
  for (int j = lane_id(); j < n; j += 64) {
    const uint32_t e = el[j];
    const uint32_t k = kof(e);
    int mv = 0;
#pragma unroll
    for (int d = 1; d <= 15; d++) {
      if (j - d >= 0 && kof(el[j - d]) > k) mv--;
      if (j + d < n && kof(el[j + d]) < k) mv++;
    }
    pos[e] = j + mv;
  }
  wave_sync<kLds>();
}

struct LineCounts {
  int sharp, less_sharp, flat, less_flat;
};

// ±5 neighbour suppression of a picked point (scanRegistration.cpp:481-504) from precomputed
// links: link[k] = |p[k+1] - p[k]|^2 <= 0.05 (float sums, compared in double); the reference's
// backward differences p[k] - p[k+1] square to the same bits.  Forward marks ind+1.. while
// link[ind], link[ind+1], ... hold (at most 5); backward marks ind-1.. while link[ind-1], ... hold.
template <bool kLds, typename BytePtr>
__device__ __forceinline__ void suppress(const BytePtr link, int ind, BytePtr picked) {
  const int lane = lane_id();
  bool brk = false;
  if (lane < 5) brk = link[ind + lane] == 0;                  // forward link ind+lane
  else if (lane < 10) brk = link[ind - 1 - (lane - 5)] == 0;  // backward link ind-1-(lane-5)
  const uint64_t bm = __ballot(brk);
  const uint64_t fwd = bm & 0x1Full, bwd = bm & 0x3E0ull;
  const int nf = fwd ? (int)first_lane(fwd) : 5;      // marked forward neighbours
  const int nb = bwd ? (int)first_lane(bwd) - 5 : 5;  // marked backward neighbours
  if (lane < nf) picked[ind + 1 + lane] = 1;
  else if (lane >= 5 && lane - 5 < nb) picked[ind - 1 - (lane - 5)] = 1;
  wave_sync<kLds>();
}

struct LineLists {
  int sharp[kCapSharpPerLine];
  int less_sharp[kCapLessSharpPerLine];
  int flat[kCapFlatPerLine];
};

// One scan line: curvature, the six-segment sharp/flat selection and the line's VoxelGrid.  The
// kernel runs it on global scratch (kLds = false) for lines longer than the register path holds;
// the VoxelGrid's key buffer layout assumes that scratch (16 B per line point).
//
// The reference sorts each segment by curvature (std::sort, scanRegistration.cpp:440-448; the
// canonical tie order is the point index) and walks it from the largest (sharp, :450-506) and
// smallest (flat, :511-568) end, skipping points already picked.  Suppression only ever adds
// picked points and the walk never revisits a position, so the k-th pick of a walk is the
// extreme (curvature, index) key among the still-unpicked points that pass the curvature test:
// each pick is one wave-wide max/min reduction instead of a sorted segment.
template <bool kLds>
__device__ __forceinline__ void line_body(const FeatureArgs& a, int s, int line, uint8_t* lds_picked, int8_t* lds_label,
                                          uint64_t* lds_keys, int* lds_list, uint8_t* lds_link, LineLists& ll,
                                          P4* stage) {
  const int lane = lane_id();
  const int N = a.N, H = a.H;
  const int* lo = a.line_off + (size_t)s * (H + 1);
  const int off = lo[line];
  const int len = lo[line + 1] - off;
  const int total = lo[H];
  const P4* cloud = a.cloud + (size_t)s * N;
  float* curv = a.curv + (size_t)s * N;
  int8_t* glabel = a.label + (size_t)s * N;
  uint8_t* picked = kLds ? lds_picked : a.scr_picked + (size_t)s * N + off;
  int8_t* label = kLds ? lds_label : glabel + off;
  uint64_t* keys = kLds ? lds_keys : a.scr_keys + 2 * ((size_t)s * N + off);  // pow2 padding <= 2 len
  float* curvL = kLds ? (float*)lds_keys : curv + off;  // the walks run before the voxel keys exist
  int* list = kLds ? lds_list : a.scr_list + (size_t)s * N + off;
  uint8_t* link = kLds ? lds_link : a.scr_link + (size_t)s * N + off;
  PHASE_BEGIN;

  // curvature (scanRegistration.cpp:397-412), left-to-right float sums
  for (int k = lane; k < len; k += 64) {
    const int i = off + k;
    float c = 0.f;
    if (i >= 5 && i < total - 5) {
      P4 q[11];
      for (int d = 0; d < 11; d++) q[d] = ld4(cloud + i - 5 + d);
      const float dX = q[0].x + q[1].x + q[2].x + q[3].x + q[4].x - 10 * q[5].x + q[6].x + q[7].x + q[8].x + q[9].x + q[10].x;
      const float dY = q[0].y + q[1].y + q[2].y + q[3].y + q[4].y - 10 * q[5].y + q[6].y + q[7].y + q[8].y + q[9].y + q[10].y;
      const float dZ = q[0].z + q[1].z + q[2].z + q[3].z + q[4].z - 10 * q[5].z + q[6].z + q[7].z + q[8].z + q[9].z + q[10].z;
      c = dX * dX + dY * dY + dZ * dZ;
    }
    curv[i] = c;
    if (kLds) curvL[k] = c;
    picked[k] = 0;
    label[k] = 0;
    uint8_t lk = 0;
    if (k + 1 < len) {
      const P4 p0 = ld4(cloud + i), p1 = ld4(cloud + i + 1);
      const float dx = p1.x - p0.x, dy = p1.y - p0.y, dz = p1.z - p0.z;
      lk = !((double)(dx * dx + dy * dy + dz * dz) > 0.05);
    }
    link[k] = lk;
  }
  wave_sync<kLds>();
  PHASE(0);

  LineCounts cnt{0, 0, 0, 0};
  P4* o_sharp = a.stg_sharp + ((size_t)s * H + line) * kCapSharpPerLine;
  P4* o_lsharp = a.stg_less_sharp + ((size_t)s * H + line) * kCapLessSharpPerLine;
  P4* o_flat = a.stg_flat + ((size_t)s * H + line) * kCapFlatPerLine;
  P4* o_lflat = a.stg_less_flat + (size_t)s * N + off;
  const int sI = 5, eI = len - 6;  // scanStartInd / scanEndInd relative to off
  int nlist = 0;
  if (eI - sI >= 6) {
    for (int j = 0; j < 6; j++) {
      const int sp = sI + (eI - sI) * j / 6;
      const int ep = sI + (eI - sI) * (j + 1) / 6 - 1;
      // keys (curvature, index) until a pick meets a tie (TIES_REFERENCE), then (std::sort's
      // position, index): the segment's sort replayed in the key buffer, which the walks leave
      // unused (line_body_reg documents the scheme)
      const bool want_replay = a.ties == LISLAM_TIES_REFERENCE;
      bool by_pos = false;  // keys are sorted positions (after a replay)
      // [n] elements, then [n + 2] index scratch / positions (past the curvature when it is LDS)
      uint32_t* seg_el = reinterpret_cast<uint32_t*>(keys) + (kLds ? len : 0);
      uint32_t* seg_pos = seg_el + (ep - sp + 1);
      auto key_of = [&](int k) -> uint64_t {
        const uint32_t hi = by_pos ? seg_pos[k - sp] : __float_as_uint(curvL[k]);
        return ((uint64_t)hi << 32) | (uint32_t)k;
      };
      auto walk_best = [&](bool largest) {
        uint64_t best = largest ? 0ull : ~0ull;
        for (int k = sp + lane; k <= ep; k += 64) {
          const float c = curvL[k];
          if (picked[k] == 0 && (largest ? (double)c > 0.1 : (double)c < 0.1)) {
            const uint64_t key = key_of(k);
            best = largest ? (key > best ? key : best) : (key < best ? key : best);
          }
        }
        return largest ? wave_max_u64(best) : wave_min_u64(best);
      };
      auto tie_at = [&](bool largest, uint64_t best) {
        const uint32_t bc = (uint32_t)(best >> 32);
        bool t = false;
        for (int k = sp + lane; k <= ep; k += 64) {
          const float c = curvL[k];
          if (picked[k] == 0 && (largest ? (double)c > 0.1 : (double)c < 0.1) && __float_as_uint(c) == bc &&
              k != (int)(uint32_t)best)
            t = true;
        }
        return __ballot(t) != 0ull;
      };
      auto replay = [&]() {
        const int n = ep - sp + 1;
        for (int i = lane; i < n; i += 64) seg_el[i] = (uint32_t)i;
        wave_sync<kLds>();
        auto kof = [&](uint32_t e) { return __float_as_uint(curvL[sp + (int)e]); };
        introsort_order<kLds>(seg_el, kof, n, seg_pos, seg_pos + (n / 2 + 1));
        wave_sync<kLds>();
        final_positions<kLds>(seg_el, kof, n, seg_pos);
        by_pos = true;
      };
      // ---- sharp picks: largest key first (:450-506); at most 20 per segment
      for (int largest = 1; largest <= 20; largest++) {
        uint64_t best = walk_best(true);
        if (best == 0) break;  // no unpicked point with curvature > 0.1 is left
        if (want_replay && !by_pos && tie_at(true, best)) {
          replay();
          best = walk_best(true);
        }
        const int ind = (int)(uint32_t)best;
        if (lane == 0) {
          if (largest <= 2) {
            label[ind] = 2;
            ll.sharp[cnt.sharp] = ind;
          } else {
            label[ind] = 1;
          }
          ll.less_sharp[cnt.less_sharp] = ind;
          picked[ind] = 1;
        }
        if (largest <= 2) cnt.sharp++;
        cnt.less_sharp++;
        wave_sync<kLds>();
        suppress<kLds>(link, ind, picked);
      }
      PHASE(2);
      // ---- flat picks: smallest key first (:511-568); the 4th pick ends the walk unmarked
      for (int smallest = 1; smallest <= 4; smallest++) {
        uint64_t best = walk_best(false);
        if (best == ~0ull) break;
        if (want_replay && !by_pos && tie_at(false, best)) {
          replay();
          best = walk_best(false);
        }
        const int ind = (int)(uint32_t)best;
        if (lane == 0) {
          label[ind] = -1;
          ll.flat[cnt.flat] = ind;
        }
        cnt.flat++;
        if (smallest == 4) break;
        if (lane == 0) picked[ind] = 1;
        wave_sync<kLds>();
        suppress<kLds>(link, ind, picked);
      }
      wave_sync<kLds>();
      PHASE(3);
      // ---- less-flat collection in index order (:570-577)
      for (int b = sp; b <= ep; b += 64) {
        const int k = b + lane;
        const bool f = k <= ep && label[k] <= 0;
        const uint64_t m = __ballot(f);
        if (f) list[nlist + __popcll(m & lanemask_lt())] = k;
        nlist += __popcll(m);
      }
      wave_sync<kLds>();
      PHASE(4);
    }
  }
  // write labels of the line (parity tests) and the picked points, in pick order
  for (int k = lane; k < len; k += 64) glabel[off + k] = label[k];
  for (int k = lane; k < cnt.sharp; k += 64) st4(o_sharp + k, ld4(cloud + off + ll.sharp[k]));
  for (int k = lane; k < cnt.less_sharp; k += 64) st4(o_lsharp + k, ld4(cloud + off + ll.less_sharp[k]));
  for (int k = lane; k < cnt.flat; k += 64) st4(o_flat + k, ld4(cloud + off + ll.flat[k]));
  wave_sync<kLds>();  // curvL aliases the key buffer
  PHASE(5);

  // ---- VoxelGrid(0.2) of the line's less-flat points (PCL VoxelGrid::applyFilter semantics)
  if (nlist > 0) {
    const float inv = 1.0f / 0.2f;
    float mn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, mx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    for (int k = lane; k < nlist; k += 64) {
      const P4 p = ld4(cloud + off + list[k]);
      mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
      mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
    }
    for (int d = 0; d < 3; d++) {
      for (int o = 32; o > 0; o >>= 1) {
        mn[d] = fminf(mn[d], __shfl_xor(mn[d], o));
        mx[d] = fmaxf(mx[d], __shfl_xor(mx[d], o));
      }
    }
    const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
    const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
    const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
    if (dx * dy * dz > (int64_t)2147483647) {  // PCL: leaf too small -> copy the input
      for (int k = lane; k < nlist; k += 64) st4(o_lflat + k, ld4(cloud + off + list[k]));
      cnt.less_flat = nlist;
    } else {
      int minb[3], divb[3];
      for (int d = 0; d < 3; d++) {
        minb[d] = (int)floorf(mn[d] * inv);
        divb[d] = (int)floorf(mx[d] * inv) - minb[d] + 1;
      }
      const int mul1 = divb[0], mul2 = divb[0] * divb[1];
      int P = 64;
      while (P < nlist) P <<= 1;
      // std::sort's order of equal voxels (introsort_order) on the list: the key buffer's 16 B per
      // line point hold the (voxel, line position) elements (second half) and the two index
      // scratches (first half) until the final keys overwrite them.
      {
        uint8_t* region = reinterpret_cast<uint8_t*>(keys);
        uint64_t* el = reinterpret_cast<uint64_t*>(region + 8 * (size_t)len);  // (voxel, line position)
        uint32_t* lidx = reinterpret_cast<uint32_t*>(region);
        uint32_t* ridx = reinterpret_cast<uint32_t*>(region + 4 * (size_t)len);
        for (int k = lane; k < nlist; k += 64) {
          const P4 p = ld4(cloud + off + list[k]);
          const int i0 = (int)(floorf(p.x * inv) - (float)minb[0]);
          const int i1 = (int)(floorf(p.y * inv) - (float)minb[1]);
          const int i2 = (int)(floorf(p.z * inv) - (float)minb[2]);
          el[k] = ((uint64_t)(uint32_t)(i0 + i1 * mul1 + i2 * mul2) << 32) | (uint32_t)list[k];
        }
        wave_sync<kLds>();
        if (a.ties == LISLAM_TIES_REFERENCE)
          introsort_order<kLds>(el, [](uint64_t e) { return (uint32_t)(e >> 32); }, nlist, lidx, ridx);
        // keys (voxel, position after the introsort loop) and the list in that order.  Key k
        // occupies bytes 8 k .. 8 k + 7 < 8 len, below the elements; the padding keys beyond the
        // list may cover the elements, so they are written afterwards.
        for (int k = lane; k < nlist; k += 64) {
          const uint64_t e = el[k];
          keys[k] = (e & 0xffffffff00000000ull) | (uint32_t)k;
          list[k] = (int)(uint32_t)e;
        }
        wave_sync<kLds>();
        for (int k = nlist + lane; k < P; k += 64) keys[k] = ~0ull;
      }
      wave_sync<kLds>();
      PHASE(6);
      bitonic_sort<kLds ? kLineCap / 128 : 0>(keys, P);
      PHASE(7);
      // centroids in sorted order (sums in input order within a voxel): 64 sorted points at a
      // time are staged in LDS; the voxel still open at the end of a window carries over.
      int nout = 0;
      P4 carry{0.f, 0.f, 0.f, 0.f};
      int carry_n = 0;
      for (int b = 0; b < nlist; b += 64) {
        const int k = b + lane;
        const int wl = min(64, nlist - b);  // window length
        const bool valid = k < nlist;
        uint32_t v = 0xffffffffu, vprev = 0xffffffffu;
        if (valid) {
          const uint64_t key = keys[k];
          v = (uint32_t)(key >> 32);
          stage[lane] = ld4(cloud + off + list[(uint32_t)key]);
          if (k > 0) vprev = (uint32_t)(keys[k - 1] >> 32);
        }
        const bool start = valid && (k == 0 || v != vprev);
        const uint64_t m = __ballot(start);
        wave_sync<kLds>();
        const bool last = b + 64 >= nlist;
        const bool cont = carry_n > 0 && !(m & 1ull);  // window opens inside the carried voxel
        int extra = 0;
        if (carry_n > 0 && (m & 1ull)) {  // the carried voxel closed exactly at the window edge
          if (lane == 0) {
            const float n = (float)carry_n;
            P4 c = carry;
            c.x /= n; c.y /= n; c.z /= n; c.i /= n;
            st4(o_lflat + nout, c);
          }
          extra = 1;
        }
        const bool head = start || (lane == 0 && cont);
        const uint64_t after = lane == 63 ? 0ull : (m >> (lane + 1)) << (lane + 1);
        const int end = after ? (int)first_lane(after) : wl;
        const bool closed = head && (end < wl || last);
        P4 c{0.f, 0.f, 0.f, 0.f};
        int n = 0;
        if (head) {
          int e = lane;
          if (start) {
            c = stage[lane];
            e = lane + 1;
            n = 1;
          } else {
            c = carry;
            n = carry_n;
          }
          for (; e < end; e++) {
            const P4 p = stage[e];
            c.x += p.x; c.y += p.y; c.z += p.z; c.i += p.i;
            n++;
          }
        }
        const uint64_t cm = __ballot(closed);
        if (closed) {
          const float fn = (float)n;
          P4 o = c;
          o.x /= fn; o.y /= fn; o.z /= fn; o.i /= fn;
          st4(o_lflat + nout + extra + __popcll(cm & lanemask_lt()), o);
        }
        nout += extra + __popcll(cm);
        // the open voxel (a head that reached the window end) becomes the carry
        const uint64_t om = __ballot(head && !closed);
        if (om) {
          const int src = (int)first_lane(om);
          carry.x = __shfl(c.x, src); carry.y = __shfl(c.y, src);
          carry.z = __shfl(c.z, src); carry.i = __shfl(c.i, src);
          carry_n = __shfl(n, src);
        } else {
          carry_n = 0;
        }
        wave_sync<kLds>();
      }
      cnt.less_flat = nout;
      PHASE(8);
    }
  }
  if (lane == 0) {
    int* c = a.line_counts + ((size_t)s * H + line) * 4;
    c[0] = cnt.sharp; c[1] = cnt.less_sharp; c[2] = cnt.flat; c[3] = cnt.less_flat;
  }
  PHASE_FLUSH;
}

// ------------------------------------------------------------------ register-resident line
// The line kernel's fast path keeps the whole line in registers: lane l holds points l + 64 t in
// slot t (t < kS), with per-lane bitmasks over the slots for the picked / label flags.  Only the
// link masks (uniform, for the suppression), the pick lists and a 64-point centroid window live
// in LDS (about 2 KiB), so occupancy is set by registers, not by a line-sized LDS footprint.

// Same results as line_body (which documents the reference semantics); the differences are only
// where the state lives.
template <int kS>
__device__ __forceinline__ void line_body_reg(const FeatureArgs& a, int s, int line, LineLists& ll, uint64_t* lmask,
                                              float* curvl, P4* stage, P4* ring, uint32_t* vel, uint16_t* vidx) {
  const int lane = lane_id();
  const int N = a.N, H = a.H;
  const int* lo = a.line_off + (size_t)s * (H + 1);
  const int off = lo[line];
  const int len = lo[line + 1] - off;
  const int total = lo[H];
  const int nsl = (len + 63) >> 6;  // slots in use
  const P4* cloud = a.cloud + (size_t)s * N;
  float* curv = a.curv + (size_t)s * N;
  int8_t* glabel = a.label + (size_t)s * N;
  PHASE_BEGIN;

  // curvature (scanRegistration.cpp:397-412) and neighbour links (suppress).  Every point of the
  // line (and the 64 before / after it) is loaded once: slot t's neighbours come from an LDS ring
  // of three 64-point slots (t - 1, t, t + 1), the next slot's load in flight meanwhile.
  uint32_t linkb = 0;
  // the box of the points inside the six segments ([sI, eI), a superset of the VoxelGrid's input)
  float bmn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, bmx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
  auto ld_slot = [&](int t) -> P4 {  // cloud point off + 64 t + lane (zero outside the cloud)
    const int i = off + 64 * t + lane;
    return (i >= 0 && i < total) ? ld4(cloud + i) : P4{0.f, 0.f, 0.f, 0.f};
  };
  auto ring_at = [&](int t) -> P4* { return ring + 64 * ((t + 3) % 3); };  // slot t >= -1
  ring_at(-1)[lane] = ld_slot(-1);
  ring_at(0)[lane] = ld_slot(0);
  P4 nxt = ld_slot(1);
#pragma unroll
  for (int t = 0; t < kS; t++) {
    if (t >= nsl) continue;
    ring_at(t + 1)[lane] = nxt;
    if (t + 1 < nsl) nxt = ld_slot(t + 2);
    wave_sync<true>();
    const int k = lane + 64 * t;
    if (k < len) {
      const int i = off + k;
      // point k + d of the line: slot t + ((lane + d + 64) >> 6) - 1, lane (lane + d) & 63
      auto nb = [&](int d) -> P4 {
        const int j = lane + d + 64;
        return ring_at(t + (j >> 6) - 1)[j & 63];
      };
      float c = 0.f;
      if (i >= 5 && i < total - 5) {
        P4 q[11];
#pragma unroll
        for (int d = 0; d < 11; d++) q[d] = nb(d - 5);
        const float dX = q[0].x + q[1].x + q[2].x + q[3].x + q[4].x - 10 * q[5].x + q[6].x + q[7].x + q[8].x + q[9].x + q[10].x;
        const float dY = q[0].y + q[1].y + q[2].y + q[3].y + q[4].y - 10 * q[5].y + q[6].y + q[7].y + q[8].y + q[9].y + q[10].y;
        const float dZ = q[0].z + q[1].z + q[2].z + q[3].z + q[4].z - 10 * q[5].z + q[6].z + q[7].z + q[8].z + q[9].z + q[10].z;
        c = dX * dX + dY * dY + dZ * dZ;
      }
      curv[i] = c;
      curvl[k] = c;
      if (k >= 5 && k < len - 6) {
        const P4 p = nb(0);
        bmn[0] = fminf(bmn[0], p.x); bmn[1] = fminf(bmn[1], p.y); bmn[2] = fminf(bmn[2], p.z);
        bmx[0] = fmaxf(bmx[0], p.x); bmx[1] = fmaxf(bmx[1], p.y); bmx[2] = fmaxf(bmx[2], p.z);
      }
      if (k + 1 < len) {
        const P4 p0 = nb(0), p1 = nb(1);
        const float dx = p1.x - p0.x, dy = p1.y - p0.y, dz = p1.z - p0.z;
        if (!((double)(dx * dx + dy * dy + dz * dz) > 0.05)) linkb |= 1u << t;
      }
    }
    wave_sync<true>();  // slot t - 1's ring entry is overwritten next
  }
  // lmask[1 + t]: link bits of points 64 t .. 64 t + 63; lmask[0] / lmask[kS + 1] stay zero
#pragma unroll
  for (int t = 0; t < kS; t++) {
    const uint64_t m = t < nsl ? __ballot((linkb >> t) & 1u) : 0ull;
    if (lane == 0) lmask[1 + t] = m;
  }
  if (lane == 0) { lmask[0] = 0; lmask[kS + 1] = 0; }
#pragma unroll
  for (int d = 0; d < 3; d++) {  // wave-uniform from here on
    for (int o = 32; o > 0; o >>= 1) {
      bmn[d] = fminf(bmn[d], __shfl_xor(bmn[d], o));
      bmx[d] = fmaxf(bmx[d], __shfl_xor(bmx[d], o));
    }
    bmn[d] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, bmn[d])));
    bmx[d] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, bmx[d])));
  }
  wave_sync<true>();
  PHASE(0);

  // The six segments are walked one at a time in a window of kW register slots: window slot u,
  // lane l holds line point wb + 64 u + l (wb = the segment's start rounded down to a slot), which
  // covers the segment and the 5 points a pick past its end can mark.  Marks below wb fall into
  // earlier segments, which no later walk reads.  The window's curvature comes from LDS (curvl);
  // the per-lane slot bitmasks of the whole line (pick / lsh / shp / flt) are shifted in and out.
  constexpr int kSeg = (64 * kS - 11 + 5) / 6;  // longest segment of a line of 64 kS points
  constexpr int kW = (68 + kSeg + 63) / 64;
  // Suppression (scanRegistration.cpp:481-504) of pick ind, ind itself included: forward marks
  // ind+1.. while link[ind], link[ind+1], ... hold (at most 5), backward ind-1.. while
  // link[ind-1], ... hold.
  uint32_t pick = 0, lsh = 0, shp = 0, flt = 0;  // per-lane slot bitmasks
  auto mark = [&](int ind, int wb, uint32_t& pw) {
    const int ti = ind >> 6, b = ind & 63;
    const uint64_t Wm = lmask[ti], W0 = lmask[ti + 1], W1 = lmask[ti + 2];
    const uint32_t fwd5 = (uint32_t)((b == 0 ? W0 : ((W0 >> b) | (W1 << (64 - b)))) & 31u);       // link[ind .. ind+4]
    const uint32_t bwd5 = (uint32_t)((b >= 5 ? (W0 >> (b - 5)) : ((W0 << (5 - b)) | (Wm >> (59 + b)))) & 31u);  // link[ind-5 .. ind-1]
    const uint32_t fz = ~fwd5 & 31u, bz = ~bwd5 & 31u;
    const int nf = fz ? (int)__builtin_ctz(fz) : 5;
    const int nb = bz ? 4 - (31 - (int)__builtin_clz(bz)) : 5;
    const int k0 = ind - nb, k1 = ind + nf;
#pragma unroll
    for (int u = 0; u < kW; u++) {
      const int k = wb + 64 * u + lane;
      if (k >= k0 && k <= k1) pw |= 1u << u;
    }
  };

  int n_sharp = 0, n_lsharp = 0, n_flat = 0;
  const int sI = 5, eI = len - 6;  // scanStartInd / scanEndInd relative to off
  const bool segs = eI - sI >= 6;
  if (segs) {
    for (int j = 0; j < 6; j++) {
      const int sp = sI + (eI - sI) * j / 6;
      const int ep = sI + (eI - sI) * (j + 1) / 6 - 1;
      const int t0 = sp >> 6, wb = 64 * t0;
      uint64_t kw[kW];
      uint32_t es = 0, ef = 0;  // window slots passing the sharp (> 0.1) / flat (< 0.1) test
#pragma unroll
      for (int u = 0; u < kW; u++) {
        const int k = wb + 64 * u + lane;
        const bool in = k >= sp && k <= ep;
        const float c = in ? curvl[k] : 0.f;
        kw[u] = ((uint64_t)__float_as_uint(c) << 32) | (uint32_t)k;
        if (in && (double)c > 0.1) es |= 1u << u;
        if (in && (double)c < 0.1) ef |= 1u << u;
      }
      uint32_t pw = (pick >> t0) & ((1u << kW) - 1u), lw = 0, sw = 0, fw = 0;
      // Equal curvatures (TIES_REFERENCE): the walks reach them in std::sort's order.  While no
      // pick meets a tie the keys stay (curvature, index); the first pick whose extreme curvature
      // is shared by another candidate replays the segment's sort (introsort_order_lds on the
      // dead curvature ring) and re-keys the window by sorted position, a refinement of the
      // curvature order, so the picks made so far stand.
      bool by_pos = a.ties != LISLAM_TIES_REFERENCE;  // true: no replay wanted / already done
      auto replay = [&]() {
        const int n = ep - sp + 1;
        uint32_t* sel = reinterpret_cast<uint32_t*>(ring);
        uint16_t* sidx = reinterpret_cast<uint16_t*>(sel + kSeg);
        for (int i = lane; i < n; i += 64) sel[i] = (uint32_t)i;
        wave_sync<true>();
        auto kof = [&](uint32_t e) { return __float_as_uint(curvl[sp + (int)e]); };
        introsort_order_lds<kS>(sel, kof, n, sidx, sidx + (n / 2 + 1));
        wave_sync<true>();
        final_positions<true>(sel, kof, n, sidx);
#pragma unroll
        for (int u = 0; u < kW; u++) {
          const int k = wb + 64 * u + lane;
          kw[u] = k >= sp && k <= ep ? ((uint64_t)sidx[k - sp] << 32) | (uint32_t)k : 0ull;
        }
        by_pos = true;
      };
      auto max_key = [&](uint32_t ok) {
        uint64_t best = 0;
#pragma unroll
        for (int u = 0; u < kW; u++)
          if ((ok >> u) & 1u) best = kw[u] > best ? kw[u] : best;
        return wave_max_u64(best);
      };
      auto min_key = [&](uint32_t ok) {
        uint64_t best = ~0ull;
#pragma unroll
        for (int u = 0; u < kW; u++)
          if ((ok >> u) & 1u) best = kw[u] < best ? kw[u] : best;
        return wave_min_u64(best);
      };
      // The extreme key over the ok slots (as max_key / min_key) and, folded into the same
      // reduction, tie_at's verdict: whether another ok candidate shares its curvature — the lanes
      // whose own extreme has the wave's extreme curvature, and how many of their slots have it.
      auto extreme_key_tie = [&](uint32_t ok, bool largest, bool& tie) {
        uint64_t best = largest ? 0ull : ~0ull;
#pragma unroll
        for (int u = 0; u < kW; u++)
          if ((ok >> u) & 1u) best = (largest ? kw[u] > best : kw[u] < best) ? kw[u] : best;
        const uint32_t bh = (uint32_t)(best >> 32), bl = (uint32_t)best;
        int cnt = 0;
#pragma unroll
        for (int u = 0; u < kW; u++) cnt += (((ok >> u) & 1u) && (uint32_t)(kw[u] >> 32) == bh) ? 1 : 0;
        const uint32_t m = largest ? wave_umax(bh) : wave_umin(bh);
        const uint64_t tm = __ballot(bh == m);
        uint32_t l;
        if (__popcll(tm) == 1) {
          const int src = (int)__builtin_ctzll(tm);
          l = (uint32_t)__builtin_amdgcn_readlane((int)bl, src);
          tie = __builtin_amdgcn_readlane(cnt, src) > 1;
        } else {
          l = largest ? wave_umax(bh == m ? bl : 0u) : wave_umin(bh == m ? bl : 0xffffffffu);
          tie = true;
        }
        return ((uint64_t)m << 32) | l;
      };
      // ---- sharp picks: largest key first (:450-506); at most 20 per segment
      for (int largest = 1; largest <= 20; largest++) {
        const uint32_t ok = es & ~pw;
        bool tie = false;
        uint64_t best = extreme_key_tie(ok, true, tie);
        if (best == 0) break;  // no unpicked point with curvature > 0.1 is left
        if (!by_pos && tie) {
          replay();
          best = max_key(ok);
        }
        const int ind = (int)(uint32_t)best;
        if (lane == 0) {
          if (largest <= 2) ll.sharp[n_sharp] = ind;
          ll.less_sharp[n_lsharp] = ind;
        }
        if (lane == (ind & 63)) {
          const uint32_t bit = 1u << ((ind - wb) >> 6);
          lw |= bit;
          if (largest <= 2) sw |= bit;
        }
        if (largest <= 2) n_sharp++;
        n_lsharp++;
        mark(ind, wb, pw);
      }
      PHASE(2);
      // ---- flat picks: smallest key first (:511-568); the 4th pick ends the walk unmarked
      for (int smallest = 1; smallest <= 4; smallest++) {
        const uint32_t ok = ef & ~pw;
        bool tie = false;
        uint64_t best = extreme_key_tie(ok, false, tie);
        if (best == ~0ull) break;
        if (!by_pos && tie) {
          replay();
          best = min_key(ok);
        }
        const int ind = (int)(uint32_t)best;
        if (lane == 0) ll.flat[n_flat] = ind;
        if (lane == (ind & 63)) fw |= 1u << ((ind - wb) >> 6);
        n_flat++;
        if (smallest == 4) break;
        mark(ind, wb, pw);
      }
      pick |= pw << t0;
      lsh |= lw << t0;
      shp |= sw << t0;
      flt |= fw << t0;
      PHASE(3);
    }
  }
  // labels (parity tests) and the picked points in pick order
#pragma unroll
  for (int t = 0; t < kS; t++) {
    const int k = lane + 64 * t;
    if (t < nsl && k < len) {
      const uint32_t bit = 1u << t;
      glabel[off + k] = (shp & bit) ? 2 : (lsh & bit) ? 1 : (flt & bit) ? -1 : 0;
    }
  }
  wave_sync<true>();  // the pick lists
  P4* o_sharp = a.stg_sharp + ((size_t)s * H + line) * kCapSharpPerLine;
  P4* o_lsharp = a.stg_less_sharp + ((size_t)s * H + line) * kCapLessSharpPerLine;
  P4* o_flat = a.stg_flat + ((size_t)s * H + line) * kCapFlatPerLine;
  P4* o_lflat = a.stg_less_flat + (size_t)s * N + off;
  {  // every pick's load in flight before the first store (<= 12 / 120 / 24 picks per line)
    static_assert(kCapSharpPerLine <= 64 && kCapLessSharpPerLine <= 128 && kCapFlatPerLine <= 64, "pick lanes");
    const P4 z{0.f, 0.f, 0.f, 0.f};
    const P4 ps = lane < n_sharp ? ld4(cloud + off + ll.sharp[lane]) : z;
    const P4 pl0 = lane < n_lsharp ? ld4(cloud + off + ll.less_sharp[lane]) : z;
    const P4 pl1 = lane + 64 < n_lsharp ? ld4(cloud + off + ll.less_sharp[lane + 64]) : z;
    const P4 pf = lane < n_flat ? ld4(cloud + off + ll.flat[lane]) : z;
    if (lane < n_sharp) st4(o_sharp + lane, ps);
    if (lane < n_lsharp) st4(o_lsharp + lane, pl0);
    if (lane + 64 < n_lsharp) st4(o_lsharp + lane + 64, pl1);
    if (lane < n_flat) st4(o_flat + lane, pf);
  }
  wave_sync<true>();  // the pick lists are dead: their LDS becomes the voxel phase's (LineLds)
  // less-flat points (:570-577): label <= 0 inside the six segments, in index order
  uint32_t lfl = 0;
  int nlist = 0;
#pragma unroll
  for (int t = 0; t < kS; t++) {
    const int k = lane + 64 * t;
    const bool f = t < nsl && segs && k >= sI && k < eI && !((lsh >> t) & 1u);
    if (f) lfl |= 1u << t;
    if (t < nsl) nlist += __popcll(__ballot(f));
  }
  PHASE(5);

  // ---- VoxelGrid(0.2) of the line's less-flat points (PCL VoxelGrid::applyFilter semantics)
  // The voxel index is a mixed-radix number (z, y, x) over the box's leaf coordinates; over any box
  // that encloses the points it orders them the same way (lexicographically in z, y, x) and is equal
  // exactly for points of one leaf, so the sort, std::sort's order of equal voxels and the centroids
  // do not depend on which enclosing box is used.  The segments' box from the curvature pass serves
  // unless its index range overflows; then the exact box of the less-flat points (PCL's own leaf-size
  // check is on that box, and it cannot fail when the larger box passes).
  int n_lflat = 0;
  if (nlist > 0) {
    const float inv = 1.0f / 0.2f;
    float mn[3] = {bmn[0], bmn[1], bmn[2]}, mx[3] = {bmx[0], bmx[1], bmx[2]};
    auto box_size = [&]() {
      const int64_t ex = (int64_t)((mx[0] - mn[0]) * inv) + 1;
      const int64_t ey = (int64_t)((mx[1] - mn[1]) * inv) + 1;
      const int64_t ez = (int64_t)((mx[2] - mn[2]) * inv) + 1;
      int64_t nv = 1;  // the index range: the leaves spanned per axis
#pragma unroll
      for (int d = 0; d < 3; d++) nv *= (int64_t)((int)floorf(mx[d] * inv) - (int)floorf(mn[d] * inv) + 1);
      return max(ex * ey * ez, nv);
    };
    if (box_size() > (int64_t)2147483647) {
#pragma unroll
      for (int d = 0; d < 3; d++) { mn[d] = 3.4e38f; mx[d] = -3.4e38f; }
#pragma unroll
      for (int t = 0; t < kS; t++) {
        if (!((lfl >> t) & 1u)) continue;
        const P4 p = ld4(cloud + off + lane + 64 * t);
        mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
        mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
      }
      for (int d = 0; d < 3; d++) {
        for (int o = 32; o > 0; o >>= 1) {
          mn[d] = fminf(mn[d], __shfl_xor(mn[d], o));
          mx[d] = fmaxf(mx[d], __shfl_xor(mx[d], o));
        }
      }
    }
    const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
    const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
    const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
    if (dx * dy * dz > (int64_t)2147483647) {  // PCL: leaf too small -> copy the input
      int base = 0;
#pragma unroll
      for (int t = 0; t < kS; t++) {
        if (t >= nsl) continue;
        const bool f = (lfl >> t) & 1u;
        const uint64_t m = __ballot(f);
        if (f) st4(o_lflat + base + __popcll(m & lanemask_lt()), ld4(cloud + off + lane + 64 * t));
        base += __popcll(m);
      }
      n_lflat = nlist;
    } else {
      int minb[3], divb[3];
      for (int d = 0; d < 3; d++) {
        minb[d] = (int)floorf(mn[d] * inv);
        divb[d] = (int)floorf(mx[d] * inv) - minb[d] + 1;
      }
      const int mul1 = divb[0], mul2 = divb[0] * divb[1];
      // keys (voxel index, point index): the point index orders like the list position
      uint64_t key[kS];
#pragma unroll
      for (int t = 0; t < kS; t++) {
        key[t] = ~0ull;
        if ((lfl >> t) & 1u) {
          const int k = lane + 64 * t;
          const P4 p = ld4(cloud + off + k);
          const int i0 = (int)(floorf(p.x * inv) - (float)minb[0]);
          const int i1 = (int)(floorf(p.y * inv) - (float)minb[1]);
          const int i2 = (int)(floorf(p.z * inv) - (float)minb[2]);
          const uint32_t idx = (uint32_t)(i0 + i1 * mul1 + i2 * mul2);
          key[t] = ((uint64_t)idx << 32) | (uint32_t)k;
        }
      }
      // std::sort's order of equal voxels (introsort_order): the list in LDS, in list order, as
      // 32-bit elements (sort key, line position), reordered as the introsort loop leaves it; the
      // keys then become (voxel, position after the loop, line position) for the stable sort
      // below.  Voxel indices below 2^21 pack with the 11-bit line position directly; otherwise a
      // first sort of (voxel, list position) numbers the voxels densely for the element.
      int sort_to = 64 * kS;  // the bitonic network's last level (none when key[] is already sorted)
      if (a.ties == LISLAM_TIES_REFERENCE) {
        uint32_t vmax = 0u;
#pragma unroll
        for (int t = 0; t < kS; t++)
          if ((lfl >> t) & 1u) vmax = max(vmax, (uint32_t)(key[t] >> 32));
        for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o));
        const bool packed = vmax < (1u << 21);
        int base = 0;
#pragma unroll
        for (int t = 0; t < kS; t++) {  // list positions: ballot prefix over the line
          if (t >= nsl) continue;
          const bool f = (lfl >> t) & 1u;
          const uint64_t m = __ballot(f);
          const int j = base + __popcll(m & lanemask_lt());
          if (f && packed) vel[j] = ((uint32_t)(key[t] >> 32) << 11) | (uint32_t)(lane + 64 * t);
          if (f && !packed)
            key[t] = (key[t] & 0xffffffff00000000ull) | ((uint32_t)j << 16) | (uint32_t)(lane + 64 * t);
          base += __popcll(m);
        }
        PHASE(6);
        if (packed) {
          wave_sync<true>();
          introsort_order_lds<kS>(vel, [](uint32_t e) { return e >> 11; }, nlist, vidx, vidx + 32 * kS + 1);
          PHASE(12);
          // std::__final_insertion_sort: the loop leaves blocks of at most 16 elements (or
          // heap-sorted ranges) in key order, and the insertion sort stably sorts each block.  An
          // element's final position is therefore its position, minus the greater keys among the
          // 15 positions before it, plus the smaller keys among the 15 after it (earlier blocks
          // hold no greater key and later blocks no smaller one, so the window needs no block
          // bounds).  The permutation is written back in place, then read in sorted order.
          // The window reads past the list's ends land on sentinels (LineLds pads vel by 16 words
          // on each side): 0 before it (no greater key), all ones after it (no smaller key), so
          // the window needs no bounds tests either; keys are compared packed, against the
          // element's own key rounded to the key field.
          if (lane < 16) {
            vel[lane - 16] = 0u;
            vel[nlist + lane] = 0xffffffffu;
          }
          wave_sync<true>();
#pragma unroll 1
          for (int t = 0; t < kS; t++) {  // final positions, into the (dead) partition scratch
            if (64 * t >= nlist) break;
            const int j = lane + 64 * t;
            if (j < nlist) {
              const uint32_t e = vel[j];
              const uint32_t gt = e | 0x7ffu;   // packed > this: a greater key
              const uint32_t lt = e & ~0x7ffu;  // packed < this: a smaller key
              int mv = 0;
#pragma unroll
              for (int d = 1; d <= 15; d++) {
                mv -= (int)(vel[j - d] > gt);
                mv += (int)(vel[j + d] < lt);
              }
              vidx[j] = (uint16_t)(j + mv);
            }
          }
          wave_sync<true>();
          uint32_t el[kS];
#pragma unroll
          for (int t = 0; t < kS; t++) el[t] = lane + 64 * t < nlist ? vel[lane + 64 * t] : 0u;
          wave_sync<true>();
#pragma unroll
          for (int t = 0; t < kS; t++)
            if (lane + 64 * t < nlist) vel[vidx[lane + 64 * t]] = el[t];
          wave_sync<true>();
#pragma unroll
          for (int t = 0; t < kS; t++) {
            const int j = lane + 64 * t;
            const uint32_t e = j < nlist ? vel[j] : 0u;
            key[t] = j < nlist ? ((uint64_t)(e >> 11) << 32) | ((uint32_t)j << 16) | (e & 0x7ffu) : ~0ull;
          }
          sort_to = 1;
        } else {
          reg_bitonic<kS>(key);
          uint32_t prev_hi = 0xffffffffu;
          int nvox = 0;
#pragma unroll
          for (int t = 0; t < kS; t++) {  // dense voxel numbers in sorted order
            if (64 * t >= nlist) continue;
            const bool valid = lane + 64 * t < nlist;
            const uint32_t v = (uint32_t)(key[t] >> 32);
            const uint32_t up1 = (uint32_t)__builtin_amdgcn_ds_bpermute(((lane + 63) & 63) << 2, (int)v);
            const uint32_t vprev = lane == 0 ? prev_hi : up1;
            prev_hi = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
            const bool start = valid && v != vprev;
            const uint64_t m = __ballot(start);
            const int num = nvox + __popcll(m & lanemask_lt()) + (int)start - 1;
            if (valid) vel[(key[t] >> 16) & 0xffffu] = ((uint32_t)num << 16) | (uint32_t)(key[t] & 0xffffu);
            nvox += __popcll(m);
          }
          wave_sync<true>();
          introsort_order_lds<kS>(vel, [](uint32_t e) { return e >> 16; }, nlist, vidx, vidx + 32 * kS + 1);
#pragma unroll
          for (int t = 0; t < kS; t++) {
            const int j = lane + 64 * t;
            const uint32_t e = j < nlist ? vel[j] : 0u;
            key[t] = j < nlist ? ((uint64_t)(e >> 16) << 32) | ((uint32_t)j << 16) | (e & 0xffffu) : ~0ull;
          }
        }
        PHASE(11);
        wave_sync<true>();
      }
      PHASE(6);
      for (int k = 2; k <= sort_to; k <<= 1) reg_bitonic_level<kS>(key, k, k >> 1, 0);  // reg_bitonic
      PHASE(7);
      // centroids in sorted order (sums in input order within a voxel): window t = sorted
      // positions 64 t .. 64 t + 63, staged in LDS; the voxel still open at the end of a window
      // carries over.
      int nout = 0;
      P4 carry{0.f, 0.f, 0.f, 0.f};
      int carry_n = 0;
      uint32_t prev_hi = 0xffffffffu;  // voxel of sorted position 64 t - 1
#pragma unroll
      for (int t = 0; t < kS; t++) {
        const int b = 64 * t;
        if (b >= nlist) continue;
        const int k = b + lane;
        const int wl = min(64, nlist - b);  // window length
        const bool valid = k < nlist;
        const uint32_t v = (uint32_t)(key[t] >> 32);
        const uint32_t up1 = (uint32_t)__builtin_amdgcn_ds_bpermute(((lane + 63) & 63) << 2, (int)v);  // lane - 1
        const uint32_t vprev = lane == 0 ? prev_hi : up1;
        prev_hi = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
        if (valid) stage[lane] = ld4(cloud + off + (int)((uint32_t)key[t] & 0xffffu));
        const bool start = valid && (k == 0 || v != vprev);
        const uint64_t m = __ballot(start);
        wave_sync<true>();
        const bool last = b + 64 >= nlist;
        const bool cont = carry_n > 0 && !(m & 1ull);  // window opens inside the carried voxel
        int extra = 0;
        if (carry_n > 0 && (m & 1ull)) {  // the carried voxel closed exactly at the window edge
          if (lane == 0) {
            const float n = (float)carry_n;
            P4 c = carry;
            c.x /= n; c.y /= n; c.z /= n; c.i /= n;
            st4(o_lflat + nout, c);
          }
          extra = 1;
        }
        const bool head = start || (lane == 0 && cont);
        const uint64_t after = lane == 63 ? 0ull : (m >> (lane + 1)) << (lane + 1);
        const int end = after ? (int)__builtin_ctzll(after) : wl;
        const bool closed = head && (end < wl || last);
        P4 c{0.f, 0.f, 0.f, 0.f};
        int n = 0;
        if (head) {
          int e = lane;
          if (start) {
            c = stage[lane];
            e = lane + 1;
            n = 1;
          } else {
            c = carry;
            n = carry_n;
          }
          for (; e < end; e++) {
            const P4 p = stage[e];
            c.x += p.x; c.y += p.y; c.z += p.z; c.i += p.i;
            n++;
          }
        }
        const uint64_t cm = __ballot(closed);
        if (closed) {
          const float fn = (float)n;
          P4 o = c;
          o.x /= fn; o.y /= fn; o.z /= fn; o.i /= fn;
          st4(o_lflat + nout + extra + __popcll(cm & lanemask_lt()), o);
        }
        nout += extra + __popcll(cm);
        // the open voxel (a head that reached the window end) becomes the carry
        const uint64_t om = __ballot(head && !closed);
        if (om) {
          const int src = (int)__builtin_ctzll(om);
          carry.x = __shfl(c.x, src); carry.y = __shfl(c.y, src);
          carry.z = __shfl(c.z, src); carry.i = __shfl(c.i, src);
          carry_n = __shfl(n, src);
        } else {
          carry_n = 0;
        }
        wave_sync<true>();
      }
      n_lflat = nout;
      PHASE(8);
    }
  }
  if (lane == 0) {
    int* c = a.line_counts + ((size_t)s * H + line) * 4;
    c[0] = n_sharp; c[1] = n_lsharp; c[2] = n_flat; c[3] = n_lflat;
  }
  PHASE_FLUSH;
}

// kS: register slots per lane of the fast path (lines up to 64 kS points); longer lines (input
// that is not ring-ordered) run line_body on global scratch.
// The wave's LDS is one union over the line's three phases, so that it bounds occupancy as little
// as possible: (sel) the curvature ring, the line's curvature, the walks' link masks and pick lists; (vox) the
// VoxelGrid's std::sort order (introsort_order: the list elements and the partition's index
// scratch); (stage) the centroid windows.  line_body_reg drains the wave's LDS traffic at each
// phase change (wave_sync).
template <int kS>
struct LineLds {
  static constexpr int kIdx = 2 * (32 * kS + 1);
  union {
    struct {
      P4 ring[3 * 64];
      LineLists ll;
      uint64_t lmask[kS + 2];
      float curv[64 * kS];
    } sel;
    struct {
      uint32_t vel[16 + 64 * kS + 16];  // the list at vel + 16; the final positions' sentinels either side
      uint16_t vidx[kIdx];
    } vox;
    P4 stage[64];
  };
};

// Waves per SIMD asked of the 1024-point lines (kS = 16): 4 (113 VGPRs, no scratch).  5 caps
// them at 96 VGPRs with 44 B of scratch per lane for one more resident wave: 2.02 -> 1.96 ms per
// 300 scans isolated in round 2 (profiles/r02v_experiments.txt), within noise on the round-3 tree
// (2.11 / 2.20 vs 2.17 / 2.18 ms, bench 8.59k / 8.56k vs 8.55k / 8.56k scans/s,
// profiles/r03s_lines_wpe_ab.txt), so the spill-free build.  Other line lengths keep the default.
#ifndef LISLAM_LINES_WPE
#define LISLAM_LINES_WPE 4
#endif

template <int kS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kS == 16 ? LISLAM_LINES_WPE : 1))) void k_scan_lines(FeatureArgs a) {
  __shared__ LineLds<kS> m;
#ifdef LISLAM_PHASE_PROF
  const uint64_t t_wave0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int s = blockIdx.x / a.H, line = blockIdx.x % a.H;
  const int* lo = a.line_off + (size_t)s * (a.H + 1);
  const int len = lo[line + 1] - lo[line];
  if (len <= 64 * kS)
    line_body_reg<kS>(a, s, line, m.sel.ll, m.sel.lmask, m.sel.curv, m.stage, m.sel.ring, m.vox.vel + 16, m.vox.vidx);
  else  // the pick lists are dead before the centroid windows are staged
    line_body<false>(a, s, line, nullptr, nullptr, nullptr, nullptr, nullptr, m.sel.ll, m.stage);
#ifdef LISLAM_PHASE_PROF
  if (g_line_log && lane_id() == 0) {  // per-wave start / end (100 MHz), line length
    unsigned long long* o = g_line_log + (size_t)blockIdx.x * 4;
    o[0] = t_wave0;
    o[1] = __builtin_amdgcn_s_memrealtime();
    o[2] = (unsigned long long)len;
    o[3] = 0;
  }
#endif
}

#ifdef LISLAM_PHASE_PROF
extern "C" int lislam_debug_line_log(unsigned long long* dev_buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_line_log), &dev_buf, sizeof(dev_buf)) == hipSuccess ? 0 : -2;
}
extern "C" int lislam_debug_phase_cycles(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_cycles), sizeof(g_phase_cycles)) != hipSuccess) return -2;
  static const unsigned long long zero[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), zero, sizeof(zero)) == hipSuccess ? 0 : -2;
}
#endif

// ------------------------------------------------------------------------------- compaction
// One wave per (scan, line): the line's offsets in the four concatenated clouds are wave sums of
// the earlier lines' counts, then the wave copies its line's staged features.
__global__ __launch_bounds__(64) void k_scan_compact(FeatureArgs a) {
  const int s = blockIdx.x / a.H, l = blockIdx.x % a.H;
  const int H = a.H, N = a.N, lane = lane_id();
  const int* lc = a.line_counts + (size_t)s * H * 4;
  int pre[4], cnt[4];
#pragma unroll
  for (int f = 0; f < 4; f++) {
    uint32_t v = 0;
    for (int k = lane; k < l; k += 64) v += (uint32_t)lc[k * 4 + f];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    pre[f] = (int)v;
    cnt[f] = lc[l * 4 + f];
  }
  if (lane == 0) {
    int* lo1 = a.feat_loff + ((size_t)s * 2 + 0) * (H + 1);
    int* lo3 = a.feat_loff + ((size_t)s * 2 + 1) * (H + 1);
    lo1[l] = pre[1];
    lo3[l] = pre[3];
    if (l == H - 1) {  // totals (sharp, less-sharp, flat, less-flat) and the closing offsets
      lo1[H] = pre[1] + cnt[1];
      lo3[H] = pre[3] + cnt[3];
      for (int f = 0; f < 4; f++) a.n_feat[s * 4 + f] = pre[f] + cnt[f];
    }
  }
  const size_t stg = (size_t)s * H + l;
  for (int k = lane; k < cnt[0]; k += 64)
    st4(a.sharp + (size_t)s * a.cap_sharp + pre[0] + k, ld4(a.stg_sharp + stg * kCapSharpPerLine + k));
  for (int k = lane; k < cnt[1]; k += 64)
    st4(a.less_sharp + (size_t)s * a.cap_less_sharp + pre[1] + k, ld4(a.stg_less_sharp + stg * kCapLessSharpPerLine + k));
  for (int k = lane; k < cnt[2]; k += 64)
    st4(a.flat + (size_t)s * a.cap_flat + pre[2] + k, ld4(a.stg_flat + stg * kCapFlatPerLine + k));
  const int off = a.line_off[(size_t)s * (H + 1) + l];
  for (int k = lane; k < cnt[3]; k += 64)
    st4(a.less_flat + (size_t)s * N + pre[3] + k, ld4(a.stg_less_flat + (size_t)s * N + off + k));
}

// ------------------------------------------------------------------------------- wire format
// sensor_msgs/PointCloud2 points <-> float4 (x, y, z, intensity): fromROSMsg's field-offset
// parsing (image_handler.h_ouster:105-106, scanRegistration.cpp:234-235) and toROSMsg of the
// feature clouds (scanRegistration.cpp:592-642) as device kernels, one thread per point.
__device__ __forceinline__ float ld_f32_bytes(const uint8_t* p) {
  uint32_t u = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
  return __uint_as_float(u);
}
__device__ __forceinline__ void st_f32_bytes(uint8_t* p, float v) {
  const uint32_t u = __float_as_uint(v);
  p[0] = (uint8_t)u; p[1] = (uint8_t)(u >> 8); p[2] = (uint8_t)(u >> 16); p[3] = (uint8_t)(u >> 24);
}
__global__ void k_unpack_layout(const uint8_t* raw, int n, WireLayout L, P4* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = raw + (size_t)i * L.step;
  if (((L.step | L.ox | L.oy | L.oz | L.oi) & 3u) == 0) {  // 4-byte aligned fields (every ROS layout): dword loads
    const float* f = reinterpret_cast<const float*>(p);
    st4(out + i, P4{f[L.ox >> 2], f[L.oy >> 2], f[L.oz >> 2], f[L.oi >> 2]});
    return;
  }
  st4(out + i, P4{ld_f32_bytes(p + L.ox), ld_f32_bytes(p + L.oy), ld_f32_bytes(p + L.oz), ld_f32_bytes(p + L.oi)});
}
// every byte of a point is written: the four fields, zeros elsewhere
__global__ void k_pack_layout(const P4* in, int n, WireLayout L, uint8_t* raw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const P4 v = ld4(in + i);
  uint8_t* p = raw + (size_t)i * L.step;
  for (uint32_t k = 0; k < L.step; k++) p[k] = 0;
  st_f32_bytes(p + L.ox, v.x);
  st_f32_bytes(p + L.oy, v.y);
  st_f32_bytes(p + L.oz, v.z);
  st_f32_bytes(p + L.oi, v.i);
}
void launch_unpack_layout(const uint8_t* raw, int n, const WireLayout& L, P4* out, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(k_unpack_layout, dim3((n + 255) / 256), dim3(256), 0, st, raw, n, L, out);
}
void launch_pack_layout(const P4* in, int n, const WireLayout& L, uint8_t* raw, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(k_pack_layout, dim3((n + 255) / 256), dim3(256), 0, st, in, n, L, raw);
}

void launch_features(const FeatureArgs& a, hipStream_t st, hipEvent_t* ev, hipEvent_t images_ready) {
  // ev (nullable): 4 events bracketing k_scan_front, k_scan_lines, k_scan_compact
  if (ev) (void)hipEventRecord(ev[0], st);
  const int fb = a.S * ((a.fr_R + kFrontWaves - 1) / kFrontWaves);
  hipLaunchKernelGGL(k_front_count, dim3(fb), dim3(64 * kFrontWaves), 0, st, a);
  if (images_ready) (void)hipEventRecord(images_ready, st);  // the a1 images are complete here
  hipLaunchKernelGGL(k_front_scan, dim3(a.S), dim3(kMaxLines), 0, st, a);
  hipLaunchKernelGGL(k_front_scatter, dim3(fb), dim3(64 * kFrontWaves), 0, st, a);
  if (ev) (void)hipEventRecord(ev[1], st);
  if (a.W <= 512)
    hipLaunchKernelGGL(k_scan_lines<8>, dim3(a.S * a.H), dim3(64), 0, st, a);
  else if (a.W <= 1024)
    hipLaunchKernelGGL(k_scan_lines<16>, dim3(a.S * a.H), dim3(64), 0, st, a);
  else
    hipLaunchKernelGGL(k_scan_lines<32>, dim3(a.S * a.H), dim3(64), 0, st, a);
  if (ev) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL(k_scan_compact, dim3(a.S * a.H), dim3(64), 0, st, a);
  if (ev) (void)hipEventRecord(ev[3], st);
}

}  // namespace lislam
