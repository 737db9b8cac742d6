// Device-wide primitives of the map path, hand-written for gfx950 (wave64): ordered compaction by
// flags, exclusive prefix sum, and the stable LSD radix sort of (key, index) pairs that the
// ikd-Tree rebuild, the A-LOAM cube map and the VoxelGrid use (lislam_map.hip).
//
// Every primitive is a few launches on the caller's stream over tiles of kTile elements
// (256 threads x 8 or 16 items, element tile_base + item * 256 + thread: coalesced):
//   count / sum per tile  ->  one workgroup scans the tile totals  ->  per tile, ranks from wave
//   ballots (mbcnt) and an LDS prefix over the 4 waves, items in input order (stable).
// The radix sort is 8 bits per pass: tile digit histograms (LDS atomics), an exclusive scan of the
// digit-major histogram (the same scan), then a scatter that ranks each item row by digit peers
// found with 8 ballots (match-any on the digit) and keeps running per-digit offsets in LDS.
// Scratch: *_temp_bytes(n) bytes of device memory, owned by the caller.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace lislam {
namespace prims {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kItems = 8;                      // compaction / scan: 2048 elements per tile
constexpr int kTile = kThreads * kItems;
constexpr int kSortItems = 16;                 // radix sort: 4096 keys per tile
constexpr int kSortTile = kThreads * kSortItems;
constexpr int kScanMax = 1024 * 16;            // tile totals one workgroup scans in registers

__device__ __forceinline__ int lane_id() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ int popc_below(uint64_t m) {  // set bits of m below this lane
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ int wave_inclusive_sum(int v) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  return v;
}
// Exclusive prefix of v over the workgroup (kThreads threads, thread order); *total = the sum.
__device__ __forceinline__ int block_exclusive_sum(int v, int* lds /*kWaves + 1*/, int* total) {
  const int lane = lane_id(), w = (int)threadIdx.x >> 6;
  const int inc = wave_inclusive_sum(v);
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  int base = 0, all = 0;
#pragma unroll
  for (int k = 0; k < kWaves; k++) {
    const int s = lds[k];
    if (k < w) base += s;
    all += s;
  }
  __syncthreads();
  *total = all;
  return base + inc - v;
}

// ---- tile totals
template <typename F>
__global__ __launch_bounds__(kThreads) void k_tile_count(const F* flags, int n, int* tile_sum) {
  __shared__ int lds[kWaves + 1];
  const int base = blockIdx.x * kTile;
  int c = 0;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const int j = base + i * kThreads + (int)threadIdx.x;
    c += (j < n && flags[j] != 0) ? 1 : 0;
  }
  int total;
  block_exclusive_sum(c, lds, &total);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}
__global__ __launch_bounds__(kThreads) void k_tile_sum(const int* in, int n, int* tile_sum) {
  __shared__ int lds[kWaves + 1];
  const int base = blockIdx.x * kTile;
  int c = 0;
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const int j = base + i * kThreads + (int)threadIdx.x;
    c += j < n ? in[j] : 0;
  }
  int total;
  block_exclusive_sum(c, lds, &total);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

// One workgroup: exclusive scan of the nt tile totals (in place), the grand total to *total.
__global__ __launch_bounds__(1024) void k_scan_tiles(int* tile, int nt, int* total) {
  __shared__ int lds[16 + 1];
  constexpr int kPer = kScanMax / 1024;
  const int t = (int)threadIdx.x, lane = lane_id(), w = t >> 6;
  int v[kPer], s = 0;
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    const int j = t * kPer + i;
    v[i] = j < nt ? tile[j] : 0;
    s += v[i];
  }
  const int inc = wave_inclusive_sum(s);
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  int base = 0, all = 0;
  for (int k = 0; k < 16; k++) {
    const int q = lds[k];
    if (k < w) base += q;
    all += q;
  }
  int run = base + inc - s;
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    const int j = t * kPer + i;
    if (j < nt) tile[j] = run;
    run += v[i];
  }
  if (t == 0 && total) *total = all;
}

// Scans of more tiles than one workgroup holds: tiles of tiles (recursive on the host side).
inline int tiles_of(int n, int tile) { return (n + tile - 1) / tile; }

// ---- ordered compaction: out[rank] = in[j] for flags[j] != 0, rank = flagged elements before j
template <typename T, typename F>
__global__ __launch_bounds__(kThreads) void k_select_scatter(const T* in, const F* flags, int n, const int* tile_off,
                                                             T* out) {
  __shared__ int lds[kWaves + 1];
  const int base = blockIdx.x * kTile;
  int run = tile_off[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const int j = base + i * kThreads + (int)threadIdx.x;
    const bool f = j < n && flags[j] != 0;
    int total;
    const int r = block_exclusive_sum(f ? 1 : 0, lds, &total);
    if (f) out[run + r] = in[j];
    run += total;
  }
}

// ---- exclusive sum: out[j] = sum of in[0..j)
__global__ __launch_bounds__(kThreads) void k_scan_scatter(const int* in, int n, const int* tile_off, int* out) {
  __shared__ int lds[kWaves + 1];
  const int base = blockIdx.x * kTile;
  int run = tile_off[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kItems; i++) {
    const int j = base + i * kThreads + (int)threadIdx.x;
    const int v = j < n ? in[j] : 0;
    int total;
    const int r = block_exclusive_sum(v, lds, &total);
    if (j < n) out[j] = run + r;
    run += total;
  }
}

// Exclusive scan of nt ints in place (device), any nt: one workgroup up to kScanMax, else tiles of
// tiles.  scratch: scan_temp_ints(nt) ints.
inline size_t scan_temp_ints(int nt) {
  size_t s = 0;
  while (nt > kScanMax) {
    const int nb = tiles_of(nt, kTile);
    s += (size_t)nb + (size_t)nt;  // tile sums + a copy
    nt = nb;
  }
  return s + 1;
}
inline void scan_inplace(int* a, int nt, int* scratch, int* total, hipStream_t st) {
  if (nt <= kScanMax) {
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, st, a, nt, total);
    return;
  }
  const int nb = tiles_of(nt, kTile);
  int* sums = scratch;
  int* copy = scratch + nb;
  hipLaunchKernelGGL(k_tile_sum, dim3(nb), dim3(kThreads), 0, st, a, nt, sums);
  scan_inplace(sums, nb, copy + nt, total, st);
  (void)hipMemcpyAsync(copy, a, sizeof(int) * (size_t)nt, hipMemcpyDeviceToDevice, st);
  hipLaunchKernelGGL(k_scan_scatter, dim3(nb), dim3(kThreads), 0, st, copy, nt, sums, a);
}

// Compaction: bytes of scratch, then the call (count: device int, the number selected).
inline size_t select_temp_bytes(int n) {
  const int nb = tiles_of(std::max(n, 1), kTile);
  return sizeof(int) * ((size_t)nb + scan_temp_ints(nb) + 4);
}
template <typename T, typename F>
hipError_t select_flagged(void* tmp, const T* in, const F* flags, T* out, int* count, int n, hipStream_t st) {
  if (n <= 0) return hipMemsetAsync(count, 0, sizeof(int), st);
  const int nb = tiles_of(n, kTile);
  int* tiles = static_cast<int*>(tmp);
  hipLaunchKernelGGL(k_tile_count<F>, dim3(nb), dim3(kThreads), 0, st, flags, n, tiles);
  scan_inplace(tiles, nb, tiles + nb, count, st);
  hipLaunchKernelGGL((k_select_scatter<T, F>), dim3(nb), dim3(kThreads), 0, st, in, flags, n, tiles, out);
  return hipGetLastError();
}

// Exclusive sum of n ints.
inline size_t exclusive_sum_temp_bytes(int n) { return select_temp_bytes(n); }
inline hipError_t exclusive_sum(void* tmp, const int* in, int* out, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int nb = tiles_of(n, kTile);
  int* tiles = static_cast<int*>(tmp);
  hipLaunchKernelGGL(k_tile_sum, dim3(nb), dim3(kThreads), 0, st, in, n, tiles);
  scan_inplace(tiles, nb, tiles + nb, nullptr, st);
  hipLaunchKernelGGL(k_scan_scatter, dim3(nb), dim3(kThreads), 0, st, in, n, tiles, out);
  return hipGetLastError();
}

// ---- stable LSD radix sort of (key, int) pairs, 8 bits per pass
template <typename K>
__global__ __launch_bounds__(kThreads) void k_radix_hist(const K* keys, int n, int shift, int nb, int* hist) {
  __shared__ int h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int base = blockIdx.x * kSortTile;
#pragma unroll 4
  for (int i = 0; i < kSortItems; i++) {
    const int j = base + i * kThreads + (int)threadIdx.x;
    if (j < n) atomicAdd(&h[(unsigned)(keys[j] >> shift) & 255u], 1);
  }
  __syncthreads();
  hist[threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];  // digit-major: the scan orders by (digit, tile)
}

template <typename K>
__global__ __launch_bounds__(kThreads) void k_radix_scatter(const K* ki, const int* vi, int n, int shift, int nb,
                                                            const int* hist_off, K* ko, int* vo) {
  __shared__ int run[256];           // running output offset of each digit
  __shared__ int wcnt[kWaves][256];  // this row's count of each digit per wave
  const int t = (int)threadIdx.x, lane = lane_id(), w = t >> 6;
  run[t] = hist_off[t * nb + blockIdx.x];
  const int base = blockIdx.x * kSortTile;
  for (int i = 0; i < kSortItems; i++) {
    const int j = base + i * kThreads + t;
    const bool ok = j < n;
    K k = ok ? ki[j] : K(0);
    const int v = ok ? vi[j] : 0;
    const unsigned d = ok ? (unsigned)(k >> shift) & 255u : 256u;
    // lanes of this wave with the same digit (match-any by 8 ballots); absent lanes match nobody
    uint64_t peers = __ballot(ok);
    if (!ok) peers = 0ull;
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const uint64_t m = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? m : ~m;
    }
    const int below = popc_below(peers);
#pragma unroll
    for (int q = 0; q < kWaves; q++) wcnt[q][t] = 0;
    __syncthreads();
    if (ok && below == 0) wcnt[w][d] = __popcll(peers);  // the first lane of each digit group
    __syncthreads();
    int pos = 0;
    if (ok) {
      pos = run[d] + below;
      for (int q = 0; q < w; q++) pos += wcnt[q][d];
      ko[pos] = k;
      vo[pos] = v;
    }
    __syncthreads();
    int add = 0;
#pragma unroll
    for (int q = 0; q < kWaves; q++) add += wcnt[q][t];
    run[t] += add;
    __syncthreads();
  }
}

inline size_t sort_temp_bytes(int n) {
  const int nb = tiles_of(std::max(n, 1), kSortTile);
  const int nh = 256 * nb;
  return sizeof(int) * ((size_t)nh + scan_temp_ints(nh) + 4);
}
// Stable sort of n (key, value) pairs by the low `bits` bits of the key (a multiple of 8): the
// result in ko / vo.  ki / vi are the other ping-pong buffer and are left modified.
template <typename K>
hipError_t sort_pairs(void* tmp, K* ki, K* ko, int* vi, int* vo, int n, int bits, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int nb = tiles_of(n, kSortTile);
  int* hist = static_cast<int*>(tmp);
  int* scr = hist + 256 * nb;
  const int passes = bits / 8;
  K* src_k = ki;
  int* src_v = vi;
  for (int p = 0; p < passes; p++) {  // pass p writes ko / vo when p is even, ki / vi when odd
    K* dst_k = (p & 1) ? ki : ko;
    int* dst_v = (p & 1) ? vi : vo;
    hipLaunchKernelGGL(k_radix_hist<K>, dim3(nb), dim3(kThreads), 0, st, src_k, n, 8 * p, nb, hist);
    scan_inplace(hist, 256 * nb, scr, nullptr, st);
    hipLaunchKernelGGL(k_radix_scatter<K>, dim3(nb), dim3(kThreads), 0, st, src_k, src_v, n, 8 * p, nb, hist, dst_k, dst_v);
    src_k = dst_k;
    src_v = dst_v;
  }
  if (src_k != ko) {  // an even number of passes ends in ki / vi
    hipError_t e = hipMemcpyAsync(ko, ki, sizeof(K) * (size_t)n, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(vo, vi, sizeof(int) * (size_t)n, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

}  // namespace prims
}  // namespace lislam
