// Developer calibration (GPU box, under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE): kernels that
// read (or write) a known number of bytes with the access patterns of the lislam kernels, so the
// counters' units can be checked per pattern.  Each kernel touches every byte of a 64 MiB buffer
// exactly once:
//   k_stream16  16 B per lane, consecutive (the streaming kernels' float4 loads)
//   k_stream4   4 B per lane, consecutive
//   k_gather16  16 B per lane at a random permutation of the 16-B elements (the target-index /
//               association gathers)
//   k_write16   16 B per lane stores, consecutive
// Prints the byte counts; compare with rocprof's per-kernel FETCH_SIZE / WRITE_SIZE (KiB).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_stream16(const float4* __restrict__ a, float* out, size_t n) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1.2345f) out[0] = acc;
}
__global__ void k_stream4(const float* __restrict__ a, float* out, size_t n) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += a[i];
  if (acc == 1.2345f) out[0] = acc;
}
__global__ void k_gather16(const float4* __restrict__ a, const unsigned* __restrict__ perm, float* out, size_t n) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[perm[i]];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1.2345f) out[0] = acc;
}
__global__ void k_write16(float4* a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_float4((float)i, 0.f, 0.f, 0.f);
}

int main() {
  const size_t bytes = (size_t)64 << 20, n16 = bytes / 16, n4 = bytes / 4;
  float4* a;
  float* out;
  unsigned* perm;
  hipMalloc(&a, bytes);
  hipMalloc(&out, 64);
  hipMalloc(&perm, n16 * 4);
  hipMemset(a, 0, bytes);
  std::vector<unsigned> p(n16);
  for (size_t i = 0; i < n16; i++) p[i] = (unsigned)i;
  unsigned long long s = 0x9E3779B97F4A7C15ull;
  for (size_t i = n16 - 1; i > 0; i--) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const size_t j = s % (i + 1);
    const unsigned t = p[i]; p[i] = p[j]; p[j] = t;
  }
  hipMemcpy(perm, p.data(), n16 * 4, hipMemcpyHostToDevice);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(256), 0, 0, a, out, n16);
  hipLaunchKernelGGL(k_stream4, dim3(4096), dim3(256), 0, 0, (const float*)a, out, n4);
  hipLaunchKernelGGL(k_gather16, dim3(4096), dim3(256), 0, 0, a, perm, out, n16);
  hipLaunchKernelGGL(k_write16, dim3(4096), dim3(256), 0, 0, a, n16);
  hipDeviceSynchronize();
  std::printf("bytes per kernel: read %zu (k_stream16, k_stream4; k_gather16 also reads %zu B of indices), "
              "write %zu (k_write16)\n", bytes, n16 * 4, bytes);
  return 0;
}
