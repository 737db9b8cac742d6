// Co-residency limits beside the engine's item workgroups (developer tool): a persistent spinner of
// (CUs - 8) workgroups x 512 threads, 128 VGPRs, 10 KB LDS (k_odom_items' footprint) on a CU-masked
// stream; then probe kernels of a given LDS size / VGPR count / workgroup size on a second stream
// with the same mask.  Prints whether each probe completes while the spinner holds the CUs.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/micro/corun2 scripts/micro/corun2.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512, 4) void spin(volatile int* flag, float* sink, unsigned long long bound) {
  __shared__ float lds[2560];  // 10 KB
  lds[threadIdx.x] = threadIdx.x;
  asm volatile("" ::: "v127");
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (*flag == 0 && __builtin_amdgcn_s_memrealtime() - t0 < bound) __builtin_amdgcn_s_sleep(8);
  if (lds[threadIdx.x ^ 1] == -1.f) sink[blockIdx.x] = 1.f;
}

#define PROBE(NAME, THREADS, LDSB, VREG)                                  \
  __global__ __launch_bounds__(THREADS) void NAME(int* out) {             \
    __shared__ int lds[(LDSB) / 4];                                       \
    lds[threadIdx.x] = threadIdx.x;                                       \
    asm volatile("" ::: VREG);                                            \
    __syncthreads();                                                      \
    if (threadIdx.x == 0) out[blockIdx.x] = lds[5] + 1;                   \
  }
PROBE(p_lds64k, 1024, 65536, "v7")
PROBE(p_lds66k, 1024, 67584, "v7")
PROBE(p_lds72k, 1024, 73728, "v7")
PROBE(p_lds80k, 1024, 81920, "v7")
PROBE(p_lds96k, 1024, 98304, "v7")
PROBE(p_1024_v64, 1024, 2048, "v63")
PROBE(p_1024_v72, 1024, 2048, "v71")
PROBE(p_1024_v112, 1024, 2048, "v111")
PROBE(p_512_v128, 512, 2048, "v127")
PROBE(p_512_v136, 512, 2048, "v135")
PROBE(p_256_v256, 256, 2048, "v255")
PROBE(p_64_v120, 64, 8192, "v119")

static hipStream_t masked(int cus, int skip) {
  const int words = (cus + 31) / 32;
  std::vector<uint32_t> m(words, 0u);
  for (int i = skip; i < cus; i++) m[i / 32] |= 1u << (i % 32);
  hipStream_t s;
  hipExtStreamCreateWithCUMask(&s, words, m.data());
  return s;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int* flag; float* sink; int* out;
  hipMalloc(&flag, 4); hipMalloc(&sink, 4096 * 4); hipMalloc(&out, 1 << 20);
  hipStream_t sa = masked(cus, 8), sb = masked(cus, 8), sc;
  hipStreamCreateWithFlags(&sc, hipStreamNonBlocking);
  struct P { const char* name; void (*k)(int*); int threads; };
  P probes[] = {{"1024 thr, LDS 64 KB", p_lds64k, 1024}, {"1024 thr, LDS 66 KB", p_lds66k, 1024},
                {"1024 thr, LDS 72 KB", p_lds72k, 1024}, {"1024 thr, LDS 80 KB", p_lds80k, 1024},
                {"1024 thr, LDS 96 KB", p_lds96k, 1024}, {"1024 thr, 64 VGPR", p_1024_v64, 1024},
                {"1024 thr, 72 VGPR", p_1024_v72, 1024}, {"1024 thr, 112 VGPR", p_1024_v112, 1024},
                {"512 thr, 128 VGPR", p_512_v128, 512}, {"512 thr, 136 VGPR", p_512_v136, 512},
                {"256 thr, 256 VGPR", p_256_v256, 256}, {"64 thr, 120 VGPR, 8 KB", p_64_v120, 64}};
  for (auto& p : probes) {
    hipMemset(flag, 0, 4);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(spin, dim3(cus - 8), dim3(512), 0, sa, flag, sink, 200000000ull);  // <= 2 s
    auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.03) {}
    hipEvent_t e;
    hipEventCreate(&e);
    t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(p.k, dim3(600), dim3(p.threads), 0, sb, out);
    hipEventRecord(e, sb);
    double dt = -1;
    for (;;) {
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (hipEventQuery(e) == hipSuccess) { dt = el; break; }
      if (el > 0.3) break;
    }
    const int one = 1;
    hipMemcpyAsync(flag, &one, 4, hipMemcpyHostToDevice, sc);
    hipDeviceSynchronize();
    printf("%-26s beside the items: %s\n", p.name, dt < 0 ? "BLOCKED (> 300 ms)" : "runs");
    hipEventDestroy(e);
  }
  return 0;
}
