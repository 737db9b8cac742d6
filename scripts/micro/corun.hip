// Co-residency probe (developer tool): does a kernel on a second stream run beside a persistent
// 248-workgroup "engine-like" kernel (512 threads, ~128 VGPRs, 10 KB LDS, spinning on a flag)?
// Prints, per probe kernel shape, how long it took to complete while the spinner held the CUs.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/corun scripts/micro/corun.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512, 4) void spin(volatile int* flag, float* sink, unsigned long long bound) {
  __shared__ float lds[2560];  // 10 KB
  float acc[80];
#pragma unroll
  for (int i = 0; i < 80; i++) acc[i] = threadIdx.x * 0.5f + i;
  lds[threadIdx.x] = acc[3];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (*flag == 0 && __builtin_amdgcn_s_memrealtime() - t0 < bound) {
#pragma unroll
    for (int i = 0; i < 80; i++) acc[i] = acc[i] * 1.0001f + lds[(threadIdx.x + i) & 511];
    __builtin_amdgcn_s_sleep(2);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 80; i++) s += acc[i];
  if (s == 12345.f) sink[blockIdx.x] = s;
}

template <int kLds>
__global__ __launch_bounds__(1024) void probe(int* out) {
  __shared__ int lds[kLds / 4];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = lds[5] + 1;
}

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
  hipMalloc(&flag, 4); hipMalloc(&sink, 4096 * 4); hipMalloc(&out, 4096 * 4);
  hipStream_t sa = masked(cus, 8), sb = masked(cus, 8), sc;
  hipStreamCreateWithFlags(&sc, hipStreamNonBlocking);
  const char* names[] = {"probe 1024 thr, 112 KB LDS", "probe 1024 thr, 64 KB LDS", "probe 1024 thr, 2 KB LDS"};
  for (int v = 0; v < 3; v++) {
    for (int mode = 0; mode < 2; mode++) {  // 0: spinner running, 1: alone
      hipMemset(flag, 0, 4);
      hipDeviceSynchronize();
      if (mode == 0) hipLaunchKernelGGL(spin, dim3(cus - 8), dim3(512), 0, sa, flag, sink, 300000000ull);  // <= 3 s
      hipEvent_t e; hipEventCreate(&e);
      // give the spinner time to be resident
      auto t0 = std::chrono::steady_clock::now();
      while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.05) {}
      t0 = std::chrono::steady_clock::now();
      if (v == 0) hipLaunchKernelGGL(probe<114688>, dim3(300), dim3(1024), 0, sb, out);
      if (v == 1) hipLaunchKernelGGL(probe<65536>, dim3(300), dim3(1024), 0, sb, out);
      if (v == 2) hipLaunchKernelGGL(probe<2048>, dim3(300), dim3(1024), 0, sb, out);
      hipEventRecord(e, sb);
      double dt = -1;
      while (true) {
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (hipEventQuery(e) == hipSuccess) { dt = el; break; }
        if (el > 1.0) break;
      }
      const int one = 1;
      hipMemcpyAsync(flag, &one, 4, hipMemcpyHostToDevice, sc);
      hipDeviceSynchronize();
      printf("%-30s %-8s: %s %.3f ms\n", names[v], mode ? "alone" : "beside", dt < 0 ? "NOT DONE after" : "done in", (dt < 0 ? 1.0 : dt) * 1e3);
      hipEventDestroy(e);
    }
  }
  return 0;
}
