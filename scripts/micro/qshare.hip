// Developer probe (GPU box): do streams created with the same CU mask share one hardware queue?
// A long spinning kernel runs on stream L; a short kernel on stream S is timed on the host.  If S
// finishes only when L does, the two streams' work went through one in-order queue.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void spin(int us) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)us * 100ull) __builtin_amdgcn_s_sleep(8);
}

static hipStream_t masked(int cus, int lo, int hi) {
  const int words = (cus + 31) / 32;
  std::vector<uint32_t> m(words, 0u);
  for (int i = lo; i < hi; i++) m[i / 32] |= 1u << (i % 32);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, words, m.data()) != hipSuccess) printf("mask stream failed\n");
  return s;
}

static double probe(hipStream_t longs, hipStream_t shorts) {
  hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, longs, 100000);  // 100 ms on 8 CUs
  const auto t0 = std::chrono::steady_clock::now();
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, shorts, 10);
  hipStreamSynchronize(shorts);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  hipDeviceSynchronize();
  return ms;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipStream_t roles = masked(cus, 0, 8), items = masked(cus, 8, cus);
  hipStream_t w1 = masked(cus, 8, cus), w2 = masked(cus, 8, cus), w3 = masked(cus, 8, cus);
  hipStream_t wd = masked(cus, 8, cus - 8);  // a different mask
  hipStream_t plain = nullptr, plain2 = nullptr, plain3 = nullptr;
  hipStreamCreateWithFlags(&plain, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&plain2, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&plain3, hipStreamNonBlocking);
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, 0, 1);
  hipDeviceSynchronize();
  printf("items -> roles      %.2f ms\n", probe(items, roles));
  printf("items -> w1 (same)  %.2f ms\n", probe(items, w1));
  printf("items -> w2 (same)  %.2f ms\n", probe(items, w2));
  printf("w1 -> w3 (same)     %.2f ms\n", probe(w1, w3));
  printf("items -> wd (diff)  %.2f ms\n", probe(items, wd));
  printf("items -> plain      %.2f ms\n", probe(items, plain));
  printf("plain -> plain2     %.2f ms\n", probe(plain, plain2));
  printf("plain -> plain3     %.2f ms\n", probe(plain, plain3));
  printf("roles -> items      %.2f ms\n", probe(roles, items));
  return 0;
}
