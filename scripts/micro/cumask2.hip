// Developer probe (GPU box): the CUs a stream masked to bits [0, n) reaches, per XCC; with more
// arguments, the mask is the bit groups [8k, 8k + 8) of each k given.
// usage: cumask2 [n] | cumask2 - k1 k2 ...
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <vector>

__global__ void probe(unsigned* out, int spin_us) {
  if (threadIdx.x == 0) {
    out[blockIdx.x * 2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);       // HW_REG_HW_ID
    out[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin_us * 100ull) __builtin_amdgcn_s_sleep(2);
  }
}

int main(int argc, char** argv) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int words = (cus + 31) / 32;
  std::vector<uint32_t> m(words, 0);
  int n = 0;
  if (argc > 2 && argv[1][0] == '-') {
    for (int a = 2; a < argc; a++)
      for (int i = 8 * atoi(argv[a]); i < 8 * atoi(argv[a]) + 8; i++) { m[i / 32] |= 1u << (i % 32); n++; }
  } else {
    n = argc > 1 ? atoi(argv[1]) : 16;
    for (int i = 0; i < n; i++) m[i / 32] |= 1u << (i % 32);
  }
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, words, m.data()) != hipSuccess) { printf("mask failed\n"); return 1; }
  const int g = 8 * n;
  unsigned* d;
  hipMalloc(&d, g * 8);
  hipLaunchKernelGGL(probe, dim3(g), dim3(64), 0, s, d, 300);
  hipDeviceSynchronize();
  std::vector<unsigned> h(g * 2);
  hipMemcpy(h.data(), d, g * 8, hipMemcpyDeviceToHost);
  std::map<unsigned, std::set<unsigned>> per;
  for (int i = 0; i < g; i++) {
    const unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 15;
    per[xcc].insert(((hw >> 13) & 7) << 8 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 15));
  }
  printf("CUs %d, %d mask bits:\n", cus, n);
  for (auto& [x, set] : per) {
    printf("  xcc %u: %zu CUs:", x, set.size());
    for (unsigned k : set) printf(" se%u.sh%u.cu%u", k >> 8, (k >> 4) & 15, k & 15);
    printf("\n");
  }
  return 0;
}
