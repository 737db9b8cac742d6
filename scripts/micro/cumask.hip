// Developer probe (GPU box): where do the workgroups of a CU-masked stream run?  Each workgroup
// records XCC_ID and HW_ID (CU, SH, SE) and spins ~50 us so the grids overlap.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

__global__ void probe(unsigned* out, int spin_us) {
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    out[blockIdx.x * 2] = hw;
    out[blockIdx.x * 2 + 1] = xcc;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin_us * 100ull) __builtin_amdgcn_s_sleep(2);
  }
}

static unsigned key(unsigned hw, unsigned xcc) {  // (xcc, se, sh, cu)
  const unsigned cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
  return (xcc & 15) << 12 | se << 8 | sh << 4 | cu;
}

int main(int argc, char** argv) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", cus);
  const int words = (cus + 31) / 32;
  const int reserve = argc > 1 ? atoi(argv[1]) : 0;  // the bit the solve stream gets
  std::vector<uint32_t> ma(words, 0), mb(words, 0xffffffffu);
  ma[reserve / 32] |= 1u << (reserve % 32);
  mb[reserve / 32] &= ~(1u << (reserve % 32));
  if (cus % 32) { mb[words - 1] &= (1u << (cus % 32)) - 1; }
  hipStream_t a, b;
  if (hipExtStreamCreateWithCUMask(&a, words, ma.data()) != hipSuccess) { printf("mask a failed\n"); return 1; }
  if (hipExtStreamCreateWithCUMask(&b, words, mb.data()) != hipSuccess) { printf("mask b failed\n"); return 1; }
  const int na = 8, nb = 2 * cus;
  unsigned *da, *db;
  hipMalloc(&da, na * 8);
  hipMalloc(&db, nb * 8);
  hipLaunchKernelGGL(probe, dim3(na), dim3(512), 0, a, da, 200);
  hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 0, b, db, 200);
  hipDeviceSynchronize();
  std::vector<unsigned> ha(na * 2), hb(nb * 2);
  hipMemcpy(ha.data(), da, na * 8, hipMemcpyDeviceToHost);
  hipMemcpy(hb.data(), db, nb * 8, hipMemcpyDeviceToHost);
  std::set<unsigned> sa, sb;
  for (int i = 0; i < na; i++) sa.insert(key(ha[2 * i], ha[2 * i + 1]));
  for (int i = 0; i < nb; i++) sb.insert(key(hb[2 * i], hb[2 * i + 1]));
  printf("stream A (bit %d): %zu distinct CUs:", reserve, sa.size());
  for (unsigned k : sa) printf(" %03x", k);
  printf("\nstream B (all other bits): %zu distinct CUs; overlap with A:", sb.size());
  int ov = 0;
  for (unsigned k : sa) if (sb.count(k)) { printf(" %03x", k); ov++; }
  printf(" (%d)\n", ov);
  // which CUs does an unmasked grid reach
  unsigned* dc;
  hipMalloc(&dc, 2 * cus * 8);
  hipLaunchKernelGGL(probe, dim3(2 * cus), dim3(512), 0, 0, dc, 200);
  hipDeviceSynchronize();
  std::vector<unsigned> hc(4 * cus);
  hipMemcpy(hc.data(), dc, 2 * cus * 8, hipMemcpyDeviceToHost);
  std::set<unsigned> sc;
  for (int i = 0; i < 2 * cus; i++) sc.insert(key(hc[2 * i], hc[2 * i + 1]));
  printf("unmasked: %zu distinct CUs; B + A cover %zu\n", sc.size(), sb.size() + sa.size() - ov);
  return 0;
}
