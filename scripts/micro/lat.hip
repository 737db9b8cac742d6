// Developer micro-benchmark (GPU box): single-wave dependent latencies on gfx950 — fp64 FMA, fp64
// sqrt and division, LDS load chains, and an s_memrealtime read — in s_memtime cycles.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_lat(double* out, unsigned long long* cyc, int n) {
  __shared__ double lds[1024];
  __shared__ int nxt[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) { lds[i] = 1.0 + i * 1e-9; nxt[i] = (i * 7 + 13) & 1023; }
  __syncthreads();
  if (threadIdx.x >= 64) return;
  double x = out[threadIdx.x], y = 1.0000001;
  unsigned long long t0 = clock64();
  for (int i = 0; i < n; i++) x = fma(x, y, 1e-9);
  unsigned long long t1 = clock64();
  double z = x;
  for (int i = 0; i < n / 10; i++) z = sqrt(z + 1.0);
  unsigned long long t2 = clock64();
  double w = z;
  for (int i = 0; i < n / 10; i++) w = 1.0 / (w + 1.0);
  unsigned long long t3 = clock64();
  int p = threadIdx.x;
  for (int i = 0; i < n / 10; i++) p = nxt[p];
  unsigned long long t4 = clock64();
  unsigned long long r = 0;
  for (int i = 0; i < n / 10; i++) r += __builtin_amdgcn_s_memrealtime();
  unsigned long long t5 = clock64();
  double q = w;
  if (threadIdx.x == 0) {  // single lane
    for (int i = 0; i < n; i++) q = fma(q, y, 1e-9);
  }
  unsigned long long t6 = clock64();
  out[threadIdx.x] = x + z + w + p + (double)r + q;
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t5 - t4; cyc[5] = t6 - t5;
  }
}

int main() {
  double* out; unsigned long long* cyc;
  hipMalloc(&out, 1024 * 8); hipMemset(out, 0, 1024 * 8);
  hipMalloc(&cyc, 64);
  const int n = 1000;
  for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, out, cyc, n);
  unsigned long long h[6];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  printf("clock64 cycles per dependent op: fma_f64 %.1f, sqrt_f64 %.1f, div_f64 %.1f, ds_read chase %.1f, "
         "s_memrealtime %.1f, fma_f64 one lane %.1f\n",
         h[0] / (double)n, h[1] / (n / 10.0), h[2] / (n / 10.0), h[3] / (n / 10.0), h[4] / (n / 10.0), h[5] / (double)n);
  return 0;
}
