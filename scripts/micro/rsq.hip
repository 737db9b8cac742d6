// Developer micro-test (GPU box): accuracy of v_rsq_f64 and of 1 / 2 Newton steps on it, in ulps
// of the correctly rounded 1 / sqrt(d), over d in [1e-12, 1e12] (log-uniform).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const double* d, double* o0, double* o1, double* o2, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = d[i];
  double y = __builtin_amdgcn_rsq(x);
  o0[i] = y;
  y = y * fma(-0.5 * x, y * y, 1.5);
  o1[i] = y;
  y = y * fma(-0.5 * x, y * y, 1.5);
  o2[i] = y;
}

int main() {
  const int n = 1 << 20;
  std::vector<double> d(n), o0(n), o1(n), o2(n);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    d[i] = std::pow(10.0, -12.0 + 24.0 * (double)(s >> 11) / 9007199254740992.0);
  }
  double *dd, *a, *b, *c;
  hipMalloc(&dd, n * 8); hipMalloc(&a, n * 8); hipMalloc(&b, n * 8); hipMalloc(&c, n * 8);
  hipMemcpy(dd, d.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dd, a, b, c, n);
  hipMemcpy(o0.data(), a, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(o1.data(), b, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(o2.data(), c, n * 8, hipMemcpyDeviceToHost);
  double e[3] = {0, 0, 0};
  for (int i = 0; i < n; i++) {
    const double r = 1.0 / std::sqrt(d[i]);
    const double ulp = std::nextafter(r, INFINITY) - r;
    const double* o[3] = {&o0[i], &o1[i], &o2[i]};
    for (int j = 0; j < 3; j++) e[j] = std::fmax(e[j], std::fabs(*o[j] - r) / ulp);
  }
  std::printf("max ulp error: rsq %.3g, +1 Newton %.3g, +2 Newton %.3g\n", e[0], e[1], e[2]);
  return 0;
}
