// Accuracy of v_rsq_f64 (__builtin_amdgcn_rsq) against 1/sqrt in double, with and without
// one Newton step, over SPD-pivot-like magnitudes.  hipcc --offload-arch=gfx950 -O3 rsq_acc.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
__global__ void k(const double* x, double* r0, double* r1, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double d = x[i];
  const double q = __builtin_amdgcn_rsq(d);
  r0[i] = q;
  r1[i] = q * (1.5 - 0.5 * d * q * q);
}
int main() {
  const int n = 1 << 22;
  std::vector<double> x(n), a(n), b(n);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double u = (double)(s >> 11) / 9007199254740992.0;
    x[i] = std::ldexp(1.0 + u, (int)(s % 80) - 40);
  }
  double *dx, *d0, *d1;
  hipMalloc(&dx, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, d0, d1, n);
  hipMemcpy(a.data(), d0, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), d1, n * 8, hipMemcpyDeviceToHost);
  double e0 = 0, e1 = 0;
  for (int i = 0; i < n; ++i) {
    const long double t = 1.0L / std::sqrt((long double)x[i]);
    e0 = std::fmax(e0, (double)std::fabs((a[i] - t) / t));
    e1 = std::fmax(e1, (double)std::fabs((b[i] - t) / t));
  }
  std::printf("max rel err: rsq %.3e  rsq+newton %.3e  (ulp %.3e)\n", e0, e1, std::ldexp(1.0, -52));
  return 0;
}
