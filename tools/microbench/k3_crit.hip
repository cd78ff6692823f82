// Microbenchmark: the critical-lane K3 block step (csrc/ba_band_cl.h) on one wave, operands
// from LDS as in the kernel, 28 dependent steps timed with s_memtime.  Variants:
//   0 full step: pivots, publish, lazy update of the sub-diagonal rows, their solve, publish,
//     next panel (u by row_shl:6, 36 broadcast FMAs), next P from LDS
//   1 pivots only
//   2 pivots + solve + next panel (no lazy update)
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I visualodometry_amd/csrc tools/microbench/k3_crit.hip -o /tmp/k3_crit
#include <hip/hip_runtime.h>

#include <cstdio>

#include "ba_band_cl.h"

using namespace vo;

constexpr int STEPS = 28;

template <int V>
__global__ void kern(double* out, unsigned long long* cyc, double seed) {
  __shared__ __attribute__((aligned(16))) double lds[4096];
  const int lane = threadIdx.x & 63, li = lane & 15;
  for (int i = lane; i < 4096; i += 64) lds[i] = (i % 7 == 0 ? 4.0 : 0.01) + seed * 1e-3 * (i & 3);
  __syncthreads();
  double a[6], pp[6], vp[6], r[6];
  for (int c = 0; c < 6; ++c) {
    a[c] = (c == li ? 10.0 : 0.1) + seed;
    pp[c] = 0.05 * c + seed;
    vp[c] = 0.02 * c;
  }
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  double chk = 0;
#pragma unroll 1
  for (int k = 0; k < STEPS; ++k) {
    const int base = (k & 7) * 384;
    cl::pivots(a, r);
    chk += r[5];
    // publish: L_kk rows / y' / r (lanes 0..5, 12; others to a dummy row)
    {
      double* d = lds + 3500 + 8 * li;
      *reinterpret_cast<double2*>(d) = make_double2(a[0], a[1]);
      *reinterpret_cast<double2*>(d + 2) = make_double2(a[2], a[3]);
      *reinterpret_cast<double2*>(d + 4) = make_double2(a[4], a[5]);
    }
    if (V == 0) {
      double u[6];
      const double* s = lds + base + 72 + 6 * (li % 6);
#pragma unroll
      for (int m = 0; m < 6; ++m) u[m] = s[m];
      cl::sub_uvt<6>(pp, u, vp);
    }
    if (V != 1) {
      cl::solve_lt(pp, a, r);
      {
        double* d = lds + 3700 + 8 * li;
        *reinterpret_cast<double2*>(d) = make_double2(pp[0], pp[1]);
        *reinterpret_cast<double2*>(d + 2) = make_double2(pp[2], pp[3]);
        *reinterpret_cast<double2*>(d + 4) = make_double2(pp[4], pp[5]);
      }
      double u[6], sh[6], b0[6];
      cl::shl6(pp, sh);
      const double* s = lds + base + 6 * (li % 6);
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        u[m] = li < 6 ? sh[m] : a[m];
        b0[m] = s[m];
      }
      cl::sub_uvt<6>(b0, u, pp);
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        vp[m] = pp[m];
        a[m] = b0[m] * 0.5 + (li == m ? 5.0 : 0.0);  // keep it SPD for the timing loop
        pp[m] = s[36 + m] * 0.01;
      }
    } else {
#pragma unroll
      for (int m = 0; m < 6; ++m) a[m] = a[m] * 0.5 + (li == m ? 5.0 : 0.0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double acc = chk;
  for (int c = 0; c < 6; ++c) acc += a[c] + pp[c] + vp[c];
  out[threadIdx.x] = acc;
  if (lane == 0) cyc[V] = (t1 - t0) / STEPS;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 8 * 8);
  hipMemset(cyc, 0, 64);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(kern<0>, dim3(1), dim3(64), 0, 0, out, cyc, 1.0);
    hipLaunchKernelGGL(kern<1>, dim3(1), dim3(64), 0, 0, out, cyc, 1.0);
    hipLaunchKernelGGL(kern<2>, dim3(1), dim3(64), 0, 0, out, cyc, 1.0);
  }
  hipDeviceSynchronize();
  unsigned long long h[8];
  hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
  std::printf("full critical step      %llu cycles/step\n", h[0]);
  std::printf("pivots only             %llu cycles/step\n", h[1]);
  std::printf("no lazy update          %llu cycles/step\n", h[2]);
  return 0;
}
