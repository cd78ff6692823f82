// Microbenchmark: dependent-chain latency of fp64 ops and LDS reads on gfx950 (one wave).
#include <hip/hip_runtime.h>
#include <cstdio>

#define N 256
__global__ void lat(double* out, unsigned long long* cyc, double seed, double b, double c, float fb, float fc) {
  __shared__ double lds[64];
  const int l = threadIdx.x;
  lds[l] = seed + l;
  __syncthreads();
  double a = seed + l;
  unsigned long long t0, t1;
  // 1. dependent fma chain
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N; ++i) a = __builtin_fma(a, b, c);
  asm volatile("" :: "v"(a));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[0] = t1 - t0;
  // 2. independent fma (8 chains)
  double v[8];
  for (int k = 0; k < 8; ++k) v[k] = a + k;
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N / 8; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = __builtin_fma(v[k], b, c);
  for (int k = 0; k < 8; ++k) asm volatile("" :: "v"(v[k]));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[1] = t1 - t0;
  // 3. dependent rsq chain
  double q = a * 1e-3 + 2.0;
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N; ++i) q = __builtin_amdgcn_rsq(q) + 1.0;
  asm volatile("" :: "v"(q));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[2] = t1 - t0;
  // 4. dependent mul chain
  double m = a;
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N; ++i) m = m * b;
  asm volatile("" :: "v"(m));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[3] = t1 - t0;
  // 5. dependent LDS read chain (pointer chase through values)
  int idx = l;
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 16
  for (int i = 0; i < 64; ++i) idx = ((int)lds[idx & 63]) & 63;
  asm volatile("" :: "v"(idx));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[4] = t1 - t0;
  // 6. dependent divide chain
  double dv = a + 3.0;
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 16
  for (int i = 0; i < 64; ++i) dv = 1.0 / dv + 1.5;
  asm volatile("" :: "v"(dv));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[5] = t1 - t0;
  // 7. f32 fma chain
  float f = (float)a;
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N; ++i) f = __builtin_fmaf(f, fb, fc);
  asm volatile("" :: "v"(f));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[6] = t1 - t0;
  out[l] = a + v[0] + q + m + idx + dv + f;
}

int main() {
  double* out; unsigned long long* cyc;
  hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 16 * 8);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, out, cyc, 1.0, 1.0000001, 1e-9, 1.0000001f, 1e-9f);
    hipDeviceSynchronize();
  }
  unsigned long long h[16];
  hipMemcpy(h, cyc, 16 * 8, hipMemcpyDeviceToHost);
  printf("fma_f64 dep    %.2f cyc/op\n", h[0] / (double)N);
  printf("fma_f64 indep8 %.2f cyc/op\n", h[1] / (double)N);
  printf("rsq_f64+add dep %.2f cyc/iter\n", h[2] / (double)N);
  printf("mul_f64 dep    %.2f cyc/op\n", h[3] / (double)N);
  printf("lds read+cvt dep %.2f cyc/iter\n", h[4] / 64.0);
  printf("div_f64+add dep %.2f cyc/iter\n", h[5] / 64.0);
  printf("fma_f32 dep    %.2f cyc/op\n", h[6] / (double)N);
  return 0;
}
