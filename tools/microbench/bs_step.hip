// Microbenchmark: one back-substitution chain step of the banded K3 on gfx950 (one wave):
// broadcast of 6 fp64 values held by 6 lanes to the whole wave, then a 6-term dot into a
// per-lane accumulator.  Variants: v_readlane pairs, LDS store + wave barrier + loads,
// DPP-free ds_bpermute.  Build: hipcc --offload-arch=gfx950 -O3 bs_step.hip -o bs_step
#include <hip/hip_runtime.h>
#include <cstdio>

#define STEPS 64
__device__ __forceinline__ double rl(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

__global__ void bench(double* out, unsigned long long* cyc, double seed) {
  __shared__ double lds[64 * 8];
  const int l = threadIdx.x;
  double g[6];
  for (int c = 0; c < 6; ++c) g[c] = 1e-3 * (l + c + 1) * seed;
  double Y = seed + l;
  unsigned long long t0, t1;
  // A: readlane broadcast
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  for (int k = 0; k < STEPS; ++k) {
    const int l0 = __builtin_amdgcn_readfirstlane(6 * (k % 8));
    double z[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) z[c] = rl(Y, l0 + c);
    Y -= g[0] * z[0] + g[1] * z[1] + g[2] * z[2] + g[3] * z[3] + g[4] * z[4] + g[5] * z[5];
  }
  asm volatile("" :: "v"(Y));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[0] = t1 - t0;
  // B: LDS broadcast
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  for (int k = 0; k < STEPS; ++k) {
    const int g0 = k % 8;
    if (l / 6 == g0) lds[8 * g0 + l % 6] = Y;
    __builtin_amdgcn_wave_barrier();
    const double2* q = reinterpret_cast<const double2*>(lds + 8 * g0);
    const double2 a0 = q[0], a1 = q[1], a2 = q[2];
    Y -= g[0] * a0.x + g[1] * a0.y + g[2] * a1.x + g[3] * a1.y + g[4] * a2.x + g[5] * a2.y;
  }
  asm volatile("" :: "v"(Y));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[1] = t1 - t0;
  // C: readlane, dot as a tree (3 levels) instead of a chain
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  for (int k = 0; k < STEPS; ++k) {
    const int l0 = __builtin_amdgcn_readfirstlane(6 * (k % 8));
    double z[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) z[c] = rl(Y, l0 + c);
    const double s0 = g[0] * z[0] + g[1] * z[1], s1 = g[2] * z[2] + g[3] * z[3], s2 = g[4] * z[4] + g[5] * z[5];
    Y -= (s0 + s1) + s2;
  }
  asm volatile("" :: "v"(Y));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[2] = t1 - t0;
  // D: 12 readlanes only (no math dependency on the result except the last)
  double acc = 0;
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  for (int k = 0; k < STEPS; ++k) {
    const int l0 = __builtin_amdgcn_readfirstlane(6 * (k % 8));
#pragma unroll
    for (int c = 0; c < 6; ++c) acc += rl(Y, l0 + c);
  }
  asm volatile("" :: "v"(acc));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[3] = t1 - t0;
  // E: dependent fp64 FMA chain of 6
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  for (int k = 0; k < STEPS; ++k) {
    Y = Y - (((((g[0] * Y + g[1]) * Y + g[2]) * Y + g[3]) * Y + g[4]) * Y + g[5]);
  }
  asm volatile("" :: "v"(Y));
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) cyc[4] = t1 - t0;
  out[l] = Y + acc;
}

int main() {
  double* d_out;
  unsigned long long* d_c;
  hipMalloc(&d_out, 64 * 8);
  hipMalloc(&d_c, 8 * 8);
  unsigned long long c[8];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(bench, dim3(1), dim3(64), 0, 0, d_out, d_c, 1.0 + rep);
    hipMemcpy(c, d_c, 8 * 8, hipMemcpyDeviceToHost);
  }
  const char* names[] = {"readlane bcast + 6-FMA chain", "LDS bcast + 6-FMA chain", "readlane + tree dot",
                         "12 readlanes only", "6 dependent fp64 FMA"};
  for (int i = 0; i < 5; ++i) printf("%-32s %7.1f cycles/step\n", names[i], (double)c[i] / STEPS);
  return 0;
}
