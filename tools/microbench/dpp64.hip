// Microbenchmark: f64 broadcasts inside a 16-lane row by DPP64 row_newbcast (gfx90a+:
// v_mov_b64_dpp / v_fmac_f64_dpp with row_newbcast:n), against the LDS broadcast, for the
// K3 chain step.  One wave; dependent chains timed with s_memtime.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/dpp64.hip -o /tmp/dpp64
#include <hip/hip_runtime.h>
#include <cstdio>

#define N 96
#define T0() __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0)
#define T1(k) __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); \
  if (l == 0) cyc[k] = t1 - t0

template <int LANE>
__device__ __forceinline__ double nb(double x) {  // lane LANE of this lane's 16-lane row
  const long v = __builtin_amdgcn_update_dpp(0l, __builtin_bit_cast(long, x), 0x150 + LANE, 0xf, 0xf, true);
  return __builtin_bit_cast(double, v);
}

// chol6 on the 6x6 block whose row r sits in lane r of this 16-lane row (a[0..5]); every lane
// receives every value by row_newbcast and factors redundantly: L (lower, 21) and 1/diag (6)
__device__ __forceinline__ void chol6_dpp(const double (&a)[6], double (&L)[21], double (&ri)[6]) {
  double A[21];
#define G(r, c) A[(r) * ((r) + 1) / 2 + (c)] = nb<r>(a[c])
  G(0, 0);
  G(1, 0); G(1, 1);
  G(2, 0); G(2, 1); G(2, 2);
  G(3, 0); G(3, 1); G(3, 2); G(3, 3);
  G(4, 0); G(4, 1); G(4, 2); G(4, 3); G(4, 4);
  G(5, 0); G(5, 1); G(5, 2); G(5, 3); G(5, 4); G(5, 5);
#undef G
#pragma unroll
  for (int p = 0; p < 6; ++p) {
    const double d = A[p * (p + 1) / 2 + p];
    double r = __builtin_amdgcn_rsq(d);
    r = __builtin_fma(0.5 * r, __builtin_fma(-(d * r), r, 1.0), r);
    ri[p] = r;
    L[p * (p + 1) / 2 + p] = d * r;
#pragma unroll
    for (int i = p + 1; i < 6; ++i) L[i * (i + 1) / 2 + p] = A[i * (i + 1) / 2 + p] * r;
#pragma unroll
    for (int i = p + 1; i < 6; ++i)
#pragma unroll
      for (int j = p + 1; j <= i; ++j)
        A[i * (i + 1) / 2 + j] = __builtin_fma(-L[i * (i + 1) / 2 + p], L[j * (j + 1) / 2 + p], A[i * (i + 1) / 2 + j]);
  }
}

__global__ void k(double* out, unsigned long long* cyc, double seed, double b, double c) {
  __shared__ double lds[1024];
  const int l = threadIdx.x & 63;
  for (int i = l; i < 1024; i += 64) lds[i] = seed + i;
  __syncthreads();
  unsigned long long t0, t1;
  double acc = 0;
  // 0 dependent v_mov_b64_dpp chain
  double a = seed + l;
  T0();
#pragma unroll
  for (int i = 0; i < N; ++i) a = nb<3>(a) + 1.0;
  asm volatile("" ::"v"(a));
  T1(0);
  acc += a;
  // 1 dependent add chain alone (to subtract)
  a = seed + l;
  T0();
#pragma unroll
  for (int i = 0; i < N; ++i) a = a + 1.0;
  asm volatile("" ::"v"(a));
  T1(1);
  acc += a;
  // 2 independent broadcasts feeding FMAs (8 chains): issue of fma(bcast(x), y, z)
  double v[8], w[8];
  for (int q = 0; q < 8; ++q) { v[q] = seed + q + l; w[q] = b + q; }
  T0();
#pragma unroll
  for (int i = 0; i < N / 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = __builtin_fma(nb<5>(w[q]), b, v[q]);
  for (int q = 0; q < 8; ++q) asm volatile("" ::"v"(v[q]));
  T1(2);
  for (int q = 0; q < 8; ++q) acc += v[q];
  // 3 the same with plain operands
  T0();
#pragma unroll
  for (int i = 0; i < N / 8; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = __builtin_fma(w[q], b, v[q]);
  for (int q = 0; q < 8; ++q) asm volatile("" ::"v"(v[q]));
  T1(3);
  for (int q = 0; q < 8; ++q) acc += v[q];
  // 4 chol6 with DPP broadcast of the block, 8 times dependent
  double row[6];
  for (int q = 0; q < 6; ++q) row[q] = (q == (l & 15) ? 10.0 : 0.5) + seed * 1e-3;
  T0();
#pragma unroll 1
  for (int it = 0; it < 8; ++it) {
    double L[21], ri[6];
    chol6_dpp(row, L, ri);
#pragma unroll
    for (int q = 0; q < 6; ++q) row[q] = row[q] + 1e-9 * (L[20 - q] + ri[q]);
  }
  for (int q = 0; q < 6; ++q) asm volatile("" ::"v"(row[q]));
  T1(4);
  for (int q = 0; q < 6; ++q) acc += row[q];
  // 5 chol6 with the block through LDS (6 lanes write, every lane reads 21 values), 8 times
  T0();
#pragma unroll 1
  for (int it = 0; it < 8; ++it) {
    if (l < 6)
      for (int q = 0; q < 6; ++q) lds[8 * l + q] = row[q];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    double A[21];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int cc = 0; cc <= r; ++cc) A[r * (r + 1) / 2 + cc] = lds[8 * r + cc];
    double L[21], ri[6];
#pragma unroll
    for (int p = 0; p < 6; ++p) {
      const double d = A[p * (p + 1) / 2 + p];
      double r = __builtin_amdgcn_rsq(d);
      r = __builtin_fma(0.5 * r, __builtin_fma(-(d * r), r, 1.0), r);
      ri[p] = r;
      L[p * (p + 1) / 2 + p] = d * r;
      for (int i = p + 1; i < 6; ++i) L[i * (i + 1) / 2 + p] = A[i * (i + 1) / 2 + p] * r;
      for (int i = p + 1; i < 6; ++i)
        for (int j = p + 1; j <= i; ++j)
          A[i * (i + 1) / 2 + j] = __builtin_fma(-L[i * (i + 1) / 2 + p], L[j * (j + 1) / 2 + p], A[i * (i + 1) / 2 + j]);
    }
#pragma unroll
    for (int q = 0; q < 6; ++q) row[q] = row[q] + 1e-9 * (L[20 - q] + ri[q]);
  }
  for (int q = 0; q < 6; ++q) asm volatile("" ::"v"(row[q]));
  T1(5);
  for (int q = 0; q < 6; ++q) acc += row[q];
  out[threadIdx.x] = acc;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 16 * 8);
  hipMemset(cyc, 0, 128);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 1.0, 0.999, 1e-3);
  unsigned long long h[16];
  hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
  const char* names[] = {"dep mov_b64_dpp+add (per op)", "dep add (per op)", "fma(bcast) 8 chains (per op)",
                         "fma plain 8 chains (per op)", "chol6 via DPP64 (per chol)", "chol6 via LDS (per chol)"};
  const double per[] = {N, N, N, N, 8, 8};
  for (int i = 0; i < 6; ++i) std::printf("%-34s %8.1f cycles (s_memtime ticks x 1)\n", names[i], h[i] / per[i]);
  return 0;
}
