// Microbenchmark: the primitives a K3 block step is built from (gfx950, one wave unless a
// row says otherwise), as dependent chains timed with s_memtime.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/k3_prims.hip -o /tmp/k3_prims
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
#define N 128
#define T0() __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0)
#define T1(k) __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); \
  if (l == 0 && wave == 0) cyc[k] = t1 - t0

__device__ __forceinline__ double rl(double x, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
  return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

__global__ void prims(double* out, unsigned long long* cyc, double seed, double b, double c) {
  __shared__ double lds[512];
  const int l = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 512; i += blockDim.x) lds[i] = seed + i;
  __syncthreads();
  double a = seed + l, acc = 0;
  unsigned long long t0, t1;
  if (wave == 0) {
    // 0 f64 fma dependent
    T0();
#pragma unroll
    for (int i = 0; i < N; ++i) a = __builtin_fma(a, b, c);
    asm volatile("" ::"v"(a));
    T1(0);
    // 1 f64 fma independent (8 chains): issue cost
    double v[8];
    for (int k = 0; k < 8; ++k) v[k] = a + k;
    T0();
#pragma unroll
    for (int i = 0; i < N / 8; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_fma(v[k], b, c);
    for (int k = 0; k < 8; ++k) asm volatile("" ::"v"(v[k]));
    T1(1);
    for (int k = 0; k < 8; ++k) acc += v[k];
    // 2 rsq f64 + Newton (3 ops) dependent: one pivot's reciprocal
    double q = a * 1e-3 + 2.0;
    T0();
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const double d = q;
      double r = __builtin_amdgcn_rsq(d);
      r = __builtin_fma(0.5 * r, __builtin_fma(-(d * r), r, 1.0), r);
      q = r + 1.5;
    }
    asm volatile("" ::"v"(q));
    T1(2);
    acc += q;
    // 3 LDS round trip: ds_write_b64 then ds_read_b64 of another lane's slot, dependent
    double x = a;
    T0();
#pragma unroll 8
    for (int i = 0; i < N; ++i) {
      lds[l] = x;
      __builtin_amdgcn_wave_barrier();
      x = lds[(l + 1) & 63] * b;
      __builtin_amdgcn_wave_barrier();
    }
    asm volatile("" ::"v"(x));
    T1(3);
    acc += x;
    // 4 readlane f64 broadcast, dependent through a VALU op
    x = a;
    T0();
#pragma unroll 8
    for (int i = 0; i < N; ++i) x = rl(x, i & 63) * b;
    asm volatile("" ::"v"(x));
    T1(4);
    acc += x;
    // 5 readlane f64 broadcast x6 independent (issue cost of a 6-value broadcast)
    double y[6];
    for (int k = 0; k < 6; ++k) y[k] = a + k;
    T0();
#pragma unroll 4
    for (int i = 0; i < N / 6; ++i)
#pragma unroll
      for (int k = 0; k < 6; ++k) y[k] = rl(y[k], (i + k) & 63) + c;
    for (int k = 0; k < 6; ++k) asm volatile("" ::"v"(y[k]));
    T1(5);
    for (int k = 0; k < 6; ++k) acc += y[k];
    // 6 DPP row_newbcast:3 f64, dependent
    x = a;
    T0();
#pragma unroll 8
    for (int i = 0; i < N; ++i) x = dpp<0x153>(x) * b;
    asm volatile("" ::"v"(x));
    T1(6);
    acc += x;
    // 7 ds_read_b128 broadcast of 6 doubles (3 reads) after a write by 6 lanes, dependent
    x = a;
    T0();
#pragma unroll 4
    for (int i = 0; i < N; ++i) {
      if (l < 6) lds[64 + l] = x;
      __builtin_amdgcn_wave_barrier();
      const double2* p = reinterpret_cast<const double2*>(lds + 64);
      const double2 u0 = p[0], u1 = p[1], u2 = p[2];
      __builtin_amdgcn_wave_barrier();
      x = u0.x + u0.y + u1.x + u1.y + u2.x + u2.y;
    }
    asm volatile("" ::"v"(x));
    T1(7);
    acc += x;
    // 8 mfma f64 16x16x4 dependent accumulator
    d4 C = {a, a, a, a};
    T0();
#pragma unroll
    for (int i = 0; i < 32; ++i) C = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, C, 0, 0, 0);
    asm volatile("" ::"v"(C));
    T1(8);
    // 9 mfma f64 16x16x4, 4 independent accumulators
    d4 D0 = C, D1 = C + 1.0, D2 = C + 2.0, D3 = C + 3.0;
    T0();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      D0 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, D0, 0, 0, 0);
      D1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, D1, 0, 0, 0);
      D2 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, D2, 0, 0, 0);
      D3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, D3, 0, 0, 0);
    }
    asm volatile("" ::"v"(D0), "v"(D1), "v"(D2), "v"(D3));
    T1(9);
    acc += D0.x + D1.y + D2.z + D3.w;
    // 10 chol6-like: 6 pivots (rsq + Newton + scale + 15 update) redundant in every lane
    double A21[21];
    for (int k = 0; k < 21; ++k) A21[k] = (k == 0 || k == 2 || k == 5 || k == 9 || k == 14 || k == 20) ? 10.0 + a : 0.1 * k;
    T0();
#pragma unroll 1
    for (int it = 0; it < 8; ++it) {
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int jj = j * (j + 1) / 2 + j;
        const double d = A21[jj];
        double r = __builtin_amdgcn_rsq(d);
        r = __builtin_fma(0.5 * r, __builtin_fma(-(d * r), r, 1.0), r);
        A21[jj] = r;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) A21[i * (i + 1) / 2 + j] *= r;
#pragma unroll
        for (int i = j + 1; i < 6; ++i)
#pragma unroll
          for (int cc = j + 1; cc <= i; ++cc) A21[i * (i + 1) / 2 + cc] -= A21[i * (i + 1) / 2 + j] * A21[cc * (cc + 1) / 2 + j];
      }
#pragma unroll
      for (int k = 0; k < 21; ++k) A21[k] = __builtin_fma(A21[k], 1e-30, (k == 0 || k == 2 || k == 5 || k == 9 || k == 14 || k == 20) ? 10.0 : 0.1);
    }
    for (int k = 0; k < 21; ++k) asm volatile("" ::"v"(A21[k]));
    T1(10);
    for (int k = 0; k < 21; ++k) acc += A21[k];
  }
  // 11 s_barrier, all 8 waves arriving together
  __syncthreads();
  T0();
#pragma unroll 8
  for (int i = 0; i < N; ++i) asm volatile("s_barrier" ::: "memory");
  T1(11);
  // 12 LDS flag handoff wave 0 -> wave 2 -> wave 0 (ping-pong through LDS, spin)
  __syncthreads();
  volatile int* fl = reinterpret_cast<volatile int*>(lds + 400);
  if (threadIdx.x == 0) { fl[0] = 0; fl[2] = 0; }
  __syncthreads();
  T0();
  if (wave == 0) {
    for (int i = 1; i <= N; ++i) {
      if (l == 0) fl[0] = i;
      for (int g = 0; g < 100000 && fl[2] != i; ++g) {}
    }
  } else if (wave == 2) {
    for (int i = 1; i <= N; ++i) {
      for (int g = 0; g < 100000 && fl[0] != i; ++g) {}
      if (l == 0) fl[2] = i;
    }
  }
  T1(12);
  out[threadIdx.x] = a + acc;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 512 * 8);
  hipMalloc(&cyc, 32 * 8);
  hipMemset(cyc, 0, 32 * 8);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(prims, dim3(1), dim3(512), 0, 0, out, cyc, 1.0, 1.0000001, 1e-9);
    hipDeviceSynchronize();
  }
  unsigned long long h[32];
  hipMemcpy(h, cyc, 32 * 8, hipMemcpyDeviceToHost);
  printf("f64 fma dependent            %.1f cyc/op\n", h[0] / (double)N);
  printf("f64 fma independent x8       %.1f cyc/op\n", h[1] / (double)N);
  printf("rsq+newton (pivot recip) dep %.1f cyc/iter\n", h[2] / (double)N);
  printf("LDS write->read round trip   %.1f cyc/iter\n", h[3] / (double)N);
  printf("readlane f64 dep             %.1f cyc/iter\n", h[4] / (double)N);
  printf("readlane f64 x6 indep        %.1f cyc/6 values\n", h[5] / (double)(N / 6));
  printf("dpp newbcast f64 dep         %.1f cyc/iter\n", h[6] / (double)N);
  printf("6-lane write + b128 bcast rd %.1f cyc/iter\n", h[7] / (double)N);
  printf("mfma f64 16x16x4 dependent   %.1f cyc/op\n", h[8] / 32.0);
  printf("mfma f64 16x16x4 indep x4    %.1f cyc/op\n", h[9] / 32.0);
  printf("chol6 redundant              %.1f cyc/chol6\n", h[10] / 8.0);
  printf("s_barrier 8 waves            %.1f cyc/barrier\n", h[11] / (double)N);
  printf("LDS flag ping-pong           %.1f cyc/round trip\n", h[12] / (double)N);
  return 0;
}
