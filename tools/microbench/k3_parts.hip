// Microbenchmark: latency of the pieces of one K3 elimination step on gfx950, one
// wave per SIMD (the K3 situation).  Build: hipcc --offload-arch=gfx950 -O3 k3_parts.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ constexpr int P6(int i, int c) { return i * (i + 1) / 2 + c; }

__device__ __forceinline__ bool chol6(double (&a)[21], double (&r)[6]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const double d = a[P6(j, j)];
    ok = ok && d > 0.0;
    const double dd = d > 0.0 ? d : 1.0;
    double q = __builtin_amdgcn_rsq(dd);
    q = q * (1.5 - 0.5 * dd * q * q);
    r[j] = q;
    a[P6(j, j)] = dd * q;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) a[P6(i, j)] *= q;
#pragma unroll
    for (int i = j + 1; i < 6; ++i)
#pragma unroll
      for (int c = j + 1; c <= i; ++c) a[P6(i, c)] -= a[P6(i, j)] * a[P6(c, j)];
  }
  return ok;
}

__device__ __forceinline__ void fwd6(const double (&L)[21], const double (&r)[6], double (&v)[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = v[i];
#pragma unroll
    for (int m = 0; m < i; ++m) s -= L[P6(i, m)] * v[m];
    v[i] = s * r[i];
  }
}

#define T0() do { __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define T1(slot, n) do { __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); if (threadIdx.x == 0) cyc[slot] = (t1 - t0) / (n); } while (0)

__global__ __launch_bounds__(256) void parts(double* out, unsigned long long* cyc, double seed) {
  __shared__ __attribute__((aligned(16))) double lds[8192];
  const int l = threadIdx.x, lane = l & 63, wave = l >> 6;
  for (int e = l; e < 8192; e += 256) lds[e] = 1.0 + 1e-3 * (e % 37);
  __syncthreads();
  unsigned long long t0 = 0, t1 = 0;
  double acc = 0.0;
  if (wave == 0) {
    // 1. chol6 -> next input (dependent chain)
    double a[21];
    for (int e = 0; e < 21; ++e) a[e] = (e == 0 || e == 2 || e == 5 || e == 9 || e == 14 || e == 20) ? 4.0 + seed : 0.1 * seed;
    double r[6];
    T0();
    for (int it = 0; it < 64; ++it) {
      chol6(a, r);
      a[0] = 4.0 + r[5] * 1e-9;
      a[2] = 4.0 + r[4] * 1e-9;
    }
    T1(0, 64);
    acc += r[5];
    // 2. fwd6 chain
    double v[6] = {1, 2, 3, 4, 5, 6};
    T0();
    for (int it = 0; it < 64; ++it) {
      fwd6(a, r, v);
      v[0] += 1e-9;
    }
    T1(1, 64);
    acc += v[5];
    // 3. 17 single-lane b128 stores then a dependent load of lane-0 data
    T0();
    for (int it = 0; it < 16; ++it) {
      if (lane == 0) {
        double2* o = reinterpret_cast<double2*>(lds + 1024 + 64 * (it & 3));
#pragma unroll
        for (int e = 0; e < 17; ++e) o[e] = make_double2(acc + e, acc);
      }
      acc += lds[1024 + 64 * (it & 3) + 2 * (lane & 15)];
    }
    T1(2, 16);
    // 4. 64-lane b128 store + dependent b128 load round trip
    T0();
    for (int it = 0; it < 16; ++it) {
      reinterpret_cast<double2*>(lds + 2048)[lane] = make_double2(acc, acc);
      acc += reinterpret_cast<double2*>(lds + 2048)[(lane + 1) & 63].x;
    }
    T1(3, 16);
    // 5. a task: 2 + 12 b128 rows (a0, a1, bq) + 2 target rows, 72 FMAs, store
    T0();
    for (int it = 0; it < 16; ++it) {
      const int qa = (lane * 5 + it) % 8, qb = (lane * 3 + it) % 8, rp = lane % 3;
      const double* A = lds + 4096 + 36 * qa + 6 * rp;
      const double* B = lds + 4096 + 36 * qb;
      double* X = lds + 6144 + 36 * ((lane * 7) % 40) + 6 * rp;
      double a0[6], a1[6], bq[6][6], x0[6], x1[6];
      for (int e = 0; e < 6; ++e) { a0[e] = A[e]; a1[e] = A[18 + e]; x0[e] = X[e]; x1[e] = X[18 + e]; }
      for (int c = 0; c < 6; ++c)
        for (int e = 0; e < 6; ++e) bq[c][e] = B[6 * c + e];
      for (int c = 0; c < 6; ++c)
        for (int e = 0; e < 6; ++e) {
          x0[c] = __builtin_fma(-a0[e], bq[c][e], x0[c]);
          x1[c] = __builtin_fma(-a1[e], bq[c][e], x1[c]);
        }
      for (int e = 0; e < 6; ++e) { X[e] = x0[e]; X[18 + e] = x1[e]; }
    }
    T1(4, 16);
  }
  if (wave == 0) {
    // 7. one side step's panel part: diag (12 b128) + yk + sv loads, chol6, fwd6 x2,
    //    3 stores of the panel row, y read-modify-write; 21 dependent steps
    T0();
    for (int it = 0; it < 21; ++it) {
      const double2* D = reinterpret_cast<const double2*>(lds + 36 * (it & 7));
      double L[21], r[6], yk[6], sv[6];
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int c = 0; c <= i; c += 2) {
          const double2 v = D[3 * i + c / 2];
          L[P6(i, c)] = v.x;
          if (c + 1 <= i) L[P6(i, c + 1)] = v.y;
        }
      for (int i = 0; i < 6; ++i) L[P6(i, i)] += 6.0;
      const double* Y = lds + 512 + 6 * (it & 3);
      for (int e = 0; e < 6; ++e) yk[e] = Y[e];
      const double* S = lds + 1024 + 36 * (lane / 6 % 8) + 6 * (lane % 6);
      for (int e = 0; e < 6; ++e) sv[e] = S[e];
      __builtin_amdgcn_sched_barrier(0);
      chol6(L, r);
      fwd6(L, r, yk);
      fwd6(L, r, sv);
      if (lane < 42) {
        double* W = lds + 3072 + 36 * (lane / 6) + 6 * (lane % 6);
        for (int e = 0; e < 6; ++e) W[e] = sv[e];
        lds[600 + lane] -= sv[0] * yk[0] + sv[1] * yk[1] + sv[2] * yk[2] + sv[3] * yk[3] + sv[4] * yk[4] + sv[5] * yk[5];
      }
      acc += lds[600 + (lane + 1) % 42];  // next step depends on this one
      lds[36 * ((it + 1) & 7)] = 1.0 + acc * 1e-12;
    }
    T1(6, 21);
  }
  if (wave == 0) {
    // 8. back-substitution step chain: L_kk (11 b128) + y'_k (3 b128) + per lane one
    //    coupled row's y' (b64) and B column (6 b64), bwd6, x by 6 lanes, y' update; 28 steps
    double* kf = lds + 4096;   // 36 doubles per k
    double* Sm = lds + 6144;
    T0();
    for (int k = 27; k >= 0; --k) {
      double Lk[21], rk[6], x[6];
      const double* o = kf + 36 * (k & 31);
      for (int e = 0; e < 20; e += 2) {
        const double2 v = reinterpret_cast<const double2*>(o)[e / 2];
        Lk[e] = v.x;
        Lk[e + 1] = v.y;
      }
      Lk[20] = o[20];
      for (int e = 0; e < 6; ++e) rk[e] = o[24 + e];
      for (int e = 0; e < 6; ++e) x[e] = o[30 + e];
      const int row = (k + 1 + lane / 6) & 31, cc = lane % 6;
      const double yv = kf[36 * row + 30 + cc];
      double col[6];
      const double* B = Sm + 36 * ((k * 7 + lane / 6) & 31) + cc;
      for (int rr = 0; rr < 6; ++rr) col[rr] = B[6 * rr];
      for (int i = 5; i >= 0; --i) {
        double s = x[i];
        for (int mm = i + 1; mm < 6; ++mm) s -= Lk[P6(mm, i)] * x[mm];
        x[i] = s * rk[i];
      }
      if (lane < 6) {
        double v = 0.0;
        for (int e = 0; e < 6; ++e) v = lane == e ? x[e] : v;
        kf[36 * (k & 31) + 30 + lane] = v;
      }
      if (lane < 42)
        kf[36 * row + 30 + cc] = yv - (col[0] * x[0] + col[1] * x[1] + col[2] * x[2] + col[3] * x[3] + col[4] * x[4] + col[5] * x[5]);
      __builtin_amdgcn_wave_barrier();
    }
    T1(7, 28);
  }
  // 6. barrier with four waves (no other work)
  __syncthreads();
  T0();
  for (int it = 0; it < 64; ++it) {
    __syncthreads();
  }
  T1(5, 64);
  out[l] = acc;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 8);
  hipMalloc(&cyc, 16 * 8);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(parts, dim3(1), dim3(256), 0, 0, out, cyc, 1.0);
    hipDeviceSynchronize();
  }
  unsigned long long h[16];
  hipMemcpy(h, cyc, 16 * 8, hipMemcpyDeviceToHost);
  printf("chol6 (dependent)              %llu cyc\n", h[0]);
  printf("fwd6 (dependent)               %llu cyc\n", h[1]);
  printf("17 x 1-lane b128 st + ld       %llu cyc\n", h[2]);
  printf("64-lane b128 st + ld           %llu cyc\n", h[3]);
  printf("task (16 b128 ld, 72 fma, st)  %llu cyc\n", h[4]);
  printf("__syncthreads, 4 waves         %llu cyc\n", h[5]);
  printf("panel part of a step (1 wave)  %llu cyc\n", h[6]);
  printf("back-substitution step         %llu cyc\n", h[7]);
  return 0;
}
