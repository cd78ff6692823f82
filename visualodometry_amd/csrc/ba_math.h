// Small fp64 kernels shared by the BA solve kernels (ba.hip, ba_band.hip): 6x6 block
// Cholesky / substitutions in registers and the left se(3) pose update.  Same operation
// order as oracle/ba_ref.py (chol of a 6x6 block, exp map).
#pragma once

#include <hip/hip_runtime.h>

namespace vo {

constexpr double kExpSeriesTh2 = 0.25;  // |phi|^2 below which the exp map uses its series

__device__ __forceinline__ void se3_exp_apply(const double* d, const double* T, double* out) {
  const double r0 = d[0], r1 = d[1], r2 = d[2], p0 = d[3], p1 = d[4], p2 = d[5];
  const double th2 = p0 * p0 + p1 * p1 + p2 * p2;
  double A, B, C;
  if (th2 < kExpSeriesTh2) {
    // A = sin(th)/th, B = (1 - cos(th))/th^2, C = (th - sin(th))/th^3 as even series in th^2
    // (8 terms: truncation < 5e-17 relative for th < 0.5), no sqrt, sincos or division on
    // the tail's chain; the closed form (oracle/ba_ref.py se3_exp) agrees to its own
    // cancellation error (~1e-16 absolute in the update)
    constexpr double cA[8] = {1.0, -1.0 / 6, 1.0 / 120, -1.0 / 5040, 1.0 / 362880, -1.0 / 39916800,
                              1.0 / 6227020800.0, -1.0 / 1307674368000.0};
    constexpr double cB[8] = {1.0 / 2, -1.0 / 24, 1.0 / 720, -1.0 / 40320, 1.0 / 3628800, -1.0 / 479001600,
                              1.0 / 87178291200.0, -1.0 / 20922789888000.0};
    constexpr double cC[8] = {1.0 / 6, -1.0 / 120, 1.0 / 5040, -1.0 / 362880, 1.0 / 39916800,
                              -1.0 / 6227020800.0, 1.0 / 1307674368000.0, -1.0 / 355687428096000.0};
    A = cA[7];
    B = cB[7];
    C = cC[7];
#pragma unroll
    for (int k = 6; k >= 0; --k) {
      A = __builtin_fma(A, th2, cA[k]);
      B = __builtin_fma(B, th2, cB[k]);
      C = __builtin_fma(C, th2, cC[k]);
    }
  } else {
    const double th = sqrt(th2);
    double s, c;
    sincos(th, &s, &c);
    const double it = 1.0 / th, it2 = it * it;
    A = s * it;
    B = (1.0 - c) * it2;
    C = (th - s) * (it2 * it);
  }
  // P = [phi]x, P2 = P P
  const double P[9] = {0, -p2, p1, p2, 0, -p0, -p1, p0, 0};
  double P2[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      P2[3 * i + j] = P[3 * i] * P[j] + P[3 * i + 1] * P[3 + j] + P[3 * i + 2] * P[6 + j];
  double Rd[9], V[9];
#pragma unroll
  for (int e = 0; e < 9; ++e) {
    const double I = (e % 4 == 0) ? 1.0 : 0.0;
    Rd[e] = I + A * P[e] + B * P2[e];
    V[e] = I + B * P[e] + C * P2[e];
  }
  const double td0 = V[0] * r0 + V[1] * r1 + V[2] * r2;
  const double td1 = V[3] * r0 + V[4] * r1 + V[5] * r2;
  const double td2 = V[6] * r0 + V[7] * r1 + V[8] * r2;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      out[3 * i + j] = Rd[3 * i] * T[j] + Rd[3 * i + 1] * T[3 + j] + Rd[3 * i + 2] * T[6 + j];
  }
  out[9] = Rd[0] * T[9] + Rd[1] * T[10] + Rd[2] * T[11] + td0;
  out[10] = Rd[3] * T[9] + Rd[4] * T[10] + Rd[5] * T[11] + td1;
  out[11] = Rd[6] * T[9] + Rd[7] * T[10] + Rd[8] * T[11] + td2;
}

// ---- 6x6 block kernels in registers (packed lower storage, P(i,c) = i(i+1)/2 + c)
#ifndef VO_CHOL_NEWTON
#define VO_CHOL_NEWTON 1
#endif
constexpr bool kCholNewton = VO_CHOL_NEWTON != 0;
__device__ __forceinline__ constexpr int P6(int i, int c) { return i * (i + 1) / 2 + c; }

// In-place Cholesky a = L L^T; r = 1/diag(L) from v_rsq_f64 + one Newton step
// (critical chain per column: rsq + 3 dependent ops instead of sqrt + divide; the
// step takes the ~2^-23 estimate to ~1e-14 relative).
// kDiag = false leaves a[P6(j, j)] unfactored: no solve reads L's diagonal (fwd6/bwd6
// use r = 1/l_jj), only the stored factor does.
template <bool kDiag = true>
__device__ __forceinline__ bool chol6(double (&a)[21], double (&r)[6]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const double d = a[P6(j, j)];
    ok = ok && d > 0.0;
    const double dd = d > 0.0 ? d : 1.0;
    double q = __builtin_amdgcn_rsq(dd);
    if (kCholNewton) q = q * (1.5 - 0.5 * dd * q * q);
    r[j] = q;
    if (kDiag) a[P6(j, j)] = dd * q;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) a[P6(i, j)] *= q;
#pragma unroll
    for (int i = j + 1; i < 6; ++i)
#pragma unroll
      for (int c = j + 1; c <= i; ++c) a[P6(i, c)] -= a[P6(i, j)] * a[P6(c, j)];
  }
  return ok;
}

// v <- L^-1 v (forward substitution); also solves x L^T = v for a row vector.
__device__ __forceinline__ void fwd6(const double (&L)[21], const double (&r)[6], double (&v)[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = v[i];
#pragma unroll
    for (int m = 0; m < i; ++m) s -= L[P6(i, m)] * v[m];
    v[i] = s * r[i];
  }
}

// v <- L^-T v (back substitution).
__device__ __forceinline__ void bwd6(const double (&L)[21], const double (&r)[6], double (&v)[6]) {
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double s = v[i];
#pragma unroll
    for (int m = i + 1; m < 6; ++m) s -= L[P6(m, i)] * v[m];
    v[i] = s * r[i];
  }
}

// 1/sqrt(d) and 1/z without the IEEE sqrt / division sequences: v_rsq_f64 (v_rcp_f64) is
// good to ~2^-23 relative; one Newton step for rsq (~1e-14, as chol6) and two for rcp
// (~1 ulp) -- a short dependent chain on the kernels' latency-bound paths.
__device__ __forceinline__ double rsq_nr(double d) {
  const double q = __builtin_amdgcn_rsq(d);
  return __builtin_fma(0.5 * q, __builtin_fma(-(d * q), q, 1.0), q);
}
// rcp_nr(+-0) = +-inf as IEEE 1/z (the Newton steps alone would give NaN: fma(-0, inf, 1)),
// so a zero-depth observation gives the oracle's infinite residual, not a NaN.
__device__ __forceinline__ double rcp_nr(double z) {
  const double r0 = __builtin_amdgcn_rcp(z);
  double r = __builtin_fma(r0, __builtin_fma(-z, r0, 1.0), r0);
  r = __builtin_fma(r, __builtin_fma(-z, r, 1.0), r);
  return __builtin_isinf(r0) ? r0 : r;
}

// v[lane] for a register array without a runtime index (a runtime index would
// put the whole array in scratch memory).
template <int N>
__device__ __forceinline__ double pick(const double (&v)[N], int lane) {
  double out = 0.0;
#pragma unroll
  for (int e = 0; e < N; ++e) out = lane == e ? v[e] : out;
  return out;
}

// Orders wave 0's own LDS (or, on the global path, memory) traffic between its
// lanes: LDS ops of one wave complete in order; global stores need a fence.
template <bool kLds>
__device__ __forceinline__ void wave_sync() {
  if (!kLds) __threadfence_block();
  __builtin_amdgcn_wave_barrier();
}

// fp64 value of lane l (wave-uniform l): two v_readlane_b32
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// ---- 6-double rows (16-byte aligned) ---------------------------------------------
__device__ __forceinline__ void ld6g(const double* p, double (&v)[6]) {
  const double2* q = reinterpret_cast<const double2*>(p);
  const double2 a0 = q[0], a1 = q[1], a2 = q[2];
  v[0] = a0.x; v[1] = a0.y; v[2] = a1.x; v[3] = a1.y; v[4] = a2.x; v[5] = a2.y;
}
__device__ __forceinline__ void st6g(double* p, const double (&v)[6]) {
  double2* q = reinterpret_cast<double2*>(p);
  q[0] = make_double2(v[0], v[1]);
  q[1] = make_double2(v[2], v[3]);
  q[2] = make_double2(v[4], v[5]);
}
__device__ __forceinline__ double dot6g(const double (&u)[6], const double* w) {
  const double2* q = reinterpret_cast<const double2*>(w);
  const double2 a0 = q[0], a1 = q[1], a2 = q[2];
  return u[0] * a0.x + u[1] * a0.y + u[2] * a1.x + u[3] * a1.y + u[4] * a2.x + u[5] * a2.y;
}

}  // namespace vo
