// Critical-lane block step of the banded K3 (ba_band.hip, kCl layout): the pieces of one
// block column's elimination that sit on the dependent chain, in one 16-lane DPP row.
//
// Lane li (0..15) of a DPP row holds one scalar row of the panel [A_kk; A_{k+1,k}; y_k]:
//   li 0..5   row li of the diagonal block A_kk (lower part meaningful),   register a[]
//   li 6..11  row li - 6 of the sub-diagonal block A_{k+1,k},              register pp[]
//   li 12     the rhs row y_k,                                            register a[]
//   li 13..15 zero rows.
// Every value another lane needs reaches it by a DPP64 row broadcast (row_newbcast:n: lane n
// of the lane's own 16-lane row), fused into the consuming v_fmac_f64 where the compiler can:
// no LDS round trip and no barrier on the chain.  The four rows of a wave run the same
// instructions on the same data (addresses from li only), so any row's result is the row-0
// result.
#pragma once

#include <hip/hip_runtime.h>

#include "ba_math.h"

namespace vo {
namespace cl {

constexpr int kNewBcast = 0x150;  // DPP row_newbcast:n (gfx90a+, DPP64-legal)
constexpr int kRowShl = 0x100;    // DPP row_shl:n: lane i reads lane i + n of its row

template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
  const long v = __builtin_amdgcn_update_dpp(0l, __builtin_bit_cast(long, x), CTRL, 0xf, 0xf, true);
  return __builtin_bit_cast(double, v);
}
// lane N of this lane's 16-lane row
template <int N>
__device__ __forceinline__ double nb(double x) {
  return dpp64<kNewBcast + N>(x);
}

// Right-looking factorisation of the panel: for each pivot p, every lane takes lane p's
// a[p] (the pivot), its reciprocal square root (v_rsq_f64 + one Newton step, as chol6), scales
// its own a[p] (lanes > p: L_lp; lane p: L_pp; lane 12: y'_p) and subtracts L_cp a[p] from a[c]
// for c > p (L_cp from lane c).  Lanes 0..5 end with the rows of L_kk, lane 12 with
// y'_k = L_kk^-1 y_k; every lane holds r = 1/diag(L_kk).  A non-positive pivot gives a NaN or
// inf r, which the caller detects (the "not SPD" outcome).
__device__ __forceinline__ void pivots(double (&a)[6], double (&r)[6]) {
#pragma unroll
  for (int p = 0; p < 6; ++p) {
    double d;
    switch (p) {
      case 0: d = nb<0>(a[0]); break;
      case 1: d = nb<1>(a[1]); break;
      case 2: d = nb<2>(a[2]); break;
      case 3: d = nb<3>(a[3]); break;
      case 4: d = nb<4>(a[4]); break;
      default: d = nb<5>(a[5]); break;
    }
    double q = __builtin_amdgcn_rsq(d);
    if (kCholNewton) q = __builtin_fma(0.5 * q, __builtin_fma(-(d * q), q, 1.0), q);
    r[p] = q;
    a[p] *= q;
#pragma unroll
    for (int c = p + 1; c < 6; ++c) {
      double l;
      switch (c) {
        case 1: l = nb<1>(a[p]); break;
        case 2: l = nb<2>(a[p]); break;
        case 3: l = nb<3>(a[p]); break;
        case 4: l = nb<4>(a[p]); break;
        default: l = nb<5>(a[p]); break;
      }
      a[c] = __builtin_fma(-l, a[p], a[c]);
    }
  }
}

// The two helpers below are single asm blocks of v_fmac_f64_dpp (the compiler does not fuse a
// 64-bit DPP move into an FMA).  Inside a block no DPP source is written; the leading s_nop 1
// gives the two wait states a DPP read needs after the VALU write of its source, wherever the
// compiler puts that write.
// x <- x - u V^T with V = the 6x6 block whose row c sits in lane B + c of v[] (broadcast; B = 6
// in the chain wave, 0 in the trailing waves); per output c the subtractions run in m order
// (x_c - u_0 V_c0 - u_1 V_c1 ...).
template <int B>
__device__ __forceinline__ void sub_uvt(double (&x)[6], const double (&u)[6], const double (&v)[6]) {
  static_assert(B == 0 || B == 6, "V rows in lanes 0..5 or 6..11");
  if constexpr (B == 6) {
    asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %0, -%6, %12 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%6, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%6, %12 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%6, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%6, %12 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%6, %12 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, -%7, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%7, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%7, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%7, %13 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%7, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%7, %13 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, -%8, %14 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%8, %14 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%8, %14 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%8, %14 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%8, %14 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%8, %14 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, -%9, %15 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%9, %15 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%9, %15 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%9, %15 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%9, %15 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%9, %15 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, -%10, %16 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%10, %16 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%10, %16 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%10, %16 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%10, %16 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%10, %16 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, -%11, %17 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%11, %17 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%11, %17 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%11, %17 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%11, %17 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%11, %17 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5])
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]),
        "v"(u[0]), "v"(u[1]), "v"(u[2]), "v"(u[3]), "v"(u[4]), "v"(u[5]));
  } else {
    asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %0, -%6, %12 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%6, %12 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%6, %12 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%6, %12 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%6, %12 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%6, %12 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, -%7, %13 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%7, %13 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%7, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%7, %13 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%7, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%7, %13 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, -%8, %14 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%8, %14 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%8, %14 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%8, %14 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%8, %14 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%8, %14 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, -%9, %15 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%9, %15 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%9, %15 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%9, %15 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%9, %15 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%9, %15 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, -%10, %16 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%10, %16 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%10, %16 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%10, %16 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%10, %16 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%10, %16 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, -%11, %17 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, -%11, %17 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%11, %17 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%11, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%11, %17 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%11, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5])
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]),
        "v"(u[0]), "v"(u[1]), "v"(u[2]), "v"(u[3]), "v"(u[4]), "v"(u[5]));
  }
}

// x <- x L_kk^-T (solve x L^T = x) with L_kk in lanes 0..5 of a[] and r = 1/diag; right-looking
// (after x_m is final every later x_j subtracts L_jm x_m), which is fwd6's operation order.
__device__ __forceinline__ void solve_lt(double (&x)[6], const double (&a)[6], const double (&r)[6]) {
  asm("s_nop 1\n\t"
      "v_mul_f64 %0, %0, %12\n\t"
      "v_fmac_f64_dpp %1, -%6, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, -%6, %0 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%6, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%6, %0 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%6, %0 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_mul_f64 %1, %1, %13\n\t"
      "v_fmac_f64_dpp %2, -%7, %1 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, -%7, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%7, %1 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%7, %1 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_mul_f64 %2, %2, %14\n\t"
      "v_fmac_f64_dpp %3, -%8, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, -%8, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%8, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_mul_f64 %3, %3, %15\n\t"
      "v_fmac_f64_dpp %4, -%9, %3 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, -%9, %3 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_mul_f64 %4, %4, %16\n\t"
      "v_fmac_f64_dpp %5, -%10, %4 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_mul_f64 %5, %5, %17\n\t"
      : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]),
        "v"(r[0]), "v"(r[1]), "v"(r[2]), "v"(r[3]), "v"(r[4]), "v"(r[5]));
}

// u for the next panel's lanes 0..5: row li of L_{k+1,k} (lane li + 6 of pp[]).
__device__ __forceinline__ void shl6(const double (&pp)[6], double (&u)[6]) {
#pragma unroll
  for (int m = 0; m < 6; ++m) u[m] = dpp64<kRowShl + 6>(pp[m]);
}

}  // namespace cl
}  // namespace vo
