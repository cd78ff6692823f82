// K2's slab reduction (shared by ba_reduce_kernel in ba.hip and the reducer workgroups of the
// fused K2 + K3 launch in ba_band.hip): arguments, fixed-order row sums, partition constants.
#pragma once

#include <hip/hip_runtime.h>

namespace vo {

// K2: fixed-order reduction of the slabs into [S profile | b | cost].
struct ReduceArgs {
  int nprof, F, nseg;
  double lambda;
  // per profile block, host-built (BAEngine::setup) so that one load level gives every
  // address: slab rows [x, y); on a diagonal block its camera's rhs slab entries [z, w)
  // (z < 0 otherwise)
  const int4* meta;
  // per profile block: output offset of its 36 values (| kRedTranspose), of its rhs (diagonal)
  const int2* out;
  const double* slab;
  const double* slab_b;
  const double* slab_cost;
  double* sys;         // output: profile [S | b | cost] or the banded K3's column layout
  long cost_off;       // output offset of the cost
  const int* status;
};
constexpr int kRedTranspose = 1 << 30;  // dst flag: store the block transposed

// Sums slab rows k0 + part + j*stride (entry e of each, rows of W doubles), j = 0, 1, ...,
// in fixed order.  K1 wrote each block's window slots to consecutive rows in prof_src order,
// so this is the former gather, bit for bit.  Rows go in batches of kRedBatch loads, all in
// flight at once: the loads are unconditional (index clamped into [k0, k1)) and a row past
// the end adds +0.0, which leaves the sum unchanged bit for bit (acc starts at +0.0, so it is
// never -0.0).  A serial tail loop here cost one global round trip per leftover row: a
// block of 40 rows took five dependent round trips in its threads.
#ifndef VO_RED_BATCH
#define VO_RED_BATCH 16
#endif
constexpr int kRedBatch = VO_RED_BATCH;
// Rows per batch: as many as the block's busiest part needs, up to kRedBatch (uniform per block:
// k0, k1 and stride are).  A batch larger than the rows only adds clamped duplicate loads (each a
// whole wave-instruction through L1: at cfg3's ~2 rows per part, 16-row batches issued 8x the
// loads); the sum adds the same rows in the same order either way.
template <int B, int W>
__device__ __forceinline__ void sum_rows_b(const double* __restrict__ slab, int k0, int k1, int part, int stride,
                                           int e, double& acc) {
  for (int k = k0 + part; k < k1; k += B * stride) {
    double v[B];
#pragma unroll
    for (int i = 0; i < B; ++i) v[i] = slab[(long)W * min(k + i * stride, k1 - 1) + e];
#pragma unroll
    for (int i = 0; i < B; ++i) acc += k + i * stride < k1 ? v[i] : 0.0;
  }
}
template <int W>
__device__ __forceinline__ double sum_rows(const double* __restrict__ slab, int k0, int k1, int part,
                                           int stride, int e) {
  double acc = 0.0;
  if (k1 <= k0) return acc;  // no rows (uniform per block)
  const int per = (k1 - k0 + stride - 1) / stride;
  if (per <= 2) sum_rows_b<2, W>(slab, k0, k1, part, stride, e, acc);
  else if (per <= 4) sum_rows_b<4, W>(slab, k0, k1, part, stride, e, acc);
  else sum_rows_b<kRedBatch, W>(slab, k0, k1, part, stride, e, acc);
  return acc;
}

// The same for 36-double S rows with 16-byte loads: lane (part, e2) sums entries 2 e2, 2 e2 + 1
// of rows k0 + part + j * stride in fixed order (18 lanes cover a row's 288 contiguous bytes).
template <int B>
__device__ __forceinline__ void sum_rows2_b(const double2* __restrict__ s2, int k0, int k1, int part, int stride,
                                            int e2, double2& acc) {
  for (int k = k0 + part; k < k1; k += B * stride) {
    double2 v[B];
#pragma unroll
    for (int i = 0; i < B; ++i) v[i] = s2[18l * min(k + i * stride, k1 - 1) + e2];
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const bool on = k + i * stride < k1;
      acc.x += on ? v[i].x : 0.0;
      acc.y += on ? v[i].y : 0.0;
    }
  }
}
__device__ __forceinline__ double2 sum_rows2(const double* __restrict__ slab, int k0, int k1, int part, int stride,
                                             int e2) {
  double2 acc = make_double2(0.0, 0.0);
  if (k1 <= k0) return acc;
  const double2* __restrict__ s2 = reinterpret_cast<const double2*>(slab);
  const int per = (k1 - k0 + stride - 1) / stride;
  if (per <= 2) sum_rows2_b<2>(s2, k0, k1, part, stride, e2, acc);
  else if (per <= 4) sum_rows2_b<4>(s2, k0, k1, part, stride, e2, acc);
  else sum_rows2_b<kRedBatch>(s2, k0, k1, part, stride, e2, acc);
  return acc;
}

#ifndef VO_RED_THREADS
#define VO_RED_THREADS 256
#endif
constexpr int kRedThreads = VO_RED_THREADS;
constexpr int kRedSParts = kRedThreads / 18;  // partial sums per S block entry (16-byte lanes: 18 per row)
constexpr int kRedBParts = kRedThreads / 6;   // partial sums per rhs entry

}  // namespace vo
