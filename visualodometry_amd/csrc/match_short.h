// Float-descriptor shortlist matcher (match_bf16.hip), launched by match_run (match.hip).
#pragma once

#include "vo_ctx.h"

namespace vo {

struct ShortArgs {
  const float* da;
  const float* db;
  __bf16* ha;           // (batch, n0_pad, Dp) bf16 query image
  __bf16* hb;           // (batch, n1_pad, Dp) bf16 train image
  float* nbq;           // (batch, n1_pad) |b'|^2, +inf for padding columns
  float* ra;            // (batch, n0_pad) |a|
  uint32_t* bmax;       // max |b| (float bits) of frame pair b at bmax[kBmaxStride b]; zero between calls
  float2* part;         // (batch, nsplit, n0_pad) top-2 of A per split
  uint32_t* mask;       // candidate bits (fsweep<2>): (batch, n0_pad / 32, ceil(n1_pad / 64), 64 lanes)
                        // words, see short_mask_word in match_bf16.hip
  int n0, n1, dim, Dp, n0_pad, n1_pad, split_w, nsplit;
  long a_bstride, b_bstride;
  const uint32_t* flag;  // [0] == gen: not SIFT integers; [1] == gen: a non-finite value
  uint32_t gen;
  int forced;            // float hint: no int8 pack ran; fpack itself flags non-finite values
  double ratio;
  int32_t* best;
  int32_t* idx2;
  float* dist2;
};

// words between two frame pairs' max |b| counters: one 128-byte line each (the fpack
// workgroups' atomicMax on one shared line cost ~15 us per call)
constexpr int kBmaxStride = 32;

// bf16 K padding of the shortlist (a multiple of 32, at most 256 for dim <= 256)
inline int short_Dp(int dim) { return (dim + 31) / 32 * 32; }
void short_launch(vo_ctx* ctx, ShortArgs& a, int batch);

}  // namespace vo
