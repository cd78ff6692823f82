// PnP kernel arguments shared by pnp.hip and pnp_group.hip (the lane-group hypothesis kernel,
// a translation unit of its own: in pnp.hip beside the batch kernel it changed that kernel's
// register allocation at its 512-register edge, 300 -> 372 B of scratch per lane).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "pnp_math.h"

namespace vo {

struct PnpArgs {
  const float* X;          // (total, 3) object points, frames back to back
  const float* uv;         // (total, 2) image points
  const int32_t* off;      // (batch + 1) frame offsets
  const int32_t* subsets;  // (batch, H, 5) RANSAC subsets (frames with n > 5)
  double* models;          // (batch, H, kModel)
  int32_t* counts;         // (batch, H) inlier counts
  double* pose;            // (batch, 6) rvec, tvec
  int32_t* status;         // (batch, 2) success, inliers
  uint8_t* mask;           // (total) inliers of the best model
  pnpm::Cam K;
  float thr2;              // (float)(reproj_err^2)
  double confidence;
  int batch, H;
};

__device__ __forceinline__ void load3(const float* X, int i, float (&M)[3]) {
  M[0] = X[3l * i];
  M[1] = X[3l * i + 1];
  M[2] = X[3l * i + 2];
}

// lanes per hypothesis of the group kernel (pnpm::Svd12Alt's groups)
constexpr int kPnpGroupLanes = pnpm::kSvdGroupLanes;
// Hypotheses [h_lo, h_hi) of every frame (of the frames with need[f] != 0), kPnpGroupLanes lanes
// each; nh = batch * (h_hi - h_lo).  Enqueued on st.
void pnp_hyp_group_launch(const PnpArgs& a, int h_lo, int h_hi, const int32_t* need, int nh, hipStream_t st);

}  // namespace vo
