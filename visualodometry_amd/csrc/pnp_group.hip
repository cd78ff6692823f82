// EPnP hypotheses on lane groups (small batches, the single frame of vo.py:135-141's tracking
// step): see pnp_hyp_group_kernel.  The rest of PnP-RANSAC is pnp.hip.
#include "pnp_args.h"

#include "vo_common.h"

#pragma clang fp contract(off)

namespace vo {
namespace {

using namespace pnpm;

// Groups of kPnpGroupLanes lanes per hypothesis (small batches, where one hypothesis per lane
// leaves the chip idle and the latency of one EPnP chain is the call's): every lane of a group
// runs the hypothesis's serial parts redundantly (same inputs, same values), and EPnP's 12 x 12
// Jacobi SVD runs on the group's lanes.  Step t of a sweep takes the pairs (i, j) with i + j == t
// (at most six, disjoint), two lanes each (half a row's elements per lane, the sums continued
// from one lane to the other in the serial order): in the cyclic order JacobiSVDImpl_ runs, every pair
// touching row i or j comes before (i, j) exactly when its index sum is below i + j, so each row
// receives the same rotations in the same order, and the result is jacobi_rows' bit for bit.  A
// sweep is 21 dependent steps instead of 66 pairs.
constexpr int kSvdDoubles = 12 * 12 + 12;

// (A kernel and translation unit of its own, not a parameter of pnp_hyp_kernel: shared code, a
// template or a folded argument, changed the batch kernel's register allocation at its
// 512-register edge: 300 -> 372..756 B of scratch per lane, the batch leg 1.5 % slower.)
__global__ __launch_bounds__(64) void pnp_hyp_group_kernel(PnpArgs a, int h_lo, int h_hi, const int32_t* need) {
  static_assert(kPnpGroupLanes == 16 && 64 % kPnpGroupLanes == 0, "Svd12Alt's lane groups are 16 lanes");
  const int hr = h_hi - h_lo;
  const int k = (blockIdx.x * 64 + threadIdx.x) / kPnpGroupLanes, r = threadIdx.x % kPnpGroupLanes;
  if (k >= a.batch * hr) return;
  const int f = k / hr, h = h_lo + (k - f * hr);
  if (need && !need[f]) return;
  const int g = f * a.H + h;
  const int o = a.off[f], n = a.off[f + 1] - o;
  double* model = a.models + (size_t)g * kModel;
  const bool run = n > kPts || (n == kPts && h == 0);
  if (!run) {
    if (r == 0) model[15] = 0.0;
    return;
  }
  __shared__ double s_cols[kEpnpColDoubles * 64];
  __shared__ __attribute__((aligned(16))) double s_svd[64 / kPnpGroupLanes][kSvdDoubles];
  EpnpState S;
  S.alphas = Col{s_cols + threadIdx.x, 64};
  S.v = Col{s_cols + kPts * 4 * 64 + threadIdx.x, 64};
#pragma unroll
  for (int p = 0; p < kPts; ++p) {
    const int i = o + (n == kPts ? p : a.subsets[(size_t)g * kPts + p]);
    float M[3];
    load3(a.X, i, M);
    S.pw[p][0] = M[0];
    S.pw[p][1] = M[1];
    S.pw[p][2] = M[2];
    S.us[p][0] = a.uv[2l * i];
    S.us[p][1] = a.uv[2l * i + 1];
  }
  double R[3][3], t[3];
  const Svd12Alt alt{s_svd[threadIdx.x / kPnpGroupLanes], r};
  const bool ok = epnp5(S, a.K, R, t, &alt);
  double rv[3], Rm[3][3];
  rodrigues_to_vec(R, rv);
  rodrigues_to_mat(rv, Rm);
  if (r == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) model[3 * i + j] = Rm[i][j];
      model[9 + i] = t[i];
      model[12 + i] = rv[i];
    }
    model[15] = ok ? 1.0 : 0.0;
  }
}

}  // namespace

void pnp_hyp_group_launch(const PnpArgs& a, int h_lo, int h_hi, const int32_t* need, int nh, hipStream_t st) {
  hipLaunchKernelGGL(pnp_hyp_group_kernel, dim3(ceil_div((int64_t)nh * kPnpGroupLanes, 64)), dim3(64), 0, st, a, h_lo,
                     h_hi, need);
  VO_HIP_CHECK(hipGetLastError());
}

}  // namespace vo
