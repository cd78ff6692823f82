// PnP-RANSAC, the reference's tracking step, on gfx950.
//
// Replaces cv2.solvePnPRansac(pnp_3d, pnp_2d, K, None, reprojectionError=...) at reference
// src/modules/vo.py:135-141 (defaults: 100 iterations, confidence 0.99,
// SOLVEPNP_ITERATIVE).  The restatement it is checked against, with every OpenCV
// routine it follows, is oracle/pnp_ref.py; this file keeps that operation order (no FMA
// contraction) so the two agree to rounding.
//
// OpenCV runs the RANSAC loop serially, but its hypotheses do not depend on each other:
// the subsets come from cv::RNG((uint64)-1) alone (drawn here on the host, ransac_subsets)
// and only the early-exit count `niters` depends on earlier inlier counts.  So every
// hypothesis of every frame is solved and scored at once, and the serial bookkeeping is
// replayed afterwards over the inlier counts, which picks exactly the model the serial
// loop picks.  Three launches per batch of frames:
//   pnp_hyp_kernel    one thread per (frame, hypothesis): EPnP on 5 points (three
//                     one-sided Jacobi SVDs, a 12x12 one among them, three beta
//                     approximations with 5 Householder Gauss-Newton steps each), then
//                     the Rodrigues round trip the model makes through (rvec, tvec);
//   pnp_score_kernel  one workgroup per (frame, group of hypotheses): float32 reprojection error
//                     of every point, inlier count;
//   pnp_final_kernel  one workgroup per frame: RANSAC replay (best model, niters update),
//                     inlier mask of the best model, Levenberg-Marquardt refinement on the
//                     inliers (fixed-order block reductions), Rodrigues to rvec.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "pnp_math.h"
#include "vo_ctx.h"

#pragma clang fp contract(off)

namespace vo {
namespace {

using namespace pnpm;

// ---------------------------------------------------------------- kernels
constexpr int kScoreGroupMax = 128;  // hypotheses scored by one workgroup, at most
constexpr int kScoreRegPts = 4;      // points per thread held in registers (frames up to 1024 points)

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
  Cam K;
  float thr2;              // (float)(reproj_err^2)
  double confidence;
  int batch, H;
};

__device__ __forceinline__ void load3(const float* X, int i, float (&M)[3]) {
  M[0] = X[3l * i];
  M[1] = X[3l * i + 1];
  M[2] = X[3l * i + 2];
}

__global__ __launch_bounds__(64) void pnp_hyp_kernel(PnpArgs a) {
  const int g = blockIdx.x * 64 + threadIdx.x;
  if (g >= a.batch * a.H) return;
  const int f = g / a.H, h = g - f * a.H;
  const int o = a.off[f], n = a.off[f + 1] - o;
  double* model = a.models + (size_t)g * kModel;
  const bool run = n > kPts || (n == kPts && h == 0);
  if (!run) {
    model[15] = 0.0;
    return;
  }
  EpnpState S;
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
  const bool ok = epnp5(S, a.K, R, t);
  double rv[3], Rm[3][3];
  rodrigues_to_vec(R, rv);
  rodrigues_to_mat(rv, Rm);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) model[3 * i + j] = Rm[i][j];
    model[9 + i] = t[i];
    model[12 + i] = rv[i];
  }
  model[15] = ok ? 1.0 : 0.0;
}

__global__ __launch_bounds__(256) void pnp_score_kernel(PnpArgs a, int group) {
  // one workgroup per (frame, group of `group` hypotheses): the frame's points stay in L1
  // across its hypotheses; the host sizes groups so the grid still fills the chip
  const int ngroups = (a.H + group - 1) / group;
  const int f = blockIdx.x / ngroups, h0 = (blockIdx.x % ngroups) * group, h1 = min(h0 + group, a.H);
  const int o = a.off[f], n = a.off[f + 1] - o;
  __shared__ int s_count[kScoreGroupMax];
  for (int h = threadIdx.x; h < h1 - h0; h += 256) s_count[h] = 0;
  __syncthreads();
  if (n > kPts && n <= kScoreRegPts * 256) {
    // the thread's points in registers for all the group's hypotheses, two hypotheses per
    // pass (independent chains through the f64 division); per point the same arithmetic
    float P[kScoreRegPts][5];
#pragma unroll
    for (int u = 0; u < kScoreRegPts; ++u) {
      const int i = min((int)threadIdx.x + 256 * u, n - 1);
      const float2 q = reinterpret_cast<const float2*>(a.uv)[o + i];
      float M[3];
      load3(a.X, o + i, M);
      P[u][0] = M[0];
      P[u][1] = M[1];
      P[u][2] = M[2];
      P[u][3] = q.x;
      P[u][4] = q.y;
    }
    auto score = [&](const double* model) __attribute__((always_inline)) {
      double R[9], t[3];
#pragma unroll
      for (int k = 0; k < 9; ++k) R[k] = model[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) t[k] = model[9 + k];
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < kScoreRegPts; ++u) {
        const float M[3] = {P[u][0], P[u][1], P[u][2]};
        cnt += ((int)threadIdx.x + 256 * u < n && is_inlier(R, t, M, P[u][3], P[u][4], a.K, a.thr2)) ? 1 : 0;
      }
      return cnt;
    };
    for (int h = h0; h < h1; h += 2) {
      const double* m0 = a.models + ((size_t)f * a.H + h) * kModel;  // uniform
      const double* m1 = a.models + ((size_t)f * a.H + min(h + 1, h1 - 1)) * kModel;
      const bool on0 = m0[15] != 0.0, on1 = h + 1 < h1 && m1[15] != 0.0;
      int c0 = on0 ? score(m0) : 0;
      int c1 = on1 ? score(m1) : 0;
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) {
        c0 += __shfl_xor(c0, m, 64);
        c1 += __shfl_xor(c1, m, 64);
      }
      if ((threadIdx.x & 63) == 0) {
        if (c0) atomicAdd(&s_count[h - h0], c0);
        if (c1) atomicAdd(&s_count[h + 1 - h0], c1);
      }
    }
  } else if (n > kPts) {
    for (int h = h0; h < h1; ++h) {
      const double* model = a.models + ((size_t)f * a.H + h) * kModel;  // uniform
      if (model[15] == 0.0) continue;
      double R[9], t[3];
#pragma unroll
      for (int k = 0; k < 9; ++k) R[k] = model[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) t[k] = model[9 + k];
      int cnt = 0;
      for (int i = threadIdx.x; i < n; i += 256) {
        const float2 q = reinterpret_cast<const float2*>(a.uv)[o + i];
        float M[3];
        load3(a.X, o + i, M);
        cnt += is_inlier(R, t, M, q.x, q.y, a.K, a.thr2) ? 1 : 0;
      }
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) cnt += __shfl_xor(cnt, m, 64);
      if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s_count[h - h0], cnt);
    }
  }
  __syncthreads();
  for (int h = threadIdx.x; h < h1 - h0; h += 256) a.counts[(size_t)f * a.H + h0 + h] = s_count[h];
}

// Sum of one double over a wave in a fixed order (butterfly).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = v + __shfl_xor(v, m, 64);
  return v;
}

// Normal equations of the inliers at (R, t): this thread's partial sums (points i = tid mod 256).
__device__ __forceinline__ void lm_accumulate(const PnpArgs& a, int o, int n, const double* R, const double* t,
                                              double (&acc)[kNe]) {
#pragma unroll
  for (int k = 0; k < kNe; ++k) acc[k] = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    if (!a.mask[o + i]) continue;
    float M[3];
    load3(a.X, o + i, M);
    const float2 q = reinterpret_cast<const float2*>(a.uv)[o + i];
    lm_point(R, t, M, q.x, q.y, a.K, acc);
  }
}

__device__ __forceinline__ void lm_reduce(double (&acc)[kNe], double* red, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kNe; ++k) {
    const double v = wave_sum(acc[k]);
    if (lane == 0) red[wave * kNe + k] = v;
  }
  __syncthreads();
  if (threadIdx.x < kNe) {
    const int k = threadIdx.x;
    out[k] = ((red[k] + red[kNe + k]) + red[2 * kNe + k]) + red[3 * kNe + k];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256, 2) void pnp_final_kernel(PnpArgs a) {  // two per CU: <= 256 VGPRs
  const int f = blockIdx.x;
  const int o = a.off[f], n = a.off[f + 1] - o;
  __shared__ int s_best, s_count, s_go;
  __shared__ double s_R[9], s_t[3];
  __shared__ double s_red[4 * kNe];
  __shared__ double s_ne[kNe];
  if (threadIdx.x == 0) {
    // the serial RANSAC loop of RANSACPointSetRegistrator::run over the precomputed counts
    int best = -1;
    if (n == kPts) {
      best = a.models[(size_t)f * a.H * kModel + 15] != 0.0 ? 0 : -1;
    } else if (n > kPts) {
      int niters = a.H, max_good = 0;
      for (int it = 0; it < niters; ++it) {
        const size_t g = (size_t)f * a.H + it;
        if (a.models[g * kModel + 15] == 0.0) continue;
        const int good = a.counts[g];
        if (good > (max_good > kPts - 1 ? max_good : kPts - 1)) {
          best = it;
          max_good = good;
          niters = update_num_iters(a.confidence, (double)(n - good) / n, kPts, niters);
        }
      }
    }
    s_best = best;
    s_count = 0;
  }
  __syncthreads();
  const int best = s_best;
  const double* model = a.models + ((size_t)f * a.H + (best < 0 ? 0 : best)) * kModel;
  if (best < 0 || n == kPts) {
    for (int i = threadIdx.x; i < n; i += 256) a.mask[o + i] = best < 0 ? 0 : 1;
    if (threadIdx.x == 0) {
      for (int k = 0; k < 3; ++k) {
        a.pose[6 * f + k] = best < 0 ? 0.0 : model[12 + k];
        a.pose[6 * f + 3 + k] = best < 0 ? 0.0 : model[9 + k];
      }
      a.status[2 * f] = best < 0 ? 0 : 1;
      a.status[2 * f + 1] = best < 0 ? 0 : n;
    }
    return;
  }
  double R[9], t[3];
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = model[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) t[k] = model[9 + k];
  int cnt = 0;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float2 q = reinterpret_cast<const float2*>(a.uv)[o + i];
    float M[3];
    load3(a.X, o + i, M);
    const bool in = is_inlier(R, t, M, q.x, q.y, a.K, a.thr2);
    a.mask[o + i] = in ? 1 : 0;
    cnt += in ? 1 : 0;
  }
  if (cnt) atomicAdd(&s_count, cnt);
  // lm_accumulate reads mask[o + i] for the same i this thread wrote (same stride).
  // Levenberg-Marquardt on the inliers: thread 0 holds the state (pnp_math.h LmState),
  // every pass evaluates the normal equations at the pose in s_R/s_t.
  double acc[kNe];
  lm_accumulate(a, o, n, R, t, acc);
  lm_reduce(acc, s_red, s_ne);
  LmState lm;
  if (threadIdx.x == 0) {
    lm.init(R, t, s_ne);
    s_go = lm.propose(s_R, s_t) ? 1 : 0;
  }
  __syncthreads();
  while (s_go) {
    double nR[9], nt[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) nR[k] = s_R[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) nt[k] = s_t[k];
    lm_accumulate(a, o, n, nR, nt, acc);
    lm_reduce(acc, s_red, s_ne);  // ends with a barrier: every thread has read s_R/s_t
    if (threadIdx.x == 0) s_go = lm.update(nR, nt, s_ne) && lm.propose(s_R, s_t) ? 1 : 0;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double Rf[3][3], rv[3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Rf[i][j] = lm.R[3 * i + j];
    rodrigues_to_vec(Rf, rv);
    for (int k = 0; k < 3; ++k) {
      a.pose[6 * f + k] = rv[k];
      a.pose[6 * f + 3 + k] = lm.t[k];
    }
    a.status[2 * f] = 1;
    a.status[2 * f + 1] = s_count;
  }
}

}  // namespace

// cv::RNG((uint64)-1) subsets of getSubset (ptsetreg.cpp) for `count` points.
void pnp_subsets(int count, int iters, int32_t* out) {
  uint64_t state = ~0ull;
  auto next = [&]() -> uint32_t {
    state = (uint64_t)(uint32_t)state * 4164903690ull + (state >> 32);
    return (uint32_t)state;
  };
  for (int it = 0; it < iters; ++it) {
    int32_t* idx = out + (size_t)it * kPts;
    for (int i = 0; i < kPts; ++i) {
      int j;
      bool dup;
      do {
        j = (int)(next() % (uint32_t)count);
        dup = false;
        for (int k = 0; k < i; ++k) dup |= idx[k] == j;
      } while (dup);
      idx[i] = j;
    }
  }
}

void pnp_run(vo_ctx* ctx, const float* d_X, const float* d_uv, const int32_t* offsets, int batch,
             const double* K, int iterations, double reproj_err, double confidence, double* d_pose,
             uint8_t* d_mask, int32_t* d_status) {
  VO_REQUIRE(batch >= 0 && offsets && K, VO_ERR_ARG, "pnp: bad arguments (batch=%d)", batch);
  VO_REQUIRE(confidence > 0 && confidence < 1, VO_ERR_ARG, "pnp: confidence %g not in (0, 1)", confidence);
  if (batch == 0) return;
  const int H = iterations > 1 ? iterations : 1;
  VO_REQUIRE(H <= 65536, VO_ERR_ARG, "pnp: iterations %d > 65536", H);
  VO_REQUIRE(offsets[0] == 0, VO_ERR_ARG, "pnp: offsets[0] must be 0");
  for (int f = 0; f < batch; ++f)
    VO_REQUIRE(offsets[f + 1] >= offsets[f], VO_ERR_ARG, "pnp: offsets not ascending at frame %d", f);
  PnpWorkspace& ws = ctx->pnp;
  // subsets depend only on (count, H): regenerate and upload when the frame layout changed
  const bool same = ws.H == H && (int)ws.offsets.size() == batch + 1 &&
                    std::memcmp(ws.offsets.data(), offsets, sizeof(int32_t) * (batch + 1)) == 0;
  if (!same) {
    std::vector<int32_t> sub((size_t)batch * H * kPts, 0);
    std::vector<int32_t> cache;
    int cached = -1;
    for (int f = 0; f < batch; ++f) {
      const int n = offsets[f + 1] - offsets[f];
      if (n <= kPts) continue;
      if (n != cached) {
        cache.resize((size_t)H * kPts);
        pnp_subsets(n, H, cache.data());
        cached = n;
      }
      std::memcpy(&sub[(size_t)f * H * kPts], cache.data(), cache.size() * sizeof(int32_t));
    }
    ws.sub.reserve(sub.size() * sizeof(int32_t));
    ws.off.reserve((size_t)(batch + 1) * sizeof(int32_t));
    VO_HIP_CHECK(hipMemcpyAsync(ws.sub.ptr, sub.data(), sub.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                                ctx->stream));
    VO_HIP_CHECK(hipMemcpyAsync(ws.off.ptr, offsets, (size_t)(batch + 1) * sizeof(int32_t),
                                hipMemcpyHostToDevice, ctx->stream));
    VO_HIP_CHECK(hipStreamSynchronize(ctx->stream));  // the host vectors go out of scope
    ws.offsets.assign(offsets, offsets + batch + 1);
    ws.H = H;
  }
  ws.models.reserve((size_t)batch * H * kModel * sizeof(double));
  ws.counts.reserve((size_t)batch * H * sizeof(int32_t));
  PnpArgs a;
  a.X = d_X;
  a.uv = d_uv;
  a.off = ws.off.as<int32_t>();
  a.subsets = ws.sub.as<int32_t>();
  a.models = ws.models.as<double>();
  a.counts = ws.counts.as<int32_t>();
  a.pose = d_pose;
  a.status = d_status;
  a.mask = d_mask;
  a.K = Cam{K[0], K[4], K[2], K[5]};
  a.thr2 = (float)(reproj_err * reproj_err);
  a.confidence = confidence;
  a.batch = batch;
  a.H = H;
  const int nh = batch * H;
  ctx->prof.begin(ctx->stream, kKPnpHyp);
  hipLaunchKernelGGL(pnp_hyp_kernel, dim3(ceil_div(nh, 64)), dim3(64), 0, ctx->stream, a);
  ctx->prof.end(ctx->stream);
  VO_HIP_CHECK(hipGetLastError());
  ctx->prof.begin(ctx->stream, kKPnpScore);
  // hypotheses per scoring workgroup: one for small batches (single-frame latency), up to
  // kScoreGroupMax while the grid keeps ~4 workgroups per CU
  const int group = std::max(1, std::min({H, kScoreGroupMax, nh / std::max(1, 4 * ctx->num_cus)}));
  const int ngroups = ceil_div(H, group);
  hipLaunchKernelGGL(pnp_score_kernel, dim3(batch * ngroups), dim3(256), 0, ctx->stream, a, group);
  ctx->prof.end(ctx->stream);
  VO_HIP_CHECK(hipGetLastError());
  ctx->prof.begin(ctx->stream, kKPnpFinal);
  hipLaunchKernelGGL(pnp_final_kernel, dim3(batch), dim3(256), 0, ctx->stream, a);
  ctx->prof.end(ctx->stream);
  VO_HIP_CHECK(hipGetLastError());
}

}  // namespace vo
