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
#include "pnp_args.h"

#pragma clang fp contract(off)

namespace vo {
namespace {

using namespace pnpm;

// ---------------------------------------------------------------- kernels
constexpr int kScoreGroupMax = 128;  // hypotheses scored by one workgroup, at most
// pnp_score: threads per workgroup and the points each holds in registers (frames up to 1024
// points take the register path); waves per SIMD the kernel's registers must allow so that one
// workgroup per frame of a 1024-frame batch is one round on 256 CUs
#ifndef VO_PNP_SCORE_THREADS
#define VO_PNP_SCORE_THREADS 256
#endif
constexpr int kScoreThreads = VO_PNP_SCORE_THREADS;
constexpr int kScoreRegPts = 1024 / kScoreThreads;
constexpr int kScoreWavesPerSimd = kScoreThreads / 64;  // four workgroups per CU
#ifndef VO_PNP_SCORE_STEP
#define VO_PNP_SCORE_STEP 8
#endif
constexpr int kScoreStep = VO_PNP_SCORE_STEP;  // hypotheses scored between two replay steps (pnp_score_kernel)
constexpr int kSplitMin = 16;        // hypotheses solved for every frame before the replay decides (pnp_run)





// Hypotheses [h_lo, h_hi) of every frame (of the frames with need[f] != 0 when need is given).
__global__ __launch_bounds__(64) void pnp_hyp_kernel(PnpArgs a, int h_lo, int h_hi, const int32_t* need) {
  const int hr = h_hi - h_lo;
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= a.batch * hr) return;
  const int f = k / hr, h = h_lo + (k - f * hr);
  if (need && !need[f]) return;
  const int g = f * a.H + h;
  const int o = a.off[f], n = a.off[f + 1] - o;
  double* model = a.models + (size_t)g * kModel;
  const bool run = n > kPts || (n == kPts && h == 0);
  if (!run) {
    model[15] = 0.0;
    return;
  }
  // alphas and v in LDS, one column per lane (one wave per workgroup)
  __shared__ double s_cols[kEpnpColDoubles * 64];
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

// The serial loop of RANSACPointSetRegistrator::run (OpenCV calib3d/src/ptsetreg.cpp) over
// precomputed inlier counts.  A hypothesis without a model (EPnP failed) has count 0, which
// never beats max(max_good, kPts - 1): the loop's skip.  State (thread 0's, in LDS): the
// iteration reached, the loop's bound niters (> h_end when it stopped at h_end: the serial loop
// would go on), the best hypothesis (-1: none) and its count.
struct ReplayState {
  int it, niters, best, max_good;
};

__device__ __forceinline__ void replay_init(const PnpArgs& a, ReplayState* st) {
  if (threadIdx.x == 0) *st = ReplayState{0, a.H, -1, 0};
}

// Hypotheses [st->it, stop) of frame f (n > kPts points) whose counts cnt[h - base] (h < stop,
// cnt holding at most kThreads) are in LDS.  Every thread first evaluates the logarithms of the
// niters update for its count (num_iters_terms: they depend on the count alone), then thread 0
// runs the loop, applying them in order.  Every thread of the workgroup calls; two barriers.
template <int kThreads>
__device__ void replay_chunk(const PnpArgs& a, int n, const int* cnt, int base, int stop, ItersTerms* s_terms,
                             ReplayState* st) {
  const int t = threadIdx.x;
  if (base + t < stop && cnt[t] > kPts - 1) s_terms[t] = num_iters_terms(a.confidence, (double)(n - cnt[t]) / n, kPts);
  __syncthreads();
  if (t == 0) {
    ReplayState r = *st;
    for (; r.it < r.niters && r.it < stop; ++r.it) {
      const int good = cnt[r.it - base];
      if (good > (r.max_good > kPts - 1 ? r.max_good : kPts - 1)) {
        r.best = r.it;
        r.max_good = good;
        r.niters = num_iters_apply(s_terms[r.it - base], r.niters);
      }
    }
    *st = r;
  }
  __syncthreads();
}

// The replay over hypotheses [0, h_end) of frame f (n > kPts) from the counts in global memory,
// staged in LDS a chunk of kThreads at a time with independent loads.  Every thread calls; on
// return every thread may read *st.
template <int kThreads>
__device__ void ransac_replay(const PnpArgs& a, int f, int n, int h_end, int* s_cnt, ItersTerms* s_terms,
                              ReplayState* st) {
  replay_init(a, st);
  const int32_t* counts = a.counts + (size_t)f * a.H;
  for (int base = 0; base < h_end; base += kThreads) {
    __syncthreads();  // *st written, the previous chunk consumed
    const int stop = min(min(st->niters, h_end), base + kThreads);  // niters only shrinks
    if (base >= stop) break;  // uniform: every thread read the same *st
    if (base + (int)threadIdx.x < stop) s_cnt[threadIdx.x] = counts[base + threadIdx.x];
    __syncthreads();
    replay_chunk<kThreads>(a, n, s_cnt, base, stop, s_terms, st);
  }
  __syncthreads();
}

// need_out (phase 1 with one workgroup per frame, h_lo = 0): the workgroup then replays the RANSAC
// loop over the counts it just made and writes need_out[f] as pnp_decide would.
// (four workgroups per CU: 1024 one-frame workgroups in one round; the replay's log/pow would
// otherwise take the kernel to 135 VGPRs)
__global__ __launch_bounds__(kScoreThreads, kScoreWavesPerSimd) void pnp_score_kernel(PnpArgs a, int group, int h_lo, int h_hi,
                                                        const int32_t* need, int32_t* need_out) {
  // one workgroup per (frame, group of `group` hypotheses of [h_lo, h_hi)): the frame's points
  // stay in L1 across its hypotheses; the host sizes groups so the grid still fills the chip
  const int ngroups = (h_hi - h_lo + group - 1) / group;
  const int f = blockIdx.x / ngroups, h0 = h_lo + (blockIdx.x % ngroups) * group, h1 = min(h0 + group, h_hi);
  if (need && !need[f]) return;  // uniform per workgroup, before any barrier
  const int o = a.off[f], n = a.off[f + 1] - o;
  __shared__ int s_count[kScoreGroupMax];
  __shared__ ItersTerms s_terms[kScoreGroupMax];
  __shared__ ReplayState s_st;
  for (int h = threadIdx.x; h < h1 - h0; h += kScoreThreads) s_count[h] = 0;
  // With need_out (phase 1, h0 = 0) the replay follows the scoring kScoreStep hypotheses at a
  // time, and the scoring stops where the serial loop stops: its later counts are never read
  // (pnp_decide and pnp_final stop at the same hypothesis).
  const bool incremental = need_out && n > kPts && n <= kScoreRegPts * kScoreThreads;  // uniform
  if (incremental) replay_init(a, &s_st);
  __syncthreads();
  if (n > kPts && n <= kScoreRegPts * kScoreThreads) {
    // the thread's points in registers for all the group's hypotheses
    float P[kScoreRegPts][5];
#pragma unroll
    for (int u = 0; u < kScoreRegPts; ++u) {
      const int i = min((int)threadIdx.x + kScoreThreads * u, n - 1);
      const float2 q = reinterpret_cast<const float2*>(a.uv)[o + i];
      float M[3];
      load3(a.X, o + i, M);
      P[u][0] = M[0];
      P[u][1] = M[1];
      P[u][2] = M[2];
      P[u][3] = q.x;
      P[u][4] = q.y;
    }
    for (int hc = h0; hc < h1;) {  // uniform
      const int hc1 = incremental ? min(hc + kScoreStep, h1) : h1;
      // one hypothesis at a time (at four waves per SIMD the other waves hide the latency of the
      // f64 division); the wave's inliers counted by ballot
      // (the next hypothesis's model is loaded while this one is scored: uniform, scalar loads)
      const double* model = a.models + ((size_t)f * a.H + hc) * kModel;
      double next[13];
#pragma unroll
      for (int k = 0; k < 12; ++k) next[k] = model[k];
      next[12] = model[15];
      for (int h = hc; h < hc1; ++h, model += kModel) {
        double R[9], t[3];
#pragma unroll
        for (int k = 0; k < 9; ++k) R[k] = next[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) t[k] = next[9 + k];
        const bool on = next[12] != 0.0;
        if (h + 1 < hc1) {
#pragma unroll
          for (int k = 0; k < 12; ++k) next[k] = model[kModel + k];
          next[12] = model[kModel + 15];
        }
        if (!on) continue;
        int cnt = 0;
#pragma unroll
        for (int u = 0; u < kScoreRegPts; ++u) {
          const float M[3] = {P[u][0], P[u][1], P[u][2]};
          // every lane tests its (clamped) point, so no lane-divergent branch; the tail lanes' bits are masked
          const bool in = (int)is_inlier(R, t, M, P[u][3], P[u][4], a.K, a.thr2) & (int)((int)threadIdx.x + kScoreThreads * u < n);
          cnt += __popcll(__ballot(in));
        }
        if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&s_count[h - h0], cnt);
      }
      if (incremental) {
        __syncthreads();  // the step's counts are in s_count
        replay_chunk<kScoreGroupMax>(a, n, s_count + (hc - h0), hc, hc1, s_terms, &s_st);
        if (s_st.niters <= hc1) break;  // the serial loop stopped in this step (uniform)
      }
      hc = hc1;
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
#pragma unroll 1  // frames over 1024 points only: kept small, so it does not set the kernel's VGPRs
      for (int i = threadIdx.x; i < n; i += kScoreThreads) {
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
  for (int h = threadIdx.x; h < h1 - h0; h += kScoreThreads) a.counts[(size_t)f * a.H + h0 + h] = s_count[h];
  if (need_out) {  // uniform; here h0 = 0 and h1 = h_hi
    if (n > kPts && !incremental) {  // uniform: frames over 1024 points replay here
      replay_init(a, &s_st);
      __syncthreads();
      replay_chunk<kScoreGroupMax>(a, n, s_count, 0, h1, s_terms, &s_st);
    }
    if (threadIdx.x == 0) need_out[f] = n > kPts && s_st.niters > h1 ? 1 : 0;
  }
}

// After the first h_end hypotheses of every frame are scored: need[f] = 1 where the serial
// loop has not stopped yet, i.e. the frames whose hypotheses [h_end, H) are solved next.
// One wave per frame.
__global__ __launch_bounds__(64) void pnp_decide_kernel(PnpArgs a, int h_end, int32_t* need) {
  __shared__ int s_cnt[64];
  __shared__ ItersTerms s_terms[64];
  __shared__ ReplayState s_st;
  const int f = blockIdx.x;
  const int n = a.off[f + 1] - a.off[f];
  if (n <= kPts) {
    if (threadIdx.x == 0) need[f] = 0;
    return;
  }
  ransac_replay<64>(a, f, n, h_end, s_cnt, s_terms, &s_st);
  if (threadIdx.x == 0) need[f] = s_st.niters > h_end ? 1 : 0;
}

// v plus the value DPP control kCtrl moves into this lane (rows outside kRowMask add +0.0).
template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ double dpp_add(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), kCtrl, kRowMask, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), kCtrl, kRowMask, 0xF, false);
  return v + __hiloint2double(hi, lo);
}

// Sum of one double over a wave in a fixed order, on DPP lane moves (no LDS traffic): quads,
// half rows, rows (every lane then holds its row's sum), rows 0 + 1 and 2 + 3 by row_bcast15,
// all four by row_bcast31 into row 3; lane 63's value broadcast.
__device__ __forceinline__ double wave_sum(double v) {
  v = dpp_add<0xB1>(v);         // quad_perm [1, 0, 3, 2]
  v = dpp_add<0x4E>(v);         // quad_perm [2, 3, 0, 1]
  v = dpp_add<0x141>(v);        // row_half_mirror
  v = dpp_add<0x140>(v);        // row_mirror
  v = dpp_add<0x142, 0xA>(v);   // row_bcast15 into rows 1 and 3
  v = dpp_add<0x143, 0xC>(v);   // row_bcast31 into rows 2 and 3
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63),
                          __builtin_amdgcn_readlane(__double2loint(v), 63));
}

// pnp_final: threads per frame.  At two waves per SIMD (<= 256 VGPRs) a CU holds 8 / kFinalWaves
// frames: with 128 threads a batch of 1024 frames is one round on 256 CUs (256 threads: two).
#ifndef VO_PNP_FINAL_THREADS
#define VO_PNP_FINAL_THREADS 128
#endif
constexpr int kFinalThreads = VO_PNP_FINAL_THREADS;
static_assert(kFinalThreads % 64 == 0 && kFinalThreads <= 256, "pnp_final: 1..4 waves");
// Small batches (the single frame of vo.py's tracking step): one frame per CU anyway, so eight
// waves share its LM passes (the normal equations' point loop is then 1 / 4 as long; the sums are
// taken in another order than at 128 threads, within the oracle's tolerance either way)
constexpr int kFinalThreadsWide = 512;
constexpr int kFinalWideBatch = 64;
constexpr int kLmStage = 1024;  // inliers pnp_final stages in LDS for its LM passes (20 KB)

// Normal equations of the inliers at (R, t): this thread's partial sums (points i = tid mod
// T).
template <int T>
__device__ __forceinline__ void lm_accumulate(const PnpArgs& a, int o, int n, const double* R, const double* t,
                                              double (&acc)[kNe]) {
#pragma unroll
  for (int k = 0; k < kNe; ++k) acc[k] = 0.0;
  for (int i = threadIdx.x; i < n; i += T) {
    if (!a.mask[o + i]) continue;
    float M[3];
    load3(a.X, o + i, M);
    const float2 q = reinterpret_cast<const float2*>(a.uv)[o + i];
    lm_point(R, t, M, q.x, q.y, a.K, acc);
  }
}

template <int T>
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
    double v = red[k];
#pragma unroll
    for (int w = 1; w < T / 64; ++w) v = v + red[w * kNe + k];
    out[k] = v;
  }
  __syncthreads();
}

template <int T>
__global__ __launch_bounds__(T, 2) void pnp_final_kernel(PnpArgs a) {  // 2 waves per SIMD
  constexpr int kFinalWaves = T / 64;
  const int f = blockIdx.x;
  const int o = a.off[f], n = a.off[f + 1] - o;
  __shared__ int s_count, s_go;
  __shared__ int s_cnt[T];
  __shared__ ItersTerms s_terms[T];
  __shared__ ReplayState s_st;
  __shared__ double s_R[9], s_t[3];
  __shared__ double s_red[kFinalWaves * kNe];
  __shared__ double s_ne[kNe];
  __shared__ float s_pt[kLmStage * 5];  // staged inliers: X, Y, Z, u, v
  __shared__ int s_wc[kFinalWaves];
  // the serial RANSAC loop over the precomputed counts (uniform branch: n is per frame)
  if (n > kPts) ransac_replay<T>(a, f, n, a.H, s_cnt, s_terms, &s_st);
  if (threadIdx.x == 0) s_count = 0;
  const int best = n > kPts ? s_st.best : n == kPts && a.models[(size_t)f * a.H * kModel + 15] != 0.0 ? 0 : -1;
  __syncthreads();
  const double* model = a.models + ((size_t)f * a.H + (best < 0 ? 0 : best)) * kModel;
  if (best < 0 || n == kPts) {
    for (int i = threadIdx.x; i < n; i += T) a.mask[o + i] = best < 0 ? 0 : 1;
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
  // The inlier mask of the best model; the inliers, in point order, staged in LDS for the LM
  // passes (a frame of more than kLmStage inliers reads them from global memory each pass).
  // Positions by ballot ranks, so the order does not depend on timing.
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int ninl = 0;  // uniform
  for (int c0 = 0; c0 < n; c0 += T) {
    const int i = c0 + (int)threadIdx.x;
    float M[3] = {0.f, 0.f, 0.f};
    float2 q = make_float2(0.f, 0.f);
    bool in = false;
    if (i < n) {
      q = reinterpret_cast<const float2*>(a.uv)[o + i];
      load3(a.X, o + i, M);
      in = is_inlier(R, t, M, q.x, q.y, a.K, a.thr2);
      a.mask[o + i] = in ? 1 : 0;
    }
    const uint64_t b = __ballot(in);
    if (lane == 0) s_wc[wave] = __popcll(b);
    __syncthreads();
    int pos = ninl + __popcll(b & ((1ull << lane) - 1)), tot = 0;
#pragma unroll
    for (int w = 0; w < kFinalWaves; ++w) {
      pos += w < wave ? s_wc[w] : 0;
      tot += s_wc[w];
    }
    if (in && pos < kLmStage) {
      float* d = &s_pt[5 * pos];
      d[0] = M[0];
      d[1] = M[1];
      d[2] = M[2];
      d[3] = q.x;
      d[4] = q.y;
    }
    ninl += tot;
    __syncthreads();  // s_wc is rewritten by the next chunk
  }
  if (threadIdx.x == 0) s_count = ninl;
  // normal equations of the inliers at (R, t), this thread's partial sums
  auto accumulate = [&](const double* Rc, const double* tc, double (&acc)[kNe]) {
    if (ninl > kLmStage) {
      lm_accumulate<T>(a, o, n, Rc, tc, acc);  // reads mask[o + i] for the i this thread wrote
      return;
    }
#pragma unroll
    for (int k = 0; k < kNe; ++k) acc[k] = 0.0;
    for (int j = threadIdx.x; j < ninl; j += T) {
      const float* d = &s_pt[5 * j];
      const float M[3] = {d[0], d[1], d[2]};
      lm_point(Rc, tc, M, d[3], d[4], a.K, acc);
    }
  };
  // Levenberg-Marquardt on the inliers: thread 0 holds the state (pnp_math.h LmState),
  // every pass evaluates the normal equations at the pose in s_R/s_t.
  double acc[kNe];
  accumulate(R, t, acc);
  lm_reduce<T>(acc, s_red, s_ne);
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
    accumulate(nR, nt, acc);
    lm_reduce<T>(acc, s_red, s_ne);  // ends with a barrier: every thread has read s_R/s_t
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
  // The serial loop stops after niters <= H hypotheses (niters shrinks as better models turn
  // up: about 17 at 25 % outliers and confidence 0.99), and one pnp_hyp thread is a long
  // dependent chain (one wave per SIMD, 512 VGPRs): a launch of more waves than SIMDs takes
  // twice as long.  So large batches solve the first h1 hypotheses of every frame (h1 sized
  // to one wave per SIMD), replay the loop over them (inside the scoring launch when one
  // workgroup scores a frame, which then also stops scoring where the loop stops; else
  // pnp_decide), and solve and score
  // hypotheses [h1, H) only for the frames whose loop has not stopped by h1.  pnp_final's
  // replay reads no count past where the loop stops, so the result is the same as solving all
  // H.  ctx->pnp_split (vo_pnp_testing_split): > 0 forces h1, -1 solves all H at once.
  const long fill = 4l * ctx->num_cus * 64;
  int h1 = H;
  if (ctx->pnp_split > 0)
    h1 = std::min(H, ctx->pnp_split);
  else if (ctx->pnp_split == 0 && (long)batch * H > fill)
    h1 = std::min(H, std::max(kSplitMin, (int)(fill / batch)));
  ws.last_h1 = h1;
  int32_t* need = nullptr;
  if (h1 < H) {
    ws.need.reserve((size_t)batch * sizeof(int32_t));
    need = ws.need.as<int32_t>();
  }
  bool decided = false;  // need written by the phase-1 scoring launch
  auto solve_and_score = [&](int h_lo, int h_hi, const int32_t* need_in, int kid_hyp, int kid_score) {
    const int hr = h_hi - h_lo, nh = batch * hr;
    ctx->prof.begin(ctx->stream, kid_hyp);
    // lane groups while they fit one wave per SIMD (small batches: the single frame of vo.py's
    // tracking step, 100 hypotheses); one lane per hypothesis beyond (the same bits either way)
    if (ctx->pnp_group > 0 || (ctx->pnp_group == 0 && (long)nh * kPnpGroupLanes <= fill))
      pnp_hyp_group_launch(a, h_lo, h_hi, need_in, nh, ctx->stream);
    else
      hipLaunchKernelGGL(pnp_hyp_kernel, dim3(ceil_div(nh, 64)), dim3(64), 0, ctx->stream, a, h_lo, h_hi, need_in);
    ctx->prof.end(ctx->stream);
    VO_HIP_CHECK(hipGetLastError());
    ctx->prof.begin(ctx->stream, kid_score);
    // hypotheses per scoring workgroup: one for small batches (single-frame latency), up to
    // kScoreGroupMax while the grid keeps ~4 workgroups per CU
    const int group = std::max(1, std::min({hr, kScoreGroupMax, nh / std::max(1, 4 * ctx->num_cus)}));
    const int ngroups = ceil_div(hr, group);
    int32_t* need_out = need && !need_in && ngroups == 1 && h_lo == 0 ? need : nullptr;
    decided |= need_out != nullptr;
    hipLaunchKernelGGL(pnp_score_kernel, dim3(batch * ngroups), dim3(kScoreThreads), 0, ctx->stream, a, group, h_lo, h_hi,
                       need_in, need_out);
    ctx->prof.end(ctx->stream);
    VO_HIP_CHECK(hipGetLastError());
  };
  solve_and_score(0, h1, nullptr, kKPnpHyp, kKPnpScore);
  if (h1 < H) {
    if (!decided) {  // phase 1 scored a frame in more than one workgroup
      ctx->prof.begin(ctx->stream, kKPnpDecide);
      hipLaunchKernelGGL(pnp_decide_kernel, dim3(batch), dim3(64), 0, ctx->stream, a, h1, need);
      ctx->prof.end(ctx->stream);
      VO_HIP_CHECK(hipGetLastError());
    }
    solve_and_score(h1, H, need, kKPnpHypTail, kKPnpScoreTail);
  }
  ctx->prof.begin(ctx->stream, kKPnpFinal);
  if (batch <= kFinalWideBatch)
    hipLaunchKernelGGL(pnp_final_kernel<kFinalThreadsWide>, dim3(batch), dim3(kFinalThreadsWide), 0, ctx->stream, a);
  else
    hipLaunchKernelGGL(pnp_final_kernel<kFinalThreads>, dim3(batch), dim3(kFinalThreads), 0, ctx->stream, a);
  ctx->prof.end(ctx->stream);
  VO_HIP_CHECK(hipGetLastError());
}

}  // namespace vo
