// Sliding-window bundle adjustment: one Gauss-Newton iteration on gfx950.
//
// The reference has no BA; the problem is build-defined and
// restated on the CPU in oracle/ba_ref.py (projection model of reference
// src/modules/frontend.py:128-140, T_cw convention of src/modules/vo.py:260-261).
//
// One GN iteration = three launches on the context stream:
//   K1 ba_lin_kernel    one workgroup per landmark segment.  Per chunk of
//                       whole landmarks (LDS-staged): [back-substitute the
//                       previous step's point update and apply it] ->
//                       reprojection residuals + 2x6 / 2x3 Jacobians (one lane
//                       per observation) -> per track entry W = Jc^T Jp and
//                       gc = Jc^T r, per landmark V = Jp^T Jp (+lambda), its
//                       3x3 Cholesky L and h = L^-1 g -> Z = W L^-T,
//                       bt = -gc + Z h -> Schur blocks U - Z_x Z_y^T
//                       accumulated into the segment's LDS window, each
//                       (slot, row) owned by one lane and summed over a static
//                       pair list in fixed order (deterministic, no atomics).
//                       The window is written once to the segment's slab.
//   K2 ba_reduce_kernel sums slab blocks into the profile-stored reduced camera
//                       matrix S, the rhs b and the cost in fixed segment order.
//   K3 ba_solve_kernel  one workgroup: right-looking 6x6-block Cholesky of the
//                       profile (LDS resident when it fits) with the forward
//                       substitution folded in, back substitution, and the
//                       left se(3) pose update T <- exp(dc^) T.
// The point update dp = L^-T(-h - sum Z^T dc) is applied by the next K1 (or a
// back-substitute-only K1), which recomputes the same linearisation bit for bit.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "ba_plan.h"
#include "vo_ctx.h"

namespace vo {

struct Comm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  ~Comm() {
    if (comm) ncclCommDestroy(comm);
  }
};

#define VO_NCCL_CHECK(expr)                                                          \
  do {                                                                               \
    ncclResult_t r_ = (expr);                                                        \
    if (r_ != ncclSuccess) {                                                         \
      ::vo::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,             \
                      ncclGetErrorString(r_));                                       \
      throw ::vo::Error{VO_ERR_RCCL};                                                \
    }                                                                                \
  } while (0)

namespace {

constexpr int kLinThreads = 128;
constexpr int kSolveThreads = 256;
constexpr double kPivotRelEps = 1e-12;  // == oracle/ba_ref.py PIVOT_REL_EPS
constexpr double kExpTaylor = 1e-4;     // == oracle/ba_ref.py EXP_TAYLOR_THETA
enum { kBacksub = 1, kAccum = 2 };

struct LinArgs {
  int n_fixed;
  double fx, fy, cx, cy, lambda;
  const float2* obs_uv;
  const int* obs_cam;
  const int* obs_te;
  const int* te_cam;
  const int* te_pt;
  const int* te_obs;
  const int16_t* te_lcam;
  const int* pt_te;
  const int* chunk_obs;
  const int* chunk_te;
  const int* chunk_pt;
  const int* chunk_slot_base;
  const int* chunk_cam_base;
  const int* slot_ptr;
  const uint16_t* pair_list;
  const int* cam_ptr;
  const uint8_t* cam_list;
  const int* seg_chunk;
  const int* seg_slot_off;
  const int* seg_cam_off;
  double* points;
  double* slab;
  double* slab_b;
  double* slab_cost;
  const double* pose_old;  // linearisation of the pending step (back-substitution)
  const double* pose_new;  // current linearisation point
  const double* dc;        // pending pose update (6 per free camera)
  const int* status;
};

struct LinShared {
  double win[kSegSlots * 36];
  double bwin[kSegCams * 6];
  double Jc[kChunkObs][12];
  double Jp[kChunkObs][6];
  double r[kChunkObs][2];
  double Z[kChunkTe][18];  // W, then Z = W L^-T
  double bt[kChunkTe][6];  // gc, then bt = -gc + Z h
  double X[kChunkPts][3];
  double L[kChunkPts][6];  // 1/l00, l10, 1/l11, l20, l21, 1/l22
  double h[kChunkPts][3];
  double red[kLinThreads];
  int obs_te[kChunkObs];
  int te_obs[kChunkTe + 1];
  int te_pt[kChunkTe];
  int te_cam[kChunkTe];
  int te_use[kChunkTe];  // free camera and valid landmark
  int te_lcam[kChunkTe];
  int pt_te[kChunkPts + 1];
  int valid[kChunkPts];
};

// R1: residual and Jacobians, one lane per observation.
__device__ __forceinline__ void lin_obs(LinShared& S, const LinArgs& A, const double* pose,
                                        int ob0, int nob, double& cost) {
  for (int o = threadIdx.x; o < nob; o += kLinThreads) {
    const int cam = A.obs_cam[ob0 + o];
    const double* T = pose + 12 * cam;
    const int q = S.te_pt[S.obs_te[o]];
    const double X0 = S.X[q][0], X1 = S.X[q][1], X2 = S.X[q][2];
    const double x = T[0] * X0 + T[1] * X1 + T[2] * X2 + T[9];
    const double y = T[3] * X0 + T[4] * X1 + T[5] * X2 + T[10];
    const double z = T[6] * X0 + T[7] * X1 + T[8] * X2 + T[11];
    const double iz = 1.0 / z;
    const float2 m = A.obs_uv[ob0 + o];
    const double r0 = A.fx * x * iz + A.cx - (double)m.x;
    const double r1 = A.fy * y * iz + A.cy - (double)m.y;
    cost += r0 * r0 + r1 * r1;
    S.r[o][0] = r0;
    S.r[o][1] = r1;
    const double j00 = A.fx * iz, j02 = -A.fx * x * iz * iz;
    const double j11 = A.fy * iz, j12 = -A.fy * y * iz * iz;
    double* jc = S.Jc[o];
    jc[0] = j00;
    jc[1] = 0.0;
    jc[2] = j02;
    jc[3] = j02 * y;
    jc[4] = j00 * z - j02 * x;
    jc[5] = -j00 * y;
    jc[6] = 0.0;
    jc[7] = j11;
    jc[8] = j12;
    jc[9] = j12 * y - j11 * z;
    jc[10] = -j12 * x;
    jc[11] = j11 * x;
    double* jp = S.Jp[o];
    jp[0] = j00 * T[0] + j02 * T[6];
    jp[1] = j00 * T[1] + j02 * T[7];
    jp[2] = j00 * T[2] + j02 * T[8];
    jp[3] = j11 * T[3] + j12 * T[6];
    jp[4] = j11 * T[4] + j12 * T[7];
    jp[5] = j11 * T[5] + j12 * T[8];
  }
}

// R2: per track entry W, gc; per landmark V (+lambda), pivot-tested Cholesky, h.
__device__ __forceinline__ void lin_reduce(LinShared& S, const LinArgs& A, int nte, int npt) {
  for (int t = threadIdx.x; t < nte; t += kLinThreads) {
    double W[18], g[6];
#pragma unroll
    for (int e = 0; e < 18; ++e) W[e] = 0.0;
#pragma unroll
    for (int e = 0; e < 6; ++e) g[e] = 0.0;
    for (int o = S.te_obs[t]; o < S.te_obs[t + 1]; ++o) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const double rk = S.r[o][k];
        const double p0 = S.Jp[o][3 * k], p1 = S.Jp[o][3 * k + 1], p2 = S.Jp[o][3 * k + 2];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
          const double jc = S.Jc[o][6 * k + a];
          W[3 * a] += jc * p0;
          W[3 * a + 1] += jc * p1;
          W[3 * a + 2] += jc * p2;
          g[a] += jc * rk;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 18; ++e) S.Z[t][e] = W[e];
#pragma unroll
    for (int e = 0; e < 6; ++e) S.bt[t][e] = g[e];
  }
  for (int p = threadIdx.x; p < npt; p += kLinThreads) {
    double v00 = 0, v01 = 0, v02 = 0, v11 = 0, v12 = 0, v22 = 0, g0 = 0, g1 = 0, g2 = 0;
    const int o0 = S.te_obs[S.pt_te[p]], o1 = S.te_obs[S.pt_te[p + 1]];
    for (int o = o0; o < o1; ++o) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const double a = S.Jp[o][3 * k], b = S.Jp[o][3 * k + 1], c = S.Jp[o][3 * k + 2];
        const double rk = S.r[o][k];
        v00 += a * a; v01 += a * b; v02 += a * c;
        v11 += b * b; v12 += b * c; v22 += c * c;
        g0 += a * rk; g1 += b * rk; g2 += c * rk;
      }
    }
    v00 += A.lambda; v11 += A.lambda; v22 += A.lambda;
    // pivot test: same sequence as oracle/ba_ref.py point_block_valid
    const double eps = kPivotRelEps * (v00 + v11 + v22);
    bool ok = v00 > eps;
    const double l00 = sqrt(ok ? v00 : 1.0);
    const double l10 = v01 / l00, l20 = v02 / l00;
    const double d1 = v11 - l10 * l10;
    ok = ok && d1 > eps;
    const double l11 = sqrt(ok ? d1 : 1.0);
    const double l21 = (v12 - l20 * l10) / l11;
    const double d2 = v22 - l20 * l20 - l21 * l21;
    ok = ok && d2 > eps;
    const double l22 = sqrt(ok ? d2 : 1.0);
    const double i00 = 1.0 / l00, i11 = 1.0 / l11, i22 = 1.0 / l22;
    S.valid[p] = ok;
    S.L[p][0] = i00; S.L[p][1] = l10; S.L[p][2] = i11;
    S.L[p][3] = l20; S.L[p][4] = l21; S.L[p][5] = i22;
    const double h0 = g0 * i00;
    const double h1 = (g1 - l10 * h0) * i11;
    const double h2 = (g2 - l20 * h0 - l21 * h1) * i22;
    S.h[p][0] = ok ? h0 : 0.0;
    S.h[p][1] = ok ? h1 : 0.0;
    S.h[p][2] = ok ? h2 : 0.0;
  }
}

// R3: Z = W L^-T and bt = -gc + Z h for track entries of valid landmarks in free
// cameras; zero otherwise (frozen landmarks leave the camera system).
__device__ __forceinline__ void lin_eliminate(LinShared& S, int nte) {
  for (int t = threadIdx.x; t < nte; t += kLinThreads) {
    const int p = S.te_pt[t];
    const bool use = S.valid[p] && S.te_lcam[t] >= 0;
    S.te_use[t] = use;
    if (!use) {
#pragma unroll
      for (int e = 0; e < 18; ++e) S.Z[t][e] = 0.0;
#pragma unroll
      for (int e = 0; e < 6; ++e) S.bt[t][e] = 0.0;
      continue;
    }
    const double i00 = S.L[p][0], l10 = S.L[p][1], i11 = S.L[p][2];
    const double l20 = S.L[p][3], l21 = S.L[p][4], i22 = S.L[p][5];
    const double h0 = S.h[p][0], h1 = S.h[p][1], h2 = S.h[p][2];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const double z0 = S.Z[t][3 * a] * i00;
      const double z1 = (S.Z[t][3 * a + 1] - l10 * z0) * i11;
      const double z2 = (S.Z[t][3 * a + 2] - l20 * z0 - l21 * z1) * i22;
      S.Z[t][3 * a] = z0;
      S.Z[t][3 * a + 1] = z1;
      S.Z[t][3 * a + 2] = z2;
      S.bt[t][a] = -S.bt[t][a] + (z0 * h0 + z1 * h1 + z2 * h2);
    }
  }
}

__device__ __forceinline__ void chunk_linearize(LinShared& S, const LinArgs& A,
                                                const double* pose, int ob0, int nob,
                                                int nte, int npt, double& cost) {
  lin_obs(S, A, pose, ob0, nob, cost);
  __syncthreads();
  lin_reduce(S, A, nte, npt);
  __syncthreads();
  lin_eliminate(S, nte);
  __syncthreads();
}

template <int MODE>
__global__ __launch_bounds__(kLinThreads) void ba_lin_kernel(LinArgs A) {
  if (A.status && *A.status) return;  // a previous solve failed: state frozen
  __shared__ LinShared S;
  const int seg = blockIdx.x, tid = threadIdx.x;
  const int nslots = A.seg_slot_off[seg + 1] - A.seg_slot_off[seg];
  const int ncams = A.seg_cam_off[seg + 1] - A.seg_cam_off[seg];
  if (MODE & kAccum) {
    for (int e = tid; e < nslots * 36; e += kLinThreads) S.win[e] = 0.0;
    for (int e = tid; e < ncams * 6; e += kLinThreads) S.bwin[e] = 0.0;
  }
  double cost = 0.0;
  for (int ch = A.seg_chunk[seg]; ch < A.seg_chunk[seg + 1]; ++ch) {
    const int ob0 = A.chunk_obs[ch], nob = A.chunk_obs[ch + 1] - ob0;
    const int te0 = A.chunk_te[ch], nte = A.chunk_te[ch + 1] - te0;
    const int p0 = A.chunk_pt[ch], npt = A.chunk_pt[ch + 1] - p0;
    __syncthreads();  // previous chunk fully consumed
    for (int o = tid; o < nob; o += kLinThreads) S.obs_te[o] = A.obs_te[ob0 + o] - te0;
    for (int t = tid; t <= nte; t += kLinThreads) S.te_obs[t] = A.te_obs[te0 + t] - ob0;
    for (int t = tid; t < nte; t += kLinThreads) {
      S.te_pt[t] = A.te_pt[te0 + t] - p0;
      S.te_cam[t] = A.te_cam[te0 + t];
      S.te_lcam[t] = A.te_lcam[te0 + t];
    }
    for (int p = tid; p <= npt; p += kLinThreads) S.pt_te[p] = A.pt_te[p0 + p] - te0;
    for (int e = tid; e < npt * 3; e += kLinThreads) S.X[e / 3][e % 3] = A.points[3l * p0 + e];
    __syncthreads();

    if (MODE & kBacksub) {
      double dummy = 0.0;
      chunk_linearize(S, A, A.pose_old, ob0, nob, nte, npt, dummy);
      for (int p = tid; p < npt; p += kLinThreads) {
        if (!S.valid[p]) continue;
        double a0 = -S.h[p][0], a1 = -S.h[p][1], a2 = -S.h[p][2];
        for (int t = S.pt_te[p]; t < S.pt_te[p + 1]; ++t) {
          if (!S.te_use[t]) continue;
          const double* d = A.dc + 6 * (S.te_cam[t] - A.n_fixed);
#pragma unroll
          for (int a = 0; a < 6; ++a) {
            a0 -= S.Z[t][3 * a] * d[a];
            a1 -= S.Z[t][3 * a + 1] * d[a];
            a2 -= S.Z[t][3 * a + 2] * d[a];
          }
        }
        const double i00 = S.L[p][0], l10 = S.L[p][1], i11 = S.L[p][2];
        const double l20 = S.L[p][3], l21 = S.L[p][4], i22 = S.L[p][5];
        const double x2 = a2 * i22;
        const double x1 = (a1 - l21 * x2) * i11;
        const double x0 = (a0 - l10 * x1 - l20 * x2) * i00;
        S.X[p][0] += x0;
        S.X[p][1] += x1;
        S.X[p][2] += x2;
        A.points[3l * (p0 + p)] = S.X[p][0];
        A.points[3l * (p0 + p) + 1] = S.X[p][1];
        A.points[3l * (p0 + p) + 2] = S.X[p][2];
      }
      __syncthreads();
    }

    if (!(MODE & kAccum)) {
      lin_obs(S, A, A.pose_new, ob0, nob, cost);  // cost at the updated state
      continue;
    }
    chunk_linearize(S, A, A.pose_new, ob0, nob, nte, npt, cost);

    // R4: Schur blocks into the window; lane owns (slot, row a) and sums its
    // slot's pair list of this chunk in fixed order.
    const int sb = A.chunk_slot_base[ch];
    for (int item = tid; item < nslots * 6; item += kLinThreads) {
      const int s = item / 6, a = item - 6 * (item / 6);
      const int e0 = A.slot_ptr[sb + s], e1 = A.slot_ptr[sb + s + 1];
      if (e0 == e1) continue;
      double out[6] = {0, 0, 0, 0, 0, 0};
      for (int e = e0; e < e1; ++e) {
        const int pr = A.pair_list[e];
        const int x = pr & 255, y = pr >> 8;
        const double za0 = S.Z[x][3 * a], za1 = S.Z[x][3 * a + 1], za2 = S.Z[x][3 * a + 2];
#pragma unroll
        for (int c = 0; c < 6; ++c)
          out[c] -= za0 * S.Z[y][3 * c] + za1 * S.Z[y][3 * c + 1] + za2 * S.Z[y][3 * c + 2];
        if (x == y && S.te_use[x]) {
          for (int o = S.te_obs[x]; o < S.te_obs[x + 1]; ++o) {
            const double ja0 = S.Jc[o][a], ja1 = S.Jc[o][6 + a];
#pragma unroll
            for (int c = 0; c < 6; ++c) out[c] += ja0 * S.Jc[o][c] + ja1 * S.Jc[o][6 + c];
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) S.win[36 * s + 6 * a + c] += out[c];
    }
    const int cb = A.chunk_cam_base[ch];
    for (int item = tid; item < ncams * 6; item += kLinThreads) {
      const int c = item / 6, a = item - 6 * (item / 6);
      double acc = 0.0;
      for (int e = A.cam_ptr[cb + c]; e < A.cam_ptr[cb + c + 1]; ++e) acc += S.bt[A.cam_list[e]][a];
      S.bwin[6 * c + a] += acc;
    }
  }
  __syncthreads();
  if (MODE & kAccum) {
    double* dst = A.slab + 36l * A.seg_slot_off[seg];
    for (int e = tid; e < nslots * 36; e += kLinThreads) dst[e] = S.win[e];
    double* dstb = A.slab_b + 6l * A.seg_cam_off[seg];
    for (int e = tid; e < ncams * 6; e += kLinThreads) dstb[e] = S.bwin[e];
  }
  S.red[tid] = cost;
  __syncthreads();
  for (int w = kLinThreads / 2; w > 0; w >>= 1) {
    if (tid < w) S.red[tid] += S.red[tid + w];
    __syncthreads();
  }
  if (tid == 0) A.slab_cost[seg] = S.red[0];
}

// K2: fixed-order reduction of the slabs into [S profile | b | cost].
struct ReduceArgs {
  int nprof, F, nseg;
  double lambda;
  const int* prof_src_ptr;
  const int* prof_src;
  const uint8_t* prof_diag;
  const int* camb_ptr;
  const int* camb_src;
  const double* slab;
  const double* slab_b;
  const double* slab_cost;
  double* sys;  // nprof*36 + 6F + 1
  const int* status;
};

__global__ __launch_bounds__(64) void ba_reduce_kernel(ReduceArgs A) {
  if (A.status && *A.status) return;
  const int blk = blockIdx.x, tid = threadIdx.x;
  if (blk < A.nprof) {
    if (tid < 36) {
      double acc = 0.0;
      for (int k = A.prof_src_ptr[blk]; k < A.prof_src_ptr[blk + 1]; ++k)
        acc += A.slab[36l * A.prof_src[k] + tid];
      if (A.prof_diag[blk] && tid % 7 == 0) acc += A.lambda;
      A.sys[36l * blk + tid] = acc;
    }
    return;
  }
  double* b = A.sys + 36l * A.nprof;
  for (int v = tid; v < 6 * A.F; v += 64) {
    const int f = v / 6, a = v - 6 * (v / 6);
    double acc = 0.0;
    for (int k = A.camb_ptr[f]; k < A.camb_ptr[f + 1]; ++k) acc += A.slab_b[6l * A.camb_src[k] + a];
    b[v] = acc;
  }
  if (tid == 0) {
    double c = 0.0;
    for (int s = 0; s < A.nseg; ++s) c += A.slab_cost[s];
    b[6 * A.F] = c;
  }
}

// K3: profile Cholesky solve S dc = b + pose update.
struct SolveArgs {
  int F, nprof, n_poses, n_fixed, iter_tag;
  const int* prof_first;
  const int* prof_off;
  const int* prof_last;
  double* sys;         // [S profile | b | cost]; factorised in place on the global path
  double* linv_glob;   // F*36 scratch (global path)
  double* dc;          // 6F out
  const double* pose_cur;
  double* pose_next;
  int* status;
};

__device__ __forceinline__ void se3_exp_apply(const double* d, const double* T, double* out) {
  const double r0 = d[0], r1 = d[1], r2 = d[2], p0 = d[3], p1 = d[4], p2 = d[5];
  const double th2 = p0 * p0 + p1 * p1 + p2 * p2;
  const double th = sqrt(th2);
  double A, B, C;
  if (th < kExpTaylor) {
    A = 1.0 - th2 / 6.0;
    B = 0.5 - th2 / 24.0;
    C = 1.0 / 6.0 - th2 / 120.0;
  } else {
    const double s = sin(th), c = cos(th);
    A = s / th;
    B = (1.0 - c) / (th * th);
    C = (th - s) / (th * th * th);
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

template <bool kLds>
__global__ __launch_bounds__(kSolveThreads) void ba_solve_kernel(SolveArgs A) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  __shared__ int s_fail;
  const int tid = threadIdx.x, F = A.F;
  const bool prior_fail = A.status && *A.status;
  double* Sm;
  double* Linv;
  double* y;
  if (kLds) {
    Sm = dyn;
    Linv = dyn + 36l * A.nprof;
    y = Linv + 36l * F;
  } else {
    Sm = A.sys;
    Linv = A.linv_glob;
    y = dyn;
  }
  int* first = reinterpret_cast<int*>(y + 6 * F);
  int* off = first + F;
  int* last = off + F + 1;
  if (tid == 0) s_fail = prior_fail ? 1 : 0;
  if (!prior_fail) {
    if (kLds)
      for (int e = tid; e < 36 * A.nprof; e += kSolveThreads) Sm[e] = A.sys[e];
    for (int e = tid; e < 6 * F; e += kSolveThreads) y[e] = A.sys[36l * A.nprof + e];
    for (int i = tid; i < F; i += kSolveThreads) {
      first[i] = A.prof_first[i];
      last[i] = A.prof_last[i];
    }
    for (int i = tid; i <= F; i += kSolveThreads) off[i] = A.prof_off[i];
  }
  __syncthreads();

  for (int k = 0; k < F && !s_fail; ++k) {
    // (A) factor the diagonal block, invert it, forward-substitute y_k
    if (tid == 0) {
      double* D = Sm + 36l * (off[k] + k - first[k]);
      double Lk[36], Li[36];
      bool ok = true;
#pragma unroll
      for (int e = 0; e < 36; ++e) Lk[e] = Li[e] = 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        double d = D[6 * j + j];
#pragma unroll
        for (int m = 0; m < j; ++m) d -= Lk[6 * j + m] * Lk[6 * j + m];
        ok = ok && d > 0.0;
        const double ljj = sqrt(d > 0.0 ? d : 1.0);
        const double inv = 1.0 / ljj;
        Lk[6 * j + j] = ljj;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
          double s = D[6 * i + j];
#pragma unroll
          for (int m = 0; m < j; ++m) s -= Lk[6 * i + m] * Lk[6 * j + m];
          Lk[6 * i + j] = s * inv;
        }
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        Li[6 * i + i] = 1.0 / Lk[6 * i + i];
#pragma unroll
        for (int j = 0; j < i; ++j) {
          double s = 0.0;
#pragma unroll
          for (int m = j; m < i; ++m) s += Lk[6 * i + m] * Li[6 * m + j];
          Li[6 * i + j] = -s * Li[6 * i + i];
        }
      }
      double yk[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        double s = 0.0;
#pragma unroll
        for (int m = 0; m <= i; ++m) s += Li[6 * i + m] * y[6 * k + m];
        yk[i] = s;
      }
#pragma unroll
      for (int e = 0; e < 36; ++e) {
        D[e] = Lk[e];
        Linv[36l * k + e] = Li[e];
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) y[6 * k + i] = yk[i];
      if (!ok || !isfinite(yk[0] + yk[1] + yk[2] + yk[3] + yk[4] + yk[5])) s_fail = 1;
    }
    __syncthreads();
    if (s_fail) break;
    const int lk = last[k];
    // (B) panel: L_ik = S_ik Linv_kk^T for rows i in (k, last] whose envelope holds k
    const double* Li = Linv + 36l * k;
    for (int item = tid; item < (lk - k) * 6; item += kSolveThreads) {
      const int i = k + 1 + item / 6, r = item % 6;
      if (first[i] > k) continue;
      double* row = Sm + 36l * (off[i] + k - first[i]) + 6 * r;
      double s[6];
#pragma unroll
      for (int m = 0; m < 6; ++m) s[m] = row[m];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m <= c; ++m) acc += s[m] * Li[6 * c + m];
        row[c] = acc;
      }
    }
    __syncthreads();
    // (C) trailing update S_ij -= L_ik L_jk^T (k < j <= i <= last) and y_i -= L_ik y_k
    const int n = lk - k;
    const int ntri = n * (n + 1) / 2;
    for (int item = tid; item < ntri * 6 + n * 6; item += kSolveThreads) {
      if (item < ntri * 6) {
        const int t = item / 6, r = item % 6;
        int di = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
        while ((di + 1) * (di + 2) / 2 <= t) ++di;
        while (di * (di + 1) / 2 > t) --di;
        const int dj = t - di * (di + 1) / 2;
        const int i = k + 1 + di, j = k + 1 + dj;
        if (first[i] > k || first[j] > k) continue;
        const double* Lik = Sm + 36l * (off[i] + k - first[i]) + 6 * r;
        const double* Ljk = Sm + 36l * (off[j] + k - first[j]);
        double* Sij = Sm + 36l * (off[i] + j - first[i]) + 6 * r;
        double li[6];
#pragma unroll
        for (int m = 0; m < 6; ++m) li[m] = Lik[m];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          double acc = 0.0;
#pragma unroll
          for (int m = 0; m < 6; ++m) acc += li[m] * Ljk[6 * c + m];
          Sij[c] -= acc;
        }
      } else {
        const int v = item - ntri * 6;
        const int i = k + 1 + v / 6, r = v % 6;
        if (first[i] > k) continue;
        const double* Lik = Sm + 36l * (off[i] + k - first[i]) + 6 * r;
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < 6; ++m) acc += Lik[m] * y[6 * k + m];
        y[6 * i + r] -= acc;
      }
    }
    __syncthreads();
  }
  // backward substitution L^T x = y (row oriented: x_k, then y_j -= L_kj^T x_k)
  if (!s_fail) {
    for (int k = F - 1; k >= 0; --k) {
      if (tid == 0) {
        const double* Li = Linv + 36l * k;
        double x[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          double acc = 0.0;
#pragma unroll
          for (int m = c; m < 6; ++m) acc += Li[6 * m + c] * y[6 * k + m];
          x[c] = acc;
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) y[6 * k + c] = x[c];
      }
      __syncthreads();
      const int nb = k - first[k];
      for (int item = tid; item < nb * 6; item += kSolveThreads) {
        const int j = first[k] + item / 6, c = item % 6;
        const double* Lkj = Sm + 36l * (off[k] + j - first[k]);
        double acc = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r) acc += Lkj[6 * r + c] * y[6 * k + r];
        y[6 * j + c] -= acc;
      }
      __syncthreads();
    }
  }
  const bool failed = s_fail != 0;
  for (int e = tid; e < 6 * F; e += kSolveThreads) A.dc[e] = failed ? 0.0 : y[e];
  for (int c = tid; c < A.n_poses; c += kSolveThreads) {
    const double* T = A.pose_cur + 12 * c;
    double* out = A.pose_next + 12 * c;
    if (failed || c < A.n_fixed) {
      for (int e = 0; e < 12; ++e) out[e] = T[e];
    } else {
      se3_exp_apply(A.dc + 6 * (c - A.n_fixed), T, out);
    }
  }
  if (tid == 0 && failed && !prior_fail) *A.status = A.iter_tag;
}

template <class T>
void upload(DevBuf& buf, const std::vector<T>& v, hipStream_t st) {
  buf.reserve(std::max<size_t>(v.size(), 1) * sizeof(T));
  if (!v.empty())
    VO_HIP_CHECK(hipMemcpyAsync(buf.ptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st));
}

size_t solve_lds_bytes(int nprof, int F) {
  return (36ull * nprof + 36ull * F + 6ull * F) * 8 + (3ull * F + 1) * 4;
}
constexpr size_t kSolveLdsMax = 150 * 1024;

}  // namespace

class BAEngine {
 public:
  explicit BAEngine(vo_ctx* ctx) : ctx_(ctx) {}

  void setup(const vo_ba_problem* prob) {
    VO_REQUIRE(prob, VO_ERR_ARG, "vo_ba_setup: null problem");
    VO_REQUIRE(prob->n_poses >= 1 && prob->n_points >= 0 && prob->n_obs >= 0, VO_ERR_ARG,
               "vo_ba_setup: bad sizes");
    VO_REQUIRE(prob->lambda >= 0.0, VO_ERR_ARG, "vo_ba_setup: lambda must be >= 0");
    VO_REQUIRE((prob->n_points == 0 || prob->point_ptr) && (prob->n_obs == 0 || (prob->obs_cam && prob->obs_uv)),
               VO_ERR_ARG, "vo_ba_setup: null arrays");
    const int target = segments_target();
    std::vector<int32_t> zero_ptr(1, 0);
    const int32_t* pp = prob->n_points ? prob->point_ptr : zero_ptr.data();
    if (prob->n_points == 0)
      VO_REQUIRE(prob->n_obs == 0, VO_ERR_ARG, "vo_ba_setup: observations without points");
    std::string err = build_plan(plan_, prob->n_poses, prob->n_points, prob->n_obs,
                                 prob->n_fixed, pp, prob->obs_cam, prob->obs_uv, target);
    VO_REQUIRE(err.empty(), VO_ERR_ARG, "vo_ba_setup: %s", err.c_str());
    std::vector<int32_t> first = local_profile_first(plan_);
    if (ctx_->comm && ctx_->comm->nranks > 1 && !first.empty()) {
      DevBuf tmp;
      upload(tmp, first, ctx_->stream);
      VO_NCCL_CHECK(ncclAllReduce(tmp.ptr, tmp.ptr, first.size(), ncclInt32, ncclMin,
                                  ctx_->comm->comm, ctx_->stream));
      VO_HIP_CHECK(hipMemcpyAsync(first.data(), tmp.ptr, first.size() * 4, hipMemcpyDeviceToHost,
                                  ctx_->stream));
      VO_HIP_CHECK(hipStreamSynchronize(ctx_->stream));
    }
    build_profile(plan_, first);
    prob_ = *prob;
    prob_.point_ptr = nullptr;
    prob_.obs_cam = nullptr;
    prob_.obs_uv = nullptr;

    hipStream_t st = ctx_->stream;
    const BAPlan& P = plan_;
    upload(d_obs_uv_, P.obs_uv, st);
    upload(d_obs_cam_, P.obs_cam, st);
    upload(d_obs_te_, P.obs_te, st);
    upload(d_te_cam_, P.te_cam, st);
    upload(d_te_pt_, P.te_pt, st);
    upload(d_te_obs_, P.te_obs, st);
    upload(d_te_lcam_, P.te_lcam, st);
    upload(d_pt_te_, P.pt_te, st);
    upload(d_chunk_obs_, P.chunk_obs, st);
    upload(d_chunk_te_, P.chunk_te, st);
    upload(d_chunk_pt_, P.chunk_pt, st);
    upload(d_chunk_slot_base_, P.chunk_slot_base, st);
    upload(d_chunk_cam_base_, P.chunk_cam_base, st);
    upload(d_slot_ptr_, P.slot_ptr, st);
    upload(d_pair_list_, P.pair_list, st);
    upload(d_cam_ptr_, P.cam_ptr, st);
    upload(d_cam_list_, P.cam_list, st);
    upload(d_seg_chunk_, P.seg_chunk, st);
    upload(d_seg_slot_off_, P.seg_slot_off, st);
    upload(d_seg_cam_off_, P.seg_cam_off, st);
    upload(d_prof_first_, P.prof_first, st);
    upload(d_prof_off_, P.prof_off, st);
    upload(d_prof_last_, P.prof_last, st);
    upload(d_prof_src_ptr_, P.prof_src_ptr, st);
    upload(d_prof_src_, P.prof_src, st);
    upload(d_prof_diag_, P.prof_diag, st);
    upload(d_camb_ptr_, P.camb_ptr, st);
    upload(d_camb_src_, P.camb_src, st);
    const int F = P.n_free;
    d_points_.reserve(std::max(1, P.n_points) * 24ull);
    d_pose_[0].reserve(P.n_poses * 96ull);
    d_pose_[1].reserve(P.n_poses * 96ull);
    d_dc_.reserve(std::max(1, F) * 48ull);
    d_slab_.reserve(std::max(1, P.n_slab_slots()) * 288ull);
    d_slab_b_.reserve(std::max<size_t>(1, P.segcam_f.size()) * 48ull);
    d_slab_cost_.reserve(std::max(1, P.n_segments()) * 8ull);
    sys_len_ = 36ull * P.n_prof_blocks() + 6ull * F + 1;
    d_sys_.reserve(sys_len_ * 8);
    d_linv_.reserve(std::max(1, F) * 288ull);
    d_status_.reserve(sizeof(int));
    VO_HIP_CHECK(hipMemsetAsync(d_status_.ptr, 0, sizeof(int), st));
    solve_lds_ = solve_lds_bytes(P.n_prof_blocks(), F) <= kSolveLdsMax;
    const size_t lds = solve_lds_ ? solve_lds_bytes(P.n_prof_blocks(), F)
                                  : (6ull * F) * 8 + (3ull * F + 1) * 4;
    VO_REQUIRE(lds <= 160 * 1024, VO_ERR_ARG,
               "vo_ba_setup: %d free poses exceed the solver's LDS budget", F);
    solve_lds_size_ = lds;
    if (solve_lds_)
      VO_HIP_CHECK(hipFuncSetAttribute((const void*)ba_solve_kernel<true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    else
      VO_HIP_CHECK(hipFuncSetAttribute((const void*)ba_solve_kernel<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    VO_HIP_CHECK(hipStreamSynchronize(st));
    have_problem_ = true;
    have_state_ = false;
    pending_ = false;
    cur_ = 0;
  }

  void set_state(const double* poses, const double* points) {
    VO_REQUIRE(have_problem_, VO_ERR_STATE, "vo_ba_set_state before vo_ba_setup");
    const BAPlan& P = plan_;
    hipStream_t st = ctx_->stream;
    VO_HIP_CHECK(hipMemcpyAsync(d_pose_[0].ptr, poses, P.n_poses * 96ull, hipMemcpyHostToDevice, st));
    std::vector<double> pts(3ull * P.n_points);
    for (int q = 0; q < P.n_points; ++q)
      for (int e = 0; e < 3; ++e) pts[3ull * q + e] = points[3ull * P.pt_perm[q] + e];
    if (P.n_points)
      VO_HIP_CHECK(hipMemcpyAsync(d_points_.ptr, pts.data(), pts.size() * 8, hipMemcpyHostToDevice, st));
    VO_HIP_CHECK(hipMemsetAsync(d_status_.ptr, 0, sizeof(int), st));
    VO_HIP_CHECK(hipStreamSynchronize(st));
    cur_ = 0;
    pending_ = false;
    have_state_ = true;
  }

  void get_state(double* poses, double* points) {
    require_state();
    finalize();
    const BAPlan& P = plan_;
    hipStream_t st = ctx_->stream;
    std::vector<double> pts(3ull * P.n_points);
    VO_HIP_CHECK(hipMemcpyAsync(poses, d_pose_[cur_].ptr, P.n_poses * 96ull, hipMemcpyDeviceToHost, st));
    if (P.n_points)
      VO_HIP_CHECK(hipMemcpyAsync(pts.data(), d_points_.ptr, pts.size() * 8, hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipStreamSynchronize(st));
    for (int q = 0; q < P.n_points; ++q)
      for (int e = 0; e < 3; ++e) points[3ull * P.pt_perm[q] + e] = pts[3ull * q + e];
  }

  // iters GN iterations; sync=true finalises and reads the costs back.
  int run(int iters, double* cost_out, bool sync) {
    require_state();
    VO_REQUIRE(iters >= 0, VO_ERR_ARG, "vo_ba_run: iters < 0");
    hipStream_t st = ctx_->stream;
    d_cost_.reserve((iters + 1) * 8ull);
    for (int it = 0; it < iters; ++it) iteration(d_cost_.as<double>() + it, it + 1);
    if (!sync) return VO_OK;
    finalize_cost(d_cost_.as<double>() + iters);
    std::vector<double> costs(iters + 1);
    int status = 0;
    VO_HIP_CHECK(hipMemcpyAsync(costs.data(), d_cost_.ptr, costs.size() * 8, hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipMemcpyAsync(&status, d_status_.ptr, sizeof(int), hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipStreamSynchronize(st));
    if (status) {
      // iteration `status` (1-based) failed: the state is its linearisation point
      for (int k = status; k <= iters; ++k) costs[k] = NAN;
      VO_HIP_CHECK(hipMemsetAsync(d_status_.ptr, 0, sizeof(int), st));
      VO_HIP_CHECK(hipStreamSynchronize(st));
    }
    if (cost_out) std::copy(costs.begin(), costs.end(), cost_out);
    if (status) {
      set_error("vo_ba_run: reduced camera system not positive definite at iteration %d",
                status - 1);
      return VO_ERR_NOT_SPD;
    }
    return VO_OK;
  }

  int step_debug(double* S_out, double* b_out, double* dc_out, double* cost_out) {
    require_state();
    hipStream_t st = ctx_->stream;
    const BAPlan& P = plan_;
    const int F = P.n_free;
    d_cost_.reserve(8);
    enqueue_lin(pending_ ? (kBacksub | kAccum) : kAccum);
    enqueue_reduce();
    std::vector<double> sys(sys_len_);
    VO_HIP_CHECK(hipMemcpyAsync(sys.data(), d_sys_.ptr, sys_len_ * 8, hipMemcpyDeviceToHost, st));
    enqueue_solve(1);
    std::vector<double> dc(6ull * F);
    int status = 0;
    if (F) VO_HIP_CHECK(hipMemcpyAsync(dc.data(), d_dc_.ptr, dc.size() * 8, hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipMemcpyAsync(&status, d_status_.ptr, sizeof(int), hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipStreamSynchronize(st));
    cur_ ^= 1;
    pending_ = true;
    if (S_out) {
      const int n = 6 * F;
      std::fill(S_out, S_out + (size_t)n * n, 0.0);
      for (int i = 0; i < F; ++i)
        for (int j = P.prof_first[i]; j <= i; ++j) {
          const double* blk = sys.data() + 36ull * (P.prof_off[i] + j - P.prof_first[i]);
          for (int r = 0; r < 6; ++r)
            for (int c = 0; c < 6; ++c) {
              S_out[(size_t)(6 * i + r) * n + 6 * j + c] = blk[6 * r + c];
              S_out[(size_t)(6 * j + c) * n + 6 * i + r] = blk[6 * r + c];
            }
        }
    }
    if (b_out) std::copy(sys.begin() + 36ull * P.n_prof_blocks(), sys.begin() + 36ull * P.n_prof_blocks() + 6 * F, b_out);
    if (dc_out) std::copy(dc.begin(), dc.end(), dc_out);
    if (cost_out) *cost_out = sys[sys_len_ - 1];
    if (status) {
      VO_HIP_CHECK(hipMemsetAsync(d_status_.ptr, 0, sizeof(int), st));
      VO_HIP_CHECK(hipStreamSynchronize(st));
      set_error("vo_ba_step_debug: reduced camera system not positive definite");
      return VO_ERR_NOT_SPD;
    }
    return VO_OK;
  }

  int stats(int64_t* out, int n) const {
    const BAPlan& P = plan_;
    const int64_t wide = 0;
    const int64_t v[8] = {P.n_chunks(), P.n_segments(), P.n_slab_slots(), (int64_t)P.slot_i.size(),
                          P.n_prof_blocks(), P.n_te, P.algorithmic_bytes_per_iter(), wide};
    const int k = std::min(n, 8);
    for (int i = 0; i < k; ++i) out[i] = v[i];
    return k;
  }

 private:
  void require_state() const {
    VO_REQUIRE(have_problem_, VO_ERR_STATE, "BA: no problem set up");
    VO_REQUIRE(have_state_, VO_ERR_STATE, "BA: no state set");
  }

  static int segments_target() {
    const char* e = getenv("VO_BA_SEGMENTS");
    return e ? std::max(1, atoi(e)) : 0;
  }

  LinArgs lin_args() {
    const BAPlan& P = plan_;
    LinArgs A;
    A.n_fixed = P.n_fixed;
    A.fx = prob_.fx; A.fy = prob_.fy; A.cx = prob_.cx; A.cy = prob_.cy;
    A.lambda = prob_.lambda;
    A.obs_uv = d_obs_uv_.as<float2>();
    A.obs_cam = d_obs_cam_.as<int>();
    A.obs_te = d_obs_te_.as<int>();
    A.te_cam = d_te_cam_.as<int>();
    A.te_pt = d_te_pt_.as<int>();
    A.te_obs = d_te_obs_.as<int>();
    A.te_lcam = d_te_lcam_.as<int16_t>();
    A.pt_te = d_pt_te_.as<int>();
    A.chunk_obs = d_chunk_obs_.as<int>();
    A.chunk_te = d_chunk_te_.as<int>();
    A.chunk_pt = d_chunk_pt_.as<int>();
    A.chunk_slot_base = d_chunk_slot_base_.as<int>();
    A.chunk_cam_base = d_chunk_cam_base_.as<int>();
    A.slot_ptr = d_slot_ptr_.as<int>();
    A.pair_list = d_pair_list_.as<uint16_t>();
    A.cam_ptr = d_cam_ptr_.as<int>();
    A.cam_list = d_cam_list_.as<uint8_t>();
    A.seg_chunk = d_seg_chunk_.as<int>();
    A.seg_slot_off = d_seg_slot_off_.as<int>();
    A.seg_cam_off = d_seg_cam_off_.as<int>();
    A.points = d_points_.as<double>();
    A.slab = d_slab_.as<double>();
    A.slab_b = d_slab_b_.as<double>();
    A.slab_cost = d_slab_cost_.as<double>();
    A.pose_old = d_pose_[cur_ ^ 1].as<double>();
    A.pose_new = d_pose_[cur_].as<double>();
    A.dc = d_dc_.as<double>();
    A.status = d_status_.as<int>();
    return A;
  }

  void enqueue_lin(int mode) {
    const int nseg = plan_.n_segments();
    if (nseg <= 0) {
      // no landmarks: empty slabs, zero cost
      VO_HIP_CHECK(hipMemsetAsync(d_slab_cost_.ptr, 0, 8, ctx_->stream));
      return;
    }
    LinArgs A = lin_args();
    dim3 g(nseg), b(kLinThreads);
    switch (mode) {
      case kAccum: hipLaunchKernelGGL(ba_lin_kernel<kAccum>, g, b, 0, ctx_->stream, A); break;
      case kBacksub | kAccum:
        hipLaunchKernelGGL((ba_lin_kernel<kBacksub | kAccum>), g, b, 0, ctx_->stream, A);
        break;
      case kBacksub: hipLaunchKernelGGL(ba_lin_kernel<kBacksub>, g, b, 0, ctx_->stream, A); break;
      default: hipLaunchKernelGGL(ba_lin_kernel<0>, g, b, 0, ctx_->stream, A); break;
    }
    VO_HIP_CHECK(hipGetLastError());
  }

  void enqueue_reduce() {
    const BAPlan& P = plan_;
    ReduceArgs R;
    R.nprof = P.n_prof_blocks();
    R.F = P.n_free;
    R.nseg = std::max(P.n_segments(), plan_.n_segments() > 0 ? 0 : 1);
    R.lambda = prob_.lambda;
    R.prof_src_ptr = d_prof_src_ptr_.as<int>();
    R.prof_src = d_prof_src_.as<int>();
    R.prof_diag = d_prof_diag_.as<uint8_t>();
    R.camb_ptr = d_camb_ptr_.as<int>();
    R.camb_src = d_camb_src_.as<int>();
    R.slab = d_slab_.as<double>();
    R.slab_b = d_slab_b_.as<double>();
    R.slab_cost = d_slab_cost_.as<double>();
    R.sys = d_sys_.as<double>();
    R.status = d_status_.as<int>();
    hipLaunchKernelGGL(ba_reduce_kernel, dim3(R.nprof + 1), dim3(64), 0, ctx_->stream, R);
    VO_HIP_CHECK(hipGetLastError());
    if (ctx_->comm && ctx_->comm->nranks > 1)
      VO_NCCL_CHECK(ncclAllReduce(d_sys_.ptr, d_sys_.ptr, sys_len_, ncclFloat64, ncclSum,
                                  ctx_->comm->comm, ctx_->stream));
  }

  void enqueue_solve(int iter_tag) {
    const BAPlan& P = plan_;
    SolveArgs A;
    A.F = P.n_free;
    A.nprof = P.n_prof_blocks();
    A.n_poses = P.n_poses;
    A.n_fixed = P.n_fixed;
    A.iter_tag = iter_tag;
    A.prof_first = d_prof_first_.as<int>();
    A.prof_off = d_prof_off_.as<int>();
    A.prof_last = d_prof_last_.as<int>();
    A.sys = d_sys_.as<double>();
    A.linv_glob = d_linv_.as<double>();
    A.dc = d_dc_.as<double>();
    A.pose_cur = d_pose_[cur_].as<double>();
    A.pose_next = d_pose_[cur_ ^ 1].as<double>();
    A.status = d_status_.as<int>();
    if (solve_lds_)
      hipLaunchKernelGGL(ba_solve_kernel<true>, dim3(1), dim3(kSolveThreads), solve_lds_size_,
                         ctx_->stream, A);
    else
      hipLaunchKernelGGL(ba_solve_kernel<false>, dim3(1), dim3(kSolveThreads), solve_lds_size_,
                         ctx_->stream, A);
    VO_HIP_CHECK(hipGetLastError());
  }

  void iteration(double* d_cost_slot, int iter_tag) {
    enqueue_lin(pending_ ? (kBacksub | kAccum) : kAccum);
    enqueue_reduce();
    VO_HIP_CHECK(hipMemcpyAsync(d_cost_slot, d_sys_.as<double>() + sys_len_ - 1, 8,
                                hipMemcpyDeviceToDevice, ctx_->stream));
    enqueue_solve(iter_tag);
    cur_ ^= 1;
    pending_ = true;
  }

  // Applies the pending point update (if any) and writes the cost at the
  // resulting state into d_cost_slot.
  void finalize_cost(double* d_cost_slot) {
    enqueue_lin(pending_ ? kBacksub : 0);
    pending_ = false;
    // cost-only reduction (S/b untouched): reuse K2's last block
    ReduceArgs R{};
    R.nprof = 0;
    R.F = 0;
    R.nseg = std::max(1, plan_.n_segments());
    R.slab_cost = d_slab_cost_.as<double>();
    R.sys = d_cost_tmp();
    R.status = d_status_.as<int>();
    hipLaunchKernelGGL(ba_reduce_kernel, dim3(1), dim3(64), 0, ctx_->stream, R);
    VO_HIP_CHECK(hipGetLastError());
    if (ctx_->comm && ctx_->comm->nranks > 1)
      VO_NCCL_CHECK(ncclAllReduce(R.sys, R.sys, 1, ncclFloat64, ncclSum, ctx_->comm->comm,
                                  ctx_->stream));
    VO_HIP_CHECK(hipMemcpyAsync(d_cost_slot, R.sys, 8, hipMemcpyDeviceToDevice, ctx_->stream));
  }

  void finalize() {
    if (!pending_) return;
    d_cost_.reserve(8);
    finalize_cost(d_cost_.as<double>());
    VO_HIP_CHECK(hipStreamSynchronize(ctx_->stream));
  }

  double* d_cost_tmp() {
    d_cost_tmp_.reserve(16);
    return d_cost_tmp_.as<double>();
  }

  vo_ctx* ctx_;
  BAPlan plan_;
  vo_ba_problem prob_{};
  bool have_problem_ = false, have_state_ = false, pending_ = false, solve_lds_ = false;
  int cur_ = 0;
  size_t sys_len_ = 0, solve_lds_size_ = 0;
  DevBuf d_obs_uv_, d_obs_cam_, d_obs_te_, d_te_cam_, d_te_pt_, d_te_obs_, d_te_lcam_, d_pt_te_;
  DevBuf d_chunk_obs_, d_chunk_te_, d_chunk_pt_, d_chunk_slot_base_, d_chunk_cam_base_;
  DevBuf d_slot_ptr_, d_pair_list_, d_cam_ptr_, d_cam_list_;
  DevBuf d_seg_chunk_, d_seg_slot_off_, d_seg_cam_off_;
  DevBuf d_prof_first_, d_prof_off_, d_prof_last_, d_prof_src_ptr_, d_prof_src_, d_prof_diag_;
  DevBuf d_camb_ptr_, d_camb_src_;
  DevBuf d_points_, d_pose_[2], d_dc_, d_slab_, d_slab_b_, d_slab_cost_, d_sys_, d_linv_;
  DevBuf d_status_, d_cost_, d_cost_tmp_;
};

// ---- entry points used by api.hip -------------------------------------------------
BAEngine* ba_engine(vo_ctx* ctx) {
  if (!ctx->ba) ctx->ba.reset(new BAEngine(ctx));
  return ctx->ba.get();
}
void ba_setup(vo_ctx* ctx, const vo_ba_problem* p) { ba_engine(ctx)->setup(p); }
void ba_set_state(vo_ctx* ctx, const double* poses, const double* pts) {
  ba_engine(ctx)->set_state(poses, pts);
}
void ba_get_state(vo_ctx* ctx, double* poses, double* pts) { ba_engine(ctx)->get_state(poses, pts); }
int ba_run(vo_ctx* ctx, int iters, double* cost, bool sync) { return ba_engine(ctx)->run(iters, cost, sync); }
int ba_step_debug(vo_ctx* ctx, double* S, double* b, double* dc, double* cost) {
  return ba_engine(ctx)->step_debug(S, b, dc, cost);
}
int ba_stats(vo_ctx* ctx, int64_t* out, int n) { return ba_engine(ctx)->stats(out, n); }

void comm_unique_id(char out[128]) {
  ncclUniqueId id;
  VO_NCCL_CHECK(ncclGetUniqueId(&id));
  static_assert(sizeof(id) == 128, "unexpected ncclUniqueId size");
  memcpy(out, &id, 128);
}

void comm_init(vo_ctx* ctx, int nranks, int rank, const char id[128]) {
  VO_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, VO_ERR_ARG, "vo_comm_init: bad rank");
  std::unique_ptr<Comm> c(new Comm);
  c->nranks = nranks;
  c->rank = rank;
  ncclUniqueId uid;
  memcpy(&uid, id, 128);
  VO_NCCL_CHECK(ncclCommInitRank(&c->comm, nranks, uid, rank));
  ctx->comm = std::move(c);
}

}  // namespace vo

vo_ctx::vo_ctx() = default;

vo_ctx::~vo_ctx() {
  ba.reset();
  comm.reset();
  if (stream) (void)hipStreamDestroy(stream);
}
