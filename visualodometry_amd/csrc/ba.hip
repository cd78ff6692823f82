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
#include <type_traits>
#include <atomic>
#include <vector>

#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>

#include "ba_band.h"
#include "ba_math.h"
#include "ba_plan.h"
#include "vo_ctx.h"

#ifndef VO_BA_FUSE
#define VO_BA_FUSE 1  // tuning build: 0 launches K2 on its own
#endif

namespace vo {

// Diagnostic build only (make EXTRA=-DVO_BA_STAMPS=1): per-phase s_memtime stamps of K1
// and the profile K3.  The product build executes none.
#ifndef VO_BA_STAMPS
#define VO_BA_STAMPS 0
#endif
constexpr bool kBaStamps = VO_BA_STAMPS != 0;
// Planner target: K1 segments per CU = K1's residency (three workgroups per CU), so the
// whole launch is one round; a tuning build may override it at compile time.
#ifndef VO_BA_SEGMENTS_PER_CU
#define VO_BA_SEGMENTS_PER_CU 3
#endif

#define VO_NCCL_CHECK(expr)                                                          \
  do {                                                                               \
    ncclResult_t r_ = (expr);                                                        \
    if (r_ != ncclSuccess) {                                                         \
      ::vo::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,             \
                      ncclGetErrorString(r_));                                       \
      throw ::vo::Error{VO_ERR_RCCL};                                                \
    }                                                                                \
  } while (0)

// In-process loopback group (vo_comm_init_loopback): N contexts of one process, each
// driven by its own host thread, stand in for N RCCL ranks so that the sharded BA path
// can be tested on one device.  Each all-reduce copies to the host, meets the others at
// a barrier and reduces in rank order (every member computes the identical result).
struct LoopGroup {
  int nranks = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::vector<char>> slot;
  int arrived = 0;
  long gen = 0;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const long g = gen;
    if (++arrived == nranks) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

struct Comm {
  ncclComm_t comm = nullptr;
  std::shared_ptr<LoopGroup> loop;
  int nranks = 1, rank = 0;
  ~Comm() {
    if (comm) ncclCommDestroy(comm);
  }
  // in-place all-reduce of n elements (int32 min or float64 sum) on the context stream
  template <class T>
  void allreduce(T* dbuf, size_t n, bool is_min, hipStream_t st);
};

template <class T>
void Comm::allreduce(T* dbuf, size_t n, bool is_min, hipStream_t st) {
  if (!loop) {
    const ncclDataType_t ty = std::is_same<T, double>::value ? ncclFloat64 : ncclInt32;
    VO_NCCL_CHECK(ncclAllReduce(dbuf, dbuf, n, ty, is_min ? ncclMin : ncclSum, comm, st));
    return;
  }
  LoopGroup& G = *loop;
  std::vector<T> mine(n);
  VO_HIP_CHECK(hipMemcpyAsync(mine.data(), dbuf, n * sizeof(T), hipMemcpyDeviceToHost, st));
  VO_HIP_CHECK(hipStreamSynchronize(st));
  {
    std::lock_guard<std::mutex> lk(G.mu);
    G.slot[rank].assign(reinterpret_cast<const char*>(mine.data()),
                        reinterpret_cast<const char*>(mine.data()) + n * sizeof(T));
  }
  G.barrier();
  std::vector<T> out(n);
  for (int r = 0; r < nranks; ++r) {
    const T* v = reinterpret_cast<const T*>(G.slot[r].data());
    for (size_t i = 0; i < n; ++i)
      out[i] = r == 0 ? v[i] : is_min ? std::min(out[i], v[i]) : out[i] + v[i];
  }
  G.barrier();  // every member has read every slot
  VO_HIP_CHECK(hipMemcpyAsync(dbuf, out.data(), n * sizeof(T), hipMemcpyHostToDevice, st));
  VO_HIP_CHECK(hipStreamSynchronize(st));
}

void* plan_host_alloc(size_t bytes, bool pinned) {
  void* p = nullptr;
  if (pinned) {
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 64), hipHostMallocDefault) != hipSuccess) throw std::bad_alloc();
    return p;
  }
  return ::operator new(std::max<size_t>(bytes, 64), std::align_val_t(64));
}

void plan_host_free(void* p, bool pinned) noexcept {
  if (!p) return;
  if (pinned) (void)hipHostFree(p);
  else ::operator delete(p, std::align_val_t(64));
}

namespace {

constexpr int kLinThreads = 256;
constexpr int kBsWindow = 10;  // K3 back substitution: register window of block rows
constexpr double kPivotRelEps = 1e-12;  // == oracle/ba_ref.py PIVOT_REL_EPS
enum { kBacksub = 1, kAccum = 2 };

struct LinArgs {
  int n_fixed;
  double fx, fy, cx, cy, lambda;
  const int4* chunk_hdr;  // kChunkHdr ints per chunk (BAPlan::chunk_hdr)
  const ChunkImg* chunk_img;  // BAPlan::chunk_img
  const int* slab_pos;        // BAPlan::slab_pos (window slot -> slab row)
  const int* cam_pos;         // BAPlan::cam_pos (window camera -> rhs slab row)
  const int* seg_hdr;     // kSegHdr ints per segment (BAPlan::seg_hdr)
  double* points;
  double* slab;
  double* slab_b;
  double* slab_cost;
  const double* pose_old;  // linearisation of the pending step (back-substitution)
  const double* pose_new;  // current linearisation point
  const double* dc;        // pending pose update (6 per free camera)
  const int* status;
  unsigned long long* stamps;  // diagnostic build only: per segment phase cycles
  int nseg;                    // segments
};

struct alignas(16) LinShared {
  ChunkImg img;  // static chunk lists (BAPlan::chunk_img), staged as one image
  int spos[kSegSlots];  // slab row of each window slot
  int cpos[kSegCams];   // rhs slab row of each window camera
  double win[kSegSlots * 36];
  double bwin[kSegCams * 6];
  double Jc[kChunkObs][12];
  double Jp[kChunkObs][6];
  double r[kChunkObs][2];
  alignas(16) double Z[kChunkTe][18];  // W, then Z = W L^-T (144-B rows, 16-B aligned)
  double bt[kChunkTe][6];  // gc, then bt = -gc + Z h
  double X[kChunkPts][3];
  double L[kChunkPts][6];  // 1/l00, l10, 1/l11, l20, l21, 1/l22
  double h[kChunkPts][3];
  double dcw[kSegCams][6];  // pending pose update of the segment's window cameras
  int te_use[kChunkTe];  // free camera and valid landmark
  int valid[kChunkPts];
  double pose_o[kSegAllCams][12];  // poses of every camera the segment sees: pending step's
  double pose_n[kSegAllCams][12];  // linearisation point (back substitution) and the new one
};
// three K1 workgroups per CU (the cfg3 plan then runs in a single round)
static_assert(sizeof(LinShared) <= 160 * 1024 / 3, "K1 LDS image");

// R1: residual and Jacobians, one lane per observation.
__device__ __forceinline__ void lin_obs(LinShared& S, const LinArgs& A, const double (*pose)[12],
                                        int nob, double& cost) {
  for (int o = threadIdx.x; o < nob; o += kLinThreads) {
    const double* T = pose[S.img.acam[o]];
    const int q = S.img.te_pt[S.img.obs_te[o]];
    const double X0 = S.X[q][0], X1 = S.X[q][1], X2 = S.X[q][2];
    const double x = T[0] * X0 + T[1] * X1 + T[2] * X2 + T[9];
    const double y = T[3] * X0 + T[4] * X1 + T[5] * X2 + T[10];
    const double z = T[6] * X0 + T[7] * X1 + T[8] * X2 + T[11];
    const double iz = rcp_nr(z);
    const float2 m = reinterpret_cast<const float2*>(S.img.uv)[o];
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

// Landmark p of the chunk: V = sum Jp^T Jp (+lambda) and g = sum Jp^T r over its
// observations (S.r may hold r + Jc dc, see chunk_backsub), the pivot-tested 3x3
// Cholesky V = L L^T (same sequence as oracle/ba_ref.py point_block_valid) and
// h = L^-1 g.  l = (1/l00, l10, 1/l11, l20, l21, 1/l22).
__device__ __forceinline__ bool point_block(const LinShared& S, const LinArgs& A, int p,
                                            double (&l)[6], double (&h)[3]) {
  double v00 = 0, v01 = 0, v02 = 0, v11 = 0, v12 = 0, v22 = 0, g0 = 0, g1 = 0, g2 = 0;
  const int o0 = S.img.te_obs[S.img.pt_te[p]], o1 = S.img.te_obs[S.img.pt_te[p + 1]];
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
  // pivots by v_rsq_f64 + one Newton step (~1e-14 relative) instead of IEEE sqrt and five
  // divisions: the same pivot tests on the same values, no division on the chain
  const double eps = kPivotRelEps * (v00 + v11 + v22);
  bool ok = v00 > eps;
  const double i00 = rsq_nr(ok ? v00 : 1.0);
  const double l10 = v01 * i00, l20 = v02 * i00;
  const double d1 = v11 - l10 * l10;
  ok = ok && d1 > eps;
  const double i11 = rsq_nr(ok ? d1 : 1.0);
  const double l21 = (v12 - l20 * l10) * i11;
  const double d2 = v22 - l20 * l20 - l21 * l21;
  ok = ok && d2 > eps;
  const double i22 = rsq_nr(ok ? d2 : 1.0);
  l[0] = i00; l[1] = l10; l[2] = i11; l[3] = l20; l[4] = l21; l[5] = i22;
  h[0] = g0 * i00;
  h[1] = (g1 - l10 * h[0]) * i11;
  h[2] = (g2 - l20 * h[0] - l21 * h[1]) * i22;
  return ok;
}

// R2: per track entry W, gc; per landmark V (+lambda), pivot-tested Cholesky, h.
// The track-entry loop (threads [0, 128)) and the landmark loop (threads [128, 256)) are
// independent and run on different waves concurrently.
__device__ __forceinline__ void lin_reduce(LinShared& S, const LinArgs& A, int nte, int npt) {
  constexpr int kHalf = kLinThreads / 2;
  static_assert(kChunkTe <= kHalf && kChunkPts <= kHalf, "one track entry / landmark per thread");
  for (int t = threadIdx.x; t < nte && t < kHalf; t += kHalf) {
    double W[18], g[6];
#pragma unroll
    for (int e = 0; e < 18; ++e) W[e] = 0.0;
#pragma unroll
    for (int e = 0; e < 6; ++e) g[e] = 0.0;
    for (int o = S.img.te_obs[t]; o < S.img.te_obs[t + 1]; ++o) {
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
  for (int p = (int)threadIdx.x - kHalf; p >= 0 && p < npt; p += kHalf) {
    double l[6], h[3];
    const bool ok = point_block(S, A, p, l, h);
    S.valid[p] = ok;
#pragma unroll
    for (int e = 0; e < 6; ++e) S.L[p][e] = l[e];
    S.h[p][0] = ok ? h[0] : 0.0;
    S.h[p][1] = ok ? h[1] : 0.0;
    S.h[p][2] = ok ? h[2] : 0.0;
  }
}

// R3: Z = W L^-T and bt = -gc + Z h for track entries of valid landmarks in free
// cameras; zero otherwise (frozen landmarks leave the camera system).
__device__ __forceinline__ void lin_eliminate(LinShared& S, int nte) {
  for (int t = threadIdx.x; t < nte; t += kLinThreads) {
    const int p = S.img.te_pt[t];
    const bool use = S.valid[p] && S.img.te_lcam[t] >= 0;
    S.te_use[t] = use;
    if (!use) {
#pragma unroll
      for (int e = 0; e < 18; ++e) S.Z[t][e] = 0.0;
#pragma unroll
      for (int e = 0; e < 6; ++e) S.bt[t][e] = 0.0;
      // frozen landmark: its observations leave U too (gc was formed from Jc already)
      for (int o = S.img.te_obs[t]; o < S.img.te_obs[t + 1]; ++o)
#pragma unroll
        for (int e = 0; e < 12; ++e) S.Jc[o][e] = 0.0;
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
                                                const double (*pose)[12], int nob,
                                                int nte, int npt, double& cost) {
  lin_obs(S, A, pose, nob, cost);
  __syncthreads();
  lin_reduce(S, A, nte, npt);
  __syncthreads();
  lin_eliminate(S, nte);
  __syncthreads();
}

// Back-substitution of the pending step at its linearisation point (pose_o):
// dp = -V^-1 sum_o Jp_o^T (r_o + Jc_o dc_cam(o)) -- algebraically the Schur
// back-substitution -V^-1 (g + sum_t W_t^T dc) without forming W or Z.  V, the pivot
// test and the Cholesky are point_block's, so a landmark frozen in the pending step's
// camera system (invalid V) is not moved; fixed cameras contribute dc = 0.
__device__ __forceinline__ void chunk_backsub(LinShared& S, const LinArgs& A, int nob, int npt,
                                              int p0) {
  for (int o = threadIdx.x; o < nob; o += kLinThreads) {
    const double* T = S.pose_o[S.img.acam[o]];
    const int te = S.img.obs_te[o];
    const int q = S.img.te_pt[te];
    const double X0 = S.X[q][0], X1 = S.X[q][1], X2 = S.X[q][2];
    const double x = T[0] * X0 + T[1] * X1 + T[2] * X2 + T[9];
    const double y = T[3] * X0 + T[4] * X1 + T[5] * X2 + T[10];
    const double z = T[6] * X0 + T[7] * X1 + T[8] * X2 + T[11];
    const double iz = rcp_nr(z);
    const float2 m = reinterpret_cast<const float2*>(S.img.uv)[o];
    double r0 = A.fx * x * iz + A.cx - (double)m.x;
    double r1 = A.fy * y * iz + A.cy - (double)m.y;
    const double j00 = A.fx * iz, j02 = -A.fx * x * iz * iz;
    const double j11 = A.fy * iz, j12 = -A.fy * y * iz * iz;
    const int lc = S.img.te_lcam[te];
    if (lc >= 0) {  // + Jc dc (rows of lin_obs's Jc)
      const double* d = S.dcw[lc];
      r0 += j00 * d[0] + j02 * d[2] + (j02 * y) * d[3] + (j00 * z - j02 * x) * d[4] - (j00 * y) * d[5];
      r1 += j11 * d[1] + j12 * d[2] + (j12 * y - j11 * z) * d[3] - (j12 * x) * d[4] + (j11 * x) * d[5];
    }
    S.r[o][0] = r0;
    S.r[o][1] = r1;
    double* jp = S.Jp[o];
    jp[0] = j00 * T[0] + j02 * T[6];
    jp[1] = j00 * T[1] + j02 * T[7];
    jp[2] = j00 * T[2] + j02 * T[8];
    jp[3] = j11 * T[3] + j12 * T[6];
    jp[4] = j11 * T[4] + j12 * T[7];
    jp[5] = j11 * T[5] + j12 * T[8];
  }
  __syncthreads();
  for (int p = threadIdx.x; p < npt; p += kLinThreads) {
    double l[6], h[3];
    if (!point_block(S, A, p, l, h)) continue;
    const double x2 = -h[2] * l[5];
    const double x1 = (-h[1] - l[4] * x2) * l[2];
    const double x0 = (-h[0] - l[1] * x1 - l[3] * x2) * l[0];
    S.X[p][0] += x0;
    S.X[p][1] += x1;
    S.X[p][2] += x2;
    A.points[3l * (p0 + p)] = S.X[p][0];
    A.points[3l * (p0 + p) + 1] = S.X[p][1];
    A.points[3l * (p0 + p) + 2] = S.X[p][2];
  }
}

// Lanes per Schur item: the largest power of two <= 8 that keeps every item's parts in
// one pass of the workgroup (parts of an item are adjacent lanes of one wave).
__device__ __forceinline__ int parts_for(int items) {
  return items * 8 <= kLinThreads ? 8 : items * 4 <= kLinThreads ? 4 : items * 2 <= kLinThreads ? 2 : 1;
}

template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), Ctrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), Ctrl, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// Sum of the np (2, 4 or 8) adjacent lanes' values, valid in the first lane of each
// group: a fixed butterfly (xor 1, xor 2 within quads, then row_shl:4), so the order of
// the additions never depends on timing.  Every lane of the wave must execute it.
__device__ __forceinline__ double sum_parts(double v, int np) {
  v += dpp_f64<0xB1>(v);               // quad_perm [1,0,3,2]
  if (np >= 4) v += dpp_f64<0x4E>(v);  // quad_perm [2,3,0,1]
  if (np >= 8) v += dpp_f64<0x104>(v); // row_shl:4 (lane 8g + 0 reads 8g + 4)
  return v;
}

// The same butterfly with a per-lane group width 2^lg (0..3): groups are aligned to their
// width, so each step only ever combines lanes of one group; lanes of narrower groups keep
// their value (select).  Every lane of the wave must execute it.
__device__ __forceinline__ double sum_parts_lane(double v, int lg) {
  const double a = dpp_f64<0xB1>(v);
  v = lg >= 1 ? v + a : v;
  const double b = dpp_f64<0x4E>(v);
  v = lg >= 2 ? v + b : v;
  const double c = dpp_f64<0x104>(v);
  return lg >= 3 ? v + c : v;
}

// Diagnostic build (VO_BA_STAMPS=1): thread 0 accumulates s_memtime deltas per
// phase; the production instantiation has kStamp = false and executes none.
// dst[i] = src[i] + add, i < n, by the workgroup: U loads per thread issued before
// any store; loads are unconditional (clamped index) so none is sunk into a branch.
template <typename T, int U, typename Src, typename V>
__device__ __forceinline__ void stage(T* dst, const Src* __restrict__ src, int n, V add) {
  if (n <= 0) return;
  for (int e = threadIdx.x; e < n; e += U * kLinThreads) {
    Src a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = src[min(e + u * kLinThreads, n - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (e + u * kLinThreads < n) dst[e + u * kLinThreads] = (T)(a[u] + add);
  }
}

enum { kPhLoad = 0, kPhBacksub, kPhLinObs, kPhReduce, kPhElim, kPhSchur, kPhWrite, kPhSchurU, kPhT0, kPhT1,
       // per-segment work counts (cost-model fitting): observations, track entries,
       // landmarks, pair-list entries, window slots, window cameras
       kPhObs, kPhTe, kPhPts, kPhPairs, kPhSlots, kPhCams, kPhCount };
template <bool kStamp>
struct Stamper {
  // the stamping lane (thread 0, or lane 0 of each one-wave segment) and its output row;
  // s_memtime counts per XCD (clocks of different XCDs are unrelated), so the row's
  // window-camera count carries the XCD id in bits 24..31
  unsigned long long t = 0, acc[kPhCount] = {};
  bool lead = false;
  int row = 0;
  __device__ __forceinline__ void start(bool ld, int r) {
    lead = kStamp && ld;
    row = r;
    if (lead) {
      acc[kPhT0] = t = __builtin_amdgcn_s_memtime();
      unsigned xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
      acc[kPhCams] = (unsigned long long)xcc << 24;
    }
  }
  __device__ __forceinline__ void start() { start(threadIdx.x == 0, blockIdx.x); }
  __device__ __forceinline__ void mark(int ph) {
    if (lead) {
      const unsigned long long n = __builtin_amdgcn_s_memtime();
      acc[ph] += n - t;
      t = n;
    }
  }
  __device__ __forceinline__ void count(int k, int v) {
    if (lead) acc[k] += (unsigned long long)v;
  }
  __device__ __forceinline__ void flush(unsigned long long* out) {
    if (lead) acc[kPhT1] = __builtin_amdgcn_s_memtime();  // absolute
    if (lead && out)
      for (int k = 0; k < kPhCount; ++k) out[(long)row * kPhCount + k] = acc[k];
  }
};

template <int MODE, bool kStamp>
__global__ __launch_bounds__(kLinThreads, 3) void ba_lin_kernel(LinArgs A) {  // 3 per CU: <= 168 VGPRs
  __shared__ LinShared S;
  Stamper<kStamp> st;
  st.start();
  const int seg = blockIdx.x, tid = threadIdx.x;
  // one load level: the status word, the segment header (uniform) and this thread's
  // camera ids (fixed offsets in the header); then poses and the pending update
  const int* SH = A.seg_hdr + (long)kSegHdr * seg;
  const int4* SH4 = reinterpret_cast<const int4*>(SH);
  const int16_t* SH16 = reinterpret_cast<const int16_t*>(SH);
  const int stat = A.status ? *A.status : 0;
  const int4 g0 = SH4[0], g1 = SH4[1];
  int4 h0 = SH4[8], h1 = SH4[9], h2 = SH4[10], h3 = SH4[11];  // first chunk's header
  const int i_acam = SH16[16 + min(tid / 12, kSegAllCams - 1)];
  const int i_wcam = SH16[32 + min(tid / 6, kSegCams - 1)];
  if (stat) return;  // a previous solve failed: state frozen
  const int nslots = g0.x, slot_off = g0.y, cam0 = g0.z, ncams = g0.w, na = g1.x;
  const int ch0 = g1.y, ch1 = g1.z;
  static_assert(12 * kSegAllCams <= kLinThreads && 6 * kSegCams <= kLinThreads,
                "one pose / update element per thread");
  if (MODE & kBacksub)
    if (tid < ncams * 6) S.dcw[tid / 6][tid % 6] = A.dc[6l * i_wcam + tid % 6];
  if (tid < 12 * na) {  // poses of the segment's cameras, once per segment
    const long g = 12l * i_acam + tid % 12;
    S.pose_n[tid / 12][tid % 12] = A.pose_new[g];
    if (MODE & kBacksub) S.pose_o[tid / 12][tid % 12] = A.pose_old[g];
  }
  if (MODE & kAccum) {
    for (int e = tid; e < nslots * 36; e += kLinThreads) S.win[e] = 0.0;
    for (int e = tid; e < ncams * 6; e += kLinThreads) S.bwin[e] = 0.0;
    if (tid < nslots) S.spos[tid] = A.slab_pos[slot_off + tid];
    if (tid < ncams) S.cpos[tid] = A.cam_pos[cam0 + tid];
  }
  double cost = 0.0;
  st.count(kPhSlots, nslots);
  st.count(kPhCams, ncams);
  // staging of a chunk: one 16-byte load of its image and of its landmark positions
  // (state) per thread, issued one chunk ahead (the next chunk's landmarks are disjoint from
  // the ones this chunk's back substitution writes); headers are read two chunks ahead
  constexpr int kImgVec = (int)(sizeof(ChunkImg) / 16);
  static_assert(kImgVec <= kLinThreads && 3 * kChunkPts <= kLinThreads, "one staging element per thread");
  const int i0 = tid;
  auto stage_img = [&](int c) { return reinterpret_cast<const uint4*>(A.chunk_img + c)[min(tid, kImgVec - 1)]; };
  auto stage_x = [&](const int4& hp) { return A.points[3l * hp.x + min(i0, max(3 * hp.y - 1, 0))]; };
  uint4 v_img = stage_img(ch0);
  double v_x = stage_x(h1);
  int4 n0, n1, n2, n3;  // the next chunk's header
  {
    const int chn = min(ch0 + 1, ch1 - 1);
    n0 = A.chunk_hdr[4l * chn];
    n1 = A.chunk_hdr[4l * chn + 1];
    n2 = A.chunk_hdr[4l * chn + 2];
    n3 = A.chunk_hdr[4l * chn + 3];
  }
  for (int ch = ch0; ch < ch1; ++ch) {
    const int chn = min(ch + 1, ch1 - 1), chn2 = min(ch + 2, ch1 - 1);
    const int4 m0 = A.chunk_hdr[4l * chn2], m1 = A.chunk_hdr[4l * chn2 + 1], m2 = A.chunk_hdr[4l * chn2 + 2],
               m3 = A.chunk_hdr[4l * chn2 + 3];
    const uint4 w_img = stage_img(chn);
    const double w_x = stage_x(n1);
    const int nob = h0.y, nte = h0.w, p0 = h1.x, npt = h1.y, e0 = h2.x, e1 = h2.y;
    st.count(kPhObs, nob);
    st.count(kPhTe, nte);
    st.count(kPhPts, npt);
    st.count(kPhPairs, e1 - e0);
    auto rotate = [&]() {
      h0 = n0;
      h1 = n1;
      h2 = n2;
      h3 = n3;
      n0 = m0;
      n1 = m1;
      n2 = m2;
      n3 = m3;
      v_img = w_img;
      v_x = w_x;
    };
    __syncthreads();  // previous chunk fully consumed
    if (tid < kImgVec) reinterpret_cast<uint4*>(&S.img)[tid] = v_img;
    if (i0 < 3 * npt) (&S.X[0][0])[i0] = v_x;
    __syncthreads();
    st.mark(kPhLoad);

    if (MODE & kBacksub) {
      chunk_backsub(S, A, nob, npt, p0);
      __syncthreads();
      st.mark(kPhBacksub);
    }

    if (!(MODE & kAccum)) {
      lin_obs(S, A, S.pose_n, nob, cost);  // cost at the updated state
      rotate();
      continue;
    }
    lin_obs(S, A, S.pose_n, nob, cost);
    __syncthreads();
    st.mark(kPhLinObs);
    lin_reduce(S, A, nte, npt);
    __syncthreads();
    st.mark(kPhReduce);
    lin_eliminate(S, nte);
    __syncthreads();
    st.mark(kPhElim);

    // R4: Schur blocks into the window.  Item (slot, row a) sums its slot's pair list of
    // this chunk; with few slots (narrow segments: two cameras, many two-view landmarks)
    // an item's list is split over np lanes (pairs e0 + part + j np) whose partial rows
    // are combined by a fixed DPP butterfly -- deterministic, no LDS scratch.  Unrolled by
    // two with two register sets: pair j+2's Z rows are fetched (16-byte LDS reads,
    // indices read two pairs ahead, clamped -- no branches) while pair j+1's 18 FMAs run.
    {
      // the chunk's active slots on balanced lanes (ChunkImg::abase / anp): lane tid -> entry
      // si (binary search over the lane bases), row a, part of 2^lgp
      // (a chunk with more than 42 active slots takes a second pass of one lane per row item)
      static_assert(kLinLanes == kLinThreads, "planner lane budget = K1 workgroup");
      const int nas = h3.z, lanes = S.img.abase[nas];
      for (int base = 0; base < lanes; base += kLinThreads) {
      const int t = base + tid;
      int si = 0;
#pragma unroll
      for (int st = 32; st > 0; st >>= 1)
        if (si + st < nas && S.img.abase[si + st] <= t) si += st;
      const bool live = t < lanes;
      const int lgp = live ? S.img.anp[si] : 0, np = 1 << lgp;
      const int off = t - S.img.abase[si], a = off >> lgp, part = off & (np - 1);
      const int s = live ? S.img.aslot[si] : 0;
        double out[6] = {0, 0, 0, 0, 0, 0};
        const int e0 = live ? S.img.slotp[si] + part : 0, e1 = live ? S.img.slotp[si] + S.img.apcnt[si] : 0;
        if (e0 < e1) {
          auto zrow = [&](int pr, double (&za)[3], double2 (&zy)[9]) {
            const double2* py = reinterpret_cast<const double2*>(S.Z[pr >> 8]);
#pragma unroll
            for (int k = 0; k < 9; ++k) zy[k] = py[k];
            const double* px = &S.Z[pr & 255][3 * a];
            za[0] = px[0];
            za[1] = px[1];
            za[2] = px[2];
          };
          auto accum = [&](const double (&za)[3], const double2 (&zy)[9]) {
            const double* zf = reinterpret_cast<const double*>(zy);
#pragma unroll
            for (int c = 0; c < 6; ++c)
              out[c] -= za[0] * zf[3 * c] + za[1] * zf[3 * c + 1] + za[2] * zf[3 * c + 2];
          };
          const int n = (e1 - e0 + np - 1) / np;  // this part's pairs
          auto pid = [&](int j) { return (int)S.img.pairs[e0 + min(j, n - 1) * np]; };
          double zaA[3], zaB[3];
          double2 zyA[9], zyB[9];
          zrow(pid(0), zaA, zyA);
          zrow(pid(1), zaB, zyB);
          int pc = pid(2), pd = pid(3);
          int j = 0;
          for (; j + 2 <= n; j += 2) {
            const int pe = pid(j + 4), pf = pid(j + 5);
            accum(zaA, zyA);
            zrow(pc, zaA, zyA);
            accum(zaB, zyB);
            zrow(pd, zaB, zyB);
            pc = pe;
            pd = pf;
          }
          if (j < n) accum(zaA, zyA);
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) out[c] = sum_parts_lane(out[c], lgp);
        if (live && part == 0)
#pragma unroll
          for (int c = 0; c < 6; ++c) S.win[36 * s + 6 * a + c] += out[c];
      }
    }
    st.mark(kPhSchur);
    __syncthreads();  // the diagonal slots receive U below
    // per window camera c, row a: U_c row a = sum over its observations of Jc^T Jc
    // (static observation list, indices read ahead) and b_c[a] = sum of bt over its
    // track entries; split over np lanes like the pairs when the window is narrow
    {
      const int items = h3.w * 6;  // the chunk's active cameras (ChunkImg::acid)
      const int np = parts_for(items);
      for (int base = 0; base < items * np; base += kLinThreads) {
        const int idx = base + tid, item = idx / np, part = idx % np;
        const int ci = item / 6, a = item - 6 * (item / 6);
        const int c = item < items ? S.img.acid[ci] : 0;
        double out[6] = {0, 0, 0, 0, 0, 0};
        double acc = 0.0;
        if (item < items) {
          const int q0 = S.img.camop[ci] + part, q1 = S.img.camop[ci + 1];
          if (q1 > q0) {
            const int ql = q1 - 1;
            int on = S.img.camol[q0];
            for (int q = q0; q < q1; q += np) {
              const int o = on;
              on = S.img.camol[min(q + np, ql)];
              const double2* jr = reinterpret_cast<const double2*>(S.Jc[o]);
              double j[12];
#pragma unroll
              for (int k = 0; k < 6; ++k) {
                const double2 v = jr[k];
                j[2 * k] = v.x;
                j[2 * k + 1] = v.y;
              }
              const double ja0 = S.Jc[o][a], ja1 = S.Jc[o][6 + a];
#pragma unroll
              for (int cc = 0; cc < 6; ++cc) out[cc] += ja0 * j[cc] + ja1 * j[6 + cc];
            }
          }
          const int e0 = S.img.camp[ci] + part, e1 = S.img.camp[ci + 1];
          if (e1 > e0) {
            const int el = e1 - 1;
            int xn = S.img.caml[e0];
            for (int e = e0; e < e1; e += np) {
              const int x = xn;
              xn = S.img.caml[min(e + np, el)];
              acc += S.bt[x][a];
            }
          }
        }
        if (np > 1) {
#pragma unroll
          for (int cc = 0; cc < 6; ++cc) out[cc] = sum_parts(out[cc], np);
          acc = sum_parts(acc, np);
        }
        if (item < items && part == 0) {
          S.bwin[6 * c + a] += acc;
          double* w = &S.win[36 * S.img.dslot[ci] + 6 * a];
#pragma unroll
          for (int cc = 0; cc < 6; ++cc) w[cc] += out[cc];
        }
      }
    }
    st.mark(kPhSchurU);
    rotate();
  }
  __syncthreads();
  if (MODE & kAccum) {  // window slots to their profile-major slab rows (K2 reads them in order)
    for (int e = tid; e < nslots * 36; e += kLinThreads) A.slab[36l * S.spos[e / 36] + e % 36] = S.win[e];
    for (int e = tid; e < ncams * 6; e += kLinThreads) A.slab_b[6l * S.cpos[e / 6] + e % 6] = S.bwin[e];
  }
  // segment cost: a fixed xor butterfly inside each wave, then the four wave sums in order
  // (deterministic; one barrier instead of a nine-barrier LDS tree)
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) cost += __shfl_xor(cost, m, 64);
  double* red = &S.Z[0][0];  // Z is dead after the last chunk: reuse it for the cost
  if ((tid & 63) == 0) red[tid >> 6] = cost;
  __syncthreads();
  if (tid == 0) {
    double c = 0.0;
    for (int w = 0; w < kLinThreads / 64; ++w) c += red[w];
    A.slab_cost[seg] = c;
  }
  st.mark(kPhWrite);
  st.flush(A.stamps);
}

// ---- K1, one wave per chunk (plans of one chunk per segment) --------------------------
// A segment is one chunk and one 64-lane workgroup: every phase of the chunk runs on one
// wave (a workgroup barrier is then only the LDS wait), and six such workgroups share a CU,
// so all of cfg3's chunks run at once instead of three four-wave workgroups per CU walking
// two chunks each behind nine barriers a chunk.  The LDS image is ~25.5 KB: the track
// entries' Z | bt region doubles as the observations' Jp | r during the linearisation and as
// the back substitution's pose_o | dc; the camera blocks U and the rhs are summed by the
// diagonal slots' lanes over their pairs' observations (a diagonal slot's pairs are exactly
// its camera's track entries), so every window item is finished in registers and written to
// its slab row once.
// Z rows of 18 doubles (36 dwords: the rows start on 16 different 4-bank offsets of gfx950's
// 64 banks, so a ds_read_b128 of 16 lanes on random rows rarely conflicts; a 24-double row of
// Z | bt started on 4 offsets only, a 4-way conflict on every Schur load)
// The one-wave K1's phase boundary: its workgroup is one wave, whose LDS operations complete
// in order, so a phase only needs its LDS writes done and the compiler kept from moving LDS
// accesses across (no s_barrier; and no workgroup fence, which would also wait for every
// outstanding global store: the back substitution's points and the slab rows).
__device__ __forceinline__ void lds_sync_wave() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

constexpr int kZbStride = 18;                  // doubles per track entry's Z row
constexpr int kZbR = 6 * kChunkObs;            // r (2 per observation) after Jp (6 per observation)
constexpr int kZbDc = kZbR + 2 * kChunkObs;    // back substitution: dc of the window cameras
constexpr int kZbPoseO = kZbDc + 6 * kSegCams; // back substitution: poses of the pending step
static_assert(kZbPoseO + 12 * kSegAllCams <= kChunkTe * kZbStride, "Zb region aliases");

struct alignas(16) LinWave {
  ChunkImg img;
  int spos[kSegSlots];
  int cpos[kSegCams];
  alignas(16) double Jc[kChunkObs][10];  // compressed camera Jacobian rows (jc_load)
  alignas(16) double zb[kChunkTe * kZbStride];
  alignas(16) double bt[kChunkTe][6];
  double X[kChunkPts][3];
  double L[kChunkPts][6];  // 1/l00, l10, 1/l11, l20, l21, 1/l22
  double h[kChunkPts][3];
  double pose_n[kSegAllCams][12];  // after the linearisation: the chunk's b sums by window camera
  uint8_t valid[kChunkPts];
  // segments of several chunks (one wave each): per window slot the scratch row of this chunk's
  // block (0xFF: not active here), per window camera whether the chunk has its b, the cost
  uint8_t srow[kSegSlots];
  uint8_t crow[kSegCams];
  double wcost;
};
// six per CU (cfg3's 1362 chunks in one round on 256 CUs); segments of two chunks: three
// workgroups of two waves, of three chunks: two of three
constexpr int kWaveSegsPerCu = 6;
static_assert(sizeof(LinWave) <= 160 * 1024 / kWaveSegsPerCu, "one-wave K1 LDS image");
static_assert(kWaveMaxChunks <= 8 && kWaveMaxChunks * sizeof(LinWave) <= 160 * 1024 &&
                  kWaveItems * 36 * sizeof(double) <= 2176 * sizeof(double),
              "the chunks of a segment fit one CU; every item's block fits the scratch rows");

// point_block over the Zb region's Jp | r (same operation order)
__device__ __forceinline__ bool point_block_w(const LinWave& S, double lambda, int p, double (&l)[6],
                                              double (&h)[3]) {
  double v00 = 0, v01 = 0, v02 = 0, v11 = 0, v12 = 0, v22 = 0, g0 = 0, g1 = 0, g2 = 0;
  const int o0 = S.img.pt_obs[p], o1 = S.img.pt_obs[p + 1];
  for (int o = o0; o < o1; ++o) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const double a = S.zb[6 * o + 3 * k], b = S.zb[6 * o + 3 * k + 1], c = S.zb[6 * o + 3 * k + 2];
      const double rk = S.zb[kZbR + 2 * o + k];
      v00 += a * a; v01 += a * b; v02 += a * c;
      v11 += b * b; v12 += b * c; v22 += c * c;
      g0 += a * rk; g1 += b * rk; g2 += c * rk;
    }
  }
  v00 += lambda; v11 += lambda; v22 += lambda;
  const double eps = kPivotRelEps * (v00 + v11 + v22);
  bool ok = v00 > eps;
  const double i00 = rsq_nr(ok ? v00 : 1.0);
  const double l10 = v01 * i00, l20 = v02 * i00;
  const double d1 = v11 - l10 * l10;
  ok = ok && d1 > eps;
  const double i11 = rsq_nr(ok ? d1 : 1.0);
  const double l21 = (v12 - l20 * l10) * i11;
  const double d2 = v22 - l20 * l20 - l21 * l21;
  ok = ok && d2 > eps;
  const double i22 = rsq_nr(ok ? d2 : 1.0);
  l[0] = i00; l[1] = l10; l[2] = i11; l[3] = l20; l[4] = l21; l[5] = i22;
  h[0] = g0 * i00;
  h[1] = (g1 - l10 * h[0]) * i11;
  h[2] = (g2 - l20 * h[0] - l21 * h[1]) * i22;
  return ok;
}

// Residual and Jacobians of observation o at pose T (lin_obs / chunk_backsub arithmetic);
// r and Jp into the Zb region, Jc (kJc) into S.Jc.  The back substitution (kBack) adds
// Jc dc for a free camera (dc non-null) and sums no cost.
template <bool kJc, bool kBack>
__device__ __forceinline__ void obs_lin_w(LinWave& S, const LinArgs& A, const double* T, int o,
                                          const double* dc, double& cost) {
  const int q = S.img.obs_pt[o];
  const double X0 = S.X[q][0], X1 = S.X[q][1], X2 = S.X[q][2];
  const double x = T[0] * X0 + T[1] * X1 + T[2] * X2 + T[9];
  const double y = T[3] * X0 + T[4] * X1 + T[5] * X2 + T[10];
  const double z = T[6] * X0 + T[7] * X1 + T[8] * X2 + T[11];
  const double iz = rcp_nr(z);
  const float2 m = reinterpret_cast<const float2*>(S.img.uv)[o];
  double r0 = A.fx * x * iz + A.cx - (double)m.x;
  double r1 = A.fy * y * iz + A.cy - (double)m.y;
  const double j00 = A.fx * iz, j02 = -A.fx * x * iz * iz;
  const double j11 = A.fy * iz, j12 = -A.fy * y * iz * iz;
  if (kBack && dc) {
    r0 += j00 * dc[0] + j02 * dc[2] + (j02 * y) * dc[3] + (j00 * z - j02 * x) * dc[4] - (j00 * y) * dc[5];
    r1 += j11 * dc[1] + j12 * dc[2] + (j12 * y - j11 * z) * dc[3] - (j12 * x) * dc[4] + (j11 * x) * dc[5];
  }
  if (!kBack) cost += r0 * r0 + r1 * r1;
  S.zb[kZbR + 2 * o] = r0;
  S.zb[kZbR + 2 * o + 1] = r1;
  if (kJc) {  // compressed rows (jc_load): row 0 without column 1, row 1 without column 0
    double2* jc = reinterpret_cast<double2*>(S.Jc[o]);
    jc[0] = make_double2(j00, j02);
    jc[1] = make_double2(j02 * y, j00 * z - j02 * x);
    jc[2] = make_double2(-j00 * y, j11);
    jc[3] = make_double2(j12, j12 * y - j11 * z);
    jc[4] = make_double2(-j12 * x, j11 * x);
  }
  double* jp = &S.zb[6 * o];
  jp[0] = j00 * T[0] + j02 * T[6];
  jp[1] = j00 * T[1] + j02 * T[7];
  jp[2] = j00 * T[2] + j02 * T[8];
  jp[3] = j11 * T[3] + j12 * T[6];
  jp[4] = j11 * T[4] + j12 * T[7];
  jp[5] = j11 * T[5] + j12 * T[8];
}

// Observation o's camera Jacobian rows from the compressed LDS row (10 doubles: row 0 without
// its structural zero at column 1, row 1 without column 0; 80-byte rows start on 16 bank
// offsets)
__device__ __forceinline__ void jc_load(const LinWave& S, int o, double (&jj)[12]) {
  const double2* jr = reinterpret_cast<const double2*>(S.Jc[o]);
  const double2 a = jr[0], b = jr[1], c = jr[2], d = jr[3], e = jr[4];
  jj[0] = a.x; jj[1] = 0.0; jj[2] = a.y; jj[3] = b.x; jj[4] = b.y; jj[5] = c.x;
  jj[6] = 0.0; jj[7] = c.y; jj[8] = d.x; jj[9] = d.y; jj[10] = e.x; jj[11] = e.y;
}

// One lane's Schur item (one-wave K1): active slot si's block, -sum over the slot's pairs of
// Z_x Z_y^T as FMA chains with both Z rows in registers (pair j+1's rows fetched while pair j
// accumulates); a diagonal slot's lane adds U over its pairs' observations (pair (x, x): track
// entry x of the slot's camera).  The block goes straight to its slab row.
template <bool kGroup, class Stamp>
__device__ __forceinline__ void schur_block(LinWave& S, const LinArgs& A, int si, bool live, Stamp& st) {
  double out[36];
#pragma unroll
  for (int e = 0; e < 36; ++e) out[e] = 0.0;
  const int e0 = S.img.slotp[si], n = live ? S.img.apcnt[si] : 0;
  const int dcam = S.img.adcam[si], s = S.img.aslot[si];
  if (n > 0) {
    auto zload = [&](int pr, double2 (&zx)[9], double2 (&zy)[9]) {
      const double2* px = reinterpret_cast<const double2*>(&S.zb[kZbStride * (pr & 255)]);
      const double2* py = reinterpret_cast<const double2*>(&S.zb[kZbStride * (pr >> 8)]);
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        zx[k] = px[k];
        zy[k] = py[k];
      }
    };
    auto accum = [&](const double2 (&zx)[9], const double2 (&zy)[9]) {
      const double* x = reinterpret_cast<const double*>(zx);
      const double* y = reinterpret_cast<const double*>(zy);
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          double v = out[6 * i + j];
          v = __builtin_fma(-x[3 * i], y[3 * j], v);
          v = __builtin_fma(-x[3 * i + 1], y[3 * j + 1], v);
          out[6 * i + j] = __builtin_fma(-x[3 * i + 2], y[3 * j + 2], v);
        }
    };
    auto pid = [&](int j) { return (int)S.img.pairs[e0 + min(j, n - 1)]; };
    double2 zxA[9], zyA[9], zxB[9], zyB[9];
    zload(pid(0), zxA, zyA);
    int pn = pid(1);
    int j = 0;
    for (; j + 2 <= n; j += 2) {
      zload(pn, zxB, zyB);
      pn = pid(j + 2);
      accum(zxA, zyA);
      zload(pn, zxA, zyA);
      pn = pid(j + 3);
      accum(zxB, zyB);
    }
    if (j < n) accum(zxA, zyA);
  }
  st.mark(kPhSchur);  // stamped builds: the pair sums
  // a diagonal item: U over its pairs' observations (camol entries [auo[si], auo[si + 1]), in
  // observation order, observation i + 1's Jc fetched while i accumulates) and its share of
  // b over its pairs (track entry x's bt row)
  double ob[6] = {0, 0, 0, 0, 0, 0};
  const int u0 = S.img.auo[si], un = live ? S.img.auo[si + 1] - u0 : 0;
  if (un > 0) {
    auto uacc = [&](const double (&jj)[12]) {
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int c = 0; c < 6; ++c)
          out[6 * i + c] = __builtin_fma(jj[6 + i], jj[6 + c], __builtin_fma(jj[i], jj[c], out[6 * i + c]));
    };
    auto oid = [&](int i) { return (int)S.img.camol[u0 + min(i, un - 1)]; };
    double jA[12], jB[12];
    jc_load(S, oid(0), jA);
    int on = oid(1);
    int i = 0;
    for (; i + 2 <= un; i += 2) {
      jc_load(S, on, jB);
      on = oid(i + 2);
      uacc(jA);
      jc_load(S, on, jA);
      on = oid(i + 3);
      uacc(jB);
    }
    if (i < un) uacc(jA);
  }
  if (n > 0 && dcam != 0xFF) {
    int xn = S.img.pairs[e0] & 255;
    for (int e = 0; e < n; ++e) {
      const double2* br = reinterpret_cast<const double2*>(S.bt[xn]);
      xn = S.img.pairs[e0 + min(e + 1, n - 1)] & 255;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double2 v = br[k];
        ob[2 * k] += v.x;
        ob[2 * k + 1] += v.y;
      }
    }
  }
  if (!live) {
    st.mark(kPhSchurU);
    return;
  }
  if (dcam != 0xFF) {  // this copy's share of the camera's b, for rhs_rows (the X | L | h region is dead)
    double2* bp = reinterpret_cast<double2*>(&S.X[0][0]) + 3 * si;
#pragma unroll
    for (int k = 0; k < 3; ++k) bp[k] = make_double2(ob[2 * k], ob[2 * k + 1]);
  }
  if (!kGroup && S.img.anp[si] <= 1) {  // a slot of one item: its slab row
    double2* w = reinterpret_cast<double2*>(&A.slab[36l * S.spos[s]]);
#pragma unroll
    for (int e = 0; e < 18; ++e) w[e] = make_double2(out[2 * e], out[2 * e + 1]);
  } else {  // a copy (or any item of a multi-chunk segment): its block to the scratch (Jc | Z | bt)
    lds_sync_wave();  // every lane's reads of that region are done (one wave, in order)
    double2* w = reinterpret_cast<double2*>(&S.Jc[0][0]) + 18 * si;
#pragma unroll
    for (int e = 0; e < 18; ++e) w[e] = make_double2(out[2 * e], out[2 * e + 1]);
  }
  st.mark(kPhSchurU);  // stamped builds: U, the b partials and the block's slab stores
}

// A slot's copies (one-wave K1): copy k of m sums entries [36 k / m, 36 (k + 1) / m) of the
// slot's m partial blocks (scratch rows of consecutive items) in copy order into the slab row
// (kGroup: into the first copy's scratch row, for the segment's combine; copy k only ever reads
// and writes entry range k of that row).
static_assert(offsetof(LinWave, zb) == offsetof(LinWave, Jc) + sizeof(LinWave::Jc) &&
                  offsetof(LinWave, bt) == offsetof(LinWave, zb) + sizeof(LinWave::zb) &&
                  sizeof(LinWave::Jc) + sizeof(LinWave::zb) + sizeof(LinWave::bt) >= 36 * sizeof(double) * kWaveItems,
              "the copies' scratch (kWaveItems items) fits the Jc | Z | bt region");
template <bool kGroup>
__device__ __forceinline__ void copy_rows(LinWave& S, const LinArgs& A, int si, bool live) {
  const int m = S.img.anp[si];
  if (!live || m <= 1) return;
  const int k = S.img.acopy[si], j0 = si - k;
  const int e0 = 36 * k / m, ne = 36 * (k + 1) / m - e0;  // <= 18 entries (m >= 2)
  double* sc = &S.Jc[0][0] + 36 * j0 + e0;
  double acc[18];
#pragma unroll
  for (int i = 0; i < 18; ++i) acc[i] = sc[min(i, ne - 1)];  // every load of a copy in flight
  int c = 1;
  for (; c + 2 <= m; c += 2) {  // two copies' loads in flight, added in copy order
    double v[18], u[18];
#pragma unroll
    for (int i = 0; i < 18; ++i) {
      v[i] = sc[36 * c + min(i, ne - 1)];
      u[i] = sc[36 * (c + 1) + min(i, ne - 1)];
    }
#pragma unroll
    for (int i = 0; i < 18; ++i) acc[i] = (acc[i] + v[i]) + u[i];
  }
  if (c < m)
#pragma unroll
    for (int i = 0; i < 18; ++i) acc[i] += sc[36 * c + min(i, ne - 1)];
  double* row = kGroup ? sc : &A.slab[36l * S.spos[S.img.aslot[si]] + e0];
#pragma unroll
  for (int i = 0; i < 18; ++i)
    if (i < ne) row[i] = acc[i];
}

// The rhs of the chunk's window cameras (one-wave K1): lane (active camera ci, row a) adds row a
// of the camera's diagonal copies' partial sums (consecutive items cdiag0 .. + cdiagn, left in
// the X | L | h region by schur_block) in item order into its slab entry (kGroup: into the dead
// pose_n region by window camera, for the segment's combine).
template <bool kGroup>
__device__ __forceinline__ void rhs_rows(LinWave& S, const LinArgs& A, int nac, int tid) {
  static_assert(sizeof(S.X) + sizeof(S.L) + sizeof(S.h) >= 6 * sizeof(double) * kWaveSlots &&
                    offsetof(LinWave, L) == offsetof(LinWave, X) + sizeof(S.X) &&
                    offsetof(LinWave, h) == offsetof(LinWave, L) + sizeof(S.L),
                "b partials of every item fit the X | L | h region");
  const double* bp = &S.X[0][0];
  for (int q = tid; q < 6 * nac; q += kLinLanesWave) {
    const int ci = q / 6, a = q - 6 * ci;
    const int j0 = S.img.cdiag0[ci], nj = S.img.cdiagn[ci];
    double acc = 0.0;
    for (int j = 0; j < nj; j += 8) {  // eight partials' loads in flight, added in item order
      double v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = bp[6 * (j0 + min(j + k, nj - 1)) + a];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (j + k < nj) acc += v[k];
    }
    if (kGroup) (&S.pose_n[0][0])[6 * S.img.acid[ci] + a] = acc;
    else A.slab_b[6l * S.cpos[S.img.acid[ci]] + a] = acc;
  }
}

// The one-wave K1 (wave plans, seg_obs == 1): one wave per chunk, NW chunks of one first-camera
// group per segment = workgroup (the plan's seg_chunks; chunk = segment * NW + wave, padded with
// empty chunks).  NW == 1: each item's block goes straight to its slab row.  NW > 1: the waves
// run on their own LDS images without waiting on each other, leave their blocks in their scratch
// rows, and after one workgroup barrier the segment's slots are summed over its chunks in chunk
// order into one slab row each (fewer rows for K2: one per segment slot, not per chunk slot).
static_assert(sizeof(LinWave::pose_n) >= kSegCams * 6 * sizeof(double), "the chunk's b sums fit pose_n");
template <int MODE, bool kStamp, int NW>
__global__ __launch_bounds__(kLinLanesWave * NW) void ba_lin_wave_kernel(LinArgs A) {
  constexpr bool kGroup = NW > 1;
  __shared__ LinWave Sw[NW];
  static_assert(kLinLanesWave == 64, "one wave");
  const int wv = kGroup ? __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6) : 0;
  LinWave& S = Sw[wv];
  const int seg = blockIdx.x, tid = (int)threadIdx.x & 63, chk = seg * NW + wv;
  Stamper<kStamp> st;
  st.start(tid == 0, chk);
  // level 1: status, segment header (uniform), this lane's camera ids (fixed header offsets)
  // and the chunk's image (chunk = segment)
  const int* SH = A.seg_hdr + (long)kSegHdr * seg;
  const int4* SH4 = reinterpret_cast<const int4*>(SH);
  const int16_t* SH16 = reinterpret_cast<const int16_t*>(SH);
  const int stat = A.status ? *A.status : 0;
  const int4 g0 = SH4[0], g1 = SH4[1];
  // this wave's chunk header: the segment header's copy (one chunk per segment), or its own
  const int4* CH = kGroup ? A.chunk_hdr + 4l * chk : SH4 + 8;
  const int4 h0 = CH[0], h1 = CH[1], h2 = CH[2], h3 = CH[3];
  constexpr int kImgVec = (int)(sizeof(ChunkImg) / 16);
  static_assert(kImgVec > 128 && kImgVec <= 192, "three 16-byte staging granules per lane");
  const uint4* img = reinterpret_cast<const uint4*>(A.chunk_img + chk);
  const uint4 img0 = img[tid], img1 = img[64 + tid], img2 = img[min(128 + tid, kImgVec - 1)];
  int i_acam[3], i_wcam[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    i_acam[k] = SH16[16 + min((tid + 64 * k) / 12, kSegAllCams - 1)];
    i_wcam[k] = SH16[32 + min((tid + 64 * k) / 6, kSegCams - 1)];
  }
  if (stat) return;  // a previous solve failed: state frozen
  const int nslots = g0.x, slot_off = g0.y, cam0 = g0.z, ncams = g0.w, na = g1.x;
  const int nob = h0.y, nte = h0.w, p0 = h1.x, npt = h1.y;
  double* dcw = &S.zb[kZbDc];
  double* pose_o = &S.zb[kZbPoseO];
  // level 2: landmarks, poses, pending update, slab rows
  double vx[2], vpn[3], vpo[3], vdc[3];
  const long xb = npt > 0 ? 3l * p0 : 0;  // an empty (padding) chunk may start past the last landmark
#pragma unroll
  for (int k = 0; k < 2; ++k) vx[k] = A.points[xb + min(tid + 64 * k, max(3 * npt - 1, 0))];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int e = tid + 64 * k;
    vpn[k] = A.pose_new[12l * i_acam[k] + e % 12];
    if (MODE & kBacksub) {
      vpo[k] = A.pose_old[12l * i_acam[k] + e % 12];
      vdc[k] = A.dc[6l * i_wcam[k] + e % 6];
    }
  }
  int vsp = 0, vcp = 0;
  if ((MODE & kAccum) && nslots > 0) {
    vsp = A.slab_pos[slot_off + min(tid, nslots - 1)];
    vcp = A.cam_pos[cam0 + min(tid, max(ncams - 1, 0))];
  }
  {
    uint4* d = reinterpret_cast<uint4*>(&S.img);
    d[tid] = img0;
    d[64 + tid] = img1;
    if (128 + tid < kImgVec) d[128 + tid] = img2;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k)
    if (tid + 64 * k < 3 * npt) (&S.X[0][0])[tid + 64 * k] = vx[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int e = tid + 64 * k;
    if (e < 12 * na) {
      (&S.pose_n[0][0])[e] = vpn[k];
      if (MODE & kBacksub) pose_o[e] = vpo[k];
    }
    if ((MODE & kBacksub) && e < 6 * ncams) dcw[e] = vdc[k];
  }
  if (MODE & kAccum) {
    if (tid < nslots) S.spos[tid] = vsp;
    if (tid < ncams) S.cpos[tid] = vcp;
    if (kGroup) {
      S.srow[tid] = 0xFF;
      if (tid < kSegCams) S.crow[tid] = 0;
    }
  }
  st.count(kPhSlots, nslots);
  st.count(kPhCams, ncams);
  st.count(kPhObs, nob);
  st.count(kPhTe, nte);
  st.count(kPhPts, npt);
  st.count(kPhPairs, h2.y - h2.x);
  double cost = 0.0;
  lds_sync_wave();
  st.mark(kPhLoad);

  if (MODE & kBacksub) {
    // the pending step at its linearisation point: r + Jc dc and Jp per observation, then
    // dp = -V^-1 sum Jp^T (r + Jc dc) per landmark (chunk_backsub)
    if (tid < nob) {
      const int lc = S.img.obs_lcam[tid];
      obs_lin_w<false, true>(S, A, &pose_o[12 * S.img.acam[tid]], tid, lc >= 0 ? &dcw[6 * lc] : nullptr, cost);
    }
    lds_sync_wave();
    if (tid < npt) {
      double l[6], h[3];
      if (point_block_w(S, A.lambda, tid, l, h)) {
        const double x2 = -h[2] * l[5];
        const double x1 = (-h[1] - l[4] * x2) * l[2];
        const double x0 = (-h[0] - l[1] * x1 - l[3] * x2) * l[0];
        S.X[tid][0] += x0;
        S.X[tid][1] += x1;
        S.X[tid][2] += x2;
        A.points[3l * (p0 + tid)] = S.X[tid][0];
        A.points[3l * (p0 + tid) + 1] = S.X[tid][1];
        A.points[3l * (p0 + tid) + 2] = S.X[tid][2];
      }
    }
    lds_sync_wave();
    st.mark(kPhBacksub);
  }

  // residuals and Jacobians at the current linearisation point (cost at the updated state)
  if (tid < nob) obs_lin_w<(MODE & kAccum) != 0, false>(S, A, S.pose_n[S.img.acam[tid]], tid, nullptr, cost);
  if (MODE & kAccum) {
    lds_sync_wave();
    st.mark(kPhLinObs);
    // per landmark: V (+lambda), its pivot-tested Cholesky and h = L^-1 g
    if (tid < npt) {
      double l[6], h[3];
      const bool ok = point_block_w(S, A.lambda, tid, l, h);
      S.valid[tid] = ok;
#pragma unroll
      for (int e = 0; e < 6; ++e) S.L[tid][e] = l[e];
      S.h[tid][0] = ok ? h[0] : 0.0;
      S.h[tid][1] = ok ? h[1] : 0.0;
      S.h[tid][2] = ok ? h[2] : 0.0;
    }
    lds_sync_wave();
    st.mark(kPhReduce);
    // per track entry: W = Jc^T Jp, gc = Jc^T r over its observations, then Z = W L^-T and
    // bt = -gc + Z h (zero, and the observations' Jc zeroed, for a frozen landmark or a
    // fixed camera); Z | bt overwrite the Jp | r every lane has read
    {
      double W[18], g[6];
#pragma unroll
      for (int e = 0; e < 18; ++e) W[e] = 0.0;
#pragma unroll
      for (int e = 0; e < 6; ++e) g[e] = 0.0;
      const int t = min(tid, max(nte - 1, 0));
      const bool live = tid < nte;
      const int oa = S.img.te_obs[t], ob = live ? S.img.te_obs[t + 1] : oa;
      for (int o = oa; o < ob; ++o) {
        double jj[12];
        jc_load(S, o, jj);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const double rk = S.zb[kZbR + 2 * o + k];
          const double q0 = S.zb[6 * o + 3 * k], q1 = S.zb[6 * o + 3 * k + 1], q2 = S.zb[6 * o + 3 * k + 2];
#pragma unroll
          for (int a = 0; a < 6; ++a) {
            const double jc = jj[6 * k + a];
            W[3 * a] += jc * q0;
            W[3 * a + 1] += jc * q1;
            W[3 * a + 2] += jc * q2;
            g[a] += jc * rk;
          }
        }
      }
      const int p = S.img.te_pt[t];
      const bool use = live && S.valid[p] && S.img.te_lcam[t] >= 0;
      const double i00 = S.L[p][0], l10 = S.L[p][1], i11 = S.L[p][2];
      const double l20 = S.L[p][3], l21 = S.L[p][4], i22 = S.L[p][5];
      const double hh0 = S.h[p][0], hh1 = S.h[p][1], hh2 = S.h[p][2];
      double bt[6];
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        const double z0 = W[3 * a] * i00;
        const double z1 = (W[3 * a + 1] - l10 * z0) * i11;
        const double z2 = (W[3 * a + 2] - l20 * z0 - l21 * z1) * i22;
        W[3 * a] = use ? z0 : 0.0;
        W[3 * a + 1] = use ? z1 : 0.0;
        W[3 * a + 2] = use ? z2 : 0.0;
        bt[a] = use ? -g[a] + (z0 * hh0 + z1 * hh1 + z2 * hh2) : 0.0;
      }
      if (live && !use)  // frozen landmark: its observations leave U too
        for (int o = oa; o < ob; ++o)
#pragma unroll
          for (int e = 0; e < 10; ++e) S.Jc[o][e] = 0.0;
      lds_sync_wave();  // every lane has read its Jp | r
      if (live) {
        double2* zr = reinterpret_cast<double2*>(&S.zb[kZbStride * t]);
#pragma unroll
        for (int e = 0; e < 9; ++e) zr[e] = make_double2(W[2 * e], W[2 * e + 1]);
        double2* br = reinterpret_cast<double2*>(S.bt[t]);
#pragma unroll
        for (int e = 0; e < 3; ++e) br[e] = make_double2(bt[2 * e], bt[2 * e + 1]);
      }
    }
    lds_sync_wave();
    st.mark(kPhElim);

    // Schur items: lane j sums active slot j's whole block (copies of a heavy slot balance
    // the lanes, each its own slab row); then the rhs by camera-row lanes
    {
      const int nas = h3.z;
      for (int j = tid; j - tid < nas; j += kLinLanesWave)
        schur_block<kGroup>(S, A, min(j, nas - 1), j < nas, st);
      lds_sync_wave();  // the copies' blocks and the diagonal items' b partials
      for (int j = tid; j - tid < nas; j += kLinLanesWave) copy_rows<kGroup>(S, A, min(j, nas - 1), j < nas);
      rhs_rows<kGroup>(S, A, h3.w, tid);
      if (kGroup) {  // where the combine finds this chunk's blocks (nas <= kWaveItems < 64 lanes)
        if (tid < nas && S.img.acopy[tid] == 0) S.srow[S.img.aslot[tid]] = (uint8_t)tid;
        if (tid < h3.w) S.crow[S.img.acid[tid]] = 1;
      }
    }
    st.mark(kPhWrite);  // stamped builds: the rhs (with the final write below)
  }  // kAccum
  // chunk cost: a fixed xor butterfly over the wave (deterministic)
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) cost += __shfl_xor(cost, m, 64);
  if (!kGroup) {
    if (tid == 0) A.slab_cost[seg] = cost;
  } else {
    if (tid == 0) S.wcost = cost;
    __syncthreads();  // every wave's blocks, b sums, maps and cost
    const int t = (int)threadIdx.x;
    if (MODE & kAccum) {
      // segment slot s, entry i: the chunks' blocks in chunk order (only the chunks that have it)
      for (int e = t; e < nslots * 36; e += 64 * NW) {
        const int s = e / 36, i = e - 36 * s;
        double acc = 0.0;
        bool any = false;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const int r = Sw[w].srow[s];
          const double v = (&Sw[w].Jc[0][0])[36 * (r == 0xFF ? 0 : r) + i];
          acc = r == 0xFF ? acc : any ? acc + v : v;
          any = any || r != 0xFF;
        }
        A.slab[36l * S.spos[s] + i] = acc;
      }
      for (int e = t; e < ncams * 6; e += 64 * NW) {
        const int c = e / 6;
        double acc = 0.0;
        bool any = false;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const bool on = Sw[w].crow[c] != 0;
          const double v = (&Sw[w].pose_n[0][0])[e];
          acc = !on ? acc : any ? acc + v : v;
          any = any || on;
        }
        A.slab_b[6l * S.cpos[c] + (e - 6 * c)] = acc;
      }
    }
    if (t == 0) {
      double c = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) c += Sw[w].wcost;
      A.slab_cost[seg] = c;
    }
  }
  st.mark(kPhWrite);
  st.flush(A.stamps);
}

// K2: fixed-order reduction of the slabs into [S profile | b | cost] (ReduceArgs, sum_rows:
// ba_reduce.h).

// One workgroup per profile block: 14 strided partial sums per S entry (16-byte loads) and, on
// a diagonal block, 42 per rhs entry of that camera, combined in fixed order (the result is
// bitwise reproducible).  The last workgroup sums the cost.  Every load of a
// workgroup is issued before the status test (a failed earlier step: nothing is written).
__global__ __launch_bounds__(kRedThreads) void ba_reduce_kernel(ReduceArgs A) {
  __shared__ __attribute__((aligned(16))) double part[kRedSParts * 36];
  __shared__ double partb[kRedBParts * 6];
  const int blk = blockIdx.x, tid = threadIdx.x;
  if (blk < A.nprof) {
    const int4 m = A.meta[blk];
    const int2 o = A.out[blk];
    const int failed = A.status ? *A.status : 0;
    const bool diag = m.z >= 0;
    double2 ps = make_double2(0.0, 0.0);
    double pb = 0.0;
    if (tid < kRedSParts * 18) ps = sum_rows2(A.slab, m.x, m.y, tid / 18, kRedSParts, tid % 18);
    if (diag && tid < kRedBParts * 6) pb = sum_rows<6>(A.slab_b, m.z, m.w, tid / 6, kRedBParts, tid % 6);
    if (failed) return;  // uniform
    if (tid < kRedSParts * 18) reinterpret_cast<double2*>(part)[tid] = ps;
    if (tid < kRedBParts * 6) partb[tid] = pb;
    __syncthreads();
    if (tid < 36) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < kRedSParts; ++q) acc += part[36 * q + tid];
      if (diag && tid % 7 == 0) acc += A.lambda;
      A.sys[(o.x & ~kRedTranspose) + ((o.x & kRedTranspose) ? 6 * (tid % 6) + tid / 6 : tid)] = acc;
    } else if (diag && tid >= 64 && tid < 70) {  // another wave: the rhs sum beside the S sum
      const int e = tid - 64;
      double acc = 0.0;
      for (int q = 0; q < kRedBParts; ++q) acc += partb[6 * q + e];
      A.sys[o.y + e] = acc;
    }
    return;
  }
  // cost: fixed-order lane-strided partial sums, then a fixed tree over the 256 lanes
  double c = 0.0;
  if (A.nseg > 0) {  // lane-strided, in order, every load of a batch in flight (sum_rows)
    for (int s = tid; s < A.nseg; s += 4 * kRedThreads) {
      double v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = A.slab_cost[min(s + i * kRedThreads, A.nseg - 1)];
#pragma unroll
      for (int i = 0; i < 4; ++i) c += s + i * kRedThreads < A.nseg ? v[i] : 0.0;
    }
  }
  if (A.status && *A.status) return;
  __shared__ double cpart[kRedThreads];
  cpart[tid] = c;
  __syncthreads();
  for (int m = kRedThreads / 2; m > 0; m >>= 1) {
    if (tid < m) cpart[tid] += cpart[tid + m];
    __syncthreads();
  }
  if (tid == 0) A.sys[A.cost_off] = cpart[0];
}

// K3: profile Cholesky solve S dc = b + pose update.
struct SolveArgs {
  int F, nprof, n_poses, n_fixed, iter_tag;
  int max_panel, max_row_span;  // most panel blocks in a column; max k - first[k]
  long lds_kf, lds_y, lds_panel, lds_pose, lds_tab;  // LDS offsets in doubles (solve_lds_layout)
  SolveTableLayout tl;
  const int* tab;      // BAPlan::solve_tab
  double* cost_out;    // if set: receives the cost of this linearisation (sys tail)
  double* sys;         // [S profile | b | cost]; factorised in place on the global path
  double* dc;          // 6F out
  const double* pose_cur;
  double* pose_next;
  int* status;
  unsigned long long* stamps;  // diagnostic build only
};



// K3.  Right-looking 6x6-block Cholesky of the profile of S with the forward
// substitution folded in, then back substitution and the pose update; one
// workgroup of four waves, one barrier per block column k:
//   every wave   reads D_k, factors it in registers (L_kk, 1/diag) and computes the
//                WHOLE panel L_ik = S_ik L_kk^-T (one lane per row) into its own
//                private LDS copy -- so the trailing update below needs no barrier;
//   trailing     S_ij -= L_ik L_jk^T over the panel's lower block triangle (this
//                includes D_{k+1}), one lane per (block, row), rows interleaved over
//                the waves, each reading only its own wave's panel copy;
//   wave 1       y_i -= L_ik y'_k with y'_k = L_kk^-1 y_k;
//   wave 2       keeps L_kk, 1/diag and y'_k for the back substitution;
//   wave 3       (next column) writes the panel into the profile blocks (i, k).
// The per-column panel rows and trailing blocks come from the host-built step
// table (BAPlan::solve_tab), staged in LDS with the profile.
enum { kS3Setup = 0, kS3Factor, kS3Backsub, kS3Tail, kS3Data, kS3Chol, kS3Panel, kS3Trail, kS3Barrier, kS3Mid, kS3Count };

// dst[i] = src[i], i < n: U loads in flight per thread.  Loads and stores are
// unconditional with a clamped index (an out-of-range slot rewrites dst[n-1] with
// src[n-1]): a predicated load is sunk into its store's branch and serialises.
template <typename T, int U>
__device__ __forceinline__ void copy_in(T* dst, const T* __restrict__ src, int n, int tid, int nthr) {
  if (n <= 0) return;
  for (int e = tid; e < n; e += U * nthr) {
    T a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = src[min(e + u * nthr, n - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) dst[min(e + u * nthr, n - 1)] = a[u];
  }
}

struct SolveLds {
  size_t prof, kf, y, panel, pose, tab, total;
};
// LDS image: [profile 36*nprof (LDS path)] [per column: L 21 + pad 3 | r 6 | y'/x 6]
// [y 6F] [4 private panels, 36 doubles per block] [step table ints]
SolveLds solve_lds_layout(bool lds_profile, int nprof, int F, int max_panel, int tab_len,
                          int n_poses) {
  SolveLds L;
  L.prof = 0;
  L.kf = lds_profile ? 36ull * nprof : 0;
  L.y = L.kf + 36ull * F;
  L.panel = L.y + 6ull * F;
  L.pose = L.panel + 4ull * 36 * std::max(1, max_panel);
  L.tab = L.pose + 12ull * n_poses;
  L.total = L.tab * 8 + 4ull * std::max(1, tab_len);
  return L;
}

template <bool kLds, bool kStamp, int NW>
__global__ __launch_bounds__(64 * NW) void ba_solve_kernel(SolveArgs A) {
  constexpr int kThr = 64 * NW;
  constexpr int wY = NW > 1 ? 1 : 0, wK = NW > 2 ? 2 : NW - 1, wC = NW - 1;  // role waves
  unsigned long long st_t = 0, st_acc[kS3Count] = {};
  auto mark = [&](int ph) {
    if (kStamp && threadIdx.x == 0) {
      const unsigned long long n = __builtin_amdgcn_s_memtime();
      if (st_t) st_acc[ph] += n - st_t;
      st_t = n;
    }
  };
  mark(0);
  // stamped build only: wait for outstanding LDS / a VALU result before a stamp
  auto settle = [&](double v) {
    if (kStamp) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      (void)__builtin_amdgcn_readfirstlane(__double2hiint(v));
    }
  };
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  __shared__ int s_fail;
  const int tid = threadIdx.x, F = A.F;
  const int wave = tid >> 6, lane = tid & 63;
  const bool prior_fail = A.status && *A.status;
  double* Sm = kLds ? dyn : A.sys;
  double* kf = dyn + A.lds_kf;       // 36 per column
  double* y = dyn + A.lds_y;         // 6F
  double* Pw = dyn + A.lds_panel + 36l * A.max_panel * wave;  // this wave's panel copy
  int* tab = reinterpret_cast<int*>(dyn + A.lds_tab);
  const int* t_diag = tab + A.tl.diag;
  const int* t_off = tab + A.tl.off;
  const int* t_first = tab + A.tl.first;
  const int* t_sptr = tab + A.tl.step_ptr;
  const int* t_pi = tab + A.tl.panel_i;
  const int* t_pblk = tab + A.tl.panel_blk;
  const int* t_iptr = tab + A.tl.item_ptr;
  const int* t_iblk = tab + A.tl.item_blk;
  const int* t_iq = tab + A.tl.item_q;
  if (tid == 0) {
    s_fail = prior_fail ? 1 : 0;
    if (A.cost_out) *A.cost_out = A.sys[36l * A.nprof + 6l * F];
  }
  if (!prior_fail) {
    // global -> LDS, every load of a batch in flight before the stores
    if (kLds) copy_in<double2, 16>(reinterpret_cast<double2*>(Sm), reinterpret_cast<const double2*>(A.sys),
                                   18 * A.nprof, tid, kThr);
    copy_in<double, 4>(y, A.sys + 36l * A.nprof, 6 * F, tid, kThr);
    copy_in<int, 8>(tab, A.tab, A.tl.len, tid, kThr);
  }
  double* pose_l = dyn + A.lds_pose;  // current poses, staged early for the tail
  copy_in<double, 4>(pose_l, A.pose_cur, 12 * A.n_poses, tid, kThr);
  __syncthreads();
  mark(kS3Setup);

  auto ld6 = [](const double* p, double (&v)[6]) {
    const double2* q = reinterpret_cast<const double2*>(p);
    const double2 a0 = q[0], a1 = q[1], a2 = q[2];
    v[0] = a0.x; v[1] = a0.y; v[2] = a1.x; v[3] = a1.y; v[4] = a2.x; v[5] = a2.y;
  };
  auto st6 = [](double* p, const double (&v)[6]) {
    double2* q = reinterpret_cast<double2*>(p);
    q[0] = make_double2(v[0], v[1]);
    q[1] = make_double2(v[2], v[3]);
    q[2] = make_double2(v[4], v[5]);
  };
  auto dot6 = [](const double (&u)[6], const double* w) {
    const double2* q = reinterpret_cast<const double2*>(w);
    const double2 a0 = q[0], a1 = q[1], a2 = q[2];
    return u[0] * a0.x + u[1] * a0.y + u[2] * a1.x + u[3] * a1.y + u[4] * a2.x + u[5] * a2.y;
  };

  // Per-column descriptors from the static step table, loaded one column ahead so
  // that after each barrier only the data loads (one LDS round trip) precede chol6.
  struct Desc {
    int p0, nb, i0, nt, diag, pblk, pi, blk0, q0;
  };
  const int tfi = lane * NW + wave;  // this lane's first trailing (block, row) item
  auto desc1 = [&](int k, Desc& d) {
    d.p0 = t_sptr[k];
    d.nb = t_sptr[k + 1] - d.p0;
    d.i0 = t_iptr[k];
    d.nt = 6 * (t_iptr[k + 1] - d.i0);
    d.diag = t_diag[k];
  };
  auto desc2 = [&](Desc& d) {
    d.pblk = d.pi = d.blk0 = d.q0 = 0;
    if (lane < 6 * d.nb) {
      d.pblk = t_pblk[d.p0 + lane / 6];
      d.pi = t_pi[d.p0 + lane / 6];
    }
    if (tfi < d.nt) {
      d.blk0 = t_iblk[d.i0 + tfi / 6];
      d.q0 = t_iq[d.i0 + tfi / 6];
    }
  };
  Desc cur{}, nxt{};
  if (F > 0 && !prior_fail) {
    desc1(0, cur);
    desc2(cur);
  }
  bool bad = false;
  bool prev_row = false;
  int prev_blk = 0, prev_p0 = 0, prev_nb = 0;
  double sv[6] = {0, 0, 0, 0, 0, 0};
  for (int k = 0; k < F && !prior_fail; ++k) {
    // wave 3: its previous panel row (still in registers) -> profile block (i, k-1), for
    // the back substitution; nobody touches blocks (i, k-1) from column k on
    if (wave == wC) {
      if (prev_row) st6(Sm + 36l * prev_blk + 6 * (lane % 6), sv);
      for (int r = lane + 64; r < 6 * prev_nb; r += 64) {
        double v[6];
        ld6(Pw + 6 * r, v);
        st6(Sm + 36l * t_pblk[prev_p0 + r / 6] + 6 * (r % 6), v);
      }
    }
    // data loads of column k
    double L[21], r[6], yk[6], s0[6];
    {
      const double* D = Sm + 36l * cur.diag;
      double dr[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        ld6(D + 6 * i, dr);
#pragma unroll
        for (int c = 0; c <= i; ++c) L[P6(i, c)] = dr[c];
      }
    }
    ld6(y + 6 * k, yk);
    const bool prow = lane < 6 * cur.nb;
    if (prow) ld6(Sm + 36l * cur.pblk + 6 * (lane % 6), sv);
    if (tfi < cur.nt) ld6(Sm + 36l * cur.blk0 + 6 * (tfi % 6), s0);
    if (k + 1 < F) desc1(k + 1, nxt);
    settle(L[0] + sv[0] + s0[0] + yk[0]);
    mark(kS3Data);
    const bool ok = chol6(L, r);
    settle(r[5]);
    mark(kS3Chol);
    if (wave == wY || wave == wK) fwd6(L, r, yk);  // y'_k: wave 1 updates y, wave 2 keeps it
    if (wave == wK && lane == 0)
      bad = bad || !ok || !isfinite(yk[0] + yk[1] + yk[2] + yk[3] + yk[4] + yk[5]);
    // panel (every wave, its own copy); wave 1 also updates y
    if (prow) {
      fwd6(L, r, sv);
      st6(Pw + 6 * lane, sv);
      if (wave == wY) y[6 * cur.pi + lane % 6] -= sv[0] * yk[0] + sv[1] * yk[1] + sv[2] * yk[2] +
                                                 sv[3] * yk[3] + sv[4] * yk[4] + sv[5] * yk[5];
    }
    for (int rr = lane + 64; rr < 6 * cur.nb; rr += 64) {  // panels wider than 10 blocks
      double v[6];
      ld6(Sm + 36l * t_pblk[cur.p0 + rr / 6] + 6 * (rr % 6), v);
      fwd6(L, r, v);
      st6(Pw + 6 * rr, v);
      if (wave == wY) y[6 * t_pi[cur.p0 + rr / 6] + rr % 6] -= v[0] * yk[0] + v[1] * yk[1] + v[2] * yk[2] +
                                                               v[3] * yk[3] + v[4] * yk[4] + v[5] * yk[5];
    }
    if (wave == wK && lane == 0) {
      double* o = kf + 36l * k;
#pragma unroll
      for (int e = 0; e < 20; e += 2) reinterpret_cast<double2*>(o)[e / 2] = make_double2(L[e], L[e + 1]);
      reinterpret_cast<double2*>(o)[10] = make_double2(L[20], 0.0);
      st6(o + 24, r);
      st6(o + 30, yk);
    }
    wave_sync<true>();
    settle(sv[5]);
    mark(kS3Panel);
    // trailing update from this wave's panel copy
    for (int t = tfi; t < cur.nt; t += kThr) {
      double s[6];
      int blk, q;
      if (t == tfi) {
#pragma unroll
        for (int c = 0; c < 6; ++c) s[c] = s0[c];
        blk = cur.blk0;
        q = cur.q0;
      } else {
        blk = t_iblk[cur.i0 + t / 6];
        q = t_iq[cur.i0 + t / 6];
        ld6(Sm + 36l * blk + 6 * (t % 6), s);
      }
      const int rr = t % 6;
      double a[6];
      ld6(Pw + 36 * (q & 0xffff) + 6 * rr, a);
      const double* B = Pw + 36 * (q >> 16);
#pragma unroll
      for (int c = 0; c < 6; ++c) s[c] -= dot6(a, B + 6 * c);
      st6(Sm + 36l * blk + 6 * rr, s);
    }
    settle(0.0);
    mark(kS3Trail);
    if (k + 1 < F) desc2(nxt);  // static table: its latency hides in the barrier wait
    prev_row = prow;
    prev_blk = cur.pblk;
    prev_p0 = cur.p0;
    prev_nb = cur.nb;
    cur = nxt;
    __syncthreads();
    mark(kS3Barrier);
  }
  if (wave == wK && lane == 0 && bad) s_fail = 1;
  __syncthreads();
  mark(kS3Factor);
  // Back substitution L^T x = y' on wave 0.
  if (!s_fail && wave == 0) {
    if (A.max_row_span < kBsWindow) {
      // Register-resident form (every row of L spans < kBsWindow blocks).  Lane
      // (g, c), g < kBsWindow, c < 6, accumulates component c of y'_j for the one block
      // row j = g (mod kBsWindow) inside the window [k - kBsWindow, k - 1] of step k.
      // Step k: y_k (group k mod W) -> 12 readlanes -> x_k = L_kk^-T y_k in every lane
      // -> each lane subtracts (L_kj^T x_k)_c for its j in row k.  L_kk, 1/diag, the
      // L_kj columns and the entering y'_{k-W} come from LDS one step ahead.
      constexpr int W = kBsWindow;
      const int g = lane / 6, c = lane % 6;
      const bool act = lane < 6 * W;
      auto jj_of = [&](int k) {  // block row of group g in the window of step k
        const int m = ((k - 1 - g) % W + W) % W;
        return k - 1 - m;
      };
      auto load_L = [&](int k, double (&Lk)[21], double (&rk)[6]) {
        const double* o = kf + 36l * k;
#pragma unroll
        for (int e2 = 0; e2 < 20; e2 += 2) {
          const double2 v = reinterpret_cast<const double2*>(o)[e2 / 2];
          Lk[e2] = v.x;
          Lk[e2 + 1] = v.y;
        }
        Lk[20] = o[20];
        ld6(o + 24, rk);
      };
      // column c of block (k, jj_of(k)) or 0; (fk, ok) = (first[k], off[k]) were read a step
      // earlier.  Loads are unconditional (clamped addresses, select afterwards): a load
      // under a branch makes the waitcnt pass drain every outstanding prefetch.
      auto load_col = [&](int k, int fk, int okk, double (&col)[6]) {
        const int jj = jj_of(k);
        const bool on = act && jj >= fk && jj < k;
        const double* b = Sm + 36l * (on ? okk + jj - fk : 0) + c;
#pragma unroll
        for (int rr = 0; rr < 6; ++rr) {
          const double v = b[6 * rr];
          col[rr] = on ? v : 0.0;
        }
      };
      double acc = 0.0;
      {
        const int jj = jj_of(F);
        if (act && jj >= 0) acc = kf[36l * jj + 30 + c];
      }
      // Two register sets used alternately (the loop is unrolled by two), so the
      // prefetched operands are never copied (each VALU op costs a wave 4 cycles).
      struct Ops {
        double L[21], r[6], col[6];
        int f, o;  // first[], off[] of the step after the one these operands serve
      };
      Ops s0, s1;
      load_L(F - 1, s0.L, s0.r);
      load_col(F - 1, t_first[F - 1], t_off[F - 1], s0.col);
      s0.f = t_first[F >= 2 ? F - 2 : 0];
      s0.o = t_off[F >= 2 ? F - 2 : 0];
      auto step = [&](int k, Ops& cur, Ops& nxt) {
        const int kn = k > 0 ? k - 1 : 0, kn2 = k > 1 ? k - 2 : 0;
        nxt.f = t_first[kn2];
        nxt.o = t_off[kn2];
        load_L(kn, nxt.L, nxt.r);
        load_col(kn, cur.f, cur.o, nxt.col);
        const int ent = k - W;  // block row entering the window of step k
        const double init_v = kf[36l * (ent >= 0 ? ent : 0) + 30 + c];
        const double init = ent >= 0 ? init_v : 0.0;
        const int src = 6 * (k % W);
        double x[6];
#pragma unroll
        for (int cc = 0; cc < 6; ++cc) {
          const int lo = __builtin_amdgcn_readlane(__double2loint(acc), src + cc);
          const int hi = __builtin_amdgcn_readlane(__double2hiint(acc), src + cc);
          x[cc] = __hiloint2double(hi, lo);
        }
        bwd6(cur.L, cur.r, x);
        if (lane == 0) st6(kf + 36l * k + 30, x);
        if (g == k % W) acc = init;
        acc -= cur.col[0] * x[0] + cur.col[1] * x[1] + cur.col[2] * x[2] + cur.col[3] * x[3] +
               cur.col[4] * x[4] + cur.col[5] * x[5];
      };
      int k = F - 1;
      for (; k >= 1; k -= 2) {
        step(k, s0, s1);
        step(k - 1, s1, s0);
      }
      if (k == 0) step(0, s0, s1);
    } else {
      // Wide rows: x_k, then y'_j -= L_kj^T x_k through LDS, one lane per (block, column).
      for (int k = F - 1; k >= 0; --k) {
        const double* o = kf + 36l * k;
        double Lk[21], rk[6], x[6];
#pragma unroll
        for (int e2 = 0; e2 < 20; e2 += 2) {
          const double2 v = reinterpret_cast<const double2*>(o)[e2 / 2];
          Lk[e2] = v.x;
          Lk[e2 + 1] = v.y;
        }
        Lk[20] = o[20];
        ld6(o + 24, rk);
        ld6(o + 30, x);
        bwd6(Lk, rk, x);
        const int fk = t_first[k], ok_ = t_off[k];
        wave_sync<true>();
        if (lane == 0) st6(kf + 36l * k + 30, x);
        for (int t = lane; t < 6 * (k - fk); t += 64) {
          const int jj = fk + t / 6, cc = t % 6;
          const double* Lkj = Sm + 36l * (ok_ + jj - fk);
          double a = 0.0;
#pragma unroll
          for (int rr = 0; rr < 6; ++rr) a += Lkj[6 * rr + cc] * x[rr];
          kf[36l * jj + 30 + cc] -= a;
        }
        wave_sync<true>();
      }
    }
  }
  __syncthreads();
  mark(kS3Backsub);
  const bool failed = s_fail != 0;
  for (int e = tid; e < 6 * F; e += kThr) A.dc[e] = failed ? 0.0 : kf[36l * (e / 6) + 30 + e % 6];
  for (int c = tid; c < A.n_poses; c += kThr) {
    const double* T = pose_l + 12 * c;
    double* out = A.pose_next + 12 * c;
    if (failed || c < A.n_fixed) {
      for (int e = 0; e < 12; ++e) out[e] = T[e];
    } else {
      const double* d6 = kf + 36l * (c - A.n_fixed) + 30;
      double d[6];
      for (int e = 0; e < 6; ++e) d[e] = d6[e];
      se3_exp_apply(d, T, out);
    }
  }
  if (tid == 0 && failed && !prior_fail) *A.status = A.iter_tag;
  mark(kS3Tail);
  if (kStamp && tid == 0 && A.stamps)
    for (int k = 0; k < kS3Count; ++k) A.stamps[k] = st_acc[k];
}


// Chunk images taken over from the previous plan: runs of consecutive chunks copied on the
// device by a kernel (hipMemcpyAsync device-to-device went through a copy engine at ~12 GB/s on
// some boxes: 0.36-0.45 ms for a slid cfg3 window's 3.5 MB).  The runs travel in the arguments.
constexpr int kImgRuns = 48;
struct ImgRuns {
  int n;                    // runs in this launch
  int src[kImgRuns], dst[kImgRuns], end[kImgRuns];  // run r: chunks [end[r-1], end[r]) of the launch
};
__global__ __launch_bounds__(64) void ba_img_copy_kernel(const uint4* __restrict__ prev, uint4* __restrict__ cur,
                                                          ImgRuns R) {
  constexpr int kVec = (int)(sizeof(ChunkImg) / 16);
  const int b = blockIdx.x;
  int r = 0;
  while (r + 1 < R.n && R.end[r] <= b) ++r;  // uniform
  const int off = b - (r ? R.end[r - 1] : 0);
  const uint4* s = prev + (long)(R.src[r] + off) * kVec;
  uint4* d = cur + (long)(R.dst[r] + off) * kVec;
  uint4 v[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) v[k] = s[min((int)threadIdx.x + 64 * k, kVec - 1)];
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if ((int)threadIdx.x + 64 * k < kVec) d[threadIdx.x + 64 * k] = v[k];
}
static_assert(sizeof(ChunkImg) / 16 <= 192, "three 16-byte pieces per lane");

template <class T, class A>
void upload(DevBuf& buf, const std::vector<T, A>& v, hipStream_t st) {
  buf.reserve(std::max<size_t>(v.size(), 1) * sizeof(T));
  if (!v.empty())
    VO_HIP_CHECK(hipMemcpyAsync(buf.ptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st));
}

constexpr size_t kSolveLdsMax = 160 * 1024 - 64;  // gfx950: 160 KiB per workgroup (+ s_fail)

std::atomic<uint64_t> g_ba_sessions{0};  // session ids, unique in the process

}  // namespace

class BAEngine {
 public:
  explicit BAEngine(vo_ctx* ctx) : ctx_(ctx) {}
  ~BAEngine() {
    if (h_state_ev_) {
      (void)hipEventSynchronize(h_state_ev_);
      (void)hipEventDestroy(h_state_ev_);
    }
  }

  // Returns the new session id.  Every argument and plan check completes before any
  // collective: with a communicator, all ranks then agree (min all-reduce of [ok, F, -F])
  // and fail together, so one rank's bad shard is an error everywhere, not a hang.
  uint64_t setup(const vo_ba_problem* prob) {
    PLAN_T_START();
    for (int64_t& v : setup_clock().ns) v = 0;
    // the previous setup's chunk-image DMA may still read the page-locked images the
    // planner is about to rewrite (a setup that failed after its upload returns unsynced)
    VO_HIP_CHECK(hipStreamSynchronize(ctx_->stream));
    PLAN_T(0, "setup: sync");
    have_problem_ = false;
    have_state_ = false;
    std::string err;
    if (!prob) err = "null problem";
    else if (!(prob->n_poses >= 1 && prob->n_points >= 0 && prob->n_obs >= 0)) err = "bad sizes";
    else if (!(prob->lambda >= 0.0)) err = "lambda must be >= 0";
    else if (!((prob->n_points == 0 || prob->point_ptr) && (prob->n_obs == 0 || (prob->obs_cam && prob->obs_uv))))
      err = "null arrays";
    else if (prob->n_points == 0 && prob->n_obs != 0) err = "observations without points";
    // the last plan whose images reached the device: the next window's plan takes over its
    // unchanged first-camera groups (ba_plan.h build_plan)
    const bool prev_ok = plan_ok_;
    plan_ok_ = false;
    if (err.empty()) {
      // K1 variant (a plan property, ba_plan.h plan_is_wave): the one-wave K1 at every size --
      // cfg4's 13.7k chunks run in nine rounds of six per CU, faster than the four-wave K1's one
      // round of two-chunk segments (148 against 222 us) -- with wave_chunks()
      // chunks per segment; the four-wave K1 over multi-chunk segments only under the testing
      // switch (vo_ba_testing_k1).  The packing target is a function of this window alone, so a
      // plan that takes groups over from the previous one is the plan a scratch setup builds
      // (take-over needs equal targets: build_plan checks).
      const bool wave = ctx_->ba_k1_variant >= 0;
      const int nw = wave ? wave_chunks(prob->n_obs) : 1;
      std::vector<int32_t> zero_ptr(1, 0);
      const int32_t* pp = prob->n_points ? prob->point_ptr : zero_ptr.data();
      std::swap(plan_, prev_plan_);
      d_chunk_img_.swap(d_chunk_img_prev_);
      const BAPlan* prev = prev_ok ? &prev_plan_ : nullptr;
      err = build_plan(plan_, prob->n_poses, prob->n_points, prob->n_obs, prob->n_fixed, pp, prob->obs_cam,
                       prob->obs_uv, seg_obs_grid(seg_obs_for(prob->n_obs, segments_target(ctx_->num_cus, wave))), prev,
                       nw);
      // six-chunk segments beyond one round (one workgroup per CU): plan with three
      if (err.empty() && wave && ctx_->ba_k1_variant == 0 && nw == kWaveChunksOneRound &&
          plan_.n_segments() > ctx_->num_cus)
        err = build_plan(plan_, prob->n_poses, prob->n_points, prob->n_obs, prob->n_fixed, pp, prob->obs_cam,
                         prob->obs_uv, seg_obs_grid(seg_obs_for(prob->n_obs, segments_target(ctx_->num_cus, wave))),
                         prev, kWaveChunksRounds);
      PLAN_T(4, "setup: returned");
      // four-wave K1: every first-camera group ends in a partial segment, so the packing target
      // may give more segments than one round holds; then pack once more, proportionally wider
      // (on the grid; a function of the plan, which does not depend on prev)
      const int round = segments_target(ctx_->num_cus, false);
      for (int k = 0; k < 4 && err.empty() && !plan_is_wave(plan_.seg_obs) && plan_.n_segments() > round; ++k) {
        const int so2 = seg_obs_grid((int64_t)plan_.seg_obs * plan_.n_segments() / round + 1);
        err = build_plan(plan_, prob->n_poses, prob->n_points, prob->n_obs, prob->n_fixed, pp, prob->obs_cam,
                         prob->obs_uv, so2, prev);
      }
    }
    if (ctx_->comm && ctx_->comm->nranks > 1) {
      const int32_t F = err.empty() ? plan_.n_free : 0;
      std::vector<int32_t> agree = {err.empty() ? 1 : 0, F, -F};
      DevBuf tmp;
      upload(tmp, agree, ctx_->stream);
      ctx_->comm->allreduce(tmp.as<int32_t>(), agree.size(), true, ctx_->stream);
      VO_HIP_CHECK(hipMemcpyAsync(agree.data(), tmp.ptr, agree.size() * 4, hipMemcpyDeviceToHost, ctx_->stream));
      VO_HIP_CHECK(hipStreamSynchronize(ctx_->stream));
      if (err.empty() && agree[0] == 0) err = "another rank's shard failed its checks";
      if (err.empty() && agree[1] != -agree[2]) err = "ranks disagree on the number of free poses";
    }
    VO_REQUIRE(err.empty(), VO_ERR_ARG, "vo_ba_setup: %s", err.c_str());
    PLAN_T(5, "setup: planned");
    // the largest plan array first: from page-locked memory the copy runs while the host
    // builds the profile and the K3 tables.  Images taken over from the previous plan are
    // copied on the device, in runs of consecutive chunks.
    {
      const BAPlan& P = plan_;
      const int nch = (int)P.chunk_img.size();
      d_chunk_img_.reserve(std::max(nch, 1) * sizeof(ChunkImg));
      ImgRuns R{};
      int copied = 0;
      auto flush = [&]() {
        if (R.n == 0) return;
        hipLaunchKernelGGL(ba_img_copy_kernel, dim3(copied), dim3(64), 0, ctx_->stream,
                           d_chunk_img_prev_.as<uint4>(), d_chunk_img_.as<uint4>(), R);
        VO_HIP_CHECK(hipGetLastError());
        R.n = 0;
        copied = 0;
      };
      for (int c0 = 0; c0 < nch;) {
        const int src = c0 < (int)P.chunk_src.size() ? P.chunk_src[c0] : -1;
        int c1 = c0 + 1;
        while (c1 < nch && (src < 0 ? P.chunk_src[c1] < 0 : P.chunk_src[c1] == src + (c1 - c0))) ++c1;
        if (src >= 0) {  // taken over: a run of the copy kernel
          if (R.n == kImgRuns) flush();
          R.src[R.n] = src;
          R.dst[R.n] = c0;
          copied += c1 - c0;
          R.end[R.n++] = copied;
        } else {  // built by this plan: from the page-locked images
          VO_HIP_CHECK(hipMemcpyAsync(d_chunk_img_.as<ChunkImg>() + c0, P.chunk_img.data() + c0,
                                      (size_t)(c1 - c0) * sizeof(ChunkImg), hipMemcpyHostToDevice, ctx_->stream));
        }
        c0 = c1;
      }
      flush();
      plan_ok_ = true;
    }
    PLAN_T(6, "setup: images");
    std::vector<int32_t> first = local_profile_first(plan_);
    if (ctx_->comm && ctx_->comm->nranks > 1 && !first.empty()) {
      DevBuf tmp;
      upload(tmp, first, ctx_->stream);
      ctx_->comm->allreduce(tmp.as<int32_t>(), first.size(), true, ctx_->stream);
      VO_HIP_CHECK(hipMemcpyAsync(first.data(), tmp.ptr, first.size() * 4, hipMemcpyDeviceToHost,
                                  ctx_->stream));
      VO_HIP_CHECK(hipStreamSynchronize(ctx_->stream));
    }
    // banded K3 when the block bandwidth and F fit it (decided on first[], before the
    // profile, whose step tables only the profile solver reads); the profile solver otherwise
    const int F = plan_.n_free;
    band_ = band_split(F, std::vector<int>(first.begin(), first.end()));
    band_on_ = F > 0 && band_supported(F, band_.w, plan_.n_poses);
    build_profile(plan_, first, !band_on_);
    PLAN_T(7, "setup: profile");
    prob_ = *prob;
    prob_.point_ptr = nullptr;
    prob_.obs_cam = nullptr;
    prob_.obs_uv = nullptr;

    hipStream_t st = ctx_->stream;
    const BAPlan& P = plan_;
    // the plan's small tables, placed in one device buffer and sent with one copy (below)
    TablePack pack;
    const size_t o_chunk_hdr = pack.add(P.chunk_hdr), o_slab_pos = pack.add(P.slab_pos),
                 o_cam_pos = pack.add(P.cam_pos), o_seg_hdr = pack.add(P.seg_hdr);
    size_t o_solve_tab = 0, o_band_tab = 0;
    PLAN_T(8, "setup: uploads");
    d_points_.reserve(std::max(1, P.n_points) * 24ull);
    d_pose_[0].reserve(P.n_poses * 96ull);
    d_pose_[1].reserve(P.n_poses * 96ull);
    d_dc_.reserve(std::max(1, F) * 48ull);
    d_slab_.reserve(std::max(1, P.n_slab_slots()) * 288ull);
    d_slab_b_.reserve(std::max<size_t>(1, P.segcam_f.size()) * 48ull);
    d_slab_cost_.reserve(std::max(1, P.n_segments()) * 8ull);
    d_linv_.reserve(std::max(1, F) * 288ull);
    if (!band_on_) {
      o_solve_tab = pack.add(P.solve_tab);
      const SolveTableLayout& TL = P.solve_layout;
      const SolveLds in_lds = solve_lds_layout(true, P.n_prof_blocks(), F, TL.max_panel, TL.len, P.n_poses);
      solve_lds_ = in_lds.total <= kSolveLdsMax;
      solve_layout_ = solve_lds_ ? in_lds : solve_lds_layout(false, P.n_prof_blocks(), F, TL.max_panel, TL.len, P.n_poses);
      VO_REQUIRE(solve_layout_.total <= kSolveLdsMax, VO_ERR_ARG,
                 "vo_ba_setup: %d free poses / panel of %d blocks exceed the solver's LDS budget", F,
                 TL.max_panel);
      solve_lds_size_ = solve_layout_.total;
    }
    PLAN_T(9, "setup: bufs");
    {
      // K2's output layout: the profile [S | b | cost], or the banded K3's columns
      const int nprof = P.n_prof_blocks();
      red_dst_.assign(std::max(1, nprof), 0);
      red_rdst_.assign(std::max(1, F), 0);
      size_t pad = 0;
      if (band_on_) {
        const int w = band_.w, CS = band_col_stride(w), top = band_.m + band_.s;
        const int base_b = top * CS;
        for (int i = 0; i < F; ++i) {
          for (int j = P.prof_first[i]; j <= i; ++j) {
            const int b = P.prof_off[i] + j - P.prof_first[i];
            red_dst_[b] = i < top ? j * CS + 36 * (i - j) : (base_b + (F - 1 - i) * CS + 36 * (i - j)) | kRedTranspose;
          }
          red_rdst_[i] = i < top ? i * CS + 36 * (w + 1) : base_b + (F - 1 - i) * CS + 36 * (w + 1);
        }
        sys_len_ = (size_t)(F + band_.s) * CS + 1;
        cost_off_ = (long)sys_len_ - 1;
        pad = band_slot_stride(w);  // the ring loader's last LDS-DMA piece reads past the end
        band_lds_ = band_lds_layout(F, band_, P.n_poses, !ctx_->ba_no_split);
        band_tab_ = band_tables(F, band_, band_lds_);
        o_band_tab = pack.add(band_tab_.tab);
        band_set_attributes(band_lds_);  // (a no-op unless the LDS size grows)
        if (!band_lds_.full || band_lds_.split) d_fac_.reserve(band_fac_doubles(F, w) * 8);
        if (band_lds_.split) {  // the split hand-offs' exchange area (front of fac); flags start clear
          const SplitXch x = split_xch(band_tab_.n_merge, band_.s);
          VO_REQUIRE((size_t)x.end() <= band_fac_doubles(F, w), VO_ERR_STATE, "band split: exchange area");
          VO_HIP_CHECK(hipMemsetAsync(d_fac_.as<double>() + x.flag, 0, 3 * 16 * sizeof(double), st));
        }
      } else {
        for (int b = 0; b < nprof; ++b) red_dst_[b] = 36 * b;
        for (int f = 0; f < F; ++f) red_rdst_[f] = 36 * nprof + 6 * f;
        sys_len_ = 36ull * nprof + 6ull * F + 1;
        cost_off_ = (long)sys_len_ - 1;
      }
      d_sys_.reserve((sys_len_ + pad) * 8);
      // entries K2 never writes (outside the profile, the bottom side's separator) stay 0
      VO_HIP_CHECK(hipMemsetAsync(d_sys_.ptr, 0, (sys_len_ + pad) * 8, st));
      // K2's per-block table: slab rows, the diagonal blocks' rhs entries, output offsets
      red_meta_.assign(std::max(1, nprof), int4{0, 0, -1, -1});
      red_out_.assign(std::max(1, nprof), int2{0, 0});
      for (int i = 0; i < F; ++i)
        for (int b = P.prof_off[i]; b < P.prof_off[i + 1]; ++b) {
          const bool diag = P.prof_diag[b] != 0;
          red_meta_[b] = int4{P.prof_src_ptr[b], P.prof_src_ptr[b + 1], diag ? P.camb_ptr[i] : -1,
                              diag ? P.camb_ptr[i + 1] : -1};
          red_out_[b] = int2{red_dst_[b], diag ? red_rdst_[i] : 0};
        }
      // the fused launch's readiness counters: the column each profile block's reducer stores
      // into (top columns j of rows i < m + s, then bottom column F - 1 - i at m + s + F - 1 - i),
      // the cost at F, and how many items each counter waits for
      red_col_.assign(std::max(1, nprof), 0);
      col_need_.assign(F + 1, 0);
      if (band_on_) {
        const int top = band_.m + band_.s;
        for (int i = 0; i < F; ++i)
          for (int b = P.prof_off[i]; b < P.prof_off[i + 1]; ++b) {
            const int j = P.prof_first[i] + (b - P.prof_off[i]);
            red_col_[b] = i < top ? j : top + (F - 1 - i);
            ++col_need_[red_col_[b]];
          }
        col_need_[F] = 1;  // the cost item
      }
      const size_t o_meta = pack.add(red_meta_), o_out = pack.add(red_out_), o_rcol = pack.add(red_col_),
                   o_need = pack.add(col_need_);
      // K2 fused into the banded K3's launch when every workgroup of it fits one round at
      // one per CU (the solver's LDS): cfg3's 356 blocks make 178 reducers + the solver on
      // MI355X's 256 CUs (fewer CUs, e.g. a partitioned device: K2 stays a launch of its own)
      // (full mode only: the ring-mode solver reads sys with plain loads, so it must come from an
      // earlier launch)
      fuse_ok_ = VO_BA_FUSE && band_on_ && band_lds_.full && !band_lds_.split &&
                 band_fused_workgroups(nprof) + 1 <= ctx_->num_cus;

      // one page-locked staging buffer, one device buffer, one copy (each table a pageable
      // copy of its own cost several µs of host time apiece); both are rewritten only after the
      // stream sync at the top of the next setup
      h_tab_.reserve(pack.bytes);
      d_tab_.reserve(pack.bytes);
      for (const TablePack::Part& q : pack.parts)
        if (q.n) std::memcpy(h_tab_.as<char>() + q.off, q.src, q.n);
      VO_HIP_CHECK(hipMemcpyAsync(d_tab_.ptr, h_tab_.ptr, pack.bytes, hipMemcpyHostToDevice, st));
      char* base = d_tab_.as<char>();
      d_chunk_hdr_.ptr = base + o_chunk_hdr;
      d_slab_pos_.ptr = base + o_slab_pos;
      d_cam_pos_.ptr = base + o_cam_pos;
      d_seg_hdr_.ptr = base + o_seg_hdr;
      d_solve_tab_.ptr = band_on_ ? nullptr : base + o_solve_tab;
      d_band_tab_.ptr = band_on_ ? base + o_band_tab : nullptr;
      d_red_meta_.ptr = base + o_meta;
      d_red_out_.ptr = base + o_out;
      d_red_col_.ptr = base + o_rcol;
      d_col_need_.ptr = base + o_need;
      // the status word, K2's fused-round counter and the zero block (masked prefetches)
      d_misc_.reserve(kMiscBytes);
      d_status_.ptr = d_misc_.ptr;
      d_zero_.ptr = d_misc_.as<char>() + 256;
      VO_HIP_CHECK(hipMemsetAsync(d_misc_.ptr, 0, kMiscBytes, st));
      colcnt_bytes_ = band_col_count_bytes(F);
      d_colcnt_.reserve(colcnt_bytes_);
      VO_HIP_CHECK(hipMemsetAsync(d_colcnt_.ptr, 0, colcnt_bytes_, st));
    }
    PLAN_T(10, "setup: band");
    if (!band_on_) {
      const int l = (int)solve_lds_size_;
      set_solve_lds<true>(l);
      set_solve_lds<false>(l);
    }
    PLAN_T(11, "setup: attrs");
    std::copy(setup_clock().ns, setup_clock().ns + kSetupSections, setup_ns_);
    // no sync: everything above is stream-ordered before the first iteration, pageable
    // sources are staged when their copy is issued, and the page-locked chunk images are
    // only rewritten after the sync at the top of the next setup
    have_problem_ = true;
    have_state_ = false;
    pending_ = false;
    cur_ = 0;
    session_ = ++g_ba_sessions;
    return session_;
  }

  // Pre-sizes what a window of about (n_poses, n_points, n_obs) needs, outside the keyframe
  // calls: both plan objects' host arrays (plan_ and prev_plan_ alternate between setups; the
  // page-locked chunk images included), every device buffer, the kernels' LDS attributes (the
  // first one also loads the library's code object) and the state staging buffer.  It sets a
  // synthetic window of that size up twice -- landmark p seen by a run of consecutive cameras,
  // the runs spread over the window -- and then drops it: the context has no problem after it,
  // and the next setup takes nothing over from it.  A later, larger window still grows what it
  // needs (every array keeps a quarter of headroom).
  void reserve(int n_poses, int n_points, int64_t n_obs, int n_fixed) {
    VO_REQUIRE(n_poses >= 2 && n_points >= 1 && n_obs >= 2 * (int64_t)n_points && n_obs <= INT32_MAX &&
                   n_fixed >= 0 && n_fixed < n_poses,
               VO_ERR_ARG, "vo_ba_reserve: bad sizes");
    VO_REQUIRE(!(ctx_->comm && ctx_->comm->nranks > 1), VO_ERR_STATE,
               "vo_ba_reserve: before vo_comm_init (a setup with a communicator is collective)");
    const int len0 = (int)std::min<int64_t>(n_poses, n_obs / n_points);
    const int64_t extra = std::min<int64_t>(n_obs - (int64_t)len0 * n_points, n_points);
    std::vector<int32_t> ptr(n_points + 1), cam;
    cam.reserve(n_obs);
    for (int p = 0; p < n_points; ++p) {
      const int len = std::min(n_poses, len0 + (p < extra ? 1 : 0));
      const int c0 = (int)((int64_t)p * (n_poses - len + 1) / n_points);
      for (int c = 0; c < len; ++c) cam.push_back(c0 + c);
      ptr[p + 1] = (int32_t)cam.size();
    }
    std::vector<float> uv(2 * cam.size(), 0.0f);
    vo_ba_problem pr{};
    pr.n_poses = n_poses;
    pr.n_points = n_points;
    pr.n_obs = (int32_t)cam.size();
    pr.n_fixed = n_fixed;
    pr.fx = pr.fy = 500.0;
    pr.lambda = 1.0;
    pr.point_ptr = ptr.data();
    pr.obs_cam = cam.data();
    pr.obs_uv = uv.data();
    for (int k = 0; k < 2; ++k) setup(&pr);
    h_state_.reserve((3ull * n_points + 12ull * n_poses) * 8);
    d_cost_.reserve(64 * 8);
    VO_HIP_CHECK(hipStreamSynchronize(ctx_->stream));
    plan_ok_ = false;  // nothing of the synthetic plan is taken over
    have_problem_ = false;
    have_state_ = false;
  }

  // The caller's session must be the engine's current problem (VO_ERR_STATE otherwise):
  // a later vo_ba_setup on the same context replaces it, and its sizes with it.
  void check_session(uint64_t s) const {
    VO_REQUIRE(have_problem_ && s == session_, VO_ERR_STATE,
               "BA session %llu is not this context's current problem (%llu): another vo_ba_setup replaced it",
               (unsigned long long)s, (unsigned long long)session_);
  }

  void set_state(const double* poses, const double* points) {
    VO_REQUIRE(have_problem_, VO_ERR_STATE, "vo_ba_set_state before vo_ba_setup");
    const BAPlan& P = plan_;
    hipStream_t st = ctx_->stream;
    // points gathered into internal order in the page-locked staging buffer, poses behind them
    const size_t np = 3ull * P.n_points;
    if (h_state_busy_) VO_HIP_CHECK(hipEventSynchronize(h_state_ev_));  // previous set_state's DMA
    h_state_busy_ = false;
    h_state_.reserve((np + 12ull * P.n_poses) * 8);
    double* pts = h_state_.as<double>();
    for (int q = 0; q < P.n_points; ++q)
      for (int e = 0; e < 3; ++e) pts[3ull * q + e] = points[3ull * P.pt_perm[q] + e];
    std::memcpy(pts + np, poses, P.n_poses * 96ull);
    VO_HIP_CHECK(hipMemcpyAsync(d_pose_[0].ptr, pts + np, P.n_poses * 96ull, hipMemcpyHostToDevice, st));
    if (P.n_points) VO_HIP_CHECK(hipMemcpyAsync(d_points_.ptr, pts, np * 8, hipMemcpyHostToDevice, st));
    // not synchronised here: the next writer of the staging buffer waits for this event
    if (!h_state_ev_) VO_HIP_CHECK(hipEventCreateWithFlags(&h_state_ev_, hipEventDisableTiming));
    VO_HIP_CHECK(hipEventRecord(h_state_ev_, st));
    h_state_busy_ = true;
    VO_HIP_CHECK(hipMemsetAsync(d_status_.ptr, 0, sizeof(int), st));
    if (fuse_ok_) VO_HIP_CHECK(hipMemsetAsync(d_colcnt_.ptr, 0, colcnt_bytes_, st));  // after a timed-out solve
    cur_ = 0;
    pending_ = false;
    have_state_ = true;
  }

  void get_state(double* poses, double* points) {
    require_state();
    finalize();
    const BAPlan& P = plan_;
    hipStream_t st = ctx_->stream;
    const size_t np = 3ull * P.n_points;
    if (h_state_busy_) VO_HIP_CHECK(hipEventSynchronize(h_state_ev_));  // before reserve() may free it
    h_state_busy_ = false;
    h_state_.reserve((np + 12ull * P.n_poses) * 8);
    double* pts = h_state_.as<double>();
    VO_HIP_CHECK(hipMemcpyAsync(pts + np, d_pose_[cur_].ptr, P.n_poses * 96ull, hipMemcpyDeviceToHost, st));
    if (P.n_points) VO_HIP_CHECK(hipMemcpyAsync(pts, d_points_.ptr, np * 8, hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipStreamSynchronize(st));
    std::memcpy(poses, pts + np, P.n_poses * 96ull);
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
    const bool timed_out = clear_timeout(status);
    if (status) {
      // iteration `status` (1-based) failed: the state is its linearisation point
      for (int k = status; k <= iters; ++k) costs[k] = NAN;
      VO_HIP_CHECK(hipMemsetAsync(d_status_.ptr, 0, sizeof(int), st));
      VO_HIP_CHECK(hipStreamSynchronize(st));
    }
    if (cost_out) std::copy(costs.begin(), costs.end(), cost_out);
    VO_REQUIRE(!timed_out, VO_ERR_HIP, "vo_ba_run: fused reduction timed out at iteration %d (a reducer workgroup never arrived)", status - 1);
    if (status) {
      set_error("vo_ba_run: reduced camera system not positive definite at iteration %d",
                status - 1);
      return VO_ERR_NOT_SPD;
    }
    return VO_OK;
  }

  // After a failed fused launch (any non-zero status; kBandStatusTimeout: the solver gave up
  // waiting for its reducers) the reducer counter is re-zeroed -- the stream is synchronised,
  // so every late reducer has counted itself by now -- and the timeout flag is stripped from
  // the status word's iteration.  Returns whether a timeout was recorded.
  bool clear_timeout(int& status) {
    if (status && fuse_ok_) VO_HIP_CHECK(hipMemsetAsync(d_colcnt_.ptr, 0, colcnt_bytes_, ctx_->stream));
    if (!(status & kBandStatusTimeout)) return false;
    status &= ~kBandStatusTimeout;
    return true;
  }

  int gn_step(double* S_out, double* b_out, double* dc_out, double* cost_out) {
    require_state();
    hipStream_t st = ctx_->stream;
    const BAPlan& P = plan_;
    const int F = P.n_free;
    d_cost_.reserve(8);
    enqueue_lin(pending_ ? (kBacksub | kAccum) : kAccum);
    enqueue_reduce();
    std::vector<double> sys(sys_len_);
    // the reduced system as K2 wrote it: before the solve (the profile solver factors it in
    // place), or after the fused K2 + K3 launch (the banded K3 only reads it)
    if (!fused()) VO_HIP_CHECK(hipMemcpyAsync(sys.data(), d_sys_.ptr, sys_len_ * 8, hipMemcpyDeviceToHost, st));
    enqueue_solve(1);
    if (fused()) VO_HIP_CHECK(hipMemcpyAsync(sys.data(), d_sys_.ptr, sys_len_ * 8, hipMemcpyDeviceToHost, st));
    std::vector<double> dc(6ull * F);
    int status = 0;
    if (F) VO_HIP_CHECK(hipMemcpyAsync(dc.data(), d_dc_.ptr, dc.size() * 8, hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipMemcpyAsync(&status, d_status_.ptr, sizeof(int), hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipStreamSynchronize(st));
    cur_ ^= 1;
    pending_ = true;
    if (S_out) {  // K2's output layout (red_dst_) back to the dense symmetric S
      const int n = 6 * F;
      std::fill(S_out, S_out + (size_t)n * n, 0.0);
      for (int i = 0; i < F; ++i)
        for (int j = P.prof_first[i]; j <= i; ++j) {
          const int d = red_dst_[P.prof_off[i] + j - P.prof_first[i]];
          const double* blk = sys.data() + (d & ~kRedTranspose);
          const bool tr = d & kRedTranspose;
          for (int r = 0; r < 6; ++r)
            for (int c = 0; c < 6; ++c) {
              const double v = blk[tr ? 6 * c + r : 6 * r + c];
              S_out[(size_t)(6 * i + r) * n + 6 * j + c] = v;
              S_out[(size_t)(6 * j + c) * n + 6 * i + r] = v;
            }
        }
    }
    if (b_out)
      for (int f = 0; f < F; ++f) std::copy(sys.begin() + red_rdst_[f], sys.begin() + red_rdst_[f] + 6, b_out + 6 * f);
    if (dc_out) std::copy(dc.begin(), dc.end(), dc_out);
    if (cost_out) *cost_out = sys[cost_off_];
    const bool timed_out = clear_timeout(status);
    if (status) {
      VO_HIP_CHECK(hipMemsetAsync(d_status_.ptr, 0, sizeof(int), st));
      VO_HIP_CHECK(hipStreamSynchronize(st));
      VO_REQUIRE(!timed_out, VO_ERR_HIP, "vo_ba_gn_step: fused reduction timed out (a reducer workgroup never arrived)");
      set_error("vo_ba_gn_step: reduced camera system not positive definite");
      return VO_ERR_NOT_SPD;
    }
    return VO_OK;
  }

  int stats(int64_t* out, int n) const {
    const BAPlan& P = plan_;
    int64_t v[12 + kSetupSections] = {P.n_chunks(), P.n_segments(), P.n_slab_slots(), (int64_t)P.slot_i.size(),
                                      P.n_prof_blocks(), P.n_te, P.algorithmic_bytes_per_iter(), band_on_ ? 1 : 0,
                                      P.reused_groups, P.reused_chunks, P.seg_obs};
    for (int i = 0; i < kSetupSections; ++i) v[11 + i] = setup_ns_[i];  // the last setup's sections
    // the banded K3's layout: 0 none (profile solver), 1 full, 2 ring, 3 split (two workgroups)
    v[11 + kSetupSections] = !band_on_ ? 0 : band_lds_.split ? 3 : band_lds_.full ? 1 : 2;
    const int k = std::min(n, 12 + kSetupSections);
    for (int i = 0; i < k; ++i) out[i] = v[i];
    return k;
  }

 private:
  void require_state() const {
    VO_REQUIRE(have_problem_, VO_ERR_STATE, "BA: no problem set up");
    VO_REQUIRE(have_state_, VO_ERR_STATE, "BA: no state set");
  }

  // Planner target of one K1 round: as many segments as resident workgroups (three per CU,
  // K1's __launch_bounds__ and LDS image).  A segment's time is about its chunk count times
  // the per-chunk latency, so one round of longer segments beats two rounds of shorter ones
  // (cfg4: 766 segments instead of 985; the cfg3 plan packs 678 either way).  Round 1's
  // sweep (profiles/r01_segment_sweep.md) predates the three-per-CU K1.
  // The one-wave K1 runs one chunk per segment: the largest target packs every
  // segment as one chunk (seg_obs = 1).
  static int segments_target(int num_cus, bool wave) {
    return wave ? (1 << 30) : VO_BA_SEGMENTS_PER_CU * std::max(1, num_cus);
  }
  // Chunks per segment of the one-wave K1's plan (the testing switch's value if it sets one).
  // Three instead of one: a third of the slab rows K2 reads for a barrier per segment; cfg3
  // 14.89k -> 15.27k GN-iters/s (42 148 -> 15 538 rows), cfg4 3.91k -> 4.04k (K2 34 -> 16 us,
  // K1 148 -> 158 us); two chunks sit between (profiles/r05_k1g).  Six (one 153 KB workgroup
  // per CU, the same six waves per CU) halves the rows again, which pays while the segments fit
  // one round: cfg3 15.71k -> 15.94k (246 segments, 8 175 rows; K1 24.7 -> 24.0 us, the fused
  // K3 43.7 -> 43.3 us), but cfg4's nine rounds of single workgroups lose the overlap of one
  // workgroup's combine with another's chunks: 4.09k -> 3.69k (profiles/r05_ab/k1_six_chunks).
  // So six for windows whose six-chunk segments are predicted to fit one round (56 observations
  // per chunk with padding, cfg3's; setup re-plans with three when they do not), else three.
  // (48-observation chunks, tuning builds: eight waves per CU, two per SIMD)
  static constexpr int kWaveChunksOneRound = std::min(kChunkObs >= 64 ? 6 : 8, kWaveMaxChunks),
                       kWaveChunksRounds = std::min(3, kWaveMaxChunks);
  int wave_chunks(int64_t n_obs) const {
    if (ctx_->ba_k1_variant >= 1) return std::min(ctx_->ba_k1_variant, kWaveMaxChunks);
    const int64_t one_round_obs = (int64_t)ctx_->num_cus * kWaveChunksOneRound * (kChunkObs * 7 / 8);
    return n_obs * 10 <= one_round_obs * 11 ? kWaveChunksOneRound : kWaveChunksRounds;
  }

  LinArgs lin_args() {
    const BAPlan& P = plan_;
    LinArgs A;
    A.n_fixed = P.n_fixed;
    A.fx = prob_.fx; A.fy = prob_.fy; A.cx = prob_.cx; A.cy = prob_.cy;
    A.lambda = prob_.lambda;
    A.chunk_hdr = d_chunk_hdr_.as<int4>();
    A.chunk_img = d_chunk_img_.as<ChunkImg>();
    A.slab_pos = d_slab_pos_.as<int>();
    A.cam_pos = d_cam_pos_.as<int>();
    A.seg_hdr = d_seg_hdr_.as<int>();
    A.points = d_points_.as<double>();
    A.slab = d_slab_.as<double>();
    A.slab_b = d_slab_b_.as<double>();
    A.slab_cost = d_slab_cost_.as<double>();
    A.pose_old = d_pose_[cur_ ^ 1].as<double>();
    A.pose_new = d_pose_[cur_].as<double>();
    A.dc = d_dc_.as<double>();
    A.status = d_status_.as<int>();
    A.stamps = nullptr;
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
    // one-wave K1 for plans of one chunk per segment (the chunk image of segment s is chunk s)
    const bool wave = plan_is_wave(plan_.seg_obs);
    const int nw = wave ? plan_.seg_chunks : 1;
    VO_REQUIRE(!wave || ((int64_t)nseg * nw == plan_.n_chunks() && nw >= 1 && nw <= kWaveMaxChunks), VO_ERR_STATE,
               "K1: segments of seg_chunks chunks expected");
    A.nseg = nseg;
    dim3 g(nseg), b(wave ? kLinLanesWave * nw : kLinThreads);
    ctx_->prof.begin(ctx_->stream, kKBaLin);
    if (stamps_on_) {  // one row per chunk (one-wave K1) or segment (four-wave K1)
      d_stamps_.reserve((size_t)plan_.n_chunks() * kPhCount * 8);
      A.stamps = d_stamps_.as<unsigned long long>();
    }
#if VO_WAVE_MAX_CHUNKS >= 8
#define VO_LIN_LAUNCH_78(M)                                                                   \
    if (wave && nw == 8)                                                                      \
      hipLaunchKernelGGL((ba_lin_wave_kernel<M, stamps_on_, 8>), g, b, 0, ctx_->stream, A);  \
    else if (wave && nw == 7)                                                                 \
      hipLaunchKernelGGL((ba_lin_wave_kernel<M, stamps_on_, 7>), g, b, 0, ctx_->stream, A);  \
    else
#else
#define VO_LIN_LAUNCH_78(M)
#endif
#define VO_LIN_LAUNCH(M)                                                                      \
  do {                                                                                        \
    VO_LIN_LAUNCH_78(M)                                                                       \
    if (wave && nw == 6)                                                                      \
      hipLaunchKernelGGL((ba_lin_wave_kernel<M, stamps_on_, 6>), g, b, 0, ctx_->stream, A);  \
    else if (wave && nw == 5)                                                                 \
      hipLaunchKernelGGL((ba_lin_wave_kernel<M, stamps_on_, 5>), g, b, 0, ctx_->stream, A);  \
    else if (wave && nw == 4)                                                                 \
      hipLaunchKernelGGL((ba_lin_wave_kernel<M, stamps_on_, 4>), g, b, 0, ctx_->stream, A);  \
    else if (wave && nw == 3)                                                                 \
      hipLaunchKernelGGL((ba_lin_wave_kernel<M, stamps_on_, 3>), g, b, 0, ctx_->stream, A);  \
    else if (wave && nw == 2)                                                                 \
      hipLaunchKernelGGL((ba_lin_wave_kernel<M, stamps_on_, 2>), g, b, 0, ctx_->stream, A);  \
    else if (wave)                                                                            \
      hipLaunchKernelGGL((ba_lin_wave_kernel<M, stamps_on_, 1>), g, b, 0, ctx_->stream, A);  \
    else                                                                                      \
      hipLaunchKernelGGL((ba_lin_kernel<M, stamps_on_>), g, b, 0, ctx_->stream, A);          \
  } while (0)
    switch (mode) {
      case kAccum: VO_LIN_LAUNCH(kAccum); break;
      case kBacksub | kAccum: VO_LIN_LAUNCH(kBacksub | kAccum); break;
      case kBacksub: VO_LIN_LAUNCH(kBacksub); break;
      default: VO_LIN_LAUNCH(0); break;
    }
#undef VO_LIN_LAUNCH
    ctx_->prof.end(ctx_->stream);
    VO_HIP_CHECK(hipGetLastError());
  }

  // K2 runs inside the banded K3's launch (one rank: no all-reduce between them)
  bool fused() const { return fuse_ok_ && !ctx_->ba_split_reduce && !(ctx_->comm && ctx_->comm->nranks > 1); }

  ReduceArgs reduce_args() const {
    const BAPlan& P = plan_;
    ReduceArgs R;
    R.nprof = P.n_prof_blocks();
    R.F = P.n_free;
    R.nseg = std::max(P.n_segments(), plan_.n_segments() > 0 ? 0 : 1);
    // damping on the camera diagonal: added once -- by rank 0 only when the partial
    // systems of the landmark shards are all-reduced
    R.lambda = (ctx_->comm && ctx_->comm->rank > 0) ? 0.0 : prob_.lambda;
    R.meta = d_red_meta_.as<int4>();
    R.out = d_red_out_.as<int2>();
    R.slab = d_slab_.as<double>();
    R.slab_b = d_slab_b_.as<double>();
    R.slab_cost = d_slab_cost_.as<double>();
    R.sys = d_sys_.as<double>();
    R.cost_off = cost_off_;
    R.status = d_status_.as<int>();
    return R;
  }

  void enqueue_reduce() {
    if (fused()) return;  // K3's reducer workgroups do it
    const ReduceArgs R = reduce_args();
    ctx_->prof.begin(ctx_->stream, kKBaReduce);
    hipLaunchKernelGGL(ba_reduce_kernel, dim3(R.nprof + 1), dim3(kRedThreads), 0, ctx_->stream, R);
    ctx_->prof.end(ctx_->stream);
    VO_HIP_CHECK(hipGetLastError());
    if (ctx_->comm && ctx_->comm->nranks > 1)
      ctx_->comm->allreduce(d_sys_.as<double>(), sys_len_, false, ctx_->stream);
  }

  void launch_solve(const SolveArgs& A) {
    if (band_on_) {
      const BAPlan& P = plan_;
      BandArgs B;
      B.F = A.F;
      B.w = band_.w;
      B.m = band_.m;
      B.nb = band_.nb;
      B.s = band_.s;
      B.nprof = A.nprof;
      B.n_poses = A.n_poses;
      B.n_fixed = A.n_fixed;
      B.iter_tag = A.iter_tag;
      B.cost_off = cost_off_;
      B.merge = band_tab_.merge;
      B.n_merge = band_tab_.n_merge;
      B.tab = d_band_tab_.as<int>();
      B.sys = A.sys;
      B.zero = d_zero_.as<double>();
      B.fac = band_lds_.full && !band_lds_.split ? nullptr : d_fac_.as<double>();
      B.seq = ++band_seq_ == 0 ? ++band_seq_ : band_seq_;  // split hand-off flags: new every launch
      B.cost_out = A.cost_out;
      B.dc = A.dc;
      B.pose_cur = A.pose_cur;
      B.pose_next = A.pose_next;
      B.status = A.status;
      B.stamps = nullptr;
      B.nred = fused() ? band_fused_workgroups(A.nprof) : 0;
      B.red_drop = B.nred > 0 ? ctx_->ba_drop_reducers : 0;
      B.red_count = d_colcnt_.as<unsigned>();
      B.red_col = d_red_col_.as<int>();
      B.col_need = d_col_need_.as<int>();
      B.red = reduce_args();
      if (stamps_on_) {  // per wave phase cycles, then realtime stamps of the solver and each reducer
        d_stamps3_.reserve((8 * kBandStamps + 8 + 4 * (B.nred + 1)) * 8);
        B.stamps = d_stamps3_.as<unsigned long long>();
      }
      (void)P;
      launch_band_solve(B, band_lds_, ctx_->stream);
      return;
    }
    if (solve_lds_)
      hipLaunchKernelGGL((ba_solve_kernel<true, kBaStamps, 4>), dim3(1), dim3(256), solve_lds_size_, ctx_->stream, A);
    else
      hipLaunchKernelGGL((ba_solve_kernel<false, kBaStamps, 4>), dim3(1), dim3(256), solve_lds_size_, ctx_->stream, A);
  }
  // the kernel's dynamic-LDS limit, raised only when a window needs more than any before it
  // (a process-wide attribute of the kernel)
  template <bool kL>
  static void set_solve_lds(int lds) {
    static std::atomic<int> set{-1};
    int cur = set.load(std::memory_order_relaxed);
    if (lds <= cur) return;
    VO_HIP_CHECK(hipFuncSetAttribute((const void*)ba_solve_kernel<kL, kBaStamps, 4>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    while (cur < lds && !set.compare_exchange_weak(cur, lds, std::memory_order_relaxed)) {
    }
  }

  void enqueue_solve(int iter_tag, double* cost_slot = nullptr) {
    const BAPlan& P = plan_;
    SolveArgs A;
    A.F = P.n_free;
    A.nprof = P.n_prof_blocks();
    A.n_poses = P.n_poses;
    A.n_fixed = P.n_fixed;
    A.iter_tag = iter_tag;
    A.max_panel = std::max(1, P.solve_layout.max_panel);
    A.max_row_span = 0;
    for (int k = 0; k < P.n_free; ++k) A.max_row_span = std::max(A.max_row_span, k - P.prof_first[k]);
    A.lds_kf = (long)solve_layout_.kf;
    A.lds_y = (long)solve_layout_.y;
    A.lds_panel = (long)solve_layout_.panel;
    A.lds_tab = (long)solve_layout_.tab;
    A.lds_pose = (long)solve_layout_.pose;
    A.tl = P.solve_layout;
    A.tab = d_solve_tab_.as<int>();
    A.cost_out = cost_slot;
    A.sys = d_sys_.as<double>();
    A.dc = d_dc_.as<double>();
    A.pose_cur = d_pose_[cur_].as<double>();
    A.pose_next = d_pose_[cur_ ^ 1].as<double>();
    A.status = d_status_.as<int>();
    A.stamps = nullptr;
    if (stamps_on_) {
      d_stamps3_.reserve(kS3Count * 8);
      A.stamps = d_stamps3_.as<unsigned long long>();
    }
    ctx_->prof.begin(ctx_->stream, kKBaSolve);
    launch_solve(A);
    ctx_->prof.end(ctx_->stream);
    VO_HIP_CHECK(hipGetLastError());
  }

  void iteration(double* d_cost_slot, int iter_tag) {
    enqueue_lin(pending_ ? (kBacksub | kAccum) : kAccum);
    enqueue_reduce();
    enqueue_solve(iter_tag, d_cost_slot);  // K3 also stores the cost (no extra copy node)
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
    R.cost_off = 0;
    R.status = d_status_.as<int>();
    hipLaunchKernelGGL(ba_reduce_kernel, dim3(1), dim3(kRedThreads), 0, ctx_->stream, R);
    VO_HIP_CHECK(hipGetLastError());
    if (ctx_->comm && ctx_->comm->nranks > 1)
      ctx_->comm->allreduce(R.sys, 1, false, ctx_->stream);
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
  BAPlan plan_{true};  // page-locked chunk images (async upload)
  BAPlan prev_plan_{true};  // the previous window's plan (group take-over), or scratch
  bool plan_ok_ = false;    // plan_ built and its images in d_chunk_img_
  int64_t setup_ns_[kSetupSections] = {};  // the last setup's host sections (vo_ba_plan_stats)
  vo_ba_problem prob_{};
  bool have_problem_ = false, have_state_ = false, pending_ = false, solve_lds_ = false;
  uint64_t session_ = 0;
  int cur_ = 0;
  size_t sys_len_ = 0, solve_lds_size_ = 0;
  SolveLds solve_layout_{};
  BandSplit band_{};
  bool band_on_ = false;
  bool fuse_ok_ = false;  // K2 fused into K3's launch (see fused())
  unsigned band_seq_ = 0;  // split-mode K3 launches so far (their hand-off flag values)
  BandLds band_lds_;
  BandTables band_tab_;
  // views into d_tab_ (the plan's small tables, one upload per setup) and d_misc_
  struct DevView {
    void* ptr = nullptr;
    template <class T>
    T* as() const {
      return static_cast<T*>(ptr);
    }
  };
  struct TablePack {  // the tables' places in d_tab_ (256-byte aligned) and their host sources
    struct Part {
      size_t off;
      const void* src;
      size_t n;
    };
    std::vector<Part> parts;
    size_t bytes = 0;
    template <class V>
    size_t add(const V& v) {
      const size_t off = (bytes + 255) & ~(size_t)255, n = v.size() * sizeof(v[0]);
      parts.push_back({off, v.data(), n});
      bytes = off + std::max<size_t>(n, 16);
      return off;
    }
  };
  HostBuf h_tab_;
  DevBuf d_tab_;
  DevView d_chunk_hdr_, d_seg_hdr_, d_slab_pos_, d_cam_pos_, d_solve_tab_, d_band_tab_, d_red_meta_, d_red_out_;
  static constexpr size_t kMiscBytes = 256 + 512;
  DevBuf d_misc_;  // [status | zero block (512 B)]
  DevView d_status_, d_zero_;
  DevBuf d_colcnt_;  // the fused launch's column readiness counters (band_col_count_bytes)
  size_t colcnt_bytes_ = 0;
  DevView d_red_col_, d_col_need_;
  std::vector<int32_t> red_col_, col_need_;
  std::vector<int4> red_meta_;
  std::vector<int2> red_out_;
  DevBuf d_fac_;
  std::vector<int32_t> red_dst_, red_rdst_;  // K2 output offsets (host copies for gn_step)
  long cost_off_ = 0;
  HostBuf h_state_;  // page-locked staging of set_state / get_state
  hipEvent_t h_state_ev_ = nullptr;  // set_state's upload from h_state_ done
  bool h_state_busy_ = false;
  DevBuf d_chunk_img_;  // K1's plan (the chunk images hold every list)
  DevBuf d_chunk_img_prev_;  // the previous plan's images (prev_plan_)
  DevBuf d_stamps_, d_stamps3_;
  static constexpr bool stamps_on_ = kBaStamps;

 public:
  // Diagnostic: per-phase cycle sums of the last K1 launch (VO_BA_STAMPS=1 builds).
  int read_stamps(uint64_t* out, int n) {
    if (!stamps_on_) return 0;
    // rows: chunks of a wave plan, segments of a four-wave plan
    const int nseg = plan_is_wave(plan_.seg_obs) ? plan_.n_chunks() : plan_.n_segments();
    std::vector<unsigned long long> h((size_t)nseg * kPhCount);
    VO_HIP_CHECK(hipStreamSynchronize(ctx_->stream));
    VO_HIP_CHECK(hipMemcpy(h.data(), d_stamps_.ptr, h.size() * 8, hipMemcpyDeviceToHost));
    if (n < 0) {  // raw per-segment rows (kPhCount values each; the last two are absolute times)
      const int k = std::min<int>(-n, (int)h.size());
      std::copy(h.begin(), h.begin() + k, out);
      return k;
    }
    int k = std::min(n, (int)kPhCount);
    for (int i = 0; i < k; ++i) {
      uint64_t acc = 0;
      for (int g = 0; g < nseg; ++g) acc += h[(size_t)g * kPhCount + i];
      out[i] = acc;
    }
    const int n3 = band_on_ ? 8 * kBandStamps : (int)kS3Count;  // K3: banded or profile solver
    if (n >= kPhCount + n3 && d_stamps3_.ptr) {
      // the banded solver's realtime stamps follow when the caller asked for them (fused launch)
      const int nx = band_on_ && fused() ? 8 + 4 * (band_fused_workgroups(plan_.n_prof_blocks()) + 1) : 0;
      const int n3x = n >= kPhCount + n3 + nx ? n3 + nx : n3;
      VO_HIP_CHECK(hipMemcpy(out + kPhCount, d_stamps3_.ptr, n3x * 8, hipMemcpyDeviceToHost));
      k += n3x;
    }
    return k;
  }

 private:
  DevBuf d_points_, d_pose_[2], d_dc_, d_slab_, d_slab_b_, d_slab_cost_, d_sys_, d_linv_;
  DevBuf d_cost_, d_cost_tmp_;
};

// ---- entry points used by api.hip -------------------------------------------------
BAEngine* ba_engine(vo_ctx* ctx) {
  if (!ctx->ba) ctx->ba.reset(new BAEngine(ctx));
  return ctx->ba.get();
}
uint64_t ba_setup(vo_ctx* ctx, const vo_ba_problem* p) { return ba_engine(ctx)->setup(p); }
void ba_reserve(vo_ctx* ctx, int n_poses, int n_points, int64_t n_obs, int n_fixed) {
  ba_engine(ctx)->reserve(n_poses, n_points, n_obs, n_fixed);
}
void ba_check_session(vo_ctx* ctx, uint64_t s) { ba_engine(ctx)->check_session(s); }
void ba_set_state(vo_ctx* ctx, const double* poses, const double* pts) {
  ba_engine(ctx)->set_state(poses, pts);
}
void ba_get_state(vo_ctx* ctx, double* poses, double* pts) { ba_engine(ctx)->get_state(poses, pts); }
int ba_run(vo_ctx* ctx, int iters, double* cost, bool sync) { return ba_engine(ctx)->run(iters, cost, sync); }
int ba_gn_step(vo_ctx* ctx, double* S, double* b, double* dc, double* cost) {
  return ba_engine(ctx)->gn_step(S, b, dc, cost);
}
int ba_stats(vo_ctx* ctx, int64_t* out, int n) { return ba_engine(ctx)->stats(out, n); }
int ba_stamps(vo_ctx* ctx, uint64_t* out, int n) { return ba_engine(ctx)->read_stamps(out, n); }

void comm_unique_id(char out[128]) {
  ncclUniqueId id;
  VO_NCCL_CHECK(ncclGetUniqueId(&id));
  static_assert(sizeof(id) == 128, "unexpected ncclUniqueId size");
  memcpy(out, &id, 128);
}

void comm_init_loopback(vo_ctx* ctx, int nranks, int rank, const char id[128]) {
  VO_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, VO_ERR_ARG, "vo_comm_init_loopback: bad rank");
  static std::mutex reg_mu;
  static std::map<std::string, std::weak_ptr<LoopGroup>> reg;
  std::shared_ptr<LoopGroup> g;
  {
    std::lock_guard<std::mutex> lk(reg_mu);
    const std::string key(id, 128);
    g = reg[key].lock();
    if (!g) {
      g = std::make_shared<LoopGroup>();
      g->nranks = nranks;
      g->slot.resize(nranks);
      reg[key] = g;
    }
  }
  VO_REQUIRE(g->nranks == nranks, VO_ERR_ARG, "vo_comm_init_loopback: group size mismatch");
  std::unique_ptr<Comm> c(new Comm);
  c->nranks = nranks;
  c->rank = rank;
  c->loop = g;
  ctx->comm = std::move(c);
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
