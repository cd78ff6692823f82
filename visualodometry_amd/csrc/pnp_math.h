// Scalar math of the PnP-RANSAC kernels (pnp.hip): EPnP, OpenCV's Jacobi SVD, Householder
// least squares, Rodrigues, the RANSAC iteration update, the se(3) exponential and a 6x6
// Cholesky solve.  Host-and-device (VO_HD) so tools/pnp_host_check.cpp can run the very
// same code on the CPU against oracle/pnp_ref.py; compiled without FMA contraction, the
// operation order of that restatement.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

#pragma clang fp contract(off)

#define VO_HD __host__ __device__ inline __attribute__((always_inline))

namespace vo {
namespace pnpm {

using std::sqrt;
using std::fabs;
using std::isfinite;

constexpr int kPts = 5;            // EPnP model points (solvePnPRansac: model_points = 5)
constexpr int kModel = 16;         // doubles per model: R (9), t (3), rvec (3), valid (1)
constexpr double kDblEps = 2.220446049250313e-16;
constexpr double kDblMin = 2.2250738585072014e-308;
constexpr double kFltEps = 1.1920928955078125e-07;
constexpr int kLmMaxIters = 20;
struct Cam {
  double fu, fv, uc, vc;
};

// ---------------------------------------------------------------- Jacobi SVD
// One pair (i, j) of JacobiSVDImpl_'s cyclic sweep (OpenCV core/lapack.cpp) on rows ai, aj of
// A and their squared norms wi, wj: rotates both rows when they are not yet orthogonal to
// eps and returns the rotation (c, s) through c_out / s_out.  jacobi_rows runs the pairs in
// the reference's order; pnp.hip's group kernel runs the same pairs on several lanes in an
// order that applies the same rotations to every row in the same sequence (bitwise equal).
template <int M>
VO_HD bool jacobi_pair(double* ai_row, double* aj_row, double& wi, double& wj, double& c_out, double& s_out) {
  constexpr double eps = 10.0 * kDblEps;
  const double a = wi, b = wj;
  double p = 0.0;
#pragma unroll
  for (int k = 0; k < M; ++k) p = p + ai_row[k] * aj_row[k];
  if (fabs(p) <= eps * sqrt(a * b)) return false;
  p = p * 2.0;
  // hypot(p, beta) from correctly rounded ops only, as the oracle: bitwise reproducible
  const double beta = a - b, gamma = sqrt(p * p + beta * beta);
  // the reference's two branches as one (same operations on the same operands), so a
  // wave whose lanes disagree on the sign of beta runs one division chain, not both:
  //   beta < 0: delta = (gamma - beta) * 0.5, s = sqrt(delta / gamma), c = p / (gamma * s * 2)
  //   else:     c = sqrt((gamma + beta) / (gamma * 2)),                s = p / (gamma * c * 2)
  const bool neg = beta < 0;
  const double num = neg ? (gamma - beta) * 0.5 : gamma + beta;
  const double den = neg ? gamma : gamma * 2.0;
  const double x = sqrt(num / den);
  const double y = p / (gamma * x * 2.0);
  const double c = neg ? y : x, s = neg ? x : y;
  double na = 0.0, nb = 0.0;
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const double ai = ai_row[k], aj = aj_row[k];
    const double t0 = c * ai + s * aj;
    const double t1 = -s * ai + c * aj;
    ai_row[k] = t0;
    aj_row[k] = t1;
    na = na + t0 * t0;
    nb = nb + t1 * t1;
  }
  wi = na;
  wj = nb;
  c_out = c;
  s_out = s;
  return true;
}

// JacobiSVDImpl_ (OpenCV core/lapack.cpp) on the rows of A (rotated in place): W[i] ends
// as the norm of row i (unsorted); Vt accumulates the rotations when WANT_V.  (The pair body is
// jacobi_pair's, operation for operation, written out here: passed row pointers, the compiler
// kept more of the batch kernel's state in scratch.)
template <int N, int M, bool WANT_V>
VO_HD void jacobi_rows(double (&A)[N][M], double (&W)[N], double (&Vt)[N][N]) {
  constexpr double eps = 10.0 * kDblEps;
  constexpr int max_sweeps = M > 30 ? M : 30;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double sd = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k) sd = sd + A[i][k] * A[i][k];
    W[i] = sd;
    if (WANT_V) {
#pragma unroll
      for (int k = 0; k < N; ++k) Vt[i][k] = i == k ? 1.0 : 0.0;
    }
  }
  for (int sweep = 0; sweep < max_sweeps; ++sweep) {
    bool changed = false;
#pragma unroll
    for (int i = 0; i < N - 1; ++i) {
#pragma unroll
      for (int j = i + 1; j < N; ++j) {
        const double a = W[i], b = W[j];
        double p = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) p = p + A[i][k] * A[j][k];
        if (!(fabs(p) <= eps * sqrt(a * b))) {
          p = p * 2.0;
          const double beta = a - b, gamma = sqrt(p * p + beta * beta);
          const bool neg = beta < 0;
          const double num = neg ? (gamma - beta) * 0.5 : gamma + beta;
          const double den = neg ? gamma : gamma * 2.0;
          const double x = sqrt(num / den);
          const double y = p / (gamma * x * 2.0);
          const double c = neg ? y : x, s = neg ? x : y;
          double na = 0.0, nb = 0.0;
#pragma unroll
          for (int k = 0; k < M; ++k) {
            const double ai = A[i][k], aj = A[j][k];
            const double t0 = c * ai + s * aj;
            const double t1 = -s * ai + c * aj;
            A[i][k] = t0;
            A[j][k] = t1;
            na = na + t0 * t0;
            nb = nb + t1 * t1;
          }
          W[i] = na;
          W[j] = nb;
          changed = true;
          if (WANT_V) {
#pragma unroll
            for (int k = 0; k < N; ++k) {
              const double vi = Vt[i][k], vj = Vt[j][k];
              Vt[i][k] = c * vi + s * vj;
              Vt[j][k] = -s * vi + c * vj;
            }
          }
        }
      }
    }
    if (!changed) break;
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double sd = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k) sd = sd + A[i][k] * A[i][k];
    W[i] = sqrt(sd);
  }
}

// The pairs of one cyclic sweep of an N-row jacobi_rows in steps: step t holds the pairs (i, j)
// with i + j == t.  A pair touching row i or j precedes (i, j) in the cyclic order exactly when
// its index sum is below i + j, and the pairs of one step are disjoint, so running the steps in
// order (the pairs of a step in any order, or at once) applies every row's rotations in the
// cyclic order: bitwise jacobi_rows.  The host restatement of pnp.hip's lane-group SVD
// (tests/test_pnp_host_math.py runs EPnP with it against the oracle).
struct Jacobi12Steps {
  VO_HD void operator()(double (&A)[12][12], double (&W)[12]) const {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      double sd = 0.0;
      for (int k = 0; k < 12; ++k) sd = sd + A[i][k] * A[i][k];
      W[i] = sd;
    }
    for (int sweep = 0; sweep < 30; ++sweep) {
      bool changed = false;
      for (int t = 1; t <= 21; ++t)
        for (int i = t - 11 > 0 ? t - 11 : 0; i < t - i; ++i) {
          double c, s;
          changed |= jacobi_pair<12>(A[i], A[t - i], W[i], W[t - i], c, s);
        }
      if (!changed) break;
    }
    for (int i = 0; i < 12; ++i) {
      double sd = 0.0;
      for (int k = 0; k < 12; ++k) sd = sd + A[i][k] * A[i][k];
      W[i] = sqrt(sd);
    }
  }
};

// EPnP's 12 x 12 SVD in the index-sum step order (Jacobi12Steps' schedule): on the device by
// the lane group of pnp.hip's group kernel (its LDS rows at lds, this lane's place in the group
// at lane), on the host (the host check) serially.  Passed to epnp5 by pointer, nullptr for the
// cyclic sweep (a template parameter instead changed the batch kernel's register allocation:
// 300 -> 532 B of scratch per lane).
constexpr int kSvdGroupLanes = 16;  // lanes per hypothesis of the lane-group SVD (Svd12Alt)
struct Svd12Alt {
  double* lds;
  int lane;
#if defined(__HIP_DEVICE_COMPILE__)
  __device__ void sweeps() const;  // the Jacobi sweeps on the group's LDS rows and squared norms
#else
  void run(double (&A)[12][12], double (&W)[12]) const;  // host: jacobi_rows in the step order
#endif
};

// Svd12Alt: 16 lanes per group on the device (pnp_group.hip), the step order serially on the
// host.  Device sweeps (svd12_group_null_space fills the rows): step t takes the pairs (i, j)
// with i + j == t (at most six, disjoint), two lanes each, on rows read from the group's LDS and
// written back; the group stops after the first sweep without a rotation (a ballot over its
// lanes).  One wave: its LDS operations complete in order, so a step's writes precede the next
// step's reads behind an lgkmcnt wait.
#if defined(__HIP_DEVICE_COMPILE__)
// 16 lanes per group: lane r takes pair slot r & 7 of a step and half r >> 3 of the pair's rows
// (elements 6h .. 6h + 5).  The dot product and the two norms stay the serial sum over the row's
// twelve elements: half 0 sums its six terms from zero, half 1 continues from half 0's partial
// (one DPP rotation by eight lanes within the 16-lane row each way), so every sum keeps its
// order; the rotation is per element.  The same values as jacobi_pair on the whole rows.
__device__ __forceinline__ double svd_xhalf(double v) {  // the value of the lane eight away in the 16-lane row
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x128, 0xF, 0xF, false);  // row_ror:8
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x128, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ inline void Svd12Alt::sweeps() const {
  constexpr double eps = 10.0 * kDblEps;
  double* A = lds;
  double* W = lds + 144;
  const int q = lane & 7, h = lane >> 3;
  const uint64_t gmask = 0xFFFFull << (threadIdx.x & 48);
  for (int sweep = 0; sweep < 30; ++sweep) {
    bool changed = false;
    for (int t = 1; t <= 21; ++t) {
      const int i = (t - 11 > 0 ? t - 11 : 0) + q, j = t - i;
      if (i < j) {  // both halves of a slot alike
        double ai[6], aj[6];
#pragma unroll
        for (int k = 0; k < 6; k += 2) {
          const double2 x = *reinterpret_cast<const double2*>(A + 12 * i + 6 * h + k);
          const double2 y = *reinterpret_cast<const double2*>(A + 12 * j + 6 * h + k);
          ai[k] = x.x;
          ai[k + 1] = x.y;
          aj[k] = y.x;
          aj[k + 1] = y.y;
        }
        const double a = W[i], b = W[j];
        double pm[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) pm[k] = ai[k] * aj[k];
        double p = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) p = p + pm[k];  // half 0: terms 0 .. 5
        p = svd_xhalf(p);
#pragma unroll
        for (int k = 0; k < 6; ++k) p = p + pm[k];  // half 1: terms 6 .. 11 after half 0's
        const double ph = svd_xhalf(p);
        p = h ? p : ph;
        if (!(fabs(p) <= eps * sqrt(a * b))) {  // jacobi_pair's rotation, the same operations
          p = p * 2.0;
          const double beta = a - b, gamma = sqrt(p * p + beta * beta);
          const bool neg = beta < 0;
          const double num = neg ? (gamma - beta) * 0.5 : gamma + beta;
          const double den = neg ? gamma : gamma * 2.0;
          const double x = sqrt(num / den);
          const double y = p / (gamma * x * 2.0);
          const double c = neg ? y : x, sn = neg ? x : y;
          double t0[6], t1[6];
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            t0[k] = c * ai[k] + sn * aj[k];
            t1[k] = -sn * ai[k] + c * aj[k];
          }
          double na = 0.0, nb = 0.0;
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            na = na + t0[k] * t0[k];
            nb = nb + t1[k] * t1[k];
          }
          na = svd_xhalf(na);
          nb = svd_xhalf(nb);
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            na = na + t0[k] * t0[k];
            nb = nb + t1[k] * t1[k];
          }
#pragma unroll
          for (int k = 0; k < 6; k += 2) {
            *reinterpret_cast<double2*>(A + 12 * i + 6 * h + k) = make_double2(t0[k], t0[k + 1]);
            *reinterpret_cast<double2*>(A + 12 * j + 6 * h + k) = make_double2(t1[k], t1[k + 1]);
          }
          if (h) {
            W[i] = na;
            W[j] = nb;
          }
          changed = true;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if ((__ballot(changed) & gmask) == 0) break;  // uniform in the group
  }
}
#else
inline void Svd12Alt::run(double (&Ar)[12][12], double (&Wr)[12]) const { Jacobi12Steps{}(Ar, Wr); }
#endif

// Position of each singular value in the descending order (the selection sort of
// JacobiSVDImpl_; equal values keep their index order, which the selection sort also
// does unless three or more tie -- never for the non-degenerate inputs used here).
template <int N>
VO_HD void desc_rank(const double (&W)[N], int (&rank)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    int r = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) r += (W[k] > W[i] || (k < i && W[k] == W[i])) ? 1 : 0;
    rank[i] = r;
  }
}

// ---------------------------------------------------------------- EPnP helpers
VO_HD double dot3(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// epnp::qr_solve (Householder least squares); X is left unchanged if a column is zero.
template <int NR, int NC>
VO_HD void qr_solve(double (&A)[NR][NC], double (&b)[NR], double (&X)[NC]) {
  double A1[NC], A2[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    double eta = fabs(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < NR; ++i) {
      const double e = fabs(A[i][k]);
      eta = eta < e ? e : eta;
    }
    if (eta == 0.0) return;
    const double inv_eta = 1.0 / eta;
    double sum2 = 0.0;
#pragma unroll
    for (int i = k; i < NR; ++i) {
      A[i][k] = A[i][k] * inv_eta;
      sum2 = sum2 + A[i][k] * A[i][k];
    }
    double sigma = sqrt(sum2);
    if (A[k][k] < 0) sigma = -sigma;
    A[k][k] = A[k][k] + sigma;
    A1[k] = sigma * A[k][k];
    A2[k] = -eta * sigma;
#pragma unroll
    for (int j = k + 1; j < NC; ++j) {
      double s = 0.0;
#pragma unroll
      for (int i = k; i < NR; ++i) s = s + A[i][k] * A[i][j];
      const double tau = s / A1[k];
#pragma unroll
      for (int i = k; i < NR; ++i) A[i][j] = A[i][j] - tau * A[i][k];
    }
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    double tau = 0.0;
#pragma unroll
    for (int i = j; i < NR; ++i) tau = tau + A[i][j] * b[i];
    tau = tau / A1[j];
#pragma unroll
    for (int i = j; i < NR; ++i) b[i] = b[i] - tau * A[i][j];
  }
  X[NC - 1] = b[NC - 1] / A2[NC - 1];
#pragma unroll
  for (int i = NC - 2; i >= 0; --i) {
    double s = 0.0;
#pragma unroll
    for (int j = i + 1; j < NC; ++j) s = s + A[i][j] * X[j];
    X[i] = (b[i] - s) / A2[i];
  }
}

// Doubles at p[k * stride]: a local array (stride 1), or on the device one lane's column of a
// wave's LDS block (stride 64), which keeps EPnP's read-mostly arrays out of the VGPRs that
// the 12x12 Jacobi sweep needs.  The arithmetic is the same either way.
struct Col {
  double* p;
  int stride;
  VO_HD double& operator[](int k) const { return p[k * stride]; }
};

struct EpnpState {
  float pw[kPts][3];  // object points (float32, as the caller holds them)
  float us[kPts][2];  // image points (float32)
  Col alphas;         // [p * 4 + c]: barycentric coordinates
  Col v;              // [i * 12 + k]: v[i] = ut row 11 - i (right singular vectors, smallest first)
  double cws[4][3];
  double L[6][10];
  double rho[6];
};
constexpr int kEpnpColDoubles = kPts * 4 + 4 * 12;  // alphas, v

#if defined(__HIP_DEVICE_COMPILE__)
// The 12 x 12 part of epnp::compute_pose on a lane group (Svd12Alt's 16 lanes), without M^T M in
// any lane's registers: lane r < 12 builds row r of M^T M straight into the group's LDS rows
// (each entry the same sum in the same order as the per-lane build), the Jacobi sweeps run on
// the group (Svd12Alt::sweeps), lane r then takes the norm of its row, and every lane reads the twelve
// norms and only the four rows it needs (v = the rows of the four smallest, each times 1 / W).
// Same values as jacobi_rows + the selection below it in epnp5.  Returns the W > DBL_MIN flag.
__device__ inline bool svd12_group_null_space(const Svd12Alt& g, EpnpState& S, const Cam& K) {
  double* A = g.lds;
  double* W = g.lds + 144;
  const int r = g.lane;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = r + kSvdGroupLanes * u;
    if (i < 12) {
      const int c = i / 3, comp = i - 3 * c;
      double row[12];
#pragma unroll
      for (int b = 0; b < 12; ++b) row[b] = 0.0;
#pragma unroll
      for (int p = 0; p < kPts; ++p) {
        double m1[12], m2[12];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          const double al = S.alphas[p * 4 + cc];
          m1[3 * cc] = al * K.fu;
          m1[3 * cc + 1] = 0.0;
          m1[3 * cc + 2] = al * (K.uc - S.us[p][0]);
          m2[3 * cc] = 0.0;
          m2[3 * cc + 1] = al * K.fv;
          m2[3 * cc + 2] = al * (K.vc - S.us[p][1]);
        }
        const double ali = S.alphas[p * 4 + c];
        const double m1i = comp == 0 ? ali * K.fu : comp == 1 ? 0.0 : ali * (K.uc - S.us[p][0]);
        const double m2i = comp == 0 ? 0.0 : comp == 1 ? ali * K.fv : ali * (K.vc - S.us[p][1]);
#pragma unroll
        for (int b = 0; b < 12; ++b) row[b] = row[b] + m1i * m1[b];
#pragma unroll
        for (int b = 0; b < 12; ++b) row[b] = row[b] + m2i * m2[b];
      }
      double sd = 0.0;
#pragma unroll
      for (int k = 0; k < 12; k += 2) {
        *reinterpret_cast<double2*>(A + 12 * i + k) = make_double2(row[k], row[k + 1]);
        sd = sd + row[k] * row[k];
        sd = sd + row[k + 1] * row[k + 1];
      }
      W[i] = sd;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  g.sweeps();
  // norms of this lane's rows (jacobi_rows' last loop), then every lane reads all twelve
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = r + kSvdGroupLanes * u;
    if (i < 12) {
      double sd = 0.0;
#pragma unroll
      for (int k = 0; k < 12; k += 2) {
        const double2 x = *reinterpret_cast<const double2*>(A + 12 * i + k);
        sd = sd + x.x * x.x;
        sd = sd + x.y * x.y;
      }
      W[i] = sqrt(sd);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  double Wr[12];
#pragma unroll
  for (int i = 0; i < 12; i += 2) {
    const double2 x = *reinterpret_cast<const double2*>(W + i);
    Wr[i] = x.x;
    Wr[i + 1] = x.y;
  }
  int rk[12];
  desc_rank<12>(Wr, rk);
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 12; ++i) ok &= Wr[i] > kDblMin;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int sel = 0;
    double wsel = Wr[0];
#pragma unroll
    for (int i = 1; i < 12; ++i) {
      sel = rk[i] == 11 - q ? i : sel;
      wsel = rk[i] == 11 - q ? Wr[i] : wsel;
    }
    const double sq = 1.0 / wsel;
    const double* rowp = A + 12 * sel;
#pragma unroll
    for (int k = 0; k < 12; k += 2) {
      const double2 x = *reinterpret_cast<const double2*>(rowp + k);
      S.v[q * 12 + k] = x.x * sq;
      S.v[q * 12 + k + 1] = x.y * sq;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's reads before the rows are reused
  return ok;
}
#endif

VO_HD double dot3f(const double* a, const float* b) {
  return a[0] * (double)b[0] + a[1] * (double)b[1] + a[2] * (double)b[2];
}

VO_HD void gauss_newton(const EpnpState& S, double (&betas)[4]) {
  double x[4] = {0.0, 0.0, 0.0, 0.0};
  for (int it = 0; it < 5; ++it) {
    double A[6][4], b[6];
    const double b0 = betas[0], b1 = betas[1], b2 = betas[2], b3 = betas[3];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double* l = S.L[i];
      A[i][0] = 2 * l[0] * b0 + l[1] * b1 + l[3] * b2 + l[6] * b3;
      A[i][1] = l[1] * b0 + 2 * l[2] * b1 + l[4] * b2 + l[7] * b3;
      A[i][2] = l[3] * b0 + l[4] * b1 + 2 * l[5] * b2 + l[8] * b3;
      A[i][3] = l[6] * b0 + l[7] * b1 + l[8] * b2 + 2 * l[9] * b3;
      b[i] = S.rho[i] - (l[0] * b0 * b0 + l[1] * b0 * b1 + l[2] * b1 * b1 + l[3] * b0 * b2 +
                         l[4] * b1 * b2 + l[5] * b2 * b2 + l[6] * b0 * b3 + l[7] * b1 * b3 +
                         l[8] * b2 * b3 + l[9] * b3 * b3);
    }
    qr_solve<6, 4>(A, b, x);
#pragma unroll
    for (int i = 0; i < 4; ++i) betas[i] = betas[i] + x[i];
  }
}

// compute_R_and_t: control points in the camera frame, sign, Procrustes, mean pixel error.
VO_HD double compute_R_and_t(const EpnpState& S, const Cam& K, const double (&betas)[4],
                                                  double (&R)[3][3], double (&t)[3]) {
  double ccs[4][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 3; ++k) ccs[j][k] = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) ccs[j][k] = ccs[j][k] + betas[i] * S.v[i * 12 + 3 * j + k];
  double pcs[kPts][3];
#pragma unroll
  for (int p = 0; p < kPts; ++p)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      pcs[p][k] = S.alphas[p * 4] * ccs[0][k] + S.alphas[p * 4 + 1] * ccs[1][k] + S.alphas[p * 4 + 2] * ccs[2][k] +
                  S.alphas[p * 4 + 3] * ccs[3][k];
  if (pcs[0][2] < 0.0) {  // solve_for_sign
#pragma unroll
    for (int p = 0; p < kPts; ++p)
#pragma unroll
      for (int k = 0; k < 3; ++k) pcs[p][k] = -pcs[p][k];
  }
  // estimate_R_and_t
  double pc0[3] = {0.0, 0.0, 0.0}, pw0[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int p = 0; p < kPts; ++p)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pc0[k] = pc0[k] + pcs[p][k];
      pw0[k] = pw0[k] + S.pw[p][k];
    }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    pc0[k] = pc0[k] / kPts;
    pw0[k] = pw0[k] / kPts;
  }
  double abt[3][3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) abt[a][b] = 0.0;
#pragma unroll
  for (int p = 0; p < kPts; ++p)
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) abt[a][b] = abt[a][b] + (pcs[p][a] - pc0[a]) * (S.pw[p][b] - pw0[b]);
  // SVD of abt: JacobiSVD on the rows of abt^T; R = U V^T = sum_k u_k v_k^T
  double At[3][3], W[3], Vt[3][3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) At[a][b] = abt[b][a];
  jacobi_rows<3, 3, true>(At, W, Vt);
  double iw[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) iw[k] = 1.0 / W[k];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 3; ++k) s = s + (At[k][i] * iw[k]) * Vt[k][j];
      R[i][j] = s;
    }
  const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                     R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
  if (det < 0) {
    R[2][0] = -R[2][0];
    R[2][1] = -R[2][1];
    R[2][2] = -R[2][2];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) t[k] = pc0[k] - dot3(R[k], pw0);
  // reprojection_error
  double err = 0.0;
#pragma unroll
  for (int p = 0; p < kPts; ++p) {
    const double Xc = dot3f(R[0], S.pw[p]) + t[0];
    const double Yc = dot3f(R[1], S.pw[p]) + t[1];
    const double inv_Zc = 1.0 / (dot3f(R[2], S.pw[p]) + t[2]);
    const double ue = K.uc + K.fu * Xc * inv_Zc;
    const double ve = K.vc + K.fv * Yc * inv_Zc;
    const double du = S.us[p][0] - ue, dv = S.us[p][1] - ve;
    err = err + sqrt(du * du + dv * dv);
  }
  return err / kPts;
}

// epnp::compute_pose on 5 correspondences.  Returns false for a degenerate subset.
VO_HD bool epnp5(EpnpState& S, const Cam& K, double (&R)[3][3], double (&t)[3], const Svd12Alt* alt = nullptr) {
  bool ok = true;
  // choose_control_points: centroid + PCA of the points
  double c0[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int p = 0; p < kPts; ++p)
#pragma unroll
    for (int k = 0; k < 3; ++k) c0[k] = c0[k] + S.pw[p][k];
#pragma unroll
  for (int k = 0; k < 3; ++k) c0[k] = c0[k] / kPts;
  {
    double P[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) P[a][b] = 0.0;
#pragma unroll
    for (int p = 0; p < kPts; ++p) {
      double d[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) d[k] = S.pw[p][k] - c0[k];
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) P[a][b] = P[a][b] + d[a] * d[b];
    }
    double At[3][3], W[3], dummy[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) At[a][b] = P[b][a];
    jacobi_rows<3, 3, false>(At, W, dummy);
    int rk[3];
    desc_rank<3>(W, rk);
#pragma unroll
    for (int k = 0; k < 3; ++k) S.cws[0][k] = c0[k];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      ok &= W[i] > kDblMin;
      const double s = 1.0 / W[i];
      const double kk = sqrt(W[i] / kPts);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        double val = c0[k] + kk * (At[i][k] * s);
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (rk[i] == q) S.cws[q + 1][k] = val;
      }
    }
  }
  // compute_barycentric_coordinates: alphas = CC^-1 (p - c0), CC^-1 from its SVD
  {
    double At[3][3], W[3], Vt[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 1; j < 4; ++j) At[j - 1][i] = S.cws[j][i] - S.cws[0][i];  // rows of CC^T
    jacobi_rows<3, 3, true>(At, W, Vt);
    double iw[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      ok &= W[k] > kDblMin;
      iw[k] = 1.0 / W[k];
    }
    double ci[3][3];  // CC^-1 = V diag(1/w) U^T
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) s = s + Vt[k][i] * iw[k] * (At[k][j] * iw[k]);
        ci[i][j] = s;
      }
#pragma unroll
    for (int p = 0; p < kPts; ++p) {
      const double d0 = S.pw[p][0] - S.cws[0][0], d1 = S.pw[p][1] - S.cws[0][1], d2 = S.pw[p][2] - S.cws[0][2];
      double al[4];
#pragma unroll
      for (int j = 0; j < 3; ++j) al[1 + j] = ci[j][0] * d0 + ci[j][1] * d1 + ci[j][2] * d2;
      al[0] = 1.0 - al[1] - al[2] - al[3];
#pragma unroll
      for (int c = 0; c < 4; ++c) S.alphas[p * 4 + c] = al[c];
    }
  }
  // compute_rho (ahead of the 12x12 SVD, so that the control points are dead during it)
  {
    constexpr int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      double e[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) e[k] = S.cws[pa[i]][k] - S.cws[pb[i]][k];
      S.rho[i] = dot3(e, e);
    }
  }
  // M (2n x 12), M^T M, its four smallest right singular vectors
#if defined(__HIP_DEVICE_COMPILE__)
  if (alt)
    ok &= svd12_group_null_space(*alt, S, K);
  else
#endif
  {
    double A[12][12];
#pragma unroll
    for (int a = 0; a < 12; ++a)
#pragma unroll
      for (int b = 0; b < 12; ++b) A[a][b] = 0.0;
#pragma unroll
    for (int p = 0; p < kPts; ++p) {
      double m1[12], m2[12];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double al = S.alphas[p * 4 + c];
        m1[3 * c] = al * K.fu;
        m1[3 * c + 1] = 0.0;
        m1[3 * c + 2] = al * (K.uc - S.us[p][0]);
        m2[3 * c] = 0.0;
        m2[3 * c + 1] = al * K.fv;
        m2[3 * c + 2] = al * (K.vc - S.us[p][1]);
      }
#pragma unroll
      for (int a = 0; a < 12; ++a)
#pragma unroll
        for (int b = 0; b < 12; ++b) A[a][b] = A[a][b] + m1[a] * m1[b];
#pragma unroll
      for (int a = 0; a < 12; ++a)
#pragma unroll
        for (int b = 0; b < 12; ++b) A[a][b] = A[a][b] + m2[a] * m2[b];
    }
    double W[12], dummy[12][12];
#if defined(__HIP_DEVICE_COMPILE__)
    jacobi_rows<12, 12, false>(A, W, dummy);  // M^T M is symmetric: its rows are A^T's
#else
    if (alt)
      alt->run(A, W);  // the lane groups' step order, serially
    else
      jacobi_rows<12, 12, false>(A, W, dummy);
#endif
    int rk[12];
    desc_rank<12>(W, rk);
    double s[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      ok &= W[i] > kDblMin;
      s[i] = 1.0 / W[i];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        double val = 0.0;
#pragma unroll
        for (int i = 0; i < 12; ++i) val = rk[i] == 11 - q ? A[i][k] * s[i] : val;
        S.v[q * 12 + k] = val;
      }
  }
  // compute_L_6x10
  {
    constexpr int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
    double dv[4][6][3];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) dv[i][j][k] = S.v[i * 12 + 3 * pa[j] + k] - S.v[i * 12 + 3 * pb[j] + k];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      double* row = S.L[i];
      row[0] = dot3(dv[0][i], dv[0][i]);
      row[1] = 2.0 * dot3(dv[0][i], dv[1][i]);
      row[2] = dot3(dv[1][i], dv[1][i]);
      row[3] = 2.0 * dot3(dv[0][i], dv[2][i]);
      row[4] = 2.0 * dot3(dv[1][i], dv[2][i]);
      row[5] = dot3(dv[2][i], dv[2][i]);
      row[6] = 2.0 * dot3(dv[0][i], dv[3][i]);
      row[7] = 2.0 * dot3(dv[1][i], dv[3][i]);
      row[8] = 2.0 * dot3(dv[2][i], dv[3][i]);
      row[9] = dot3(dv[3][i], dv[3][i]);
    }
  }
  // three beta approximations, each refined by Gauss-Newton; keep the lowest error
  auto run_kind = [&](int kind, double (&Rk)[3][3], double (&tk)[3]) __attribute__((always_inline)) -> double {
    double betas[4] = {0.0, 0.0, 0.0, 0.0};
    double rho[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) rho[i] = S.rho[i];
    if (kind == 1) {  // [B11 B12 B13 B14]
      double A[6][4], x[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        A[i][0] = S.L[i][0];
        A[i][1] = S.L[i][1];
        A[i][2] = S.L[i][3];
        A[i][3] = S.L[i][6];
      }
      qr_solve<6, 4>(A, rho, x);
      if (x[0] < 0) {
        betas[0] = sqrt(-x[0]);
        betas[1] = -x[1] / betas[0];
        betas[2] = -x[2] / betas[0];
        betas[3] = -x[3] / betas[0];
      } else {
        betas[0] = sqrt(x[0]);
        betas[1] = x[1] / betas[0];
        betas[2] = x[2] / betas[0];
        betas[3] = x[3] / betas[0];
      }
    } else if (kind == 2) {  // [B11 B12 B22]
      double A[6][3], x[3] = {0.0, 0.0, 0.0};
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) A[i][c] = S.L[i][c];
      qr_solve<6, 3>(A, rho, x);
      if (x[0] < 0) {
        betas[0] = sqrt(-x[0]);
        betas[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
      } else {
        betas[0] = sqrt(x[0]);
        betas[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0) betas[0] = -betas[0];
    } else {  // [B11 B12 B22 B13 B23]
      double A[6][5], x[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int c = 0; c < 5; ++c) A[i][c] = S.L[i][c];
      qr_solve<6, 5>(A, rho, x);
      if (x[0] < 0) {
        betas[0] = sqrt(-x[0]);
        betas[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
      } else {
        betas[0] = sqrt(x[0]);
        betas[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0) betas[0] = -betas[0];
      betas[2] = x[3] / betas[0];
    }
    gauss_newton(S, betas);
    return compute_R_and_t(S, K, betas, Rk, tk);
  };
  double bestR[3][3], bestt[3], best_err = 0.0;
#if defined(__HIP_DEVICE_COMPILE__)
  if (alt) {
    // lane groups: lane r of the group refines kind r + 1 (lanes 3.. repeat kind 3), the three
    // results meet in the group's LDS (free after the SVD; one wave: its LDS operations
    // complete in order) and every lane takes the serial loop's choice from them: kind 1, then
    // a later kind only if its error is strictly lower.  The kinds' Gauss-Newton and pose
    // passes run once, side by side, instead of three times on every lane.
    double Rk[3][3], tk[3];
    const int my = alt->lane < 3 ? alt->lane + 1 : 3;
    const double e = run_kind(my, Rk, tk);
    double* x = alt->lds;
    if (alt->lane < 3) {
      double* d = x + 13 * alt->lane;
#pragma unroll
      for (int q = 0; q < 9; ++q) d[q] = Rk[q / 3][q % 3];
#pragma unroll
      for (int q = 0; q < 3; ++q) d[9 + q] = tk[q];
      d[12] = e;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int pick = 0;
    best_err = x[12];
    if (x[13 + 12] < best_err) {
      best_err = x[13 + 12];
      pick = 1;
    }
    if (x[26 + 12] < best_err) {
      best_err = x[26 + 12];
      pick = 2;
    }
    const double* d = x + 13 * pick;
#pragma unroll
    for (int q = 0; q < 9; ++q) bestR[q / 3][q % 3] = d[q];
#pragma unroll
    for (int q = 0; q < 3; ++q) bestt[q] = d[9 + q];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's reads before the group's LDS is reused
  } else
#endif
  for (int kind = 1; kind <= 3; ++kind) {
    // keeps the reads of S.alphas / S.v (LDS on the device) inside the loop: hoisted out of
    // it they would take registers across all three kinds
    asm volatile("" ::: "memory");
    double Rk[3][3], tk[3];
    const double e = run_kind(kind, Rk, tk);
    if (kind == 1 || e < best_err) {
      best_err = e;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        bestt[a] = tk[a];
#pragma unroll
        for (int b = 0; b < 3; ++b) bestR[a][b] = Rk[a][b];
      }
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    t[a] = bestt[a];
    ok &= isfinite(t[a]);
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      R[a][b] = bestR[a][b];
      ok &= isfinite(R[a][b]);
    }
  }
  return ok;
}

// ---------------------------------------------------------------- Rodrigues
// Matrix -> vector (calibration.cpp); R's columns are first scaled to unit norm, which is
// what OpenCV's U Vt re-orthonormalisation does to an already orthonormal R.
VO_HD void rodrigues_to_vec(const double (&Rin)[3][3], double (&r)[3]) {
  double R[3][3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double nrm = sqrt(Rin[0][j] * Rin[0][j] + Rin[1][j] * Rin[1][j] + Rin[2][j] * Rin[2][j]);
#pragma unroll
    for (int i = 0; i < 3; ++i) R[i][j] = Rin[i][j] / nrm;
  }
  const double rx = R[2][1] - R[1][2], ry = R[0][2] - R[2][0], rz = R[1][0] - R[0][1];
  const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0][0] + R[1][1] + R[2][2] - 1) * 0.5;
  c = c > 1. ? 1. : c < -1. ? -1. : c;
  const double theta = acos(c);
  if (s < 1e-5) {
    if (c > 0) {
      r[0] = r[1] = r[2] = 0.0;
    } else {
      double t = (R[0][0] + 1) * 0.5;
      double r0 = sqrt(t > 0. ? t : 0.);
      t = (R[1][1] + 1) * 0.5;
      double r1 = sqrt(t > 0. ? t : 0.) * (R[0][1] < 0 ? -1. : 1.);
      t = (R[2][2] + 1) * 0.5;
      double r2 = sqrt(t > 0. ? t : 0.) * (R[0][2] < 0 ? -1. : 1.);
      if (fabs(r0) < fabs(r1) && fabs(r0) < fabs(r2) && (R[1][2] > 0) != (r1 * r2 > 0)) r2 = -r2;
      const double th = theta / sqrt(r0 * r0 + r1 * r1 + r2 * r2);
      r[0] = r0 * th;
      r[1] = r1 * th;
      r[2] = r2 * th;
    }
  } else {
    double vth = 1 / (2 * s);
    vth = vth * theta;
    r[0] = rx * vth;
    r[1] = ry * vth;
    r[2] = rz * vth;
  }
}

VO_HD void rodrigues_to_mat(const double (&r)[3], double (&R)[3][3]) {
  const double theta = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (theta < kDblEps) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) R[i][j] = i == j ? 1.0 : 0.0;
    return;
  }
  const double c = cos(theta), s = sin(theta), c1 = 1.0 - c;
  const double it = 1.0 / theta;
  const double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  const double rrt[3][3] = {{x * x, x * y, x * z}, {x * y, y * y, y * z}, {x * z, y * z, z * z}};
  const double rx[3][3] = {{0.0, -z, y}, {z, 0.0, -x}, {-y, x, 0.0}};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) R[i][j] = c * (i == j ? 1.0 : 0.0) + c1 * rrt[i][j] + s * rx[i][j];
}

// RANSACUpdateNumIters (ptsetreg.cpp), in two parts: the logarithms depend only on the
// inlier fraction, so a replay can evaluate them for many counts at once and apply them in
// the serial order (num_iters_apply is the rest of the function, the max_iters cap).
struct ItersTerms {
  double num, denom;
  bool zero;  // denom < DBL_MIN: the function returns 0
};
VO_HD ItersTerms num_iters_terms(double p, double ep, int model_points) {
  p = p > 0. ? p : 0.;
  p = p < 1. ? p : 1.;
  ep = ep > 0. ? ep : 0.;
  ep = ep < 1. ? ep : 1.;
  double num = 1. - p;
  num = num > kDblMin ? num : kDblMin;
  double denom = 1. - pow(1. - ep, (double)model_points);
  if (denom < kDblMin) return {0.0, 0.0, true};
  return {log(num), log(denom), false};
}
VO_HD int num_iters_apply(const ItersTerms& t, int max_iters) {
  if (t.zero) return 0;
  return t.denom >= 0 || -t.num >= max_iters * (-t.denom) ? max_iters : (int)rint(t.num / t.denom);
}
VO_HD int update_num_iters(double p, double ep, int model_points, int max_iters) {
  return num_iters_apply(num_iters_terms(p, ep, model_points), max_iters);
}

VO_HD void se3_exp(const double (&d)[6], double (&R)[3][3], double (&t)[3]) {
  const double px = d[3], py = d[4], pz = d[5];
  const double th = sqrt(px * px + py * py + pz * pz);
  const double K[3][3] = {{0.0, -pz, py}, {pz, 0.0, -px}, {-py, px, 0.0}};
  double K2[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) K2[i][j] = K[i][0] * K[0][j] + K[i][1] * K[1][j] + K[i][2] * K[2][j];
  double a, b, c;
  if (th < 1e-4) {
    a = 1.0;
    b = 0.5;
    c = 1.0 / 6.0;
  } else {
    a = sin(th) / th;
    b = (1 - cos(th)) / (th * th);
    c = (th - sin(th)) / (th * th * th);
  }
  double V[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double I = i == j ? 1.0 : 0.0;
      R[i][j] = I + a * K[i][j] + b * K2[i][j];
      V[i][j] = I + b * K[i][j] + c * K2[i][j];
    }
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = V[i][0] * d[0] + V[i][1] * d[1] + V[i][2] * d[2];
}

// 6x6 SPD solve (Cholesky); false if not positive definite.
VO_HD bool chol_solve6(double (&A)[6][6], const double (&b)[6], double (&x)[6]) {
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double d = A[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) d = d - A[j][k] * A[j][k];
    if (!(d > 0.0)) return false;
    d = sqrt(d);
    A[j][j] = d;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double s = A[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) s = s - A[i][k] * A[j][k];
      A[i][j] = s / d;
    }
  }
  double y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s = s - A[i][k] * y[k];
    y[i] = s / A[i][i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) s = s - A[k][i] * x[k];
    x[i] = s / A[i][i];
  }
  return true;
}



// ---------------------------------------------------------------- scoring and refinement
// cvProjectPoints2Internal without distortion: X = R M + t left to right, z = 1/Z, float32.
VO_HD void project_f32(const double* R, const double* t, const float* M, const Cam& K, float& u, float& v) {
  const double X = M[0], Y = M[1], Z = M[2];
  const double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
  const double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
  const double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
  const double zi = z != 0.0 ? 1.0 / z : 1.0;
  u = (float)((x * zi) * K.fu + K.uc);
  v = (float)((y * zi) * K.fv + K.vc);
}

// PnPRansacCallback::computeError + findInliers: float32 dx*dx + dy*dy <= (float)thr^2.
VO_HD bool is_inlier(const double* R, const double* t, const float* M, float qx, float qy, const Cam& K,
                     float thr2) {
  float u, v;
  project_f32(R, t, M, K, u, v);
  const float dx = qx - u, dy = qy - v;
  const float e = dx * dx + dy * dy;
  return e <= thr2;
}

constexpr int kNe = 28;  // normal equations: 21 (upper J^T J) + 6 (J^T r) + 1 (cost)

// Adds one inlier's terms to the normal equations at (R, t): J = [J_proj | -J_proj [pc]x]
// (left se(3) increment), r = projection - measurement (oracle/pnp_ref.py _normal_eq).
VO_HD void lm_point(const double* R, const double* t, const float* M, float qx, float qy, const Cam& K,
                    double (&acc)[kNe]) {
  const double X = M[0], Y = M[1], Z = M[2];
  const double pc0 = R[0] * X + R[1] * Y + R[2] * Z + t[0];
  const double pc1 = R[3] * X + R[4] * Y + R[5] * Z + t[1];
  const double pc2 = R[6] * X + R[7] * Y + R[8] * Z + t[2];
  const double zi = 1.0 / pc2;
  const double r0 = K.fu * pc0 * zi + K.uc - (double)qx;
  const double r1 = K.fv * pc1 * zi + K.vc - (double)qy;
  const double Jp[2][3] = {{K.fu * zi, 0.0, -K.fu * pc0 * zi * zi}, {0.0, K.fv * zi, -K.fv * pc1 * zi * zi}};
  const double sk[3][3] = {{0.0, -pc2, pc1}, {pc2, 0.0, -pc0}, {-pc1, pc0, 0.0}};
  double J0[6], J1[6];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    J0[c] = Jp[0][c];
    J1[c] = Jp[1][c];
    J0[3 + c] = -(Jp[0][0] * sk[0][c] + Jp[0][1] * sk[1][c] + Jp[0][2] * sk[2][c]);
    J1[3 + c] = -(Jp[1][0] * sk[0][c] + Jp[1][1] * sk[1][c] + Jp[1][2] * sk[2][c]);
  }
  int e = 0;
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int c = r; c < 6; ++c) acc[e++] += J0[r] * J0[c] + J1[r] * J1[c];
#pragma unroll
  for (int r = 0; r < 6; ++r) acc[21 + r] += J0[r] * r0 + J1[r] * r1;
  acc[27] += r0 * r0 + r1 * r1;
}

// 10^e for CvLevMarq's lambda, e in [-16, 16] (decimal literals: correctly rounded, equal to
// Python's 10.0 ** e).
VO_HD double pow10i(int e) {
  switch (e) {
    case -16: return 1e-16; case -15: return 1e-15; case -14: return 1e-14; case -13: return 1e-13;
    case -12: return 1e-12; case -11: return 1e-11; case -10: return 1e-10; case -9: return 1e-9;
    case -8: return 1e-8;   case -7: return 1e-7;   case -6: return 1e-6;   case -5: return 1e-5;
    case -4: return 1e-4;   case -3: return 1e-3;   case -2: return 1e-2;   case -1: return 1e-1;
    case 0: return 1e0;     case 1: return 1e1;     case 2: return 1e2;     case 3: return 1e3;
    case 4: return 1e4;     case 5: return 1e5;     case 6: return 1e6;     case 7: return 1e7;
    case 8: return 1e8;     case 9: return 1e9;     case 10: return 1e10;   case 11: return 1e11;
    case 12: return 1e12;   case 13: return 1e13;   case 14: return 1e14;   case 15: return 1e15;
    default: return 1e16;
  }
}

// Levenberg-Marquardt control of oracle/pnp_ref.py refine_lm (CvLevMarq's schedule): the
// caller evaluates the normal equations at the poses this proposes.
struct LmState {
  double R[9], t[3], A[21], g[6], cost, delta[6];
  int lg, accepted;

  VO_HD void init(const double* R0, const double* t0, const double* ne) {
    for (int k = 0; k < 9; ++k) R[k] = R0[k];
    for (int k = 0; k < 3; ++k) t[k] = t0[k];
    for (int k = 0; k < 21; ++k) A[k] = ne[k];
    for (int k = 0; k < 6; ++k) g[k] = ne[21 + k];
    cost = ne[27];
    lg = -3;
    accepted = 0;
  }
  // Candidate (nR, nt) = exp(delta^) (R, t) with (A + lambda diag A) delta = -g; false when
  // the refinement is over (20 accepted steps, or the damped system is not SPD).
  VO_HD bool propose(double* nR, double* nt) {
    if (accepted >= kLmMaxIters) return false;
    const double lam = pow10i(lg);
    double An[6][6];
    int e = 0;
    for (int r = 0; r < 6; ++r)
      for (int c = r; c < 6; ++c) {
        An[r][c] = A[e];
        An[c][r] = A[e];
        ++e;
      }
    for (int r = 0; r < 6; ++r) An[r][r] = An[r][r] * (1.0 + lam);
    double ng[6];
    for (int r = 0; r < 6; ++r) ng[r] = -g[r];
    if (!chol_solve6(An, ng, delta)) return false;
    double dR[3][3], dt[3];
    se3_exp(delta, dR, dt);
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) nR[3 * i + j] = dR[i][0] * R[j] + dR[i][1] * R[3 + j] + dR[i][2] * R[6 + j];
      nt[i] = dR[i][0] * t[0] + dR[i][1] * t[1] + dR[i][2] * t[2] + dt[i];
    }
    return true;
  }
  // Accepts or rejects the candidate given its normal equations; false when done.
  VO_HD bool update(const double* nR, const double* nt, const double* ne) {
    const double costn = ne[27];
    if (costn <= cost) {
      const double dn = sqrt(delta[0] * delta[0] + delta[1] * delta[1] + delta[2] * delta[2] +
                             delta[3] * delta[3] + delta[4] * delta[4] + delta[5] * delta[5]);
      const double tn = sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
      const bool small = dn <= kFltEps * (1.0 + tn);
      for (int k = 0; k < 9; ++k) R[k] = nR[k];
      for (int k = 0; k < 3; ++k) t[k] = nt[k];
      for (int k = 0; k < 21; ++k) A[k] = ne[k];
      for (int k = 0; k < 6; ++k) g[k] = ne[21 + k];
      cost = costn;
      lg = lg - 1 > -16 ? lg - 1 : -16;
      ++accepted;
      return !small;
    }
    ++lg;
    return lg <= 16;
  }
};

}  // namespace pnpm
}  // namespace vo
