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
//   pnp_score_kernel  one workgroup per (frame, hypothesis): float32 reprojection error
//                     of every point, inlier count;
//   pnp_final_kernel  one workgroup per frame: RANSAC replay (best model, niters update),
//                     inlier mask of the best model, Levenberg-Marquardt refinement on the
//                     inliers (fixed-order block reductions), Rodrigues to rvec.
#include <cmath>
#include <cstring>
#include <vector>

#include "vo_ctx.h"

#pragma clang fp contract(off)

namespace vo {
namespace {

constexpr int kPts = 5;            // EPnP model points (solvePnPRansac: model_points = 5)
constexpr int kModel = 16;         // doubles per model: R (9), t (3), rvec (3), valid (1)
constexpr double kDblEps = 2.220446049250313e-16;
constexpr double kDblMin = 2.2250738585072014e-308;
constexpr double kFltEps = 1.1920928955078125e-07;
constexpr int kLmMaxIters = 20;
// CvLevMarq's lambda = 10^lg, lg in [-16, 16] (decimal literals: correctly rounded)
__constant__ double kPow10[33] = {1e-16, 1e-15, 1e-14, 1e-13, 1e-12, 1e-11, 1e-10, 1e-9, 1e-8, 1e-7, 1e-6,
                                  1e-5,  1e-4,  1e-3,  1e-2,  1e-1,  1e0,   1e1,   1e2,  1e3,  1e4,  1e5,
                                  1e6,   1e7,   1e8,   1e9,   1e10,  1e11,  1e12,  1e13, 1e14, 1e15, 1e16};

struct Cam {
  double fu, fv, uc, vc;
};

// ---------------------------------------------------------------- Jacobi SVD
// JacobiSVDImpl_ (OpenCV core/lapack.cpp) on the rows of A (rotated in place): W[i] ends
// as the norm of row i (unsorted); Vt accumulates the rotations when WANT_V.
template <int N, int M, bool WANT_V>
__device__ __forceinline__ void jacobi_rows(double (&A)[N][M], double (&W)[N], double (&Vt)[N][N]) {
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
          const double beta = a - b, gamma = hypot(p, beta);
          double c, s;
          if (beta < 0) {
            const double delta = (gamma - beta) * 0.5;
            s = sqrt(delta / gamma);
            c = p / (gamma * s * 2.0);
          } else {
            c = sqrt((gamma + beta) / (gamma * 2.0));
            s = p / (gamma * c * 2.0);
          }
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

// Position of each singular value in the descending order (the selection sort of
// JacobiSVDImpl_; equal values keep their index order, which the selection sort also
// does unless three or more tie -- never for the non-degenerate inputs used here).
template <int N>
__device__ __forceinline__ void desc_rank(const double (&W)[N], int (&rank)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    int r = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) r += (W[k] > W[i] || (k < i && W[k] == W[i])) ? 1 : 0;
    rank[i] = r;
  }
}

// ---------------------------------------------------------------- EPnP helpers
__device__ __forceinline__ double dot3(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// epnp::qr_solve (Householder least squares); X is left unchanged if a column is zero.
template <int NR, int NC>
__device__ __forceinline__ void qr_solve(double (&A)[NR][NC], double (&b)[NR], double (&X)[NC]) {
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

struct EpnpState {
  double pw[kPts][3];
  double us[kPts][2];
  double alphas[kPts][4];
  double cws[4][3];
  double v[4][12];  // v[i] = ut row 11 - i (right singular vectors, smallest first)
  double L[6][10];
  double rho[6];
};

__device__ __forceinline__ void gauss_newton(const EpnpState& S, double (&betas)[4]) {
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
__device__ __forceinline__ double compute_R_and_t(const EpnpState& S, const Cam& K, const double (&betas)[4],
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
      for (int k = 0; k < 3; ++k) ccs[j][k] = ccs[j][k] + betas[i] * S.v[i][3 * j + k];
  double pcs[kPts][3];
#pragma unroll
  for (int p = 0; p < kPts; ++p)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      pcs[p][k] = S.alphas[p][0] * ccs[0][k] + S.alphas[p][1] * ccs[1][k] + S.alphas[p][2] * ccs[2][k] +
                  S.alphas[p][3] * ccs[3][k];
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
    const double Xc = dot3(R[0], S.pw[p]) + t[0];
    const double Yc = dot3(R[1], S.pw[p]) + t[1];
    const double inv_Zc = 1.0 / (dot3(R[2], S.pw[p]) + t[2]);
    const double ue = K.uc + K.fu * Xc * inv_Zc;
    const double ve = K.vc + K.fv * Yc * inv_Zc;
    const double du = S.us[p][0] - ue, dv = S.us[p][1] - ve;
    err = err + sqrt(du * du + dv * dv);
  }
  return err / kPts;
}

// epnp::compute_pose on 5 correspondences.  Returns false for a degenerate subset.
__device__ bool epnp5(EpnpState& S, const Cam& K, double (&R)[3][3], double (&t)[3]) {
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
#pragma unroll
      for (int j = 0; j < 3; ++j) S.alphas[p][1 + j] = ci[j][0] * d0 + ci[j][1] * d1 + ci[j][2] * d2;
      S.alphas[p][0] = 1.0 - S.alphas[p][1] - S.alphas[p][2] - S.alphas[p][3];
    }
  }
  // M (2n x 12), M^T M, its four smallest right singular vectors
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
        const double al = S.alphas[p][c];
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
    jacobi_rows<12, 12, false>(A, W, dummy);  // M^T M is symmetric: its rows are A^T's
    int rk[12];
    desc_rank<12>(W, rk);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      ok &= W[i] > kDblMin;
      const double s = 1.0 / W[i];
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        const double val = A[i][k] * s;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (rk[i] == 11 - q) S.v[q][k] = val;
      }
    }
  }
  // compute_L_6x10, compute_rho
  {
    constexpr int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
    double dv[4][6][3];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j)
#pragma unroll
        for (int k = 0; k < 3; ++k) dv[i][j][k] = S.v[i][3 * pa[j] + k] - S.v[i][3 * pb[j] + k];
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
      double e[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) e[k] = S.cws[pa[i]][k] - S.cws[pb[i]][k];
      S.rho[i] = dot3(e, e);
    }
  }
  // three beta approximations, each refined by Gauss-Newton; keep the lowest error
  double bestR[3][3], bestt[3], best_err = 0.0;
  for (int kind = 1; kind <= 3; ++kind) {
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
    double Rk[3][3], tk[3];
    const double e = compute_R_and_t(S, K, betas, Rk, tk);
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
__device__ void rodrigues_to_vec(const double (&Rin)[3][3], double (&r)[3]) {
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

__device__ void rodrigues_to_mat(const double (&r)[3], double (&R)[3][3]) {
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

// ---------------------------------------------------------------- kernels
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

__device__ __forceinline__ float2 project_f32(const double* R, const double* t, float3 Xf, const Cam& K) {
  const double X = Xf.x, Y = Xf.y, Z = Xf.z;
  const double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
  const double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
  const double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
  const double zi = z != 0.0 ? 1.0 / z : 1.0;
  return make_float2((float)((x * zi) * K.fu + K.uc), (float)((y * zi) * K.fv + K.vc));
}

__device__ __forceinline__ bool is_inlier(const double* R, const double* t, float3 X, float2 q, const Cam& K,
                                          float thr2) {
  const float2 p = project_f32(R, t, X, K);
  const float dx = q.x - p.x, dy = q.y - p.y;
  const float e = dx * dx + dy * dy;
  return e <= thr2;
}

__device__ __forceinline__ float3 load3(const float* X, int i) {
  return make_float3(X[3l * i], X[3l * i + 1], X[3l * i + 2]);
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
    const float3 X = load3(a.X, i);
    S.pw[p][0] = X.x;
    S.pw[p][1] = X.y;
    S.pw[p][2] = X.z;
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

__global__ __launch_bounds__(256) void pnp_score_kernel(PnpArgs a) {
  const int g = blockIdx.x;  // (frame, hypothesis)
  const int f = g / a.H;
  const int o = a.off[f], n = a.off[f + 1] - o;
  const double* model = a.models + (size_t)g * kModel;
  __shared__ int s_count;
  if (threadIdx.x == 0) s_count = 0;
  __syncthreads();
  if (model[15] != 0.0 && n > kPts) {
    double R[9], t[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = model[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = model[9 + k];
    int cnt = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
      const float2 q = reinterpret_cast<const float2*>(a.uv)[o + i];
      cnt += is_inlier(R, t, load3(a.X, o + i), q, a.K, a.thr2) ? 1 : 0;
    }
    if (cnt) atomicAdd(&s_count, cnt);
  }
  __syncthreads();
  if (threadIdx.x == 0) a.counts[g] = s_count;
}

// RANSACUpdateNumIters (ptsetreg.cpp)
__device__ int update_num_iters(double p, double ep, int model_points, int max_iters) {
  p = p > 0. ? p : 0.;
  p = p < 1. ? p : 1.;
  ep = ep > 0. ? ep : 0.;
  ep = ep < 1. ? ep : 1.;
  double num = 1. - p;
  num = num > kDblMin ? num : kDblMin;
  double denom = 1. - pow(1. - ep, (double)model_points);
  if (denom < kDblMin) return 0;
  num = log(num);
  denom = log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)rint(num / denom);
}

// Sum of one double over a wave in a fixed order (butterfly).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = v + __shfl_xor(v, m, 64);
  return v;
}

constexpr int kNe = 28;  // 21 (upper J^T J) + 6 (J^T r) + 1 (cost)

// Normal equations of the inliers at (R, t): the partial sums of this thread.
__device__ __forceinline__ void lm_accumulate(const PnpArgs& a, int o, int n, const double* R, const double* t,
                                              double (&acc)[kNe]) {
#pragma unroll
  for (int k = 0; k < kNe; ++k) acc[k] = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    if (!a.mask[o + i]) continue;
    const float3 Xf = load3(a.X, o + i);
    const float2 q = reinterpret_cast<const float2*>(a.uv)[o + i];
    const double X = Xf.x, Y = Xf.y, Z = Xf.z;
    const double pc0 = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    const double pc1 = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    const double pc2 = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    const double zi = 1.0 / pc2;
    const double r0 = a.K.fu * pc0 * zi + a.K.uc - (double)q.x;
    const double r1 = a.K.fv * pc1 * zi + a.K.vc - (double)q.y;
    // J = [J_proj | -J_proj [pc]x]  (left se(3) increment, as oracle/pnp_ref.py _normal_eq)
    const double Jp[2][3] = {{a.K.fu * zi, 0.0, -a.K.fu * pc0 * zi * zi}, {0.0, a.K.fv * zi, -a.K.fv * pc1 * zi * zi}};
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

__device__ void se3_exp(const double (&d)[6], double (&R)[3][3], double (&t)[3]) {
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
__device__ bool chol_solve6(double (&A)[6][6], const double (&b)[6], double (&x)[6]) {
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

__global__ __launch_bounds__(256) void pnp_final_kernel(PnpArgs a) {
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
    const bool in = is_inlier(R, t, load3(a.X, o + i), q, a.K, a.thr2);
    a.mask[o + i] = in ? 1 : 0;
    cnt += in ? 1 : 0;
  }
  if (cnt) atomicAdd(&s_count, cnt);
  // lm_accumulate reads mask[o + i] for the same i this thread wrote (same stride)
  // Levenberg-Marquardt on the inliers (oracle/pnp_ref.py refine_lm)
  double acc[kNe];
  lm_accumulate(a, o, n, R, t, acc);
  lm_reduce(acc, s_red, s_ne);
  // thread 0 keeps the LM state
  double cR[3][3], ct[3], A[21], g[6], cost = 0.0;
  int lg = -3, accepted = 0;
  double delta[6];
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      ct[i] = t[i];
#pragma unroll
      for (int j = 0; j < 3; ++j) cR[i][j] = R[3 * i + j];
    }
#pragma unroll
    for (int k = 0; k < 21; ++k) A[k] = s_ne[k];
#pragma unroll
    for (int k = 0; k < 6; ++k) g[k] = s_ne[21 + k];
    cost = s_ne[27];
  }
  for (;;) {
    if (threadIdx.x == 0) {
      int go = 0;
      if (accepted < kLmMaxIters) {
        const double lam = kPow10[lg + 16];
        double An[6][6];
        int e = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
          for (int c = r; c < 6; ++c) {
            An[r][c] = An[c][r] = A[e++];
          }
#pragma unroll
        for (int r = 0; r < 6; ++r) An[r][r] = An[r][r] * (1.0 + lam);
        double ng[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) ng[r] = -g[r];
        if (chol_solve6(An, ng, delta)) {
          double dR[3][3], dt[3];
          se3_exp(delta, dR, dt);
#pragma unroll
          for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = 0; j < 3; ++j) s_R[3 * i + j] = dR[i][0] * cR[0][j] + dR[i][1] * cR[1][j] + dR[i][2] * cR[2][j];
            s_t[i] = dR[i][0] * ct[0] + dR[i][1] * ct[1] + dR[i][2] * ct[2] + dt[i];
          }
          go = 1;
        }
      }
      s_go = go;
    }
    __syncthreads();
    if (!s_go) break;
    double nR[9], nt[3];
#pragma unroll
    for (int k = 0; k < 9; ++k) nR[k] = s_R[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) nt[k] = s_t[k];
    lm_accumulate(a, o, n, nR, nt, acc);
    lm_reduce(acc, s_red, s_ne);
    int stop = 0;
    if (threadIdx.x == 0) {
      const double costn = s_ne[27];
      if (costn <= cost) {
        const double dn = sqrt(delta[0] * delta[0] + delta[1] * delta[1] + delta[2] * delta[2] +
                               delta[3] * delta[3] + delta[4] * delta[4] + delta[5] * delta[5]);
        const double tn = sqrt(ct[0] * ct[0] + ct[1] * ct[1] + ct[2] * ct[2]);
        const bool small = dn <= kFltEps * (1.0 + tn);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          ct[i] = nt[i];
#pragma unroll
          for (int j = 0; j < 3; ++j) cR[i][j] = nR[3 * i + j];
        }
#pragma unroll
        for (int k = 0; k < 21; ++k) A[k] = s_ne[k];
#pragma unroll
        for (int k = 0; k < 6; ++k) g[k] = s_ne[21 + k];
        cost = costn;
        lg = lg - 1 > -16 ? lg - 1 : -16;
        ++accepted;
        stop = small ? 1 : 0;
      } else {
        ++lg;
        stop = lg > 16 ? 1 : 0;
      }
      s_go = !stop;
    }
    __syncthreads();
    if (!s_go) break;
  }
  if (threadIdx.x == 0) {
    double rv[3];
    rodrigues_to_vec(cR, rv);
    for (int k = 0; k < 3; ++k) {
      a.pose[6 * f + k] = rv[k];
      a.pose[6 * f + 3 + k] = ct[k];
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
  hipLaunchKernelGGL(pnp_score_kernel, dim3(nh), dim3(256), 0, ctx->stream, a);
  ctx->prof.end(ctx->stream);
  VO_HIP_CHECK(hipGetLastError());
  ctx->prof.begin(ctx->stream, kKPnpFinal);
  hipLaunchKernelGGL(pnp_final_kernel, dim3(batch), dim3(256), 0, ctx->stream, a);
  ctx->prof.end(ctx->stream);
  VO_HIP_CHECK(hipGetLastError());
}

}  // namespace vo
