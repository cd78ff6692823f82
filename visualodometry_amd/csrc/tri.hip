// Two-view triangulation with the reference's filters on gfx950.
//
// Replaces triangulate_points (reference src/modules/frontend.py:115-148): the DLT of
// cv2.triangulatePoints (OpenCV icvTriangulatePoints: for each point the 4x4 matrix
// rows x_j P_j[2] - P_j[0] and y_j P_j[2] - P_j[1] in double, the right singular vector
// of its smallest singular value as the homogeneous point, stored as float32 like the
// image points), the float32 dehomogenisation (:131), the depth test in camera 2
// (:134-135) and the reprojection error of cv2.projectPoints in image 2 (:139-143).
// One thread per point; the 4x4 SVD is a one-sided Jacobi iteration in fp64 on the
// columns of A (no normal equations: A^T A would square the conditioning).  The
// projection follows OpenCV's cvProjectPoints2Internal with no distortion operation
// for operation (no FMA contraction), so masks match the restatement in
// oracle/triangulate_ref.py.
#include "vo_ctx.h"

namespace vo {
namespace {

struct TriArgs {
  double P1[12], P2[12], R2[9], t2[3];
  double fx, fy, cx, cy, min_depth;
  float max_err;
  int n;
  const float2* pts1;
  const float2* pts2;
  float* pts3d;    // n x 3
  uint8_t* mask;   // n
};

constexpr int kTriSweeps = 12;  // cap on one-sided Jacobi sweeps (4 columns: converged in ~5)

__global__ __launch_bounds__(256) void tri_kernel(TriArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const float2 q1 = a.pts1[i], q2 = a.pts2[i];
  // DLT rows (double, two roundings each as in OpenCV)
  double A[4][4];
  {
    const double x1 = q1.x, y1 = q1.y, x2 = q2.x, y2 = q2.y;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      A[0][k] = __dsub_rn(__dmul_rn(x1, a.P1[8 + k]), a.P1[k]);
      A[1][k] = __dsub_rn(__dmul_rn(y1, a.P1[8 + k]), a.P1[4 + k]);
      A[2][k] = __dsub_rn(__dmul_rn(x2, a.P2[8 + k]), a.P2[k]);
      A[3][k] = __dsub_rn(__dmul_rn(y2, a.P2[8 + k]), a.P2[4 + k]);
    }
  }
  double V[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) V[r][c] = r == c ? 1.0 : 0.0;
  // one-sided Jacobi: rotate column pairs of A (and V) until they are orthogonal
  for (int sweep = 0; sweep < kTriSweeps; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        double al = 0.0, be = 0.0, ga = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          al += A[r][p] * A[r][p];
          be += A[r][q] * A[r][q];
          ga += A[r][p] * A[r][q];
        }
        if (fabs(ga) > 1e-15 * sqrt(al * be)) {  // columns not yet orthogonal to ~4 ulp
          rotated = true;
          const double zeta = (be - al) / (2.0 * ga);
          const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
          const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double ap = A[r][p], aq = A[r][q];
            A[r][p] = c * ap - s * aq;
            A[r][q] = s * ap + c * aq;
            const double vp = V[r][p], vq = V[r][q];
            V[r][p] = c * vp - s * vq;
            V[r][q] = s * vp + c * vq;
          }
        }
      }
    if (!__any(rotated)) break;  // the whole wave has converged
  }
  // the column of V whose image has the smallest norm (smallest singular value)
  double best = 0.0, h[4] = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const double nrm = A[0][c] * A[0][c] + A[1][c] * A[1][c] + A[2][c] * A[2][c] + A[3][c] * A[3][c];
    const bool take = c == 0 || nrm < best;
    best = take ? nrm : best;
#pragma unroll
    for (int r = 0; r < 4; ++r) h[r] = take ? V[r][c] : h[r];
  }
  // points4D is float32; dehomogenise in float32 (sign of h cancels)
  const float hw = (float)h[3];
  const float X = __fdiv_rn((float)h[0], hw), Y = __fdiv_rn((float)h[1], hw), Z = __fdiv_rn((float)h[2], hw);
  a.pts3d[3l * i] = X;
  a.pts3d[3l * i + 1] = Y;
  a.pts3d[3l * i + 2] = Z;
  const double Xd = X, Yd = Y, Zd = Z;
  // cv2.projectPoints(pts3d, R2, t2, K, None): X = R M + t left to right, z = 1/Z, x *= z
  const double* R = a.R2;
  const double xc = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(R[0], Xd), __dmul_rn(R[1], Yd)), __dmul_rn(R[2], Zd)), a.t2[0]);
  const double yc = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(R[3], Xd), __dmul_rn(R[4], Yd)), __dmul_rn(R[5], Zd)), a.t2[1]);
  const double zc = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(R[6], Xd), __dmul_rn(R[7], Yd)), __dmul_rn(R[8], Zd)), a.t2[2]);
  const double zi = zc != 0.0 ? __ddiv_rn(1.0, zc) : 1.0;
  const double xn = __dmul_rn(xc, zi), yn = __dmul_rn(yc, zi);
  const float u = (float)__dadd_rn(__dmul_rn(xn, a.fx), a.cx);
  const float v = (float)__dadd_rn(__dmul_rn(yn, a.fy), a.cy);
  const float du = __fsub_rn(u, q2.x), dv = __fsub_rn(v, q2.y);
  // correctly rounded sqrtf (__fsqrt_rn is the approximate native sqrt in this HIP)
  const float err = (float)sqrt((double)__fadd_rn(__fmul_rn(du, du), __fmul_rn(dv, dv)));
  a.mask[i] = (zc > a.min_depth && err < a.max_err) ? 1 : 0;
}

}  // namespace

void tri_run(vo_ctx* ctx, const double* P1, const double* P2, const double* T_cw2, const double* K,
             const float* d_pts1, const float* d_pts2, int n, double min_depth, double max_reproj_err,
             float* d_pts3d, uint8_t* d_mask) {
  VO_REQUIRE(n >= 0, VO_ERR_ARG, "triangulate: n=%d", n);
  if (n == 0) return;
  TriArgs a;
  for (int e = 0; e < 12; ++e) {
    a.P1[e] = P1[e];
    a.P2[e] = P2[e];
  }
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) a.R2[3 * r + c] = T_cw2[4 * r + c];
    a.t2[r] = T_cw2[4 * r + 3];
  }
  a.fx = K[0];
  a.cx = K[2];
  a.fy = K[4];
  a.cy = K[5];
  a.min_depth = min_depth;
  a.max_err = (float)max_reproj_err;  // err (float32) < threshold: the comparison numpy makes
  a.n = n;
  a.pts1 = reinterpret_cast<const float2*>(d_pts1);
  a.pts2 = reinterpret_cast<const float2*>(d_pts2);
  a.pts3d = d_pts3d;
  a.mask = d_mask;
  ctx->prof.begin(ctx->stream, kKTriangulate);
  hipLaunchKernelGGL(tri_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, ctx->stream, a);
  ctx->prof.end(ctx->stream);
  VO_HIP_CHECK(hipGetLastError());
}

}  // namespace vo
