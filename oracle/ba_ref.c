/*
 * CPU oracle / CPU baseline for the sliding-window BA Gauss-Newton step --
 * TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py
 * cpu_baseline leg); never linked into the product library.
 *
 * The reference has no BA (pyceres/pycolmap declared in pyproject.toml:11-12,
 * never imported): parity with the reference is unpinned.  This
 * is a second, independent restatement of oracle/ba_ref.py (same model:
 * projection of reference src/modules/frontend.py:128-140, T_cw convention of
 * src/modules/vo.py:260-261), written the straightforward dense way: explicit
 * 3x3 inverses V^-1, a dense reduced camera matrix S accumulated per thread,
 * a dense right-looking Cholesky.  tests/test_oracle_ba.py pins it against the
 * numpy oracle, which is itself pinned by finite differences, a full-system
 * solve and scipy.optimize.least_squares.
 *
 * Layouts: poses (N,12) = R_cw row-major (9) + t_cw (3); points (L,3);
 * observations CSR by point (point_ptr), obs_uv (M,2) float32.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PIVOT_REL_EPS 1e-12 /* == ba_ref.py */
#define EXP_TAYLOR 1e-4     /* == ba_ref.py */

typedef struct {
  double pc[3], r[2], Jc[12], Jp[6];
} lin_t;

static void linearize(const double* T, const double* X, const float* uv, double fx, double fy,
                      double cx, double cy, lin_t* o) {
  const double x = T[0] * X[0] + T[1] * X[1] + T[2] * X[2] + T[9];
  const double y = T[3] * X[0] + T[4] * X[1] + T[5] * X[2] + T[10];
  const double z = T[6] * X[0] + T[7] * X[1] + T[8] * X[2] + T[11];
  o->pc[0] = x; o->pc[1] = y; o->pc[2] = z;
  o->r[0] = fx * x / z + cx - (double)uv[0];
  o->r[1] = fy * y / z + cy - (double)uv[1];
  /* Jproj = [[fx/z, 0, -fx x/z^2], [0, fy/z, -fy y/z^2]];  d pc / d(rho,phi) = [I | -[pc]x] */
  const double P[2][3] = {{fx / z, 0.0, -fx * x / (z * z)}, {0.0, fy / z, -fy * y / (z * z)}};
  const double D[3][6] = {{1, 0, 0, 0, z, -y}, {0, 1, 0, -z, 0, x}, {0, 0, 1, y, -x, 0}};
  for (int k = 0; k < 2; ++k) {
    for (int c = 0; c < 6; ++c)
      o->Jc[6 * k + c] = P[k][0] * D[0][c] + P[k][1] * D[1][c] + P[k][2] * D[2][c];
    for (int c = 0; c < 3; ++c)
      o->Jp[3 * k + c] = P[k][0] * T[c] + P[k][1] * T[3 + c] + P[k][2] * T[6 + c];
  }
}

static int point_valid(const double V[9]) {
  const double eps = PIVOT_REL_EPS * (V[0] + V[4] + V[8]);
  int ok = V[0] > eps;
  const double l00 = sqrt(ok ? V[0] : 1.0);
  const double l10 = V[1] / l00, l20 = V[2] / l00;
  const double d1 = V[4] - l10 * l10;
  ok = ok && d1 > eps;
  const double l11 = sqrt(ok ? d1 : 1.0);
  const double l21 = (V[5] - l20 * l10) / l11;
  const double d2 = V[8] - l20 * l20 - l21 * l21;
  return ok && d2 > eps;
}

static void inv3(const double m[9], double o[9]) {
  const double c00 = m[4] * m[8] - m[5] * m[7], c01 = m[5] * m[6] - m[3] * m[8],
               c02 = m[3] * m[7] - m[4] * m[6];
  const double det = m[0] * c00 + m[1] * c01 + m[2] * c02, id = 1.0 / det;
  o[0] = c00 * id; o[1] = (m[2] * m[7] - m[1] * m[8]) * id; o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
  o[3] = c01 * id; o[4] = (m[0] * m[8] - m[2] * m[6]) * id; o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
  o[6] = c02 * id; o[7] = (m[1] * m[6] - m[0] * m[7]) * id; o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

static void se3_apply(const double d[6], const double* T, double* out) {
  const double th2 = d[3] * d[3] + d[4] * d[4] + d[5] * d[5], th = sqrt(th2);
  double A, B, C;
  if (th < EXP_TAYLOR) {
    A = 1.0 - th2 / 6.0; B = 0.5 - th2 / 24.0; C = 1.0 / 6.0 - th2 / 120.0;
  } else {
    A = sin(th) / th; B = (1.0 - cos(th)) / (th * th); C = (th - sin(th)) / (th * th * th);
  }
  const double K[9] = {0, -d[5], d[4], d[5], 0, -d[3], -d[4], d[3], 0};
  double K2[9], R[9], V[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      K2[3 * i + j] = K[3 * i] * K[j] + K[3 * i + 1] * K[3 + j] + K[3 * i + 2] * K[6 + j];
  for (int e = 0; e < 9; ++e) {
    const double I = (e % 4 == 0) ? 1.0 : 0.0;
    R[e] = I + A * K[e] + B * K2[e];
    V[e] = I + B * K[e] + C * K2[e];
  }
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      out[3 * i + j] = R[3 * i] * T[j] + R[3 * i + 1] * T[3 + j] + R[3 * i + 2] * T[6 + j];
    out[9 + i] = R[3 * i] * T[9] + R[3 * i + 1] * T[10] + R[3 * i + 2] * T[11] +
                 V[3 * i] * d[0] + V[3 * i + 1] * d[1] + V[3 * i + 2] * d[2];
  }
}

/* Lower Cholesky in place + solve; returns 0 if S is not positive definite.  The
 * arithmetic is the dense algorithm's, term for term; entries outside the envelope of S
 * (left of each row's first nonzero, which the factor keeps) are exact zeros, and the
 * loops skip them, so the result is bitwise the dense one at O(n bw^2) instead of O(n^3)
 * (the CPU baseline then pays for the arithmetic S needs, not for zeros). */
static int chol_solve(double* S, int n, double* x, int nthreads) {
  (void)nthreads;
  int* first = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  int* last = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  for (int i = 0; i < n; ++i) {
    int f = i;
    for (int j = 0; j < i; ++j)
      if (S[(int64_t)i * n + j] != 0.0) {
        f = j;
        break;
      }
    first[i] = f;
    last[i] = i;
  }
  for (int i = 0; i < n; ++i)
    for (int k = first[i]; k < i; ++k)
      if (last[k] < i) last[k] = i;
  int ok = 1;
  for (int k = 0; k < n && ok; ++k) {
    const double d = S[(int64_t)k * n + k];
    if (!(d > 0.0)) {
      ok = 0;
      break;
    }
    const double l = sqrt(d), il = 1.0 / l;
    S[(int64_t)k * n + k] = l;
    for (int i = k + 1; i <= last[k]; ++i) S[(int64_t)i * n + k] *= il;
    for (int i = k + 1; i <= last[k]; ++i) {
      if (first[i] > k) continue;  /* l_ik == 0 */
      const double lik = S[(int64_t)i * n + k];
      double* row = S + (int64_t)i * n;
      for (int j = k + 1; j <= i; ++j)
        if (first[j] <= k) row[j] -= lik * S[(int64_t)j * n + k];
    }
  }
  if (ok) {
    for (int i = 0; i < n; ++i) {
      double s = x[i];
      for (int m = first[i]; m < i; ++m) s -= S[(int64_t)i * n + m] * x[m];
      x[i] = s / S[(int64_t)i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
      double s = x[i];
      for (int m = i + 1; m <= last[i]; ++m) s -= S[(int64_t)m * n + i] * x[m];
      x[i] = s / S[(int64_t)i * n + i];
    }
  }
  free(first);
  free(last);
  return ok;
}

typedef struct {
  double* S;  /* n*n */
  double* b;  /* n */
  double cost;
} partial_t;

/* One GN step.  Outputs (may be NULL): S_out (n*n, before factorisation), b_out,
 * dc_out (n).  Returns 1 on success, 0 if S is not SPD (state unchanged). */
int oracle_ba_step(int N, int L, int n_fixed, double fx, double fy, double cx, double cy,
                   double lam, const int32_t* point_ptr, const int32_t* obs_cam,
                   const float* obs_uv, double* poses, double* points, double* cost_out,
                   double* S_out, double* b_out, double* dc_out, int nthreads) {
  const int F = N - n_fixed, n = 6 * F;
  const int M = point_ptr[L];
  double* Wobs = (double*)malloc(sizeof(double) * 18 * (size_t)(M > 0 ? M : 1));
  double* Vinv = (double*)calloc(9 * (size_t)(L > 0 ? L : 1), sizeof(double));
  double* gp = (double*)calloc(3 * (size_t)(L > 0 ? L : 1), sizeof(double));
  unsigned char* pvalid = (unsigned char*)calloc((size_t)(L > 0 ? L : 1), 1);
  int nt = nthreads > 0 ? nthreads : 1;
  partial_t* part = (partial_t*)calloc(nt, sizeof(partial_t));
#pragma omp parallel num_threads(nt)
  {
    const int tid = omp_get_thread_num();
    partial_t* P = &part[tid];
    P->S = (double*)calloc((size_t)n * n + 1, sizeof(double));
    P->b = (double*)calloc((size_t)n + 1, sizeof(double));
    P->cost = 0.0;
    lin_t lin;
#pragma omp for schedule(static)
    for (int p = 0; p < L; ++p) {
      const int o0 = point_ptr[p], o1 = point_ptr[p + 1];
      double V[9] = {0}, g[3] = {0};
      for (int o = o0; o < o1; ++o) {
        linearize(poses + 12 * obs_cam[o], points + 3 * p, obs_uv + 2 * o, fx, fy, cx, cy, &lin);
        P->cost += lin.r[0] * lin.r[0] + lin.r[1] * lin.r[1];
        for (int i = 0; i < 3; ++i) {
          g[i] += lin.Jp[i] * lin.r[0] + lin.Jp[3 + i] * lin.r[1];
          for (int j = 0; j < 3; ++j) V[3 * i + j] += lin.Jp[i] * lin.Jp[j] + lin.Jp[3 + i] * lin.Jp[3 + j];
        }
        double* W = Wobs + 18 * (int64_t)o;
        for (int a = 0; a < 6; ++a)
          for (int c = 0; c < 3; ++c) W[3 * a + c] = lin.Jc[a] * lin.Jp[c] + lin.Jc[6 + a] * lin.Jp[3 + c];
      }
      V[0] += lam; V[4] += lam; V[8] += lam;
      memcpy(gp + 3 * p, g, sizeof g);
      if (!point_valid(V)) continue;  /* frozen: leaves the camera system */
      pvalid[p] = 1;
      double Vi[9];
      inv3(V, Vi);
      memcpy(Vinv + 9 * p, Vi, sizeof Vi);
      for (int o = o0; o < o1; ++o) {
        const int ci = obs_cam[o] - n_fixed;
        if (ci < 0) continue;
        linearize(poses + 12 * obs_cam[o], points + 3 * p, obs_uv + 2 * o, fx, fy, cx, cy, &lin);
        const double* Wo = Wobs + 18 * (int64_t)o;
        double Y[18];
        for (int a = 0; a < 6; ++a)
          for (int c = 0; c < 3; ++c)
            Y[3 * a + c] = Wo[3 * a] * Vi[c] + Wo[3 * a + 1] * Vi[3 + c] + Wo[3 * a + 2] * Vi[6 + c];
        for (int a = 0; a < 6; ++a) {
          P->b[6 * ci + a] += -(lin.Jc[a] * lin.r[0] + lin.Jc[6 + a] * lin.r[1]) +
                              Y[3 * a] * g[0] + Y[3 * a + 1] * g[1] + Y[3 * a + 2] * g[2];
          for (int c = 0; c < 6; ++c)
            P->S[(int64_t)(6 * ci + a) * n + 6 * ci + c] +=
                lin.Jc[a] * lin.Jc[c] + lin.Jc[6 + a] * lin.Jc[6 + c];
        }
        for (int o2 = o0; o2 < o1; ++o2) {
          const int cj = obs_cam[o2] - n_fixed;
          if (cj < 0) continue;
          const double* W2 = Wobs + 18 * (int64_t)o2;
          for (int a = 0; a < 6; ++a)
            for (int c = 0; c < 6; ++c)
              P->S[(int64_t)(6 * ci + a) * n + 6 * cj + c] -=
                  Y[3 * a] * W2[3 * c] + Y[3 * a + 1] * W2[3 * c + 1] + Y[3 * a + 2] * W2[3 * c + 2];
        }
      }
    }
  }
  double* S = part[0].S;
  double* b = part[0].b;
  double cost = part[0].cost;
  /* thread partials summed in thread order per entry (entries in parallel) */
#pragma omp parallel for schedule(static) num_threads(nt)
  for (int64_t e = 0; e < (int64_t)n * n; ++e)
    for (int t = 1; t < nt; ++t) S[e] += part[t].S[e];
  for (int t = 1; t < nt; ++t) {
    for (int e = 0; e < n; ++e) b[e] += part[t].b[e];
    cost += part[t].cost;
  }
  for (int i = 0; i < n; ++i) S[(int64_t)i * n + i] += lam;
  if (cost_out) *cost_out = cost;
  if (S_out) memcpy(S_out, S, sizeof(double) * (size_t)n * n);
  if (b_out) memcpy(b_out, b, sizeof(double) * n);
  double* dc = (double*)malloc(sizeof(double) * (n + 1));
  memcpy(dc, b, sizeof(double) * n);
  const int ok = chol_solve(S, n, dc, nt);
  if (ok) {
    if (dc_out) memcpy(dc_out, dc, sizeof(double) * n);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int p = 0; p < L; ++p) {
      double acc[3] = {-gp[3 * p], -gp[3 * p + 1], -gp[3 * p + 2]};
      const double* Vi = Vinv + 9 * p;
      if (!pvalid[p]) continue;  /* frozen */
      for (int o = point_ptr[p]; o < point_ptr[p + 1]; ++o) {
        const int ci = obs_cam[o] - n_fixed;
        if (ci < 0) continue;
        const double* W = Wobs + 18 * (int64_t)o;
        for (int c = 0; c < 3; ++c)
          for (int a = 0; a < 6; ++a) acc[c] -= W[3 * a + c] * dc[6 * ci + a];
      }
      for (int i = 0; i < 3; ++i)
        points[3 * p + i] += Vi[3 * i] * acc[0] + Vi[3 * i + 1] * acc[1] + Vi[3 * i + 2] * acc[2];
    }
    for (int c = n_fixed; c < N; ++c) {
      double out[12];
      se3_apply(dc + 6 * (c - n_fixed), poses + 12 * c, out);
      memcpy(poses + 12 * c, out, sizeof out);
    }
  }
  for (int t = 0; t < nt; ++t) {
    free(part[t].S);
    free(part[t].b);
  }
  free(part);
  free(dc);
  free(Wobs);
  free(Vinv);
  free(gp);
  free(pvalid);
  return ok;
}

double oracle_ba_cost(int L, double fx, double fy, double cx, double cy, const int32_t* point_ptr,
                      const int32_t* obs_cam, const float* obs_uv, const double* poses,
                      const double* points, int nthreads) {
  double cost = 0.0;
#pragma omp parallel for reduction(+ : cost) schedule(static) num_threads(nthreads)
  for (int p = 0; p < L; ++p) {
    lin_t lin;
    for (int o = point_ptr[p]; o < point_ptr[p + 1]; ++o) {
      linearize(poses + 12 * obs_cam[o], points + 3 * p, obs_uv + 2 * o, fx, fy, cx, cy, &lin);
      cost += lin.r[0] * lin.r[0] + lin.r[1] * lin.r[1];
    }
  }
  return cost;
}

/* iters GN steps; cost_out[iters+1]; returns the number of successful steps. */
int oracle_ba_solve(int N, int L, int n_fixed, double fx, double fy, double cx, double cy,
                    double lam, const int32_t* point_ptr, const int32_t* obs_cam,
                    const float* obs_uv, double* poses, double* points, int iters,
                    double* cost_out, int nthreads) {
  int it = 0;
  for (; it < iters; ++it) {
    if (!oracle_ba_step(N, L, n_fixed, fx, fy, cx, cy, lam, point_ptr, obs_cam, obs_uv, poses,
                        points, cost_out ? cost_out + it : NULL, NULL, NULL, NULL, nthreads))
      break;
  }
  if (cost_out)
    cost_out[it] = oracle_ba_cost(L, fx, fy, cx, cy, point_ptr, obs_cam, obs_uv, poses, points,
                                  nthreads);
  return it;
}
