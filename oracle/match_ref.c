/*
 * CPU oracle for the descriptor matcher -- TEST INFRASTRUCTURE ONLY (tests/,
 * __graft_entry__.smoke(), bench.py cpu_baseline leg).  Never linked into the
 * product library.
 *
 * Restates, for one frame pair:
 *   reference src/modules/frontend.py:101   matcher.knnMatch(des0, des1, k=2)
 *     with matcher = cv2.BFMatcher(cv2.NORM_L2, crossCheck=False) (:34), i.e.
 *     OpenCV 4.12 (opencv-python==4.12.0.88, uv.lock:742-743, not vendored)
 *     BFMatcher::knnMatchImpl -> batchDistance(..., K=2): per query row the
 *     distances dist[j] = sqrtf(normL2Sqr(q, t_j)) for j = 0..n1-1, then an
 *     insertion scan that keeps the K best with a STRICT '<' test, so an equal
 *     distance never displaces an earlier (lower) train index.
 *   reference src/modules/frontend.py:103-109 the ratio loop: keep
 *     (queryIdx, trainIdx) when len(m_n) == 2 and m.distance < 0.75*n.distance
 *     (Python compares the float32 distances promoted to double).
 * normL2Sqr is the k-ordered fmaf chain acc = fmaf(d_k, d_k, acc), d_k = a_k - b_k;
 * for OpenCV SIFT descriptors (integers 0..255) every partial sum is an exact
 * integer below 2^24, so the result equals OpenCV's SIMD sum bit for bit.  For
 * non-integer descriptors the summation order is build-defined.
 *
 * Parity pin: no cv2 in this image and the reference holds no fixtures
 * (SURVEY.md §4); pinned by the hand-built known-answer tests of
 * tests/test_oracle_match.py (ties, N1 < 2, duplicates, sqrt collisions).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>

static void knn2_row(const float* q, const float* train, int n1, int dim, int32_t* idx,
                     float* dist) {
  float d0 = FLT_MAX, d1 = FLT_MAX;
  int32_t i0 = -1, i1 = -1;
  for (int j = 0; j < n1; ++j) {
    const float* t = train + (int64_t)j * dim;
    float acc = 0.0f;
    for (int k = 0; k < dim; ++k) {
      const float df = q[k] - t[k];
      acc = fmaf(df, df, acc);
    }
    const float d = sqrtf(acc);
    if (d < d1) {          /* batchDistance: if (d < dist[K-1]) */
      if (d0 > d) {        /* shift while dist[k] > d           */
        d1 = d0;
        i1 = i0;
        d0 = d;
        i0 = j;
      } else {
        d1 = d;
        i1 = j;
      }
    }
  }
  idx[0] = i0;
  idx[1] = i1;
  dist[0] = d0;
  dist[1] = d1;
}

/* idx: (n0,2) int32 (-1 = fewer neighbours), dist: (n0,2) float32. */
void oracle_knn2(const float* des0, int n0, const float* des1, int n1, int dim, int32_t* idx,
                 float* dist, int nthreads) {
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
  for (int i = 0; i < n0; ++i)
    knn2_row(des0 + (int64_t)i * dim, des1, n1, dim, idx + 2 * (int64_t)i, dist + 2 * (int64_t)i);
}

/* Ratio test over knn2 output: best[i] = train index kept for query i, or -1. */
void oracle_ratio(const int32_t* idx, const float* dist, int n0, double ratio, int32_t* best) {
  for (int i = 0; i < n0; ++i) {
    const int ok = idx[2 * i + 1] >= 0 && (double)dist[2 * i] < ratio * (double)dist[2 * i + 1];
    best[i] = ok ? idx[2 * i] : -1;
  }
}

/* Full match_frames restatement: pairs (query, train) ascending query; returns count. */
int oracle_match(const float* des0, int n0, const float* des1, int n1, int dim, double ratio,
                 int32_t* pairs, int32_t* idx_scratch, float* dist_scratch, int nthreads) {
  if (n0 == 0 || n1 == 0) return 0;
  oracle_knn2(des0, n0, des1, n1, dim, idx_scratch, dist_scratch, nthreads);
  int m = 0;
  for (int i = 0; i < n0; ++i) {
    if (idx_scratch[2 * i + 1] >= 0 &&
        (double)dist_scratch[2 * i] < ratio * (double)dist_scratch[2 * i + 1]) {
      pairs[2 * m] = i;
      pairs[2 * m + 1] = idx_scratch[2 * i];
      ++m;
    }
  }
  return m;
}
