// Runs the PnP kernels' scalar math (pnp_math.h) on the host, for
// tests/test_pnp_host_math.py to compare with oracle/pnp_ref.py without a GPU.
// Diagnostic build only: never part of libvo_hip.so.
//   pnp_host_check [steps] in.bin out.bin   per hypothesis (what pnp_hyp_kernel computes; steps: the
//                                        12 x 12 SVD in the lane-group kernel's step order)
// in:  int32 count, double K[4] (fu, fv, uc, vc), then count x (pw[5][3], us[5][2]) doubles
// out: count x (R[9] of EPnP, t[3], rvec[3], Rm[9] = Rodrigues(rvec), ok) doubles
//   pnp_host_check full in.bin out.bin   one frame through the three kernels' logic, with
//                                        pnp_final_kernel's 256-thread reduction emulated
// in:  int32 n, int32 H, double K[4], float thr2, double confidence, float X[n][3],
//      float uv[n][2], int32 subsets[H][5]
// out: double rvec[3], tvec[3], int32 success, int32 inliers, uint8 mask[n]
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "pnp_math.h"

using namespace vo::pnpm;

namespace {

// pnp_final_kernel's lm_accumulate + lm_reduce: 256 strided partial sums, a butterfly per
// 64-lane wave (v += v[lane ^ m], m = 32 .. 1), then waves 0..3 added in order.
void block_normal_eq(const std::vector<float>& X, const std::vector<float>& uv, const std::vector<uint8_t>& mask,
                     int n, const double* R, const double* t, const Cam& K, double* ne) {
  std::vector<double> part((size_t)256 * kNe, 0.0);
  for (int th = 0; th < 256; ++th) {
    double acc[kNe];
    for (int k = 0; k < kNe; ++k) acc[k] = 0.0;
    for (int i = th; i < n; i += 256)
      if (mask[i]) lm_point(R, t, &X[3 * (size_t)i], uv[2 * (size_t)i], uv[2 * (size_t)i + 1], K, acc);
    for (int k = 0; k < kNe; ++k) part[(size_t)th * kNe + k] = acc[k];
  }
  double wsum[4][kNe];
  for (int k = 0; k < kNe; ++k) {
    for (int w = 0; w < 4; ++w) {
      double v[64];
      for (int l = 0; l < 64; ++l) v[l] = part[(size_t)(64 * w + l) * kNe + k];
      for (int m = 32; m >= 1; m >>= 1) {
        double nv[64];
        for (int l = 0; l < 64; ++l) nv[l] = v[l] + v[l ^ m];
        for (int l = 0; l < 64; ++l) v[l] = nv[l];
      }
      wsum[w][k] = v[0];
    }
    ne[k] = ((wsum[0][k] + wsum[1][k]) + wsum[2][k]) + wsum[3][k];
  }
}

int run_full(const char* in_path, const char* out_path) {
  FILE* fi = std::fopen(in_path, "rb");
  if (!fi) return 2;
  int n = 0, H = 0;
  double k[4], confidence = 0;
  float thr2 = 0;
  if (std::fread(&n, 4, 1, fi) != 1 || std::fread(&H, 4, 1, fi) != 1 || std::fread(k, 8, 4, fi) != 4 ||
      std::fread(&thr2, 4, 1, fi) != 1 || std::fread(&confidence, 8, 1, fi) != 1)
    return 2;
  std::vector<float> X((size_t)3 * n), uv((size_t)2 * n);
  std::vector<int32_t> sub((size_t)5 * H);
  if (std::fread(X.data(), 4, X.size(), fi) != X.size() || std::fread(uv.data(), 4, uv.size(), fi) != uv.size() ||
      std::fread(sub.data(), 4, sub.size(), fi) != sub.size())
    return 2;
  std::fclose(fi);
  const Cam K{k[0], k[1], k[2], k[3]};
  // pnp_hyp_kernel + pnp_score_kernel
  const int nh = n == kPts ? 1 : (n > kPts ? H : 0);
  std::vector<double> models((size_t)16 * (nh ? nh : 1), 0.0);
  std::vector<int> counts(nh ? nh : 1, 0);
  for (int h = 0; h < nh; ++h) {
    EpnpState S;
    double cols[kEpnpColDoubles];
    S.alphas = Col{cols, 1};
    S.v = Col{cols + kPts * 4, 1};
    for (int p = 0; p < kPts; ++p) {
      const int i = n == kPts ? p : sub[5 * (size_t)h + p];
      for (int c = 0; c < 3; ++c) S.pw[p][c] = X[3 * (size_t)i + c];
      for (int c = 0; c < 2; ++c) S.us[p][c] = uv[2 * (size_t)i + c];
    }
    double R[3][3], t[3], rv[3], Rm[3][3];
    const bool ok = epnp5(S, K, R, t);
    rodrigues_to_vec(R, rv);
    rodrigues_to_mat(rv, Rm);
    double* m = &models[16 * (size_t)h];
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) m[3 * i + j] = Rm[i][j];
      m[9 + i] = t[i];
      m[12 + i] = rv[i];
    }
    m[15] = ok ? 1.0 : 0.0;
    if (ok && n > kPts)
      for (int i = 0; i < n; ++i)
        counts[h] += is_inlier(m, m + 9, &X[3 * (size_t)i], uv[2 * (size_t)i], uv[2 * (size_t)i + 1], K, thr2);
  }
  // pnp_final_kernel
  int best = -1;
  if (n == kPts) {
    best = models[15] != 0.0 ? 0 : -1;
  } else if (n > kPts) {
    int niters = H, max_good = 0;
    for (int it = 0; it < niters; ++it) {
      if (models[16 * (size_t)it + 15] == 0.0) continue;
      const int good = counts[it];
      if (good > (max_good > kPts - 1 ? max_good : kPts - 1)) {
        best = it;
        max_good = good;
        niters = update_num_iters(confidence, (double)(n - good) / n, kPts, niters);
      }
    }
  }
  double pose[6] = {0, 0, 0, 0, 0, 0};
  int32_t status[2] = {0, 0};
  std::vector<uint8_t> mask(n, 0);
  if (best >= 0 && n == kPts) {
    for (int k2 = 0; k2 < 3; ++k2) {
      pose[k2] = models[12 + k2];
      pose[3 + k2] = models[9 + k2];
    }
    status[0] = 1;
    status[1] = n;
    for (int i = 0; i < n; ++i) mask[i] = 1;
  } else if (best >= 0) {
    const double* m = &models[16 * (size_t)best];
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
      mask[i] = is_inlier(m, m + 9, &X[3 * (size_t)i], uv[2 * (size_t)i], uv[2 * (size_t)i + 1], K, thr2);
      cnt += mask[i];
    }
    double ne[kNe], nR[9], nt[3];
    block_normal_eq(X, uv, mask, n, m, m + 9, K, ne);
    LmState lm;
    lm.init(m, m + 9, ne);
    bool go = lm.propose(nR, nt);
    while (go) {
      block_normal_eq(X, uv, mask, n, nR, nt, K, ne);
      go = lm.update(nR, nt, ne) && lm.propose(nR, nt);
    }
    double Rf[3][3], rv[3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Rf[i][j] = lm.R[3 * i + j];
    rodrigues_to_vec(Rf, rv);
    for (int k2 = 0; k2 < 3; ++k2) {
      pose[k2] = rv[k2];
      pose[3 + k2] = lm.t[k2];
    }
    status[0] = 1;
    status[1] = cnt;
  }
  FILE* fo = std::fopen(out_path, "wb");
  if (!fo) return 2;
  std::fwrite(pose, 8, 6, fo);
  std::fwrite(status, 4, 2, fo);
  std::fwrite(mask.data(), 1, mask.size(), fo);
  std::fclose(fo);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc == 4 && std::string(argv[1]) == "full") return run_full(argv[2], argv[3]);
  // "steps": EPnP's 12 x 12 SVD in the lane-group kernel's step order (Jacobi12Steps)
  const bool steps = argc == 4 && std::string(argv[1]) == "steps";
  if (steps) ++argv;
  else if (argc != 3) {
    std::fprintf(stderr, "usage: %s [steps] in.bin out.bin\n", argv[0]);
    return 2;
  }
  FILE* fi = std::fopen(argv[1], "rb");
  if (!fi) return 2;
  int count = 0;
  double k[4];
  if (std::fread(&count, 4, 1, fi) != 1 || std::fread(k, 8, 4, fi) != 4) return 2;
  std::vector<double> in((size_t)count * 25), out((size_t)count * 25);
  if (std::fread(in.data(), 8, in.size(), fi) != in.size()) return 2;
  std::fclose(fi);
  const Cam K{k[0], k[1], k[2], k[3]};
  for (int h = 0; h < count; ++h) {
    const double* src = &in[(size_t)h * 25];
    EpnpState S;
    double cols[kEpnpColDoubles];
    S.alphas = Col{cols, 1};
    S.v = Col{cols + kPts * 4, 1};
    for (int p = 0; p < kPts; ++p) {
      for (int c = 0; c < 3; ++c) S.pw[p][c] = src[3 * p + c];
      for (int c = 0; c < 2; ++c) S.us[p][c] = src[15 + 2 * p + c];
    }
    double R[3][3], t[3], rv[3], Rm[3][3];
    const Svd12Alt alt{nullptr, 0};  // the host: the lane groups' step order, serially
    const bool ok = epnp5(S, K, R, t, steps ? &alt : nullptr);
    rodrigues_to_vec(R, rv);
    rodrigues_to_mat(rv, Rm);
    double* dst = &out[(size_t)h * 25];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        dst[3 * i + j] = R[i][j];
        dst[15 + 3 * i + j] = Rm[i][j];
      }
    for (int i = 0; i < 3; ++i) {
      dst[9 + i] = t[i];
      dst[12 + i] = rv[i];
    }
    dst[24] = ok ? 1.0 : 0.0;
  }
  FILE* fo = std::fopen(argv[2], "wb");
  if (!fo) return 2;
  std::fwrite(out.data(), 8, out.size(), fo);
  std::fclose(fo);
  return 0;
}
