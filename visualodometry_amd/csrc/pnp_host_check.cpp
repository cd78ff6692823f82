// Runs the PnP kernels' scalar math (pnp_math.h, the code pnp_hyp_kernel executes per
// hypothesis) on the host, for tests/test_pnp_host_math.py to compare with oracle/pnp_ref.py
// without a GPU.  Diagnostic build only: never part of libvo_hip.so.
//   pnp_host_check in.bin out.bin
// in:  int32 count, double K[4] (fu, fv, uc, vc), then count x (pw[5][3], us[5][2]) doubles
// out: count x (R[9] of EPnP, t[3], rvec[3], Rm[9] = Rodrigues(rvec), ok) doubles
#include <cstdio>
#include <vector>

#include "pnp_math.h"

using namespace vo::pnpm;

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]);
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
    for (int p = 0; p < kPts; ++p) {
      for (int c = 0; c < 3; ++c) S.pw[p][c] = src[3 * p + c];
      for (int c = 0; c < 2; ++c) S.us[p][c] = src[15 + 2 * p + c];
    }
    double R[3][3], t[3], rv[3], Rm[3][3];
    const bool ok = epnp5(S, K, R, t);
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
