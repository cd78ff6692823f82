// Runs the SIFT orientation kernel's per-keypoint math (sift_math.h, sift_orient_kernel's
// sample evaluation and per-bin accumulation order) on the host, for
// tests/test_sift_host_math.py to compare with oracle/sift_ref.py without a GPU.
// Diagnostic build only: never part of libvo_hip.so.
//   sift_host_check in.bin out.bin
// in:  int32 rows, cols; float img[rows][cols]; int32 n; n x (int32 row, col; float scl)
// out: n x float hist[36] (smoothed)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "sift_math.h"

using namespace vo::siftm;

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  FILE* fi = std::fopen(argv[1], "rb");
  if (!fi) return 2;
  int32_t rows = 0, cols = 0, n = 0;
  if (std::fread(&rows, 4, 1, fi) != 1 || std::fread(&cols, 4, 1, fi) != 1) return 2;
  std::vector<float> img((size_t)rows * cols);
  if (std::fread(img.data(), 4, img.size(), fi) != img.size() || std::fread(&n, 4, 1, fi) != 1) return 2;
  ExpTab tab;
  for (int j = 0; j < 64; ++j) tab.v[j] = (float)(std::pow(2.0, j / 64.0) * kExpA0);
  std::vector<float> out((size_t)n * 36);
  for (int q = 0; q < n; ++q) {
    int32_t pr = 0, pc = 0;
    float scl = 0;
    if (std::fread(&pr, 4, 1, fi) != 1 || std::fread(&pc, 4, 1, fi) != 1 || std::fread(&scl, 4, 1, fi) != 1) return 2;
    const int radius = (int)std::rint(4.5f * scl);
    const float sigma = 1.5f * scl;
    const float expf_scale = -1.f / (2.f * sigma * sigma);
    float th[40] = {0};
    for (int i = -radius; i <= radius; ++i)
      for (int j = -radius; j <= radius; ++j) {
        const int y = pr + i, x = pc + j;
        if (!(y > 0 && y < rows - 1 && x > 0 && x < cols - 1)) continue;
        const float dx = img[(size_t)y * cols + x + 1] - img[(size_t)y * cols + x - 1];
        const float dy = img[(size_t)(y - 1) * cols + x] - img[(size_t)(y + 1) * cols + x];
        const float w = exp32f((float)(i * i + j * j) * expf_scale, tab.v);
        const float ori = fast_atan2_deg(dy, dx);
        const float mag = sqrt_rn(dx * dx + dy * dy);
        int bin = (int)std::rint((36.f / 360.f) * ori);
        if (bin >= 36) bin -= 36;
        if (bin < 0) bin += 36;
        th[bin + 2] = th[bin + 2] + w * mag;
      }
    th[0] = th[36];
    th[1] = th[37];
    th[38] = th[2];
    th[39] = th[3];
    for (int l = 0; l < 36; ++l) {
      const float* T = th + 2 + l;
      out[(size_t)q * 36 + l] = (T[-2] + T[2]) * (1.f / 16.f) + (T[-1] + T[1]) * (4.f / 16.f) + T[0] * (6.f / 16.f);
    }
  }
  std::fclose(fi);
  FILE* fo = std::fopen(argv[2], "wb");
  if (!fo) return 2;
  std::fwrite(out.data(), 4, out.size(), fo);
  std::fclose(fo);
  return 0;
}
