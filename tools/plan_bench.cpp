// Host-only timing of the BA planner (csrc/ba_plan.cpp build_plan + build_profile) on a sequence
// of sliding windows, as vo_ba_setup runs it per keyframe: each window planned from scratch, and
// each window after the previous one (taking its unchanged first-camera groups over).
// Build: g++ -O3 -std=c++17 -pthread tools/plan_bench.cpp visualodometry_amd/csrc/ba_plan.cpp -o /tmp/plan_bench
// Input (binary, tools/plan_bench.py writes it): int32 n_windows, then per window int32 n_poses,
// n_points, n_obs, n_fixed; point_ptr; obs_cam; float32 obs_uv.
// Usage: plan_bench <file> <seg_obs> <seg_chunks> <reps>; prints one JSON line (medians, ms).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <new>
#include <vector>

#include "../visualodometry_amd/csrc/ba_plan.h"

namespace vo {
void* plan_host_alloc(size_t b, bool) { return ::operator new(b < 64 ? 64 : b, std::align_val_t(64)); }
void plan_host_free(void* p, bool) noexcept {
  if (p) ::operator delete(p, std::align_val_t(64));
}
}  // namespace vo

struct Win {
  int n, L, M, nf;
  std::vector<int32_t> ptr, cam;
  std::vector<float> uv;
};

static double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  const int so = std::atoi(argv[2]), sc = std::atoi(argv[3]), reps = std::atoi(argv[4]);
  int32_t nw = 0;
  if (std::fread(&nw, 4, 1, f) != 1) return 2;
  std::vector<Win> ws(nw);
  for (Win& w : ws) {
    int32_t h[4];
    if (std::fread(h, 4, 4, f) != 4) return 2;
    w.n = h[0], w.L = h[1], w.M = h[2], w.nf = h[3];
    w.ptr.resize(w.L + 1);
    w.cam.resize(w.M);
    w.uv.resize(2 * (size_t)w.M);
    if (std::fread(w.ptr.data(), 4, w.L + 1, f) != (size_t)w.L + 1 || std::fread(w.cam.data(), 4, w.M, f) != (size_t)w.M ||
        std::fread(w.uv.data(), 4, 2 * (size_t)w.M, f) != 2 * (size_t)w.M)
      return 2;
  }
  std::fclose(f);
  vo::BAPlan A, B;
  auto plan = [&](vo::BAPlan& P, const Win& w, const vo::BAPlan* prev) {
    const std::string err = vo::build_plan(P, w.n, w.L, w.M, w.nf, w.ptr.data(), w.cam.data(), w.uv.data(), so, prev, sc);
    if (!err.empty()) {
      std::fprintf(stderr, "plan: %s\n", err.c_str());
      std::exit(1);
    }
    vo::build_profile(P, vo::local_profile_first(P));
  };
  std::vector<double> scratch, slide;
  long reused = 0, chunks = 0;
  for (int r = 0; r < reps; ++r)
    for (int i = 0; i < nw; ++i) {
      auto t0 = std::chrono::steady_clock::now();
      plan(A, ws[i], nullptr);  // from scratch
      scratch.push_back(ms_since(t0));
      if (i + 1 < nw) {
        t0 = std::chrono::steady_clock::now();
        plan(B, ws[i + 1], &A);  // the next window after this one
        slide.push_back(ms_since(t0));
        reused += B.reused_chunks;
        chunks += B.n_chunks();
      }
    }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
  };
  std::printf("{\"scratch_ms\": %.4f, \"slide_ms\": %.4f, \"reused_frac\": %.3f, \"windows\": %d, \"reps\": %d}\n",
              med(scratch), med(slide), chunks ? (double)reused / chunks : 0.0, nw, reps);
  return 0;
}
