// Host check of the one-wave K1's chunk images (tests/test_plan_wave_lanes.py): builds the
// plan of a window and walks each chunk's Schur lanes exactly as ba_lin_wave_kernel assigns
// them (passes of kLinLanes, binary search over abase, 2^anp lanes per row), checking that
//   - every pair of every active slot is summed exactly once per row, by one part;
//   - every row's parts are aligned lanes of one pass (the four-wave K1's butterfly groups);
//   - the one-wave K1 (seg_obs 1): one lane per slot block, copies splitting heavy slots;
//   - a diagonal slot's pairs (over its copies) are (x, x) over exactly its camera's track entries
//     (so its lanes' U sums equal the camera lists'), adcam names the camera, off-diagonal 0xFF;
//     one-wave K1: each item's U observation range (auo) is exactly its pairs' observations;
//   - one-wave K1: every window slot is active and every window camera has a diagonal slot in
//     some chunk of its segment (every slab row and rhs entry is written); a segment of several
//     chunks (seg_chunks > 1) has exactly seg_chunks of them (padded with empty chunks), all of
//     one first-camera group, at most kWaveItems window slots and items per chunk (the combine's
//     scratch rows).
// Input (binary): int32 n_poses, n_points, n_obs, n_fixed, seg_obs; point_ptr; obs_cam; obs_uv.
// Optional argv[2]: seg_chunks (wave plans; default 1).
// Prints "ok <chunks> <segments> <passes> <max chain (pair rows)>" or the first violation.
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "ba_plan.h"

namespace vo {
void* plan_host_alloc(size_t b, bool) { return ::operator new(b < 64 ? 64 : b, std::align_val_t(64)); }
void plan_host_free(void* p, bool) noexcept {
  if (p) ::operator delete(p, std::align_val_t(64));
}
}  // namespace vo

#define FAIL(...)                      \
  do {                                 \
    std::printf("fail: " __VA_ARGS__); \
    std::printf("\n");                 \
    return 1;                          \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t hd[5];
  if (std::fread(hd, 4, 5, f) != 5) return 2;
  const int N = hd[0], L = hd[1], M = hd[2], nf = hd[3], so = hd[4];
  std::vector<int32_t> ptr(L + 1), cam(M);
  std::vector<float> uv(2 * (size_t)M);
  if (std::fread(ptr.data(), 4, L + 1, f) != (size_t)L + 1 || std::fread(cam.data(), 4, M, f) != (size_t)M ||
      std::fread(uv.data(), 4, 2 * (size_t)M, f) != 2 * (size_t)M)
    return 2;
  std::fclose(f);
  vo::BAPlan P;
  const bool wave = vo::plan_is_wave(so);
  const int sc = argc > 2 ? std::atoi(argv[2]) : 1;
  const std::string err = vo::build_plan(P, N, L, M, nf, ptr.data(), cam.data(), uv.data(), so, nullptr, sc);
  if (!err.empty()) FAIL("plan: %s", err.c_str());
  if (wave && P.seg_chunks != sc) FAIL("plan seg_chunks %d, asked %d", P.seg_chunks, sc);
  long passes = 0;
  int max_chain = 0;
  for (int si = 0; si < P.n_segments(); ++si) {
    const int32_t* sh = &P.seg_hdr[(size_t)si * vo::kSegHdr];
    const int nslots = sh[0], so_ = sh[1], co = sh[2], ncams = sh[3];
    std::vector<int> slot_seen(nslots, 0), cam_diag(ncams, 0);
    if (wave) {
      if (sh[6] - sh[5] != sc || sh[5] != si * sc) FAIL("segment %d: chunks [%d, %d), seg_chunks %d", si, sh[5], sh[6], sc);
      if (sc > 1 && nslots > vo::kWaveItems) FAIL("segment %d: %d window slots", si, nslots);
      // one first-camera group: the segment's landmarks inside one group's range
      const int q0 = P.chunk_pt[sh[5]], q1 = P.chunk_pt[sh[6]];
      int g = 0;
      while (g + 1 < (int)P.group_q.size() && P.group_q[g + 1] <= q0 && P.group_q[g + 1] < q1) ++g;
      if (q1 > q0 && (q0 < P.group_q[g] || q1 > P.group_q[g + 1])) FAIL("segment %d crosses a first-camera group", si);
    }
    for (int ch = sh[5]; ch < sh[6]; ++ch) {
      const int32_t* h = &P.chunk_hdr[(size_t)ch * vo::kChunkHdr];
      const vo::ChunkImg& g = P.chunk_img[ch];
      const int nas = h[14], lanes = g.abase[nas], npairs = h[9] - h[8];
      if (wave && sc > 1 && nas > vo::kWaveItems) FAIL("chunk %d: %d items", ch, nas);
      std::vector<int> cover(6 * (size_t)npairs, 0);
      const int plane = wave ? vo::kLinLanesWave : vo::kLinLanes;
      for (int base = 0; base < lanes; base += plane, ++passes) {
        for (int tid = 0; tid < plane; ++tid) {
          const int t = base + tid;
          if (t >= lanes) continue;
          int s = 0;
          for (int sp = 32; sp > 0; sp >>= 1)
            if (s + sp < nas && g.abase[s + sp] <= t) s += sp;
          const int off = t - g.abase[s];
          int r0, r1, part, np;
          if (wave) {  // lane = item: the whole block over the item's pairs
            if (off != 0) FAIL("chunk %d: lane %d is not item %d", ch, t, s);
            r0 = 0;
            r1 = 6;
            part = 0;
            np = 1;
          } else {  // lane = (row a, part)
            const int lgp = g.anp[s];
            np = 1 << lgp;
            const int a = off >> lgp;
            part = off & (np - 1);
            if (a >= 6) FAIL("chunk %d lane %d: row %d", ch, t, a);
            if ((t - part) / plane != (t - part + np - 1) / plane || (t - part) % np)
              FAIL("chunk %d slot item %d: parts not aligned in one pass", ch, s);
            r0 = a;
            r1 = a + 1;
          }
          int n = 0;
          for (int e = g.slotp[s] + part; e < g.slotp[s] + g.apcnt[s]; e += np, ++n)
            for (int r = r0; r < r1; ++r) ++cover[6 * (size_t)e + r];
          max_chain = std::max(max_chain, n * (r1 - r0));
        }
      }
      for (size_t k = 0; k < cover.size(); ++k)
        if (cover[k] != 1) FAIL("chunk %d: pair %zu row %zu summed %d times", ch, k / 6, k % 6, cover[k]);
      if (g.slotp[nas] != npairs) FAIL("chunk %d: active slots end at %d of %d pairs", ch, (int)g.slotp[nas], npairs);
      const int te0 = h[2];
      std::vector<std::vector<int>> upairs(ncams);
      for (int s = 0; s < nas; ++s) {
        const int ws = g.aslot[s];
        slot_seen[ws] = 1;
        const int ci = P.slot_i[so_ + ws], cj = P.slot_j[so_ + ws];
        if (ci != cj) {
          if (g.adcam[s] != 0xFF) FAIL("chunk %d: off-diagonal slot %d marked camera %d", ch, ws, (int)g.adcam[s]);
          if (wave && g.auo[s] != g.auo[s + 1]) FAIL("chunk %d: off-diagonal item %d with U observations", ch, s);
          continue;
        }
        const int wc = g.adcam[s];
        if (wc >= ncams || P.segcam_f[co + wc] != ci) FAIL("chunk %d: diagonal slot %d camera %d", ch, ws, wc);
        cam_diag[wc] = 1;
        // its pairs: (x, x) over the chunk's track entries of that camera, each once
        std::vector<int> tes, uobs;
        for (int e = g.slotp[s]; e < g.slotp[s] + g.apcnt[s]; ++e) {
          const int x = g.pairs[e] & 255, y = g.pairs[e] >> 8;
          if (x != y) FAIL("chunk %d: diagonal slot pair (%d, %d)", ch, x, y);
          tes.push_back(x);
          for (int o = g.te_obs[x]; o < g.te_obs[x + 1]; ++o) uobs.push_back(o);
        }
        // one-wave K1: the item's U observations (camol range) are exactly its pairs' ones
        if (wave) {
          std::vector<int> got;
          for (int i = g.auo[s]; i < g.auo[s + 1]; ++i) got.push_back(g.camol[i]);
          if (got != uobs) FAIL("chunk %d item %d: U observations differ from its pairs'", ch, s);
        }
        upairs[wc].insert(upairs[wc].end(), tes.begin(), tes.end());
      }
      for (int wc = 0; wc < ncams; ++wc) {
        std::vector<int> want;
        for (int t = te0; t < te0 + h[3]; ++t)
          if (P.te_lcam[t] == wc) want.push_back(t - te0);
        std::sort(upairs[wc].begin(), upairs[wc].end());
        if (!upairs[wc].empty() && upairs[wc] != want) FAIL("chunk %d: camera %d track entries (U) differ", ch, wc);
      }
    }
    if (wave) {
      for (int s = 0; s < nslots; ++s)
        if (!slot_seen[s]) FAIL("segment %d: window slot %d never written", si, s);
      for (int c = 0; c < ncams; ++c)
        if (!cam_diag[c]) FAIL("segment %d: window camera %d without a diagonal slot", si, c);
    }
  }
  std::printf("ok %d %d %ld %d\n", P.n_chunks(), P.n_segments(), passes, max_chain);
  std::fprintf(stderr, "slab_slots %d\n", P.n_slab_slots());
  return 0;
}
