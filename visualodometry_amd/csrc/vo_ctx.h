// vo_ctx: one HIP device + stream, the matcher workspace and the BA engine.
#pragma once

#include <memory>
#include <vector>

#include "vo_common.h"

namespace vo {

struct MatchWorkspace {
  DevBuf des;       // staging for host descriptors (des0 then des1)
  DevBuf q8;        // packed int8 (a - 128) descriptors, query then train
  DevBuf norms;     // int32 squared norms of the packed rows
  DevBuf colconst;  // uint32 per train column (see match.hip)
  DevBuf partial;   // per (split, row) top-2 partials
  DevBuf best;      // int32 (batch, n0) best train index or -1
  DevBuf top2;      // int32 (n0, 2) + float (n0, 2)
  DevBuf pairs;     // int32 (n0, 2) compacted pairs + count
  DevBuf flag;      // uint32: == gen when this call's descriptors are not 0..255 integers
  DevBuf tri;       // triangulation staging: pts1, pts2, pts3d, mask
  DevBuf hbf;       // float path: bf16 images of both sides (match_bf16.hip)
  DevBuf fnorm;     // float path: |b'|^2 per train row, |a| per query row
  DevBuf fpart;     // float path: top-2 of A per (split, row), the sweeps' own split
  DevBuf bmax;      // float path: max |b| per batch entry (zero between calls)
  DevBuf cand;      // float path: candidate lists + counts
  uint32_t gen = 0;         // generation tag of the current call
  int kind_hint = 0;        // VO_DESC_* (vo_match_hint)
  bool flag_fresh = true;   // flag not yet zeroed
};

// The matcher's cached query side (vo_match_knn2_ratio_dev / _q with a nonzero tag): the
// reference matches every frame against the same keyframe (vo.py:64-65), so the keyframe's
// packed int8 rows, norms and integer verdict are kept across calls.  Keyed on (tag, source
// pointer, n0, dim, device or host source); host sources also keep their float copy (the
// exact sweep and the float path read it).
struct MatchQueryCache {
  DevBuf des;    // host sources: the query's float32 rows on the device
  DevBuf q8;     // packed int8 (a - 128) rows (n0_pad x Dp)
  DevBuf norms;  // int32 squared norms
  DevBuf flag;   // [0] 1 = a value is not a 0..255 integer, [1] 1 = a value is not finite
  uint64_t tag = 0;
  const void* src = nullptr;
  int n0 = -1, dim = -1;
  bool device_src = false;
  bool valid = false;
};

// PnP-RANSAC workspace (pnp.hip): RANSAC subsets cached per frame layout.
struct PnpWorkspace {
  DevBuf sub;     // int32 (batch, H, 5) subsets
  DevBuf off;     // int32 (batch + 1) frame offsets
  DevBuf models;  // double (batch, H, 16)
  DevBuf counts;  // int32 (batch, H)
  DevBuf need;    // int32 (batch): frames whose hypotheses past the first h1 are solved
  DevBuf stage;   // host-call staging: points, outputs
  HostBuf hstage; // its page-locked mirror: one upload and one download per host call
  std::vector<int32_t> offsets;  // layout the cached subsets were made for
  int H = 0;
  int last_h1 = 0;  // hypotheses solved for every frame by the last call (pnp_run)
};

// SIFT detection workspace (sift.hip): Gaussian and DoG pyramids of a batch.
struct SiftWorkspace {
  DevBuf g, d;     // float pyramids (pitched, all octaves)
  DevBuf img;      // host-call staging: the uint8 image
  DevBuf kp;       // host-call staging: keypoints + count
  DevBuf cand_ext; // packed 26-neighbour extrema awaiting refinement + their count
  DevBuf cand;     // detectAndCompute: refined extrema (float + int records, count)
  DevBuf okp;      // oriented keypoints (batch, capacity, 8 floats)
  DevBuf keys;     // uint64 sort keys in / out
  DevBuf vals;     // uint32 record indices in / out, then the selection
  DevBuf segs;     // int32 per-image counts, segment bounds, kept counts
  DevBuf sort_tmp; // rocprim temporary storage
  DevBuf out;      // host-call staging: keypoints, descriptors, count
  // The overlapped pyramid (sift_run): octave o + 1's down-sample and first levels on the
  // context stream while octave o's last two levels and its extrema test run on this one.
  hipStream_t side = nullptr;
  hipEvent_t side_ev[17] = {};  // per octave (its level n_layers done), then the join
  SiftWorkspace() = default;
  SiftWorkspace(const SiftWorkspace&) = delete;
  SiftWorkspace& operator=(const SiftWorkspace&) = delete;
  ~SiftWorkspace() {
    if (side) (void)hipStreamSynchronize(side);
    for (hipEvent_t e : side_ev)
      if (e) (void)hipEventDestroy(e);
    if (side) (void)hipStreamDestroy(side);
  }
};

class BAEngine;   // ba.hip
struct Comm;      // ba.hip (RCCL communicator)

// Kernel ids of the event profiler (vo_profile_* in include/vo_hip.h).
enum KernelId {
  kKBaLin = 0, kKBaReduce, kKBaSolve, kKMatchPack, kKMatchI8, kKMatchF32, kKMatchMerge,
  kKTriangulate, kKPnpHyp, kKPnpScore, kKPnpFinal, kKSiftPyramid, kKSiftExtrema, kKSiftOrient, kKSiftSelect,
  kKSiftDesc, kKMatchRerank, kKPnpDecide, kKPnpHypTail, kKPnpScoreTail, kKCount
};

// HIP-event timing of individual kernels on the context stream (off by default).
struct Profiler {
  bool on = false;
  struct Rec { int id; hipEvent_t start, stop; };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  hipEvent_t get();
  void begin(hipStream_t st, int id);  // records a start event if on
  void end(hipStream_t st);            // records the matching stop event
  void read(double* ms, int64_t* counts);  // after a stream sync; clears the records
  ~Profiler();
};

}  // namespace vo

struct vo_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int num_cus = 0;
  vo::MatchWorkspace match;
  vo::MatchQueryCache match_q;
  vo::PnpWorkspace pnp;
  vo::SiftWorkspace sift;
  vo::Profiler prof;
  std::unique_ptr<vo::BAEngine> ba;
  std::unique_ptr<vo::Comm> comm;
  bool ba_split_reduce = false;  // test/tool switch (vo_ba_split_reduce): K2 never fused into K3
  int ba_drop_reducers = 0;      // test switch (vo_ba_testing_drop_reducers): fused launches short of reducers
  bool ba_no_split = false;      // test switch (vo_ba_testing_no_split): no split band layout at setup
  int pnp_group = 0;      // test switch (vo_pnp_testing_group): 0 auto, 1 lane groups, -1 one lane per hypothesis
  int pnp_split = 0;      // test/tool switch (vo_pnp_testing_split): 0 auto, -1 never, n > 0 first n hypotheses
  int ba_k1_variant = 0;  // test switch (vo_ba_testing_k1): -1 four-wave K1, n >= 1 one-wave K1 of n chunks per segment
  vo_ctx();
  ~vo_ctx();
};

namespace vo {
// Matcher entry points (match.hip).
void match_run(vo_ctx* ctx, const float* d_des0, const float* d_des1, int batch, int n0,
               int n1, int dim, double ratio, int32_t* d_best, int32_t* d_idx2,
               float* d_dist2, const MatchQueryCache* qc = nullptr);
void match_pack_query(vo_ctx* ctx, const float* d_des0, int n0, int dim, MatchQueryCache& qc);
void compact_pairs(vo_ctx* ctx, const int32_t* d_best, int n0, int32_t* d_pairs,
                   int32_t* d_count);
// Triangulation entry point (tri.hip): host matrices, device points.
void tri_run(vo_ctx* ctx, const double* P1, const double* P2, const double* T_cw2, const double* K,
             const float* d_pts1, const float* d_pts2, int n, double min_depth, double max_reproj_err,
             float* d_pts3d, uint8_t* d_mask);
// PnP-RANSAC entry point (pnp.hip): device points, host offsets and K.
void pnp_run(vo_ctx* ctx, const float* d_X, const float* d_uv, const int32_t* offsets, int batch,
             const double* K, int iterations, double reproj_err, double confidence, double* d_pose,
             uint8_t* d_mask, int32_t* d_status);
void pnp_subsets(int count, int iters, int32_t* out);
// SIFT detection (sift.hip): device images, device keypoint outputs (unsorted).
void sift_run(vo_ctx* ctx, const uint8_t* d_img, int batch, int h, int w, double contrast, double edge,
              double sigma, int n_layers, int capacity, float* d_kpf, int32_t* d_kpi, int32_t* d_count,
              float** g_out, float** d_out, int64_t* layout);
int sift_layout(int h, int w, int n_layers, int64_t* out, int n);
// SIFT orientation, filtering and descriptors (sift_desc.hip) of sift_run's candidates.
int sift_max_capacity();  // largest per-image keypoint capacity of sift_describe
void sift_describe(vo_ctx* ctx, int batch, int h, int w, int n_layers, double sigma, int nfeatures, int cap_img,
                   const float* cand_f, const int32_t* cand_i, const int32_t* cand_count, int cand_cap,
                   const float* G, vo_sift_keypoint* d_kp, float* d_desc, int32_t* d_count);
}  // namespace vo
