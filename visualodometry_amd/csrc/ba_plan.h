// Static execution plan of the BA Gauss-Newton step (host side, built once per
// window structure by vo_ba_setup).  See DESIGN.md §BA for the data layout.
//
// Terminology (domain names):
//   track entry (te): one (landmark, camera) pair with >= 1 observation; the
//                     observations of a landmark are grouped by camera so that
//                     duplicate (landmark, camera) observations simply sum.
//   chunk:            a run of whole landmarks processed together by one K1
//                     workgroup pass (<= kChunkObs obs, <= kChunkTe te,
//                     <= kChunkPts landmarks).
//   segment:          the run of chunks owned by one K1 workgroup.  Its camera
//                     window (the free cameras its landmarks see) and its
//                     camera-pair slots (blocks (i, j), i >= j, of the reduced
//                     camera matrix S it touches) are accumulated in LDS and
//                     written once to the slab.
//   slab:             per-segment partial blocks of S (36 doubles per slot),
//                     of b (6 per window camera) and of the cost.
//   profile:          lower block-envelope storage of S: block row i holds
//                     block columns first[i]..i.  Cholesky preserves it.
#pragma once

#include <cstdint>
#include <memory>
#include <new>
#include <type_traits>
#include <utility>
#include <string>
#include <vector>
// Host setup sections: PLAN_T(i, name) records the time since the previous mark of the calling
// thread as section i (kSetupSections, read back by vo_ba_plan_stats; a steady_clock read, tens
// of nanoseconds); diagnostic builds (EXTRA=-DVO_PLAN_TIMING) also print it to stderr.
#include <chrono>
#include <cstdio>
namespace vo {
constexpr int kSetupSections = 12;  // sync, order, segments, lists, returned, planned, images, profile,
                                    // uploads, bufs, band, attrs
struct SetupClock {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  int64_t ns[kSetupSections] = {};
};
inline SetupClock& setup_clock() {
  static thread_local SetupClock c;
  return c;
}
}  // namespace vo
#ifdef VO_PLAN_TIMING
#define PLAN_T_PRINT(name, ns) std::fprintf(stderr, "  %-14s %8.3f ms\n", name, (ns) * 1e-6)
#else
#define PLAN_T_PRINT(name, ns) \
  do {                         \
  } while (0)
#endif
#define PLAN_T(i, name)                                                                             \
  do {                                                                                              \
    ::vo::SetupClock& c_ = ::vo::setup_clock();                                                     \
    const auto n_ = std::chrono::steady_clock::now();                                               \
    const int64_t d_ = std::chrono::duration_cast<std::chrono::nanoseconds>(n_ - c_.t).count();     \
    c_.ns[i] = d_;                                                                                  \
    c_.t = n_;                                                                                      \
    PLAN_T_PRINT(name, d_);                                                                         \
  } while (0)
#define PLAN_T_START() (::vo::setup_clock().t = std::chrono::steady_clock::now())

namespace vo {

#ifndef VO_CHUNK_OBS
#define VO_CHUNK_OBS 64  // 64-observation chunks: ~50 KB LDS per K1 workgroup, 3 per CU (profiles/r01_chunk_sweep.md)
#endif
constexpr int kChunkObs = VO_CHUNK_OBS;
constexpr int kChunkTe = VO_CHUNK_OBS;
constexpr int kChunkPts = VO_CHUNK_OBS / 2;
constexpr int kChunkPairs = 8 * VO_CHUNK_OBS;  // camera-pair (x, y) entries of one chunk, staged in LDS
constexpr int kSegSlots = 64;
// K1 variants (a plan property): wave plans (seg_obs == 1) run the one-wave K1, one 64-lane wave
// per chunk, one lane per Schur slot block; a segment holds seg_chunks chunks of one
// first-camera group (padded with empty chunks: chunk = segment * seg_chunks + wave), whose
// waves share one workgroup and sum their slot blocks in LDS in chunk order (one slab row per
// segment slot).  Any other packing runs the four-wave K1 walking its segment's chunks (one
// pass of 256 lanes, one lane per block row).
constexpr int kLinLanesWave = 64;   // one-wave K1 lanes (ba.hip ba_lin_wave_kernel)
constexpr int kLinLanes = 256;      // four-wave K1 lanes per Schur pass (ba.hip kLinThreads)
inline bool plan_is_wave(int seg_obs) { return seg_obs == 1; }
#ifndef VO_WAVE_MAX_CHUNKS
#define VO_WAVE_MAX_CHUNKS 6
#endif
constexpr int kWaveMaxChunks = VO_WAVE_MAX_CHUNKS;  // chunks (waves) per segment of a wave plan (ba.hip instantiates 1..6)
// one-wave K1 lanes for slot items: the combine's scratch rows (36 doubles each) alias the chunk's
// Jc | Z | bt region (34 doubles per observation), 60 at 64-observation chunks
constexpr int kWaveItems = VO_CHUNK_OBS * 34 / 36 < 60 ? VO_CHUNK_OBS * 34 / 36 : 60;
// window slots of a one-chunk wave segment: every item's b partial (6 doubles) fits the chunk's
// X | L | h region (12 doubles per landmark), all 64 at 64-observation chunks
constexpr int kWaveSlots = kChunkPts * 12 / 6 < kSegSlots ? kWaveItems : kSegSlots;
constexpr int kChunkHdr = 16;

constexpr int kSegCams = 24;     // free (window) cameras of a segment
constexpr int kSegAllCams = 16;  // all cameras its observations reference (poses staged in LDS)
constexpr int kPlanTableCams = 512;  // planner: flat lookup tables up to this many free cameras

// Per segment, kSegHdr ints: [0] nslots [1] slot offset [2] first window camera [3] window
// cameras [4] cameras seen [5] first chunk [6] end chunk [7] spare | [8..15] cameras seen
// (16 x int16) | [16..27] free camera of each window camera (24 x int16) | [28..31] spare |
// [32..47] the first chunk's header.  One uniform load level gives K1 every segment
// offset; per-thread camera ids sit at fixed offsets (no dependent load).
constexpr int kSegHdr = 48;

// Per chunk header (kChunkHdr ints): ob0 nob te0 nte p0 npt sb cb e0 e1 c0 c1 q0 q1, then the
// chunk's active window slots and active window cameras (ChunkImg).
// Per chunk, the static part of K1's LDS staging as one image (offsets already made
// chunk-relative, types as K1 reads them): staging a chunk is one 16-byte load and one
// LDS store per thread instead of a load per list.  Unused entries are zero.
struct alignas(16) ChunkImg {
  // byte-wide lists (every index < 64 and every count <= 64, kChunkObs): the image, and K1's
  // LDS with it, stays under a third of the CU after the LDS allocation granule
  uint8_t obs_te[kChunkObs];       // observation -> chunk track entry
  uint8_t te_obs[kChunkTe + 1];    // track entry -> first chunk observation
  uint8_t te_pt[kChunkTe];         // track entry -> chunk landmark
  int8_t te_lcam[kChunkTe];        // track entry -> window camera, -1 if fixed
  uint8_t pt_te[kChunkPts + 1];    // landmark -> first chunk track entry
  // the same relations one LDS level shorter (one-wave K1)
  uint8_t obs_pt[kChunkObs];       // observation -> chunk landmark
  int8_t obs_lcam[kChunkObs];      // observation -> window camera, -1 if fixed
  uint8_t pt_obs[kChunkPts + 1];   // landmark -> first chunk observation
  // Only the window slots and cameras this chunk touches (header ints 14 and 15 count them),
  // so K1's Schur loops run over the chunk's own items, not the whole segment window.
  uint16_t slotp[kSegSlots + 1];   // active slot i -> its first pair-list entry
  uint8_t camp[kSegCams + 1];      // active camera i -> first track-entry list entry
  uint8_t camop[kSegCams + 1];     // active camera i -> first observation list entry
  uint8_t dslot[kSegCams];         // active camera i -> its diagonal slot
  uint8_t aslot[kSegSlots];        // active slot i -> window slot
  uint8_t acid[kSegCams];          // active camera i -> window camera
  // Schur-pair lanes.  Four-wave K1: active slot i (ordered by lanes per item descending) sums
  // its apcnt[i] pairs from slotp[i] on 6 << anp[i] lanes starting at abase[i] (2^anp lanes per
  // row, their strided partial sums combined by an aligned butterfly).  One-wave K1: lane i sums
  // item i's whole block over its apcnt[i] pairs from slotp[i] (abase[i] = i); the items of a
  // slot are its anp[i] copies (acopy[i] = 0 .. anp[i] - 1, consecutive ranges of the slot's
  // pairs, consecutive items), summed in copy order inside K1; a diagonal slot's items add U
  // over their pairs' observations.  abase[nas] = lanes used
  uint16_t apcnt[kSegSlots];
  uint16_t abase[kSegSlots + 1];  // up to 6 x 64 lanes (two passes of the workgroup)
  uint8_t anp[kSegSlots];
  uint8_t adcam[kSegSlots];        // active slot i -> window camera if diagonal, else 0xFF
  uint8_t acopy[kSegSlots];        // one-wave K1: item i's copy index (anp[i] = the slot's copies)
  uint8_t cdiag0[kSegCams];        // one-wave K1: active camera i -> its first diagonal item
  uint8_t cdiagn[kSegCams];        //   and the number of copies (consecutive items)
  uint8_t auo[kSegSlots + 1];      // one-wave K1: item i's U observations, camol entries
                                   //   [auo[i], auo[i + 1]) (empty off the diagonal)
  alignas(2) uint16_t pairs[kChunkPairs];  // (te_x | te_y << 8) by slot
  uint8_t caml[kChunkTe];          // track entries by window camera
  uint8_t camol[kChunkObs];        // observations by window camera
  alignas(8) float uv[2 * kChunkObs];
  uint8_t acam[kChunkObs];         // observation -> camera seen (pose index in LDS)
};
static_assert(sizeof(ChunkImg) % 16 == 0, "16-byte staging granules");
static_assert(kChunkObs <= 64 && kChunkTe <= 64 && kChunkPairs <= 65535, "byte-wide chunk lists");

// Host memory of the chunk images (defined in ba.hip): page-locked (hipHostMalloc) for the
// BA engine's plan, so vo_ba_setup's upload of the largest plan array is an asynchronous
// DMA that overlaps the rest of setup; ordinary heap memory for the plans the digest and
// probe entry points build (they run on hosts without a GPU).  Throws std::bad_alloc.
void* plan_host_alloc(size_t bytes, bool pinned);
void plan_host_free(void* p, bool pinned) noexcept;

// Allocator of the chunk images: resize() default-initialises (leaves a trivial type
// unwritten; the planner writes every image in full, on its worker threads), and the
// memory kind is part of the allocator's state.
template <class T>
struct PlanHostAlloc {
  using value_type = T;
  using propagate_on_container_move_assignment = std::true_type;
  using propagate_on_container_swap = std::true_type;
  bool pinned = false;
  PlanHostAlloc() = default;
  explicit PlanHostAlloc(bool p) noexcept : pinned(p) {}
  template <class U>
  PlanHostAlloc(const PlanHostAlloc<U>& o) noexcept : pinned(o.pinned) {}
  T* allocate(size_t n) { return static_cast<T*>(plan_host_alloc(n * sizeof(T), pinned)); }
  void deallocate(T* p, size_t) noexcept { plan_host_free(p, pinned); }
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... Args>
  void construct(U* p, Args&&... args) {
    ::new (static_cast<void*>(p)) U(std::forward<Args>(args)...);
  }
  friend bool operator==(const PlanHostAlloc& a, const PlanHostAlloc& b) { return a.pinned == b.pinned; }
  friend bool operator!=(const PlanHostAlloc& a, const PlanHostAlloc& b) { return a.pinned != b.pinned; }
};

// Allocator whose resize() leaves trivial elements unwritten, for the plan arrays the planner
// writes in full on its worker threads (a value-initialising resize would zero them serially
// first).  Every element of such an array is written before it is read, uploaded or digested.
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = DefaultInitAlloc<U>;
  };
  DefaultInitAlloc() = default;
  template <class U>
  DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... Args>
  void construct(U* p, Args&&... args) {
    ::new (static_cast<void*>(p)) U(std::forward<Args>(args)...);
  }
};
template <class T>
using PlanArr = std::vector<T, DefaultInitAlloc<T>>;

struct PlanScratch;  // ba_plan.cpp

struct SolveTableLayout {
  int diag = 0, off = 0, first = 0, step_ptr = 0, panel_i = 0, panel_blk = 0, item_ptr = 0,
      item_blk = 0, item_q = 0, len = 0;
  int max_panel = 0;  // most panel blocks in one column
};

struct BAPlan {
  int n_poses = 0, n_points = 0, n_obs = 0, n_fixed = 0, n_free = 0, n_te = 0;
  // internal order -> caller order
  PlanArr<int32_t> pt_perm;   // internal point q -> caller point index
  // observations in internal order (points by first camera, then camera)
  PlanArr<float> obs_uv;      // 2 per obs
  PlanArr<int32_t> obs_cam, obs_te;
  // track entries
  PlanArr<int32_t> te_cam, te_pt, te_obs;  // te_obs: n_te+1
  PlanArr<int16_t> te_lcam;                    // segment-local free camera, -1 if fixed
  PlanArr<int32_t> pt_te;                  // n_points+1
  // chunks
  std::vector<int32_t> chunk_obs, chunk_te, chunk_pt;  // n_chunks+1
  std::vector<int32_t> chunk_slot_base, chunk_cam_base;  // index into slot_ptr / cam_ptr
  // per chunk, kChunkHdr ints: every offset K1 needs to stage the chunk, so that one
  // (uniform) load precedes all list loads -- see ChunkHdr in ba.hip
  std::vector<int32_t> chunk_hdr;
  // slab positions: window slot s of the plan -> its row in the profile-major slab
  // (the inverse of prof_src), window camera e -> its row in the camera-major rhs slab
  // (the inverse of camb_src); K1 writes there so K2 reads contiguous rows
  std::vector<int32_t> slab_pos, cam_pos;
  std::vector<int32_t> seg_hdr;  // kSegHdr ints per segment
  std::vector<ChunkImg, PlanHostAlloc<ChunkImg>> chunk_img;
  PlanArr<int32_t> slot_ptr;   // per chunk: nslots(seg)+1 offsets into pair_list
  PlanArr<uint16_t> pair_list; // (te_x_local | te_y_local << 8)
  PlanArr<int32_t> cam_ptr;    // per chunk: ncams(seg)+1 offsets into cam_list
  PlanArr<uint8_t> cam_list;   // te local index
  PlanArr<int32_t> camo_ptr;   // same indexing as cam_ptr: offsets into camo_list
  PlanArr<uint8_t> camo_list;  // observation local index (U = Jc^T Jc of the camera)
  // segments
  std::vector<int32_t> seg_chunk, seg_slot_off, seg_cam_off;  // n_seg+1
  PlanArr<int32_t> slot_i, slot_j;   // per slab slot: global free-camera block (i >= j)
  PlanArr<int32_t> segcam_f;         // per slab b entry: free camera
  PlanArr<int32_t> segcam_diag;      // per slab b entry: its diagonal slot within the segment
  std::vector<int32_t> seg_acam_off, seg_acam;  // per segment: every camera its observations see
  std::vector<uint8_t> obs_acam;                // per observation: index into its segment's seg_acam
  // profile of S (block rows over free cameras)
  std::vector<int32_t> prof_first, prof_off, prof_last;  // F, F+1, F
  std::vector<int32_t> prof_src_ptr, prof_src;  // per profile block: slab slots
  std::vector<uint8_t> prof_diag;               // per profile block: 1 if i == j
  std::vector<int32_t> camb_ptr, camb_src;      // per free camera: slab b entries
  // K3 step tables (one packed int array, staged in LDS): for block column k,
  //   panel rows   i in (k, last[k]] with first[i] <= k       -> i, profile block (i, k)
  //   trailing     blocks (i_q1, i_q2), q2 <= q1 of the panel  -> profile block, q1 | q2 << 16
  // plus diag[k] (profile block (k, k)), off[k], first[k].
  std::vector<int32_t> solve_tab;
  SolveTableLayout solve_layout;
  // slide-stable packing: landmarks are ordered by first camera, and every first-camera
  // group is packed on its own (segments never cross a group), with seg_obs observations per
  // segment as the packing target.  group_q / group_chunk / group_seg: per first camera c
  // (0 .. N; N = landmarks without observations) its first landmark, chunk and segment.
  int seg_obs = 0;
  int seg_chunks = 0;  // wave plans: chunks per segment (1 .. kWaveMaxChunks); 0 otherwise
  std::vector<int32_t> group_q, group_chunk, group_seg;
  // Not part of the plan (never digested): how it was built.  chunk_src[c] = the chunk of
  // the previous plan whose image chunk c copies (an incremental build), -1 if rebuilt;
  // reused_groups / reused_chunks count the groups and chunks taken over.
  std::vector<int32_t> chunk_src;
  int reused_groups = 0, reused_chunks = 0;
  // true when this plan's host chunk_img holds stale bytes for the chunks it took over: a plan
  // with page-locked images takes them over on the device only (ba.hip setup), so its host copy
  // is not the plan a scratch build makes.  plan_digest and any other host reader of chunk_img
  // refuse such a plan (host-only plans, digests and probes, always copy the images).
  bool host_images_partial = false;
  // planner scratch (never digested; kept across plans so a session's next window reuses it)
  PlanArr<int32_t> scr_sorted;
  std::shared_ptr<PlanScratch> scratch;  // the planner's working containers (ba_plan.cpp)

  BAPlan() = default;
  explicit BAPlan(bool pinned_images) : chunk_img(PlanHostAlloc<ChunkImg>(pinned_images)) {}
  void reset();  // empty every array, keep its capacity (a session's next window reuses it)
  int n_chunks() const { return (int)chunk_obs.size() - 1; }
  int n_segments() const { return (int)seg_chunk.size() - 1; }
  int n_slab_slots() const { return (int)slot_i.size(); }
  int n_prof_blocks() const { return prof_off.empty() ? 0 : prof_off.back(); }
  int64_t algorithmic_bytes_per_iter() const;
};

// The packing target of a window of n_obs observations for target_segments K1 workgroups.
int seg_obs_for(int64_t n_obs, int target_segments);
// The smallest packing target of a fixed geometric grid (ceil(2^(k/8)), steps of ~9 %) that is
// >= x: a function of x alone, so windows of nearly equal size (consecutive keyframes) share a
// target, which group take-over needs, without making a plan depend on the window before it.
int seg_obs_grid(int64_t x);
// Builds everything except the profile (needs the global first[] on multi-GPU).
// Returns an empty string on success, else the error message.  With prev (the plan of the
// previous window on the same engine, built with the same seg_obs and n_fixed), every
// first-camera group whose landmarks equal a group of prev one camera later (the window slid
// by one keyframe) or at the same camera (the window grew, or the same window again) takes
// over that group's chunks and segments: lists and images copied, offsets and camera ids
// shifted, nothing repacked.  The result is the same plan, byte for byte, as without prev --
// except that a plan with page-locked images (the BA engine's) leaves the host copies of the
// images it takes over unwritten: the engine copies them from the previous plan's device images.
// seg_chunks: chunks per segment of a wave plan (seg_obs == 1; ignored otherwise).
std::string build_plan(BAPlan& plan, int n_poses, int n_points, int n_obs, int n_fixed,
                       const int32_t* point_ptr, const int32_t* obs_cam, const float* obs_uv,
                       int seg_obs, const BAPlan* prev = nullptr, int seg_chunks = 1);
// first[i] of each free block row touched by this plan (i if untouched).
std::vector<int32_t> local_profile_first(const BAPlan& plan);
// Builds the profile and the K2 reduction index from a (possibly all-reduced) first[];
// step_tables: also the profile solver's K3 step tables (solve_tab; skipped when the banded
// solver takes the window).
void build_profile(BAPlan& plan, const std::vector<int32_t>& first, bool step_tables = true);
// 64-bit FNV-1a over every plan array in a fixed order (vo_ba_plan_digest).
uint64_t plan_digest(const BAPlan& plan);

}  // namespace vo
