// Brute-force descriptor matcher: knn k=2 + Lowe ratio test on gfx950.
//
// Replaces cv2.BFMatcher(cv2.NORM_L2, crossCheck=False).knnMatch(k=2) and the
// Python ratio loop of FeatureFrontend.match_frames (reference
// src/modules/frontend.py:86-111).  Semantics:
//   dist(i,j) = sqrtf(d2(i,j)); the two nearest train rows per query are the two
//   smallest keys (dist, j) (equal distances keep the lower j -- OpenCV's
//   insertion scan with strict '<'); keep (i, j1) iff (double)dist1 < ratio *
//   (double)dist2.
//
// Integer path (all values integers in [0,255], as OpenCV SIFT produces): the
// descriptors are shifted to int8 (a - 128) -- d2 is shift invariant -- and
// d2 = |a'|^2 + |b'|^2 - 2 a'.b' is computed EXACTLY with
// v_mfma_i32_16x16x64_i8 (i32 accumulate).  The per-pair epilogue packs
// (d2 - |a'|^2 + Dp*2^14, column tile) into one u32 so that the running top-2 per
// (row, lane) is two branch-free ops: m2 = med3(m1, m2, p); m1 = min(m1, p).
// sqrtf can merge two integer d2 values only when they differ by 1 and are
// >= 2^22; rows whose second-best d2 reaches 2^22 are re-scanned exactly with
// sqrt-domain keys (never the case for real SIFT, whose d2 stays below ~1.1e6).
//
// Float path (any other values, e.g. SuperPoint): d2 is the k-ordered fmaf
// chain sum((a_k - b_k)^2) in fp32 and keys are (sqrtf(d2), j) directly.
#include "match_short.h"
#include <type_traits>

#ifndef VO_MATCH_WGS_PER_CU
#define VO_MATCH_WGS_PER_CU (VO_MATCH_MT == 2 ? 1 : 2)
#endif
// Tuning builds only (EXTRA=-D...): columns per LDS-staged B chunk (64 or 128) and
// s_setprio around each tile's MFMA issue.
#ifndef VO_MATCH_CHUNK
#define VO_MATCH_CHUNK (VO_MATCH_MT == 2 ? 128 : 64)
#endif
#ifndef VO_MATCH_PRIO
#define VO_MATCH_PRIO 0
#endif

namespace vo {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kKStep = 64;          // K of v_mfma_i32_16x16x64_i8
constexpr int kMaxDpInt = 256;      // int path keeps A fragments in registers
// M tiles of 16 query rows per wave (tuning builds: EXTRA=-DVO_MATCH_MT=2 gives 32-row waves,
// eight per workgroup, 128-column B chunks)
#ifndef VO_MATCH_MT
#define VO_MATCH_MT 2
#endif
constexpr int kMT = VO_MATCH_MT;
static_assert(kMT == 2 || kMT == 4, "two or four M tiles per wave");
constexpr int kRowsPerWave = 16 * kMT;
constexpr int kRowsPerWG = 256;     // 4 or 8 waves
constexpr int kMatchThreads = 64 * kRowsPerWG / kRowsPerWave;
constexpr int kMatchChunk = VO_MATCH_CHUNK;
constexpr bool kMatchPrio = VO_MATCH_PRIO != 0;
static_assert(kMatchChunk == 64 || kMatchChunk == 128, "B chunk of 64 or 128 columns");
// Key range: |a'|^2 <= Dp * 128^2 and d2 - |a'|^2 = sum(b'^2 - 2 a'b') <= Dp * 48896, so
// d2 - |a'|^2 lies in [-Dp * 16384, Dp * 48896]: 24 key bits + 8 column-tile bits.
// int8 path keys are kept in max form: ((2 a'.b' - |b'|^2 + off) << 8) | (255 - tile)
// = ((off - (d2 - |a'|^2)) << 8) | (255 - tile), off = Dp * 48896 + 1, so a valid key is
// in [1 << 8, (Dp * 65280 + 1) << 8] (< 2^32 for Dp <= 256) and larger = closer; ties in
// d2 prefer the lower column tile (lower train index), and 0 (padding) never wins.  One
// v_lshl_add_u32 forms a key from the MFMA dot product.
__host__ __device__ constexpr uint32_t max_off(int Dp) { return (uint32_t)Dp * 48896u + 1u; }
constexpr int kCollide = 1 << 22;   // sqrtf(n) == sqrtf(n+1) needs n >= 2^22
constexpr int kFloatTile = 64;      // float path: 64 rows x kFloatCols columns per WG tile
constexpr int kFloatCols = 128;     //   (4 rows x 8 columns per thread)
constexpr int kFloatKC = 16;        // float path: k-chunk staged in LDS

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  // not volatile: a pure function the scheduler may interleave with the MFMAs
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ uint32_t max3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_max3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// One step of a 16-lane top-2 reduction on u32 keys (larger = better): merge this
// lane's (M1 >= M2) with the pair of the lane `Ctrl` (a DPP row rotation) away.
// second(a1, a2, b1, b2) = med3(a1, b1, max(a2, b2)) since max(a2, b2) <= max(a1, b1).
template <int Ctrl>
__device__ __forceinline__ void row_top2_step(uint32_t& M1, uint32_t& M2) {
  const uint32_t b1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)M1, Ctrl, 0xF, 0xF, false);
  const uint32_t b2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)M2, Ctrl, 0xF, 0xF, false);
  M2 = med3_u32(M1, b1, max(M2, b2));
  M1 = max(M1, b1);
}

// Correctly rounded sqrtf: the f64 sqrt expansion is correctly rounded and
// 53 >= 2*24 + 2 makes the f64 -> f32 double rounding innocuous.
__device__ __forceinline__ float sqrtf_rn(float x) { return (float)sqrt((double)x); }

__device__ __forceinline__ uint64_t key64(uint32_t d, uint32_t j) {
  return ((uint64_t)d << 32) | j;
}

__device__ __forceinline__ void merge2(uint64_t& a1, uint64_t& a2, uint64_t b1, uint64_t b2) {
  const uint64_t lo = a1 < b1 ? a1 : b1;
  const uint64_t hi = a1 < b1 ? b1 : a1;
  const uint64_t m = a2 < b2 ? a2 : b2;
  a1 = lo;
  a2 = hi < m ? hi : m;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)v, m, 64);
  const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}

// ---- packing: f32 -> int8 (a - 128), squared norms, u8-valued check --------
// One launch packs both sides (workgroups [0, a.wgs) the queries, the rest the train
// rows).  16 threads per row, each moving 4 consecutive elements per step (one float4
// when the rows are 16-byte aligned).  A value that is not an integer in [0,255]
// stamps the call's generation into *flag: every later kernel of the call then takes
// the fp32 path, and no memset is needed between calls.
struct PackSide {
  const float* des;
  int n, n_pad, wgs;
  long in_bstride, q_bstride;
  int8_t* q8;
  int* norms;
  uint32_t* colconst;  // train side only
};

__global__ __launch_bounds__(256) void pack_kernel(PackSide sa, PackSide sb, int dim, int Dp,
                                                   int vec4, uint32_t* __restrict__ flag,
                                                   uint32_t gen, const uint32_t* __restrict__ qflag) {
  // a cached query side (sa.wgs == 0; packed by an earlier call into its own buffers): its
  // integer / finiteness verdicts (qflag, 1 = seen) join this call's flag
  if (qflag && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    if (qflag[0]) flag[0] = gen;
    if (qflag[1]) flag[1] = gen;
  }
  const bool is_b = (int)blockIdx.x >= sa.wgs;
  const PackSide P = is_b ? sb : sa;
  const int b = blockIdx.y;
  const int row = (((int)blockIdx.x - (is_b ? sa.wgs : 0)) * 256 + (int)threadIdx.x) >> 4;
  const int sub = threadIdx.x & 15;
  if (row >= P.n_pad) return;
  const bool live_row = row < P.n;
  const float* src = P.des + b * P.in_bstride + (long)row * dim;
  int8_t* dst = P.q8 + b * P.q_bstride + (long)row * Dp;
  int acc = 0;
  bool bad = false, nonfinite = false;
  for (int e = sub * 4; e < Dp; e += 64) {
    float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (live_row) {
      if (vec4) {
        if (e < dim) {
          const float4 t = *reinterpret_cast<const float4*>(src + e);
          v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        }
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (e + u < dim) v[u] = src[e + u];
      }
    }
    int q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool live = live_row && e + u < dim;
      const bool ok = (v[u] == rintf(v[u])) && v[u] >= 0.0f && v[u] <= 255.0f;
      bad |= live && !ok;
      nonfinite |= live && !isfinite(v[u]);
      q[u] = live && ok ? (int)v[u] - 128 : 0;
      acc += q[u] * q[u];
    }
    const uint32_t packed = (uint32_t)(q[0] & 255) | ((uint32_t)(q[1] & 255) << 8) |
                            ((uint32_t)(q[2] & 255) << 16) | ((uint32_t)(q[3] & 255) << 24);
    *reinterpret_cast<uint32_t*>(dst + e) = packed;
  }
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) acc += __shfl_xor(acc, m, 64);
  if (__any(bad) && (threadIdx.x & 63) == 0) flag[0] = gen;  // every writer stores the same value
  if (__any(nonfinite) && (threadIdx.x & 63) == 0) flag[1] = gen;  // the exact sweep handles it
  if (sub == 0) {
    P.norms[b * (long)P.n_pad + row] = acc;
    if (is_b) {
      P.colconst[b * (long)P.n_pad + row] =
          live_row ? ((max_off(Dp) - (uint32_t)acc) << 8) | (255u - ((uint32_t)(row >> 4) & 255u)) : 0u;
    }
  }
}

// ---- fused sweep + merge + ratio test ----------------------------------------
// Grid (n0_pad / 256, nsplit, batch); a workgroup owns 256 query rows x one split of
// train columns (split width w | 4096, so a split never straddles a 4096-column block
// and the 8-bit column-tile tag in the packed key is monotone in j inside a split).
// It writes one top-2 partial per row; merge_kernel combines the nsplit partials.
struct MatchArgs {
  const int8_t* qa;
  const int8_t* qb;
  const uint32_t* colconst;
  const int* norma;
  const float* da;
  const float* db;
  int n0, n1, dim, Dp, n0_pad, n1_pad, split_w, force_f32;
  int short_ok;  // float calls take the bf16 shortlist (match_bf16.hip) unless non-finite
  int exact_in_merge;  // int8 launch: merge_kernel runs the exact fp32 sweep for float values
  long qa_bstride, qb_bstride, a_bstride, b_bstride;
  uint4* partial;
  const uint32_t* flag;
  uint32_t gen;
  double ratio;
  int32_t* best;
  int32_t* idx2;
  float* dist2;
};

// Slot swizzle of the B chunk image (see sweep_i8), found by exhaustive search over strides
// and linear XOR patterns for the two gfx950 access patterns.
template <int KS>
__device__ __forceinline__ int i8_swz(int row) {
  if constexpr (KS == 1) return ((row >> 2) & 1) * 2;
  if constexpr (KS == 2) return (row * 5) & 7;
  if constexpr (KS == 4) return (row * 6) & 15;
  return 0;
}

// int8 MFMA sweep of one workgroup: 4 waves x 64 query rows
template <int KS>
__device__ __forceinline__ void sweep_i8(const MatchArgs& p) {
  const int8_t* qa = p.qa;
  const int8_t* qb = p.qb;
  const uint32_t* colconst = p.colconst;
  const int* norma = p.norma;
  const int n0_pad = p.n0_pad, n1_pad = p.n1_pad, split_w = p.split_w;
  const long qa_bstride = p.qa_bstride, qb_bstride = p.qb_bstride;
  uint4* partial = p.partial;
  constexpr int Dp = KS * kKStep;
  constexpr uint32_t kOffMax = max_off(Dp);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int b = blockIdx.z;
  const int split = blockIdx.y;
  const int nsplit = gridDim.y;
  const int rowbase = blockIdx.x * kRowsPerWG + wave * kRowsPerWave;
  const int8_t* A = qa + b * qa_bstride;
  const int8_t* B = qb + b * qb_bstride;
  const uint32_t* cc = colconst + b * (long)n1_pad;

  v4i afrag[kMT][KS];
#pragma unroll
  for (int mt = 0; mt < kMT; ++mt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      afrag[mt][ks] = *reinterpret_cast<const v4i*>(
          A + (long)(rowbase + mt * 16 + (lane & 15)) * Dp + ks * kKStep + 16 * (lane >> 4));

  uint32_t m1[kMT][4], m2[kMT][4];
#pragma unroll
  for (int mt = 0; mt < kMT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) m1[mt][r] = m2[mt][r] = 0u;

  const int c0 = split * split_w;
  const int c1 = min(c0 + split_w, n1_pad);
  // B is staged per chunk in LDS, shared by the workgroup's waves (one global fetch per
  // workgroup instead of one per wave).  Row r of the image holds column r's Dp bytes as Dp/16
  // slots of 16 bytes, slot s at s ^ i8_swz<KS>(r); staging thread t moves slots t & 3,
  // (t & 3) + 4, ... of row t >> 2 (four lanes load 64 contiguous bytes of a column).  For
  // KS = 1, 2, 4 the swizzle makes both gfx950 access patterns bank-conflict free with
  // unpadded rows: the ds_write_b128 staging (8 x 8 contiguous lanes, banks (a/4) mod 32) and
  // the fragment reads (ds_read_b128, 16-lane groups {0-3,12-15,20-27}, ..., banks (a/4) mod
  // 64; lane l: row l & 15, slot (l >> 4) + 4 ks).  Other KS: rows padded by 32 bytes.
  constexpr bool kSwz = KS == 1 || KS == 2 || KS == 4;
  constexpr int kRow = kSwz ? Dp : Dp + 32;
  constexpr int kCols = kMatchChunk;           // columns per staged chunk
  constexpr int kPieceCols = kMatchThreads / 4;  // columns one staging round covers
  constexpr int kNH = kCols / kPieceCols;       // staging rounds per chunk
  static_assert(kNH >= 1 && kCols % kPieceCols == 0, "B chunk staging");
  __shared__ __attribute__((aligned(16))) int8_t sB[2][kCols * kRow];
  __shared__ uint32_t sC[2][kCols];
  const int tid = threadIdx.x;
  auto gload = [&](int cbase, v4i (&g)[kNH][KS], uint32_t& gc) {
#pragma unroll
    for (int h = 0; h < kNH; ++h) {
      const int col = min(cbase + kPieceCols * h + (tid >> 2), c1 - 1);  // clamped, unconditional
      const int8_t* src = B + (long)col * Dp + 16 * (tid & 3);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) g[h][ks] = *reinterpret_cast<const v4i*>(src + 64 * ks);  // slot (t & 3) + 4 ks
    }
    gc = cc[min(cbase + (tid & (kCols - 1)), c1 - 1)];
  };
  static_assert(kPieceCols % 16 == 0, "the swizzle of row kPieceCols h + r is that of r");
  int st_off[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    st_off[ks] = (tid >> 2) * kRow + 16 * (((tid & 3) + 4 * ks) ^ (kSwz ? i8_swz<KS>(tid >> 2) : 0));
  auto sstore = [&](int buf, const v4i (&g)[kNH][KS], uint32_t gc) {
#pragma unroll
    for (int h = 0; h < kNH; ++h) {
      int8_t* dst = &sB[buf][kPieceCols * h * kRow];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) *reinterpret_cast<v4i*>(dst + st_off[ks]) = g[h][ks];
    }
    if (tid < kCols) sC[buf][tid] = gc;
  };
  // One 16-column tile: its B fragments and column constants from LDS (frag), the
  // four row tiles' MFMAs into separate accumulators (mm), then the top-2 update
  // (epi: v_lshl_add_u32 + v_med3_u32 + v_max_u32 per pair).
  struct Frag {
    v4i bf[KS];
    uint32_t cc;
  };
  struct Acc {
    v4i v[kMT];
  };
  // this lane's fragment offsets inside a 16-row tile (the swizzle of row 16 u + (lane & 15)
  // depends on lane & 15 only), and its staging offsets inside the image
  int rd_off[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    rd_off[ks] = (lane & 15) * kRow + 16 * (((lane >> 4) + 4 * ks) ^ (kSwz ? i8_swz<KS>(lane & 15) : 0));
  auto frag = [&](int buf, int u) {
    Frag f;
    const int8_t* fp = &sB[buf][16 * u * kRow];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) f.bf[ks] = *reinterpret_cast<const v4i*>(fp + rd_off[ks]);
    f.cc = sC[buf][16 * u + (lane & 15)];
    return f;
  };
  auto mm = [&](const Frag& f) {
    Acc a;
#pragma unroll
    for (int mt = 0; mt < kMT; ++mt) a.v[mt] = v4i{0, 0, 0, 0};
    if (kMatchPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mt = 0; mt < kMT; ++mt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        a.v[mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag[mt][ks], f.bf[ks], a.v[mt], 0, 0, 0);
    if (kMatchPrio) __builtin_amdgcn_s_setprio(0);
    return a;
  };
  auto epi = [&](const Acc& a, uint32_t ccol) {
#pragma unroll
    for (int mt = 0; mt < kMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t p = ((uint32_t)a.v[mt][r] << 9) + ccol;
        m2[mt][r] = med3_u32(m1[mt][r], m2[mt][r], p);
        m1[mt][r] = max(m1[mt][r], p);
      }
  };
  // two keys p, q of one (row, lane) at once (keys are unique, larger = better): the new best
  // is max3(m1, p, q) and the new second max(m2, med3(m1, p, q)) (m2 <= m1, so m2 can only be
  // second by beating the middle of the three)
  auto epi2 = [&](const Acc& a, uint32_t ca, const Acc& b, uint32_t cbk) {
#pragma unroll
    for (int mt = 0; mt < kMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t p = ((uint32_t)a.v[mt][r] << 9) + ca;
        const uint32_t q = ((uint32_t)b.v[mt][r] << 9) + cbk;
        m2[mt][r] = max(m2[mt][r], med3_u32(m1[mt][r], p, q));
        m1[mt][r] = max3_u32(m1[mt][r], p, q);
      }
  };
  if (c0 < c1) {  // uniform over the workgroup (split bounds)
    const int nchunk = (c1 - c0 + kCols - 1) / kCols;
    v4i g[kNH][KS];
    uint32_t gc;
    gload(c0, g, gc);
    sstore(0, g, gc);
    __syncthreads();
    // One chunk: its tiles in pairs, the two tiles' keys entering the top-2 together (epi2:
    // 5 VALU ops for two pairs of the same (row, lane) instead of 6); a lone last tile takes
    // epi.  Whole chunks (every tile in range) run as a loop of their own with no bounds
    // branch: the per-tile branches' joins made the compiler copy the 16 top-2 registers
    // of each tile pair (16 v_mov per 40 VALU ops of the epilogue).
    auto chunk = [&](int ch, auto whole) __attribute__((always_inline)) {
      const int buf = ch & 1, cb = c0 + kCols * ch;
      if (ch + 1 < nchunk) gload(cb + kCols, g, gc);  // in flight during this chunk
#pragma unroll
      for (int u = 0; u < kCols / 16; u += 2) {
        if (decltype(whole)::value || cb + 16 * (u + 1) < c1) {
          const Frag f0 = frag(buf, u), f1 = frag(buf, u + 1);
          epi2(mm(f0), f0.cc, mm(f1), f1.cc);
        } else if (cb + 16 * u < c1) {
          const Frag f = frag(buf, u);
          epi(mm(f), f.cc);
        }
      }
      if (ch + 1 < nchunk) sstore(buf ^ 1, g, gc);
      __syncthreads();
    };
    const int nwhole = (c1 - c0) / kCols;
    int ch = 0;
    for (; ch < nwhole; ++ch) chunk(ch, std::true_type{});
    for (; ch < nchunk; ++ch) chunk(ch, std::false_type{});
  }

  // Merge the 16 lanes that share each row (one DPP row) on the u32 keys: within a
  // split they are comparable across lanes, and equal keys mean equal d2 and tile, where
  // the lower lane (lower j) must win -- recovered by ballot after the value reduction.
  // Rotations by 1, 2, 4, 8 combine disjoint lane sets, so the top-2 merge is exact.
  const int jblock = c0 & ~4095;
  const int gshift = lane & 48;  // this lane's 16-lane group in a ballot mask
#pragma unroll
  for (int mt = 0; mt < kMT; ++mt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t a1 = m1[mt][r], a2 = m2[mt][r];
      uint32_t M1 = a1, M2 = a2;
      row_top2_step<0x121>(M1, M2);  // row_ror:1
      row_top2_step<0x122>(M1, M2);  // row_ror:2
      row_top2_step<0x124>(M1, M2);  // row_ror:4
      row_top2_step<0x128>(M1, M2);  // row_ror:8
      const uint32_t g1 = (uint32_t)(__ballot(a1 == M1) >> gshift) & 0xFFFFu;
      const uint32_t g2 = (uint32_t)(__ballot(a1 == M2 || a2 == M2) >> gshift) & 0xFFFFu;
      const uint32_t l1 = __builtin_ctz(g1 | 0x10000u);
      // M2 == M1 (two lanes tie exactly): the next such lane; else the lowest holder of M2
      const uint32_t l2 = __builtin_ctz((M2 == M1 ? g1 & ~(1u << l1) : g2) | 0x10000u);
      if ((lane & 15) == 0) {
        const int row = rowbase + mt * 16 + (lane >> 4) * 4 + r;
        const int na = norma[b * (long)n0_pad + row];
        uint4 q = make_uint4(~0u, ~0u, ~0u, ~0u);
        if (M1 != 0u) {
          q.x = kOffMax - (M1 >> 8) + na;
          q.y = jblock + 16 * (255u - (M1 & 255u)) + l1;
        }
        if (M2 != 0u) {
          q.z = kOffMax - (M2 >> 8) + na;
          q.w = jblock + 16 * (255u - (M2 & 255u)) + l2;
        }
        partial[((long)b * nsplit + split) * n0_pad + row] = q;
      }
    }
  }
}

// fp32 sweep of one 64-row tile: thread (ty, tx) owns rows 4ty..4ty+3 and columns
// tx + 16c.  Each pair's d2 is the fmaf chain over k in ascending order.  Per thread
// the columns arrive in ascending j, so a candidate can only enter the top-2 if
// d2 < d2(second): sqrtf is evaluated only then (exact filter, see header).
__device__ __forceinline__ void sweep_f32(const MatchArgs& p, int rowbase, int b, int split, int nsplit, int c0,
                                          int c1) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const float* da = p.da;
  const float* db = p.db;
  const int n0 = p.n0, dim = p.dim, n0_pad = p.n0_pad;
  const long a_bstride = p.a_bstride, b_bstride = p.b_bstride;
  uint4* partial = p.partial;
  // k-major tiles (rows padded by 16 bytes): a thread reads its 4 rows and its 8 columns
  // of one k as one and two 16-byte loads
  __shared__ __attribute__((aligned(16))) float sa[kFloatKC][kFloatTile + 4];
  __shared__ __attribute__((aligned(16))) float sb[kFloatKC][kFloatCols + 4];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const float* A = da + b * a_bstride;
  const float* B = db + b * b_bstride;

  float s1[4], s2[4], d1st[4], d2nd[4];
  int j1[4], j2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s1[i] = s2[i] = d1st[i] = d2nd[i] = __builtin_huge_valf();
    j1[i] = j2[i] = -1;
  }
  for (int ct = c0; ct < c1; ct += kFloatCols) {
    // acc[i][q] = the k-ordered fmaf chains of rows ty*4+i, columns tx*8+2q, tx*8+2q+1:
    // packed fp32 (v_pk_add_f32 / v_pk_fma_f32 are the same IEEE operations per element)
    f2 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[i][q] = f2{0.0f, 0.0f};
    for (int k0 = 0; k0 < dim; k0 += kFloatKC) {
      __syncthreads();
      for (int e = threadIdx.x; e < kFloatKC * kFloatTile; e += 256) {
        const int rr = e / kFloatKC, kk = e % kFloatKC;
        const int ga = rowbase + rr, gk = k0 + kk;
        sa[kk][rr] = (ga < n0 && gk < dim) ? A[(long)ga * dim + gk] : 0.0f;
      }
      for (int e = threadIdx.x; e < kFloatKC * kFloatCols; e += 256) {
        const int rr = e / kFloatKC, kk = e % kFloatKC;
        const int gb = ct + rr, gk = k0 + kk;
        sb[kk][rr] = (gb < c1 && gk < dim) ? B[(long)gb * dim + gk] : 0.0f;
      }
      __syncthreads();
      const int kc = min(kFloatKC, dim - k0);
      for (int kk = 0; kk < kc; ++kk) {
        const float4 a4 = *reinterpret_cast<const float4*>(&sa[kk][ty * 4]);
        const float4 bl = *reinterpret_cast<const float4*>(&sb[kk][tx * 8]);
        const float4 bh = *reinterpret_cast<const float4*>(&sb[kk][tx * 8 + 4]);
        const f2 bv[4] = {f2{bl.x, bl.y}, f2{bl.z, bl.w}, f2{bh.x, bh.y}, f2{bh.z, bh.w}};
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f2 a2 = f2{av[i], av[i]};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f2 df = a2 - bv[q];
            acc[i][q] = __builtin_elementwise_fma(df, df, acc[i][q]);
          }
        }
      }
    }
    // this lane's columns in ascending j (strict '<' keeps the lower j on equal s)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int j = ct + tx * 8 + c;
      if (j >= c1) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = (c & 1) ? acc[i][c >> 1].y : acc[i][c >> 1].x;
        if (d < d2nd[i]) {  // d2 >= d2(second) implies s >= s2: cannot enter
          const float s = sqrtf_rn(d);
          if (s < s1[i]) {
            s2[i] = s1[i]; j2[i] = j1[i]; d2nd[i] = d1st[i];
            s1[i] = s; j1[i] = j; d1st[i] = d;
          } else if (s < s2[i]) {
            s2[i] = s; j2[i] = j; d2nd[i] = d;
          }
        }
      }
    }
  }
  // merge across the 16 tx lanes of each row (keys: float bits of s, j)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint64_t k1 = j1[i] < 0 ? ~0ull : key64(__float_as_uint(s1[i]), (uint32_t)j1[i]);
    uint64_t k2 = j2[i] < 0 ? ~0ull : key64(__float_as_uint(s2[i]), (uint32_t)j2[i]);
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) merge2(k1, k2, shfl_xor64(k1, m), shfl_xor64(k2, m));
    const int row = rowbase + ty * 4 + i;
    if (tx == 0 && row < n0_pad) {
      partial[((long)b * nsplit + split) * n0_pad + row] =
          make_uint4((uint32_t)(k1 >> 32), (uint32_t)k1, (uint32_t)(k2 >> 32), (uint32_t)k2);
    }
  }
}

// Merge of the nsplit partials, one thread per query row (256-row workgroups), then
// the exact near-tie rescan (rare; a whole wave per flagged row) and the ratio test.
__global__ __launch_bounds__(256) void merge_kernel(MatchArgs p, int nsplit) {
  const bool fpath = p.force_f32 || p.flag[0] == p.gen;  // uniform
  if (fpath && p.short_ok && p.flag[1] != p.gen) return;  // frerank_kernel writes the outputs
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerWG + threadIdx.x;
  if (fpath && p.exact_in_merge) {
    // an int8-path launch whose values turned out not SIFT integers (or not finite): the
    // exact fp32 sweep of this block's rows over every train column here, as split 0 of 1
    // (rare; the int8 kernel keeps its registers to itself)
#pragma unroll 1
    for (int t = 0; t < kRowsPerWG / kFloatTile; ++t)
      sweep_f32(p, blockIdx.x * kRowsPerWG + t * kFloatTile, b, 0, 1, 0, p.n1);
    __syncthreads();  // the partials of this block's rows, written by this workgroup
    nsplit = 1;
  }
  uint64_t k1 = ~0ull, k2 = ~0ull;
  for (int s = 0; s < nsplit; ++s) {
    const uint4 q = p.partial[((long)b * nsplit + s) * p.n0_pad + row];
    merge2(k1, k2, key64(q.x, q.y), key64(q.z, q.w));
  }
  float s1 = __builtin_huge_valf(), s2 = __builtin_huge_valf();
  if (!fpath) {
    // (d2, j) order equals (sqrtf(d2), j) order unless sqrtf merges two
    // consecutive integers, which needs d2 >= 2^22 (see header).
    const bool rescan = row < p.n0 && k2 != ~0ull && (uint32_t)(k2 >> 32) >= (uint32_t)kCollide;
    uint64_t todo = __ballot(rescan);
    if (rescan) {
      k1 = k2 = ~0ull;
    } else {
      if (k1 != ~0ull) s1 = sqrtf_rn((float)(uint32_t)(k1 >> 32));
      if (k2 != ~0ull) s2 = sqrtf_rn((float)(uint32_t)(k2 >> 32));
    }
    // the whole wave re-scans each flagged row with sqrt-domain keys
    const int8_t* bb = p.qb + b * p.qb_bstride;
    while (todo) {
      const int l = __builtin_ctzll(todo);
      todo &= todo - 1;
      const int8_t* a = p.qa + b * p.qa_bstride + (long)(row - lane + l) * p.Dp;
      uint64_t r1 = ~0ull, r2 = ~0ull;
      for (int j = lane; j < p.n1; j += 64) {
        int d = 0;
        for (int e = 0; e < p.Dp; ++e) {
          const int df = (int)a[e] - (int)bb[(long)j * p.Dp + e];
          d += df * df;
        }
        merge2(r1, r2, key64(__float_as_uint(sqrtf_rn((float)d)), (uint32_t)j), ~0ull);
      }
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) merge2(r1, r2, shfl_xor64(r1, m), shfl_xor64(r2, m));
      if (lane == l) {
        k1 = r1;
        k2 = r2;
        if (k1 != ~0ull) s1 = __uint_as_float((uint32_t)(k1 >> 32));
        if (k2 != ~0ull) s2 = __uint_as_float((uint32_t)(k2 >> 32));
      }
    }
  } else {
    if (k1 != ~0ull) s1 = __uint_as_float((uint32_t)(k1 >> 32));
    if (k2 != ~0ull) s2 = __uint_as_float((uint32_t)(k2 >> 32));
  }
  if (row < p.n0) {
    const int j1 = k1 == ~0ull ? -1 : (int)(uint32_t)k1;
    const int j2 = k2 == ~0ull ? -1 : (int)(uint32_t)k2;
    const long o = (long)b * p.n0 + row;
    if (p.best) p.best[o] = (j2 >= 0 && (double)s1 < p.ratio * (double)s2) ? j1 : -1;
    if (p.idx2) {
      p.idx2[2 * o] = j1;
      p.idx2[2 * o + 1] = j2;
      p.dist2[2 * o] = j1 >= 0 ? s1 : 3.402823466e+38f;
      p.dist2[2 * o + 1] = j2 >= 0 ? s2 : 3.402823466e+38f;
    }
  }
}

// The int8 sweep only: a call whose values are not SIFT integers (decided on the device by
// pack_kernel) takes the exact fp32 sweep inside merge_kernel, so this kernel's registers and
// LDS are its own, not the maximum of both paths'.
template <int KS>
__global__ __launch_bounds__(kMatchThreads) void match_kernel(MatchArgs p) {
  const bool fpath = p.force_f32 || p.flag[0] == p.gen;  // uniform
  if (!fpath) sweep_i8<KS>(p);
}

// descriptors wider than the int8 kernel takes (Dp > 256): the exact fp32 sweep is the path
__global__ __launch_bounds__(256) void match_f32_kernel(MatchArgs p) {
  const int c0 = blockIdx.y * p.split_w, c1 = min(c0 + p.split_w, p.n1);
#pragma unroll 1
  for (int t = 0; t < kRowsPerWG / kFloatTile; ++t)
    sweep_f32(p, blockIdx.x * kRowsPerWG + t * kFloatTile, blockIdx.z, blockIdx.y, gridDim.y, c0, c1);
}

// n1 == 0: no query has a neighbour
__global__ void no_train_kernel(int total, int32_t* best, int32_t* idx2, float* dist2) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= total) return;
  if (best) best[o] = -1;
  if (idx2) {
    idx2[2 * o] = idx2[2 * o + 1] = -1;
    dist2[2 * o] = dist2[2 * o + 1] = 3.402823466e+38f;
  }
}

// ---- stream compaction of best[] into ascending (query, train) pairs ---------
__global__ __launch_bounds__(1024) void compact_kernel(const int32_t* __restrict__ best,
                                                       int n0, int32_t* __restrict__ pairs,
                                                       int32_t* __restrict__ count) {
  __shared__ int wsum[16];
  __shared__ int base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int start = 0; start < n0; start += 1024) {
    const int i = start + threadIdx.x;
    const int v = i < n0 ? best[i] : -1;
    const unsigned long long mask = __ballot(v >= 0);
    const int pre = __popcll(mask & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(mask);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wave; ++w) off += wsum[w];
    if (v >= 0) {
      pairs[2 * (off + pre)] = i;
      pairs[2 * (off + pre) + 1] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int w = 0; w < 16; ++w) t += wsum[w];
      base += t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = base;
}

int pow2_floor(int x) {
  int p = 1;
  while (p * 2 <= x) p *= 2;
  return p;
}

}  // namespace

// Packs one query side (batch 1) into the cache's own buffers, with its own flag words
// (generation 1: [0] = 1 if a value is not an integer in [0, 255], [1] = 1 if one is not finite).
void match_pack_query(vo_ctx* ctx, const float* d_des0, int n0, int dim, MatchQueryCache& qc) {
  hipStream_t st = ctx->stream;
  const int Dp = ceil_div(dim, kKStep) * kKStep;
  const int n0_pad = ceil_div(std::max(n0, 1), kRowsPerWG) * kRowsPerWG;
  qc.q8.reserve((size_t)n0_pad * Dp);
  qc.norms.reserve((size_t)n0_pad * sizeof(int));
  qc.flag.reserve(2 * sizeof(uint32_t));
  VO_HIP_CHECK(hipMemsetAsync(qc.flag.ptr, 0, 2 * sizeof(uint32_t), st));
  PackSide pa{d_des0, n0, n0_pad, ceil_div((int64_t)n0_pad * 16, 256), (long)n0 * dim, (long)n0_pad * Dp,
              qc.q8.as<int8_t>(), qc.norms.as<int>(), nullptr};
  PackSide pb{nullptr, 0, 0, 0, 0, 0, nullptr, nullptr, nullptr};
  const int vec4 = dim % 4 == 0 && (uintptr_t)d_des0 % 16 == 0;
  ctx->prof.begin(st, kKMatchPack);
  hipLaunchKernelGGL(pack_kernel, dim3(pa.wgs, 1), dim3(256), 0, st, pa, pb, dim, Dp, vec4, qc.flag.as<uint32_t>(),
                     1u, (const uint32_t*)nullptr);
  ctx->prof.end(st);
  VO_HIP_CHECK(hipGetLastError());
}

void match_run(vo_ctx* ctx, const float* d_des0, const float* d_des1, int batch, int n0,
               int n1, int dim, double ratio, int32_t* d_best, int32_t* d_idx2,
               float* d_dist2, const MatchQueryCache* qc) {
  VO_REQUIRE(batch >= 1 && n0 >= 0 && n1 >= 0 && dim >= 1, VO_ERR_ARG,
             "match: bad shape batch=%d n0=%d n1=%d dim=%d", batch, n0, n1, dim);
  if (n0 == 0) return;
  hipStream_t st = ctx->stream;
  MatchWorkspace& ws = ctx->match;
  const int Dp = ceil_div(dim, kKStep) * kKStep;
  const bool int_ok = Dp <= kMaxDpInt;
  const int n0_pad = ceil_div(n0, kRowsPerWG) * kRowsPerWG;
  const int n1_pad = ceil_div(std::max(n1, 1), 16) * 16;

  // split the train columns so the grid fills the chip (w | 4096, w >= 64); the split
  // count does not change any result (splits merge on exact (d^2, j) keys)
  const int row_wgs = n0_pad / kRowsPerWG;
  constexpr int wgs_per_cu = VO_MATCH_WGS_PER_CU;  // tuning builds: EXTRA=-DVO_MATCH_WGS_PER_CU=n
  const int want = std::max(1, ceil_div(wgs_per_cu * ctx->num_cus, (int64_t)row_wgs * batch));
  int w = pow2_floor(std::max(1, n1_pad / want));
  w = std::max(256, std::min(4096, w));
  const int nsplit = std::max(1, ceil_div(n1_pad, w));

  ws.flag.reserve(2 * sizeof(uint32_t));
  ws.partial.reserve((size_t)batch * nsplit * n0_pad * sizeof(uint4));
  // generation tag of this call (see pack_kernel); 0 is the reset value of the flag
  if (++ws.gen == 0 || ws.flag_fresh) {
    VO_HIP_CHECK(hipMemsetAsync(ws.flag.ptr, 0, 2 * sizeof(uint32_t), st));
    ws.gen = 1;
    ws.flag_fresh = false;
  }
  uint32_t* flag = ws.flag.as<uint32_t>();

  MatchArgs a{};
  a.da = d_des0;
  a.db = d_des1;
  a.n0 = n0;
  a.n1 = n1;
  a.dim = dim;
  a.Dp = Dp;
  a.n0_pad = n0_pad;
  a.n1_pad = n1_pad;
  a.split_w = w;
  // dim <= 256: the shortlist's A fragments fit in VGPRs; a SIFT hint leaves it unlaunched
  // (float values then take the exact sweep).  A float hint skips the int8 pack and its
  // integer check: the shortlist is exact for any finite values, SIFT integers included (their
  // fp32 chains of <= 256 squared byte differences stay below 2^24, so F = the integer d^2 and
  // the (sqrtf, j) keys order as the integer path's), and fpack flags non-finite values itself.
  const bool float_hint = int_ok && ws.kind_hint == VO_DESC_FLOAT;
  a.force_f32 = int_ok && !float_hint ? 0 : 1;
  a.short_ok = int_ok && ws.kind_hint != VO_DESC_SIFT ? 1 : 0;
  a.exact_in_merge = int_ok ? 1 : 0;
  a.a_bstride = (long)n0 * dim;
  a.b_bstride = (long)n1 * dim;
  a.partial = ws.partial.as<uint4>();
  a.flag = flag;
  a.gen = ws.gen;
  a.ratio = ratio;
  a.best = d_best;
  a.idx2 = d_idx2;
  a.dist2 = d_dist2;
  if (n1 == 0) {
    const int total = batch * n0;
    hipLaunchKernelGGL(no_train_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, st, total,
                       d_best, d_idx2, d_dist2);
    VO_HIP_CHECK(hipGetLastError());
    return;
  }
  if (int_ok && !float_hint) {
    // a cached query side (batch 1: match_pack_query packed it for an earlier call) is read
    // from the cache's buffers; only the train side is packed
    const bool cached = qc != nullptr && batch == 1;
    a.qa_bstride = (long)n0_pad * Dp;
    a.qb_bstride = (long)n1_pad * Dp;
    ws.q8.reserve((size_t)batch * (a.qa_bstride + a.qb_bstride));
    ws.norms.reserve((size_t)batch * (n0_pad + n1_pad) * sizeof(int));
    ws.colconst.reserve((size_t)batch * n1_pad * sizeof(uint32_t));
    int8_t* qa = cached ? qc->q8.as<int8_t>() : ws.q8.as<int8_t>();
    int8_t* qb = ws.q8.as<int8_t>() + batch * a.qa_bstride;
    int* na = cached ? qc->norms.as<int>() : ws.norms.as<int>();
    int* nb = ws.norms.as<int>() + (size_t)batch * n0_pad;
    a.qa = qa;
    a.qb = qb;
    a.colconst = ws.colconst.as<uint32_t>();
    a.norma = na;
    PackSide pa{d_des0, n0, n0_pad, cached ? 0 : ceil_div((int64_t)n0_pad * 16, 256), a.a_bstride,
                a.qa_bstride, qa, na, nullptr};
    PackSide pb{d_des1, n1, n1_pad, ceil_div((int64_t)n1_pad * 16, 256), a.b_bstride,
                a.qb_bstride, qb, nb, ws.colconst.as<uint32_t>()};
    const int vec4 = dim % 4 == 0 && (uintptr_t)d_des0 % 16 == 0 && (uintptr_t)d_des1 % 16 == 0;
    ctx->prof.begin(st, kKMatchPack);
    hipLaunchKernelGGL(pack_kernel, dim3(pa.wgs + pb.wgs, batch), dim3(256), 0, st, pa, pb, dim,
                       Dp, vec4, flag, ws.gen, cached ? qc->flag.as<uint32_t>() : (const uint32_t*)nullptr);
    ctx->prof.end(st);
  }
  auto sweep = [&]() {  // int8 sweep, and the exact fp32 sweep (float calls the shortlist cannot take)
    dim3 grid(row_wgs, nsplit, batch);
    if (int_ok) {
      ctx->prof.begin(st, kKMatchI8);
      switch (Dp / kKStep) {
        case 1: hipLaunchKernelGGL(match_kernel<1>, grid, dim3(kMatchThreads), 0, st, a); break;
        case 2: hipLaunchKernelGGL(match_kernel<2>, grid, dim3(kMatchThreads), 0, st, a); break;
        case 3: hipLaunchKernelGGL(match_kernel<3>, grid, dim3(kMatchThreads), 0, st, a); break;
        default: hipLaunchKernelGGL(match_kernel<4>, grid, dim3(kMatchThreads), 0, st, a); break;
      }
      ctx->prof.end(st);
    } else {
      ctx->prof.begin(st, kKMatchF32);
      hipLaunchKernelGGL(match_f32_kernel, grid, dim3(256), 0, st, a);
      ctx->prof.end(st);
    }
  };
  // under the float hint no exact sweep or merge is launched: fpack raises the non-finite
  // flag and frerank_kernel then answers the call by an exact scan itself
  if (!float_hint) sweep();
  if (a.short_ok) {  // float calls: bf16 MFMA shortlist + exact re-rank (match_bf16.hip)
    ShortArgs s{};
    s.da = d_des0;
    s.db = d_des1;
    s.n0 = n0;
    s.n1 = n1;
    s.dim = dim;
    s.Dp = short_Dp(dim);
    s.n0_pad = n0_pad;
    s.n1_pad = n1_pad;
    s.split_w = w;
    s.nsplit = nsplit;
    s.a_bstride = a.a_bstride;
    s.b_bstride = a.b_bstride;
    s.flag = flag;
    s.gen = ws.gen;
    s.forced = float_hint ? 1 : 0;
    s.ratio = ratio;
    s.best = d_best;
    s.idx2 = d_idx2;
    s.dist2 = d_dist2;
    ws.hbf.reserve((size_t)batch * (n0_pad + n1_pad) * s.Dp * 2);
    s.ha = ws.hbf.as<__bf16>();
    s.hb = s.ha + (size_t)batch * n0_pad * s.Dp;
    ws.fnorm.reserve((size_t)batch * (n0_pad + n1_pad) * sizeof(float));
    s.nbq = ws.fnorm.as<float>();
    s.ra = s.nbq + (size_t)batch * n1_pad;
    if (ws.bmax.bytes < (size_t)batch * kBmaxStride * sizeof(uint32_t)) {
      ws.bmax.reserve((size_t)batch * kBmaxStride * sizeof(uint32_t));
      VO_HIP_CHECK(hipMemsetAsync(ws.bmax.ptr, 0, ws.bmax.bytes, st));
    }
    s.bmax = ws.bmax.as<uint32_t>();
    // (batch, nsplit_f, n0_pad) float2; short_launch picks nsplit_f <= ceil(n1_pad / 64)
    ws.fpart.reserve((size_t)batch * ceil_div(n1_pad, 64) * n0_pad * sizeof(float2));
    s.part = ws.fpart.as<float2>();
    ws.cand.reserve((size_t)batch * (n0_pad / 32) * ceil_div(n1_pad, 64) * 64 * sizeof(uint32_t));
    s.mask = ws.cand.as<uint32_t>();
    short_launch(ctx, s, batch);
  }
  if (!float_hint) {
    ctx->prof.begin(st, kKMatchMerge);
    hipLaunchKernelGGL(merge_kernel, dim3(row_wgs, batch), dim3(256), 0, st, a, nsplit);
    ctx->prof.end(st);
  }
  VO_HIP_CHECK(hipGetLastError());
}

void compact_pairs(vo_ctx* ctx, const int32_t* d_best, int n0, int32_t* d_pairs,
                   int32_t* d_count) {
  hipLaunchKernelGGL(compact_kernel, dim3(1), dim3(1024), 0, ctx->stream, d_best, n0,
                     d_pairs, d_count);
  VO_HIP_CHECK(hipGetLastError());
}

}  // namespace vo
