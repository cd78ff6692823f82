// Float-descriptor matcher (SuperPoint-like, BASELINE config 5) on the matrix cores:
// a bf16 MFMA shortlist followed by an exact fp32 re-rank, bit-exact against
// oracle/match_ref.c (k-ordered fmaf chain, keys (sqrtf(d2), j), OpenCV's tie rule).
// Replaces the same cv2.BFMatcher(NORM_L2).knnMatch(k=2) + ratio loop as the integer
// path (reference src/modules/frontend.py:86-111; the LightGlue branch :80-84 is what
// config 5 swaps for brute force).
//
// Why a shortlist is exact.  Let D_j be the exact squared distance of query a to train
// row b_j, F_j the fp32 fmaf chain the oracle computes, and A_j the shortlist value
// |b'_j|^2 - 2 a'.b'_j + |a'|^2 with a', b' the bf16 (round to nearest even, unit
// roundoff 2^-8) images, products exact in fp32 and sums in fp32 (the row constant
// |a'|^2 is dropped: it does not change a row's ranking).  Then
//   |A_j - D_j| <= 2^-8 (|a| + |b_j|)^2 (2 + 2^-8) + (n + 4) 2^-24 (|a| + |b_j|)^2,
//   |F_j - D_j| <= (n + 4) 2^-24 (|a| + |b_j|)^2                     (n = dim <= 256),
// so |A_j - F_j| <= E = c (|a| + max_j |b_j|)^2 with c = 1.25 (2^-7 + 4e-5) (a 25 %
// margin).  With m2 the second smallest A of the row, the second smallest F is at most
// m2 + E, and every j whose F does not exceed it has A_j <= m2 + 2E.  So the candidate set
// {j : A_j <= m2 + 2E} holds every pair the exact top-2 can take (ties included), and
// ranking the candidates by their exact fp32 chains reproduces the oracle.  Candidates
// are recorded as bit masks (one 32-bit word per lane and 64-column chunk), so the set is
// complete whatever its size, and the re-rank is deterministic.
//
// Kernels (one call, every launch exits at once unless the call's descriptors took the
// float path -- pack_kernel's device-side flag -- and are finite, dim <= 256):
//   fpack   bf16 images of both sides, |b'|^2 per train row (+inf for padding), |a| and
//           max |b| (the bound)
//   fsweep<1>  v_mfma_f32_16x16x32_bf16 sweep, top-2 of A per (row, split)
//   fsweep<2>  the same sweep again: every A <= m2 + 2E marked in its lane's chunk word
//   frerank    one workgroup per 16 query rows: exact fmaf chains of the pooled candidates, top-2 by
//              (sqrtf(d2), j), ratio test (the merge_kernel outputs)
#include "match_short.h"

namespace vo {

typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int kShortMT = 2;                      // 16-row M tiles per wave (4: 256 VGPRs + AGPRs, one wave per SIMD, 180 us for both sweeps against 133)
constexpr int kShortRowsPerWG = 64 * kShortMT;  // 4 waves x 16 kShortMT query rows
constexpr float kShortC = 1.25f * (0.0078125f + 4e-5f);

namespace {

__device__ __forceinline__ bool short_active(const ShortArgs& p) {
  return (p.forced || p.flag[0] == p.gen) && p.flag[1] != p.gen;  // uniform
}

// Candidate masks of fsweep<2>: per (frame pair, 32-row wave group, 64-column chunk) one
// 32-bit word per lane; bit 8 u + 4 mt + r = row 32 rg + 16 mt + 4 (lane >> 4) + r, column
// 64 ch + 16 u + (lane & 15).  Index of the chunk's first word:
static_assert(kShortMT == 2, "32 candidate bits per lane and chunk: 4 tiles x 2 M tiles x 4 rows");
__device__ __forceinline__ long short_mask_word(const ShortArgs& p, int b, int rg, int ch) {
  return (((long)b * (p.n0_pad / 32) + rg) * ((p.n1_pad + 63) / 64) + ch) * 64;
}

__device__ __forceinline__ float med3_f32(float a, float b, float c) {
  float r;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// IEEE minNum without fminf's operand canonicalisation (the compiler quiets a loop-carried
// operand with v_max_f32 x, x, x before every v_min_f32): the running minima here come from
// v_min / v_med3 and the keys from v_fma, never signalling NaNs, so the result is the same
__device__ __forceinline__ float min_f32(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// ---- bf16 images, norms ------------------------------------------------------------
// 16 threads per row, 8 consecutive elements per thread and step.  Rows past n are
// written as zeros (train padding rows get |b'|^2 = +inf: never a candidate).
__global__ __launch_bounds__(256) void fpack_kernel(ShortArgs p, int a_wgs, int v4) {
  if (!p.forced && !short_active(p)) return;
  const bool is_b = (int)blockIdx.x >= a_wgs;
  const int b = blockIdx.y;
  const int n = is_b ? p.n1 : p.n0, n_pad = is_b ? p.n1_pad : p.n0_pad;
  const int row = (((int)blockIdx.x - (is_b ? a_wgs : 0)) * 256 + (int)threadIdx.x) >> 4;
  const int sub = threadIdx.x & 15;
  const bool in = row < n_pad;  // every thread reaches the workgroup reduction below
  const bool live = row < n;
  const float* src = (is_b ? p.db + b * p.b_bstride : p.da + b * p.a_bstride) + (long)row * p.dim;
  __bf16* dst = (is_b ? p.hb + (long)b * p.n1_pad * p.Dp : p.ha + (long)b * p.n0_pad * p.Dp) + (long)row * p.Dp;
  float q2 = 0.0f, x2 = 0.0f;
  bool nonfinite = false;
  if (v4 && p.dim == p.Dp && n > 0) {
    // fast path (16-byte rows, dim a multiple of 32): a thread's <= two groups of 8 elements
    // (k = 8 sub and 8 sub + 128), all four float4 loads issued first from a clamped row
    // (dead rows read row n - 1 and convert zeros), no per-element guard
    const float* s0 = (is_b ? p.db + b * p.b_bstride : p.da + b * p.a_bstride) + (long)min(row, n - 1) * p.dim;
    const int k0 = 8 * sub, k1 = k0 + 128;
    const bool g0 = in && k0 < p.Dp, g1 = in && k1 < p.Dp;
    const float4* q = reinterpret_cast<const float4*>(s0);
    const float4 x0 = q[min(k0, p.Dp - 8) / 4], x1 = q[min(k0, p.Dp - 8) / 4 + 1];
    const float4 x2v = q[min(k1, p.Dp - 8) / 4], x3 = q[min(k1, p.Dp - 8) / 4 + 1];
    const float vv[16] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w,
                          x2v.x, x2v.y, x2v.z, x2v.w, x3.x, x3.y, x3.z, x3.w};
#pragma unroll
    for (int gi = 0; gi < 2; ++gi) {
      const bool use = (gi == 0 ? g0 : g1) && live;
      v8bf h;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float v = use ? vv[8 * gi + u] : 0.0f;
        const __bf16 hv = (__bf16)v;
        const float hf = (float)hv;
        h[u] = hv;
        q2 = fmaf(hf, hf, q2);
        x2 = fmaf(v, v, x2);
        nonfinite |= !isfinite(v);
      }
      if (gi == 0 ? g0 : g1) *reinterpret_cast<v8bf*>(dst + (gi == 0 ? k0 : k1)) = h;
    }
    // the row's 16 lanes: quad_perm xor 1, xor 2, then row_half_mirror and row_mirror (every
    // lane ends with the row sum; a fixed order, inside the bound's summation allowance)
    auto rsum = [](float v) __attribute__((always_inline)) {
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
      return v;
    };
    q2 = rsum(q2);
    x2 = rsum(x2);
  } else {
  for (int e = sub * 8; in && e < p.Dp; e += 128) {
    v8bf h;
    float vv[8];
    if (v4 && live && e + 8 <= p.dim) {
      const float4 x0 = *reinterpret_cast<const float4*>(src + e);
      const float4 x1 = *reinterpret_cast<const float4*>(src + e + 4);
      vv[0] = x0.x; vv[1] = x0.y; vv[2] = x0.z; vv[3] = x0.w;
      vv[4] = x1.x; vv[5] = x1.y; vv[6] = x1.z; vv[7] = x1.w;
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) vv[u] = (live && e + u < p.dim) ? src[e + u] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float v = vv[u];
      const __bf16 hv = (__bf16)v;
      const float hf = (float)hv;
      h[u] = hv;
      q2 = fmaf(hf, hf, q2);
      x2 = fmaf(v, v, x2);
      nonfinite |= !isfinite(v);  // padding is 0
    }
    *reinterpret_cast<v8bf*>(dst + e) = h;
  }
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) {
    q2 += __shfl_xor(q2, m, 64);
    x2 += __shfl_xor(x2, m, 64);
  }
  }
  // float hint (no int8 pack): a non-finite value sends the call to the exact fp32 sweep
  if (p.forced && __any(nonfinite) && (threadIdx.x & 63) == 0) const_cast<uint32_t*>(p.flag)[1] = p.gen;
  // norms rounded up by a few ulps: the bound only needs upper estimates
  const float r = sqrtf(x2) * 1.0001f;
  if (sub == 0 && in) {
    if (is_b) p.nbq[(long)b * p.n1_pad + row] = live ? q2 : __builtin_huge_valf();
    else p.ra[(long)b * p.n0_pad + row] = r;
  }
  if (!is_b) return;
  // max |b| of the workgroup's 16 rows, then one atomic per workgroup (not per row: same-
  // address atomics serialise)
  uint32_t m = live ? __float_as_uint(r) : 0u;
#pragma unroll
  for (int k = 16; k < 64; k <<= 1) m = max(m, (uint32_t)__shfl_xor((int)m, k, 64));
  __shared__ uint32_t wmax[4];
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
    if (m) atomicMax(p.bmax + kBmaxStride * b, m);
  }
}

// ---- bf16 MFMA sweep ---------------------------------------------------------------
// Grid (n0_pad / kShortRowsPerWG, nsplit, batch).  Wave w holds the A fragments of query rows
// rowbase .. rowbase + 16 kShortMT - 1 (kShortMT M tiles: every B fragment read from LDS feeds
// kShortMT MFMAs) in VGPRs; train columns arrive in 64-column chunks staged in
// LDS (one global fetch per workgroup, double-buffered, rows padded by 16 bytes).  A
// 16-column tile: B fragments from LDS, KS MFMAs per M tile, then per (row, column)
// A' = |b'|^2 - 2 a'.b' and PASS 1: running top-2 (v_min_f32 + v_med3_f32), PASS 2: the
// candidate test.
template <int PASS, int KS>
__global__ __launch_bounds__(256) void fsweep_kernel(ShortArgs p) {
  if (!short_active(p)) return;
  constexpr int Dp = 32 * KS;
  // B chunk image in LDS: rows of Dp + 32 bf16 (Dp / 8 + 4 16-byte slots), slot s of row r
  // stored at slot s ^ ((2 r) & (Dp / 8 - 1)) (power-of-two Dp / 8).  The staging thread t
  // moves slots t & 3, (t & 3) + 4, ... of row t >> 2 (so four lanes load 64 contiguous bytes
  // of a row), and with this stride and swizzle both gfx950 access patterns are bank-conflict
  // free: the ds_write_b128 staging (8 x 8 contiguous lanes, banks (a/4) mod 32) and the
  // fragment reads (ds_read_b128, 16-lane groups {0-3,12-15,20-27}, ..., banks (a/4) mod 64;
  // lane l: row l & 15, slot l >> 4).  Round 2's Dp + 8 rows with 128 contiguous bytes per
  // thread were 4-way on every staging store and 2-way on every fragment read.
  constexpr int kRow = Dp + 32;
  constexpr int kNS = Dp / 8;
  constexpr int kSwz = (kNS & (kNS - 1)) == 0 ? kNS - 1 : 0;
  auto swz = [](int row, int slot) { return slot ^ ((2 * row) & kSwz); };
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int b = blockIdx.z, split = blockIdx.y, nsplit = p.nsplit;
  const int rowbase = blockIdx.x * kShortRowsPerWG + wave * 16 * kShortMT;
  const __bf16* A = p.ha + (long)b * p.n0_pad * Dp;
  const __bf16* B = p.hb + (long)b * p.n1_pad * Dp;
  const float* nbq = p.nbq + (long)b * p.n1_pad;

  v8bf af[kShortMT][KS];
#pragma unroll
  for (int mt = 0; mt < kShortMT; ++mt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      af[mt][ks] = *reinterpret_cast<const v8bf*>(A + (long)(rowbase + 16 * mt + (lane & 15)) * Dp + 32 * ks +
                                                  8 * (lane >> 4));

  // this lane's rows: 16 mt + 4 (lane >> 4) + r
  float m1[kShortMT][4], m2[kShortMT][4], thr[kShortMT][4];
  if (PASS == 1) {
#pragma unroll
    for (int mt = 0; mt < kShortMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) m1[mt][r] = m2[mt][r] = __builtin_huge_valf();
  } else {
    const float bm = __uint_as_float(p.bmax[kBmaxStride * b]);
#pragma unroll
    for (int mt = 0; mt < kShortMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rowbase + 16 * mt + 4 * (lane >> 4) + r;
        float a1 = __builtin_huge_valf(), a2 = __builtin_huge_valf();
        for (int s = 0; s < nsplit; ++s) {
          const float2 q = p.part[((long)b * nsplit + s) * p.n0_pad + row];
          a2 = med3_f32(a1, q.x, fminf(a2, q.y));
          a1 = fminf(a1, q.x);
        }
        const float ra = p.ra[(long)b * p.n0_pad + row] + bm;
        // +inf when the row has < 2 columns; padding rows take nothing
        thr[mt][r] = row < p.n0 ? a2 + 2.0f * kShortC * ra * ra : -__builtin_huge_valf();
      }
  }

  const int c0 = split * p.split_w;
  const int c1 = min(c0 + p.split_w, p.n1_pad);
  __shared__ __attribute__((aligned(16))) __bf16 sB[2][64 * kRow];
  __shared__ float sN[2][64];
  typedef int v4i __attribute__((ext_vector_type(4)));
  auto gload = [&](int cbase, v4i (&g)[KS], float& gn) {
    const int col = min(cbase + (tid >> 2), c1 - 1);
    const __bf16* src = B + (long)col * Dp + 8 * (tid & 3);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) g[ks] = *reinterpret_cast<const v4i*>(src + 32 * ks);  // slot (t & 3) + 4 ks
    gn = nbq[min(cbase + (tid & 63), c1 - 1)];
  };
  auto sstore = [&](int buf, const v4i (&g)[KS], float gn) {
    const int row = tid >> 2;
    __bf16* dst = &sB[buf][row * kRow];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) *reinterpret_cast<v4i*>(dst + 8 * swz(row, (tid & 3) + 4 * ks)) = g[ks];
    if (tid < 64) sN[buf][tid] = gn;
  };
  if (c0 < c1) {
    const int nchunk = (c1 - c0 + 63) / 64;
    v4i g[KS];
    float gn;
    gload(c0, g, gn);
    sstore(0, g, gn);
    __syncthreads();
    for (int ch = 0; ch < nchunk; ++ch) {
      const int buf = ch & 1, cb = c0 + 64 * ch;
      if (ch + 1 < nchunk) gload(cb + 64, g, gn);
      uint32_t bits = 0;  // PASS 2: this lane's candidates of the chunk, bit 8 u + 4 mt + r
      // the chunk's four 16-column tiles x four M tiles: sixteen independent accumulators,
      // k-step outer, so consecutive MFMAs never wait on each other
      v4f acc[4][kShortMT];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int mt = 0; mt < kShortMT; ++mt) acc[u][mt] = v4f{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        v8bf bf[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          bf[u] = *reinterpret_cast<const v8bf*>(
              &sB[buf][(16 * u + (lane & 15)) * kRow + 8 * swz(lane & 15, (lane >> 4) + 4 * ks)]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int mt = 0; mt < kShortMT; ++mt)
            acc[u][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt][ks], bf[u], acc[u][mt], 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (cb + 16 * u >= c1) continue;  // uniform
        const float nc = sN[buf][16 * u + (lane & 15)];
        const int col = cb + 16 * u + (lane & 15);
#pragma unroll
        for (int mt = 0; mt < kShortMT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = fmaf(-2.0f, acc[u][mt][r], nc);
            if (PASS == 1) {
              m2[mt][r] = med3_f32(m1[mt][r], m2[mt][r], v);
              m1[mt][r] = min_f32(m1[mt][r], v);
            } else {
              // row 16 mt + 4 g + r (g = lane >> 4), column cb + 16 u + (lane & 15)
              bits |= (v <= thr[mt][r] && col < p.n1) ? 1u << (8 * u + 4 * mt + r) : 0u;
            }
          }
      }
      // one word per lane and chunk, every chunk: no ballot, no branch, nothing to clear
      if (PASS == 2) p.mask[short_mask_word(p, b, rowbase >> 5, cb >> 6) + lane] = bits;
      if (ch + 1 < nchunk) sstore(buf ^ 1, g, gn);
      __syncthreads();
    }
  }
  if (PASS == 1) {
    // top-2 over the 16 lanes of a row (one DPP row): second = med3(a1, b1, min(a2, b2))
#pragma unroll
    for (int mt = 0; mt < kShortMT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float M1 = m1[mt][r], M2 = m2[mt][r];
#define VO_TOP2_STEP(CTRL)                                                                             \
  {                                                                                                    \
    const float b1 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(M1), CTRL, 0xF, 0xF, false)); \
    const float b2 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(M2), CTRL, 0xF, 0xF, false)); \
    M2 = med3_f32(M1, b1, fminf(M2, b2));                                                              \
    M1 = fminf(M1, b1);                                                                                \
  }
        VO_TOP2_STEP(0x121)
        VO_TOP2_STEP(0x122)
        VO_TOP2_STEP(0x124)
        VO_TOP2_STEP(0x128)
#undef VO_TOP2_STEP
        if ((lane & 15) == 0) {
          const int row = rowbase + 16 * mt + 4 * (lane >> 4) + r;
          p.part[((long)b * nsplit + split) * p.n0_pad + row] = make_float2(M1, M2);
        }
      }
  }
}

// ---- exact re-rank -----------------------------------------------------------------
__device__ __forceinline__ float sqrtf_rn2(float x) { return (float)sqrt((double)x); }

__device__ __forceinline__ uint64_t key64s(uint32_t d, uint32_t j) { return ((uint64_t)d << 32) | j; }

__device__ __forceinline__ void merge2s(uint64_t& a1, uint64_t& a2, uint64_t b1, uint64_t b2) {
  const uint64_t lo = a1 < b1 ? a1 : b1;
  const uint64_t hi = a1 < b1 ? b1 : a1;
  const uint64_t m = a2 < b2 ? a2 : b2;
  a1 = lo;
  a2 = hi < m ? hi : m;
}

// One workgroup per block of 16 query rows (the rows one set of candidate masks covers).
// The block's candidates (row, column) are pooled into one LDS list, so every lane of
// every wave has a candidate: thread c loads candidate c's train row (two halves of 32
// float4, all in flight) and runs the exact k-ordered fmaf chain against its query row
// (staged in LDS), keys (sqrtf(d2), j) go to LDS, and thread r merges row r's keys.  The
// candidate set is complete (masks have no capacity); a block with more than kPool
// candidates takes its rows one at a time through the same code.
// 384 candidates: the kernel's LDS (40 KB) then admits four workgroups per CU, the limit its
// 118 VGPRs set (at 512 it took 42 KB: three)
constexpr int kPool = 384;
constexpr int kQStr = 260;  // floats per staged query row
#ifndef VO_CHAIN_SPAN
#define VO_CHAIN_SPAN 128
#endif
constexpr int kChainSpan = VO_CHAIN_SPAN;  // train-row elements loaded before their chain

__device__ __forceinline__ float chain_regs(const float* x, const float* y, int dim) {
  // the oracle's distance: sum over k ascending of fmaf(x_k - y_k, x_k - y_k, acc); the
  // train row y (global) arrives kChainSpan elements at a time, every load in flight first
  float acc = 0.0f;
  for (int h = 0; h < dim; h += kChainSpan) {
    float4 yr[kChainSpan / 4];
#pragma unroll
    for (int t = 0; t < kChainSpan / 4; ++t)
      yr[t] = h + 4 * t < dim ? *reinterpret_cast<const float4*>(y + h + 4 * t) : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int t = 0; t < kChainSpan / 4; ++t) {
      if (h + 4 * t >= dim) break;
      const float4 xv = *reinterpret_cast<const float4*>(x + h + 4 * t);
      float d = xv.x - yr[t].x;
      acc = fmaf(d, d, acc);
      d = xv.y - yr[t].y;
      acc = fmaf(d, d, acc);
      d = xv.z - yr[t].z;
      acc = fmaf(d, d, acc);
      d = xv.w - yr[t].w;
      acc = fmaf(d, d, acc);
    }
  }
  return acc;
}

// Exact chains of the wave's (up to) 64 candidates, candidate c0 + lane, with the train rows
// staged through LDS: a span of kRerankSpan elements of 16 rows per load instruction (4
// lanes x 16 bytes per row: 16 x 64 contiguous bytes, not 64 rows' scattered 16 bytes), every
// load of a span in flight, then each lane continues its own k-ordered fmaf chain from its
// row's staged span and its query row (LDS).  Rows are padded by 16 bytes so the per-lane row
// reads spread over the banks.  Returns lane's d2 (garbage for c0 + lane >= total).
constexpr int kRerankSpan = 16;                 // floats per span (4 float4 per row)
constexpr int kSpanF4 = kRerankSpan / 4, kSpanRows = 64 / kSpanF4;  // per load instruction
// Staged rows of kRerankSpan floats (4 16-byte slots), slot s of row r stored at s ^ ((r >> 2) & 3):
// conflict-free on gfx950 both for the staging ds_write_b128 (8 x 8 contiguous lanes, four per
// row) and for each lane reading its own row (ds_read_b128 16-lane groups {0-3,12-15,20-27},
// ...); the former 16-byte row padding was 2-way on every staging store
constexpr int kRerankRowStr = kRerankSpan;
static_assert(kRerankSpan == 16, "the slot swizzle assumes 4 slots per staged row");
__device__ __forceinline__ int rr_slot(int row, int slot) { return slot ^ ((row >> 2) & 3); }
__device__ __forceinline__ float chain_staged(const float* __restrict__ B, const float* sq, const int* slist,
                                              const int* scol, float* sbuf, int c0, int total, int dim) {
  const int lane = threadIdx.x & 63;
  const int c = min(c0 + lane, total - 1);
  const float* x = sq + slist[c] * kQStr;
  // loader role: instruction t stages rows kSpanRows t + lane / kSpanF4, float4 lane % kSpanF4
  int jrow[kSpanF4];
#pragma unroll
  for (int t = 0; t < kSpanF4; ++t) jrow[t] = scol[min(c0 + kSpanRows * t + lane / kSpanF4, total - 1)];
  // three spans in flight: span h's loads were issued two spans earlier
  auto fetch = [&](int h, float4 (&v)[kSpanF4]) __attribute__((always_inline)) {
    const int k4 = h / 4 + lane % kSpanF4;
    if (h + kRerankSpan <= dim) {  // a whole span (uniform): unconditional loads
#pragma unroll
      for (int t = 0; t < kSpanF4; ++t)
        v[t] = reinterpret_cast<const float4*>(B + (long)jrow[t] * dim)[k4];
      return;
    }
    const bool in = 4 * k4 < dim;
#pragma unroll
    for (int t = 0; t < kSpanF4; ++t)
      v[t] = in ? reinterpret_cast<const float4*>(B + (long)jrow[t] * dim)[k4] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto consume = [&](int h, const float4 (&v)[kSpanF4], float& acc) __attribute__((always_inline)) {
    __builtin_amdgcn_wave_barrier();  // every lane's reads of the previous span are done (in-order LDS)
#pragma unroll
    for (int t = 0; t < kSpanF4; ++t) {
      const int row = kSpanRows * t + lane / kSpanF4;
      *reinterpret_cast<float4*>(sbuf + row * kRerankRowStr + 4 * rr_slot(row, lane % kSpanF4)) = v[t];
    }
    __builtin_amdgcn_wave_barrier();
    const float* y = sbuf + lane * kRerankRowStr;
    auto step4 = [&](const float4& xv, const float4& yv) __attribute__((always_inline)) {
      float d = xv.x - yv.x;
      acc = fmaf(d, d, acc);
      d = xv.y - yv.y;
      acc = fmaf(d, d, acc);
      d = xv.z - yv.z;
      acc = fmaf(d, d, acc);
      d = xv.w - yv.w;
      acc = fmaf(d, d, acc);
    };
    if (h + kRerankSpan <= dim) {  // a whole span (uniform): all eight LDS reads in flight at once
      float4 xv[kSpanF4], yv[kSpanF4];
#pragma unroll
      for (int q = 0; q < kSpanF4; ++q) {
        xv[q] = *reinterpret_cast<const float4*>(x + h + 4 * q);
        yv[q] = *reinterpret_cast<const float4*>(y + 4 * rr_slot(lane, q));
      }
#pragma unroll
      for (int q = 0; q < kSpanF4; ++q) step4(xv[q], yv[q]);
    } else {
      const int n = dim - h;
      for (int k = 0; k < n; k += 4)
        step4(*reinterpret_cast<const float4*>(x + h + k), *reinterpret_cast<const float4*>(y + 4 * rr_slot(lane, k / 4)));
    }
  };
  float acc = 0.0f;
  float4 v0[kSpanF4], v1[kSpanF4], v2[kSpanF4];
  fetch(0, v0);
  if (kRerankSpan < dim) fetch(kRerankSpan, v1);
  for (int h = 0; h < dim; h += 3 * kRerankSpan) {
    if (h + 2 * kRerankSpan < dim) fetch(h + 2 * kRerankSpan, v2);
    consume(h, v0, acc);
    if (h + kRerankSpan >= dim) break;
    if (h + 3 * kRerankSpan < dim) fetch(h + 3 * kRerankSpan, v0);
    consume(h + kRerankSpan, v1, acc);
    if (h + 2 * kRerankSpan >= dim) break;
    if (h + 4 * kRerankSpan < dim) fetch(h + 4 * kRerankSpan, v1);
    consume(h + 2 * kRerankSpan, v2, acc);
  }
  return acc;
}

__device__ __forceinline__ const float* B_row(const ShortArgs& p, int b, int j) {
  return p.db + b * p.b_bstride + (long)j * p.dim;
}

__device__ __forceinline__ float chain_scalar(const float* x, const float* y, int dim) {
  float acc = 0.0f;
  for (int k = 0; k < dim; ++k) {
    const float d = x[k] - y[k];
    acc = fmaf(d, d, acc);
  }
  return acc;
}

// Grid: 8 * ceil(nR * batch / 8) workgroups, remapped XCD-major (workgroup L runs on XCD L mod
// 8 by round-robin dispatch): XCD x takes the contiguous items [x per, (x + 1) per) of the
// (pair, 16-row block) list, so the blocks of one frame pair share one L2 and its train rows
// (2 MB at 2048 x 256) are fetched from the fabric once per XCD instead of by every XCD.
// Under the float hint no exact sweep is launched: a call with non-finite values (fpack's
// flag) is answered here by an exact scan of every train row instead (rare; see below).
// Waves that run candidate chains (each stages train rows in its own 4 KB of LDS) and the
// workgroups per CU the kernel is compiled for (tuning builds: EXTRA=-DVO_RERANK_CW=n /
// -DVO_RERANK_WGS=n)
#ifndef VO_RERANK_CW
#define VO_RERANK_CW 4
#endif
#ifndef VO_RERANK_WGS
#define VO_RERANK_WGS 4
#endif
constexpr int kChainWaves = VO_RERANK_CW;
static_assert(kChainWaves >= 1 && kChainWaves <= 4, "chain waves of a 256-thread workgroup");
__global__ __launch_bounds__(256, VO_RERANK_WGS) void frerank_kernel(ShortArgs p, int v4, int nR, int nitems) {
  const bool exact_scan = p.forced && p.flag[1] == p.gen;  // uniform
  if (!exact_scan && !short_active(p)) return;
  const int per = (nitems + 7) / 8, L = blockIdx.x, item = (L & 7) * per + (L >> 3);
  if (item >= nitems) return;
  const int b = item / nR, R = item - b * nR, tid = threadIdx.x;
  if (R == 0 && tid == 0) p.bmax[kBmaxStride * b] = 0u;  // fsweep<2> is done with it
  __shared__ __attribute__((aligned(16))) float sq[16 * kQStr];
  __shared__ __attribute__((aligned(8))) int slist[kPool];  // row_local << 16 | column tile bit position (see below)
  __shared__ int scol[kPool];
  __shared__ uint64_t skey[kPool];
  __shared__ int sscan[256];
  __shared__ __attribute__((aligned(16))) float sbuf[kChainWaves][64 * kRerankRowStr];  // per-wave row staging
  const int row0 = 16 * R;
  if (v4) {  // the block's 16 query rows as float4s, every load in flight before the stores
    const int nv = p.dim / 4, nall = 16 * nv;  // dim <= 256: at most 4 per thread
    float4 tq[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, rl = e / max(nv, 1), k4 = e - rl * nv;
      tq[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < nall && row0 + rl < p.n0)
        tq[u] = reinterpret_cast<const float4*>(p.da + b * p.a_bstride + (long)(row0 + rl) * p.dim)[k4];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, rl = e / max(nv, 1), k4 = e - rl * nv;
      if (e < nall) *reinterpret_cast<float4*>(sq + rl * kQStr + 4 * k4) = tq[u];
    }
  } else {
    for (int e = tid; e < 16 * p.dim; e += 256) {
      const int rl = e / p.dim, k = e - rl * p.dim;
      sq[rl * kQStr + k] = row0 + rl < p.n0 ? p.da[b * p.a_bstride + (long)(row0 + rl) * p.dim + k] : 0.0f;
    }
  }
  uint64_t k1 = ~0ull, k2 = ~0ull;
  if (exact_scan) {
    // the exact fp32 sweep's answer (match.hip sweep_f32 + merge_kernel): the two smallest
    // (sqrtf(d2), j) keys over the train rows whose k-ordered fmaf chain d2 is finite (a NaN or
    // +inf d2 never enters a top-2 there).  Thread (r, part) scans rows part, part + 16, ...
    // for query row r; the 16 partial top-2s of a row merge as below.
    __syncthreads();
    const int r = tid & 15, part = tid >> 4;
    uint64_t a1 = ~0ull, a2 = ~0ull;
    if (row0 + r < p.n0)
      for (int j = part; j < p.n1; j += 16) {
        const float d = chain_scalar(sq + r * kQStr, B_row(p, b, j), p.dim);
        if (d < __builtin_huge_valf()) merge2s(a1, a2, key64s(__float_as_uint(sqrtf_rn2(d)), (uint32_t)j), ~0ull);
      }
    uint64_t* pt = reinterpret_cast<uint64_t*>(&sbuf[0][0]);  // the row staging is idle here
    static_assert(sizeof(sbuf) >= 512 * sizeof(uint64_t), "the partial top-2s fit the staging buffer");
    pt[tid] = a1;
    pt[256 + tid] = a2;
    __syncthreads();
    if (tid < 16)
      for (int q = 0; q < 16; ++q) merge2s(k1, k2, pt[tid + 16 * q], pt[256 + tid + 16 * q]);
  } else {
  // the block's 16 rows are M tile mt = R & 1 of wave row group R >> 1: in each of its
  // nch x 64 words, bits 8 u + 4 mt + r
  const int nch = (p.n1_pad + 63) / 64, nw = 64 * nch;
  const uint32_t* mblk = p.mask + short_mask_word(p, b, R >> 1, 0);
  const uint32_t msel = 0x0F0F0F0Fu << (4 * (R & 1));
  const float* B = p.db + b * p.b_bstride;
  // this thread's words (e = tid + 256 i), kept for the list pass: up to 8 (n1 <= 2048);
  // wider train sets re-read the rest
  constexpr int kWordRegs = 8;
  uint32_t wr[kWordRegs];
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < kWordRegs; ++i) {
    const int e = tid + 256 * i;
    wr[i] = e < nw ? mblk[e] & msel : 0u;
    cnt += __popc(wr[i]);
  }
  for (int e = tid + 256 * kWordRegs; e < nw; e += 256) cnt += __popc(mblk[e] & msel);
  // workgroup exclusive prefix of the counts: inclusive scan inside each wave (fixed shuffle
  // pattern), the four wave totals through LDS, one barrier
  const int lane = tid & 63, wv = tid >> 6;
  int incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int v = __shfl_up(incl, d, 64);
    incl += lane >= d ? v : 0;
  }
  if (lane == 63) sscan[wv] = incl;
  __syncthreads();
  int wbase = 0, total = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    wbase += w < wv ? sscan[w] : 0;
    total += sscan[w];
  }
  int pos = wbase + incl - cnt;
  const bool pooled = total <= kPool;
  if (pooled) {
    auto emit = [&](int e, uint32_t m) {
      const int ch = e >> 6, ln = e & 63;
      for (; m; m &= m - 1) {
        const int bit = __builtin_ctz(m);
        slist[pos] = 4 * (ln >> 4) + (bit & 3);  // row_local = 4 g + r
        scol[pos] = 64 * ch + 16 * (bit >> 3) + (ln & 15);
        ++pos;
      }
    };
#pragma unroll
    for (int i = 0; i < kWordRegs; ++i) emit(tid + 256 * i, wr[i]);
    for (int e = tid + 256 * kWordRegs; e < nw; e += 256) emit(e, mblk[e] & msel);
  }
  __syncthreads();
  if (pooled) {
    if (v4) {
      // wave w takes candidates 64 (w + 4 q) + lane (the loop bound is wave-uniform)
      const int wv = tid >> 6;
      for (int c0 = 64 * wv; wv < kChainWaves && c0 < total; c0 += 64 * kChainWaves) {
        const float d = chain_staged(B, sq, slist, scol, sbuf[wv], c0, total, p.dim);
        const int c = c0 + (tid & 63);
        if (c < total) skey[c] = key64s(__float_as_uint(sqrtf_rn2(d)), (uint32_t)scol[c]);
      }
    } else {
      for (int c = tid; c < total; c += 256) {
        const int rl = slist[c], j = scol[c];
        const float d = chain_scalar(sq + rl * kQStr, B + (long)j * p.dim, p.dim);
        skey[c] = key64s(__float_as_uint(sqrtf_rn2(d)), (uint32_t)j);
      }
    }
    __syncthreads();
    // row r's keys merged by 16 threads (r + 16 part, every 16th pooled candidate), then
    // their 16 partial top-2s by thread r (keys are unique: the order does not matter)
    {
      const int r = tid & 15, part = tid >> 4;
      uint64_t a1 = ~0ull, a2 = ~0ull;
      for (int c = part; c < total; c += 16)
        if (slist[c] == r) merge2s(a1, a2, skey[c], ~0ull);
      uint64_t* pt = reinterpret_cast<uint64_t*>(&sbuf[0][0]);  // the row staging is idle now
      pt[tid] = a1;
      pt[256 + tid] = a2;
      __syncthreads();
      if (tid < 16)
        for (int q = 0; q < 16; ++q) merge2s(k1, k2, pt[tid + 16 * q], pt[256 + tid + 16 * q]);
    }
  } else if (tid < 16) {  // rare: thread rl walks row rl's candidates itself
    const int g = tid >> 2, r = tid & 3;
    for (int e = 16 * g; e < nw; e += (e & 15) == 15 ? 49 : 1) {  // the 16 lanes of group g of every chunk
      const int ch = e >> 6, ln = e & 63;
      for (int u = 0; u < 4; ++u)
        if ((mblk[e] >> (8 * u + 4 * (R & 1) + r)) & 1u) {
          const int j = 64 * ch + 16 * u + (ln & 15);
          const float d = chain_scalar(sq + tid * kQStr, B + (long)j * p.dim, p.dim);
          merge2s(k1, k2, key64s(__float_as_uint(sqrtf_rn2(d)), (uint32_t)j), ~0ull);
        }
    }
  }
  }
  const int row = row0 + tid;
  if (tid >= 16 || row >= p.n0) return;
  const float s1 = k1 == ~0ull ? __builtin_huge_valf() : __uint_as_float((uint32_t)(k1 >> 32));
  const float s2 = k2 == ~0ull ? __builtin_huge_valf() : __uint_as_float((uint32_t)(k2 >> 32));
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

}  // namespace

#ifndef VO_FSWEEP_WGS_PER_CU
#define VO_FSWEEP_WGS_PER_CU 2  // tuning builds: EXTRA=-DVO_FSWEEP_WGS_PER_CU=n
#endif

void short_launch(vo_ctx* ctx, ShortArgs& a, int batch) {
  hipStream_t st = ctx->stream;
  {
    // the sweeps' own column split: a workgroup loads 64 KB of A fragments (128 rows x 256
    // bf16) before its first MFMA, so it should sweep as many columns as the grid allows --
    // about VO_FSWEEP_WGS_PER_CU workgroups per CU, one round (splits are multiples of 64
    // columns, the staging chunk; the split never changes a result)
    const int64_t row_blocks = (int64_t)(a.n0_pad / kShortRowsPerWG) * batch;
    const int want = (int)std::max<int64_t>(1, ceil_div((int64_t)VO_FSWEEP_WGS_PER_CU * ctx->num_cus, row_blocks));
    const int w = std::max(64, ((a.n1_pad + want - 1) / want + 63) / 64 * 64);
    a.split_w = w;
    a.nsplit = (a.n1_pad + w - 1) / w;
  }
  const int a_wgs = (int)ceil_div((int64_t)a.n0_pad * 16, 256);
  const int b_wgs = (int)ceil_div((int64_t)a.n1_pad * 16, 256);
  ctx->prof.begin(st, kKMatchPack);
  const int v4 = a.dim % 4 == 0 && (uintptr_t)a.da % 16 == 0 && (uintptr_t)a.db % 16 == 0;
  hipLaunchKernelGGL(fpack_kernel, dim3(a_wgs + b_wgs, batch), dim3(256), 0, st, a, a_wgs, v4);
  ctx->prof.end(st);
  const dim3 grid(a.n0_pad / kShortRowsPerWG, a.nsplit, batch);
  ctx->prof.begin(st, kKMatchF32);
  switch (a.Dp / 32) {
#define VO_SWEEPS(KS)                                                                \
  case KS:                                                                           \
    hipLaunchKernelGGL((fsweep_kernel<1, KS>), grid, dim3(256), 0, st, a);           \
    hipLaunchKernelGGL((fsweep_kernel<2, KS>), grid, dim3(256), 0, st, a);           \
    break;
    VO_SWEEPS(1)
    VO_SWEEPS(2)
    VO_SWEEPS(3)
    VO_SWEEPS(4)
    VO_SWEEPS(5)
    VO_SWEEPS(6)
    VO_SWEEPS(7)
    VO_SWEEPS(8)
#undef VO_SWEEPS
  }
  ctx->prof.end(st);
  ctx->prof.begin(st, kKMatchRerank);
  const int nR = a.n0_pad / 16, nitems = nR * batch;
  hipLaunchKernelGGL(frerank_kernel, dim3(8 * ((nitems + 7) / 8)), dim3(256), 0, st, a, v4, nR, nitems);
  ctx->prof.end(st);
}

}  // namespace vo
