// SIFT orientation assignment, keypoint filtering and descriptors on gfx950.
//
// The second half of cv2.SIFT_create(nfeatures, contrastThreshold, edgeThreshold, sigma)
// .detectAndCompute(gray, None) (reference src/modules/frontend.py:27-32,55; OpenCV 4.12
// sift.simd.hpp calcOrientationHist / calcSIFTDescriptor, sift.dispatch.cpp
// detectAndCompute, keypoint.cpp removeDuplicatedSorted / retainBest), restated in
// oracle/sift_ref.py.  FMA contraction is off and every histogram bin is summed in
// OpenCV's sample order (row-major over the window), so orientations and descriptors are
// bitwise the oracle's.
//
// After sift_run (sift.hip) has left the refined extrema in a candidate list:
//   sift_orient_kernel    one 64-lane workgroup per extremum: the window's samples are
//                         evaluated 64 at a time into LDS (bin, weighted magnitude), then
//                         lane b < 36 sums the samples of bin b in sample order; [1 4 6 4 1]
//                         smoothing, peaks >= 0.8 max appended per image with the
//                         parabolic angle
//   sift_keys_kernel      64-bit sort keys (image | x bits | y bits, 10 + 27 + 27 bits)
//   rocprim radix sort of the whole batch at once: image, then x asc, then y asc
//   sift_select_kernel    one workgroup per image: runs of equal (x, y) ordered by (size
//                         desc, angle asc, response desc, octave desc), duplicates in
//                         (x, y, size, angle) dropped (removeDuplicatedSorted), the
//                         nfeatures-th largest response found by a 4-pass radix select
//                         (retainBest keeps every response >= it), ordered compaction
//   sift_desc_kernel      one 256-thread workgroup per kept keypoint: the square window's
//                         positions are classified by the cheap geometry test and the valid
//                         ones compacted in order (about half lie outside the rotated
//                         square); then, 256 valid samples at a time, each thread evaluates one sample
//                         (gradient, fastAtan2, magnitude, exp32f, trilinear shares) and
//                         appends it to the stable LDS lists of the (up to 4) interior
//                         cells it votes into as (o0, share to o0, share to o0 + 1) (one
//                         ballot per cell and wave); then wave w owns descriptor cell row
//                         w + 1, lanes 0..35 its (column, orientation) bins, and each lane
//                         walks its cell's list in window order adding its share; finally the circular
//                         orientation bins are folded, clipped at 0.2 of the norm,
//                         renormalised to 512 and rounded.
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "sift_math.h"
#include "vo_ctx.h"

#pragma clang fp contract(off)

namespace vo {
namespace {

using namespace siftm;

constexpr int kMaxOct = 16;
constexpr int kOriBins = 36;
constexpr int kOriChunk = 1024;
constexpr int kOriPerLane = kOriChunk / 64;  // chunk samples per lane of the one-wave workgroup
constexpr int kD = 4, kN = 8, kDesc = kD * kD * kN;
constexpr int kCountStride = 64;                // ints between per-image append counters (own 256-byte line)
constexpr int kOkpFloats = 8;                   // x, y, size, angle, response (doubled-image units), octave word
constexpr float kFltEps = 1.1920928955078125e-07f;

struct Octaves {
  int oh[kMaxOct], ow[kMaxOct], op[kMaxOct];
  long off[kMaxOct];  // floats from the image's G base to the octave's level 0
  long g_img;         // floats per image
  int n_layers;
};

__device__ __forceinline__ const float* level_ptr(const float* G, const Octaves& O, int b, int o, int layer) {
  return G + (long)b * O.g_img + O.off[o] + (long)layer * O.oh[o] * O.op[o];
}

// Inclusive prefix sum over the 64 lanes of a wave in DPP (no LDS round trips): row_shr
// 1/2/4/8 inside each 16-lane row, then row_bcast:15 and row_bcast:31 across rows (GFX9).
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// ---- orientation -------------------------------------------------------------------
struct OriArgs {
  const float* G;
  Octaves O;
  const float* cand_f;        // sift_run records (x, y, size, response, xi) in doubled-image units
  const int32_t* cand_i;      // (image, octave word, cand level, level, row, col, cand row, cand col)
  const int32_t* cand_count;
  int cand_cap, cap_img;
  float* okp;                 // (batch, cap_img, 8)
  int32_t* img_count;         // (batch) at stride kCountStride
  ExpTab tab;
};

// resident one-wave workgroups per CU; the loop is persistent, so the grid must not exceed
// what fits (a second, late half of the grid would double the wall time)
#ifndef VO_ORI_WG_PER_CU
#define VO_ORI_WG_PER_CU 24
#endif
constexpr int kOriWgPerCu = VO_ORI_WG_PER_CU;

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kOriWgPerCu / 4)))
void sift_orient_kernel(OriArgs A) {
  __shared__ float s_val[kOriChunk];  // the chunk's terms grouped by bin, window order inside a bin
  __shared__ int s_run[kOriBins], s_base[kOriBins];
  __shared__ float s_th[kOriBins + 4];
  __shared__ float s_h[kOriBins];
  const int lane = threadIdx.x;
  // an extrema list overflowed (sift_refine_kernel's flag bit): records past the flag were not
  // written, so nothing is read; the selection kernel reports the overflow
  const int cc = *A.cand_count;
  const int ncand = (cc & (1 << 30)) ? 0 : min(cc, A.cand_cap);
  for (int ci = blockIdx.x; ci < ncand; ci += gridDim.x) {
    const float* F = A.cand_f + (long)ci * 8;
    const int32_t* Q = A.cand_i + (long)ci * 8;
    const int b = Q[0], word = Q[1], layer = Q[3], pr = Q[4], pc = Q[5];
    const int o = word & 255;
    const float size2 = F[2];
    const float scl = size2 * 0.5f / (float)(1 << o);
    const int radius = (int)rintf(4.5f * scl);
    const float sigma = 1.5f * scl;
    const float expf_scale = __fdiv_rn(-1.f, 2.f * sigma * sigma);
    const float* img = level_ptr(A.G, A.O, b, o, layer);
    const int rows = A.O.oh[o], cols = A.O.ow[o], pitch = A.O.op[o];
    const int side = 2 * radius + 1, len = side * side;
    float acc = 0.0f;
    for (int k0 = 0; k0 < len; k0 += kOriChunk) {
      const int kn = min(kOriChunk, len - k0);
      // samples t = lane + 64 u of the chunk (window order = (u, lane)); each is ranked
      // inside its bin by a stable counting sort: peers (same bin) from six bit ballots, the
      // rank among earlier peers by mbcnt, the bin's running count in s_run
      if (lane < kOriBins) s_run[lane] = 0;
      float vv[kOriPerLane];
      int bb[kOriPerLane], rk[kOriPerLane];
#pragma unroll
      for (int u = 0; u < kOriPerLane; ++u) {
        const int t = lane + 64 * u;
        const int k = k0 + t, i = k / side - radius, j = k % side - radius;
        const int y = pr + i, x = pc + j;
        int bin = -1;
        float v = 0.0f;
        if (t < kn && y > 0 && y < rows - 1 && x > 0 && x < cols - 1) {
          const float dx = img[(long)y * pitch + x + 1] - img[(long)y * pitch + x - 1];
          const float dy = img[(long)(y - 1) * pitch + x] - img[(long)(y + 1) * pitch + x];
          const float w = exp32f((float)(i * i + j * j) * expf_scale, A.tab.v);
          const float ori = fast_atan2_deg(dy, dx);
          const float mag = sqrt_rn(dx * dx + dy * dy);
          bin = (int)rintf(((float)kOriBins / 360.f) * ori);
          if (bin >= kOriBins) bin -= kOriBins;
          if (bin < 0) bin += kOriBins;
          v = w * mag;
        }
        const int key = bin < 0 ? 63 : bin;  // 63: no bin (outside the image or the chunk)
        uint64_t peers = ~0ull;
#pragma unroll
        for (int bit = 0; bit < 6; ++bit) {
          const uint64_t m = __ballot((key >> bit) & 1);
          peers &= ((key >> bit) & 1) ? m : ~m;
        }
        const int r = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
        rk[u] = bin >= 0 ? s_run[bin] + r : 0;
        // the last peer carries the group's count (one wave: LDS keeps its accesses in order)
        if (bin >= 0 && (peers >> lane) == 1ull) s_run[bin] = rk[u] + 1;
        bb[u] = bin;
        vv[u] = v;
      }
      // bin b's list starts at the sum of the earlier bins' counts
      const int cnt = lane < kOriBins ? s_run[lane] : 0, incl = wave_incl_scan(cnt);
      if (lane < kOriBins) s_base[lane] = incl - cnt;
#pragma unroll
      for (int u = 0; u < kOriPerLane; ++u)
        if (bb[u] >= 0) s_val[s_base[bb[u]] + rk[u]] = vv[u];
      __syncthreads();
      // lane b sums bin b's samples in window order
      if (lane < kOriBins) {
        const float* P = s_val + (incl - cnt);
        int t = 0;
        for (; t + 4 <= cnt; t += 4) {
          float e[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) e[u] = P[t + u];
#pragma unroll
          for (int u = 0; u < 4; ++u) acc = acc + e[u];
        }
        for (; t < cnt; ++t) acc = acc + P[t];
      }
      __syncthreads();
    }
    if (lane < kOriBins) s_th[lane + 2] = acc;
    __syncthreads();
    if (lane < 2) {
      s_th[lane] = s_th[kOriBins + lane];             // temphist[-2], [-1]
      s_th[kOriBins + 2 + lane] = s_th[2 + lane];     // temphist[n], [n+1]
    }
    __syncthreads();
    float h = 0.0f;
    if (lane < kOriBins) {
      const float* T = s_th + 2 + lane;
      h = (T[-2] + T[2]) * (1.f / 16.f) + (T[-1] + T[1]) * (4.f / 16.f) + T[0] * (6.f / 16.f);
      s_h[lane] = h;
    }
    float m = lane < kOriBins ? h : -1.0f;
    for (int s = 32; s >= 1; s >>= 1) m = fmaxf(m, __shfl_xor(m, s));
    __syncthreads();
    if (lane < kOriBins) {
      const float mag_thr = m * 0.8f;
      const int l = lane > 0 ? lane - 1 : kOriBins - 1, r2 = lane < kOriBins - 1 ? lane + 1 : 0;
      const float hl = s_h[l], hr = s_h[r2];
      if (h > hl && h > hr && h >= mag_thr) {
        float bin = (float)lane + __fdiv_rn(0.5f * (hl - hr), (hl - 2.0f * h) + hr);
        bin = bin < 0 ? (float)kOriBins + bin : (bin >= kOriBins ? bin - (float)kOriBins : bin);
        float angle = 360.f - (360.f / kOriBins) * bin;
        if (fabsf(angle - 360.f) < kFltEps) angle = 0.f;
        const int slot = atomicAdd(A.img_count + b * kCountStride, 1);
        if (slot < A.cap_img) {
          float* R = A.okp + ((long)b * A.cap_img + slot) * kOkpFloats;
          R[0] = F[0];
          R[1] = F[1];
          R[2] = size2;
          R[3] = angle;
          R[4] = F[3];
          R[5] = __int_as_float(word);
          R[6] = 0.0f;
          R[7] = 0.0f;
        }
      }
    }
    __syncthreads();
  }
}

// ---- sort keys, segments -------------------------------------------------------------
__global__ __launch_bounds__(256) void sift_keys_kernel(const float* __restrict__ okp, const int32_t* __restrict__ img_count,
                                                        int cap_img, int batch, uint64_t* __restrict__ keys,
                                                        uint32_t* __restrict__ vals) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  const int b = (int)(g / cap_img), s = (int)(g - (long)b * cap_img);
  if (b >= batch) return;
  vals[g] = (uint32_t)g;
  if (s >= min(img_count[b * kCountStride], cap_img)) {
    keys[g] = ~0ull;  // unused slot: after every image
    return;
  }
  const float* R = okp + g * kOkpFloats;
  // x, y in [4.5, 32768) doubled-image pixels: their float bits minus those of 2.0 fit in
  // 27 bits and order like the values
  const uint64_t xb = __float_as_uint(R[0]) - 0x40000000u, yb = __float_as_uint(R[1]) - 0x40000000u;
  keys[g] = ((uint64_t)b << 54) | (xb << 27) | yb;
}

// ---- removeDuplicatedSorted + retainBest + ordered compaction ------------------------
struct SelArgs {
  const float* okp;
  const uint64_t* keys;  // sorted per image
  uint32_t* vals;        // sorted per image (ties re-ordered in place)
  const int32_t* img_count;
  const int32_t* cand_count;
  int cand_cap, cap_img, nfeatures;
  uint32_t* sel;         // (batch, cap_img) record indices in output order
  int32_t* sel_count;    // (batch): kept, or -(the capacity needed) when one overflowed
  uint32_t* resp;        // (batch, cap_img) scratch: response bits in sorted order
  int32_t* work;         // the descriptor kernel's keypoint counter (zeroed here)
};

__device__ __forceinline__ bool kp_less2(const float* a, const float* b) {
  // KeyPoint12_LessThan after equal (x, y): size desc, angle asc, response desc, octave desc
  if (a[2] != b[2]) return a[2] > b[2];
  if (a[3] != b[3]) return a[3] < b[3];
  if (a[4] != b[4]) return a[4] > b[4];
  return __float_as_int(a[5]) > __float_as_int(b[5]);
}

constexpr int kSelThreads = 1024;
constexpr int kSelUnroll = 4;  // records per thread and round of the select passes
constexpr int kRunMax = 8;     // equal-(x, y) runs sorted in registers (longer: insertion sort)
constexpr int kLongQueue = 2048;  // runs of >= 3 records sorted after the pass (more: inline)
constexpr int kMaxCapImg = 131072;  // keep[] in LDS: 128 KiB of the select kernel's 160

// A run of >= 3 records with equal (x, y) starting at i: ordered by kp_less2 (the stable
// insertion sort's order), its duplicates (equal size and angle after the order) flagged in
// keep, its response bits copied to R; returns the records kept.  Up to kRunMax records are
// loaded in three batches (keys, indices, records) and sorted in registers by odd-even
// transposition (adjacent swaps only when strictly less: stable); longer runs (rare) take an
// insertion sort in place.
__device__ __forceinline__ int sort_run(const SelArgs& A, const uint64_t* K, uint32_t* V, uint32_t* R,
                                                  uint8_t* keep, int i, int n) {
  const uint64_t key = K[i];
  uint64_t kr[kRunMax];
#pragma unroll
  for (int u = 1; u < kRunMax; ++u) kr[u] = K[min(i + u, n - 1)];
  int len = 1;
#pragma unroll
  for (int u = 1; u < kRunMax; ++u) len += (len == u && i + u < n && kr[u] == key) ? 1 : 0;
  const bool fits = len < kRunMax || i + kRunMax >= n || K[i + kRunMax] != key;
  if (fits) {
    uint32_t vr[kRunMax];
    float f[kRunMax][6];
#pragma unroll
    for (int u = 0; u < kRunMax; ++u) vr[u] = u < len ? V[i + u] : 0u;
#pragma unroll
    for (int u = 0; u < kRunMax; ++u) {
      if (u >= len) continue;
      const float4* r = reinterpret_cast<const float4*>(A.okp + (long)vr[u] * kOkpFloats);
      const float4 x0 = r[0], x1 = r[1];
      f[u][0] = x0.x;
      f[u][1] = x0.y;
      f[u][2] = x0.z;
      f[u][3] = x0.w;
      f[u][4] = x1.x;
      f[u][5] = x1.y;
    }
#pragma unroll
    for (int round = 0; round < kRunMax; ++round) {
#pragma unroll
      for (int u = round & 1; u + 1 < kRunMax; u += 2) {
        if (u + 1 < len && kp_less2(f[u + 1], f[u])) {
#pragma unroll
          for (int c = 0; c < 6; ++c) {
            const float t = f[u][c];
            f[u][c] = f[u + 1][c];
            f[u + 1][c] = t;
          }
          const uint32_t t = vr[u];
          vr[u] = vr[u + 1];
          vr[u + 1] = t;
        }
      }
    }
    int kept = 0;
#pragma unroll
    for (int u = 0; u < kRunMax; ++u) {
      if (u >= len) continue;
      const bool k = u == 0 || !(f[u][2] == f[u - 1][2] && f[u][3] == f[u - 1][3]);
      V[i + u] = vr[u];
      keep[i + u] = k;
      R[i + u] = __float_as_uint(f[u][4]);
      kept += k;
    }
    return kept;
  }
  int e = i + 1;
  while (e < n && K[e] == key) ++e;
  for (int p = i + 1; p < e; ++p) {
    const uint32_t v = V[p];
    const float* rv = A.okp + (long)v * kOkpFloats;
    int q = p - 1;
    while (q >= i && kp_less2(rv, A.okp + (long)V[q] * kOkpFloats)) {
      V[q + 1] = V[q];
      --q;
    }
    V[q + 1] = v;
  }
  int kept = 0;
  for (int p = i; p < e; ++p) {
    const float* c = A.okp + (long)V[p] * kOkpFloats;
    const bool k = p == i || !(c[2] == A.okp[(long)V[p - 1] * kOkpFloats + 2] &&
                               c[3] == A.okp[(long)V[p - 1] * kOkpFloats + 3]);
    keep[p] = k;
    R[p] = __float_as_uint(c[4]);
    kept += k;
  }
  return kept;
}


__global__ __launch_bounds__(kSelThreads) void sift_select_kernel(SelArgs A) {
  __shared__ uint8_t keep[kMaxCapImg];
  __shared__ int s_hist[256];
  __shared__ int s_scan[kSelThreads];
  __shared__ int s_total;
  __shared__ uint32_t s_prefix, s_rank;
  __shared__ int s_nlong, s_long[kLongQueue];  // starts of runs of >= 3 records
  const int b = blockIdx.x, tid = threadIdx.x;
  const long base = (long)b * A.cap_img;
  const int cnt = A.img_count[b * kCountStride];
  if (b == 0 && tid == 0) *A.work = 0;
  long sbase = 0;  // this image's first element in the batch-wide sorted order
  for (int q = 0; q < b; ++q) sbase += min(A.img_count[q * kCountStride], A.cap_img);
  if (*A.cand_count > A.cand_cap || cnt > A.cap_img) {
    // the counters kept counting past their capacities: report the per-image working
    // capacity they ask for, so the host retries at that size instead of growing step by
    // step.  With every candidate kept, cnt is exact; when candidates were dropped, cnt only
    // counts the oriented keypoints of the kept ones, so ask for two per candidate (a second
    // orientation peak is common, more are rare; a short guess costs one more pass).
    const long ncand = *A.cand_count;
    const long need = ncand > A.cand_cap ? max((long)cnt, 2 * ((ncand + gridDim.x - 1) / gridDim.x)) : (long)cnt;
    if (tid == 0) A.sel_count[b] = -(int)min(max(need, 1l), (long)INT32_MAX);
    return;
  }
  const int n = cnt;
  const uint64_t* K = A.keys + sbase;
  uint32_t* V = A.vals + sbase;
  // One pass over the sorted keys does removeDuplicatedSorted's work: runs of equal (x, y)
  // are put in comparator order (size desc, angle asc, response desc, octave desc) and, since
  // duplicates share (x, y), flagged inside their run; every record's response bits are copied
  // out in sorted order for the selection passes (read coalesced there).  A record that starts
  // no run is kept (its predecessor differs in x or y).  Almost every run is one point's two
  // orientation peaks: one compare-and-swap, its loads issued with the round's other records.
  // Longer runs are queued and sorted after the pass, one per thread.  Four records per thread
  // and round; the thread of a run's first record owns the run.
  uint32_t* R = A.resp + base;
  int local = 0;
  if (tid == 0) s_nlong = 0;
  __syncthreads();
  for (int i0 = tid; i0 < n; i0 += kSelUnroll * kSelThreads) {
    uint64_t kp[kSelUnroll], kc[kSelUnroll], kn[kSelUnroll], kn2[kSelUnroll];
#pragma unroll
    for (int j = 0; j < kSelUnroll; ++j) {
      const int i = min(i0 + j * kSelThreads, n - 1);
      kp[j] = K[max(i - 1, 0)];
      kc[j] = K[i];
      kn[j] = K[min(i + 1, n - 1)];
      kn2[j] = K[min(i + 2, n - 1)];
    }
    bool single[kSelUnroll], pair[kSelUnroll];
#pragma unroll
    for (int j = 0; j < kSelUnroll; ++j) {
      const int i = i0 + j * kSelThreads;
      const bool head = i < n && (i == 0 || kp[j] != kc[j]);  // first record of its (x, y)
      const bool start = head && i + 1 < n && kn[j] == kc[j];
      pair[j] = start && (i + 2 >= n || kn2[j] != kc[j]);
      single[j] = head && !start;
      if (start && !pair[j]) {
        const int q = atomicAdd(&s_nlong, 1);
        if (q < kLongQueue) s_long[q] = i;
      }
    }
    uint32_t va[kSelUnroll], vb[kSelUnroll];
#pragma unroll
    for (int j = 0; j < kSelUnroll; ++j) {
      const int i = min(i0 + j * kSelThreads, max(n - 2, 0));
      va[j] = single[j] || pair[j] ? V[min(i0 + j * kSelThreads, n - 1)] : 0u;
      vb[j] = pair[j] ? V[i + 1] : 0u;
    }
    float4 a0[kSelUnroll], a1[kSelUnroll], b0[kSelUnroll], b1[kSelUnroll];
    float rs[kSelUnroll];
#pragma unroll
    for (int j = 0; j < kSelUnroll; ++j) {
      rs[j] = 0.0f;
      if (single[j]) rs[j] = A.okp[(long)va[j] * kOkpFloats + 4];
      if (!pair[j]) continue;
      const float4* ra = reinterpret_cast<const float4*>(A.okp + (long)va[j] * kOkpFloats);
      const float4* rb = reinterpret_cast<const float4*>(A.okp + (long)vb[j] * kOkpFloats);
      a0[j] = ra[0];
      a1[j] = ra[1];
      b0[j] = rb[0];
      b1[j] = rb[1];
    }
#pragma unroll
    for (int j = 0; j < kSelUnroll; ++j) {
      const int i = i0 + j * kSelThreads;
      if (single[j]) {
        keep[i] = 1;
        R[i] = __float_as_uint(rs[j]);
        ++local;
      }
      if (!pair[j]) continue;
      const float fa[6] = {a0[j].x, a0[j].y, a0[j].z, a0[j].w, a1[j].x, a1[j].y};
      const float fb[6] = {b0[j].x, b0[j].y, b0[j].z, b0[j].w, b1[j].x, b1[j].y};
      const bool sw = kp_less2(fb, fa);  // the stable insertion sort of two records
      const float* f0 = sw ? fb : fa;
      const float* f1 = sw ? fa : fb;
      if (sw) {
        V[i] = vb[j];
        V[i + 1] = va[j];
      }
      const bool k1 = !(f1[2] == f0[2] && f1[3] == f0[3]);  // (x, y) equal within the run
      keep[i] = 1;
      keep[i + 1] = k1;
      R[i] = __float_as_uint(f0[4]);
      R[i + 1] = __float_as_uint(f1[4]);
      local += 1 + k1;
    }
  }
  __syncthreads();
  const int nlong = s_nlong;
  if (nlong <= kLongQueue) {
    for (int q = tid; q < nlong; q += kSelThreads) local += sort_run(A, K, V, R, keep, s_long[q], n);
  } else {  // more than the queue holds (not seen on real images): every start found again
    for (int i = tid; i < n; i += kSelThreads)
      if ((i == 0 || K[i - 1] != K[i]) && i + 2 < n && K[i + 1] == K[i] && K[i + 2] == K[i])
        local += sort_run(A, K, V, R, keep, i, n);
  }
  __threadfence_block();
  __syncthreads();
  if (tid == 0) s_total = 0;
  __syncthreads();
  atomicAdd(&s_total, local);
  __syncthreads();
  const int kept = s_total;
  if (A.nfeatures > 0 && kept > A.nfeatures) {
    // the nfeatures-th largest response among the kept: radix select, 8 bits per pass
    if (tid == 0) {
      s_prefix = 0;
      s_rank = (uint32_t)A.nfeatures;
    }
    uint32_t mask = 0;
    for (int pass = 3; pass >= 0; --pass) {
      if (tid < 256) s_hist[tid] = 0;
      __syncthreads();
      const uint32_t prefix = s_prefix;
      for (int i0 = tid; i0 < n; i0 += kSelUnroll * kSelThreads) {
        uint32_t bits[kSelUnroll];
#pragma unroll
        for (int j = 0; j < kSelUnroll; ++j) bits[j] = R[min(i0 + j * kSelThreads, n - 1)];
#pragma unroll
        for (int j = 0; j < kSelUnroll; ++j) {
          const int i = i0 + j * kSelThreads;
          if (i < n && keep[i] && (bits[j] & mask) == prefix) atomicAdd(&s_hist[(bits[j] >> (8 * pass)) & 255], 1);
        }
      }
      __syncthreads();
      // the digit: the largest d whose count from 255 down to d reaches the rank (0 when none
      // above 0 does); wave 0, lane L holding digits 255 - 4L .. 252 - 4L
      if (tid < 64) {
        const uint32_t rank = s_rank;
        uint32_t c4[4], lsum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          c4[q] = (uint32_t)s_hist[255 - 4 * tid - q];
          lsum += c4[q];
        }
        const uint32_t incl = (uint32_t)wave_incl_scan((int)lsum);
        const uint64_t reach = __ballot(incl >= rank);
        const int L = reach ? __ffsll((unsigned long long)reach) - 1 : 63;
        if (tid == L) {
          uint32_t cum = incl - lsum;
          int q = 0;
          while (q < 3 && cum + c4[q] < rank) cum += c4[q++];
          s_rank = rank - cum;
          s_prefix = prefix | ((uint32_t)(255 - 4 * L - q) << (8 * pass));
        }
      }
      mask |= 255u << (8 * pass);
      __syncthreads();
    }
    const uint32_t thr = s_prefix;
    for (int i0 = tid; i0 < n; i0 += kSelUnroll * kSelThreads) {
      uint32_t bits[kSelUnroll];
#pragma unroll
      for (int j = 0; j < kSelUnroll; ++j) bits[j] = R[min(i0 + j * kSelThreads, n - 1)];
#pragma unroll
      for (int j = 0; j < kSelUnroll; ++j) {
        const int i = i0 + j * kSelThreads;
        if (i < n && bits[j] < thr) keep[i] = 0;
      }
    }
    __syncthreads();
  }
  // ordered compaction: thread t owns [t * per, (t + 1) * per)
  const int per = (n + kSelThreads - 1) / kSelThreads;
  const int lo = min(tid * per, n), hi = min(lo + per, n);
  int c = 0;
  for (int i = lo; i < hi; ++i) c += keep[i];
  s_scan[tid] = c;
  __syncthreads();
  for (int off = 1; off < kSelThreads; off <<= 1) {
    const int v = tid >= off ? s_scan[tid - off] : 0;
    __syncthreads();
    s_scan[tid] += v;
    __syncthreads();
  }
  int pos = s_scan[tid] - c;
  for (int i = lo; i < hi; ++i)
    if (keep[i]) A.sel[base + pos++] = V[i];
  if (tid == kSelThreads - 1) A.sel_count[b] = s_scan[tid];
}

// ---- descriptors ---------------------------------------------------------------------
struct DescArgs {
  const float* G;
  Octaves O;
  const float* okp;
  const uint32_t* sel;
  const int32_t* sel_count;
  int batch, cap_img;
  vo_sift_keypoint* kp_out;   // (batch, cap_img)
  float* desc_out;            // (batch, cap_img, 128)
  int32_t* count_out;         // (batch)
  int32_t* work;              // keypoints taken past the first gridDim.x (zeroed by the select kernel)
  ExpTab tab;
};

#ifndef VO_DESC_THREADS
#define VO_DESC_THREADS 256
#endif
constexpr int kDescThreads = VO_DESC_THREADS;  // samples per block (one per thread)
constexpr int kClassify = 2;  // window positions classified per thread and iteration
// compacted window positions per pass (uint16: windows < 65536): a carried partial block plus
// kClassify blocks always fit, and a pass ends with >= 2 full blocks
constexpr int kPosCap = (kClassify + 2) * kDescThreads;
constexpr int kMaxBatch = 256;
constexpr int kLists = 16 * 9;   // (interior cell, orientation slot 0..8) bins
constexpr int kOwn = (kLists + kDescThreads - 1) / kDescThreads;  // lists summed per thread
constexpr int kMskSlots = 26;    // 16 cell masks, a zero guard, 8 bin masks, a zero guard
// resident descriptor workgroups per CU: every phase of a block is a short latency chain
// (barriers, LDS round trips), so throughput comes from workgroups overlapping (8: 2017 ->
// 1680 us per 8 images against 4, with a 72-byte register spill)
#ifndef VO_DESC_WG_PER_CU
#define VO_DESC_WG_PER_CU 8
#endif
constexpr int kDescWgPerCu = VO_DESC_WG_PER_CU;

__global__ __launch_bounds__(kDescThreads) __attribute__((amdgpu_waves_per_eu(kDescWgPerCu * kDescThreads / 256)))
void sift_desc_kernel(DescArgs A) {
  // per 256-position block of the window: for each of the 144 (cell, orientation slot) bins,
  // the terms it receives, in window order
  __shared__ float s_pool[kDescThreads * 8];           // list terms: <= 4 cells x 2 slots per sample
  __shared__ uint64_t s_msk[kDescThreads / 64][kMskSlots];
  __shared__ int s_lc[kDescThreads / 64][kLists];      // per-wave entry counts
  __shared__ int s_wb[kDescThreads / 64][kLists];      // per-wave write bases
  __shared__ int s_lb[kLists], s_lt[kLists];           // list base and length
  __shared__ uint16_t s_pos[kPosCap];  // valid window positions of the current pass, in order
  __shared__ int s_wc[kClassify][kDescThreads / 64];
  __shared__ float s_h[16 * 9];
  __shared__ float4 s_raw4[kDesc / 4];
  __shared__ int s_off[kMaxBatch + 1];
  __shared__ float s_scale[2];
  __shared__ int s_next;
  float* s_raw = reinterpret_cast<float*>(s_raw4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    int acc = 0;
    for (int b = 0; b < A.batch; ++b) {
      s_off[b] = acc;
      acc += max(A.sel_count[b], 0);
    }
    s_off[A.batch] = acc;
  }
  if (blockIdx.x == 0 && tid < A.batch) A.count_out[tid] = A.sel_count[tid];
  __syncthreads();
  const int total = s_off[A.batch];
  // list ownership: thread t < 144 sums bin t = cell * 9 + slot (slot 9 never receives:
  // o0 + 1 <= n)
  // Keypoints are taken from a counter after each workgroup's first (blockIdx.x): window sizes
  // vary about 4x with the scale, and a fixed stride left the workgroups that drew two large
  // windows running long after the rest had finished.
  for (int g = blockIdx.x; g < total;) {
    int b = 0;
    while (s_off[b + 1] <= g) ++b;
    const int pos = g - s_off[b];
    const float* R = A.okp + (long)A.sel[(long)b * A.cap_img + pos] * kOkpFloats;
    const float x2 = R[0], y2 = R[1], size2 = R[2], angle = R[3], response = R[4];
    const int word = __float_as_int(R[5]);
    const int o = word & 255, layer = (word >> 8) & 255;
    const float s = 1.0f / (float)(1 << o);
    const float ptx = x2 * s, pty = y2 * s, scl = (size2 * s) * 0.5f;
    float ori = 360.f - angle;
    if (fabsf(ori - 360.f) < kFltEps) ori = 0.f;
    const float* img = level_ptr(A.G, A.O, b, o, layer);
    const int rows = A.O.oh[o], cols = A.O.ow[o], pitch = A.O.op[o];
    const int px = (int)rintf(ptx), py = (int)rintf(pty);
    const float a_rad = ori * (float)(3.14159265358979323846 / 180);
    const float cos0 = (float)cos((double)a_rad), sin0 = (float)sin((double)a_rad);
    const float bins_per_rad = (float)kN / 360.f;
    const float exp_scale = -1.f / (kD * kD * 0.5f);
    const float hist_width = 3.f * scl;
    int radius = (int)rintf(hist_width * 1.4142135623730951f * (float)(kD + 1) * 0.5f);
    radius = min(radius, (int)sqrt((double)cols * cols + (double)rows * rows));
    const float cos_t = __fdiv_rn(cos0, hist_width), sin_t = __fdiv_rn(sin0, hist_width);
    const int side = 2 * radius + 1, len = side * side;
    float acc[kOwn];  // the sums of lists tid + w * kDescThreads
  #pragma unroll
    for (int w = 0; w < kOwn; ++w) acc[w] = 0.0f;
    // The window's positions, in order, are classified 256 at a time by the cheap geometry
    // test and the valid ones compacted into s_pos (about half of the square window lies
    // outside the rotated descriptor square); the sample work then runs on dense blocks.
    // While the window has positions left, only full blocks are processed and the remainder
    // (< one block, ahead of every later position) is carried to the front of s_pos.
    int kk0 = 0, n = 0;
    while (kk0 < len || n > 0) {
      while (kk0 < len && n + kClassify * kDescThreads <= kPosCap) {
        // kClassify * 256 positions per iteration, position kk0 + p * 256 + tid in slot p
        bool v[kClassify];
        uint64_t bal[kClassify];
  #pragma unroll
        for (int p = 0; p < kClassify; ++p) {
          const int k = kk0 + p * kDescThreads + tid;
          v[p] = false;
          if (k < len) {
            const int i = k / side - radius, j = k % side - radius;
            const float c_rot = (float)j * cos_t - (float)i * sin_t;
            const float r_rot = (float)j * sin_t + (float)i * cos_t;
            const float rbin = r_rot + (float)(kD / 2) - 0.5f, cbin = c_rot + (float)(kD / 2) - 0.5f;
            const int r = py + i, c = px + j;
            v[p] = rbin > -1 && rbin < kD && cbin > -1 && cbin < kD && r > 0 && r < rows - 1 && c > 0 && c < cols - 1;
          }
          bal[p] = __ballot(v[p]);
          if (lane == 0) s_wc[p][wave] = __popcll(bal[p]);
        }
        __syncthreads();
        int base = n;
  #pragma unroll
        for (int p = 0; p < kClassify; ++p) {
          int off = base, tot = 0;
  #pragma unroll
          for (int w = 0; w < kDescThreads / 64; ++w) {
            off += w < wave ? s_wc[p][w] : 0;
            tot += s_wc[p][w];
          }
          if (v[p]) s_pos[off + __popcll(bal[p] & ((1ull << lane) - 1ull))] = (uint16_t)(kk0 + p * kDescThreads + tid);
          base += tot;
        }
        n = base;
        kk0 += kClassify * kDescThreads;
        __syncthreads();
      }
      const int nproc = kk0 < len ? (n & ~(kDescThreads - 1)) : n;
      for (int t0 = 0; t0 < nproc; t0 += kDescThreads) {
        const bool valid = t0 + tid < nproc;
        int r0 = -9, c0 = -9;
        float ob = 0.0f, v_r0 = 0.0f, v_r1 = 0.0f, cb = 0.0f;
        int o0 = 0;
        {
          if (valid) {
            const int k = s_pos[t0 + tid];
            const int i = k / side - radius, j = k % side - radius;
            const float c_rot = (float)j * cos_t - (float)i * sin_t;
            const float r_rot = (float)j * sin_t + (float)i * cos_t;
            const float rbin = r_rot + (float)(kD / 2) - 0.5f, cbin = c_rot + (float)(kD / 2) - 0.5f;
            const int r = py + i, c = px + j;
            const float dx = img[(long)r * pitch + c + 1] - img[(long)r * pitch + c - 1];
            const float dy = img[(long)(r - 1) * pitch + c] - img[(long)(r + 1) * pitch + c];
            const float w = exp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale, A.tab.v);
            const float Ori = fast_atan2_deg(dy, dx);
            const float Mag = sqrt_rn(dx * dx + dy * dy);
            const float obin = (Ori - ori) * bins_per_rad;
            const float mag = Mag * w;
            o0 = (int)floorf(obin);
            ob = obin - (float)o0;
            if (o0 < 0) o0 += kN;
            if (o0 >= kN) o0 -= kN;
            r0 = (int)floorf(rbin);
            c0 = (int)floorf(cbin);
            const float rb = rbin - (float)r0;
            cb = cbin - (float)c0;
            v_r1 = mag * rb;
            v_r0 = mag - v_r1;
          }
        }
        // (cell, slot) lists: the sample adds v_o0 to slot o0 and v_o1 to slot o0 + 1 of each
        // interior cell q = (r0 + dr) * 4 + (c0 + dc) it votes into (dr, dc in {0, 1}; cell row
        // r0 + 1 + dr of the (d+2)^2 grid).  List L = q * 9 + slot holds exactly the terms bin
        // L receives from this block, in window order: a wave's entries are ranked by ballot
        // (lanes are in window order), and a scan lays the waves' runs and the lists out in one
        // pool.  The owner of L then sums a dense list.
        uint32_t hit = 0;
        if (valid) {
  #pragma unroll
          for (int dr = 0; dr < 2; ++dr)
  #pragma unroll
            for (int dc = 0; dc < 2; ++dc) {
              const int rr = r0 + dr, cc = c0 + dc;
              if ((unsigned)rr < 4u && (unsigned)cc < 4u) hit |= 1u << (rr * 4 + cc);
            }
        }
        // the wave's masks: cells (s_msk[0..15]) and lower orientation bins (s_msk[17 + k]),
        // with zero guards at 16 and 25 for the bins -1 and 8
        uint64_t bal[16];
        uint64_t mv = 0;
  #pragma unroll
        for (int q = 0; q < 16; ++q) {
          bal[q] = __ballot((hit >> q) & 1u);
          mv = lane == q ? bal[q] : mv;
        }
  #pragma unroll
        for (int k = 0; k < kN; ++k) {
          const uint64_t ob_k = __ballot(hit != 0u && o0 == k);
          mv = lane == 17 + k ? ob_k : mv;
        }
        if (lane < kMskSlots) s_msk[wave][lane] = mv;
        __syncthreads();
        // per-wave entry counts of the 144 lists: the wave's samples voting into cell q whose
        // o0 is the slot or the slot - 1
        for (int L = lane; L < kLists; L += 64) {
          const int q = L / 9, sl = L - 9 * q;
          s_lc[wave][L] = __popcll(s_msk[wave][q] & (s_msk[wave][17 + sl] | s_msk[wave][16 + sl]));
        }
        __syncthreads();
        // wave 0 lays the lists out: lane l owns lists 3l .. 3l + 2 (l < 48)
        if (wave == 0) {
          int t3[3], sum = 0;
  #pragma unroll
          for (int u = 0; u < 3; ++u) {
            const int L = 3 * lane + u;
            int t = 0;
  #pragma unroll
            for (int w = 0; w < kDescThreads / 64; ++w) t += L < kLists ? s_lc[w][L] : 0;
            t3[u] = t;
            sum += t3[u];
          }
          const int incl = wave_incl_scan(sum);
          int base = incl - sum;
  #pragma unroll
          for (int u = 0; u < 3; ++u) {
            const int L = 3 * lane + u;
            if (L < kLists) {
              s_lb[L] = base;
              s_lt[L] = t3[u];
              int wb = base;
  #pragma unroll
              for (int w = 0; w < kDescThreads / 64; ++w) {
                s_wb[w][L] = wb;
                wb += s_lc[w][L];
              }
            }
            base += t3[u];
          }
        }
        __syncthreads();
        if (hit) {
          // samples of this wave feeding slot o0 (their o0 is o0 or o0 - 1) and slot o0 + 1
          const uint64_t m_s0 = s_msk[wave][17 + o0] | s_msk[wave][16 + o0];
          const uint64_t m_s1 = s_msk[wave][18 + o0] | s_msk[wave][17 + o0];
          auto rank = [](uint64_t m) {
            return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          };
  #pragma unroll
          for (int q = 0; q < 16; ++q) {
            if ((hit >> q) & 1u) {
              const int dr = q / 4 - r0, dc = q % 4 - c0;
              const float vr = dr ? v_r1 : v_r0;
              const float v_c1 = vr * cb, v_c0 = vr - v_c1;
              const float vc = dc ? v_c1 : v_c0;
              const float v_o1 = vc * ob, v_o0 = vc - v_o1;
              const int L = q * 9 + o0;
              s_pool[s_wb[wave][L] + rank(bal[q] & m_s0)] = v_o0;
              s_pool[s_wb[wave][L + 1] + rank(bal[q] & m_s1)] = v_o1;
            }
          }
        }
        __syncthreads();
        // the owner of list L adds its terms in order.  No barrier follows: the next block
        // writes s_pool, s_lb and s_lt only after two barriers every owner must reach first.
        if (tid < kLists) {
  #pragma unroll
          for (int w = 0; w < kOwn; ++w) {
            const int L = tid + w * kDescThreads;
            if (L < kLists) {
              const float* P = s_pool + s_lb[L];
              const int nl = s_lt[L];
              float a = acc[w];
              int t = 0;
              for (; t + 4 <= nl; t += 4) {
                float e[4];
  #pragma unroll
                for (int u = 0; u < 4; ++u) e[u] = P[t + u];
  #pragma unroll
                for (int u = 0; u < 4; ++u) a = a + e[u];
              }
              for (; t < nl; ++t) a = a + P[t];
              acc[w] = a;
            }
          }
        }
      }
      const int rem = n - nproc;  // uniform
      if (rem > 0) {
        const uint16_t keep = tid < rem ? s_pos[nproc + tid] : (uint16_t)0;
        __syncthreads();
        if (tid < rem) s_pos[tid] = keep;
        __syncthreads();
      }
      n = rem;
    }
  #pragma unroll
    for (int w = 0; w < kOwn; ++w)
      if (tid + w * kDescThreads < kLists) s_h[tid + w * kDescThreads] = acc[w];
    __syncthreads();
    if (tid < kDesc) {
      const int q = tid / kN, k = tid % kN;
      float v = s_h[q * 9 + k];
      if (k == 0) v = v + s_h[q * 9 + kN];  // hist[idx] += hist[idx + n] (slot n + 1 is zero)
      s_raw[tid] = v;
    }
    __syncthreads();
    if (tid == 0) {
      // the two norms in element order (OpenCV's scalar loops)
      float n2 = 0.0f;
#pragma unroll 8
      for (int k = 0; k < kDesc / 4; ++k) {
        const float4 v = s_raw4[k];
        n2 = n2 + v.x * v.x;
        n2 = n2 + v.y * v.y;
        n2 = n2 + v.z * v.z;
        n2 = n2 + v.w * v.w;
      }
      const float thr = sqrt_rn(n2) * 0.2f;
      n2 = 0.0f;
#pragma unroll 8
      for (int k = 0; k < kDesc / 4; ++k) {
        const float4 v = s_raw4[k];
        const float a = fminf(v.x, thr), bb = fminf(v.y, thr), c = fminf(v.z, thr), d = fminf(v.w, thr);
        n2 = n2 + a * a;
        n2 = n2 + bb * bb;
        n2 = n2 + c * c;
        n2 = n2 + d * d;
      }
      s_scale[0] = thr;
      s_scale[1] = __fdiv_rn(512.f, fmaxf(sqrt_rn(n2), kFltEps));
    }
    __syncthreads();
    const long out = (long)b * A.cap_img + pos;
    if (tid < kDesc) {
      const float v = fminf(s_raw[tid], s_scale[0]) * s_scale[1];
      A.desc_out[out * kDesc + tid] = fminf(fmaxf(rintf(v), 0.0f), 255.0f);
    }
    if (tid == 0) {
      vo_sift_keypoint kp;
      kp.x = x2 * 0.5f;
      kp.y = y2 * 0.5f;
      kp.size = size2 * 0.5f;
      kp.angle = angle;
      kp.response = response;
      kp.octave = (word & ~255) | ((o - 1) & 255);  // first octave -1
      kp.image = b;
      kp.reserved = 0;
      A.kp_out[out] = kp;
    }
    if (tid == 0) s_next = (int)gridDim.x + atomicAdd(A.work, 1);
    __syncthreads();
    g = s_next;
  }
}

}  // namespace

ExpTab make_exp_tab() {
  ExpTab t;
  for (int j = 0; j < 64; ++j) t.v[j] = (float)(std::pow(2.0, j / 64.0) * kExpA0);
  return t;
}

// Orientation, filtering and descriptors of the candidates sift_run left in the workspace.
int sift_max_capacity() { return kMaxCapImg; }

void sift_describe(vo_ctx* ctx, int batch, int h, int w, int n_layers, double sigma, int nfeatures, int cap_img,
                   const float* cand_f, const int32_t* cand_i, const int32_t* cand_count, int cand_cap,
                   const float* G, vo_sift_keypoint* d_kp, float* d_desc, int32_t* d_count) {
  VO_REQUIRE(batch >= 1 && batch <= kMaxBatch, VO_ERR_ARG, "sift: batch %d outside 1..%d", batch, kMaxBatch);
  VO_REQUIRE(cap_img >= 1 && cap_img <= kMaxCapImg, VO_ERR_ARG, "sift: capacity %d outside 1..%d", cap_img,
             kMaxCapImg);
  VO_REQUIRE(h <= 16383 && w <= 16383, VO_ERR_ARG, "sift: image %dx%d larger than 16383 pixels a side", h, w);
  // descriptor windows are indexed in 16 bits: (2 radius + 1)^2 < 65536, radius <= 127, with
  // radius <= 3 scl sqrt2 (d + 1) / 2 + 1 and scl <= sigma 2^((n_layers + 0.5) / n_layers)
  const double scl_max = sigma * std::pow(2.0, (n_layers + 0.5) / n_layers);
  VO_REQUIRE(3.0 * scl_max * 1.4142135623730951 * (kD + 1) * 0.5 + 1.0 <= 127.0, VO_ERR_ARG,
             "sift: sigma %g with %d layers gives descriptor windows over 255 samples a side", sigma, n_layers);
  std::vector<int64_t> lay(3 + 5 * kMaxOct);
  const int nv = sift_layout(h, w, n_layers, lay.data(), (int)lay.size());
  VO_REQUIRE(nv <= (int)lay.size(), VO_ERR_ARG, "sift: %dx%d has too many octaves", h, w);
  Octaves O{};
  const int n_oct = (int)lay[0];
  O.g_img = lay[1];
  O.n_layers = n_layers;
  for (int o = 0; o < n_oct; ++o) {
    O.oh[o] = (int)lay[3 + 5 * o];
    O.ow[o] = (int)lay[4 + 5 * o];
    O.op[o] = (int)lay[5 + 5 * o];
    O.off[o] = lay[6 + 5 * o];
  }
  SiftWorkspace& ws = ctx->sift;
  const size_t slots = (size_t)batch * cap_img;
  ws.okp.reserve(slots * kOkpFloats * sizeof(float));
  ws.keys.reserve(slots * 2 * sizeof(uint64_t));
  ws.vals.reserve(slots * 4 * sizeof(uint32_t));
  ws.segs.reserve(((size_t)(kCountStride + 1) * batch + kCountStride) * sizeof(int32_t));
  float* okp = ws.okp.as<float>();
  uint64_t* keys_in = ws.keys.as<uint64_t>();
  uint64_t* keys_out = keys_in + slots;
  uint32_t* vals_in = ws.vals.as<uint32_t>();
  uint32_t* vals_out = vals_in + slots;
  uint32_t* sel = vals_out + slots;
  uint32_t* resp = sel + slots;
  int32_t* img_count = ws.segs.as<int32_t>();
  int32_t* sel_count = img_count + (size_t)batch * kCountStride;
  int32_t* work = sel_count + batch;  // read only by the kernels after select (which zeros it)
  hipStream_t st = ctx->stream;
  const ExpTab tab = make_exp_tab();

  ctx->prof.begin(st, kKSiftOrient);
  VO_HIP_CHECK(hipMemsetAsync(img_count, 0, (size_t)batch * kCountStride * sizeof(int32_t), st));
  OriArgs oa;
  oa.G = G;
  oa.O = O;
  oa.cand_f = cand_f;
  oa.cand_i = cand_i;
  oa.cand_count = cand_count;
  oa.cand_cap = cand_cap;
  oa.cap_img = cap_img;
  oa.okp = okp;
  oa.img_count = img_count;
  oa.tab = tab;
  // persistent: 64-lane workgroups looping over the candidates (count is on the device)
  const int ori_blocks = std::max(1, std::min(cand_cap, ctx->num_cus * kOriWgPerCu));
  hipLaunchKernelGGL(sift_orient_kernel, dim3(ori_blocks), dim3(64), 0, st, oa);
  VO_HIP_CHECK(hipGetLastError());
  ctx->prof.end(st);

  ctx->prof.begin(st, kKSiftSelect);
  hipLaunchKernelGGL(sift_keys_kernel, dim3(ceil_div((int64_t)slots, 256)), dim3(256), 0, st, okp, img_count, cap_img,
                     batch, keys_in, vals_in);
  // image bits 54.. (ceil(log2(batch + 1)) of them; unused slots are all ones)
  int img_bits = 1;
  while ((1 << img_bits) <= batch) ++img_bits;
  const unsigned end_bit = 54u + (unsigned)img_bits;
  size_t tmp_bytes = 0;
  VO_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, keys_in, keys_out, vals_in, vals_out, slots, 0u, end_bit,
                                         st));
  ws.sort_tmp.reserve(tmp_bytes);
  VO_HIP_CHECK(rocprim::radix_sort_pairs(ws.sort_tmp.ptr, tmp_bytes, keys_in, keys_out, vals_in, vals_out, slots, 0u,
                                         end_bit, st));
  SelArgs sa;
  sa.okp = okp;
  sa.keys = keys_out;
  sa.vals = vals_out;
  sa.img_count = img_count;
  sa.cand_count = cand_count;
  sa.cand_cap = cand_cap;
  sa.cap_img = cap_img;
  sa.nfeatures = nfeatures;
  sa.sel = sel;
  sa.sel_count = sel_count;
  sa.resp = resp;
  sa.work = work;
  hipLaunchKernelGGL(sift_select_kernel, dim3(batch), dim3(kSelThreads), 0, st, sa);
  VO_HIP_CHECK(hipGetLastError());
  ctx->prof.end(st);

  ctx->prof.begin(st, kKSiftDesc);
  DescArgs da;
  da.G = G;
  da.O = O;
  da.okp = okp;
  da.sel = sel;
  da.sel_count = sel_count;
  da.batch = batch;
  da.cap_img = cap_img;
  da.kp_out = d_kp;
  da.desc_out = d_desc;
  da.count_out = d_count;
  da.work = work;
  da.tab = tab;
  hipLaunchKernelGGL(sift_desc_kernel, dim3(std::max(1, ctx->num_cus * kDescWgPerCu)), dim3(kDescThreads), 0, st, da);
  VO_HIP_CHECK(hipGetLastError());
  ctx->prof.end(st);
}

}  // namespace vo
