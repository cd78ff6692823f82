// SIFT keypoint detection (scale space, DoG, extrema, sub-pixel refinement) on gfx950.
//
// The detection stage (scale space and refined extrema) of
// cv2.SIFT_create(...).detectAndCompute(gray, None) at
// reference src/modules/frontend.py:27-32,55 (OpenCV 4.12 sift.dispatch.cpp /
// sift.simd.hpp), restated with its arithmetic in oracle/sift_ref.py; this file keeps that
// operation order in float32 with FMA contraction off, so every pyramid level is bitwise
// the oracle's and the extremum decisions are exact.
//
// A batch of equally sized images is processed level by level (one launch per pyramid
// level for the whole batch, grid.z = image):
//   sift_upsample_kernel  uint8 -> float32 doubled image (INTER_LINEAR, exact)
//   sift_blur_r_kernel<R> one Gaussian level for tap radius R <= 16 (sift_blur_kernel for
//                         wider kernels): a 64 x 16 output tile, its (16 + 2r) x
//                         (64 + 2r) input tile staged in LDS (BORDER_REFLECT_101), the row
//                         pass for the tile's rows into LDS, the column pass (4 outputs per
//                         thread from registers in both passes), and the DoG
//                         D_{i-1} = G_i - G_{i-1} written beside G_i (HBM-bound: 16 B/pixel)
//   sift_down_kernel      next octave's level 0 = every other pixel of level nOctaveLayers
//   sift_extrema_kernel   per octave: one thread per DoG pixel of levels 1..nOctaveLayers,
//                         the 26-neighbour test; extrema appended to a candidate list
//   sift_refine_kernel    adjustLocalExtrema, one thread per candidate of every octave;
//                         accepted keypoints appended with an atomic counter and put in
//                         (image, octave, level, row, column) order on the host.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "vo_ctx.h"

#pragma clang fp contract(off)

namespace vo {
namespace {

constexpr int kBorder = 5;        // SIFT_IMG_BORDER
constexpr int kMaxInterp = 5;     // SIFT_MAX_INTERP_STEPS
constexpr int kTileW = 64, kTileH = 16, kMaxR = 32;
#ifndef VO_TILE_HR
#define VO_TILE_HR 16
#endif
constexpr int kTileHR = VO_TILE_HR;  // tile height of the radius-specialised blur (16 or 32)
constexpr int kRowsPT = kTileHR / 4;  // column-pass outputs per thread
constexpr int kKpFloats = 8;      // x, y, size, response, xi, (pad) per keypoint
constexpr int kKpInts = 8;        // image, octave word, candidate level, level, row, col, cand row, cand col

struct Taps {
  float k[2 * kMaxR + 1];
  int r;
};

__global__ __launch_bounds__(256) void sift_upsample_kernel(const uint8_t* __restrict__ src, int h, int w,
                                                            int src_stride, float* __restrict__ dst, int pitch,
                                                            long dst_stride) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.z;
  const int W2 = 2 * w, H2 = 2 * h;
  if (x >= W2 || y >= H2) return;
  // source coordinate (d + 0.5) / 2 - 0.5: even d -> (d/2 - 1, 3/4), odd -> (d/2, 1/4);
  // clamped to the edge pixel at both borders
  auto axis = [](int d, int n, int& s0, int& s1, float& a0, float& a1) {
    const int s = (d & 1) ? (d >> 1) : (d >> 1) - 1;
    float f = (d & 1) ? 0.25f : 0.75f;
    if (s < 0 || s + 1 >= n) f = 0.0f;
    s0 = s < 0 ? 0 : (s + 1 >= n ? n - 1 : s);
    s1 = s + 1 < n ? (s + 1 < 0 ? 0 : s + 1) : n - 1;
    a0 = 1.0f - f;
    a1 = f;
  };
  int x0, x1, y0, y1;
  float ax0, ax1, ay0, ay1;
  axis(x, w, x0, x1, ax0, ax1);
  axis(y, h, y0, y1, ay0, ay1);
  const uint8_t* S = src + (long)b * src_stride;
  const float r0 = (float)S[(long)y0 * w + x0] * ax0 + (float)S[(long)y0 * w + x1] * ax1;
  const float r1 = (float)S[(long)y1 * w + x0] * ax0 + (float)S[(long)y1 * w + x1] * ax1;
  dst[(long)b * dst_stride + (long)y * pitch + x] = r0 * ay0 + r1 * ay1;
}

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  const int period = 2 * n - 2;
  i = i < 0 ? -i : i;
  i = i % period;
  return i >= n ? period - i : i;
}

// One Gaussian level (and the DoG beside it when prev != nullptr).
__global__ __launch_bounds__(256) void sift_blur_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                        const float* __restrict__ prev, float* __restrict__ dog,
                                                        int h, int w, int pitch, long stride, long dog_stride,
                                                        Taps T) {
  __shared__ float in[(kTileH + 2 * kMaxR) * (kTileW + 2 * kMaxR)];
  __shared__ float tmp[(kTileH + 2 * kMaxR) * kTileW];
  const int r = T.r, tw = kTileW + 2 * r, th = kTileH + 2 * r;
  const int x0 = blockIdx.x * kTileW, y0 = blockIdx.y * kTileH;
  const long base = (long)blockIdx.z * stride;
  const float* S = src + base;
  for (int e = threadIdx.x; e < tw * th; e += 256) {
    const int ty = e / tw, tx = e - ty * tw;
    const int gy = reflect101(y0 + ty - r, h), gx = reflect101(x0 + tx - r, w);
    in[e] = S[(long)gy * pitch + gx];
  }
  __syncthreads();
  // row pass for every staged row: tmp(ty, tx) = sum_j k_j in(ty, tx + j)
  for (int e = threadIdx.x; e < th * kTileW; e += 256) {
    const int ty = e / kTileW, tx = e - ty * kTileW;
    const float* row = in + ty * tw + tx;
    float s = 0.0f;
    for (int j = 0; j <= 2 * r; ++j) s = s + T.k[j] * row[j];
    tmp[e] = s;
  }
  __syncthreads();
  // column pass: 64 columns x 16 rows, 4 rows per thread
  const int tx = threadIdx.x & 63, ty0 = threadIdx.x >> 6;
  const int gx = x0 + tx;
  for (int q = 0; q < kTileH / 4; ++q) {
    const int ty = ty0 + 4 * q, gy = y0 + ty;
    float s = 0.0f;
    for (int j = 0; j <= 2 * r; ++j) s = s + T.k[j] * tmp[(ty + j) * kTileW + tx];
    if (gx < w && gy < h) {
      const long o = base + (long)gy * pitch + gx;
      dst[o] = s;
      // the DoG buffer holds n_layers + 2 levels per image against G's n_layers + 3
      if (prev) dog[(long)blockIdx.z * dog_stride + (long)gy * pitch + gx] = s - prev[o];
    }
  }
}

// The same level for tap radius R known at compile time: staging with the reflected row
// and column indices computed once per row / column (none for interior tiles), and 4
// outputs per thread in both passes from registers (float4 LDS reads); every output is
// still s = 0, s = s + k_j x_j left to right, so the result is bitwise the generic kernel's.
template <int R>
__global__ __launch_bounds__(256) void sift_blur_r_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                          const float* __restrict__ prev, float* __restrict__ dog,
                                                          int h, int w, int pitch, long stride, long dog_stride,
                                                          Taps T) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  constexpr int TW = kTileW + 2 * R, TWP = (TW + 3) & ~3, TH = kTileHR + 2 * R;
  constexpr int NXR = 4 + 2 * R, NXC = kRowsPT + 2 * R;
  __shared__ float4 in4[TH * TWP / 4];
  __shared__ float4 tmp4[TH * kTileW / 4];
  float* in = reinterpret_cast<float*>(in4);
  float* tmp = reinterpret_cast<float*>(tmp4);
  const int x0 = blockIdx.x * kTileW, y0 = blockIdx.y * kTileHR;
  const long base = (long)blockIdx.z * stride;
  const float* S = src + base;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const bool interior = x0 - R >= 0 && x0 + kTileW + R <= w && y0 - R >= 0 && y0 + kTileHR + R <= h;
  int gx0 = x0 + tx - R, gx1 = x0 + tx + 64 - R;
  if (!interior) {
    gx0 = reflect101(gx0, w);
    gx1 = reflect101(gx1, w);
  }
  for (int r = ty; r < TH; r += 4) {
    const int gy = interior ? y0 + r - R : reflect101(y0 + r - R, h);
    const float* row = S + (long)gy * pitch;
    in[r * TWP + tx] = row[gx0];
    if (tx + 64 < TW) in[r * TWP + tx + 64] = row[gx1];
  }
  __syncthreads();
  float k[2 * R + 1];
#pragma unroll
  for (int j = 0; j <= 2 * R; ++j) k[j] = T.k[j];
  // row pass: TH rows x 16 column quads; outputs in pairs as packed fp32 (v_pk_mul_f32 and
  // v_pk_add_f32: per element the same IEEE multiply and add, no FMA)
  for (int t = threadIdx.x; t < TH * 16; t += 256) {
    const int r = t >> 4, q = (t & 15) * 4;
    const float4* p = in4 + (r * TWP + q) / 4;
    float x[(NXR + 3) & ~3];
#pragma unroll
    for (int m = 0; m < (NXR + 3) / 4; ++m) {
      const float4 v = p[m];
      x[4 * m] = v.x;
      x[4 * m + 1] = v.y;
      x[4 * m + 2] = v.z;
      x[4 * m + 3] = v.w;
    }
    f2 s01 = f2{0.0f, 0.0f}, s23 = f2{0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j <= 2 * R; ++j) {
      const f2 kj = f2{k[j], k[j]};
      s01 = s01 + kj * f2{x[j], x[j + 1]};
      s23 = s23 + kj * f2{x[j + 2], x[j + 3]};
    }
    tmp4[(r * kTileW + q) / 4] = make_float4(s01.x, s01.y, s23.x, s23.y);
  }
  __syncthreads();
  // column pass: column tx, rows kRowsPT ty .. kRowsPT (ty + 1) - 1, in pairs
  float x[NXC];
#pragma unroll
  for (int m = 0; m < NXC; ++m) x[m] = tmp[(kRowsPT * ty + m) * kTileW + tx];
  const int gx = x0 + tx;
#pragma unroll
  for (int u = 0; u < kRowsPT; u += 2) {
    f2 s = f2{0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j <= 2 * R; ++j) s = s + f2{k[j], k[j]} * f2{x[u + j], x[u + 1 + j]};
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int gy = y0 + kRowsPT * ty + u + e;
      const float v = e ? s.y : s.x;
      if (gx < w && gy < h) {
        const long o = base + (long)gy * pitch + gx;
        dst[o] = v;
        if (prev) dog[(long)blockIdx.z * dog_stride + (long)gy * pitch + gx] = v - prev[o];
      }
    }
  }
}

// One Gaussian level through the radius-specialised kernel when there is one.
void launch_blur(dim3 grid, hipStream_t st, const float* src, float* dst, const float* prev, float* dog, int h,
                 int w, int pitch, long stride, long dog_stride, const Taps& T) {
  const dim3 gridr(grid.x, ceil_div(h, kTileHR), grid.z);
#define VO_BLUR_CASE(RR)                                                                                        \
  case RR:                                                                                                      \
    hipLaunchKernelGGL(sift_blur_r_kernel<RR>, gridr, dim3(256), 0, st, src, dst, prev, dog, h, w, pitch, stride, \
                       dog_stride, T);                                                                          \
    return;
  switch (T.r) {
    VO_BLUR_CASE(1) VO_BLUR_CASE(2) VO_BLUR_CASE(3) VO_BLUR_CASE(4) VO_BLUR_CASE(5) VO_BLUR_CASE(6)
    VO_BLUR_CASE(7) VO_BLUR_CASE(8) VO_BLUR_CASE(9) VO_BLUR_CASE(10) VO_BLUR_CASE(11) VO_BLUR_CASE(12)
    VO_BLUR_CASE(13) VO_BLUR_CASE(14) VO_BLUR_CASE(15) VO_BLUR_CASE(16)
    default:
      hipLaunchKernelGGL(sift_blur_kernel, grid, dim3(256), 0, st, src, dst, prev, dog, h, w, pitch, stride,
                         dog_stride, T);
  }
#undef VO_BLUR_CASE
}

__global__ __launch_bounds__(256) void sift_down_kernel(const float* __restrict__ src, int src_pitch, long src_stride,
                                                        float* __restrict__ dst, int h, int w, int pitch, long stride) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= w || y >= h) return;
  dst[(long)blockIdx.z * stride + (long)y * pitch + x] =
      src[(long)blockIdx.z * src_stride + (long)(2 * y) * src_pitch + 2 * x];
}

constexpr int kMaxOctaves = 16;
constexpr int kCandRegions = 64;  // candidate appends spread over this many counters
constexpr int kExtRun = 8;        // rows per thread of the extrema test
constexpr int kCandStride = 64;   // ints between two candidate counters (own 256-byte line)

// Per-octave DoG geometry of a batch (all octaves in one launch of the refinement).
struct DogGeom {
  const float* dog;                 // DoG pyramid base
  long img_stride;                  // floats per image
  long off[kMaxOctaves];            // octave's first DoG level
  int h[kMaxOctaves], w[kMaxOctaves], pitch[kMaxOctaves];
};

struct ExtArgs {
  const float* dog;  // octave's DoG levels: level l of image b at dog + b * img_stride + l * lvl_stride
  long img_stride, lvl_stride;
  int h, w, pitch, n_layers, octave, threshold;
  uint64_t* cand;    // packed (image, octave, level, row, column) of the 26-neighbour extrema:
  int cand_cap;      //   kCandRegions regions of cand_cap entries,
  int32_t* cand_n;   //   each with its own append counter
};

struct RefArgs {
  DogGeom G;
  int n_layers, capacity;
  float contrast, edge, sigma;
  const uint64_t* cand;  // kCandRegions x cand_cap
  int cand_cap;
  const int32_t* cand_n;  // kCandRegions counters
  float* kp_f;       // (capacity, kKpFloats)
  int32_t* kp_i;     // (capacity, kKpInts)
  int32_t* count;
};

__device__ __forceinline__ uint64_t pack_cand(int b, int o, int layer, int r, int c) {
  return ((uint64_t)b << 48) | ((uint64_t)o << 44) | ((uint64_t)layer << 40) | ((uint64_t)r << 20) | (uint64_t)c;
}

__device__ __forceinline__ float at(const float* L, int pitch, int r, int c) { return L[(long)r * pitch + c]; }

// Matx33f::solve(DECOMP_LU): Cramer's rule with the determinant in float; zeros if singular.
__device__ __forceinline__ void solve3(const float (&a)[3][3], const float (&b)[3], float (&x)[3]) {
  const float det = a[0][0] * (a[1][1] * a[2][2] - a[2][1] * a[1][2]) - a[0][1] * (a[1][0] * a[2][2] - a[2][0] * a[1][2]) +
                    a[0][2] * (a[1][0] * a[2][1] - a[2][0] * a[1][1]);
  if (det == 0.0f) {
    x[0] = x[1] = x[2] = 0.0f;
    return;
  }
  const float d = __fdiv_rn(1.0f, det);
  x[0] = d * (b[0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) - a[0][1] * (b[1] * a[2][2] - a[1][2] * b[2]) +
              a[0][2] * (b[1] * a[2][1] - a[1][1] * b[2]));
  x[1] = d * (a[0][0] * (b[1] * a[2][2] - a[1][2] * b[2]) - b[0] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
              a[0][2] * (a[1][0] * b[2] - b[1] * a[2][0]));
  x[2] = d * (a[0][0] * (a[1][1] * b[2] - b[1] * a[2][1]) - a[0][1] * (a[1][0] * b[2] - b[1] * a[2][0]) +
              b[0] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]));
}

struct ExtView {
  long lvl_stride;
  int h, w, pitch, n_layers, octave, capacity;
  float contrast, edge, sigma;
  float* kp_f;
  int32_t* kp_i;
  int32_t* count;
};

// adjustLocalExtrema of one candidate: true and the keypoint record (F, Q) when accepted.
__device__ __forceinline__ bool refine_one(const ExtView& A, const float* D, int b, int layer0, int r, int c,
                                           float (&F)[kKpFloats], int32_t (&Q)[kKpInts]) {
  // adjustLocalExtrema (oracle/sift_ref.py adjust_local_extremum)
  const float img_scale = 1.0f / 255.0f;
  const float deriv_scale = img_scale * 0.5f, second = img_scale, cross = img_scale * 0.25f;
  float xi = 0.0f, xr = 0.0f, xc = 0.0f;
  int layer = layer0, rr = r, cc = c, i = 0;
  for (; i < kMaxInterp; ++i) {
    const float* I = D + (long)layer * A.lvl_stride;
    const float* P = I - A.lvl_stride;
    const float* N = I + A.lvl_stride;
    const int p = A.pitch;
    const float dD[3] = {(at(I, p, rr, cc + 1) - at(I, p, rr, cc - 1)) * deriv_scale,
                         (at(I, p, rr + 1, cc) - at(I, p, rr - 1, cc)) * deriv_scale,
                         (at(N, p, rr, cc) - at(P, p, rr, cc)) * deriv_scale};
    const float v2 = at(I, p, rr, cc) * 2.0f;
    const float dxx = (at(I, p, rr, cc + 1) + at(I, p, rr, cc - 1) - v2) * second;
    const float dyy = (at(I, p, rr + 1, cc) + at(I, p, rr - 1, cc) - v2) * second;
    const float dss = (at(N, p, rr, cc) + at(P, p, rr, cc) - v2) * second;
    const float dxy = (at(I, p, rr + 1, cc + 1) - at(I, p, rr + 1, cc - 1) - at(I, p, rr - 1, cc + 1) +
                       at(I, p, rr - 1, cc - 1)) * cross;
    const float dxs = (at(N, p, rr, cc + 1) - at(N, p, rr, cc - 1) - at(P, p, rr, cc + 1) + at(P, p, rr, cc - 1)) * cross;
    const float dys = (at(N, p, rr + 1, cc) - at(N, p, rr - 1, cc) - at(P, p, rr + 1, cc) + at(P, p, rr - 1, cc)) * cross;
    const float H[3][3] = {{dxx, dxy, dxs}, {dxy, dyy, dys}, {dxs, dys, dss}};
    float X[3];
    solve3(H, dD, X);
    xi = -X[2];
    xr = -X[1];
    xc = -X[0];
    if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
    const float lim = (float)(2147483647 / 3);
    if (fabsf(xi) > lim || fabsf(xr) > lim || fabsf(xc) > lim) return false;
    cc += (int)rint(xc);
    rr += (int)rint(xr);
    layer += (int)rint(xi);
    if (layer < 1 || layer > A.n_layers || cc < kBorder || cc >= A.w - kBorder || rr < kBorder || rr >= A.h - kBorder)
      return false;
  }
  if (i >= kMaxInterp) return false;
  const float* I = D + (long)layer * A.lvl_stride;
  const float* P = I - A.lvl_stride;
  const float* N = I + A.lvl_stride;
  const int p = A.pitch;
  const float dD[3] = {(at(I, p, rr, cc + 1) - at(I, p, rr, cc - 1)) * deriv_scale,
                       (at(I, p, rr + 1, cc) - at(I, p, rr - 1, cc)) * deriv_scale,
                       (at(N, p, rr, cc) - at(P, p, rr, cc)) * deriv_scale};
  const float t = (0.0f + dD[0] * xc + dD[1] * xr) + dD[2] * xi;
  const float contr = at(I, p, rr, cc) * img_scale + t * 0.5f;
  if (fabsf(contr) * (float)A.n_layers < A.contrast) return false;
  const float v2 = at(I, p, rr, cc) * 2.0f;
  const float dxx = (at(I, p, rr, cc + 1) + at(I, p, rr, cc - 1) - v2) * second;
  const float dyy = (at(I, p, rr + 1, cc) + at(I, p, rr - 1, cc) - v2) * second;
  const float dxy = (at(I, p, rr + 1, cc + 1) - at(I, p, rr + 1, cc - 1) - at(I, p, rr - 1, cc + 1) +
                     at(I, p, rr - 1, cc - 1)) * cross;
  const float tr = dxx + dyy, det = dxx * dyy - dxy * dxy;
  if (det <= 0.0f || tr * tr * A.edge >= (A.edge + 1.0f) * (A.edge + 1.0f) * det) return false;
  const float scale = (float)(1 << A.octave);
  F[0] = ((float)cc + xc) * scale;
  F[1] = ((float)rr + xr) * scale;
  // powf(2, e) as (float)exp2((double)e): correctly rounded on host and device alike
  F[2] = A.sigma * (float)exp2((double)(((float)layer + xi) / (float)A.n_layers)) * scale * 2.0f;
  F[3] = fabsf(contr);
  F[4] = xi;
  F[5] = F[6] = F[7] = 0.0f;
  Q[0] = b;
  Q[1] = A.octave + (layer << 8) + ((int)rint(((double)xi + 0.5) * 255) << 16);
  Q[2] = layer0;
  Q[3] = layer;
  Q[4] = rr;
  Q[5] = cc;
  Q[6] = r;
  Q[7] = c;
  return true;
}

// One thread per DoG pixel of levels 1..n_layers: the 26-neighbour test; extrema are
// appended to the candidate list (refined by sift_refine_kernel, all octaves at once, so
// the few candidates do not hold a whole wave each through the Newton steps).
__global__ __launch_bounds__(256) void sift_extrema_kernel(ExtArgs A) {
  // thread = one column and a run of kExtRun rows; the 3 x 3 x 3 neighbourhood slides down
  // the run in registers (a ring of three rows per level, static slots after unrolling):
  // 9 loads per pixel instead of 27
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * (4 * kExtRun) + (threadIdx.x >> 6) * kExtRun;
  const int lz = blockIdx.z % A.n_layers, b = blockIdx.z / A.n_layers;
  const int layer0 = lz + 1;
  const int rs = max(r0, kBorder), re = min(r0 + kExtRun, A.h - kBorder);
  const bool colok = c >= kBorder && c < A.w - kBorder;
  const int cc = colok ? c : kBorder;  // loads stay inside the image
  const float* L1 = A.dog + (long)b * A.img_stride + (long)layer0 * A.lvl_stride;
  const float* Lv[3] = {L1 - A.lvl_stride, L1, L1 + A.lvl_stride};
  float W[3][3][3];  // [level][ring slot][column - 1]
  auto ld = [&](int slot, int r) {
    const long ro = (long)min(max(r, 0), A.h - 1) * A.pitch + cc;
#pragma unroll
    for (int l = 0; l < 3; ++l) {
      W[l][slot][0] = Lv[l][ro - 1];
      W[l][slot][1] = Lv[l][ro];
      W[l][slot][2] = Lv[l][ro + 1];
    }
  };
  ld(0, r0 - 1);
  ld(1, r0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ int s_off[4][kExtRun];
  __shared__ int s_base;
  uint64_t bal[kExtRun];
#pragma unroll
  for (int u = 0; u < kExtRun; ++u) {
    const int r = r0 + u;
    ld((u + 2) % 3, r + 1);
    const int sl[3] = {u % 3, (u + 1) % 3, (u + 2) % 3};  // rows r - 1, r, r + 1
    const float val = W[1][sl[1]][1];
    bool ext = false;
    if (colok && r >= rs && r < re && fabsf(val) > (float)A.threshold) {
      bool is_max = val > 0, is_min = val < 0;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const float a = W[0][sl[dy]][dx], n = W[2][sl[dy]][dx];
          is_max = is_max && val >= a && val >= n;
          is_min = is_min && val <= a && val <= n;
          if (dy != 1 || dx != 1) {
            const float sv = W[1][sl[dy]][dx];
            is_max = is_max && val >= sv;
            is_min = is_min && val <= sv;
          }
        }
      bool flat = false;
      if (is_max || is_min) {  // (rare: the flatness test only for the points that passed)
        flat = true;
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            if (dy != 1 || dx != 1) flat = flat && W[1][sl[dy]][dx] == val;
      }
      // A point whose own level is constant over its 3 x 3 neighbourhood (a flat or saturated
      // region: a constant image has constant DoG levels, and at a zero threshold every pixel
      // of such a level can pass the 26-neighbour test) is one adjustLocalExtrema always
      // rejects: dx = dy = dxx = dyy = dxy = 0 there, so the offset solve is singular (X = 0,
      // the point stays) and the edge test sees det = dxx dyy - dxy^2 = 0 <= 0.  Dropping it
      // here keeps such regions from flooding the candidate lists.
      ext = (is_max || is_min) && !flat;
    }
    bal[u] = __ballot(ext);
    if (lane == 0) s_off[wave][u] = __popcll(bal[u]);
  }
  // the workgroup's candidates in (wave, row, lane) order: one atomic per workgroup, on one
  // of kCandRegions counters (each on its own 256-byte line)
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int q = 0; q < 4 * kExtRun; ++q) {
      const int v = s_off[q / kExtRun][q % kExtRun];
      s_off[q / kExtRun][q % kExtRun] = acc;
      acc += v;
    }
    const int region = (int)((blockIdx.x + 7u * blockIdx.y + 13u * blockIdx.z) % kCandRegions);
    s_base = acc ? atomicAdd(A.cand_n + region * kCandStride, acc) : 0;
    s_off[0][0] = region;  // (offset 0 of the first group is always 0)
  }
  __syncthreads();
  const int region = s_off[0][0], base = s_base;
  const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int u = 0; u < kExtRun; ++u) {
    if ((bal[u] >> lane) & 1ull) {
      const int slot = base + (wave == 0 && u == 0 ? 0 : s_off[wave][u]) + __popcll(bal[u] & lt);
      if (slot < A.cand_cap) A.cand[(long)region * A.cand_cap + slot] = pack_cand(b, A.octave, layer0, r0 + u, c);
    }
  }
}

// adjustLocalExtrema for every candidate of the batch, one thread each (grid-stride over
// the device-side count); accepted keypoints appended with an atomic counter.
__global__ __launch_bounds__(256) void sift_refine_kernel(RefArgs RA) {
  const int region = blockIdx.y;
  const int ncand = RA.cand_n[region * kCandStride];
  if (ncand > RA.cand_cap) {  // candidates were dropped: poison the count (host raises)
    // (a flag bit, set idempotently: one addition per overflowing region wrapped the count
    // around to a small or negative number once four or more regions overflowed)
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(RA.count, 1 << 30);
    return;
  }
  const uint64_t* cand = RA.cand + (long)region * RA.cand_cap;
  const int lane = threadIdx.x & 63;
  // wave-uniform loop: accepted keypoints are appended with one atomic per wave
  for (int wbase = blockIdx.x * 256 + (int)(threadIdx.x & ~63u); wbase < ncand; wbase += gridDim.x * 256) {
    const int ci = wbase + lane;
    bool ok = false;
    float F[kKpFloats];
    int32_t Q[kKpInts];
    if (ci < ncand) {
      const uint64_t pc = cand[ci];
      const int b = (int)(pc >> 48), o = (int)((pc >> 44) & 15), layer0 = (int)((pc >> 40) & 15);
      const int r = (int)((pc >> 20) & 0xFFFFF), c = (int)(pc & 0xFFFFF);
      ExtView A;
      A.h = RA.G.h[o];
      A.w = RA.G.w[o];
      A.pitch = RA.G.pitch[o];
      A.lvl_stride = (long)A.h * A.pitch;
      A.n_layers = RA.n_layers;
      A.octave = o;
      A.capacity = RA.capacity;
      A.contrast = RA.contrast;
      A.edge = RA.edge;
      A.sigma = RA.sigma;
      A.kp_f = RA.kp_f;
      A.kp_i = RA.kp_i;
      A.count = RA.count;
      const float* D = RA.G.dog + (long)b * RA.G.img_stride + RA.G.off[o];
      ok = refine_one(A, D, b, layer0, r, c, F, Q);
    }
    const uint64_t bal = __ballot(ok);
    if (bal == 0) continue;
    const int leader = __ffsll((unsigned long long)bal) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(RA.count, __popcll(bal));
    base = __shfl(base, leader);
    if (ok) {
      const int slot = base + __popcll(bal & ((1ull << lane) - 1ull));
      if ((unsigned)slot < (unsigned)RA.capacity) {
#pragma unroll
        for (int e = 0; e < kKpFloats; ++e) RA.kp_f[(long)slot * kKpFloats + e] = F[e];
#pragma unroll
        for (int e = 0; e < kKpInts; ++e) RA.kp_i[(long)slot * kKpInts + e] = Q[e];
      }
    }
  }
}

Taps make_taps(double sigma) {
  // getGaussianKernelBitExact's structure in double (oracle/sift_ref.py gaussian_kernel)
  const int n = (int)std::nearbyint(sigma * 4 * 2 + 1) | 1;
  VO_REQUIRE(n <= 2 * kMaxR + 1, VO_ERR_ARG, "sift: sigma %g needs %d taps (max %d)", sigma, n, 2 * kMaxR + 1);
  const double scale2x = -0.125 / (sigma * sigma);
  const int n2 = (n - 1) / 2;
  std::vector<double> vals(n2);
  double total = 0.0;
  int x = 1 - n;
  for (int i = 0; i < n2; ++i, x += 2) {
    vals[i] = std::exp((double)(x * x) * scale2x);
    total += vals[i];
  }
  total *= 2.0;
  total += 1.0;
  if ((n & 1) == 0) total += 1.0;
  const double mul1 = 1.0 / total;
  Taps T;
  T.r = n / 2;
  for (int i = 0; i < n2; ++i) T.k[i] = T.k[n - 1 - i] = (float)(vals[i] * mul1);
  for (int i = n2; i <= n - 1 - n2; ++i) T.k[i] = (float)mul1;
  return T;
}

}  // namespace

// Pyramid geometry of a batch (host): octave sizes, pitches and buffer offsets.
struct SiftGeom {
  int h2, w2, n_oct, n_layers;
  std::vector<int> oh, ow, op;        // per octave
  std::vector<long> g_off, d_off;     // per octave: first level's offset (floats) in G / DoG
  long g_img, d_img;                  // floats per image
};

static SiftGeom sift_geom(int h, int w, int n_layers) {
  SiftGeom g;
  g.h2 = 2 * h;
  g.w2 = 2 * w;
  g.n_layers = n_layers;
  g.n_oct = (int)std::nearbyint(std::log((double)std::min(g.h2, g.w2)) / std::log(2.0) - 2) + 1;
  long go = 0, dofs = 0;
  int oh = g.h2, ow = g.w2;
  for (int o = 0; o < g.n_oct; ++o) {
    if (o) {
      oh /= 2;
      ow /= 2;
    }
    const int pitch = ((ow + 63) / 64) * 64;
    g.oh.push_back(oh);
    g.ow.push_back(ow);
    g.op.push_back(pitch);
    g.g_off.push_back(go);
    g.d_off.push_back(dofs);
    go += (long)(n_layers + 3) * oh * pitch;
    dofs += (long)(n_layers + 2) * oh * pitch;
  }
  g.g_img = go;
  g.d_img = dofs;
  return g;
}

void sift_run(vo_ctx* ctx, const uint8_t* d_img, int batch, int h, int w, double contrast, double edge,
              double sigma, int n_layers, int capacity, float* d_kpf, int32_t* d_kpi, int32_t* d_count,
              float** g_out, float** d_out, int64_t* layout) {
  VO_REQUIRE(batch >= 1 && h >= 1 && w >= 1 && n_layers >= 1 && n_layers <= 8 && sigma > 0 && capacity >= 0,
             VO_ERR_ARG, "sift: bad arguments (batch %d, %dx%d, layers %d, sigma %g)", batch, h, w, n_layers, sigma);
  const SiftGeom g = sift_geom(h, w, n_layers);
  VO_REQUIRE(g.n_oct >= 1, VO_ERR_ARG, "sift: image %dx%d too small", h, w);
  SiftWorkspace& ws = ctx->sift;
  ws.g.reserve((size_t)batch * g.g_img * sizeof(float));
  ws.d.reserve((size_t)batch * g.d_img * sizeof(float));
  float* G = ws.g.as<float>();
  float* Dg = ws.d.as<float>();
  hipStream_t st = ctx->stream;
  VO_HIP_CHECK(hipMemsetAsync(d_count, 0, sizeof(int32_t), st));
  const std::vector<double> sig = [&] {
    std::vector<double> s(n_layers + 3);
    s[0] = sigma;
    const double k = std::pow(2.0, 1.0 / n_layers);
    for (int i = 1; i < n_layers + 3; ++i) {
      const double prev = std::pow(k, (double)(i - 1)) * sigma, total = prev * k;
      s[i] = std::sqrt(total * total - prev * prev);
    }
    return s;
  }();
  const float sf = (float)sigma;
  const float sig_diff = sqrtf(std::max(sf * sf - 0.5f * 0.5f * 4, 0.01f));
  const int threshold = (int)std::floor(0.5 * contrast / n_layers * 255);
  // candidate lists of the 26-neighbour extrema (kCandRegions regions with their own
  // counters): at most one per 9 pixels of a level, bounded here by a quarter of the
  // candidate levels' pixels (overflow poisons the keypoint count)
  int64_t cand_px = 0;
  for (int o = 0; o < g.n_oct; ++o) cand_px += (int64_t)g.oh[o] * g.ow[o];
  const int cand_cap = (int)std::min<int64_t>(((int64_t)batch * n_layers * cand_px / 4) / kCandRegions + 1024,
                                              (int64_t)1 << 26);  // per region
  ws.cand_ext.reserve((size_t)kCandRegions * cand_cap * sizeof(uint64_t) +
                      (size_t)kCandRegions * kCandStride * sizeof(int32_t));
  uint64_t* cand = ws.cand_ext.as<uint64_t>();
  int32_t* cand_n = reinterpret_cast<int32_t*>(cand + (size_t)kCandRegions * cand_cap);
  VO_HIP_CHECK(hipMemsetAsync(cand_n, 0, (size_t)kCandRegions * kCandStride * sizeof(int32_t), st));
  auto launch_extrema = [&](int o, hipStream_t s) {
    const int oh = g.oh[o], ow = g.ow[o];
    if (oh <= 2 * kBorder || ow <= 2 * kBorder) return;
    ExtArgs A;
    A.dog = Dg + g.d_off[o];
    A.img_stride = g.d_img;
    A.lvl_stride = (long)oh * g.op[o];
    A.h = oh;
    A.w = ow;
    A.pitch = g.op[o];
    A.n_layers = n_layers;
    A.octave = o;
    A.threshold = threshold;
    A.cand = cand;
    A.cand_cap = cand_cap;
    A.cand_n = cand_n;
    hipLaunchKernelGGL(sift_extrema_kernel, dim3(ceil_div(ow, 64), ceil_div(oh, 4 * kExtRun), batch * n_layers),
                       dim3(256), 0, s, A);
  };
  // The chain from octave to octave runs through level n_layers (the next octave's base), so
  // octave o's last two levels and its extrema test (which needs every DoG level of the
  // octave) go to a second stream once level n_layers is done, beside octave o + 1's chain;
  // the context stream joins it before the refinement.  Under the event profiler (per-phase
  // spans on one stream) every launch stays on the context stream.
  const bool overlap = !ctx->prof.on && g.n_oct < (int)(sizeof(ws.side_ev) / sizeof(ws.side_ev[0]));
  if (overlap && !ws.side) {
    VO_HIP_CHECK(hipStreamCreateWithFlags(&ws.side, hipStreamNonBlocking));
    for (hipEvent_t& e : ws.side_ev) VO_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  ctx->prof.begin(st, kKSiftPyramid);
  for (int o = 0; o < g.n_oct; ++o) {
    const int oh = g.oh[o], ow = g.ow[o], op = g.op[o];
    const long lvl = (long)oh * op;
    float* Go = G + g.g_off[o];
    float* Do = Dg + g.d_off[o];
    const dim3 px(ceil_div(ow, 64), ceil_div(oh, 4), batch);
    const dim3 tiles(ceil_div(ow, kTileW), ceil_div(oh, kTileH), batch);
    if (o == 0) {
      // the doubled image goes to level 1's slot, which its own blur overwrites later
      hipLaunchKernelGGL(sift_upsample_kernel, px, dim3(256), 0, st, d_img, h, w, h * w, Go + lvl, op, g.g_img);
      launch_blur(tiles, st, Go + lvl, Go, nullptr, nullptr, oh, ow, op, g.g_img, g.d_img,
                  make_taps((double)sig_diff));
    } else {
      const long src = g.g_off[o - 1] + (long)n_layers * g.oh[o - 1] * g.op[o - 1];
      hipLaunchKernelGGL(sift_down_kernel, px, dim3(256), 0, st, G + src, g.op[o - 1], g.g_img, Go, oh, ow, op,
                         g.g_img);
    }
    const int split = overlap ? n_layers + 1 : n_layers + 3;  // levels [1, split) on the context stream
    for (int i = 1; i < split; ++i)
      launch_blur(tiles, st, Go + (i - 1) * lvl, Go + i * lvl, Go + (i - 1) * lvl, Do + (i - 1) * lvl, oh, ow, op,
                  g.g_img, g.d_img, make_taps(sig[i]));
    if (overlap) {
      VO_HIP_CHECK(hipEventRecord(ws.side_ev[o], st));
      VO_HIP_CHECK(hipStreamWaitEvent(ws.side, ws.side_ev[o], 0));
      for (int i = split; i < n_layers + 3; ++i)
        launch_blur(tiles, ws.side, Go + (i - 1) * lvl, Go + i * lvl, Go + (i - 1) * lvl, Do + (i - 1) * lvl, oh, ow,
                    op, g.g_img, g.d_img, make_taps(sig[i]));
      launch_extrema(o, ws.side);
    }
    VO_HIP_CHECK(hipGetLastError());
  }
  ctx->prof.end(st);
  ctx->prof.begin(st, kKSiftExtrema);
  if (overlap) {
    VO_HIP_CHECK(hipEventRecord(ws.side_ev[g.n_oct], ws.side));
    VO_HIP_CHECK(hipStreamWaitEvent(st, ws.side_ev[g.n_oct], 0));
  } else {
    for (int o = 0; o < g.n_oct; ++o) launch_extrema(o, st);
  }
  if (capacity > 0 || d_kpf) {
    RefArgs R{};
    R.G.dog = Dg;
    R.G.img_stride = g.d_img;
    for (int o = 0; o < g.n_oct; ++o) {
      R.G.off[o] = g.d_off[o];
      R.G.h[o] = g.oh[o];
      R.G.w[o] = g.ow[o];
      R.G.pitch[o] = g.op[o];
    }
    R.n_layers = n_layers;
    R.capacity = capacity;
    R.contrast = (float)contrast;
    R.edge = (float)edge;
    R.sigma = sf;
    R.cand = cand;
    R.cand_cap = cand_cap;
    R.cand_n = cand_n;
    R.kp_f = d_kpf;
    R.kp_i = d_kpi;
    R.count = d_count;
    hipLaunchKernelGGL(sift_refine_kernel, dim3(std::max(1, ctx->num_cus / 4), kCandRegions), dim3(256), 0, st, R);
  }
  ctx->prof.end(st);
  VO_HIP_CHECK(hipGetLastError());
  if (g_out) *g_out = G;
  if (d_out) *d_out = Dg;
  if (layout) {
    layout[0] = g.n_oct;
    layout[1] = g.g_img;
    layout[2] = g.d_img;
  }
}

// Host: the pyramid geometry (n_oct, then per octave h, w, pitch, G offset, DoG offset).
int sift_layout(int h, int w, int n_layers, int64_t* out, int n) {
  const SiftGeom g = sift_geom(h, w, n_layers);
  std::vector<int64_t> v = {g.n_oct, g.g_img, g.d_img};
  for (int o = 0; o < g.n_oct; ++o) {
    v.push_back(g.oh[o]);
    v.push_back(g.ow[o]);
    v.push_back(g.op[o]);
    v.push_back(g.g_off[o]);
    v.push_back(g.d_off[o]);
  }
  const int m = std::min<int>(n, (int)v.size());
  for (int i = 0; i < m; ++i) out[i] = v[i];
  return (int)v.size();
}

}  // namespace vo
