// Scalar math of the SIFT orientation / descriptor kernels (sift_desc.hip), host and
// device (VO_HD) so that tools and tests can run it on the CPU (sift_host_check.cpp):
// OpenCV 4.12's cv::hal::exp32f and cv::fastAtan2, scalar paths, no FMA (oracle/sift_ref.py
// exp32f, fast_atan2).  Float division is correctly rounded on gfx950 by default
// (-fhip-fp32-correctly-rounded-divide-sqrt), as on the host.  Float sqrt is not
// __fsqrt_rn, which this HIP maps to the approximate native sqrt: sqrt_rn below.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>

#pragma clang fp contract(off)

#ifndef VO_HD
#define VO_HD __host__ __device__ inline __attribute__((always_inline))
#endif

namespace vo {
namespace siftm {

VO_HD float as_float(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// cv::hal::exp32f constants (core/src/mathfuncs_core.simd.hpp), scalar path
constexpr double kExpA0 = .9670371139572337719125840413672004409288e-2;
constexpr float kExpA4 = (float)(1.000000000000002438532970795181890933776 / kExpA0);
constexpr float kExpA3 = (float)(.6931471805521448196800669615864773144641 / kExpA0);
constexpr float kExpA2 = (float)(.2402265109513301490103372422686535526573 / kExpA0);
constexpr float kExpA1 = (float)(.5550339366753125211915322047004666939128e-1 / kExpA0);
constexpr double kExpPre = 1.4426950408889634073599246810019 * 64;
constexpr float kExpPrescale = (float)kExpPre;
constexpr float kExpPostscale = (float)(1.0 / 64);
constexpr float kExpMin = (float)(-3000.0 * 64 / kExpPre);
constexpr float kExpMax = (float)(3000.0 * 64 / kExpPre);

// cv::fastAtan2 constants: float literal times (float)(180 / pi), in float
constexpr float kRad2Deg = (float)(180.0 / 3.14159265358979323846);
constexpr float kAtP1 = (float)0.9997878412794807 * kRad2Deg;
constexpr float kAtP3 = (float)-0.3258083974640975 * kRad2Deg;
constexpr float kAtP5 = (float)0.1555786518463281 * kRad2Deg;
constexpr float kAtP7 = (float)-0.04432655554792128 * kRad2Deg;
constexpr float kDblEpsF = (float)2.220446049250313e-16;

// Correctly rounded sqrtf on host and device. On gfx950 `sqrtf` is LLVM's correctly rounded
// expansion (v_sqrt_f32, then the fma residuals of the neighbouring floats pick the result);
// __fsqrt_rn is not (it maps to the native approximation unless OCML_BASIC_ROUNDED_OPERATIONS).
VO_HD float sqrt_rn(float x) { return sqrtf(x); }

struct ExpTab {
  float v[64];
};

VO_HD float exp32f(float x, const float* tab) {
  x = fminf(fmaxf(x, kExpMin), kExpMax);
  x = x * kExpPrescale;
  const int xi = (int)rintf(x);  // saturate_cast<int>(float): round half to even
  x = (x - (float)xi) * kExpPostscale;
  int t = (xi >> 6) + 127;
  t = !(t & ~255) ? t : (t < 0 ? 0 : 255);
  const float buf = as_float((uint32_t)t << 23);
  return buf * tab[xi & 63] * ((((x + kExpA1) * x + kExpA2) * x + kExpA3) * x + kExpA4);
}

VO_HD float fast_atan2_deg(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  float a;
  if (ax >= ay) {
    const float c = ay / (ax + kDblEpsF), c2 = c * c;
    a = (((kAtP7 * c2 + kAtP5) * c2 + kAtP3) * c2 + kAtP1) * c;
  } else {
    const float c = ax / (ay + kDblEpsF), c2 = c * c;
    a = 90.f - (((kAtP7 * c2 + kAtP5) * c2 + kAtP3) * c2 + kAtP1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

}  // namespace siftm
}  // namespace vo
