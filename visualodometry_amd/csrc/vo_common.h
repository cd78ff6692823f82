// Shared helpers for the vo_hip library (gfx950 only; no CUDA/HIP dual paths).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/vo_hip.h"

namespace vo {

// Thread-local last-error message returned by vo_last_error().
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
const char* last_error();

struct Error {
  int code;
};

#define VO_HIP_CHECK(expr)                                                        \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) {                                                       \
      ::vo::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,          \
                      hipGetErrorString(e_));                                     \
      throw ::vo::Error{e_ == hipErrorOutOfMemory ? VO_ERR_NOMEM : VO_ERR_HIP};   \
    }                                                                             \
  } while (0)

#define VO_REQUIRE(cond, code, ...)   \
  do {                                \
    if (!(cond)) {                    \
      ::vo::set_error(__VA_ARGS__);   \
      throw ::vo::Error{code};        \
    }                                 \
  } while (0)

// Growth of the on-demand buffers: a quarter of headroom, so a window that grows by a few
// landmarks per keyframe does not free (an implicit device synchronisation) and reallocate
// its buffers on most calls.
inline size_t buf_grow(size_t n) { return ((n ? n : 16) + n / 4 + 255) & ~(size_t)255; }

// Device buffer that grows on demand and is freed with its owner.
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  void reserve(size_t n) {
    if (n <= bytes) return;
    if (ptr) VO_HIP_CHECK(hipFree(ptr));
    ptr = nullptr;
    bytes = 0;
    const size_t b = buf_grow(n);
    VO_HIP_CHECK(hipMalloc(&ptr, b));
    bytes = b;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(ptr);
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
  void swap(DevBuf& o) noexcept {
    std::swap(ptr, o.ptr);
    std::swap(bytes, o.bytes);
  }
  ~DevBuf() { release(); }
};

// Page-locked host staging buffer that grows on demand (asynchronous DMA, no page faults).
struct HostBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  void reserve(size_t n) {
    if (n <= bytes) return;
    if (ptr) VO_HIP_CHECK(hipHostFree(ptr));
    ptr = nullptr;
    bytes = 0;
    const size_t b = buf_grow(n);
    VO_HIP_CHECK(hipHostMalloc(&ptr, b, hipHostMallocDefault));
    bytes = b;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(ptr);
  }
  ~HostBuf() {
    if (ptr) (void)hipHostFree(ptr);
  }
};

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Runs `fn`, converting vo::Error into the status code (message already set).
template <class F>
int guarded(F&& fn) {
  try {
    fn();
    return VO_OK;
  } catch (const Error& e) {
    return e.code;
  } catch (const std::exception& e) {
    set_error("internal error: %s", e.what());
    return VO_ERR_HIP;
  }
}

}  // namespace vo
