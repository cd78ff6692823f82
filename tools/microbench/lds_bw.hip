// Microbenchmark: LDS throughput of ds_read_b128 on gfx950 with 8 waves hammering LDS at once,
// for the access shapes K3 uses: uniform address per wave (broadcast), lane-contiguous,
// lane stride 48 B (a 6-double row per lane), and 6-of-64 active lanes writing.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/lds_bw.hip -o tools/microbench/bin/lds_bw
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 256
typedef double d2 __attribute__((ext_vector_type(2)));

typedef int i4 __attribute__((ext_vector_type(4)));
#define R16(a)                                                                                          \
  asm volatile(                                                                                         \
      "ds_read_b128 %0, %16 offset:0\n ds_read_b128 %1, %16 offset:1024\n"                              \
      "ds_read_b128 %2, %16 offset:2048\n ds_read_b128 %3, %16 offset:3072\n"                           \
      "ds_read_b128 %4, %16 offset:4096\n ds_read_b128 %5, %16 offset:5120\n"                           \
      "ds_read_b128 %6, %16 offset:6144\n ds_read_b128 %7, %16 offset:7168\n"                           \
      "ds_read_b128 %8, %16 offset:8192\n ds_read_b128 %9, %16 offset:9216\n"                           \
      "ds_read_b128 %10, %16 offset:10240\n ds_read_b128 %11, %16 offset:11264\n"                       \
      "ds_read_b128 %12, %16 offset:12288\n ds_read_b128 %13, %16 offset:13312\n"                       \
      "ds_read_b128 %14, %16 offset:14336\n ds_read_b128 %15, %16 offset:15360\n s_waitcnt lgkmcnt(0)" \
      : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]),    \
        "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15]) \
      : "v"(a)                                                                                          \
      : "memory")

template <int MODE>
__global__ void bw(double* out, unsigned long long* cyc, int nw) {
  __shared__ __attribute__((aligned(16))) double lds[8192];
  const int l = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) lds[i] = i;
  __syncthreads();
  i4 r[16], acc = {0, 0, 0, 0};
  // byte address: wave base in the first 32 KB (offsets add up to 15 KB), per-lane part by mode
  const unsigned base = (unsigned)(uintptr_t)lds + (wave & 1) * 1024 * 0;
  const unsigned a = base + (MODE == 0 ? 0 : MODE == 1 ? 16 * l : 48 * (l & 15) + 16 * (l >> 4) * 0 + 768 * (l >> 4) / 4);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (wave < nw) {
    for (int i = 0; i < ITERS / 16; ++i) {
      R16(a);
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += r[k];
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) cyc[wave] = t1 - t0;
  out[threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

typedef int i2 __attribute__((ext_vector_type(2)));
// 16 writes (b128 or b64) from one asm block, then lgkmcnt(0)
template <int ACTIVE, int B128>
__global__ void wr(double* out, unsigned long long* cyc, int nw) {
  __shared__ __attribute__((aligned(16))) double lds[8192];
  const int l = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned a = (unsigned)(uintptr_t)lds + 16 * l;
  i4 v = {l, wave, 1, 2};
  i2 v2 = {l, wave};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (wave < nw && l < ACTIVE) {
    for (int i = 0; i < ITERS / 16; ++i) {
      if (B128)
        asm volatile(
            "ds_write_b128 %0, %1 offset:0\n ds_write_b128 %0, %1 offset:1024\n ds_write_b128 %0, %1 offset:2048\n"
            "ds_write_b128 %0, %1 offset:3072\n ds_write_b128 %0, %1 offset:4096\n ds_write_b128 %0, %1 offset:5120\n"
            "ds_write_b128 %0, %1 offset:6144\n ds_write_b128 %0, %1 offset:7168\n ds_write_b128 %0, %1 offset:8192\n"
            "ds_write_b128 %0, %1 offset:9216\n ds_write_b128 %0, %1 offset:10240\n ds_write_b128 %0, %1 offset:11264\n"
            "ds_write_b128 %0, %1 offset:12288\n ds_write_b128 %0, %1 offset:13312\n ds_write_b128 %0, %1 offset:14336\n"
            "ds_write_b128 %0, %1 offset:15360\n s_waitcnt lgkmcnt(0)" ::"v"(a), "v"(v) : "memory");
      else
        asm volatile(
            "ds_write_b64 %0, %1 offset:0\n ds_write_b64 %0, %1 offset:1024\n ds_write_b64 %0, %1 offset:2048\n"
            "ds_write_b64 %0, %1 offset:3072\n ds_write_b64 %0, %1 offset:4096\n ds_write_b64 %0, %1 offset:5120\n"
            "ds_write_b64 %0, %1 offset:6144\n ds_write_b64 %0, %1 offset:7168\n ds_write_b64 %0, %1 offset:8192\n"
            "ds_write_b64 %0, %1 offset:9216\n ds_write_b64 %0, %1 offset:10240\n ds_write_b64 %0, %1 offset:11264\n"
            "ds_write_b64 %0, %1 offset:12288\n ds_write_b64 %0, %1 offset:13312\n ds_write_b64 %0, %1 offset:14336\n"
            "ds_write_b64 %0, %1 offset:15360\n s_waitcnt lgkmcnt(0)" ::"v"(a), "v"(v2) : "memory");
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) cyc[wave] = t1 - t0;
  __syncthreads();
  out[threadIdx.x] = lds[threadIdx.x];
}
// 16 ds_read_b64, uniform address
__global__ void rd64(double* out, unsigned long long* cyc, int nw) {
  __shared__ __attribute__((aligned(16))) double lds[8192];
  const int l = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) lds[i] = i;
  __syncthreads();
  const unsigned a = (unsigned)(uintptr_t)lds;
  i2 r[16], acc = {0, 0};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (wave < nw) {
    for (int i = 0; i < ITERS / 16; ++i) {
      asm volatile(
          "ds_read_b64 %0, %16 offset:0\n ds_read_b64 %1, %16 offset:1024\n"
          "ds_read_b64 %2, %16 offset:2048\n ds_read_b64 %3, %16 offset:3072\n"
          "ds_read_b64 %4, %16 offset:4096\n ds_read_b64 %5, %16 offset:5120\n"
          "ds_read_b64 %6, %16 offset:6144\n ds_read_b64 %7, %16 offset:7168\n"
          "ds_read_b64 %8, %16 offset:8192\n ds_read_b64 %9, %16 offset:9216\n"
          "ds_read_b64 %10, %16 offset:10240\n ds_read_b64 %11, %16 offset:11264\n"
          "ds_read_b64 %12, %16 offset:12288\n ds_read_b64 %13, %16 offset:13312\n"
          "ds_read_b64 %14, %16 offset:14336\n ds_read_b64 %15, %16 offset:15360\n s_waitcnt lgkmcnt(0)"
          : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7]),
            "=v"(r[8]), "=v"(r[9]), "=v"(r[10]), "=v"(r[11]), "=v"(r[12]), "=v"(r[13]), "=v"(r[14]), "=v"(r[15])
          : "v"(a)
          : "memory");
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += r[k];
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) cyc[wave] = t1 - t0;
  out[threadIdx.x] = acc.x + acc.y;
}

int main() {
  double* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 512 * 8);
  (void)hipMalloc(&cyc, 8 * 8);
  unsigned long long h[8];
  const char* names[3] = {"uniform (broadcast)", "contiguous 16B/lane", "stride 48B/lane"};
  for (int mode = 0; mode < 3; ++mode)
    for (int nw : {1, 8}) {
      for (int rep = 0; rep < 3; ++rep) {
        if (mode == 0) hipLaunchKernelGGL(bw<0>, dim3(1), dim3(512), 0, 0, out, cyc, nw);
        if (mode == 1) hipLaunchKernelGGL(bw<1>, dim3(1), dim3(512), 0, 0, out, cyc, nw);
        if (mode == 2) hipLaunchKernelGGL(bw<2>, dim3(1), dim3(512), 0, 0, out, cyc, nw);
        (void)hipDeviceSynchronize();
      }
      (void)hipMemcpy(h, cyc, 64, hipMemcpyDeviceToHost);
      printf("ds_read_b128 %-22s waves %d: %.1f cyc per wave-instruction (wave 0)\n", names[mode], nw, h[0] / (double)ITERS);
    }
  for (int b128 : {1, 0})
    for (int act : {6, 64})
      for (int nw : {1, 8}) {
        for (int rep = 0; rep < 3; ++rep) {
          if (b128 && act == 6) hipLaunchKernelGGL((wr<6, 1>), dim3(1), dim3(512), 0, 0, out, cyc, nw);
          if (b128 && act == 64) hipLaunchKernelGGL((wr<64, 1>), dim3(1), dim3(512), 0, 0, out, cyc, nw);
          if (!b128 && act == 6) hipLaunchKernelGGL((wr<6, 0>), dim3(1), dim3(512), 0, 0, out, cyc, nw);
          if (!b128 && act == 64) hipLaunchKernelGGL((wr<64, 0>), dim3(1), dim3(512), 0, 0, out, cyc, nw);
          (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(h, cyc, 64, hipMemcpyDeviceToHost);
        printf("ds_write_b%d %2d active lanes, waves %d: %.1f cyc per wave-instruction\n", b128 ? 128 : 64, act, nw,
               h[0] / (double)ITERS);
      }
  for (int nw : {1, 8}) {
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(rd64, dim3(1), dim3(512), 0, 0, out, cyc, nw);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, cyc, 64, hipMemcpyDeviceToHost);
    printf("ds_read_b64 uniform, waves %d: %.1f cyc per wave-instruction\n", nw, h[0] / (double)ITERS);
  }
  return 0;
}
