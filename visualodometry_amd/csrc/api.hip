// extern "C" entry points of libvo_hip.so (declared in include/vo_hip.h).
#include <cstdarg>
#include <algorithm>
#include <array>
#include <cstring>
#include <vector>

#include "ba_band.h"
#include "ba_plan.h"
#include "vo_ctx.h"
#include "../../include/vo_hip_testing.h"

namespace vo {

namespace {
thread_local std::string g_err;
}

void set_error(const char* f, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, f);
  std::vsnprintf(buf, sizeof buf, f, ap);
  va_end(ap);
  g_err = buf;
}
const char* last_error() { return g_err.c_str(); }

hipEvent_t Profiler::get() {
  if (used == pool.size()) {
    hipEvent_t e;
    VO_HIP_CHECK(hipEventCreate(&e));
    pool.push_back(e);
  }
  return pool[used++];
}

void Profiler::begin(hipStream_t st, int id) {
  if (!on) return;
  Rec r{id, get(), get()};
  VO_HIP_CHECK(hipEventRecord(r.start, st));
  recs.push_back(r);
}

void Profiler::end(hipStream_t st) {
  if (!on || recs.empty()) return;
  VO_HIP_CHECK(hipEventRecord(recs.back().stop, st));
}

static_assert(kKCount == VO_PROFILE_KERNELS, "profiler ids match include/vo_hip.h");

void Profiler::read(double* ms, int64_t* counts) {
  for (int k = 0; k < kKCount; ++k) {
    ms[k] = 0.0;
    counts[k] = 0;
  }
  for (const Rec& r : recs) {
    float t = 0.0f;
    VO_HIP_CHECK(hipEventElapsedTime(&t, r.start, r.stop));
    ms[r.id] += t;
    counts[r.id] += 1;
  }
  recs.clear();
  used = 0;
}

Profiler::~Profiler() {
  for (hipEvent_t e : pool) (void)hipEventDestroy(e);
}

// ba.hip
uint64_t ba_setup(vo_ctx*, const vo_ba_problem*);
void ba_reserve(vo_ctx*, int, int, int64_t, int);
void ba_check_session(vo_ctx*, uint64_t);
void ba_set_state(vo_ctx*, const double*, const double*);
void ba_get_state(vo_ctx*, double*, double*);
int ba_run(vo_ctx*, int, double*, bool);
int ba_gn_step(vo_ctx*, double*, double*, double*, double*);
int ba_stats(vo_ctx*, int64_t*, int);
int ba_stamps(vo_ctx*, uint64_t*, int);
void comm_unique_id(char out[128]);
void comm_init(vo_ctx*, int, int, const char*);
void comm_init_loopback(vo_ctx*, int, int, const char*);

namespace {

void bind(vo_ctx* ctx) {
  VO_REQUIRE(ctx, VO_ERR_ARG, "null vo_ctx");
  VO_HIP_CHECK(hipSetDevice(ctx->device));
}

// Host-array matcher call: descriptors staged into the workspace, results copied back.
// A caller's device pointer must be device memory of the context's GPU, known to this HIP runtime,
// whose allocation covers [p, p + bytes).
void check_device_range(vo_ctx* ctx, const void* p, size_t bytes, const char* what) {
  if (bytes == 0) return;
  VO_REQUIRE(p != nullptr, VO_ERR_ARG, "%s: null device pointer", what);
  hipPointerAttribute_t at{};
  const hipError_t e = hipPointerGetAttributes(&at, p);
  if (e != hipSuccess) (void)hipGetLastError();
  VO_REQUIRE(e == hipSuccess && at.type == hipMemoryTypeDevice && at.device == ctx->device, VO_ERR_ARG,
             "%s: not device memory of device %d in this process's HIP runtime", what, ctx->device);
  void* base = nullptr;
  size_t size = 0;
  const hipError_t e2 = hipMemGetAddressRange(&base, &size, const_cast<void*>(p));
  if (e2 != hipSuccess) (void)hipGetLastError();
  VO_REQUIRE(e2 == hipSuccess && (const char*)p + bytes <= (const char*)base + size, VO_ERR_ARG,
             "%s: %zu bytes past its allocation", what, bytes);
}

void match_host(vo_ctx* ctx, const float* des0, int n0, const float* des1, int n1, int dim,
                double ratio, int32_t* pairs, int32_t* count, int32_t* idx2, float* dist2, uint64_t q_tag = 0,
                bool device_src = false) {
  VO_REQUIRE(n0 >= 0 && n1 >= 0 && dim >= 1, VO_ERR_ARG, "match: bad shape n0=%d n1=%d dim=%d",
             n0, n1, dim);
  VO_REQUIRE((n0 == 0 || des0) && (n1 == 0 || des1), VO_ERR_ARG, "match: null descriptors");
  if (count) *count = 0;
  if (n0 == 0) return;
  hipStream_t st = ctx->stream;
  MatchWorkspace& ws = ctx->match;
  MatchQueryCache& qc = ctx->match_q;
  // the query side's cache (a nonzero tag; the int8 path's dimensions): a hit skips the query's
  // upload and packing, a miss packs it into the cache first
  const bool use_cache = q_tag != 0 && n1 > 0 && dim <= 256;
  const bool hit = use_cache && qc.valid && qc.tag == q_tag && qc.src == (const void*)des0 && qc.n0 == n0 &&
                   qc.dim == dim && qc.device_src == device_src;
  const size_t b0 = (size_t)n0 * dim * 4, b1 = (size_t)n1 * dim * 4;
  const float* d0 = des0;
  const float* d1 = des1;
  if (!device_src) {
    ws.des.reserve((use_cache ? 0 : b0) + b1 + 16);
    float* stage1 = ws.des.as<float>() + (use_cache ? 0 : (size_t)n0 * dim);
    if (use_cache) {
      if (!hit) {
        qc.des.reserve(b0);
        VO_HIP_CHECK(hipMemcpyAsync(qc.des.ptr, des0, b0, hipMemcpyHostToDevice, st));
      }
      d0 = qc.des.as<float>();
    } else {
      VO_HIP_CHECK(hipMemcpyAsync(ws.des.ptr, des0, b0, hipMemcpyHostToDevice, st));
      d0 = ws.des.as<float>();
    }
    if (n1) VO_HIP_CHECK(hipMemcpyAsync(stage1, des1, b1, hipMemcpyHostToDevice, st));
    d1 = stage1;
  }
  if (use_cache && !hit) {
    qc.valid = false;
    match_pack_query(ctx, d0, n0, dim, qc);
    qc.tag = q_tag;
    qc.src = des0;
    qc.n0 = n0;
    qc.dim = dim;
    qc.device_src = device_src;
    qc.valid = true;
  }
  ws.best.reserve((size_t)n0 * 4);
  int32_t* d_idx2 = nullptr;
  float* d_dist2 = nullptr;
  if (idx2) {
    ws.top2.reserve((size_t)n0 * 16);
    d_idx2 = ws.top2.as<int32_t>();
    d_dist2 = reinterpret_cast<float*>(d_idx2 + 2 * (size_t)n0);
  }
  match_run(ctx, d0, d1, 1, n0, n1, dim, ratio, ws.best.as<int32_t>(), d_idx2, d_dist2, use_cache ? &qc : nullptr);
  if (pairs) {
    ws.pairs.reserve((size_t)n0 * 8 + 16);
    int32_t* d_pairs = ws.pairs.as<int32_t>();
    int32_t* d_count = d_pairs + 2 * (size_t)n0;
    compact_pairs(ctx, ws.best.as<int32_t>(), n0, d_pairs, d_count);
    // the count and all n0 pair slots (out_pairs' capacity; the slots past the count are left
    // unspecified) in one round trip: 8 n0 bytes more over PCIe instead of a second sync
    VO_HIP_CHECK(hipMemcpyAsync(count, d_count, 4, hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipMemcpyAsync(pairs, d_pairs, (size_t)n0 * 8, hipMemcpyDeviceToHost, st));
  }
  if (idx2) {
    VO_HIP_CHECK(hipMemcpyAsync(idx2, d_idx2, (size_t)n0 * 8, hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipMemcpyAsync(dist2, d_dist2, (size_t)n0 * 8, hipMemcpyDeviceToHost, st));
  }
  VO_HIP_CHECK(hipStreamSynchronize(st));
}

}  // namespace
}  // namespace vo

using vo::guarded;

extern "C" {

int vo_abi_version(void) { return VO_ABI_VERSION; }

const char* vo_last_error(void) { return vo::last_error(); }

vo_ctx* vo_create(int device, int flags) {
  (void)flags;
  vo_ctx* out = nullptr;
  int rc = guarded([&] {
    int n = 0;
    VO_HIP_CHECK(hipGetDeviceCount(&n));
    VO_REQUIRE(device >= 0 && device < n, VO_ERR_NODEV, "vo_create: device %d not present (%d devices)",
               device, n);
    hipDeviceProp_t prop;
    VO_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    VO_REQUIRE(std::strncmp(prop.gcnArchName, "gfx950", 6) == 0, VO_ERR_NODEV,
               "vo_create: device %d is %s; this library is built for gfx950 only", device,
               prop.gcnArchName);
    VO_HIP_CHECK(hipSetDevice(device));
    std::unique_ptr<vo_ctx> c(new vo_ctx);
    c->device = device;
    c->num_cus = prop.multiProcessorCount;
    VO_HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    out = c.release();
  });
  return rc == VO_OK ? out : nullptr;
}

void vo_destroy(vo_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  delete ctx;
}

void* vo_stream(vo_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int vo_synchronize(vo_ctx* ctx) {
  return guarded([&] {
    vo::bind(ctx);
    VO_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  });
}

void* vo_device_alloc(vo_ctx* ctx, uint64_t bytes) {
  void* p = nullptr;
  int rc = guarded([&] {
    vo::bind(ctx);
    VO_HIP_CHECK(hipMalloc(&p, bytes ? bytes : 16));
  });
  return rc == VO_OK ? p : nullptr;
}

int vo_device_free(vo_ctx* ctx, void* ptr) {
  return guarded([&] {
    vo::bind(ctx);
    VO_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (ptr) VO_HIP_CHECK(hipFree(ptr));
  });
}

int vo_memcpy_h2d(vo_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
  return guarded([&] {
    vo::bind(ctx);
    VO_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    VO_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  });
}

int vo_memcpy_d2h(vo_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
  return guarded([&] {
    vo::bind(ctx);
    VO_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    VO_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  });
}

int vo_match_knn2_ratio(vo_ctx* ctx, const float* des0, int n0, const float* des1, int n1,
                        int dim, double ratio, int32_t* out_pairs, int32_t* out_count) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(out_pairs && out_count, VO_ERR_ARG, "vo_match_knn2_ratio: null outputs");
    vo::match_host(ctx, des0, n0, des1, n1, dim, ratio, out_pairs, out_count, nullptr, nullptr);
  });
}

int vo_match_knn2_ratio_q(vo_ctx* ctx, const float* des0, int n0, uint64_t des0_tag, const float* des1, int n1,
                          int dim, double ratio, int32_t* out_pairs, int32_t* out_count) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(out_pairs && out_count, VO_ERR_ARG, "vo_match_knn2_ratio_q: null outputs");
    vo::match_host(ctx, des0, n0, des1, n1, dim, ratio, out_pairs, out_count, nullptr, nullptr, des0_tag, false);
  });
}

int vo_match_knn2_ratio_dev(vo_ctx* ctx, const float* d_des0, int n0, uint64_t des0_tag, const float* d_des1,
                            int n1, int dim, double ratio, int32_t* out_pairs, int32_t* out_count) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(out_pairs && out_count, VO_ERR_ARG, "vo_match_knn2_ratio_dev: null outputs");
    VO_REQUIRE(n0 >= 0 && n1 >= 0 && dim >= 1, VO_ERR_ARG, "vo_match_knn2_ratio_dev: bad shape");
    // no kernel reads a pointer this runtime does not know as device memory of the context's GPU
    // covering the rows (a pointer of another HIP runtime instance, or of host memory, is refused)
    vo::check_device_range(ctx, d_des0, (size_t)n0 * dim * 4, "des0");
    vo::check_device_range(ctx, d_des1, (size_t)n1 * dim * 4, "des1");
    vo::match_host(ctx, d_des0, n0, d_des1, n1, dim, ratio, out_pairs, out_count, nullptr, nullptr, des0_tag, true);
  });
}

int vo_match_knn2(vo_ctx* ctx, const float* des0, int n0, const float* des1, int n1, int dim,
                  int32_t* idx_out, float* dist_out) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(idx_out && dist_out, VO_ERR_ARG, "vo_match_knn2: null outputs");
    vo::match_host(ctx, des0, n0, des1, n1, dim, 0.0, nullptr, nullptr, idx_out, dist_out);
  });
}

int vo_triangulate(vo_ctx* ctx, const double* P1, const double* P2, const double* T_cw2,
                   const double* K, const float* pts1, const float* pts2, int n,
                   double min_depth, double max_reproj_err, float* pts3d_out, uint8_t* mask_out) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(P1 && P2 && T_cw2 && K && n >= 0, VO_ERR_ARG, "vo_triangulate: bad arguments");
    if (n == 0) return;
    VO_REQUIRE(pts1 && pts2 && pts3d_out && mask_out, VO_ERR_ARG, "vo_triangulate: null arrays");
    const size_t in = (size_t)n * 2 * sizeof(float), out3 = (size_t)n * 3 * sizeof(float);
    ctx->match.tri.reserve(2 * in + out3 + (size_t)n + 64);
    char* base = ctx->match.tri.as<char>();
    float* d1 = reinterpret_cast<float*>(base);
    float* d2 = reinterpret_cast<float*>(base + in);
    float* d3 = reinterpret_cast<float*>(base + 2 * in);
    uint8_t* dm = reinterpret_cast<uint8_t*>(base + 2 * in + out3);
    hipStream_t st = ctx->stream;
    VO_HIP_CHECK(hipMemcpyAsync(d1, pts1, in, hipMemcpyHostToDevice, st));
    VO_HIP_CHECK(hipMemcpyAsync(d2, pts2, in, hipMemcpyHostToDevice, st));
    vo::tri_run(ctx, P1, P2, T_cw2, K, d1, d2, n, min_depth, max_reproj_err, d3, dm);
    VO_HIP_CHECK(hipMemcpyAsync(pts3d_out, d3, out3, hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipMemcpyAsync(mask_out, dm, (size_t)n, hipMemcpyDeviceToHost, st));
    VO_HIP_CHECK(hipStreamSynchronize(st));
  });
}

int vo_triangulate_async(vo_ctx* ctx, const double* P1, const double* P2, const double* T_cw2,
                         const double* K, const float* d_pts1, const float* d_pts2, int n,
                         double min_depth, double max_reproj_err, float* d_pts3d, uint8_t* d_mask) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(P1 && P2 && T_cw2 && K && n >= 0, VO_ERR_ARG, "vo_triangulate_async: bad arguments");
    if (n == 0) return;
    VO_REQUIRE(d_pts1 && d_pts2 && d_pts3d && d_mask, VO_ERR_ARG, "vo_triangulate_async: null arrays");
    vo::tri_run(ctx, P1, P2, T_cw2, K, d_pts1, d_pts2, n, min_depth, max_reproj_err, d_pts3d, d_mask);
  });
}

int vo_pnp_ransac(vo_ctx* ctx, const float* objpts, const float* imgpts, int n, const double* K,
                  int iterations, double reproj_err, double confidence, double* rvec_out,
                  double* tvec_out, uint8_t* mask_out, int32_t* success_out) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(K && n >= 0 && rvec_out && tvec_out && success_out, VO_ERR_ARG,
               "vo_pnp_ransac: bad arguments");
    VO_REQUIRE(n == 0 || (objpts && imgpts && mask_out), VO_ERR_ARG, "vo_pnp_ransac: null arrays");
    *success_out = 0;
    for (int k = 0; k < 3; ++k) rvec_out[k] = tvec_out[k] = 0.0;
    if (n == 0) return;
    // device and page-locked host staging share one layout, X | uv | pose | status | mask: the
    // points go up in one copy and the results come back in one
    const size_t bx = (size_t)n * 12, bu = (size_t)n * 8, bp = 64, bm = (size_t)n;
    const size_t po = (bx + bu + 15) & ~size_t(15), total = po + bp + 16 + bm;
    vo::DevBuf& st = ctx->pnp.stage;
    vo::HostBuf& hs = ctx->pnp.hstage;
    st.reserve(total + 64);
    hs.reserve(total + 64);
    char* base = st.as<char>();
    char* hbase = hs.as<char>();
    float* dX = reinterpret_cast<float*>(base);
    float* dU = reinterpret_cast<float*>(base + bx);
    double* dP = reinterpret_cast<double*>(base + po);
    int32_t* dS = reinterpret_cast<int32_t*>(base + po + bp);
    uint8_t* dM = reinterpret_cast<uint8_t*>(dS + 4);
    hipStream_t s = ctx->stream;
    std::memcpy(hbase, objpts, bx);
    std::memcpy(hbase + bx, imgpts, bu);
    VO_HIP_CHECK(hipMemcpyAsync(base, hbase, bx + bu, hipMemcpyHostToDevice, s));
    const int32_t offs[2] = {0, n};
    vo::pnp_run(ctx, dX, dU, offs, 1, K, iterations, reproj_err, confidence, dP, dM, dS);
    VO_HIP_CHECK(hipMemcpyAsync(hbase + po, dP, total - po, hipMemcpyDeviceToHost, s));
    VO_HIP_CHECK(hipStreamSynchronize(s));
    const double* pose = reinterpret_cast<const double*>(hbase + po);
    const int32_t* status = reinterpret_cast<const int32_t*>(hbase + po + bp);
    std::memcpy(mask_out, hbase + po + bp + 16, bm);
    for (int k = 0; k < 3; ++k) {
      rvec_out[k] = pose[k];
      tvec_out[k] = pose[3 + k];
    }
    *success_out = status[0];
  });
}

int vo_pnp_ransac_batch_async(vo_ctx* ctx, const float* d_objpts, const float* d_imgpts,
                              const int32_t* offsets, int batch, const double* K, int iterations,
                              double reproj_err, double confidence, double* d_pose, uint8_t* d_mask,
                              int32_t* d_status) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(offsets && K && batch >= 0 && d_pose && d_status, VO_ERR_ARG,
               "vo_pnp_ransac_batch_async: bad arguments");
    VO_REQUIRE(batch == 0 || offsets[batch] == 0 || (d_objpts && d_imgpts && d_mask), VO_ERR_ARG,
               "vo_pnp_ransac_batch_async: null arrays");
    vo::pnp_run(ctx, d_objpts, d_imgpts, offsets, batch, K, iterations, reproj_err, confidence, d_pose,
                d_mask, d_status);
  });
}

int vo_sift_detect(vo_ctx* ctx, const uint8_t* img, int h, int w, double contrast, double edge, double sigma,
                   int n_layers, int capacity, float* kp_f, int32_t* kp_i, int32_t* count) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(img && count && capacity >= 0 && (capacity == 0 || (kp_f && kp_i)), VO_ERR_ARG,
               "vo_sift_detect: bad arguments");
    VO_REQUIRE(h >= 1 && w >= 1, VO_ERR_ARG, "vo_sift_detect: empty image %dx%d", h, w);
    vo::SiftWorkspace& ws = ctx->sift;
    const size_t nimg = (size_t)h * w;
    const size_t cap = (size_t)std::max(capacity, 1);
    ws.img.reserve(nimg);
    ws.kp.reserve(cap * 64 + 64);
    float* dF = ws.kp.as<float>();
    int32_t* dI = reinterpret_cast<int32_t*>(dF + cap * 8);
    int32_t* dC = dI + cap * 8;
    hipStream_t s = ctx->stream;
    VO_HIP_CHECK(hipMemcpyAsync(ws.img.ptr, img, nimg, hipMemcpyHostToDevice, s));
    vo::sift_run(ctx, ws.img.as<uint8_t>(), 1, h, w, contrast, edge, sigma, n_layers, capacity, dF, dI, dC, nullptr,
                 nullptr, nullptr);
    int32_t found = 0;
    VO_HIP_CHECK(hipMemcpyAsync(&found, dC, 4, hipMemcpyDeviceToHost, s));
    VO_HIP_CHECK(hipStreamSynchronize(s));
    const int k = std::min(found, capacity);
    *count = found;
    if (k == 0) return;
    std::vector<float> F((size_t)k * 8);
    std::vector<int32_t> I((size_t)k * 8);
    VO_HIP_CHECK(hipMemcpyAsync(F.data(), dF, F.size() * 4, hipMemcpyDeviceToHost, s));
    VO_HIP_CHECK(hipMemcpyAsync(I.data(), dI, I.size() * 4, hipMemcpyDeviceToHost, s));
    VO_HIP_CHECK(hipStreamSynchronize(s));
    // (image, octave, candidate level, candidate row, candidate column): OpenCV's loop order
    std::vector<int> ord(k);
    for (int i = 0; i < k; ++i) ord[i] = i;
    auto key = [&](int i) {
      const int32_t* q = &I[(size_t)i * 8];
      return std::array<int64_t, 6>{q[0], q[1] & 255, q[2], q[6], q[7], i};
    };
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return key(a) < key(b); });
    for (int i = 0; i < k; ++i) {
      std::memcpy(kp_f + (size_t)i * 8, &F[(size_t)ord[i] * 8], 32);
      std::memcpy(kp_i + (size_t)i * 8, &I[(size_t)ord[i] * 8], 32);
    }
  });
}

int vo_sift_detect_batch_async(vo_ctx* ctx, const uint8_t* d_imgs, int batch, int h, int w, double contrast,
                               double edge, double sigma, int n_layers, int capacity, float* d_kpf,
                               int32_t* d_kpi, int32_t* d_count) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(d_imgs && d_count && capacity >= 0 && (capacity == 0 || (d_kpf && d_kpi)), VO_ERR_ARG,
               "vo_sift_detect_batch_async: bad arguments");
    vo::sift_run(ctx, d_imgs, batch, h, w, contrast, edge, sigma, n_layers, capacity, d_kpf, d_kpi, d_count,
                 nullptr, nullptr, nullptr);
  });
}

int vo_sift_pyramid(vo_ctx* ctx, const uint8_t* img, int h, int w, double sigma, int n_layers, float* g_out,
                    int64_t g_floats, float* d_out, int64_t d_floats) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(img && g_out && d_out && h >= 1 && w >= 1, VO_ERR_ARG, "vo_sift_pyramid: bad arguments");
    int64_t lay[3];
    vo::sift_layout(h, w, n_layers, lay, 3);
    VO_REQUIRE(g_floats >= lay[1] && d_floats >= lay[2], VO_ERR_ARG,
               "vo_sift_pyramid: outputs too small (%lld/%lld floats needed)", (long long)lay[1], (long long)lay[2]);
    vo::SiftWorkspace& ws = ctx->sift;
    ws.img.reserve((size_t)h * w);
    ws.kp.reserve(64);
    hipStream_t s = ctx->stream;
    VO_HIP_CHECK(hipMemcpyAsync(ws.img.ptr, img, (size_t)h * w, hipMemcpyHostToDevice, s));
    float *G = nullptr, *D = nullptr;
    vo::sift_run(ctx, ws.img.as<uint8_t>(), 1, h, w, 0.04, 10.0, sigma, n_layers, 0, nullptr, nullptr,
                 ws.kp.as<int32_t>(), &G, &D, nullptr);
    VO_HIP_CHECK(hipMemcpyAsync(g_out, G, (size_t)lay[1] * 4, hipMemcpyDeviceToHost, s));
    VO_HIP_CHECK(hipMemcpyAsync(d_out, D, (size_t)lay[2] * 4, hipMemcpyDeviceToHost, s));
    VO_HIP_CHECK(hipStreamSynchronize(s));
  });
}

// detectAndCompute of a device batch: detection into the workspace's candidate list, then
// orientation / filtering / descriptors into the caller's buffers.
static void sift_full(vo_ctx* ctx, const uint8_t* d_imgs, int batch, int h, int w, int nfeatures, double contrast,
               double edge, double sigma, int n_layers, int capacity, vo_sift_keypoint* d_kps, float* d_desc,
               int32_t* d_counts) {
  VO_REQUIRE(d_imgs && d_kps && d_desc && d_counts && batch >= 1 && capacity >= 1 && nfeatures >= 0, VO_ERR_ARG,
             "sift detectAndCompute: bad arguments");
  vo::SiftWorkspace& ws = ctx->sift;
  const int cand_cap = (int)std::min<int64_t>((int64_t)batch * capacity, 1 << 24);
  ws.cand.reserve((size_t)cand_cap * 64 + 64);
  float* cf = ws.cand.as<float>();
  int32_t* ci = reinterpret_cast<int32_t*>(cf + (size_t)cand_cap * 8);
  int32_t* cc = ci + (size_t)cand_cap * 8;
  float* G = nullptr;
  vo::sift_run(ctx, d_imgs, batch, h, w, contrast, edge, sigma, n_layers, cand_cap, cf, ci, cc, &G, nullptr,
               nullptr);
  vo::sift_describe(ctx, batch, h, w, n_layers, sigma, nfeatures, capacity, cf, ci, cc, cand_cap, G, d_kps, d_desc,
                    d_counts);
}

int vo_sift_detect_and_compute(vo_ctx* ctx, const uint8_t* img, int h, int w, int nfeatures, double contrast,
                               double edge, double sigma, int n_layers, int capacity, vo_sift_keypoint* kps,
                               float* desc, int32_t* count) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(img && kps && desc && count && capacity >= 1 && h >= 1 && w >= 1, VO_ERR_ARG,
               "vo_sift_detect_and_compute: bad arguments");
    vo::SiftWorkspace& ws = ctx->sift;
    const size_t nimg = (size_t)h * w;
    ws.img.reserve(nimg);
    hipStream_t s = ctx->stream;
    VO_HIP_CHECK(hipMemcpyAsync(ws.img.ptr, img, nimg, hipMemcpyHostToDevice, s));
    // The working capacity (oriented keypoints before duplicate removal and retainBest)
    // starts at the caller's; an overflowing pass reports the capacity it needed (-n) and the
    // next pass takes that (at least twice the last, at most the kernel limit: OpenCV has no
    // cap); only the final keypoints must fit the caller's buffers.
    int cap = std::min(capacity, vo::sift_max_capacity()), n = -1;
    vo_sift_keypoint* dK = nullptr;
    float* dD = nullptr;
    for (;;) {
      ws.out.reserve((size_t)cap * (sizeof(vo_sift_keypoint) + 128 * sizeof(float)) + 64);
      dK = ws.out.as<vo_sift_keypoint>();
      dD = reinterpret_cast<float*>(dK + cap);
      int32_t* dC = reinterpret_cast<int32_t*>(dD + (size_t)cap * 128);
      sift_full(ctx, ws.img.as<uint8_t>(), 1, h, w, nfeatures, contrast, edge, sigma, n_layers, cap, dK, dD, dC);
      VO_HIP_CHECK(hipMemcpyAsync(&n, dC, 4, hipMemcpyDeviceToHost, s));
      VO_HIP_CHECK(hipStreamSynchronize(s));
      if (n >= 0 || cap >= vo::sift_max_capacity()) break;
      cap = (int)std::min<int64_t>(std::max<int64_t>(-(int64_t)n, 2ll * cap), vo::sift_max_capacity());
    }
    VO_REQUIRE(n >= 0, VO_ERR_ARG, "vo_sift_detect_and_compute: more than %d keypoints in one image", cap);
    VO_REQUIRE(n <= capacity, VO_ERR_ARG, "vo_sift_detect_and_compute: %d keypoints exceed capacity=%d", n,
               capacity);
    *count = n;
    if (n == 0) return;
    VO_HIP_CHECK(hipMemcpyAsync(kps, dK, (size_t)n * sizeof(vo_sift_keypoint), hipMemcpyDeviceToHost, s));
    VO_HIP_CHECK(hipMemcpyAsync(desc, dD, (size_t)n * 128 * sizeof(float), hipMemcpyDeviceToHost, s));
    VO_HIP_CHECK(hipStreamSynchronize(s));
  });
}

int vo_sift_detect_and_compute_dev(vo_ctx* ctx, const uint8_t* img, int h, int w, int nfeatures, double contrast,
                                   double edge, double sigma, int n_layers, int capacity, vo_sift_keypoint* d_kps,
                                   float* d_desc, int32_t* count) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(img && d_kps && d_desc && count && capacity >= 1 && h >= 1 && w >= 1, VO_ERR_ARG,
               "vo_sift_detect_and_compute_dev: bad arguments");
    // the caller's buffers: device memory of this runtime on the context's GPU, capacity entries each
    vo::check_device_range(ctx, d_kps, (size_t)capacity * sizeof(vo_sift_keypoint), "kps");
    vo::check_device_range(ctx, d_desc, (size_t)capacity * 128 * sizeof(float), "desc");
    vo::SiftWorkspace& ws = ctx->sift;
    const size_t nimg = (size_t)h * w;
    ws.img.reserve(nimg);
    hipStream_t s = ctx->stream;
    VO_HIP_CHECK(hipMemcpyAsync(ws.img.ptr, img, nimg, hipMemcpyHostToDevice, s));
    // the working capacity and its retries as vo_sift_detect_and_compute's
    // (before retainBest the oriented keypoints outnumber the output many times: the working
    // capacity starts at 32768, as the host entry's default buffers do)
    int cap = std::min(std::max(capacity, 1 << 15), vo::sift_max_capacity()), n = -1;
    vo_sift_keypoint* dK = nullptr;
    float* dD = nullptr;
    for (;;) {
      ws.out.reserve((size_t)cap * (sizeof(vo_sift_keypoint) + 128 * sizeof(float)) + 64);
      dK = ws.out.as<vo_sift_keypoint>();
      dD = reinterpret_cast<float*>(dK + cap);
      int32_t* dC = reinterpret_cast<int32_t*>(dD + (size_t)cap * 128);
      sift_full(ctx, ws.img.as<uint8_t>(), 1, h, w, nfeatures, contrast, edge, sigma, n_layers, cap, dK, dD, dC);
      VO_HIP_CHECK(hipMemcpyAsync(&n, dC, 4, hipMemcpyDeviceToHost, s));
      VO_HIP_CHECK(hipStreamSynchronize(s));
      if (n >= 0 || cap >= vo::sift_max_capacity()) break;
      cap = (int)std::min<int64_t>(std::max<int64_t>(-(int64_t)n, 2ll * cap), vo::sift_max_capacity());
    }
    VO_REQUIRE(n >= 0, VO_ERR_ARG, "vo_sift_detect_and_compute_dev: more than %d keypoints in one image", cap);
    VO_REQUIRE(n <= capacity, VO_ERR_ARG, "vo_sift_detect_and_compute_dev: %d keypoints exceed capacity=%d", n,
               capacity);
    *count = n;
    if (n == 0) return;
    VO_HIP_CHECK(hipMemcpyAsync(d_kps, dK, (size_t)n * sizeof(vo_sift_keypoint), hipMemcpyDeviceToDevice, s));
    VO_HIP_CHECK(hipMemcpyAsync(d_desc, dD, (size_t)n * 128 * sizeof(float), hipMemcpyDeviceToDevice, s));
    VO_HIP_CHECK(hipStreamSynchronize(s));
  });
}

int vo_sift_detect_and_compute_batch_async(vo_ctx* ctx, const uint8_t* d_imgs, int batch, int h, int w,
                                           int nfeatures, double contrast, double edge, double sigma,
                                           int n_layers, int capacity, vo_sift_keypoint* d_kps, float* d_desc,
                                           int32_t* d_counts) {
  return guarded([&] {
    vo::bind(ctx);
    sift_full(ctx, d_imgs, batch, h, w, nfeatures, contrast, edge, sigma, n_layers, capacity, d_kps, d_desc,
              d_counts);
  });
}

int vo_sift_layout(int h, int w, int n_layers, int64_t* out, int n) {
  int rc = 0;
  const int st = guarded([&] {
    VO_REQUIRE(h >= 1 && w >= 1 && n_layers >= 1 && out && n >= 0, VO_ERR_ARG, "vo_sift_layout: bad arguments");
    rc = vo::sift_layout(h, w, n_layers, out, n);
  });
  return st == VO_OK ? rc : st;
}

int vo_pnp_subsets(int count, int iterations, int32_t* out) {
  return guarded([&] {
    VO_REQUIRE(count > 5 && iterations >= 0 && out, VO_ERR_ARG, "vo_pnp_subsets: need count > 5");
    vo::pnp_subsets(count, iterations, out);
  });
}

int vo_match_batch_async(vo_ctx* ctx, const float* d_des0, const float* d_des1, int batch,
                         int n0, int n1, int dim, double ratio, int32_t* d_best) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(d_best && (n0 == 0 || d_des0) && (n1 == 0 || d_des1), VO_ERR_ARG,
               "vo_match_batch_async: null pointers");
    vo::match_run(ctx, d_des0, d_des1, batch, n0, n1, dim, ratio, d_best, nullptr, nullptr);
  });
}

int vo_match_hint(vo_ctx* ctx, int kind) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(kind == VO_DESC_AUTO || kind == VO_DESC_SIFT || kind == VO_DESC_FLOAT, VO_ERR_ARG,
               "vo_match_hint: unknown kind %d", kind);
    ctx->match.kind_hint = kind;
  });
}

int vo_ba_setup(vo_ctx* ctx, const vo_ba_problem* prob, uint64_t* session_out) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(session_out, VO_ERR_ARG, "vo_ba_setup: null session_out");
    *session_out = 0;
    *session_out = vo::ba_setup(ctx, prob);
  });
}

int vo_ba_reserve(vo_ctx* ctx, int n_poses, int n_points, int64_t n_obs, int n_fixed) {
  return guarded([&] {
    vo::bind(ctx);
    vo::ba_reserve(ctx, n_poses, n_points, n_obs, n_fixed);
  });
}

int vo_ba_set_state(vo_ctx* ctx, uint64_t session, const double* poses, const double* points) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(poses && points, VO_ERR_ARG, "vo_ba_set_state: null arrays");
    vo::ba_check_session(ctx, session);
    vo::ba_set_state(ctx, poses, points);
  });
}

int vo_ba_get_state(vo_ctx* ctx, uint64_t session, double* poses, double* points) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(poses && points, VO_ERR_ARG, "vo_ba_get_state: null arrays");
    vo::ba_check_session(ctx, session);
    vo::ba_get_state(ctx, poses, points);
  });
}

int vo_ba_run(vo_ctx* ctx, uint64_t session, int iters, double* cost_out) {
  int rc = VO_OK;
  int g = guarded([&] {
    vo::bind(ctx);
    vo::ba_check_session(ctx, session);
    rc = vo::ba_run(ctx, iters, cost_out, true);
  });
  return g != VO_OK ? g : rc;
}

int vo_ba_run_async(vo_ctx* ctx, uint64_t session, int iters) {
  return guarded([&] {
    vo::bind(ctx);
    vo::ba_check_session(ctx, session);
    vo::ba_run(ctx, iters, nullptr, false);
  });
}

int vo_ba_gn_step(vo_ctx* ctx, uint64_t session, double* S_out, double* b_out, double* dc_out,
                  double* cost_out) {
  int rc = VO_OK;
  int g = guarded([&] {
    vo::bind(ctx);
    vo::ba_check_session(ctx, session);
    rc = vo::ba_gn_step(ctx, S_out, b_out, dc_out, cost_out);
  });
  return g != VO_OK ? g : rc;
}

int vo_ba_solve(vo_ctx* ctx, const vo_ba_problem* prob, double* poses, double* points, int iters,
                double* cost_out) {
  uint64_t s = 0;
  int rc = vo_ba_setup(ctx, prob, &s);
  if (rc) return rc;
  rc = vo_ba_set_state(ctx, s, poses, points);
  if (rc) return rc;
  const int run_rc = vo_ba_run(ctx, s, iters, cost_out);
  if (run_rc && run_rc != VO_ERR_NOT_SPD) return run_rc;
  rc = vo_ba_get_state(ctx, s, poses, points);
  return rc ? rc : run_rc;
}

int vo_ba_plan_stats(vo_ctx* ctx, int64_t* out, int n) {
  int k = 0;
  int g = guarded([&] {
    vo::bind(ctx);
    k = vo::ba_stats(ctx, out, n);
  });
  return g != VO_OK ? g : k;
}

int vo_profile_enable(vo_ctx* ctx, int on) {
  return guarded([&] {
    vo::bind(ctx);
    VO_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    ctx->prof.on = on != 0;
    ctx->prof.recs.clear();
    ctx->prof.used = 0;
  });
}

int vo_profile_read(vo_ctx* ctx, double* ms_out, int64_t* counts_out) {
  return guarded([&] {
    vo::bind(ctx);
    VO_REQUIRE(ms_out && counts_out, VO_ERR_ARG, "vo_profile_read: null outputs");
    VO_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    ctx->prof.read(ms_out, counts_out);
  });
}

int vo_ba_debug_stamps(vo_ctx* ctx, uint64_t* out, int n) {
  int k = 0;
  int g = guarded([&] {
    vo::bind(ctx);
    k = vo::ba_stamps(ctx, out, n);
  });
  return g != VO_OK ? g : k;
}

int vo_ba_plan_digest(const vo_ba_problem* prob, int target_segments, uint64_t* digest) {
  return guarded([&] {
    VO_REQUIRE(prob && digest, VO_ERR_ARG, "vo_ba_plan_digest: null argument");
    std::vector<int32_t> zero(1, 0);
    vo::BAPlan P;
    std::string err = vo::build_plan(P, prob->n_poses, prob->n_points, prob->n_obs, prob->n_fixed,
                                     prob->n_points ? prob->point_ptr : zero.data(), prob->obs_cam,
                                     prob->obs_uv, vo::seg_obs_for(prob->n_obs, target_segments));
    VO_REQUIRE(err.empty(), VO_ERR_ARG, "vo_ba_plan_digest: %s", err.c_str());
    vo::build_profile(P, vo::local_profile_first(P));
    *digest = vo::plan_digest(P);
  });
}

int vo_ba_testing_plan_slide(const vo_ba_problem* prev, const vo_ba_problem* cur, int seg_obs, int seg_chunks,
                             uint64_t* digest, int64_t* reused_chunks) {
  return guarded([&] {
    VO_REQUIRE(cur && digest && seg_obs >= 1, VO_ERR_ARG, "vo_ba_testing_plan_slide: bad argument");
    std::vector<int32_t> zero(1, 0);
    vo::BAPlan A, B;
    auto build = [&](vo::BAPlan& P, const vo_ba_problem* p, const vo::BAPlan* from) {
      std::string err = vo::build_plan(P, p->n_poses, p->n_points, p->n_obs, p->n_fixed,
                                       p->n_points ? p->point_ptr : zero.data(), p->obs_cam, p->obs_uv, seg_obs, from,
                                       seg_chunks);
      VO_REQUIRE(err.empty(), VO_ERR_ARG, "vo_ba_testing_plan_slide: %s", err.c_str());
      vo::build_profile(P, vo::local_profile_first(P));
    };
    if (prev) build(A, prev, nullptr);
    build(B, cur, prev ? &A : nullptr);
    *digest = vo::plan_digest(B);
    if (reused_chunks) *reused_chunks = B.reused_chunks;
  });
}

int vo_ba_group_by_point(int n_points, int n_obs, const int32_t* obs_pt, int32_t* order, int32_t* point_ptr) {
  int grouped = 1;
  const int rc = guarded([&] {
    VO_REQUIRE(n_points >= 0 && n_obs >= 0, VO_ERR_ARG, "vo_ba_group_by_point: bad sizes");
    VO_REQUIRE(point_ptr && (n_obs == 0 || obs_pt), VO_ERR_ARG, "vo_ba_group_by_point: null argument");
    if (!order) {  // already grouped (nondecreasing obs_pt)?  then only point_ptr
      const int32_t* __restrict op = obs_pt;
      int32_t* __restrict pp = point_ptr;
      unsigned descending = 0;  // branch-free scan
      for (int o = 1; o < n_obs; ++o) descending |= op[o] < op[o - 1];
      // nondecreasing: in range iff the ends are; otherwise every entry is checked
      unsigned out_of_range = n_obs > 0 && ((unsigned)op[0] >= (unsigned)n_points ||
                                            (unsigned)op[n_obs - 1] >= (unsigned)n_points);
      if (descending)
        for (int o = 0; o < n_obs; ++o) out_of_range |= (unsigned)op[o] >= (unsigned)n_points;
      if (out_of_range) {
        int o = 0;
        while ((unsigned)op[o] < (unsigned)n_points) ++o;
        VO_REQUIRE(false, VO_ERR_ARG, "vo_ba_group_by_point: obs_pt[%d]=%d out of range", o, op[o]);
      }
      if (descending) {
        grouped = 0;
        return;
      }
      // grouped: landmark p's run starts at its first observation, or (none) where the next
      // landmark's does.  Branch-free, and no per-observation read-modify-write: the first
      // observations stored from the back, then a running minimum from the last landmark.
      std::fill(pp, pp + n_points + 1, n_obs);
      for (int o = n_obs - 1; o >= 0; --o) pp[op[o]] = o;
      int run = n_obs;
      for (int p = n_points - 1; p >= 0; --p) {
        run = std::min(run, pp[p]);
        pp[p] = run;
      }
      return;
    }
    std::fill(point_ptr, point_ptr + n_points + 1, 0);
    for (int o = 0; o < n_obs; ++o) {
      VO_REQUIRE(obs_pt[o] >= 0 && obs_pt[o] < n_points, VO_ERR_ARG, "vo_ba_group_by_point: obs_pt[%d]=%d out of range",
                 o, obs_pt[o]);
      ++point_ptr[obs_pt[o] + 1];
    }
    for (int p = 0; p < n_points; ++p) point_ptr[p + 1] += point_ptr[p];
    std::vector<int32_t> next(point_ptr, point_ptr + std::max(n_points, 1));
    for (int o = 0; o < n_obs; ++o) order[next[obs_pt[o]]++] = o;  // stable: caller order within a landmark
  });
  return rc == VO_OK && !grouped ? 1 : rc;
}

int vo_ba_plan_probe(const vo_ba_problem* prob, int target_segments, int64_t* out, int n) {
  int k = 0;
  int g = guarded([&] {
    VO_REQUIRE(prob && out, VO_ERR_ARG, "vo_ba_plan_probe: null argument");
    std::vector<int32_t> zero(1, 0);
    vo::BAPlan P;
    std::string err = vo::build_plan(P, prob->n_poses, prob->n_points, prob->n_obs, prob->n_fixed,
                                     prob->n_points ? prob->point_ptr : zero.data(), prob->obs_cam,
                                     prob->obs_uv, vo::seg_obs_for(prob->n_obs, target_segments));
    VO_REQUIRE(err.empty(), VO_ERR_ARG, "vo_ba_plan_probe: %s", err.c_str());
    vo::build_profile(P, vo::local_profile_first(P));
    int64_t max_pairs = 0, max_slots = 0, max_cams = 0;
    for (int c = 0, s = 0; c < P.n_chunks(); ++c) {
      while (s + 1 < P.n_segments() + 1 && P.seg_chunk[s + 1] <= c) ++s;
      const int ns = P.seg_slot_off[s + 1] - P.seg_slot_off[s];
      const int b = P.chunk_slot_base[c];
      max_pairs = std::max<int64_t>(max_pairs, P.slot_ptr[b + ns] - P.slot_ptr[b]);
    }
    for (int s = 0; s < P.n_segments(); ++s) {
      max_slots = std::max<int64_t>(max_slots, P.seg_slot_off[s + 1] - P.seg_slot_off[s]);
      max_cams = std::max<int64_t>(max_cams, P.seg_cam_off[s + 1] - P.seg_cam_off[s]);
    }
    int span = 0;
    for (int r = 0; r < P.n_free; ++r) span = std::max(span, r - P.prof_first[r]);
    std::vector<int> first(P.prof_first.begin(), P.prof_first.end());
    const vo::BandSplit T = vo::band_split(P.n_free, first);
    const int64_t v[14] = {P.n_chunks(), P.n_segments(), P.n_slab_slots(), P.n_prof_blocks(),
                           P.n_te, max_pairs, max_slots, max_cams, P.n_free, span,
                           vo::band_supported(P.n_free, T.w, P.n_poses) ? 1 : 0, T.m, T.s, T.nb};
    k = std::min(n, 14);
    for (int i = 0; i < k; ++i) out[i] = v[i];
  });
  return g != VO_OK ? g : k;
}

int vo_comm_unique_id(char out[128]) {
  return guarded([&] { vo::comm_unique_id(out); });
}

int vo_comm_init(vo_ctx* ctx, int nranks, int rank, const char id[128]) {
  return guarded([&] {
    vo::bind(ctx);
    vo::comm_init(ctx, nranks, rank, id);
  });
}

// test-only (include/vo_hip_testing.h)
int vo_ba_split_reduce(vo_ctx* ctx, int on) {
  return guarded([&] {
    VO_REQUIRE(ctx != nullptr, VO_ERR_ARG, "vo_ba_split_reduce: null context");
    ctx->ba_split_reduce = on != 0;
  });
}

int vo_ba_testing_drop_reducers(vo_ctx* ctx, int n) {
  return guarded([&] {
    VO_REQUIRE(ctx != nullptr, VO_ERR_ARG, "vo_ba_testing_drop_reducers: null context");
    VO_REQUIRE(n >= 0, VO_ERR_ARG, "vo_ba_testing_drop_reducers: n < 0");
    ctx->ba_drop_reducers = n;
  });
}

int vo_ba_testing_no_split(vo_ctx* ctx, int on) {
  return guarded([&] {
    VO_REQUIRE(ctx != nullptr, VO_ERR_ARG, "vo_ba_testing_no_split: null context");
    ctx->ba_no_split = on != 0;
  });
}

int vo_ba_testing_k1(vo_ctx* ctx, int variant) {
  return guarded([&] {
    VO_REQUIRE(ctx != nullptr, VO_ERR_ARG, "vo_ba_testing_k1: null context");
    VO_REQUIRE(variant >= -1 && variant <= vo::kWaveMaxChunks, VO_ERR_ARG, "vo_ba_testing_k1: variant %d outside -1..%d",
               variant, vo::kWaveMaxChunks);
    ctx->ba_k1_variant = variant;
  });
}

int vo_pnp_testing_group(vo_ctx* ctx, int mode) {
  return guarded([&] {
    VO_REQUIRE(ctx != nullptr, VO_ERR_ARG, "vo_pnp_testing_group: null context");
    VO_REQUIRE(mode >= -1 && mode <= 1, VO_ERR_ARG, "vo_pnp_testing_group: mode %d outside -1..1", mode);
    ctx->pnp_group = mode;
  });
}

int vo_pnp_testing_split(vo_ctx* ctx, int h1) {
  return guarded([&] {
    VO_REQUIRE(ctx != nullptr, VO_ERR_ARG, "vo_pnp_testing_split: null context");
    VO_REQUIRE(h1 >= -1, VO_ERR_ARG, "vo_pnp_testing_split: h1 %d < -1", h1);
    ctx->pnp_split = h1;
  });
}

int vo_pnp_testing_last_split(vo_ctx* ctx, int* h1, int* tail_frames) {
  return guarded([&] {
    VO_REQUIRE(ctx != nullptr && h1 && tail_frames, VO_ERR_ARG, "vo_pnp_testing_last_split: bad arguments");
    vo::bind(ctx);
    vo::PnpWorkspace& ws = ctx->pnp;
    const int batch = (int)ws.offsets.size() - 1;
    *h1 = ws.last_h1;
    *tail_frames = 0;
    if (batch <= 0 || ws.last_h1 >= ws.H) return;
    std::vector<int32_t> need(batch);
    VO_HIP_CHECK(hipMemcpyAsync(need.data(), ws.need.ptr, sizeof(int32_t) * batch, hipMemcpyDeviceToHost, ctx->stream));
    VO_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    for (int v : need) *tail_frames += v != 0;
  });
}

int vo_comm_init_loopback(vo_ctx* ctx, int nranks, int rank, const char id[128]) {
  return guarded([&] {
    vo::bind(ctx);
    vo::comm_init_loopback(ctx, nranks, rank, id);
  });
}

}  // extern "C"
