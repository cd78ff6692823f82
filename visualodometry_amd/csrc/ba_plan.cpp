// Host-side static planner for the BA Gauss-Newton step (see ba_plan.h).
#include "ba_plan.h"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <stdexcept>
#include <functional>
#include <mutex>
#include <thread>

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <numeric>

namespace vo {

namespace {

std::string fmt(const char* f, long a = 0, long b = 0, long c = 0) {
  char buf[256];
  std::snprintf(buf, sizeof buf, f, a, b, c);
  return buf;
}


}  // namespace

int64_t BAPlan::algorithmic_bytes_per_iter() const {
  // obs (uv f32x2 + two i32) read by linearise and back-substitute,
  // points read twice + written once + CSR offset, poses read and written,
  // S written and read by the solve, rhs written and read.
  const int64_t F6 = 6ll * n_free;
  return 2ll * n_obs * 16 + (int64_t)n_points * (2 * 24 + 24 + 4) + (int64_t)n_poses * 2 * 96 +
         2 * F6 * F6 * 8 + F6 * 8 * 2;
}

namespace {

// Host threads the planner may use: the CPU affinity, capped by a cgroup v2 CPU quota (a
// GPU box's container sees every CPU of the machine but is granted a share of them) and by
// kPlanMaxThreads.  The plan itself never depends on it.
#ifndef VO_PLAN_MAX_THREADS
#define VO_PLAN_MAX_THREADS 16
#endif
constexpr int kPlanMaxThreads = VO_PLAN_MAX_THREADS;
int host_threads() {
  static const int n = [] {
    long c = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) c = std::max(1, CPU_COUNT(&set));
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char quota[32] = {0};
      long period = 0;
      if (std::fscanf(f, "%31s %ld", quota, &period) == 2 && std::strcmp(quota, "max") != 0 && period > 0)
        c = std::min(c, std::max(1L, (std::atol(quota) + period - 1) / period));
      std::fclose(f);
    }
    return (int)std::min<long>(c, kPlanMaxThreads);
  }();
  return n;
}

// fn(t) for t = 0 .. n - 1, each exactly once, on the caller and the pool's workers.  The items
// are claimed from a counter, so a phase ends when its items are done, not when every worker has
// arrived: a worker that wakes late finds them taken (the first phase of a plan follows a futex
// wake of every worker, and on a loaded host the slowest wake had set that phase's length).
// Every use writes disjoint, precomputed ranges per item, so the plan never depends on the
// thread count or timing.  Workers persist across plans (thread creation would cost more than a
// small phase); a caller that finds the pool busy (another context planning) starts its own
// threads.  While a plan is being built (PlanSession, one build_plan call: about half a
// millisecond of consecutive phases tens of microseconds apart), the workers poll for the next
// phase instead of sleeping on the condition variable; between plans they sleep (polling there
// would eat the job's CPU quota).  Tuning build: -DVO_PLAN_SESSION_SPIN=0 never polls.
#ifndef VO_PLAN_SESSION_SPIN
#define VO_PLAN_SESSION_SPIN 1
#endif
constexpr bool kPlanSessionSpin = VO_PLAN_SESSION_SPIN != 0;


inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#endif
}
// Every spin is bounded: past kSpinYield pauses (tens of microseconds) a waiting caller yields its
// core on each further check, and a polling worker goes back to its condition variable.  With
// several ranks per node each sizing its pool to the cgroup quota, an unbounded spinner could hold
// a core that a throttled or preempted worker needs to finish the item the spinner waits for.
constexpr long kSpinYield = 1L << 14;
inline void spin_wait(long& spins) {
  if (++spins < kSpinYield) cpu_relax();
  else std::this_thread::yield();
}

class PlanPool {
 public:
  static PlanPool& get() {
    static PlanPool pool;
    return pool;
  }
  // Exceptions (bad_alloc in a phase) never escape a thread: each item is caught, the first
  // exception is kept, every item still runs, then the caller rethrows it (guarded() maps it to
  // an error code).
  template <class Fn>
  void run(int n, Fn&& fn) {
    std::exception_ptr first;
    std::mutex emu;
    auto safe = [&](int t) {
      try {
        fn(t);
      } catch (...) {
        std::lock_guard<std::mutex> lk(emu);
        if (!first) first = std::current_exception();
      }
    };
    // a forked child inherits the pool object but not its threads: it plans on its own
    std::unique_lock<std::mutex> busy(use_, std::defer_lock);
    if (getpid() != owner_ || !busy.try_lock()) {
      std::vector<std::thread> pool;
      try {
        for (int t = 1; t < n; ++t) pool.emplace_back([&safe, t] { safe(t); });
      } catch (...) {  // thread creation failed: the rest of the phase on this thread
        for (int t = (int)pool.size() + 1; t < n; ++t) safe(t);
      }
      safe(0);
      for (auto& th : pool) th.join();
      if (first) std::rethrow_exception(first);
      return;
    }
    std::function<void(int)> job = [&safe](int t) { safe(t); };
    // publish: the job's fields are written while the pool is retired (a worker that enters now
    // backs off without reading them), then opened with a new generation
    job_ = &job;
    n_items_ = n;
    next_.store(0, std::memory_order_relaxed);
    ndone_.store(0, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(mu_);
      retired_.store(false, std::memory_order_seq_cst);
      gen_.fetch_add(1, std::memory_order_seq_cst);
    }
    cv_.notify_all();  // (cheap when every worker is polling: no waiter to wake)
    work();
    long spins = 0;
    while (ndone_.load(std::memory_order_acquire) < n) spin_wait(spins);
    // retire: workers inside the job finish their (claimed-nothing) loop; later ones back off
    retired_.store(true, std::memory_order_seq_cst);
    spins = 0;
    while (entered_.load(std::memory_order_seq_cst) != 0) spin_wait(spins);
    job_ = nullptr;
    if (first) std::rethrow_exception(first);
  }
  // a plan is being built: workers poll between its phases (see kPlanSessionSpin).  (Waking
  // them at the start of vo_ba_setup, before the plan, measured slower: 0.66 -> 0.83 ms per
  // cfg3 setup, the polling threads competing with the setup thread.)
  void begin_session() {
    if (kPlanSessionSpin) session_.fetch_add(1, std::memory_order_acq_rel);
  }
  void end_session() {
    if (kPlanSessionSpin) session_.fetch_sub(1, std::memory_order_acq_rel);
  }
  ~PlanPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& th : workers_) th.join();
  }

 private:
  PlanPool() : owner_(getpid()) {
    for (int t = 1; t < host_threads(); ++t) workers_.emplace_back([this] { loop(); });
  }
  // items of the current job until none is left (the caller, and workers that entered it)
  void work() {
    for (;;) {
      const int t = next_.fetch_add(1, std::memory_order_relaxed);
      if (t >= n_items_) return;
      (*job_)(t);
      ndone_.fetch_add(1, std::memory_order_release);
    }
  }
  void loop() {
    long seen = 0;
    for (;;) {
      // poll while a plan is being built, for at most kSpinYield pauses, then sleep
      for (long spins = 0; spins < kSpinYield && session_.load(std::memory_order_acquire) > 0 &&
                           gen_.load(std::memory_order_acquire) == seen;
           ++spins)
        cpu_relax();
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_.load(std::memory_order_relaxed) != seen; });
        if (stop_) return;
        seen = gen_.load(std::memory_order_relaxed);
      }
      entered_.fetch_add(1, std::memory_order_seq_cst);
      if (!retired_.load(std::memory_order_seq_cst)) work();
      entered_.fetch_sub(1, std::memory_order_seq_cst);
    }
  }
  pid_t owner_;
  std::vector<std::thread> workers_;
  std::mutex use_, mu_;
  std::condition_variable cv_;
  // the current job: written only while retired_ is true and no worker is inside it
  std::function<void(int)>* job_ = nullptr;
  int n_items_ = 0;
  std::atomic<int> next_{0}, ndone_{0}, entered_{0};
  std::atomic<bool> retired_{true};
  std::atomic<long> gen_{0};
  std::atomic<int> session_{0};  // plans being built (begin_session / end_session)
  bool stop_ = false;
};

// The polling window of one build_plan call (plans of one thread start no session).
struct PlanSession {
  bool on;
  explicit PlanSession(bool multi) : on(multi) {
    if (on) PlanPool::get().begin_session();
  }
  ~PlanSession() {
    if (on) PlanPool::get().end_session();
  }
  PlanSession(const PlanSession&) = delete;
  PlanSession& operator=(const PlanSession&) = delete;
};

template <class Fn>
void run_parallel(int n, Fn&& fn) {
  if (n <= 1) return fn(0);
  PlanPool::get().run(n, fn);
}

// Plan arrays grow with a quarter of headroom: consecutive keyframe windows differ by a few
// landmarks, and an exact-size reallocation (fresh pages to fault in; for the page-locked chunk
// images a hipHostMalloc) on most calls cost more than the phase that fills the array.
template <class V>
void fit(V& v, size_t n) {
  if (v.capacity() >= n) return;
  v.clear();
  v.reserve(n + n / 4 + 64);
}
template <class V>
void sized(V& v, size_t n) {
  fit(v, n);
  v.resize(n);
}
template <class V, class T>
void filled(V& v, size_t n, const T& x) {
  fit(v, n);
  v.assign(n, x);
}

int plan_threads(int64_t work) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), work / 2048 + 1));
}

}  // namespace

// A vector of at most N trivially copyable elements stored inline (a segment's windows are
// bounded by kSegCams / kSegAllCams / kSegSlots, checked before anything is added): no heap
// allocation per segment, so a plan frees nothing per segment either.
template <class T, int N>
struct FixVec {
  T v[N];
  int n = 0;
  int size() const { return n; }
  bool empty() const { return n == 0; }
  void clear() { n = 0; }
  void push_back(const T& x) {
    if (n >= N) throw std::length_error("plan: segment window overflow");
    v[n++] = x;
  }
  T& operator[](int i) { return v[i]; }
  const T& operator[](int i) const { return v[i]; }
  T* begin() { return v; }
  T* end() { return v + n; }
  const T* begin() const { return v; }
  const T* end() const { return v + n; }
};

template <class V, class X>
int find_or_neg(const V& v, const X& x) {
  for (int i = 0; i < (int)v.size(); ++i)
    if (v[i] == x) return i;
  return -1;
}

struct PlanSeg {
  int chunk0 = 0;                           // first chunk (global index after the merge)
  int src = -1;                             // taken over: the previous plan's segment
  FixVec<int32_t, kSegCams> cams;           // free cameras (unsorted while growing)
  FixVec<int32_t, kSegAllCams> acams;       // all cameras its observations see
  FixVec<std::pair<int32_t, int32_t>, kSegSlots> slots;
  FixVec<int32_t, kSegSlots> slot_cnt;      // pairs per slot (while packing)
  PlanSeg() = default;
  PlanSeg(int c0, int s) : chunk0(c0), src(s) {}
};

// one first-camera group's greedy packing: chunks (first landmark, pair count, free track
// entries, free observations) and segments (first chunk, local index); a group taken over
// from the previous plan (src >= 0) copies them from there
struct PlanPart {
  std::vector<int32_t> chunk_q, chunk_pairs, chunk_fte, chunk_fobs;
  std::vector<PlanSeg> segs;
  int src = -1, shift = 0;
  int err_q = -1;
  std::string err;
  void reset() {  // empty, capacity kept (the plan's next window reuses it)
    chunk_q.clear();
    chunk_pairs.clear();
    chunk_fte.clear();
    chunk_fobs.clear();
    segs.clear();
    src = -1;
    shift = 0;
    err_q = -1;
    err.clear();
  }
};

// The planner's working containers, kept across the plans of one BAPlan (ba_plan.h).
struct PlanScratch {
  std::vector<PlanPart> parts;
  std::vector<PlanSeg*> segp;  // the plan's segments in order (into parts[].segs)
  std::vector<int32_t> first, tecnt, hist, seg_of, pair_base, cl_base, col_base, ch_pairs, ch_fte, ch_fobs;
};

// One-wave K1: weighted chain below which a slot's pairs stay on one lane (copies split longer
// ones).  15 with three-chunk segments (same-box A/B, profiles/r05_ab/copy_chain*.txt: K1 cfg3
// 24.69 -> 24.51 us, cfg4 158.5 -> 155.8 us against 21; 9, 12 and 30 slower).
#ifndef VO_BA_COPY_CHAIN
#define VO_BA_COPY_CHAIN 15
#endif
constexpr int kCopyChain = VO_BA_COPY_CHAIN;

int seg_obs_for(int64_t n_obs, int target_segments) {
  const int64_t t = std::max(1, target_segments);
  return (int)std::max<int64_t>(1, std::min<int64_t>((n_obs + t - 1) / t, 1 << 30));
}

int seg_obs_grid(int64_t x) {
  if (x <= 1) return 1;
  double g = 1.0;
  while (std::ceil(g) < (double)x && g < (double)(1 << 30)) g *= 1.0905077326652577;  // 2^(1/8)
  return (int)std::min<double>(std::ceil(g), 1 << 30);
}

void BAPlan::reset() {
  n_poses = n_points = n_obs = n_fixed = n_free = n_te = 0;
  seg_obs = seg_chunks = reused_groups = reused_chunks = 0;
  host_images_partial = false;
  group_q.clear();
  group_chunk.clear();
  group_seg.clear();
  chunk_src.clear();
  for (auto* v : {&pt_perm, &obs_cam, &obs_te, &te_cam, &te_pt, &te_obs, &pt_te, &slot_ptr, &cam_ptr, &camo_ptr,
                  &slot_i, &slot_j, &segcam_f, &segcam_diag})
    v->clear();
  for (auto* v : {&chunk_obs, &chunk_te, &chunk_pt, &chunk_slot_base, &chunk_cam_base, &chunk_hdr, &slab_pos,
                  &cam_pos, &seg_hdr, &seg_chunk, &seg_slot_off, &seg_cam_off, &seg_acam_off, &seg_acam,
                  &prof_first, &prof_off, &prof_last, &prof_src_ptr, &prof_src, &camb_ptr, &camb_src, &solve_tab})
    v->clear();
  obs_uv.clear();
  te_lcam.clear();
  chunk_img.clear();
  pair_list.clear();
  cam_list.clear();
  camo_list.clear();
  obs_acam.clear();
  prof_diag.clear();
  solve_layout = SolveTableLayout();
}

std::string build_plan(BAPlan& P, int N, int L, int M, int n_fixed, const int32_t* point_ptr,
                       const int32_t* obs_cam, const float* obs_uv, int seg_obs, const BAPlan* prev,
                       int seg_chunks) {
  P.reset();
  if (N < 1 || L < 0 || M < 0) return fmt("bad sizes n_poses=%ld n_points=%ld n_obs=%ld", N, L, M);
  if (N > 32767) return fmt("n_poses=%ld exceeds the 32767 camera ids of a segment header", N);
  if (n_fixed < 0 || n_fixed > N) return fmt("bad n_fixed=%ld (n_poses=%ld)", n_fixed, N);
  if (point_ptr[0] != 0 || point_ptr[L] != M) return "point_ptr must start at 0 and end at n_obs";
  // point_ptr monotone and obs_cam in range: checked by the first parallel pass below

  P.n_poses = N;
  P.n_points = L;
  P.n_obs = M;
  P.n_fixed = n_fixed;
  P.n_free = N - n_fixed;
  P.seg_obs = std::max(1, seg_obs);
  const bool wave = plan_is_wave(P.seg_obs);  // the one-wave K1's images
  if (wave && (seg_chunks < 1 || seg_chunks > kWaveMaxChunks))
    return fmt("seg_chunks=%ld outside 1..%ld", seg_chunks, kWaveMaxChunks);
  P.seg_chunks = wave ? seg_chunks : 0;
  // wave plans of several chunks per segment: segments padded to seg_chunks chunks, and a
  // window of at most kWaveItems slots (every chunk's blocks fit the combine's scratch rows)
  const int group_nch = wave && seg_chunks > 1 ? seg_chunks : 0;
  const int max_slots = group_nch || (wave && kWaveSlots < kSegSlots) ? kWaveItems : kSegSlots;
  const int nthr = plan_threads(M);
  PlanSession session(nthr > 1);
  if (!P.scratch) P.scratch = std::make_shared<PlanScratch>();
  PlanScratch& X = *P.scratch;

#ifdef VO_PLAN_TIMING  // diagnostic builds: the order pass's own steps
  auto sub_t0 = std::chrono::steady_clock::now();
  auto sub = [&](const char* name) {
    const auto n = std::chrono::steady_clock::now();
    std::fprintf(stderr, "    %-12s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(n - sub_t0).count());
    sub_t0 = n;
  };
#else
  auto sub = [](const char*) {};
#endif
  PlanArr<int32_t>& sorted = P.scr_sorted;
  sized(sorted, std::max(M, 1));
  // Landmarks ordered by first camera (stable counting sort; no observation: last), which
  // keeps each workgroup's camera window narrow, and their observations grouped by (landmark,
  // camera) into track entries.  Pass 1 over landmark ranges: the checks, each landmark's first
  // camera and track-entry count, and per (range, camera) the landmarks, observations and track
  // entries; offsets in (camera, range) order; pass 2 over the same ranges: each landmark takes
  // its internal index and its observation and track-entry slots from its bucket's running
  // offsets, sorts its observations by camera (stable) into them and writes every array.
  {
    std::vector<int32_t>&first = X.first, &tecnt = X.tecnt, &hist = X.hist;
    sized(first, L);
    sized(tecnt, L);
    const int nt = std::max(1, std::min(nthr, L / 1024 + 1));
    const size_t nb = (size_t)nt * (N + 1);
    filled(hist, 3 * nb, 0);  // landmarks | observations | track entries per (range, camera)
    std::vector<int32_t> bad_ptr(nt, -1), bad_obs(nt, -1);  // first violation of each range
    auto lrange = [&](int t) { return std::make_pair((int)((int64_t)L * t / nt), (int)((int64_t)L * (t + 1) / nt)); };
    run_parallel(nt, [&](int t) {
      const auto [pa, pb] = lrange(t);
      for (int p = pa; p < pb; ++p)
        if (point_ptr[p + 1] < point_ptr[p]) {
          bad_ptr[t] = p;
          return;
        }
      // locally monotone but outside [0, M]: another range is not monotone (reported there)
      if (point_ptr[pa] < 0 || point_ptr[pb] > M) return;
      for (int o = point_ptr[pa]; o < point_ptr[pb]; ++o)
        if (obs_cam[o] < 0 || obs_cam[o] >= N) {
          bad_obs[t] = o;
          return;
        }
      int32_t* h = &hist[(size_t)t * (N + 1)];
      int32_t* ho = h + nb;
      int32_t* ht = ho + nb;
      for (int p = pa; p < pb; ++p) {
        // first camera and track entries (distinct cameras; tracks are short)
        int f = N, nte = 0;
        const int o0 = point_ptr[p], o1 = point_ptr[p + 1];
        for (int o = o0; o < o1; ++o) {
          const int c = obs_cam[o];
          f = std::min(f, c);
          bool fresh = true;
          for (int u = o0; u < o; ++u) fresh = fresh && obs_cam[u] != c;
          nte += fresh;
        }
        first[p] = f;
        tecnt[p] = nte;
        ++h[f];
        ho[f] += o1 - o0;
        ht[f] += nte;
      }
    });
    sub("pass 1");
    for (int t = 0; t < nt; ++t)  // the lowest violation, as a serial scan would find it
      if (bad_ptr[t] >= 0) return fmt("point_ptr not monotone at %ld", bad_ptr[t]);
    for (int t = 0; t < nt; ++t)
      if (bad_obs[t] >= 0) return fmt("obs_cam[%ld]=%ld out of range", bad_obs[t], obs_cam[bad_obs[t]]);
    int32_t off = 0, ooff = 0, toff = 0;
    sized(P.group_q, N + 2);
    for (int c = 0; c <= N; ++c) {
      P.group_q[c] = off;
      for (int t = 0; t < nt; ++t) {
        int32_t* h = &hist[(size_t)t * (N + 1) + c];
        const int32_t n = h[0], no = h[nb], ne = h[2 * nb];
        h[0] = off;
        h[nb] = ooff;
        h[2 * nb] = toff;
        off += n;
        ooff += no;
        toff += ne;
      }
    }
    P.group_q[N + 1] = off;
    P.n_te = toff;
    sized(P.pt_perm, L);
    sized(P.obs_uv, 2 * (size_t)M);
    sized(P.obs_cam, M);
    sized(P.obs_te, M);
    sized(P.te_cam, P.n_te);
    sized(P.te_pt, P.n_te);
    sized(P.te_obs, P.n_te + 1);
    sized(P.te_lcam, P.n_te);
    sized(P.pt_te, L + 1);
    run_parallel(nt, [&](int t) {
      const auto [pa, pb] = lrange(t);
      int32_t* h = &hist[(size_t)t * (N + 1)];
      int32_t* ho = h + nb;
      int32_t* ht = ho + nb;
      for (int p = pa; p < pb; ++p) {
        const int c = first[p], n = point_ptr[p + 1] - point_ptr[p];
        const int32_t q = h[c]++, ob = ho[c], te0 = ht[c];
        ho[c] += n;
        ht[c] += tecnt[p];
        P.pt_perm[q] = p;
        P.pt_te[q] = te0;
        int32_t* idx = &sorted[ob];
        for (int i = 0; i < n; ++i) {  // stable insertion sort by camera (tracks are short)
          const int32_t v = point_ptr[p] + i;
          int j = i;
          while (j > 0 && obs_cam[idx[j - 1]] > obs_cam[v]) {
            idx[j] = idx[j - 1];
            --j;
          }
          idx[j] = v;
        }
        int te = te0 - 1;
        for (int pos = ob; pos < ob + n; ++pos) {
          const int o = sorted[pos];
          if (pos == ob || obs_cam[o] != obs_cam[sorted[pos - 1]]) {
            ++te;
            P.te_cam[te] = obs_cam[o];
            P.te_pt[te] = q;
            P.te_obs[te] = pos;
            P.te_lcam[te] = -1;  // window camera: set by the packing (free cameras)
          }
          P.obs_uv[2 * (size_t)pos] = obs_uv[2 * (size_t)o];
          P.obs_uv[2 * (size_t)pos + 1] = obs_uv[2 * (size_t)o + 1];
          P.obs_cam[pos] = obs_cam[o];
          P.obs_te[pos] = te;
        }
      }
    });
  }
  sub("pass 2");
  P.pt_te[L] = P.n_te;
  P.te_obs[P.n_te] = M;
  PLAN_T(1, "order + track entries");

  // ---- chunks and segments: each first-camera group packed greedily on its own (so a
  // group's packing depends on its own landmarks only), or taken over from prev
  const int64_t seg_obs_target = P.seg_obs;
  const int Nf = N - n_fixed;
  const bool tables = Nf <= kPlanTableCams;
  const int nparts = N + 1;
  std::vector<PlanPart>& parts = X.parts;
  parts.resize(nparts);
  for (PlanPart& R : parts) R.reset();
  const bool reuse = prev && prev != &P && prev->seg_obs == P.seg_obs && prev->seg_chunks == P.seg_chunks &&
                     prev->n_fixed == n_fixed &&
                     (int)prev->group_q.size() == prev->n_poses + 2;
  // group g equals the previous plan's group g + s: the same landmarks in the same order, their
  // cameras s lower, the same observations (uv bit for bit)
  auto same_group = [&](int g, int src, int s) {
    const BAPlan& Q = *prev;
    const int q0 = P.group_q[g], q1 = P.group_q[g + 1], pq0 = Q.group_q[src], pq1 = Q.group_q[src + 1];
    if (q1 - q0 != pq1 - pq0 || q1 == q0) return false;
    const int t0 = P.pt_te[q0], t1 = P.pt_te[q1], pt0 = Q.pt_te[pq0];
    if (t1 - t0 != Q.pt_te[pq1] - pt0) return false;
    const int o0 = P.te_obs[t0], o1 = P.te_obs[t1], po0 = Q.te_obs[pt0];
    if (o1 - o0 != Q.te_obs[Q.pt_te[pq1]] - po0) return false;
    for (int i = 0; i < q1 - q0; ++i)
      if (P.pt_te[q0 + i] - t0 != Q.pt_te[pq0 + i] - pt0) return false;
    for (int i = 0; i < t1 - t0; ++i)
      if (P.te_cam[t0 + i] + s != Q.te_cam[pt0 + i] || P.te_obs[t0 + i] - o0 != Q.te_obs[pt0 + i] - po0) return false;
    return std::memcmp(&P.obs_uv[2 * (size_t)o0], &Q.obs_uv[2 * (size_t)po0], 8 * (size_t)(o1 - o0)) == 0;
  };
  // the previous plan's packing of group src, moved to group g (cameras s lower)
  auto take_over = [&](PlanPart& R, int g, int src, int s) {
    const BAPlan& Q = *prev;
    R.src = src;
    R.shift = s;
    const int pc0 = Q.group_chunk[src], pc1 = Q.group_chunk[src + 1];
    for (int pc = pc0; pc < pc1; ++pc) {
      const int32_t* h = &Q.chunk_hdr[(size_t)pc * kChunkHdr];
      R.chunk_q.push_back(Q.chunk_pt[pc] - Q.group_q[src] + P.group_q[g]);
      R.chunk_pairs.push_back(h[9] - h[8]);
      R.chunk_fte.push_back(h[11] - h[10]);
      R.chunk_fobs.push_back(h[13] - h[12]);
    }
    for (int ps = Q.group_seg[src]; ps < Q.group_seg[src + 1]; ++ps) {
      R.segs.emplace_back(Q.seg_chunk[ps] - pc0, ps);
      PlanSeg& sg = R.segs.back();
      for (int e = Q.seg_cam_off[ps]; e < Q.seg_cam_off[ps + 1]; ++e) sg.cams.push_back(Q.segcam_f[e] - s);
      for (int e = Q.seg_acam_off[ps]; e < Q.seg_acam_off[ps + 1]; ++e) sg.acams.push_back(Q.seg_acam[e] - s);
      for (int e = Q.seg_slot_off[ps]; e < Q.seg_slot_off[ps + 1]; ++e)
        sg.slots.push_back(std::make_pair(Q.slot_i[e] - s, Q.slot_j[e] - s));
    }
  };
  auto pack = [&](int pi) {
    PlanPart& R = parts[pi];
    const int qa = P.group_q[pi], qb = P.group_q[pi + 1];
    // groups of free cameras only (no camera changes between fixed and free with the shift);
    // the slide (s = 1) first, then the same camera (a growing or repeated window)
    if (reuse && pi >= n_fixed && pi < N)
      for (int s = 1; s >= 0; --s)
        if (pi + s < prev->n_poses && same_group(pi, pi + s, s)) {
          take_over(R, pi, pi + s, s);
          return;
        }
    // membership of the open segment's cameras and camera pairs: stamp tables (stamp = the
    // segment's local number) when the free cameras are few, the linear searches otherwise
    std::vector<int32_t> cam_stamp(tables ? N : 0, -1), fcam_stamp(tables ? std::max(Nf, 1) : 0, -1);
    std::vector<int32_t> pair_stamp(tables ? (size_t)std::max(Nf, 1) * std::max(Nf, 1) : 0, -1);
    std::vector<int32_t> pair_sidx(tables ? (size_t)std::max(Nf, 1) * std::max(Nf, 1) : 0, 0);
    std::vector<int32_t> cq;
    int c_obs = 0, c_te = 0, c_pts = 0, c_pairs = 0, s_nch = 0;
    int64_t s_obs = 0;
    bool seg_open = false;
    auto open_chunk = [&](int q) {
      R.chunk_q.push_back(q);
      R.chunk_pairs.push_back(0);
      R.chunk_fte.push_back(0);
      R.chunk_fobs.push_back(0);
      c_obs = c_te = c_pts = c_pairs = 0;
      ++s_nch;
    };
    // the open segment padded to group_nch chunks by empty chunks at landmark q (none of its
    // landmarks: q starts the next chunk)
    auto pad_segment = [&](int q) {
      if (!seg_open) return;
      while (s_nch < group_nch) open_chunk(q);
    };
    for (int q = qa; q < qb; ++q) {
      const int t0 = P.pt_te[q], t1 = P.pt_te[q + 1];
      const int nob = P.te_obs[t1] - P.te_obs[t0], nte = t1 - t0;
      cq.clear();
      int fobs = 0;
      for (int t = t0; t < t1; ++t)
        if (P.te_cam[t] >= n_fixed) {
          cq.push_back(P.te_cam[t] - n_fixed);
          fobs += P.te_obs[t + 1] - P.te_obs[t];
        }
      if (t1 - t0 > kSegAllCams) {
        R.err_q = q;
        R.err = fmt("landmark %ld is too wide (%ld cameras); limit: %ld cameras per landmark", P.pt_perm[q], t1 - t0,
                    (long)kSegAllCams);
        return;
      }
      const int k = (int)cq.size();
      if (nob > kChunkObs || nte > kChunkTe || k > kSegCams || k * (k + 1) / 2 > kSegSlots) {
        R.err_q = q;
        R.err = fmt("landmark %ld is too wide (%ld observations, %ld free cameras); "
                    "limits: 64 observations, 10 free cameras per landmark",
                    P.pt_perm[q], nob, k);
        return;
      }
      const int npairs = k * (k + 1) / 2;
      const bool chunk_fits = seg_open && c_obs + nob <= kChunkObs && c_te + nte <= kChunkTe &&
                              c_pts + 1 <= kChunkPts && c_pairs + npairs <= kChunkPairs;
      bool seg_fits = seg_open;
      if (seg_open) {
        PlanSeg& s = R.segs.back();
        const int32_t sid = (int32_t)R.segs.size() - 1;
        int ncams = (int)s.cams.size(), nslots = (int)s.slots.size(), nacams = (int)s.acams.size();
        if (tables) {
          for (int c : cq) ncams += fcam_stamp[c] != sid;
          for (int a = 0; a < k; ++a)
            for (int b = 0; b <= a; ++b)
              nslots += pair_stamp[(size_t)std::max(cq[a], cq[b]) * Nf + std::min(cq[a], cq[b])] != sid;
          for (int t = t0; t < t1; ++t) nacams += cam_stamp[P.te_cam[t]] != sid;
        } else {
          for (int c : cq) ncams += find_or_neg(s.cams, c) < 0;
          for (int a = 0; a < k; ++a)
            for (int b = 0; b <= a; ++b) {
              const auto pr = std::make_pair(std::max(cq[a], cq[b]), std::min(cq[a], cq[b]));
              nslots += std::find(s.slots.begin(), s.slots.end(), pr) == s.slots.end();
            }
          for (int t = t0; t < t1; ++t) nacams += find_or_neg(s.acams, P.te_cam[t]) < 0;
        }
        seg_fits = ncams <= kSegCams && nslots <= max_slots && nacams <= kSegAllCams;
      }
      if (!seg_fits || (!chunk_fits && (group_nch ? s_nch >= group_nch : s_obs >= seg_obs_target))) {
        pad_segment(q);
        R.segs.emplace_back((int)R.chunk_q.size(), -1);
        seg_open = true;
        s_obs = 0;
        s_nch = 0;
        open_chunk(q);
      } else if (!chunk_fits) {
        open_chunk(q);
      }
      PlanSeg& s = R.segs.back();
      const int32_t sid = (int32_t)R.segs.size() - 1;
      if (tables) {
        for (int c : cq)
          if (fcam_stamp[c] != sid) {
            fcam_stamp[c] = sid;
            s.cams.push_back(c);
          }
        for (int t = t0; t < t1; ++t)
          if (cam_stamp[P.te_cam[t]] != sid) {
            cam_stamp[P.te_cam[t]] = sid;
            s.acams.push_back(P.te_cam[t]);
          }
        for (int a = 0; a < k; ++a)
          for (int b = 0; b <= a; ++b) {
            const int32_t hi = std::max(cq[a], cq[b]), lo = std::min(cq[a], cq[b]);
            int32_t& st = pair_stamp[(size_t)hi * Nf + lo];
            int32_t& si = pair_sidx[(size_t)hi * Nf + lo];
            if (st != sid) {
              st = sid;
              si = (int32_t)s.slots.size();
              s.slots.push_back(std::make_pair(hi, lo));
              s.slot_cnt.push_back(0);
            }
            ++s.slot_cnt[si];
          }
      } else {
        for (int c : cq)
          if (find_or_neg(s.cams, c) < 0) s.cams.push_back(c);
        for (int t = t0; t < t1; ++t)
          if (find_or_neg(s.acams, P.te_cam[t]) < 0) s.acams.push_back(P.te_cam[t]);
        for (int a = 0; a < k; ++a)
          for (int b = 0; b <= a; ++b) {
            const auto pr = std::make_pair(std::max(cq[a], cq[b]), std::min(cq[a], cq[b]));
            const auto it = std::find(s.slots.begin(), s.slots.end(), pr);
            if (it == s.slots.end()) {
              s.slots.push_back(pr);
              s.slot_cnt.push_back(1);
            } else {
              ++s.slot_cnt[it - s.slots.begin()];
            }
          }
      }
      c_obs += nob;
      c_te += nte;
      c_pts += 1;
      c_pairs += npairs;
      s_obs += nob;
      R.chunk_pairs.back() += npairs;
      R.chunk_fte.back() += k;
      R.chunk_fobs.back() += fobs;
    }
    pad_segment(qb);
  };
  {  // groups handed out one at a time (taken-over groups cost little, packed ones more)
    std::atomic<int> next{0};
    run_parallel(std::min(nparts, nthr), [&](int) {
      for (int pi = next.fetch_add(1); pi < nparts; pi = next.fetch_add(1)) pack(pi);
    });
  }
  for (const PlanPart& R : parts)  // the first error in landmark order
    if (R.err_q >= 0) return R.err;
  // merge the groups: chunks and segments in landmark order
  std::vector<PlanSeg*>& segs = X.segp;  // (pointers into the groups' segment lists)
  std::vector<int32_t>&ch_pairs = X.ch_pairs, &ch_fte = X.ch_fte, &ch_fobs = X.ch_fobs;
  segs.clear();
  ch_pairs.clear();
  ch_fte.clear();
  ch_fobs.clear();
  sized(P.group_chunk, nparts + 1);
  sized(P.group_seg, nparts + 1);
  for (int pi = 0; pi < nparts; ++pi) {
    PlanPart& R = parts[pi];
    const int base = (int)P.chunk_pt.size();
    P.group_chunk[pi] = base;
    P.group_seg[pi] = (int)segs.size();
    for (size_t c = 0; c < R.chunk_q.size(); ++c)
      P.chunk_src.push_back(R.src >= 0 ? prev->group_chunk[R.src] + (int)c : -1);
    if (R.src >= 0) {
      ++P.reused_groups;
      P.reused_chunks += (int)R.chunk_q.size();
      if (P.chunk_img.get_allocator().pinned && !R.chunk_q.empty()) P.host_images_partial = true;
    }
    for (size_t c = 0; c < R.chunk_q.size(); ++c) {
      const int q = R.chunk_q[c];
      P.chunk_obs.push_back(P.te_obs[P.pt_te[q]]);
      P.chunk_te.push_back(P.pt_te[q]);
      P.chunk_pt.push_back(q);
    }
    ch_pairs.insert(ch_pairs.end(), R.chunk_pairs.begin(), R.chunk_pairs.end());
    ch_fte.insert(ch_fte.end(), R.chunk_fte.begin(), R.chunk_fte.end());
    ch_fobs.insert(ch_fobs.end(), R.chunk_fobs.begin(), R.chunk_fobs.end());
    for (PlanSeg& s : R.segs) {
      s.chunk0 += base;
      segs.push_back(&s);
    }
  }
  P.group_chunk[nparts] = (int)P.chunk_pt.size();
  P.group_seg[nparts] = (int)segs.size();
  P.chunk_obs.push_back(M);
  P.chunk_te.push_back(P.n_te);
  P.chunk_pt.push_back(L);
  PLAN_T(2, "segments");

  // ---- per segment: sorted windows, slab offsets, per chunk pair and camera lists,
  // chunk headers and LDS images, segment headers.  Offsets first (prefix sums over
  // segments and chunks), then segment ranges filled in parallel.
  const int nchunks = (int)P.chunk_obs.size() - 1;
  const int nseg = (int)segs.size();
  std::vector<int32_t>& seg_of = X.seg_of;
  filled(seg_of, std::max(nchunks, 1), 0);
  sized(P.seg_chunk, nseg + 1);
  sized(P.seg_slot_off, nseg + 1);
  sized(P.seg_cam_off, nseg + 1);
  sized(P.seg_acam_off, nseg + 1);
  P.seg_chunk[0] = P.seg_slot_off[0] = P.seg_cam_off[0] = P.seg_acam_off[0] = 0;
  for (int si = 0; si < nseg; ++si) {
    const PlanSeg& s = *segs[si];
    const int ch1 = si + 1 < nseg ? segs[si + 1]->chunk0 : nchunks;
    for (int ch = s.chunk0; ch < ch1; ++ch) seg_of[ch] = si;
    P.seg_chunk[si + 1] = ch1;
    P.seg_slot_off[si + 1] = P.seg_slot_off[si] + (int)s.slots.size();
    P.seg_cam_off[si + 1] = P.seg_cam_off[si] + (int)s.cams.size();
    P.seg_acam_off[si + 1] = P.seg_acam_off[si] + (int)s.acams.size();
  }
  // per chunk: its slot_ptr / cam_ptr rows and its pair / camera list ranges
  std::vector<int32_t>&pair_base = X.pair_base, &cl_base = X.cl_base, &col_base = X.col_base;
  sized(pair_base, nchunks + 1);
  sized(cl_base, nchunks + 1);
  sized(col_base, nchunks + 1);
  sized(P.chunk_slot_base, nchunks);
  sized(P.chunk_cam_base, nchunks);
  {
    int32_t sb = 0, cb = 0;
    pair_base[0] = cl_base[0] = col_base[0] = 0;
    for (int ch = 0; ch < nchunks; ++ch) {
      const PlanSeg& s = *segs[seg_of[ch]];
      P.chunk_slot_base[ch] = sb;
      P.chunk_cam_base[ch] = cb;
      sb += (int)s.slots.size() + 1;
      cb += (int)s.cams.size() + 1;
      pair_base[ch + 1] = pair_base[ch] + ch_pairs[ch];
      cl_base[ch + 1] = cl_base[ch] + ch_fte[ch];
      col_base[ch + 1] = col_base[ch] + ch_fobs[ch];
    }
    sized(P.slot_ptr, sb);
    sized(P.cam_ptr, cb);
    sized(P.camo_ptr, cb);
  }
  sized(P.slot_i, P.seg_slot_off[nseg]);
  sized(P.slot_j, P.seg_slot_off[nseg]);
  sized(P.segcam_f, P.seg_cam_off[nseg]);
  sized(P.segcam_diag, P.seg_cam_off[nseg]);
  sized(P.seg_acam, P.seg_acam_off[nseg]);
  filled(P.obs_acam, std::max(M, 1), 0);
  sized(P.pair_list, pair_base[nchunks]);
  sized(P.cam_list, cl_base[nchunks]);
  sized(P.camo_list, col_base[nchunks]);
  filled(P.chunk_hdr, (size_t)std::max(nchunks, 1) * kChunkHdr, 0);
  sized(P.chunk_img, (size_t)std::max(nchunks, 1));
  if (nchunks == 0) P.chunk_img[0] = ChunkImg();
  filled(P.seg_hdr, (size_t)std::max(nseg, 1) * kSegHdr, 0);
  // chunk header: ob0 nob te0 nte p0 npt sb cb e0 e1 c0 c1 q0 q1 (14, 15: active slots and cameras)
  auto chunk_header = [&](int ch, int ns, int nc) {
    int32_t* h = &P.chunk_hdr[(size_t)ch * kChunkHdr];
    const int sb = P.chunk_slot_base[ch], cb = P.chunk_cam_base[ch];
    h[0] = P.chunk_obs[ch];
    h[1] = P.chunk_obs[ch + 1] - h[0];
    h[2] = P.chunk_te[ch];
    h[3] = P.chunk_te[ch + 1] - h[2];
    h[4] = P.chunk_pt[ch];
    h[5] = P.chunk_pt[ch + 1] - P.chunk_pt[ch];
    h[6] = sb;
    h[7] = cb;
    h[8] = P.slot_ptr[sb];
    h[9] = P.slot_ptr[sb + ns];
    h[10] = P.cam_ptr[cb];
    h[11] = P.cam_ptr[cb + nc];
    h[12] = P.camo_ptr[cb];
    h[13] = P.camo_ptr[cb + nc];
    return h;
  };
  // segment header (kSegHdr)
  auto seg_header = [&](int si, const PlanSeg& s) {
    int32_t* h = &P.seg_hdr[(size_t)si * kSegHdr];
    const int ch0 = P.seg_chunk[si], ch1 = P.seg_chunk[si + 1];
    h[0] = (int)s.slots.size();
    h[1] = P.seg_slot_off[si];
    h[2] = P.seg_cam_off[si];
    h[3] = (int)s.cams.size();
    h[4] = (int)s.acams.size();
    h[5] = ch0;
    h[6] = ch1;
    int16_t* h16 = reinterpret_cast<int16_t*>(h);
    for (int i = 0; i < h[4]; ++i) h16[16 + i] = (int16_t)s.acams[i];
    for (int i = 0; i < h[3]; ++i) h16[32 + i] = (int16_t)s.cams[i];
    if (ch1 > ch0) std::copy(&P.chunk_hdr[(size_t)ch0 * kChunkHdr], &P.chunk_hdr[(size_t)(ch0 + 1) * kChunkHdr], h + 32);
  };
  // a segment taken over from the previous plan: its lists and images copied, their offsets
  // moved to this plan's (the values fill() would compute from the same landmarks)
  const bool host_images_pinned = P.chunk_img.get_allocator().pinned;
  auto fill_taken = [&](int si, const PlanSeg& s) {
    const BAPlan& Q = *prev;
    const int ps = s.src;
    const int ch0 = P.seg_chunk[si], ch1 = P.seg_chunk[si + 1], pch0 = Q.seg_chunk[ps];
    const int so = P.seg_slot_off[si], co = P.seg_cam_off[si];
    const int ns = (int)s.slots.size(), nc = (int)s.cams.size();
    for (int i = 0; i < ns; ++i) {
      P.slot_i[so + i] = s.slots[i].first;
      P.slot_j[so + i] = s.slots[i].second;
    }
    std::copy(s.acams.begin(), s.acams.end(), P.seg_acam.begin() + P.seg_acam_off[si]);
    const int ob0 = P.chunk_obs[ch0], pob0 = Q.chunk_obs[pch0];
    std::memcpy(P.obs_acam.data() + ob0, Q.obs_acam.data() + pob0, P.chunk_obs[ch1] - ob0);
    for (int i = 0; i < nc; ++i) {
      P.segcam_f[co + i] = s.cams[i];
      P.segcam_diag[co + i] = Q.segcam_diag[Q.seg_cam_off[ps] + i];
    }
    for (int ch = ch0; ch < ch1; ++ch) {
      const int pc = pch0 + (ch - ch0);
      const int te0 = P.chunk_te[ch], pte0 = Q.chunk_te[pc];
      std::copy(Q.te_lcam.data() + pte0, Q.te_lcam.data() + pte0 + (P.chunk_te[ch + 1] - te0), P.te_lcam.data() + te0);
      const int sb = P.chunk_slot_base[ch], psb = Q.chunk_slot_base[pc];
      const int32_t pb = pair_base[ch], qpb = Q.slot_ptr[psb];
      for (int sl = 0; sl <= ns; ++sl) P.slot_ptr[sb + sl] = Q.slot_ptr[psb + sl] - qpb + pb;
      std::memcpy(P.pair_list.data() + pb, Q.pair_list.data() + qpb, sizeof(uint16_t) * (pair_base[ch + 1] - pb));
      const int cb = P.chunk_cam_base[ch], pcb = Q.chunk_cam_base[pc];
      const int32_t clb = cl_base[ch], qcl = Q.cam_ptr[pcb], cob = col_base[ch], qco = Q.camo_ptr[pcb];
      for (int c = 0; c <= nc; ++c) {
        P.cam_ptr[cb + c] = Q.cam_ptr[pcb + c] - qcl + clb;
        P.camo_ptr[cb + c] = Q.camo_ptr[pcb + c] - qco + cob;
      }
      std::memcpy(P.cam_list.data() + clb, Q.cam_list.data() + qcl, cl_base[ch + 1] - clb);
      std::memcpy(P.camo_list.data() + cob, Q.camo_list.data() + qco, col_base[ch + 1] - cob);
      int32_t* h = chunk_header(ch, ns, nc);
      h[14] = Q.chunk_hdr[(size_t)pc * kChunkHdr + 14];
      h[15] = Q.chunk_hdr[(size_t)pc * kChunkHdr + 15];
      // the engine's plans keep their images in page-locked memory, uncached for the CPU (a
      // read is slow): they take images over on the device (d_chunk_img_prev_ -> d_chunk_img_)
      // and leave the host copy unwritten; host-only plans (digests, probes) copy it
      if (!host_images_pinned) std::memcpy(&P.chunk_img[ch], &Q.chunk_img[pc], sizeof(ChunkImg));
    }
    seg_header(si, s);
  };
  // segments handed out in batches from a shared counter (dynamic scheduling: on a slide the
  // freshly packed segments, the expensive ones, are the newest groups, all at the end)
  std::atomic<int> fill_next{0};
  constexpr int kFillBatch = 4;
  auto fill = [&]() {
    // per-thread lookup tables (camera -> window index, camera pair -> slot) and counting-sort buffers
    std::vector<int32_t> fcam_idx(tables ? std::max(Nf, 1) : 0, -1), acam_idx(tables ? N : 0, -1);
    std::vector<int32_t> pair_slot(tables ? (size_t)std::max(Nf, 1) * std::max(Nf, 1) : 0, -1);
    int32_t cnt[std::max(kSegSlots, kSegCams) + 1], cnt2[kSegCams + 1], pslot[kChunkPairs];
    uint16_t ptmp[kChunkPairs];
    for (int sa = fill_next.fetch_add(kFillBatch); sa < nseg; sa = fill_next.fetch_add(kFillBatch))
    for (int si = sa; si < std::min(sa + kFillBatch, nseg); ++si) {
      PlanSeg& s = *segs[si];
      if (s.src >= 0) {
        fill_taken(si, s);
        continue;
      }
      std::sort(s.cams.begin(), s.cams.end());
      std::sort(s.slots.begin(), s.slots.end());
      std::sort(s.acams.begin(), s.acams.end());
      const int ch0 = P.seg_chunk[si], ch1 = P.seg_chunk[si + 1];
      const int so = P.seg_slot_off[si], co = P.seg_cam_off[si];
      for (int i = 0; i < s.slots.size(); ++i) {
        P.slot_i[so + i] = s.slots[i].first;
        P.slot_j[so + i] = s.slots[i].second;
      }
      if (tables) {
        for (int i = 0; i < s.cams.size(); ++i) fcam_idx[s.cams[i]] = (int32_t)i;
        for (int i = 0; i < s.acams.size(); ++i) acam_idx[s.acams[i]] = (int32_t)i;
        for (int i = s.slots.size(); i-- > 0;)  // the first of equal slots (copies)
          pair_slot[(size_t)s.slots[i].first * Nf + s.slots[i].second] = (int32_t)i;
      }
      auto lcam_of = [&](int32_t c) {  // window index of free camera c
        return tables ? fcam_idx[c] : (int32_t)(std::lower_bound(s.cams.begin(), s.cams.end(), c) - s.cams.begin());
      };
      auto slot_of = [&](const std::pair<int32_t, int32_t>& pr) {
        return tables ? pair_slot[(size_t)pr.first * Nf + pr.second]
                      : (int32_t)(std::lower_bound(s.slots.begin(), s.slots.end(), pr) - s.slots.begin());
      };
      std::copy(s.acams.begin(), s.acams.end(), P.seg_acam.begin() + P.seg_acam_off[si]);
      for (int o = P.chunk_obs[ch0]; o < P.chunk_obs[ch1]; ++o)
        P.obs_acam[o] = (uint8_t)(tables ? acam_idx[P.obs_cam[o]]
                                         : std::lower_bound(s.acams.begin(), s.acams.end(), P.obs_cam[o]) -
                                               s.acams.begin());
      for (int i = 0; i < s.cams.size(); ++i) {
        P.segcam_f[co + i] = s.cams[i];
        P.segcam_diag[co + i] = slot_of(std::make_pair(s.cams[i], s.cams[i]));
      }
      const int ns = (int)s.slots.size(), nc = (int)s.cams.size();
      for (int ch = ch0; ch < ch1; ++ch) {
        const int te0 = P.chunk_te[ch];
        for (int t = te0; t < P.chunk_te[ch + 1]; ++t)
          if (P.te_cam[t] >= n_fixed) P.te_lcam[t] = (int16_t)lcam_of(P.te_cam[t] - n_fixed);
        // pair lists by slot: a stable counting sort of the (x, y) pairs in generation order
        // (a landmark's track entries are sorted by camera, so (cam x, cam y) is (hi, lo))
        int npair = 0;
        std::fill(cnt, cnt + ns + 1, 0);
        for (int q = P.chunk_pt[ch]; q < P.chunk_pt[ch + 1]; ++q) {
          const int ta = P.pt_te[q], tb = P.pt_te[q + 1];
          for (int x = ta; x < tb; ++x) {
            const int32_t cx = P.te_cam[x] - n_fixed;
            if (cx < 0) continue;
            for (int y = ta; y <= x; ++y) {
              const int32_t cy = P.te_cam[y] - n_fixed;
              if (cy < 0) continue;
              const int32_t sl = slot_of(std::make_pair(cx, cy));
              pslot[npair] = sl;
              ptmp[npair++] = (uint16_t)((x - te0) | ((y - te0) << 8));
              ++cnt[sl + 1];
            }
          }
        }
        for (int sl = 0; sl < ns; ++sl) cnt[sl + 1] += cnt[sl];
        const int32_t pbase = pair_base[ch];
        int32_t* sp = &P.slot_ptr[P.chunk_slot_base[ch]];
        for (int sl = 0; sl <= ns; ++sl) sp[sl] = pbase + cnt[sl];
        for (int e = 0; e < npair; ++e) P.pair_list[pbase + cnt[pslot[e]]++] = ptmp[e];
        // camera lists: track entries and observations by window camera, in order
        std::fill(cnt, cnt + nc + 1, 0);
        std::fill(cnt2, cnt2 + nc + 1, 0);
        for (int t = te0; t < P.chunk_te[ch + 1]; ++t)
          if (P.te_lcam[t] >= 0) ++cnt[P.te_lcam[t] + 1];
        const int ob0 = P.chunk_obs[ch];
        for (int o = ob0; o < P.chunk_obs[ch + 1]; ++o)
          if (P.te_lcam[P.obs_te[o]] >= 0) ++cnt2[P.te_lcam[P.obs_te[o]] + 1];
        for (int c = 0; c < nc; ++c) {
          cnt[c + 1] += cnt[c];
          cnt2[c + 1] += cnt2[c];
        }
        const int32_t cbase = cl_base[ch], obase = col_base[ch];
        int32_t* cp = &P.cam_ptr[P.chunk_cam_base[ch]];
        int32_t* op = &P.camo_ptr[P.chunk_cam_base[ch]];
        for (int c = 0; c <= nc; ++c) {
          cp[c] = cbase + cnt[c];
          op[c] = obase + cnt2[c];
        }
        for (int t = te0; t < P.chunk_te[ch + 1]; ++t)
          if (P.te_lcam[t] >= 0) P.cam_list[cbase + cnt[P.te_lcam[t]]++] = (uint8_t)(t - te0);
        for (int o = ob0; o < P.chunk_obs[ch + 1]; ++o) {
          const int lc = P.te_lcam[P.obs_te[o]];
          if (lc >= 0) P.camo_list[obase + cnt2[lc]++] = (uint8_t)(o - ob0);
        }
        int32_t* h = chunk_header(ch, ns, nc);
        const int sb = P.chunk_slot_base[ch], cb = P.chunk_cam_base[ch];
        // the chunk's LDS image (chunk-relative offsets, unused entries zero), built in a local
        // buffer and copied out whole: the engine's images are page-locked memory, which the CPU
        // reads uncached (the build reads its own fields back) and writes best in whole lines
        ChunkImg g{};
        const int nob = h[1], nte = h[3], p0 = h[4], npt = h[5];
        const int e0 = h[8], e1 = h[9], c0 = h[10], c1 = h[11], q0 = h[12], q1 = h[13];
        for (int i = 0; i < nob; ++i) {
          g.obs_te[i] = P.obs_te[ob0 + i] - te0;
          g.uv[2 * i] = P.obs_uv[2 * (ob0 + i)];
          g.uv[2 * i + 1] = P.obs_uv[2 * (ob0 + i) + 1];
          g.acam[i] = P.obs_acam[ob0 + i];
        }
        for (int i = 0; i <= nte; ++i) g.te_obs[i] = P.te_obs[te0 + i] - ob0;
        for (int i = 0; i < nte; ++i) {
          g.te_pt[i] = P.te_pt[te0 + i] - p0;
          g.te_lcam[i] = P.te_lcam[te0 + i];
        }
        for (int i = 0; i <= npt; ++i) {
          g.pt_te[i] = P.pt_te[p0 + i] - te0;
          g.pt_obs[i] = P.te_obs[P.pt_te[p0 + i]] - ob0;
        }
        for (int i = 0; i < nob; ++i) {
          g.obs_pt[i] = g.te_pt[g.obs_te[i]];
          g.obs_lcam[i] = g.te_lcam[g.obs_te[i]];
        }
        // the slots with pairs in this chunk and the cameras with track entries or observations
        // in it, compacted in window order (their lists keep their order)
        int nas = 0, nac = 0;
        {
          // active slots.  Four-wave K1: lanes per row item (2^lg) doubled greedily for the slot
          // with the longest per-lane pair chain while 6 lanes x the sum fit its 256 lanes (more
          // than 42 active slots take one lane per row item, in two passes), items ordered by
          // lanes per row descending (every item group starts at a multiple of its own width).
          // One-wave K1: lane j = active slot j (copies of heavy slots made at packing).
          int sl[kSegSlots], cntp[kSegSlots], lg[kSegSlots];
          for (int i = 0; i < ns; ++i)
            if (P.slot_ptr[sb + i + 1] > P.slot_ptr[sb + i]) {
              sl[nas] = i;
              cntp[nas] = P.slot_ptr[sb + i + 1] - P.slot_ptr[sb + i];
              lg[nas++] = 0;
            }
          int ord[kSegSlots];
          for (int i = 0; i < nas; ++i) ord[i] = i;
          int base = 0;
          if (!wave) {
            int used = nas;
            for (;;) {
              int best = -1, chain = 0;
              for (int i = 0; i < nas; ++i) {
                const int c = (cntp[i] + (1 << lg[i]) - 1) >> lg[i];
                if (c > chain) {
                  chain = c;
                  best = i;
                }
              }
              if (best < 0 || chain <= 1 || lg[best] == 3 || 6 * (used + (1 << lg[best])) > kLinLanes) break;
              used += 1 << lg[best];
              ++lg[best];
            }
            std::stable_sort(ord, ord + nas, [&](int a, int b) { return lg[a] > lg[b]; });
            for (int j = 0; j < nas; ++j) {
              const int i = ord[j];
              g.aslot[j] = (uint8_t)sl[i];
              g.slotp[j] = P.slot_ptr[sb + sl[i]] - e0;
              g.apcnt[j] = (uint16_t)cntp[i];
              g.anp[j] = (uint8_t)lg[i];
              g.acopy[j] = 0;
              g.adcam[j] = P.slot_i[so + sl[i]] == P.slot_j[so + sl[i]] ? (uint8_t)lcam_of(P.slot_i[so + sl[i]]) : 0xFF;
              g.abase[j] = (uint16_t)base;
              base += 6 << lg[i];
            }
          } else {
            // One-wave K1: an item is a copy of an active slot on one lane (the block over a
            // consecutive range of the slot's pairs); each slot gets the fewest copies that bring
            // its per-lane chain (pairs per copy, a diagonal pair weighted 5 against 3 for its U
            // and b) within kCopyChain, or, past kWaveItems lanes, copies go one at a time to the
            // slot of longest chain.  The copies' blocks are summed in copy order inside K1 (one
            // slab row per window slot).
            int cp[kSegSlots];
            auto wgt = [&](int i) { return P.slot_i[so + sl[i]] == P.slot_j[so + sl[i]] ? 5 : 3; };
            auto chain = [&](int i) { return (cntp[i] + cp[i] - 1) / cp[i] * wgt(i); };
            int lanes = 0;
            for (int i = 0; i < nas; ++i) {
              const int per = std::max(1, kCopyChain / wgt(i));
              cp[i] = std::max(1, (cntp[i] + per - 1) / per);
              lanes += cp[i];
            }
            if (lanes > kWaveItems) {
              for (int i = 0; i < nas; ++i) cp[i] = 1;
              for (lanes = nas; lanes < kWaveItems; ++lanes) {
                int best = 0;
                for (int i = 1; i < nas; ++i)
                  if (chain(i) > chain(best)) best = i;
                if (chain(best) <= kCopyChain || cntp[best] <= cp[best]) break;
                ++cp[best];
              }
            }
            int j = 0;
            for (int i = 0; i < nas; ++i)
              for (int c = 0; c < cp[i]; ++c, ++j) {
                const int lo = (int)((int64_t)cntp[i] * c / cp[i]), hi = (int)((int64_t)cntp[i] * (c + 1) / cp[i]);
                g.aslot[j] = (uint8_t)sl[i];
                g.slotp[j] = (uint16_t)(P.slot_ptr[sb + sl[i]] - e0 + lo);
                g.apcnt[j] = (uint16_t)(hi - lo);
                g.anp[j] = (uint8_t)cp[i];   // copies of the slot
                g.acopy[j] = (uint8_t)c;     // this item's copy index
                g.adcam[j] = P.slot_i[so + sl[i]] == P.slot_j[so + sl[i]] ? (uint8_t)lcam_of(P.slot_i[so + sl[i]]) : 0xFF;
                g.abase[j] = (uint16_t)j;
              }
            nas = j;
            base = j;
          }
          g.abase[nas] = (uint16_t)base;
          g.slotp[nas] = e1 - e0;
        }
        for (int i = 0; i < e1 - e0; ++i) g.pairs[i] = P.pair_list[e0 + i];
        for (int i = 0; i < nc; ++i)
          if (P.cam_ptr[cb + i + 1] > P.cam_ptr[cb + i] || P.camo_ptr[cb + i + 1] > P.camo_ptr[cb + i]) {
            g.acid[nac] = (uint8_t)i;
            g.camp[nac] = P.cam_ptr[cb + i] - c0;
            g.camop[nac] = P.camo_ptr[cb + i] - q0;
            g.dslot[nac++] = P.segcam_diag[co + i];
          }
        g.camp[nac] = c1 - c0;
        g.camop[nac] = q1 - q0;
        if (wave) {  // each active camera's diagonal items (its copies are consecutive)
          for (int ci = 0; ci < nac; ++ci) {
            int j0 = -1, nj = 0;
            for (int j = 0; j < nas; ++j)
              if (g.adcam[j] == g.acid[ci]) {
                if (j0 < 0) j0 = j;
                ++nj;
              }
            g.cdiag0[ci] = (uint8_t)std::max(j0, 0);
            g.cdiagn[ci] = (uint8_t)nj;
          }
          // the diagonal items' U observations: a diagonal slot's pairs (x, x) run over its
          // camera's track entries in order, so copy k's observations are the next entries of
          // the camera's observation list; diagonal items come in camera order (the slot of
          // (c, c) is the last of row c), so the ranges tile camol and an off-diagonal item
          // gets the empty range at the next diagonal item's start
          g.auo[nas] = (uint8_t)(q1 - q0);
          int run = 0;
          for (int ci = 0, j = 0; ci < nac; ++ci) {
            run = g.camop[ci];
            for (; j < g.cdiag0[ci] + g.cdiagn[ci] && j < nas; ++j) {
              if (g.adcam[j] != g.acid[ci]) continue;
              g.auo[j] = (uint8_t)run;
              for (int e = g.slotp[j]; e < g.slotp[j] + g.apcnt[j]; ++e) {
                const int x = g.pairs[e] & 255;
                run += g.te_obs[x + 1] - g.te_obs[x];
              }
            }
          }
          for (int j = nas; j-- > 0;)
            if (g.adcam[j] == 0xFF) g.auo[j] = g.auo[j + 1];
        }
        for (int i = 0; i < c1 - c0; ++i) g.caml[i] = P.cam_list[c0 + i];
        for (int i = 0; i < q1 - q0; ++i) g.camol[i] = P.camo_list[q0 + i];
        std::memcpy(&P.chunk_img[ch], &g, sizeof g);
        h[14] = nas;
        h[15] = nac;
      }
      seg_header(si, s);
      if (tables) {  // clear this segment's table entries for the next one
        for (int32_t c : s.cams) fcam_idx[c] = -1;
        for (int32_t c : s.acams) acam_idx[c] = -1;
        for (const auto& pr : s.slots) pair_slot[(size_t)pr.first * Nf + pr.second] = -1;
      }
    }
  };
  {
    const int nt = std::max(1, std::min(nthr, (nseg + kFillBatch - 1) / kFillBatch));
    run_parallel(nt, [&](int) { fill(); });
  }
  if (P.pair_list.empty()) P.pair_list.push_back(0);  // keep device arrays non-empty
  if (P.cam_list.empty()) P.cam_list.push_back(0);
  if (P.camo_list.empty()) P.camo_list.push_back(0);
  if (P.segcam_diag.empty()) P.segcam_diag.push_back(0);
  PLAN_T(3, "lists+images");
  return "";
}

std::vector<int32_t> local_profile_first(const BAPlan& P) {
  std::vector<int32_t> first(P.n_free);
  for (int i = 0; i < P.n_free; ++i) first[i] = i;
  for (size_t s = 0; s < P.slot_i.size(); ++s)
    first[P.slot_i[s]] = std::min(first[P.slot_i[s]], P.slot_j[s]);
  return first;
}

void build_profile(BAPlan& P, const std::vector<int32_t>& first, bool step_tables) {
  const int F = P.n_free;
  P.prof_first = first;
  filled(P.prof_off, F + 1, 0);
  for (int i = 0; i < F; ++i) P.prof_off[i + 1] = P.prof_off[i] + (i - first[i] + 1);
  filled(P.prof_last, F, 0);
  for (int k = 0; k < F; ++k) P.prof_last[k] = k;
  for (int i = 0; i < F; ++i)
    for (int k = first[i]; k <= i; ++k) P.prof_last[k] = std::max(P.prof_last[k], i);
  const int nb = P.prof_off[F];
  filled(P.prof_diag, nb, 0);
  for (int i = 0; i < F; ++i) P.prof_diag[P.prof_off[i] + (i - first[i])] = 1;
  // per profile block its slab slots, per free camera its rhs entries: stable counting
  // sorts (slots / entries in plan order within a block), and the inverse positions
  const size_t nslot = P.slot_i.size(), nent = P.segcam_f.size();
  std::vector<int32_t> sblk(nslot);
  filled(P.prof_src_ptr, nb + 1, 0);
  for (size_t s = 0; s < nslot; ++s) {
    sblk[s] = P.prof_off[P.slot_i[s]] + (P.slot_j[s] - first[P.slot_i[s]]);
    ++P.prof_src_ptr[sblk[s] + 1];
  }
  for (int b = 0; b < nb; ++b) P.prof_src_ptr[b + 1] += P.prof_src_ptr[b];
  sized(P.prof_src, nslot);
  filled(P.slab_pos, std::max<size_t>(nslot, 1), 0);
  {
    std::vector<int32_t> next(P.prof_src_ptr.begin(), P.prof_src_ptr.end() - 1);
    for (size_t s = 0; s < nslot; ++s) {
      const int32_t k = next[sblk[s]]++;
      P.prof_src[k] = (int32_t)s;
      P.slab_pos[s] = k;
    }
  }
  filled(P.camb_ptr, F + 1, 0);
  for (size_t e = 0; e < nent; ++e) ++P.camb_ptr[P.segcam_f[e] + 1];
  for (int f = 0; f < F; ++f) P.camb_ptr[f + 1] += P.camb_ptr[f];
  sized(P.camb_src, nent);
  filled(P.cam_pos, std::max<size_t>(nent, 1), 0);
  {
    std::vector<int32_t> next(P.camb_ptr.begin(), P.camb_ptr.end() - 1);
    for (size_t e = 0; e < nent; ++e) {
      const int32_t k = next[P.segcam_f[e]]++;
      P.camb_src[k] = (int32_t)e;
      P.cam_pos[e] = k;
    }
  }
  if (P.prof_src.empty()) P.prof_src.push_back(0);
  if (P.camb_src.empty()) P.camb_src.push_back(0);

  // K3 step tables (the profile solver's; the banded solver has its own)
  if (!step_tables) {
    P.solve_tab.assign(1, 0);
    P.solve_layout = SolveTableLayout();
    return;
  }
  auto blk = [&](int i, int j) { return P.prof_off[i] + (j - first[i]); };
  std::vector<int32_t> sptr{0}, pi, pblk, iptr{0}, iblk, iq;
  int maxnb = 0;
  for (int k = 0; k < F; ++k) {
    std::vector<int> rows;
    for (int i = k + 1; i <= P.prof_last[k]; ++i)
      if (first[i] <= k) rows.push_back(i);
    const int nb = (int)rows.size();
    maxnb = std::max(maxnb, nb);
    for (int i : rows) {
      pi.push_back(i);
      pblk.push_back(blk(i, k));
    }
    sptr.push_back((int32_t)pi.size());
    for (int q1 = 0; q1 < nb; ++q1)
      for (int q2 = 0; q2 <= q1; ++q2) {
        iblk.push_back(blk(rows[q1], rows[q2]));
        iq.push_back(q1 | (q2 << 16));
      }
    iptr.push_back((int32_t)iblk.size());
  }
  SolveTableLayout& L = P.solve_layout;
  std::vector<int32_t>& T = P.solve_tab;
  T.clear();
  auto put = [&](int& o, const std::vector<int32_t>& v) {
    o = (int)T.size();
    T.insert(T.end(), v.begin(), v.end());
  };
  std::vector<int32_t> diag(F), offv(P.prof_off.begin(), P.prof_off.begin() + F);
  for (int k = 0; k < F; ++k) diag[k] = blk(k, k);
  put(L.diag, diag);
  put(L.off, offv);
  put(L.first, first);
  put(L.step_ptr, sptr);
  put(L.panel_i, pi);
  put(L.panel_blk, pblk);
  put(L.item_ptr, iptr);
  put(L.item_blk, iblk);
  put(L.item_q, iq);
  L.len = (int)T.size();
  L.max_panel = maxnb;
  if (T.empty()) T.push_back(0);
}

uint64_t plan_digest(const BAPlan& P) {
  if (P.host_images_partial)
    throw std::logic_error("plan_digest: the plan's host chunk images are partial (taken over on the device)");
  uint64_t h = 1469598103934665603ull;
  auto bytes = [&](const void* p, size_t n) {
    const unsigned char* c = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  };
  auto vec = [&](const auto& v) {
    const uint64_t n = v.size();
    bytes(&n, sizeof n);
    if (n) bytes(v.data(), n * sizeof(v[0]));
  };
  const int32_t sizes[6] = {P.n_poses, P.n_points, P.n_obs, P.n_fixed, P.n_free, P.n_te};
  bytes(sizes, sizeof sizes);
  vec(P.pt_perm); vec(P.obs_uv); vec(P.obs_cam); vec(P.obs_te); vec(P.te_cam); vec(P.te_pt); vec(P.te_obs);
  vec(P.te_lcam); vec(P.pt_te); vec(P.chunk_obs); vec(P.chunk_te); vec(P.chunk_pt); vec(P.chunk_slot_base);
  vec(P.chunk_cam_base); vec(P.chunk_hdr); vec(P.slab_pos); vec(P.cam_pos); vec(P.seg_hdr); vec(P.chunk_img);
  vec(P.slot_ptr); vec(P.pair_list); vec(P.cam_ptr); vec(P.cam_list); vec(P.camo_ptr); vec(P.camo_list);
  vec(P.seg_chunk); vec(P.seg_slot_off); vec(P.seg_cam_off); vec(P.slot_i); vec(P.slot_j); vec(P.segcam_f);
  vec(P.segcam_diag); vec(P.seg_acam_off); vec(P.seg_acam); vec(P.obs_acam); vec(P.prof_first); vec(P.prof_off);
  vec(P.prof_last); vec(P.prof_src_ptr); vec(P.prof_src); vec(P.prof_diag); vec(P.camb_ptr); vec(P.camb_src);
  vec(P.solve_tab);
  const int32_t so = P.seg_obs;
  bytes(&so, sizeof so);
  if (P.seg_chunks > 1) bytes(&P.seg_chunks, sizeof P.seg_chunks);  // (plans of one chunk per segment: as before)
  vec(P.group_q); vec(P.group_chunk); vec(P.group_seg);
  return h;
}

}  // namespace vo
