// K3 for banded reduced camera systems: S dc = b by a two-sided block Cholesky, then the
// left se(3) pose update T <- exp(dc^) T.  Build-defined solve (the reference has no BA,
// SURVEY.md §8 a9-a10); same arithmetic contract as oracle/ba_ref.py gn_step (dense
// Cholesky of S, exp map of oracle/ba_ref.py se3_exp), checked to 1e-5 over whole runs.
//
// The window's reduced camera matrix is block banded: a landmark track spans at most
// w + 1 consecutive keyframes, so block (i, j) is zero for i - j > w (w = 7 for the
// BASELINE windows).  Rows are split into top [0, m), separator [m, m + w) and bottom
// [m + w, F); the top is eliminated top-down and the bottom bottom-up (the same
// algorithm on the block-reversed matrix) at the same time, then the separator, which
// receives both sides' Schur updates, continues the top side.  The chain of dependent
// block steps is max(m, nb) + w instead of F.
//
// One workgroup of eight waves (two per SIMD), four roles per side:
//   chain   holds the block column being factored in registers, one lane per scalar row
//           (lane 6 g + r: row r of block row g).  Step k: the diagonal block's rows go
//           through LDS to every lane, each lane factors it (chol6) and solves its own panel
//           row, the panel goes to LDS; after the workgroup barrier the lane loads its row
//           of column k + 1 and applies step k's update to it.
//   trail   after the barrier: the rest of step k's trailing update (blocks (i, j),
//           k + 2 <= j <= i <= k + w); ring mode: then column k - 1's factor record to
//           global memory.
//   fwd     the forward substitution of step k (y'_k = L_kk^-1 y_k, y_i -= L_ik y'_k).
//   loader  column k + w + 2 by LDS-DMA (ring mode: into the slot of column k - 2).
// Back substitution as a z recurrence (z_k = y'_k - sum_q L_{k+q,k}^T x_{k+q}); x_k =
// L_kk^-T z_k for every row at the end (see the back-substitution section below).
//
// LDS: full mode (the cfg3 window) keeps every column of both sides; ring mode (cfg4:
// F = 98, a 225 KB profile) keeps w + 4 column slots per side and writes the factor
// records to global memory.  Plus z (6F), the poses and the merge table.
#include <atomic>
#include "ba_band.h"

#include <algorithm>
#include <climits>

#include "ba_math.h"
#include "vo_common.h"

namespace vo {

BandSplit band_split(int F, const std::vector<int>& first) {
  BandSplit b;
  int w = 0;
  for (int i = 0; i < F; ++i) w = std::max(w, i - first[i]);
  b.w = w;
  if (F >= 2 * w + 2) {
    b.s = w;
    b.nb = (F - w) / 2;
    b.m = F - w - b.nb;
  } else {
    b.m = F;
  }
  return b;
}

static size_t band_lds_total(const BandLds& L, int F, int n_poses) {
  return 8 * (2 * ((size_t)L.rc * L.ss + L.pad) + 6 * (size_t)F + 12 * (size_t)n_poses + 104);
}

BandLds band_lds_layout(int F, const BandSplit& b, int n_poses, bool allow_split) {
  BandLds L;
  const int CS = band_col_stride(b.w);
  L.full = true;
  L.rc = std::max(b.m + b.s, b.nb + b.s);
  L.ss = CS;
  L.pad = 128;
  L.bytes = band_lds_total(L, F, n_poses);
  if (L.bytes <= kBandLdsMax) return L;
  // split: each side's columns in full in its own workgroup's LDS (plus the bottom's staged copy
  // of the top's separator records), two workgroups on two CUs
  if (b.s > 0 && allow_split) {
    L.split = true;
    L.bytes = 8 * ((size_t)L.rc * L.ss + L.pad + 6 * (size_t)F + 12 * (size_t)n_poses + 104 + 42 * (size_t)b.s);
    if (L.bytes <= kBandLdsMax) return L;
    L.split = false;
  }
  L.full = false;
  L.rc = b.w + 4;
  L.ss = band_slot_stride(b.w);
  L.pad = 0;
  L.bytes = band_lds_total(L, F, n_poses);
  return L;
}

BandTables band_tables(int F, const BandSplit& b, const BandLds& L) {
  const int w = b.w, R = w + 1, RC = L.rc, SS = L.ss, m = b.m, sp = b.s;
  const int offB = RC * SS + L.pad;
  BandTables T;
  T.merge = 0;
  for (int jj = 0; jj < sp; ++jj)
    for (int qq = 0; qq < sp - jj; ++qq) {
      const int j = m + jj, i = j + qq;
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) {
          // the bottom side stores its blocks transposed; a diagonal block is symmetric, so its
          // own lower triangle is the source (the critical-lane trailing tiles keep only the
          // lower triangle of a diagonal block that straddles two 16-row tiles up to date)
          T.tab.push_back((j % RC) * SS + 36 * qq + 6 * r + c);
          T.tab.push_back(offB + ((F - 1 - i) % RC) * SS + 36 * qq + (qq == 0 ? 6 * r + c : 6 * c + r));
        }
    }
  for (int d = 0; d < sp; ++d) {
    const int i = m + d;
    for (int r = 0; r < 6; ++r) {
      T.tab.push_back((i % RC) * SS + 36 * R + r);
      T.tab.push_back(offB + ((F - 1 - i) % RC) * SS + 36 * R + r);
    }
  }
  T.n_merge = (int)T.tab.size() / 2;
  if (T.tab.empty()) T.tab.push_back(0);
  return T;
}

size_t band_fac_doubles(int F, int w) { return (size_t)std::max(F, 1) * band_col_stride(w); }

bool band_supported(int F, int w, int n_poses) {
  if (w < 0 || w > kBandMaxW || F > kBandMaxF) return false;
  BandSplit b;
  b.w = w;
  b.m = F;  // the ring layout's size does not depend on the split
  return band_lds_layout(F, b, n_poses).bytes <= kBandLdsMax;
}

namespace {

// chol6 (ba_math.h) without the per-pivot positivity test on the dependent chain: a
// non-positive pivot gives a NaN / inf reciprocal (v_rsq_f64), which the caller detects
// from r afterwards (the same "not SPD" outcome).  The diagonal of L is not stored.
__device__ __forceinline__ void chol6_nochk(double (&a)[21], double (&r)[6]) {
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const double d = a[P6(j, j)];
    double q = __builtin_amdgcn_rsq(d);
    // one Newton step, q + (q / 2)(1 - d q^2): three dependent operations on the chain
    if (kCholNewton) q = __builtin_fma(0.5 * q, __builtin_fma(-(d * q), q, 1.0), q);
    r[j] = q;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) a[P6(i, j)] *= q;
#pragma unroll
    for (int i = j + 1; i < 6; ++i)
#pragma unroll
      for (int c = j + 1; c <= i; ++c) a[P6(i, c)] -= a[P6(i, j)] * a[P6(c, j)];
  }
}

constexpr int kBandWaves = 8;
constexpr int kBandThreads = 64 * kBandWaves;
constexpr int kLdRegs = 6;      // ring loader: elements per lane of one column
constexpr int kTaskRounds = 2;  // trailing (block, row pair) tasks per lane
constexpr int kProLoads = 8;    // prologue: 16-byte pieces per thread (columns 0 .. w + 1 of both sides)
static_assert(36 * (kBandMaxW + 1) + 12 <= 64 * kLdRegs, "one column per loader wave");
static_assert(3 * (kBandMaxW - 1) * kBandMaxW / 2 <= 64 * kTaskRounds, "trailing tasks per helper wave");
static_assert(6 * (kBandMaxW + 1) <= 64, "one lane per panel row");
static_assert(36 * (kBandMaxW + 1) + 12 <= 3 * 128, "at most three 1 KiB LDS-DMA pieces per column");
static_assert((kBandMaxW + 2) * (36 * (kBandMaxW + 1) + 12) <= kProLoads * kBandThreads, "prologue");
// Wave roles (wave = 2 * role + side; wave w runs on SIMD w mod 4, so each side's chain
// shares its SIMD only with that side's loader, which mostly waits on memory).
enum { kChain = 0, kTrail = 1, kLoad = 2, kFwd = 3 };

// LDS writes of every wave complete, then the workgroup barrier.  Global loads and
// stores stay in flight (__syncthreads would drain them: the ring loader's prefetch).
__device__ __forceinline__ void band_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#ifndef VO_BA_STAMPS
#define VO_BA_STAMPS 0
#endif
// Diagnostic build only (EXTRA=-DVO_BA_STAMPS=1): lane 0 of each wave accumulates
// s_memtime deltas per phase; the product build executes none.
#if VO_BA_STAMPS
#define BST(i)                                                    \
  do {                                                            \
    if (lane == 0) {                                              \
      const unsigned long long n_ = __builtin_amdgcn_s_memtime(); \
      st_acc[i] += n_ - st_t;                                     \
      st_t = n_;                                                  \
    }                                                             \
  } while (0)
// value x computed (and every LDS access retired) before the next stamp
#define BSETTLE(x)                                                                        \
  do {                                                                                    \
    int d_;                                                                               \
    asm volatile("s_waitcnt lgkmcnt(0)\n\tv_mov_b32 %0, %1" : "=v"(d_) : "v"(__double2loint(x))); \
  } while (0)
#if VO_BA_STAMPS >= 2  // fine stamps: each one drains the wave's LDS queue (s_memtime)
#define BSTF(i) BST(i)
#else
#define BSTF(i) \
  do {          \
  } while (0)
#undef BSETTLE
#define BSETTLE(x) \
  do {             \
  } while (0)
#endif
#else
#define BSTF(i) \
  do {          \
  } while (0)
#define BST(i) \
  do {         \
  } while (0)
#define BSETTLE(x) \
  do {             \
  } while (0)
#endif

// ---- fused K2: the reducer workgroups (BandArgs::nred).  Each 256-thread half of a
// workgroup runs ba_reduce_kernel's work for one item (a profile block, or the cost after
// the last block) with K2's partition and order, so sys gets the same bits as from K2.  The
// outputs go write-through (sc1: the solver reads them on another CU, maybe another XCD),
// every storing wave drains them, and one lane counts the workgroup in red_count after the
// workgroup barrier (MI355X_MICROARCH.md, hand-off rows: sc1 stores + vmcnt(0) + barrier +
// one agent-scope atomic add; the solver polls relaxed, then one agent-scope acquire).
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
constexpr int kRedScr = kRedSParts * 36 + kRedBParts * 6 + kRedThreads;  // LDS doubles per half

__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void band_reduce_wg(const BandArgs& B, int r, double* scr) {
  static_assert(kRedThreads * kBandRedItems == 512, "two K2 items per 512-thread workgroup");
  const ReduceArgs& A = B.red;
  const int tid = threadIdx.x, h = tid / kRedThreads, t = tid % kRedThreads;
  const int blk = kBandRedItems * r + h;
  double* part = scr + h * kRedScr;
  double* partb = part + kRedSParts * 36;
  double* cpart = partb + kRedBParts * 6;
  const bool isblk = blk < A.nprof, iscost = blk == A.nprof;
  int4 m = make_int4(0, 0, -1, 0);
  int2 o = make_int2(0, 0);
  double2 ps = make_double2(0.0, 0.0);
  double pb = 0.0, c = 0.0;
#if VO_BA_STAMPS  // diagnostic build: reducer r's realtime stamps (start, loads in, stored, counted)
  unsigned long long* rst = B.stamps ? B.stamps + 8 * kBandStamps + 8 + 4 * r : nullptr;
  if (rst && tid == 0) rst[0] = __builtin_amdgcn_s_memrealtime();
#endif
  // the readiness counter this item counts itself in (loaded beside its meta: no extra latency)
  const int col = isblk ? B.red_col[blk] : B.F;
  if (isblk) {
    m = A.meta[blk];
    o = A.out[blk];
    if (t < kRedSParts * 18) ps = sum_rows2(A.slab, m.x, m.y, t / 18, kRedSParts, t % 18);
    if (m.z >= 0 && t < kRedBParts * 6) pb = sum_rows<6>(A.slab_b, m.z, m.w, t / 6, kRedBParts, t % 6);
  } else if (iscost && A.nseg > 0) {
    for (int s = t; s < A.nseg; s += 4 * kRedThreads) {
      double v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = A.slab_cost[min(s + i * kRedThreads, A.nseg - 1)];
#pragma unroll
      for (int i = 0; i < 4; ++i) c += s + i * kRedThreads < A.nseg ? v[i] : 0.0;
    }
  }
  const bool failed = A.status && *A.status;  // a failed earlier step: nothing is written
  if (isblk) {
    if (t < kRedSParts * 18) reinterpret_cast<double2*>(part)[t] = ps;
    if (t < kRedBParts * 6) partb[t] = pb;
  } else if (iscost) {
    cpart[t] = c;
  }
  __syncthreads();
#if VO_BA_STAMPS
  if (rst && tid == 0) rst[1] = __builtin_amdgcn_s_memrealtime();
#endif
  if (isblk && !failed) {
    const bool diag = m.z >= 0;
    if (t < 36) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < kRedSParts; ++q) acc += part[36 * q + t];
      if (diag && t % 7 == 0) acc += A.lambda;
      st_sc1(A.sys + (o.x & ~kRedTranspose) + ((o.x & kRedTranspose) ? 6 * (t % 6) + t / 6 : t), acc);
    } else if (diag && t >= 64 && t < 70) {
      const int e = t - 64;
      double acc = 0.0;
      for (int q = 0; q < kRedBParts; ++q) acc += partb[6 * q + e];
      st_sc1(A.sys + o.y + e, acc);
    }
  }
  // the cost: K2's tree, in the one workgroup that holds the cost item (uniform per workgroup)
  if (A.nprof >= kBandRedItems * r && A.nprof < kBandRedItems * (r + 1))
    for (int mm = kRedThreads / 2; mm > 0; mm >>= 1) {
      if (iscost && t < mm) cpart[t] += cpart[t + mm];
      __syncthreads();
    }
  if (iscost && t == 0 && !failed) st_sc1(A.sys + A.cost_off, cpart[0]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores done
  __syncthreads();
  // one lane counts the workgroup, behind every storing wave's drain: with write-through (sc1)
  // stores and a consumer that reads every handed-off byte by sc1 loads, no release fence
  // (MI355X_MICROARCH.md, inter-workgroup visibility, hand-off table row 1, a sharded counter;
  // a fence here cost each reducer ~1.7 us of write-back on the solver's path)
  // lane 0 of each half counts its item in its column's counter, behind the barrier that follows
  // every storing wave's drain (the column's consumer loads only what the items it counted stored)
#if VO_BA_STAMPS
  if (rst && tid == 0) rst[2] = __builtin_amdgcn_s_memrealtime();
#endif
  if (t == 0 && (isblk || iscost)) {
    const unsigned v = __hip_atomic_fetch_add((gu32*)(B.red_count + kBandRedShardStride * col), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
#if VO_BA_STAMPS
    if (rst && tid == 0) rst[3] = __builtin_amdgcn_s_memrealtime() + (v & 0);
#endif
    (void)v;
  }
}

// Solver side of the fused launch: a column's readiness.  A polling wave reads the column's
// counter by relaxed sc1 loads, s_sleep between reads, bounded, until it holds col_need[c]; then
// takes the count back off (zero between launches).  No acquire: every load of sys is an sc1
// load (SysLoads), and a wave loads a column only after its own poll of that column matched;
// other waves read the column from LDS after a workgroup barrier (MI355X_MICROARCH.md,
// hand-off table row 1, one counter per column).  A timeout fails the solve ("failed"), which
// then uses nothing it read.
// Columns [c0, c1) at once, one lane each (64 per round): the loader's check of the columns after
// the prologue's (by step 0 their reducers are long done).  Wave-uniform loop.
__device__ __forceinline__ bool band_cols_wait(const BandArgs& A, int c0, int c1) {
  const int lane = threadIdx.x & 63;
  for (int b = c0; b < c1; b += 64) {
    const int c = b + lane;
    const bool on = c < c1;
    const unsigned need = on ? (unsigned)A.col_need[c] : 0u;
    gu32* cnt = (gu32*)(A.red_count + kBandRedShardStride * (on ? c : 0));
    unsigned spins = 0;
    for (;;) {
      const unsigned v = need ? __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      if (__builtin_amdgcn_ballot_w64(v < need) == 0) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) return false;
    }
    if (need) __hip_atomic_fetch_sub(cnt, need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

// The solver reads sys (written by the fused launch's reducers, or by K2) only by sc1 buffer
// loads: L2-served, never a stale L1 line, so the in-launch hand-off needs no acquire fence.
// Offsets in doubles; past the buffer's end a buffer load returns zero.
struct SysLoads {
  __amdgpu_buffer_rsrc_t r;
  __device__ explicit SysLoads(const double* sys, long n) {
    r = __builtin_amdgcn_make_buffer_rsrc((void*)sys, (short)0, (int)min(n * 8, (long)0x7fffffff), 0x00020000);
  }
  __device__ __forceinline__ double2 ld2(long off) const {  // 16 bytes at sys[off] (off even)
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off * 8), 0, 16);
    return __builtin_bit_cast(double2, v);
  }
  __device__ __forceinline__ double ld(long off) const {
    typedef int v2i __attribute__((ext_vector_type(2)));
    const v2i v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(off * 8), 0, 16);
    return __builtin_bit_cast(double, v);
  }
};

// Split mode's hand-offs between the two workgroups (same protocol as the fused reducers': the
// producer's stores write-through (sc1) and drained, then one relaxed agent-scope store of the
// flag; the consumer polls the flag relaxed and reads the data by sc1 loads only, after a
// workgroup barrier behind its poll).  Bounded: false after ~seconds (a workgroup that never
// arrived fails the solve instead of hanging it).
__device__ __forceinline__ void xch_flag_set(double* fac, long flag, unsigned seq) {
  __hip_atomic_store((gu32*)(fac + flag), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool xch_flag_wait(const double* fac, long flag, unsigned seq) {
  unsigned spins = 0;
  while (__hip_atomic_load((gu32*)(fac + flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != seq) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1u << 22)) return false;
  }
  return true;
}

// Loads below never feed a select or branch before their first real use: a value that
// must be zero is loaded from the zero block (A.zero) instead, so the waitcnt pass can
// leave every prefetch in flight.
// kMode: 0 ring (one workgroup, factor records in global memory), 1 full (one workgroup, both
// sides' columns in LDS), 2 split (one workgroup of four waves per side, each side's columns in
// its own CU's LDS; the separator's bottom contributions, the top's separator records and the
// separator's z cross over through global memory once each: see the split hand-offs below).
template <int kMode>
__global__ __launch_bounds__(kBandThreads) void ba_band_kernel(BandArgs A) {
  constexpr bool kFull = kMode != 0, kSplit = kMode == 2;
  constexpr int NT = kSplit ? kBandThreads / 2 : kBandThreads;  // threads of this workgroup
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  __shared__ int s_fail;
  __shared__ __attribute__((aligned(16))) double s_zero[40];   // full mode's zero block
#if VO_BA_STAMPS
  unsigned long long st_acc[kBandStamps] = {}, st_t = __builtin_amdgcn_s_memtime();
#endif
  // wave (so role and side) is wave-uniform: readfirstlane lets the compiler branch on SGPRs
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  // split mode: workgroup s is side s, its four waves the side's four roles
  if (A.nred > 0 && blockIdx.x > 0) {  // fused K2: a reducer workgroup (uniform branch)
    band_reduce_wg(A, blockIdx.x - 1, dyn);
    return;
  }
  // CS: doubles per column (K2 layout, factor record; full mode: SS == CS); SS per slot (ring mode: whole 1 KiB
  // pieces), RC slots per side (band_lds_layout)
  const int F = A.F, w = A.w, R = w + 1, CS = 36 * R + 12, CSP = (CS + 127) / 128 * 128;
  const int m = A.m, nb = A.nb, sp = A.s;
  const int ncolT = m + sp, ncolB = nb + sp;
  const int SS = kFull ? CS : CSP, RC = kFull ? max(ncolT, ncolB) : w + 4, SPAD = kFull ? 128 : 0;
  const int prior_word = A.status ? *A.status : 0;
  const bool prior_status = prior_word != 0;
  double* ringT = dyn;
  double* ringB = kSplit ? dyn : ringT + RC * SS + SPAD;  // split: each workgroup holds its own side
  double* zs = ringB + RC * SS + SPAD;  // back substitution: z (6F)
  double* pose_l = zs + 6 * F;
  // a zero block (masked loads) and a dummy row (masked stores), dyn offsets
  const int ZOFF = (int)(pose_l - dyn) + 12 * A.n_poses, DOFF = ZOFF + 40;
  // split mode, bottom workgroup: the top's separator records, 42 doubles a row (L_kk, 1/diag)
  double* const sepT = dyn + DOFF + 64;
  const SplitXch xch = split_xch(A.n_merge, A.s);

  const int side = kSplit ? (int)blockIdx.x : wave & 1, role = kSplit ? wave : wave >> 1;
  const bool sbot = side == 1;
  // this wave's side: ring (column v in slot v mod RC), factor records (column v at v *
  // CS: global memory, or the full-mode slots themselves), column sources, columns
  // factored before the merge, columns loaded into the ring
  double* const sring = sbot ? ringB : ringT;
  const double* const recT = kFull ? ringT : A.fac;  // the top side's records
  const double* const sfac = kFull ? sring : sbot ? A.fac + (long)ncolT * CS : A.fac;
  const long sbase = sbot ? (long)ncolT * CS : 0;  // this side's columns in sys (K2)
  const SysLoads sysl(A.sys, kFull ? A.cost_off + 1 : 0);
  const int sna = sbot ? nb : m, snload = sbot ? ncolB : ncolT;

  if (tid < 40) s_zero[tid] = 0.0;
  if (tid < 40) dyn[ZOFF + tid] = 0.0;
  // the poses for the tail's update, staged now (their load latency under the prologue's,
  // or under the wait for the fused launch's reducers)
  for (int e = tid; e < 12 * A.n_poses; e += NT) pose_l[e] = A.pose_cur[e];
  // fused K2 (one rank): sys is read column by column, each after its reducers have counted
  // themselves (the prologue's poll loop); a timeout fails the solve (status) without using what was read
  const bool fused = kFull && !kSplit && A.nred > 0;
  __shared__ int s_late;  // a column's reducers never arrived
  if (fused || kSplit) {  // (split mode: a hand-off that never arrived)
    if (tid == 0) s_late = 0;
    __syncthreads();
  }
#if VO_BA_STAMPS
  unsigned long long* sst = A.stamps ? A.stamps + 8 * kBandStamps : nullptr;
  if (sst && tid == 0) sst[0] = __builtin_amdgcn_s_memrealtime();
#endif
  if (fused) {
    // Prologue of a fused launch: the prologue columns (top 0 .. nTc - 1, then bottom 0 .. nBc -
    // 1) are dealt to the waves, column pc to wave pc mod 8; a wave issues a column's loads as soon
    // as that column's counter is full, keeping every issued column in flight while it polls the
    // next, so the loads overlap the later reducers.  Each loader wave then checks the rest of
    // its side's columns (the top one also the cost, which it hands to cost_out) -- their first
    // loads follow at step 0 -- and every wave stores its columns into the rings.
    const int nTc = min(w + 2, ncolT), nBc = min(w + 2, ncolB), np = nTc + nBc;
    static_assert(36 * (kBandMaxW + 1) + 12 <= 2 * 3 * 64, "three 16-byte pieces per lane and column");
    static_assert(2 * (kBandMaxW + 2) <= 3 * kBandWaves, "three prologue columns per wave");
    double2 pv[3][3];
    bool ok = true;
    // this wave's prologue columns u = 0..2 (pc = wave + 8 u): side, column and counter (-1: a
    // bottom separator column, which K2 does not write: no wait)
    int uc[3], ucid[3];
    bool utop[3];
    unsigned pend = 0;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int pc = wave + kBandWaves * u;
      utop[u] = pc < nTc;
      uc[u] = utop[u] ? pc : pc - nTc;
      ucid[u] = pc >= np ? -1 : utop[u] ? uc[u] : (uc[u] < nb ? ncolT + uc[u] : -1);
      if (pc < np) pend |= 1u << u;
    }
    auto issue = [&](int u) __attribute__((always_inline)) {
      const long base = (utop[u] ? 0 : (long)ncolT * CS) + (long)uc[u] * CS;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int piece = lane + 64 * t;
        pv[u][t] = sysl.ld2(base + 2 * (long)min(piece, CS / 2 - 1));
      }
    };
    // One poll of every pending column per round -- lane u < 3 this wave's prologue column u, and
    // on the loader waves lanes 3.. the rest of their side's columns (whose loads follow from step
    // 0) and, on the top loader, the cost -- so a wave pays one round trip per round, not one per
    // column; a prologue column's loads are issued in the round its counter is found full, so the
    // first columns' loads overlap the wait for the slower reducers.
    const int r0 = sbot ? ncolT + nBc : nTc, r1 = sbot ? ncolT + nb : ncolT;  // the loader's rest
    const int nrest = role == kLoad ? min(max(r1 - r0, 0), 60) + (sbot ? 0 : 1) : 0;  // + the cost (top)
    const int lcid = lane < 3 ? (lane == 0 ? ucid[0] : lane == 1 ? ucid[1] : ucid[2])
                     : lane - 3 < nrest ? (lane - 3 < min(max(r1 - r0, 0), 60) ? r0 + lane - 3 : F) : -1;
    bool lpend = lcid >= 0 && (lane >= 3 || ((pend >> lane) & 1u));
    const unsigned need = lpend ? (unsigned)A.col_need[lcid] : 0u;
    gu32* const cnt = (gu32*)(A.red_count + kBandRedShardStride * (lcid >= 0 ? lcid : 0));
    if (need == 0) lpend = false;
    // prologue columns with nothing to wait for (K2 writes no bottom separator column): at once
    const unsigned waiting = (unsigned)__builtin_amdgcn_ballot_w64(lpend) & 7u;
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (((pend >> u) & 1u) && !((waiting >> u) & 1u)) issue(u);
    unsigned spins = 0;
    for (;;) {
      const unsigned v = lpend ? __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      const bool now = lpend && v >= need;
      const uint64_t nowb = __builtin_amdgcn_ballot_w64(now);
      if (nowb & 1u) issue(0);
      if (nowb & 2u) issue(1);
      if (nowb & 4u) issue(2);
      if (now) __hip_atomic_fetch_sub(cnt, need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lpend = lpend && !now;
      if (__builtin_amdgcn_ballot_w64(lpend) == 0) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {  // seconds (a reducer never arrived): fail, do not hang
        ok = false;
        break;
      }
    }
    if (role == kLoad && ok && r1 - r0 > 60) ok = band_cols_wait(A, r0 + 60, r1);  // wide windows only
    if (role == kLoad && !sbot && ok && lane == 0 && A.cost_out) *A.cost_out = sysl.ld(A.cost_off);
    if (!ok && lane == 0) s_late = 1;
    BST(15);
#if VO_BA_STAMPS
    if (sst && tid == 0) sst[1] = __builtin_amdgcn_s_memrealtime();
#endif
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int pc = wave + kBandWaves * u;
      if (pc < np) {
        const bool top = pc < nTc;
        const int c = top ? pc : pc - nTc;
        double* dst = (top ? ringT : ringB) + c * SS;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const int piece = lane + 64 * t;
          if (piece < CS / 2) *reinterpret_cast<double2*>(dst + 2 * piece) = pv[u][t];
        }
      }
    }
  } else {
    if (tid == 0 && A.cost_out && side == 0) *A.cost_out = A.sys[A.cost_off];  // plain-sys-read: not fused
    // Prologue: columns 0 .. w + 1 of both sides (contiguous in K2's layout), every 16-byte
    // load in flight, then the stores.  The loads do not wait for the status word (one
    // global round trip less on the launch's path); a failed earlier solve only skips the
    // stores.
    // (split mode: each workgroup its own side's columns)
    const int nT = kSplit && sbot ? 0 : min(w + 2, ncolT) * CS / 2;  // double2 pieces
    const int nB = kSplit && !sbot ? 0 : min(w + 2, ncolB) * CS / 2;
    static_assert((kBandMaxW + 2) * (36 * (kBandMaxW + 1) + 12) / 2 <= kProLoads * kBandThreads / 2,
                  "split prologue: one side's columns per four-wave workgroup");
    double2 v[kProLoads];
#pragma unroll
    for (int u = 0; u < kProLoads; ++u) {
      const int e = tid + u * NT;
      const long o2 = e < nT ? e : (long)ncolT * CS / 2 + (e - nT);
      v[u] = e < nT + nB ? reinterpret_cast<const double2*>(A.sys)[o2] : make_double2(0.0, 0.0);  // plain-sys-read: not fused
    }
    if (!prior_status)
#pragma unroll
    for (int u = 0; u < kProLoads; ++u) {
      const int e = tid + u * NT;
      const bool top = e < nT;
      const int x = 2 * (top ? e : e - nT), col = x / CS;
      if (e < nT + nB)
        *reinterpret_cast<double2*>((top ? ringT : ringB) + col * SS + x - col * CS) = v[u];
    }
  }

  // ---- loader wave, nDma 1 KiB wave pieces (16 bytes per lane) per column.  In a fused launch
  // (full mode; sys from this launch's reducers): sc1 register loads, written into the column's
  // LDS slot one step later (the loads in flight across the barrier); otherwise (sys from an
  // earlier launch): LDS-DMA.  The ring-mode kernel carries no sc1 path (its registers and the
  // buffer descriptor pushed it past 256 VGPRs into spills: cfg4 K3 77 -> 89 us).
  const int nDma = CSP / 128;
  const bool ld_sc1 = kFull && !kSplit && A.nred > 0;
  static_assert(36 * (kBandMaxW + 1) + 12 <= 3 * 128, "at most three 1 KiB pieces per column");
  double2 ldv[3];
  int ld_pend = -1;  // the column whose pieces are in ldv
  auto col_issue = [&](int v) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 3; ++t) ldv[t] = sysl.ld2(sbase + (long)v * CS + 2 * lane + 128 * t);
    ld_pend = v;
  };
  auto col_write = [&]() __attribute__((always_inline)) {
    if (ld_pend < 0) return;
    double* slot = sring + (kFull ? ld_pend : ld_pend % RC) * SS;
#pragma unroll
    for (int t = 0; t < 3; ++t)
      if (t < nDma && 128 * t + 2 * lane < CS) *reinterpret_cast<double2*>(slot + 128 * t + 2 * lane) = ldv[t];
    ld_pend = -1;
  };
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) const void gbl_void;
  auto dma_col = [&](int v, double* slot) __attribute__((always_inline)) {
    const double* src = A.sys + sbase + (long)v * CS + 2 * lane;  // plain-sys-read: LDS-DMA, not fused (ld_sc1 false)
    for (int t = 0; t < nDma; ++t)
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + 128 * t), (lds_void*)(slot + 128 * t), 16, 0, 0);
  };
  // every DMA but the last column's nDma pieces complete
  auto dma_wait_prev = [&]() __attribute__((always_inline)) {
    if (nDma == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if (nDma == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  };
  // ---- trailing wave: task lane + 64 h = block (k + qi, k + qj), rows r and r + 3
  // (blocks by qj, then qi): target column offset qj, offsets of the target row r, of
  // L_{k+qi,k} row r, of L_{k+qj,k}
  int tk_qj[kTaskRounds], tk_o[kTaskRounds], tk_a[kTaskRounds], tk_b[kTaskRounds];
  {
    const int nt = 3 * (w - 1) * w / 2;
#pragma unroll
    for (int h = 0; h < kTaskRounds; ++h) {
      const int t = lane + 64 * h;
      int qj = 0, qi = 0, r = 0;
      if (t < nt) {
        int b = t / 3;
        r = t - 3 * b;
        qj = 2;
        while (b >= w - qj + 1) {
          b -= w - qj + 1;
          ++qj;
        }
        qi = qj + b;
      }
      tk_qj[h] = t < nt ? qj : -1;
      tk_o[h] = 36 * (qi - qj) + 6 * r;
      tk_a[h] = 36 * qi + 6 * r;
      tk_b[h] = 36 * qj;
    }
  }
  band_barrier();
  BST(0);
#if VO_BA_STAMPS
  if (sst && tid == 0) sst[2] = __builtin_amdgcn_s_memrealtime();
#endif
  // every wave's polls are behind the barrier: one verdict for the whole solve
  const bool reduced = !fused || s_late == 0;
  const bool prior_fail = prior_status || !reduced;
  if (tid == 0) s_fail = prior_fail ? 1 : 0;

  // ---- chain wave: lane 6 g + sr holds row sr of block (k + q, k), q = (g - k) mod R
  const bool act = role == kChain && lane < 6 * R;
  const int g = lane / 6, sr = lane % 6;
  int q = act ? g : 0;
  double P[6] = {0, 0, 0, 0, 0, 0};
  double L1[6][6];  // L_{k+1,k}, read at the end of step k's factor phase
  bool bad = false;
  if (act && !prior_fail && sna > 0) ld6g(sring + 36 * g + 6 * sr, P);  // column 0 (slot 0), block g

  // Step k, before the barrier (column k in slot sk): factor the diagonal block, solve
  // this lane's panel row, write the panel and 1/diag into the ring.
  auto chain_pre = [&](int k, int sk) __attribute__((always_inline)) {
    double* col = sring + sk * SS;
    const int ocol = (int)(col - dyn);
    double L[21], r[6];
    // the diagonal block's rows (group q == 0) to every lane through LDS (other lanes
    // store to the dummy row: no divergent code on the chain)
    {
      int o = (act & (q == 0)) ? ocol + 6 * sr : DOFF;
      asm volatile("" : "+v"(o));
      st6g(dyn + o, P);
    }
    wave_sync<true>();
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int c = 0; c <= i; c += 2) {
        const double2 v = reinterpret_cast<const double2*>(col + 6 * i)[c / 2];
        L[P6(i, c)] = v.x;
        if (c + 1 <= i) L[P6(i, c + 1)] = v.y;
      }
    BSETTLE(L[20]);
    BSTF(17);
    chol6_nochk(L, r);
    bad = bad | !(isfinite(r[0] + r[1] + r[2] + r[3] + r[4] + r[5]));
    BSETTLE(r[5]);
    BSTF(18);
    fwd6(L, r, P);  // x L_kk^T = row; on the diagonal group: row sr of L_kk
    BSETTLE(P[5]);
    BSTF(19);
    {
      int o = act ? ocol + 36 * q + 6 * sr : DOFF;
      int o2 = (act & (q == 0)) ? ocol + 36 * R + 6 + sr : DOFF + 8;
      asm volatile("" : "+v"(o), "+v"(o2));
      st6g(dyn + o, P);
      dyn[o2] = pick<6>(r, sr);
    }
    wave_sync<true>();
    // L_{k+1,k} for the update after the barrier: issued now, its latency under the wait
    if (w >= 1)
#pragma unroll
      for (int c = 0; c < 6; ++c) ld6g(col + 36 + 6 * c, L1[c]);
  };
  // Step k, after the barrier: this lane's row of column k + 1 (every earlier step's
  // update applied by the trailing wave) minus L_{i,k} L_{k+1,k}^T.
  auto chain_post = [&](int sk1) __attribute__((always_inline)) {
    const int q1 = q == 0 ? w : q - 1;
    double N[6];
    int o = act ? (int)(sring - dyn) + sk1 * SS + 36 * q1 + 6 * sr : ZOFF;
    asm volatile("" : "+v"(o));
    ld6g(dyn + o, N);
    BSETTLE(N[5]);
    BSTF(22);
    if (w >= 1) {
      const bool upd = q != 0;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        double u = N[c] - (P[0] * L1[c][0] + P[1] * L1[c][1] + P[2] * L1[c][2] + P[3] * L1[c][3] +
                           P[4] * L1[c][4] + P[5] * L1[c][5]);
        asm volatile("" : "+v"(u));
        N[c] = upd ? u : N[c];
      }
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) P[c] = N[c];  // non-chain lanes load the zero block
    q = q1;
    BSETTLE(P[5]);
    BSTF(23);
  };
  // Forward-substitution wave, step k: y'_k = L_kk^-1 y_k into the record, y_i -= L_ik
  // y'_k for the rows below (lane 6 qf + rf, qf = 1..w), then the factor record of column
  // k (blocks, y'_k, 1/diag) to global memory.
  auto fwd_step = [&](int k, int sk) __attribute__((always_inline)) {
    double* col = sring + sk * SS;
    double L[21], r[6], y[6], row[6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int c = 0; c <= i; c += 2) {
        const double2 v = reinterpret_cast<const double2*>(col + 6 * i)[c / 2];
        L[P6(i, c)] = v.x;
        if (c + 1 <= i) L[P6(i, c + 1)] = v.y;
      }
    ld6g(col + 36 * R + 6, r);
    ld6g(col + 36 * R, y);
    const int qf = lane / 6, rf = lane % 6;
    const bool on = (qf >= 1) & (qf < R) & (k + qf < snload);  // rows past the side: none
    ld6g(col + (on ? 36 * qf + 6 * rf : 0), row);
    // the rhs entry this lane updates, read with the other operands (its latency under fwd6)
    const int st = sk + qf < RC ? sk + qf : sk + qf - RC;
    int o = on ? (int)(sring - dyn) + st * SS + 36 * R + rf : DOFF + lane;
    int o2 = lane < 6 ? (int)(col - dyn) + 36 * R + lane : DOFF + lane;
    asm volatile("" : "+v"(o), "+v"(o2));
    const double yo = dyn[o];
    BSETTLE(row[5]);
    BSTF(24);
    fwd6(L, r, y);
    bad = bad | !isfinite(y[0] + y[1] + y[2] + y[3] + y[4] + y[5]);
    BSETTLE(y[5]);
    BSTF(25);
    dyn[o] = yo - (row[0] * y[0] + row[1] * y[1] + row[2] * y[2] + row[3] * y[3] + row[4] * y[4] + row[5] * y[5]);
    dyn[o2] = pick<6>(y, lane);
    BSETTLE(y[0]);
    BSTF(27);
  };
  // Ring mode: the factor record of column kc (blocks, y', 1/diag; in slot sc) to global
  // memory, by the trailing wave one step after its forward substitution (the fwd wave is
  // the ring's slowest role otherwise).  The ring has w + 4 slots, so the loader refills
  // column kc's slot only a step later, after the barrier that retires these reads.
  // The three 16-byte pieces per lane go out in one asm block: issued together from three
  // register tuples (compiled stores would share one tuple and wait for each other), after
  // all of the wave's LDS work of the step; they complete under the next barrier and the
  // vmcnt(0) drain after the elimination covers them.
  typedef __attribute__((ext_vector_type(4))) int i32x4;
  auto rec_load = [&](int sc, i32x4 (&v2)[3]) __attribute__((always_inline)) {
    const i32x4* s2 = reinterpret_cast<const i32x4*>(sring + sc * SS);
#pragma unroll
    for (int t = 0; t < 3; ++t) v2[t] = s2[min(lane + 64 * t, CS / 2 - 1)];
  };
  auto rec_store = [&](int kc, const i32x4 (&v2)[3]) __attribute__((always_inline)) {
    i32x4* d2 = reinterpret_cast<i32x4*>(const_cast<double*>(sfac) + (long)kc * CS);
    const bool t2 = lane + 128 < CS / 2;
    i32x4* a0 = d2 + lane;
    i32x4* a1 = d2 + lane + 64;
    i32x4* a2 = d2 + (t2 ? lane + 128 : lane);  // masked lanes rewrite their first piece
    const i32x4 v2b = t2 ? v2[2] : v2[0];
    asm volatile(
        "global_store_dwordx4 %0, %3, off\n\t"
        "global_store_dwordx4 %1, %4, off\n\t"
        "global_store_dwordx4 %2, %5, off" ::"v"(a0),
        "v"(a1), "v"(a2), "v"(v2[0]), "v"(v2[1]), "v"(v2b)
        : "memory");
  };
  // Trailing wave, step k: blocks (i, j), k + 2 <= j <= i <= k + w, minus L_ik L_jk^T.
  auto trail_step = [&](int k, int sk) __attribute__((always_inline)) {
    const double* col = sring + sk * SS;
#pragma unroll
    for (int h = 0; h < kTaskRounds; ++h) {
      if (tk_qj[h] < 0 || k + tk_qj[h] >= snload) continue;  // no column past the side
      const int st = sk + tk_qj[h] < RC ? sk + tk_qj[h] : sk + tk_qj[h] - RC;
      double* out = sring + st * SS + tk_o[h];
      double o0[6], o1[6], a0[6], a1[6], B[6][6];
      ld6g(out, o0);
      ld6g(out + 18, o1);
      ld6g(col + tk_a[h], a0);
      ld6g(col + tk_a[h] + 18, a1);
#pragma unroll
      for (int c = 0; c < 6; ++c) ld6g(col + tk_b[h] + 6 * c, B[c]);
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        o0[c] -= a0[0] * B[c][0] + a0[1] * B[c][1] + a0[2] * B[c][2] + a0[3] * B[c][3] + a0[4] * B[c][4] +
                 a0[5] * B[c][5];
        o1[c] -= a1[0] * B[c][0] + a1[1] * B[c][1] + a1[2] * B[c][2] + a1[3] * B[c][3] + a1[4] * B[c][4] +
                 a1[5] * B[c][5];
      }
      st6g(out, o0);
      st6g(out + 18, o1);
    }
  };
  // Loader wave, step k, sc1: the column loaded at step k - 1 (k + w + 1) into its slot (ring
  // mode: column c in slot c mod (w + 4), i.e. column k - 3's, whose record the trailing wave
  // copied two steps ago; first read at step k + 1, after this step's barrier), then the loads
  // of column k + w + 2.  LDS-DMA: column k + w + 2 issued into its slot (column k - 2's, whose
  // record the trailing wave copied a step ago), then the previous column's pieces retired.
  auto load_step = [&](int k) __attribute__((always_inline)) {
    if (kFull && ld_sc1) {
      col_write();
      BSTF(21);
      if (k + w + 2 < snload) col_issue(k + w + 2);
      BSTF(20);
    } else if (k + w + 2 < snload) {
      dma_col(k + w + 2, sring + (kFull ? k + w + 2 : (k + w + 2) % RC) * SS);
      BSTF(20);
      dma_wait_prev();
      BSTF(21);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };
  auto side_step = [&](int p, int sk, int skm) __attribute__((always_inline)) {
    if (role == kTrail) {
      // ring mode: column p - 1's record read first (its latency under the trailing
      // update), stored to global memory last
      i32x4 v2[3];
      if (!kFull && p >= 1) rec_load(skm, v2);
      trail_step(p, sk);
      if (!kFull && p >= 1) rec_store(p - 1, v2);
    } else if (role == kFwd) {
      fwd_step(p, sk);
    } else if (role == kLoad) {
      load_step(p);
    }
  };

  // Full mode: every block L_{k,i} (k - w <= i < k) is replaced by G = L_kk^-1 L_{k,i}
  // before the back substitution, one block column per thread (L_kk from this side's
  // record, or for the bottom side's separator rows from the top's).  Item e = 6 b + s2:
  // column s2 of block b of the lists: set 0 = the rows final after phase A (top rows < m,
  // then bottom rows < nb; done by the idle bottom waves during the separator phase),
  // set 1 = the separator rows (top rows m .. m + s, then the bottom side's pseudo rows
  // nb .. nb + s).
  auto g_item = [&](int set, int e) __attribute__((always_inline)) {
    const int bi = e / 6, s2 = e - 6 * bi;
    const int nt = (set == 0 ? m : sp) * w;
    const bool eb = bi >= nt;
    const int e2 = eb ? bi - nt : bi, k = e2 / w + (set == 0 ? 0 : eb ? nb : m), qq = e2 % w + 1, i = k - qq;
    if (i < 0 || (eb && i >= nb)) return;
    double* fs = eb ? ringB : ringT;
    // the bottom side's pseudo rows take the top's separator record (split mode: its staged copy,
    // 42 doubles a row with 1/diag at 36)
    const bool xrec = eb && k >= nb;
    const double* rec = xrec ? (kSplit ? sepT + 42l * (F - 1 - k - m) : ringT + (long)(F - 1 - k) * CS) : fs + (long)k * CS;
    const int roff = kSplit && xrec ? 36 : 36 * R + 6;
    double L[21], r[6], gv[6];
#pragma unroll
    for (int ii = 0; ii < 6; ++ii)
#pragma unroll
      for (int c = 0; c <= ii; c += 2) {
        const double2 v = reinterpret_cast<const double2*>(rec + 6 * ii)[c / 2];
        L[P6(ii, c)] = v.x;
        if (c + 1 <= ii) L[P6(ii, c + 1)] = v.y;
      }
    ld6g(rec + roff, r);
    double* col = fs + (long)i * CS + 36 * qq + s2;
#pragma unroll
    for (int c = 0; c < 6; ++c) gv[c] = col[6 * c];
    fwd6(L, r, gv);
#pragma unroll
    for (int c = 0; c < 6; ++c) col[6 * c] = gv[c];
  };

  if (!prior_fail) {
    const int PA = kSplit ? sna : max(m, nb);
    int sk = 0, skm = RC - 1;
    for (int p = 0; p < PA; ++p) {
      const bool on = p < sna;
      const int sk1 = sk + 1 == RC ? 0 : sk + 1;
      if (role == kChain && on) chain_pre(p, sk);
      BST(1);
      band_barrier();
      BST(2);
      if (on) {
        if (role == kChain) {
          if (p + 1 < snload) chain_post(sk1);
        } else {
          side_step(p, sk, skm);
          // split mode: the loader (half idle: its DMA waits) forms the G blocks of row p - 1,
          // final since step p - 1 (its diagonal block) and unused by any later step; a side's
          // last row follows after phase A
          if (kSplit && role == kLoad && p >= 1 && lane < 6 * w) g_item(0, 6 * ((sbot ? m * w : 0) + (p - 1) * w) + lane);
        }
      }
      BST(3);
      skm = sk;
      sk = sk1;
    }
    if (sp > 0) {
      // both sides' state of the separator into the rings, the bottom's contributions
      // merged into the top's (fixed order), then the top continues through the separator
      if (act) st6g(sring + (sna % RC) * SS + 36 * q + 6 * sr, P);
      if constexpr (kSplit) {
        // split hand-off 0: the bottom's separator contributions (the merge table's sources,
        // at their offsets in a two-ring layout less offB) and its failure word go out; the
        // top adds them in the table's order, as the one-workgroup merge does
        const int offB = RC * SS + SPAD;
        if (lane == 0 && bad) s_fail = 1;
        __syncthreads();
        if (sbot) {
          for (int e = tid; e < A.n_merge; e += NT) {
            const int2 d = reinterpret_cast<const int2*>(A.tab + A.merge)[e];
            st_sc1(A.fac + xch.merge + e, dyn[d.y - offB]);
          }
          if (tid == 0) st_sc1(A.fac + xch.fail, s_fail ? 1.0 : 0.0);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid == 0) xch_flag_set(A.fac, xch.flag, A.seq);
          // the G blocks of the bottom's last row (the loader formed the others during phase A)
          for (int e = tid; e < 6 * w; e += NT) g_item(0, 6 * (m * w + (nb - 1) * w) + e);
        } else {
          if (tid == 0 && !xch_flag_wait(A.fac, xch.flag, A.seq)) s_late = 1;
          for (int e = tid; e < 6 * w; e += NT) g_item(0, 6 * (m - 1) * w + e);  // the top's last row
          __syncthreads();
          const SysLoads xl(A.fac, xch.end());
          for (int e = tid; e < A.n_merge; e += NT) {
            const int2 d = reinterpret_cast<const int2*>(A.tab + A.merge)[e];
            dyn[d.x] += xl.ld(xch.merge + e);
          }
          if (tid == 0 && (s_late || xl.ld(xch.fail) != 0.0)) s_fail = 1;
          __syncthreads();
          if (act) ld6g(ringT + (m % RC) * SS + 36 * q + 6 * sr, P);
        }
      } else {
        __syncthreads();
        for (int e = tid; e < A.n_merge; e += NT) {
          const int2 d = reinterpret_cast<const int2*>(A.tab + A.merge)[e];
          dyn[d.x] += dyn[d.y];
        }
        __syncthreads();
        if (act && side == 0) ld6g(ringT + (m % RC) * SS + 36 * q + 6 * sr, P);
      }
      BST(4);
      int sk = m % RC, skm = sk == 0 ? RC - 1 : sk - 1;
      for (int p = m; p < (kSplit && sbot ? m : m + sp); ++p) {
        const int sk1 = sk + 1 == RC ? 0 : sk + 1;
        if (role == kChain && side == 0) chain_pre(p, sk);
        BST(5);
        band_barrier();
        BST(6);
        if (side == 0) {
          if (role == kChain) {
            if (p + 1 < ncolT) chain_post(sk1);
          } else {
            side_step(p, sk, skm);
          }
        } else if (kFull) {
          const int n0 = 6 * (m + nb) * w, chunk = (n0 + sp - 1) / sp, t = p - m;
          const int e1 = min(n0, (t + 1) * chunk);
          for (int e = t * chunk + 64 * role + lane; e < e1; e += 256) g_item(0, e);
        }
        BST(7);
        skm = sk;
        sk = sk1;
      }
    }
  }
  if (!kFull && !prior_fail) {  // each side's last record (no later step copies it)
    band_barrier();
    const int last = sbot ? nb - 1 : ncolT - 1;
    if (role == kTrail && last >= 0) {
      i32x4 v2[3];
      rec_load(last % RC, v2);
      rec_store(last, v2);
    }
  }
  if (lane == 0 && bad) s_fail = 1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // factor records written
  BST(8);
  __syncthreads();
  if constexpr (kSplit) {
    // split hand-off 1: the top's separator records (L_kk's rows and 1/diag: the bottom's pseudo
    // rows form their G blocks from them) and the top's failure word (both sides' phase-A state
    // and the separator's) out; the bottom stages the records in sepT
    if (!prior_fail && sp > 0) {
      if (!sbot) {
        for (int e = tid; e < 42 * sp; e += NT) {
          const int k = m + e / 42, o = e % 42;
          st_sc1(A.fac + xch.rec + e, ringT[(long)k * SS + (o < 36 ? o : 36 * R + 6 + (o - 36))]);
        }
        if (tid == 0) st_sc1(A.fac + xch.fail + 1, s_fail ? 1.0 : 0.0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) xch_flag_set(A.fac, xch.flag + 16, A.seq);
      } else {
        if (tid == 0 && !xch_flag_wait(A.fac, xch.flag + 16, A.seq)) s_late = 1;
        __syncthreads();
        const SysLoads xl(A.fac, xch.end());
        for (int e = tid; e < 42 * sp; e += NT) sepT[e] = xl.ld(xch.rec + e);
        if (tid == 0 && (s_late || xl.ld(xch.fail + 1) != 0.0)) s_fail = 1;
        __syncthreads();
      }
    }
  }
  BST(9);
  const bool failed = s_fail != 0;

  // ---- back substitution L^T x = y'.  z_k = y'_k - sum_{q=1..w} L_{k+q,k}^T x_{k+q} runs
  // down the chain; x_k = L_kk^-T z_k is taken off it: x_k's share of the lane's row
  // j = k - q is g . z_k with g = L_kk^-1 (column sr of L_{k,j}), formed from operands
  // fetched two steps ahead.  A chain step is the readlane broadcast of z_k from the
  // lanes holding it plus 6 FMAs; every x_k is formed in parallel at the end from z (LDS)
  // and the factor records.
  // Full mode, the rest of the G blocks (rows the separator phase finalised: the top's
  // separator rows and the bottom side's pseudo rows), then the back substitution.
  if (kFull && !failed) {
    if constexpr (kSplit) {  // the top: its separator rows
      if (!sbot) {  // (its rows before the separator: during phase A and after it)
        for (int e = tid; e < 6 * sp * w; e += NT) g_item(1, e);
      } else {  // the bottom: its pseudo rows (its own rows: during phase A and after it)
        for (int e = 6 * sp * w + tid; e < 12 * sp * w; e += NT) g_item(1, e);
      }
    } else {
      const int nR = 6 * (sp > 0 ? 2 * sp * w : m * w);  // one-sided windows: every top row here
      for (int e = tid; e < nR; e += NT) g_item(sp > 0 ? 1 : 0, e);
    }
    __syncthreads();
  }
  BST(16);
  // masked operands come from a zero block in the records' address space (LDS loads stay
  // ds_read, not flat)
  const double* const zsrc = kFull ? s_zero : A.zero;
  double Yb = 0.0;
  int qb = 0;  // this lane's window row at the current step k is k - qb
  auto bs_init = [&](int khi, int kp) __attribute__((always_inline)) {
    qb = act ? ((khi - g) % R + R) % R : 0;
    if (act) {
      const int i = khi - qb;
      const bool on = i >= 0 && i < kp;
      Yb = *(on ? sfac + (long)i * CS + 36 * R + sr : zsrc);
    }
  };
  struct BsOps {
    double L[21], r[6], Lc[6], yin;
  };
  // operands of step k for a lane at window position qk: L_kk and 1/diag (this side's
  // record k, clamped; for the bottom side's separator rows k >= kp, the top's record
  // F - 1 - k), column sr of L_{k,k-qk} (zero unless the lane's row is live), and the y'
  // of the row entering the window (k - w - 1) for the lane leaving it.
  auto bs_fetch = [&](int k, int qk, int kp, BsOps& o) __attribute__((always_inline)) {
    if (!kFull) {  // full mode: g precomputed in place of the block
    const double* rec = k >= kp ? recT + (long)(F - 1 - k) * CS : sfac + (long)max(k, 0) * CS;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int c = 0; c <= i; c += 2) {
        const double2 v = reinterpret_cast<const double2*>(rec + 6 * i)[c / 2];
        o.L[P6(i, c)] = v.x;
        if (c + 1 <= i) o.L[P6(i, c + 1)] = v.y;
      }
    ld6g(rec + 36 * R + 6, o.r);
    }
    const int i = k - qk;
    const bool on = act && qk >= 1 && i >= 0 && i < kp;
    const double* rc = on ? sfac + (long)i * CS + 36 * qk + sr : zsrc;
#pragma unroll
    for (int c = 0; c < 6; ++c) o.Lc[c] = rc[6 * c];
    const int ie = k - R;
    const bool on2 = act && qk == 0 && ie >= 0 && ie < kp;
    o.yin = *(on2 ? sfac + (long)ie * CS + 36 * R + sr : zsrc);
  };
  auto bs_step = [&](int k, int kp, int g0, BsOps& o) __attribute__((always_inline)) {
    if (!kFull) fwd6(o.L, o.r, o.Lc);  // g, independent of z_k
    double z[6];
    const int G = sbot ? F - 1 - k : k;
    // z's LDS accesses in asm: a compiled LDS access here would first wait for every
    // outstanding global load (LDS-DMA shares the counter), i.e. for the prefetched operands
    // of the next two steps
    if (k >= kp) {
      const uint32_t a = (uint32_t)(uintptr_t)(zs + 6 * G);  // the separator's z (top side)
      asm volatile(
          "ds_read_b128 %0, %3\n\t"
          "ds_read_b128 %1, %3 offset:16\n\t"
          "ds_read_b128 %2, %3 offset:32\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=v"(*reinterpret_cast<double2*>(&z[0])), "=v"(*reinterpret_cast<double2*>(&z[2])),
            "=v"(*reinterpret_cast<double2*>(&z[4]))
          : "v"(a)
          : "memory");
    } else {
      // z_k to every lane through LDS (the lanes holding it store it, the others to the dummy
      // row; LDS ops of one wave complete in order): one round trip instead of 12 v_readlanes
      // and their SGPR hazards (~17 cycles per dword measured)
      (void)g0;
      const uint32_t aw = (uint32_t)(uintptr_t)((act && qb == 0) ? zs + 6 * G + sr : dyn + DOFF + lane);
      const uint32_t ar = (uint32_t)(uintptr_t)(zs + 6 * G);
      asm volatile(
          "ds_write_b64 %3, %4\n\t"
          "ds_read_b128 %0, %5\n\t"
          "ds_read_b128 %1, %5 offset:16\n\t"
          "ds_read_b128 %2, %5 offset:32\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(*reinterpret_cast<double2*>(&z[0])), "=&v"(*reinterpret_cast<double2*>(&z[2])),
            "=&v"(*reinterpret_cast<double2*>(&z[4]))
          : "v"(aw), "v"(Yb), "v"(ar)
          : "memory");
    }
    if (act && qb >= 1)
      Yb -= o.Lc[0] * z[0] + o.Lc[1] * z[1] + o.Lc[2] * z[2] + o.Lc[3] * z[3] + o.Lc[4] * z[4] + o.Lc[5] * z[5];
    if (act && qb == 0) Yb = o.yin;
    qb = qb == 0 ? w : qb - 1;
  };
  auto dec = [&](int x) __attribute__((always_inline)) { return x == 0 ? w : x - 1; };
  auto bs_run = [&](int khi, int klo, int kp) __attribute__((always_inline)) {
    BsOps o0, o1;
    int qa = dec(dec(qb)), qc = dec(qa);  // window positions of steps khi - 2, khi - 3
    bs_fetch(khi, qb, kp, o0);
    bs_fetch(khi - 1, dec(qb), kp, o1);
    int g0 = khi % R;  // the group at window position 0 (holding z_k) at step k
    int k = khi;
    for (; k - 1 >= klo; k -= 2) {
      bs_step(k, kp, g0, o0);
      bs_fetch(k - 2, qa, kp, o0);
      g0 = dec(g0);
      bs_step(k - 1, kp, g0, o1);
      bs_fetch(k - 3, qc, kp, o1);
      g0 = dec(g0);
      BSTF(26);
      qa = dec(dec(qa));
      qc = dec(dec(qc));
    }
    if (k >= klo) bs_step(k, kp, g0, o0);
  };
  // Full mode: the same steps with LDS operands and no divergent code.  A lane's row j =
  // k - qb stays fixed while it crosses the window, so its g address is its row's record
  // plus 36 per step; z_k goes through LDS (the qb == 0 lanes store it, every lane reads
  // it back: the store is the one zs needs anyway).
  auto bs_run_full = [&](int khi, int klo, int kp) __attribute__((always_inline)) {
    // offsets into dyn; selects kept opaque so that they stay v_cndmask, not branches
    const int sbase = (int)(sring - dyn);
    int qf = qb, kf = khi;
    int pf = sbase + (khi - qb) * CS + 36 * qb + sr;  // g of the step being fetched (if live)
    auto fetch = [&](double (&gv)[6], double& yin) __attribute__((always_inline)) {
      const int jf = kf - qf;
      const bool on = act & (qf >= 1) & (jf >= 0) & (jf < kp);
      int og = on ? pf : ZOFF;
      asm volatile("" : "+v"(og));
      const double* pg = dyn + og;
      gv[0] = pg[0]; gv[1] = pg[6]; gv[2] = pg[12]; gv[3] = pg[18]; gv[4] = pg[24]; gv[5] = pg[30];
      int oy = kf - R >= 0 ? sbase + (kf - R) * CS + 36 * R + sr : ZOFF;
      asm volatile("" : "+v"(oy));
      yin = dyn[oy];
      --kf;
      const bool wrap = qf == 0;
      qf = wrap ? w : qf - 1;
      pf = wrap ? pf - R * CS + 36 * w : pf - 36;
    };
    int zk = (int)(zs - dyn) + 6 * (sbot ? F - 1 - khi : khi);  // z_k of the current step
    const int dz = sbot ? 6 : -6;
    // a step also fetches the operands of the step two ahead, issued after its z reads: LDS
    // reads of one wave complete in order, so reads issued before them would delay z_k
    auto step = [&](int k, const double (&gv)[6], double yin, double (&gn)[6], double& yn) __attribute__((always_inline)) {
      int ow = ((k < kp) & act & (qb == 0)) ? zk + sr : DOFF + lane;
      asm volatile("" : "+v"(ow));
      dyn[ow] = Yb;
      double z[6];
      ld6g(dyn + zk, z);
      asm volatile("" ::: "memory");
      fetch(gn, yn);
      double d = gv[0] * z[0] + gv[1] * z[1] + gv[2] * z[2] + gv[3] * z[3] + gv[4] * z[4] + gv[5] * z[5];
      asm volatile("" : "+v"(d));
      Yb = qb == 0 ? yin : Yb - d;
      qb = qb == 0 ? w : qb - 1;
      zk += dz;
    };
    int k = khi;
    double gA[6], gB[6], yA, yB;
    fetch(gA, yA);
    // pseudo steps (the bottom side's separator rows, k >= kp): z_k is the top side's,
    // already in zs, so nothing is stored, and every operand of a step (z, g, y) is loaded
    // during the step before it: the steps are independent subtractions whose loads are in
    // flight while the previous one computes, not LDS round trips.  The operands fetched
    // past the last pseudo step are the first regular step's.
    if (k >= kp && k >= klo) {
      double zc[6];
      ld6g(dyn + zk, zc);
      for (; k >= kp && k >= klo; --k) {
        double zn[6];
        int on = k - 1 >= kp ? zk + dz : zk;
        asm volatile("" : "+v"(on));
        ld6g(dyn + on, zn);
        fetch(gB, yB);
        double d = gA[0] * zc[0] + gA[1] * zc[1] + gA[2] * zc[2] + gA[3] * zc[3] + gA[4] * zc[4] + gA[5] * zc[5];
        asm volatile("" : "+v"(d));
        Yb = qb == 0 ? yA : Yb - d;
        qb = qb == 0 ? w : qb - 1;
        zk += dz;
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          zc[c] = zn[c];
          gA[c] = gB[c];
        }
        yA = yB;
      }
    }
    fetch(gB, yB);
    // three operand sets in rotation (a step's set is in use while the one two steps ahead
    // loads), unrolled by three so that no set is copied; the fetches past the last step read
    // in-bounds (zero) operands
    double gC[6], yC;
    for (; k - 2 >= klo; k -= 3) {
      step(k, gA, yA, gC, yC);
      step(k - 1, gB, yB, gA, yA);
      step(k - 2, gC, yC, gB, yB);
    }
    if (k >= klo) step(k, gA, yA, gC, yC);
    if (k - 1 >= klo) step(k - 1, gB, yB, gA, yA);
  };
  auto bs_go = [&](int khi, int klo, int kp) __attribute__((always_inline)) {
    if constexpr (kFull) bs_run_full(khi, klo, kp);
    else bs_run(khi, klo, kp);
  };
  if (!failed) {
    if (role == kChain && side == 0 && sp > 0) {
      bs_init(m + sp - 1, INT_MAX);
      bs_go(m + sp - 1, m, INT_MAX);
    }
    BST(10);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the asm z stores retired
    __syncthreads();  // the separator's z in LDS
    if constexpr (kSplit) {
      // split hand-off 2: the separator's z (the bottom's pseudo steps read it)
      if (!sbot) {
        for (int e = tid; e < 6 * sp; e += NT) st_sc1(A.fac + xch.z + e, zs[6 * m + e]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) xch_flag_set(A.fac, xch.flag + 32, A.seq);
      } else {
        if (tid == 0 && !xch_flag_wait(A.fac, xch.flag + 32, A.seq)) s_late = 1;
        __syncthreads();
        const SysLoads xl(A.fac, xch.end());
        for (int e = tid; e < 6 * sp; e += NT) zs[6 * m + e] = xl.ld(xch.z + e);
        __syncthreads();
      }
    }
    BST(11);
    if (role == kChain && side == 0 && m > 0) {
      if (sp == 0) bs_init(m - 1, INT_MAX);
      bs_go(m - 1, 0, INT_MAX);
    }
    if (role == kChain && side == 1 && nb > 0) {
      bs_init(nb + sp - 1, nb);
      bs_go(nb + sp - 1, 0, nb);
    }
  }
  BST(12);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  BST(13);

  // x_k = L_kk^-T z_k for every row at once, then the pose update
  const double* const recB = kFull ? ringB : A.fac + (long)ncolT * CS;
  // (split mode: the late flag of a hand-off the bottom waited on after its failure verdict)
  const bool failed2 = failed || (kSplit && s_late != 0);
  for (int c = tid; c < A.n_poses; c += NT) {
    if (kSplit && (c >= A.n_fixed && c - A.n_fixed >= ncolT) != sbot) continue;  // the other side's poses
    const double* T = pose_l + 12 * c;
    double* out = A.pose_next + 12l * c;
    if (failed2 || c < A.n_fixed) {
      for (int e = 0; e < 12; ++e) out[e] = T[e];
      if (c >= A.n_fixed)
        for (int e = 0; e < 6; ++e) A.dc[6 * (c - A.n_fixed) + e] = 0.0;
    } else {
      const int G = c - A.n_fixed;
      const double* rec = G < ncolT ? recT + (long)G * CS : recB + (long)(F - 1 - G) * CS;
      double L[21], r[6], d[6];
#pragma unroll
      for (int ii = 0; ii < 6; ++ii)
#pragma unroll
        for (int cc = 0; cc <= ii; cc += 2) {
          const double2 v = reinterpret_cast<const double2*>(rec + 6 * ii)[cc / 2];
          L[P6(ii, cc)] = v.x;
          if (cc + 1 <= ii) L[P6(ii, cc + 1)] = v.y;
        }
      ld6g(rec + 36 * R + 6, r);
      ld6g(zs + 6 * G, d);
      bwd6(L, r, d);
      st6g(A.dc + 6 * G, d);
      se3_exp_apply(d, T, out);
    }
  }
  // A timeout is recorded whatever the earlier status (the counter then holds this launch's
  // reducers: the host re-zeroes it when it reads the flag); a failed factorisation only when
  // no earlier step failed (the status names the first failed iteration).
  // (split mode: either workgroup records a hand-off that never arrived; the factorisation's
  // verdict, which both hold, by the top one)
  const bool late = !reduced || (kSplit && s_late != 0);
  if (tid == 0 && (late || !kSplit || !sbot)) {
    if (late) *A.status = (prior_status ? prior_word : A.iter_tag) | kBandStatusTimeout;
    else if (failed && !prior_status) *A.status = A.iter_tag;
  }
  BST(14);
#if VO_BA_STAMPS
  if (lane == 0 && A.stamps)
    for (int i = 0; i < kBandStamps; ++i) A.stamps[kBandStamps * (kSplit ? 2 * wave + side : wave) + i] = st_acc[i];
#endif
}

}  // namespace

// A fused launch's reducer workgroups need their K2 scratch (two halves) even when the
// solver's own layout is smaller (narrow windows).
static size_t band_launch_lds(const BandLds& L, bool fused) {
  return fused ? std::max(L.bytes, (size_t)kBandRedItems * kRedScr * sizeof(double)) : L.bytes;
}

// The kernels' dynamic-LDS limit (process-wide), raised only when a window needs more than
// any before it: a hipFuncSetAttribute costs host time on every keyframe otherwise.
void band_set_attributes(const BandLds& L) {
  static std::atomic<int> set{-1};
  const int lds = (int)band_launch_lds(L, true);
  int cur = set.load(std::memory_order_relaxed);
  if (lds <= cur) return;
  const void* fs[3] = {(const void*)ba_band_kernel<0>, (const void*)ba_band_kernel<1>, (const void*)ba_band_kernel<2>};
  for (const void* f : fs) VO_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  while (cur < lds && !set.compare_exchange_weak(cur, lds, std::memory_order_relaxed)) {
  }
}

void launch_band_solve(const BandArgs& A, const BandLds& L, hipStream_t st) {
  // the solver first, then the fused K2's reducers (a test build of the context may launch
  // fewer than the solver waits for: vo_ba_testing_drop_reducers)
  const dim3 grid(1 + std::max(A.nred - std::max(A.red_drop, 0), 0));
  const size_t lds = band_launch_lds(L, A.nred > 0);
  if (L.split)  // one workgroup of four waves per side (K2 never fused: BAEngine::fused)
    hipLaunchKernelGGL((ba_band_kernel<2>), dim3(2), dim3(kBandThreads / 2), lds, st, A);
  else if (L.full)
    hipLaunchKernelGGL((ba_band_kernel<1>), grid, dim3(kBandThreads), lds, st, A);
  else
    hipLaunchKernelGGL((ba_band_kernel<0>), grid, dim3(kBandThreads), lds, st, A);
}

}  // namespace vo
