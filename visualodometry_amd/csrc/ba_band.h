// K3 for banded reduced camera systems (ba_band.hip), launched by the BA engine (ba.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <vector>

#include "ba_reduce.h"

namespace vo {

// Widest block bandwidth (max_i i - first[i]) the banded solver takes: one chain wave
// holds the panel of a block column, one lane per scalar row, (w + 1) * 6 <= 64.
constexpr int kBandMaxW = 9;
constexpr int kBandMaxF = 512;
constexpr int kBandStamps = 32;
constexpr size_t kBandLdsMax = 160 * 1024 - 1024;  // static LDS: flags, zero block  // dynamic LDS of the one workgroup  // diagnostic build: phase slots per wave

// Split of the F free block rows: top rows [0, m) eliminated top-down, bottom rows
// [F - nb, F) bottom-up, concurrently; the separator [m, m + s) (s = w) last, top-down.
// One-sided (nb = s = 0, m = F) when F is too small for two sides.
struct BandSplit {
  int w = 0, m = 0, nb = 0, s = 0;
};
BandSplit band_split(int F, const std::vector<int>& first);

// Merge pairs of one window structure (host-built, uploaded once): (destination, source)
// LDS offsets (doubles) of the separator's blocks and rhs, top ring += bottom ring.
struct BandTables {
  std::vector<int> tab;
  int merge = 0, n_merge = 0;
};
// LDS layout of the two column stores.  Ring mode: w + 4 slots per side, each padded to
// whole 1 KiB LDS-DMA pieces; factor records go to global memory.  Full mode (when it
// fits): every column of a side in its own slot at the K2 stride, so the factor stays
// in LDS for the back substitution (a DMA's last piece spills into the next slot, or into
// the 1 KiB pad after the side, with the K2 values of the following column).
struct BandLds {
  bool full = false;
  bool split = false;  // two workgroups, one per side, each side's columns in full in its own LDS
  int rc = 0, ss = 0, pad = 0;  // slots per side, doubles per slot, doubles after each side
  size_t bytes = 0;
};
BandLds band_lds_layout(int F, const BandSplit& b, int n_poses, bool allow_split = true);
BandTables band_tables(int F, const BandSplit& b, const BandLds& L);

// K2 writes the reduced camera system in the banded layout (ba.hip, red_dst_): per side,
// column v = band_col_stride(w) doubles -- block (v + q, v) of the side's coordinates
// row-major at 36 q (the bottom side's blocks transposed), the rhs of row v at 36 (w + 1),
// 6 zero doubles; top columns [0, m + s), then bottom columns [0, nb + s), then the cost.
struct BandArgs {
  int F, w, m, nb, s;
  int nprof, n_poses, n_fixed, iter_tag;
  int merge, n_merge;     // merge pairs in tab (BandTables)
  long cost_off;          // the cost in sys
  const int* tab;
  const double* sys;      // K2's banded layout (above), padded by one ring slot
  const double* zero;     // 64 zero doubles: the source of masked prefetches
  double* fac;            // factor records: F columns x band_col_stride(w) doubles
  double* cost_out;       // if set: receives the cost of this linearisation (sys tail)
  double* dc;             // 6F out
  const double* pose_cur;
  double* pose_next;
  int* status;
  unsigned long long* stamps;  // diagnostic build: 4 waves x kBandStamps phase cycles
  // Fused K2 (nred > 0, one rank): workgroups 1..nred of the launch reduce the slabs into sys
  // (two profile blocks each, the cost in the item after the last block: K2's sums bit for
  // bit), store them write-through (sc1) and count themselves in red_count's shards; workgroup
  // 0, the solver, reads sys (by sc1 loads only) after every shard reached its count, and takes
  // the counts back off (zero between launches).
  unsigned seq;  // split mode: this launch's hand-off flag value (nonzero, new every launch)
  int nred;
  int red_drop;  // test switch (host only): reducer workgroups left out of the launch
  unsigned* red_count;   // F + 1 column readiness counters, kBandRedShardStride words apart
  const int* red_col;    // per reduction item (profile block): its column's counter
  const int* col_need;   // per counter: the items that store into that column (F + 1)
  ReduceArgs red;
};
// Split mode's exchange area at the front of BandArgs::fac (doubles): the bottom's merge sources
// (n_merge), the top's separator records (42 doubles a row: L_kk's six rows, 1/diag), the
// separator's z (6 s), two failure words, and three hand-off flags 128 bytes apart (each set to
// the launch's seq once its data is out).
struct SplitXch {
  long merge, rec, z, fail, flag;
  __host__ __device__ long end() const { return flag + 3 * 16; }
};
__host__ __device__ inline SplitXch split_xch(int n_merge, int s) {
  SplitXch x;
  x.merge = 0;
  x.rec = (n_merge + 15) / 16 * 16;
  x.z = x.rec + (42L * s + 15) / 16 * 16;
  x.fail = x.z + (6L * s + 15) / 16 * 16;
  x.flag = x.fail + 16;
  return x;
}
// Status word flag: the fused launch's solver gave up waiting for its reducers (the low bits
// are the iteration, as for a failed factorisation).
constexpr int kBandStatusTimeout = 1 << 30;
// Reducer workgroups of a fused launch: items (profile blocks + the cost) per workgroup.
constexpr int kBandRedItems = 2;
// The fused launch's hand-off is per column of K2's banded layout: one readiness counter per
// column that K2 writes (top columns 0 .. m + s - 1, then bottom columns 0 .. nb - 1: F counters)
// and one for the cost, each on a 128-byte line of its own (kBandRedShardStride words).  A reducer
// item counts itself in its column's counter; the solver starts loading a column as soon as its
// counter holds the column's item count (col_need), so the prologue's loads overlap the slower
// reducers instead of waiting for the last one.  (One counter for all took the 178 arrivals of
// cfg3 one after another at the memory side: MI355X_MICROARCH.md, fanin row.)
constexpr int kBandRedShardStride = 32;
inline size_t band_col_count_bytes(int F) { return (size_t)(F + 1) * kBandRedShardStride * 4; }
inline int band_fused_workgroups(int nprof) { return (nprof + 1 + kBandRedItems - 1) / kBandRedItems; }

// Doubles per ring slot / factor record: (w + 1) blocks of 36, the rhs row (6) and the
// reciprocal diagonal (6).
inline int band_col_stride(int w) { return 36 * (w + 1) + 12; }
// Doubles per LDS ring slot: the column padded to whole 1 KiB LDS-DMA wave pieces.
inline int band_slot_stride(int w) { return (band_col_stride(w) + 127) / 128 * 128; }
size_t band_fac_doubles(int F, int w);
// true if the window fits the kernel (lane budget, LDS budget)
bool band_supported(int F, int w, int n_poses);
void band_set_attributes(const BandLds& L);
void launch_band_solve(const BandArgs& A, const BandLds& L, hipStream_t st);

}  // namespace vo
