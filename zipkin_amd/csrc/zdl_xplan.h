// zdl_xplan.h — the host-side bookkeeping of libzdl's multi-GPU combines, kept
// free of HIP / RCCL so that tests/xplan_check.cpp compiles it with g++ and runs it against
// simulated ranks on the CPU (tests/test_xplan.py).
//
// 1. Sparse lists (contexts above 1024 services keep one sorted (cell, call, err) list each):
//    the lists are gathered with exact lengths - rank k's list lands at at[k] of every
//    receiver (a job: every rank; a device group: the first device), in rank order - and then
//    summed per cell (DependencyLinker.merge's sum, DependencyLinker.java:189-204).
//    A job (one list per rank) sums by reduce-scatter instead (range_split / slice_plan below):
//    rank k sums the cells of the k-th cell range over every list, then the reduced ranges are
//    gathered with gather_plan - ascending ranges in rank order, so the concatenation is sorted.
// 2. Insertion order across the ranks of a job: the job's list is DependencyLinker.merge over
//    the ranks' link() lists concatenated in rank order (DependencyLinker.java:189-204: a
//    LinkedHashMap keyed by (parent, child), so a pair sits where it is first seen). Each rank's
//    first-seen rank of a pair (ord_rank: (put position + breadth-first index) << 1 | k) is
//    tagged with the rank number above it, and one element-wise MIN over the ranks (ncclMin,
//    next to the sums) gives every pair its first rank in the concatenation.
#pragma once

#include <algorithm>
#include <cstdint>
#include <utility>
#include <vector>

#ifdef __HIP__  // libzdl's kernels call ord_tag too; the CPU check compiles this with g++
#define ZDL_XPLAN_HD __host__ __device__
#else
#define ZDL_XPLAN_HD
#endif

namespace zdl_xplan {

// Rank tags: ord ranks ((position + breadth-first index) << 1 | k) stay below 2^58 (span
// positions below 2^56, ORD_POS_LIMIT) so that 6 bits of job rank fit above them; an empty cell
// (~0) stays the largest value.
constexpr int ORD_TAG_SHIFT = 58;
constexpr uint64_t ORD_POS_LIMIT = 1ull << 56;
constexpr int ORD_MAX_WORLD = 64;
ZDL_XPLAN_HD inline uint64_t ord_tag(uint64_t first, int rank) {
  return first == ~0ull ? first : (first | ((uint64_t)rank << ORD_TAG_SHIFT));
}

// One transfer: `n` entries of rank `src`'s list from its offset `from` to `dst`'s buffer at `at`.
struct Xfer {
  int src, dst;
  uint64_t n, at, from;
};

// The exact-length gather of W lists (lengths n[0..W)): every list k lands at at[k] (the
// exclusive prefix of n) of each receiver. all = true (a job: every rank receives every list,
// its own by a local copy); all = false (a device group: only rank 0 receives). Empty lists
// move nothing. The plan lists every point-to-point transfer; the caller issues rank me's
// sends (src == me) and receives (dst == me) inside one ncclGroupStart / ncclGroupEnd, and
// its own list (src == dst == me) as a device copy.
struct Plan {
  std::vector<uint64_t> at;  // W + 1 offsets; at[W] = total
  std::vector<Xfer> ops;
  uint64_t total() const { return at.empty() ? 0 : at.back(); }
};

inline Plan gather_plan(const uint64_t* n, int W, bool all) {
  Plan p;
  p.at.assign((size_t)W + 1, 0);
  for (int k = 0; k < W; ++k) p.at[k + 1] = p.at[k] + n[k];
  for (int dst = 0; dst < W; ++dst) {
    if (!all && dst != 0) continue;
    for (int src = 0; src < W; ++src)
      if (n[src]) p.ops.push_back(Xfer{src, dst, n[src], p.at[src], 0});
  }
  return p;
}

// ---- the sparse reduce-scatter of a job (zdl.hip comm_sum_sparse) ----
constexpr int MAX_WORLD = 1024;          // ranks of a sparse job (k_x_slices' LDS bounds)
constexpr uint32_t SPLIT_SAMPLES = 64;  // sampled cells per rank

// The W + 1 cell-range bounds every rank derives from the same gathered samples: meta holds W
// rows of 1 + q words, [list length, the cells at the middle of each of q equal parts of the
// sorted list]. A sample stands for length / q entries; bound k (0 < k < W) is the first sample
// (in cell order) at which the samples' cumulative weight reaches k / W of the total, so each
// range holds about 1 / W of all entries. bound 0 = 0, bound W = 2^32 (past every u32 cell).
// Bounds never decrease; equal bounds leave a rank an empty range (a cell is never split).
inline std::vector<uint64_t> range_split(const uint64_t* meta, int W, uint32_t q) {
  std::vector<std::pair<uint64_t, uint64_t>> smp;  // (cell, weight)
  uint64_t T = 0;
  for (int r = 0; r < W; ++r) {
    const uint64_t* row = meta + (size_t)r * (1 + q);
    if (!row[0]) continue;
    for (uint32_t i = 0; i < q; ++i) smp.push_back({row[1 + i], row[0]});
    T += row[0] * q;
  }
  std::sort(smp.begin(), smp.end());
  std::vector<uint64_t> b((size_t)W + 1, 1ull << 32);
  b[0] = 0;
  uint64_t cum = 0;
  int k = 1;
  for (const auto& e : smp) {
    cum += e.second;
    while (k < W && cum * (uint64_t)W >= (uint64_t)k * T) b[(size_t)k++] = e.first;
  }
  return b;
}

// Rank me's transfers of the all-to-all of slices: cnt is the W x W matrix (row r: the lengths
// of rank r's slices 0..W-1, i.e. what r sends to each rank). Rank r's slice k starts at
// `from` = its slices 0..k-1, and lands at `at` = the slices k receives from ranks 0..r-1. The
// plan lists me's sends (src == me, itself included) and receives (dst == me); at[0..W] are
// me's receive offsets per sender (at[W] = what me receives in all).
inline Plan slice_plan(const uint64_t* cnt, int W, int me) {
  Plan p;
  auto C = [&](int r, int k) { return cnt[(size_t)r * W + k]; };
  p.at.assign((size_t)W + 1, 0);
  for (int j = 0; j < W; ++j) p.at[(size_t)j + 1] = p.at[(size_t)j] + C(j, me);
  uint64_t from = 0;
  for (int k = 0; k < W; ++k) {  // sends, in destination order
    uint64_t at = 0;
    for (int i = 0; i < me; ++i) at += C(i, k);
    if (C(me, k)) p.ops.push_back(Xfer{me, k, C(me, k), at, from});
    from += C(me, k);
  }
  for (int j = 0; j < W; ++j) {  // receives, in source order
    if (j == me || !C(j, me)) continue;
    uint64_t f = 0;
    for (int l = 0; l < me; ++l) f += C(j, l);
    p.ops.push_back(Xfer{j, me, C(j, me), p.at[(size_t)j], f});
  }
  return p;
}

}  // namespace zdl_xplan
