// zdl_xplan.h — the host-side bookkeeping of libzdl's multi-GPU combines, kept
// free of HIP / RCCL so that tests/xplan_check.cpp compiles it with g++ and runs it against
// simulated ranks on the CPU (tests/test_xplan.py).
//
// 1. Sparse lists (contexts above 1024 services keep one sorted (cell, call, err) list each):
//    the lists are gathered with exact lengths - rank k's list lands at at[k] of every
//    receiver (a job: every rank; a device group: the first device), in rank order - and then
//    summed per cell (DependencyLinker.merge's sum, DependencyLinker.java:189-204).
// 2. Insertion order across the ranks of a job: the job's list is DependencyLinker.merge over
//    the ranks' link() lists concatenated in rank order (DependencyLinker.java:189-204: a
//    LinkedHashMap keyed by (parent, child), so a pair sits where it is first seen). Each rank's
//    first-seen rank of a pair (ord_rank: put position << 24 | breadth-first index << 1 | k) is
//    tagged with the rank number above it, and one element-wise MIN over the ranks (ncclMin,
//    next to the sums) gives every pair its first rank in the concatenation.
#pragma once

#include <cstdint>
#include <vector>

#ifdef __HIP__  // libzdl's kernels call ord_tag too; the CPU check compiles this with g++
#define ZDL_XPLAN_HD __host__ __device__
#else
#define ZDL_XPLAN_HD
#endif

namespace zdl_xplan {

// Rank tags: ord ranks stay below 2^58 (span positions below 2^34, ORD_POS_LIMIT) so that 6
// bits of job rank fit above them; an empty cell (~0) stays the largest value.
constexpr int ORD_TAG_SHIFT = 58;
constexpr uint64_t ORD_POS_LIMIT = 1ull << 34;
constexpr int ORD_MAX_WORLD = 64;
ZDL_XPLAN_HD inline uint64_t ord_tag(uint64_t first, int rank) {
  return first == ~0ull ? first : (first | ((uint64_t)rank << ORD_TAG_SHIFT));
}

// One transfer of a gather: `n` entries of rank `src`'s list to `dst`'s buffer at `at`.
struct Xfer {
  int src, dst;
  uint64_t n, at;
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
      if (n[src]) p.ops.push_back(Xfer{src, dst, n[src], p.at[src]});
  }
  return p;
}

}  // namespace zdl_xplan
