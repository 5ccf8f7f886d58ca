// zdl_sparse.h — the sparse link table (zdl_sparse.hip) for large service dictionaries.
//
// At C5's 10 000 services the S x S table has 10^8 cells (1.6 GB of u64 call and error
// counts, zeroed on every reset and scanned on every link) while a put holds a few million
// distinct (parent, child) pairs. A sparse context keeps instead the accumulated links as one
// list sorted by cell = parent * S + child: the DependencyLinker count maps
// (DependencyLinker.java:39-40, 166-182) as sorted arrays. Each put's links arrive as a log of
// (cell << 1 | error) entries; they are radix-sorted, reduced per cell (call = entries,
// error = odd entries) and merged into the list with the counts of equal cells summed - the
// DependencyLinker.merge reduce (DependencyLinker.java:189-204). Everything is on the stream;
// each step reads its output length back (hipcub sizes are host values).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace zdl {

struct SparseTable {
  uint32_t* cell = nullptr;
  unsigned long long* call = nullptr;
  unsigned long long* err = nullptr;
  size_t n = 0, cap = 0;
  void release();
};

struct SparseWork {
  void* tmp = nullptr;  // hipcub scratch
  size_t tmp_bytes = 0;
  uint32_t* keys = nullptr;  // sorted log
  size_t keys_cap = 0;
  // the put's reduced list, then the merge buffers
  uint32_t* bcell = nullptr;
  unsigned long long* bcall = nullptr;
  unsigned long long* berr = nullptr;
  size_t b_cap = 0;
  uint32_t* mcell = nullptr;
  uint32_t* midx = nullptr;
  unsigned long long* vcall = nullptr;  // A's then B's counts, indexed by the merge's idx
  unsigned long long* verr = nullptr;
  size_t m_cap = 0;
  SparseTable next;  // the merged list (swapped with the context's)
  uint64_t* d_count = nullptr;
  uint64_t* h_count = nullptr;  // pinned
  uint32_t* idx_sorted = nullptr;  // sparse_add: the cells' sort permutation
  size_t idx_cap = 0;
  void release();
};

// Adds the links of E log entries (cell << 1 | error, any order; overwritten as scratch) to t.
// key_bits: significant bits of an entry (1 + bits of the largest cell).
hipError_t sparse_accumulate(SparseWork& w, SparseTable& t, uint32_t* log, uint64_t E, int key_bits,
                             hipStream_t s);

// Adds n pre-aggregated links (cells in any order, repeats allowed) to t.
hipError_t sparse_add(SparseWork& w, SparseTable& t, const uint32_t* cells, const unsigned long long* call,
                      const unsigned long long* err, uint64_t n, int cell_bits, hipStream_t s);

// Capacity for n entries in t (its contents are dropped when it grows).
hipError_t sparse_reserve(SparseTable& t, size_t n);

}  // namespace zdl
