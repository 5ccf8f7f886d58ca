// zdl_group.h — on-device grouping of ungrouped spans by low trace id (zdl_group.hip).
//
// InMemoryStorage.getDependencies groups the stored spans by lowTraceId
// (InMemoryStorage.java:323-332, 448-467) in storage order. Here: a stable radix sort of the
// span positions by trace_lo (after one by `ord` when the caller gives a storage order),
// then the run heads become the CSR trace offsets. Everything stays on the context stream.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace zdl {

struct GroupWork {
  void* tmp = nullptr;  // hipcub scratch
  size_t tmp_bytes = 0;
  uint64_t* keys[2] = {};
  uint32_t* idx[2] = {};
  uint32_t* ord_keys[2] = {};
  uint64_t* off = nullptr;    // n_traces + 1 offsets (capacity n + 1)
  uint64_t* count = nullptr;  // device: number of traces
  uint32_t* perm = nullptr;   // points into idx[]: the sorted span positions
  size_t cap = 0;
  void release();
};

// Groups n spans (n < 2^32) by trace_lo, stable in `ord` order when ord != nullptr, else
// in input order. On success g.perm[i] is the input position of the i-th grouped span,
// g.off[0..*g.count] the trace offsets (device memory).
hipError_t group_spans(GroupWork& g, const uint64_t* trace_lo, const uint32_t* ord, uint64_t n,
                       hipStream_t s);

// The non-zero cells of an S x S count table as link records, on the device, in output
// order: cell order (= (parent id, child id)), or by (rank[parent], rank[child]) when a rank
// table is given (a stable 32-bit radix sort; ids past the table rank as themselves).
// Replaces an atomic-counter compaction plus a host sort (7 ms at 250 000 links).
struct LinkWork {
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  uint32_t* sel[2] = {};
  uint32_t* keys[2] = {};
  uint64_t* count = nullptr;
  uint64_t* h_count = nullptr;  // pinned
  size_t cap = 0;
  void release();
};
hipError_t compact_links(LinkWork& w, const unsigned long long* call, const unsigned long long* err, uint64_t SS,
                         uint32_t S, const int32_t* rank, uint32_t nrank, int32_t* parent, int32_t* child,
                         int64_t* call_out, int64_t* err_out, uint64_t* n_out, hipStream_t s);
// The same in two steps, so that the caller can size the output by the link count first:
// compact_select selects the non-zero cells and returns their number (one stream sync);
// compact_records writes the m records (the output may be mapped pinned host memory).
hipError_t compact_select(LinkWork& w, const unsigned long long* call, uint64_t SS, uint64_t* n_out, hipStream_t s);
// A sparse context's sorted (cell, call, err) list as link records (zdl_sparse.h), in rank
// order when a rank table is given.
hipError_t compact_sparse(LinkWork& w, const uint32_t* cell, const unsigned long long* call,
                          const unsigned long long* err, uint64_t m, uint32_t S, const int32_t* rank, uint32_t nrank,
                          int32_t* parent, int32_t* child, int64_t* call_out, int64_t* err_out, hipStream_t s);
hipError_t compact_records(LinkWork& w, const unsigned long long* call, const unsigned long long* err, uint64_t m,
                           uint32_t S, const int32_t* rank, uint32_t nrank, int32_t* parent, int32_t* child,
                           int64_t* call_out, int64_t* err_out, hipStream_t s);

}  // namespace zdl
