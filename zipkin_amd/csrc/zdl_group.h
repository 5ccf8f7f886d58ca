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

}  // namespace zdl
