// zdl_store_index.h — InMemoryStorage's trace index on the device (zdl_store.hip).
//
// The store keeps, per stored span, its low and high trace id, its timestamp and an alive
// byte, and a resident index over them that accept keeps current (index_update: the batch is
// radix-sorted and merged in, like the reference's TreeMap inserts at accept, IMS:156-181):
//   bk  every stored position by (lowTraceId, timestamp, arrival)  - the spansByTraceId keys
//   st  by (lowTraceId, first arrival of the span's (lowTraceId, timestamp) key, arrival)
// Evicted spans stay in the index and are filtered by their alive byte; a compaction renumbers
// the positions and the next update rebuilds it. From these:
//   - eviction (evictToRecoverSpans / deleteOldestTrace, InMemoryStorage.java:184-211): the
//     last key of TIMESTAMP_DESCENDING is the smallest (timestamp, lowTraceId), so traces go
//     in ascending (their smallest timestamp, lowTraceId) order until enough spans are freed;
//   - storage order inside a low trace id (spansByTraceId, :448-454): its distinct
//     (lowTraceId, timestamp) keys in first-seen order, each key's spans in arrival order;
//   - trace order: getDependencies(endTs, lookback) walks TIMESTAMP_DESCENDING keys, so a
//     trace comes at its newest key (timestamp, then lowTraceId, descending; :272-291,
//     356-366); getTraces() walks lowTraceIds ascending (:251-262), split by the full trace id
//     in first-seen order when strictTraceId (strictByTraceId, :241-249).
// Nothing of this runs on the host; only counts cross PCIe.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace zdl {

enum : int { SEL_NEWEST = 0, SEL_ALL = 1, SEL_ALL_STRICT = 2 };

struct IndexWork {
  void* tmp = nullptr;  // hipCUB scratch
  size_t tmp_bytes = 0;
  uint64_t* k[2] = {};   // 64-bit sort keys
  uint32_t* v[2] = {};   // span positions
  uint32_t* u[4] = {};   // 32-bit scratch: flags, scans, ranks
  uint64_t* seg = nullptr;  // segment (trace) offsets, cap + 1
  uint64_t* sk[2] = {};  // segment-level sort keys
  uint32_t* sv[2] = {};  // segment-level sort values
  uint8_t* flag = nullptr;
  uint32_t* bc = nullptr;  // offsets_of: per-workgroup flag counts, then their exclusive prefix
  uint64_t* d = nullptr;  // device scalars [4]
  uint64_t* h = nullptr;  // pinned host scalars [4]
  size_t cap = 0;
  // the resident index (index_update)
  uint32_t* bk = nullptr;  // positions [0, ni) by (low id, timestamp, arrival)
  uint32_t* st = nullptr;  // by (low id, first arrival of its (low id, timestamp) key, arrival)
  uint32_t* fs = nullptr;  // per position: that first arrival
  uint32_t* mo = nullptr;  // merge output
  size_t rcap = 0;
  uint64_t ni = 0;         // positions indexed
  void release();
};

// Brings the resident index to positions [0, n): the new ones [ni, n) are sorted and merged in.
// ni > n (the store was compacted or cleared) rebuilds it from scratch.
hipError_t index_update(IndexWork& w, const uint64_t* lo, const int64_t* ts, uint64_t n, hipStream_t s);

// The alive spans of positions [0, n) as a selection: perm[0..n_sel) (device, capacity n) in
// the mode's order, off[0..n_traces] (device, capacity n + 1) the CSR trace offsets.
// n_alive == n: no span is evicted (the alive filter is skipped).
hipError_t index_select(IndexWork& w, const uint64_t* lo, const uint64_t* hi, const int64_t* ts,
                        const uint8_t* alive, uint64_t n, uint64_t n_alive, int mode, uint32_t* perm,
                        uint64_t* off, uint64_t* n_sel, uint64_t* n_traces, hipStream_t s);

// deleteOldestTrace until at least to_recover (> 0) spans are gone: clears their alive bytes
// and returns their number. exhausted: the store ran empty first (every span is evicted, as
// the reference's loop does before TreeMap.lastKey throws NoSuchElementException).
hipError_t index_evict(IndexWork& w, const uint64_t* lo, const int64_t* ts, uint8_t* alive, uint64_t n,
                       uint64_t n_alive, uint64_t to_recover, uint64_t* evicted, bool* exhausted, hipStream_t s);

// The alive positions, ascending, into out (device, capacity n); their number into *m.
hipError_t index_alive(IndexWork& w, const uint8_t* alive, uint64_t n, uint32_t* out, uint64_t* m,
                       hipStream_t s);

}  // namespace zdl
