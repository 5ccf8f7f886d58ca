// zdl_sparse.hip — sorted-list link table for large service dictionaries (zdl_sparse.h).
#include "zdl_sparse.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <utility>

namespace zdl {
namespace {

#define STRY(expr)                   \
  do {                               \
    hipError_t _e = (expr);          \
    if (_e != hipSuccess) return _e; \
  } while (0)

template <class T>
hipError_t grow(T*& p, size_t& cap, size_t n) {
  if (n <= cap && p) return hipSuccess;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  const size_t c = std::max<size_t>(n + n / 4, 1024);
  STRY(hipMalloc((void**)&p, c * sizeof(T)));
  cap = c;
  return hipSuccess;
}

struct CellOf {
  __host__ __device__ uint32_t operator()(uint32_t k) const { return k >> 1; }
};
// one log entry as (call 1 << 32 | error bit): a single reduce by key sums both counts (a put
// holds < 2^31 entries, so neither half overflows)
struct PackOf {
  __host__ __device__ unsigned long long operator()(uint32_t k) const { return (1ull << 32) | (k & 1u); }
};
struct Gather {
  const unsigned long long* v;
  __host__ __device__ unsigned long long operator()(uint32_t i) const { return v[i]; }
};

using CellIt = hipcub::TransformInputIterator<uint32_t, CellOf, const uint32_t*>;
using PackIt = hipcub::TransformInputIterator<unsigned long long, PackOf, const uint32_t*>;
using GatherIt = hipcub::TransformInputIterator<unsigned long long, Gather, const uint32_t*>;
using IdxIt = hipcub::CountingInputIterator<uint32_t>;

// (call << 32 | err) -> call, err (in place for call)
__global__ void k_unpack(unsigned long long* call, unsigned long long* err, const uint64_t* n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *n) return;
  const unsigned long long v = call[i];
  call[i] = v >> 32;
  err[i] = v & 0xFFFFFFFFull;
}

__global__ void k_iota32(uint32_t* p, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (uint32_t)i;
}

hipError_t scratch(SparseWork& w, size_t need) {
  if (need <= w.tmp_bytes) return hipSuccess;
  if (w.tmp) (void)hipFree(w.tmp);
  w.tmp = nullptr;
  w.tmp_bytes = 0;
  STRY(hipMalloc(&w.tmp, need));
  w.tmp_bytes = need;
  return hipSuccess;
}

hipError_t read_count(SparseWork& w, hipStream_t s, uint64_t* out) {
  STRY(hipMemcpyAsync(w.h_count, w.d_count, 8, hipMemcpyDeviceToHost, s));
  STRY(hipStreamSynchronize(s));
  *out = *w.h_count;
  return hipSuccess;
}

hipError_t ensure_table(SparseTable& t, size_t n) {
  if (n <= t.cap && t.cell) return hipSuccess;
  t.release();
  const size_t c = std::max<size_t>(n + n / 4, 1024);
  STRY(hipMalloc((void**)&t.cell, c * 4));
  STRY(hipMalloc((void**)&t.call, c * 8));
  STRY(hipMalloc((void**)&t.err, c * 8));
  t.cap = c;
  return hipSuccess;
}

// t += (cellB, callB, errB)[0..U): both sorted by cell, each cell once.
hipError_t merge_into(SparseWork& w, SparseTable& t, const uint32_t* cellB, const unsigned long long* callB,
                      const unsigned long long* errB, uint64_t U, hipStream_t s) {
  if (U == 0) return hipSuccess;
  if (t.n == 0) {
    STRY(ensure_table(t, U));
    STRY(hipMemcpyAsync(t.cell, cellB, U * 4, hipMemcpyDeviceToDevice, s));
    STRY(hipMemcpyAsync(t.call, callB, U * 8, hipMemcpyDeviceToDevice, s));
    STRY(hipMemcpyAsync(t.err, errB, U * 8, hipMemcpyDeviceToDevice, s));
    t.n = U;
    return hipSuccess;
  }
  const uint64_t n = t.n, M = n + U;
  size_t mcap = w.m_cap, c2 = w.m_cap, c3 = w.m_cap, c4 = w.m_cap;
  STRY(grow(w.mcell, mcap, M));
  STRY(grow(w.midx, c2, M));
  STRY(grow(w.vcall, c3, M));
  STRY(grow(w.verr, c4, M));
  w.m_cap = std::min(std::min(mcap, c2), std::min(c3, c4));
  STRY(ensure_table(w.next, M));
  STRY(hipMemcpyAsync(w.vcall, t.call, n * 8, hipMemcpyDeviceToDevice, s));
  STRY(hipMemcpyAsync(w.vcall + n, callB, U * 8, hipMemcpyDeviceToDevice, s));
  STRY(hipMemcpyAsync(w.verr, t.err, n * 8, hipMemcpyDeviceToDevice, s));
  STRY(hipMemcpyAsync(w.verr + n, errB, U * 8, hipMemcpyDeviceToDevice, s));
  size_t a = 0, b = 0;
  STRY(hipcub::DeviceMerge::MergePairs(nullptr, a, t.cell, IdxIt(0), (int)n, cellB, IdxIt((uint32_t)n), (int)U,
                                       w.mcell, w.midx, ::rocprim::less<uint32_t>(), s));
  STRY(hipcub::DeviceReduce::ReduceByKey(nullptr, b, (const uint32_t*)w.mcell, w.next.cell,
                                         GatherIt(w.midx, Gather{w.vcall}), w.next.call, w.d_count, hipcub::Sum(),
                                         (int)M, s));
  STRY(scratch(w, std::max(a, b)));
  size_t bytes = w.tmp_bytes;
  STRY(hipcub::DeviceMerge::MergePairs(w.tmp, bytes, t.cell, IdxIt(0), (int)n, cellB, IdxIt((uint32_t)n), (int)U,
                                       w.mcell, w.midx, ::rocprim::less<uint32_t>(), s));
  bytes = w.tmp_bytes;
  STRY(hipcub::DeviceReduce::ReduceByKey(w.tmp, bytes, (const uint32_t*)w.mcell, w.next.cell,
                                         GatherIt(w.midx, Gather{w.vcall}), w.next.call, w.d_count, hipcub::Sum(),
                                         (int)M, s));
  bytes = w.tmp_bytes;
  STRY(hipcub::DeviceReduce::ReduceByKey(w.tmp, bytes, (const uint32_t*)w.mcell, w.next.cell,
                                         GatherIt(w.midx, Gather{w.verr}), w.next.err, w.d_count, hipcub::Sum(),
                                         (int)M, s));
  uint64_t m = 0;
  STRY(read_count(w, s, &m));
  std::swap(t, w.next);
  t.n = m;
  return hipSuccess;
}

hipError_t counters(SparseWork& w) {
  if (!w.d_count) STRY(hipMalloc((void**)&w.d_count, 8));
  if (!w.h_count) STRY(hipHostMalloc((void**)&w.h_count, 8, hipHostMallocDefault));
  return hipSuccess;
}

}  // namespace

void SparseTable::release() {
  if (cell) (void)hipFree(cell);
  if (call) (void)hipFree(call);
  if (err) (void)hipFree(err);
  cell = nullptr;
  call = nullptr;
  err = nullptr;
  n = cap = 0;
}

void SparseWork::release() {
  for (void* p : {(void*)tmp, (void*)keys, (void*)bcell, (void*)bcall, (void*)berr, (void*)mcell, (void*)midx,
                  (void*)vcall, (void*)verr, (void*)d_count, (void*)idx_sorted})
    if (p) (void)hipFree(p);
  if (h_count) (void)hipHostFree(h_count);
  tmp = nullptr;
  keys = nullptr;
  bcell = nullptr;
  bcall = nullptr;
  berr = nullptr;
  mcell = nullptr;
  midx = nullptr;
  vcall = nullptr;
  verr = nullptr;
  d_count = nullptr;
  h_count = nullptr;
  idx_sorted = nullptr;
  tmp_bytes = keys_cap = b_cap = m_cap = idx_cap = 0;
  next.release();
}

hipError_t sparse_accumulate(SparseWork& w, SparseTable& t, uint32_t* log, uint64_t E, int key_bits,
                             hipStream_t s) {
  if (E == 0) return hipSuccess;
  if (E >= (1ull << 31)) return hipErrorInvalidValue;
  STRY(counters(w));
  size_t c1 = w.keys_cap;
  STRY(grow(w.keys, c1, E));
  w.keys_cap = c1;
  size_t b1 = w.b_cap, b2 = w.b_cap, b3 = w.b_cap;
  STRY(grow(w.bcell, b1, E));
  STRY(grow(w.bcall, b2, E));
  STRY(grow(w.berr, b3, E));
  w.b_cap = std::min(b1, std::min(b2, b3));
  size_t a = 0, b = 0;
  STRY(hipcub::DeviceRadixSort::SortKeys(nullptr, a, log, w.keys, (int)E, 0, key_bits, s));
  STRY(hipcub::DeviceReduce::ReduceByKey(nullptr, b, CellIt(w.keys, CellOf{}), w.bcell, PackIt(w.keys, PackOf{}),
                                         w.bcall, w.d_count, hipcub::Sum(), (int)E, s));
  STRY(scratch(w, std::max(a, b)));
  size_t bytes = w.tmp_bytes;
  STRY(hipcub::DeviceRadixSort::SortKeys(w.tmp, bytes, log, w.keys, (int)E, 0, key_bits, s));
  bytes = w.tmp_bytes;  // per cell: call = entries, error = odd entries, in one pass
  STRY(hipcub::DeviceReduce::ReduceByKey(w.tmp, bytes, CellIt(w.keys, CellOf{}), w.bcell, PackIt(w.keys, PackOf{}),
                                         w.bcall, w.d_count, hipcub::Sum(), (int)E, s));
  hipLaunchKernelGGL(k_unpack, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, w.bcall, w.berr, w.d_count);
  STRY(hipGetLastError());
  uint64_t U = 0;
  STRY(read_count(w, s, &U));
  return merge_into(w, t, w.bcell, w.bcall, w.berr, U, s);
}

hipError_t sparse_add(SparseWork& w, SparseTable& t, const uint32_t* cells, const unsigned long long* call,
                      const unsigned long long* err, uint64_t n, int cell_bits, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n >= (1ull << 31)) return hipErrorInvalidValue;
  STRY(counters(w));
  size_t c1 = w.keys_cap;
  STRY(grow(w.keys, c1, n));
  w.keys_cap = c1;
  size_t b1 = w.b_cap, b2 = w.b_cap, b3 = w.b_cap;
  STRY(grow(w.bcell, b1, 2 * n));  // the cells' sort: sorted keys, then sorted indices behind them
  STRY(grow(w.bcall, b2, n));
  STRY(grow(w.berr, b3, n));
  w.b_cap = std::min(b1 / 2, std::min(b2, b3));
  uint32_t* idx = w.bcell + n;  // scratch: iota, sorted by cell into keys' partner
  size_t icap = w.idx_cap;
  STRY(grow(w.idx_sorted, icap, n));  // kept in the work area: no allocation per combine, no leak
  w.idx_cap = icap;
  uint32_t* idx_sorted = w.idx_sorted;
  hipLaunchKernelGGL(k_iota32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, idx, n);
  STRY(hipGetLastError());
  size_t a = 0, b = 0;
  STRY(hipcub::DeviceRadixSort::SortPairs(nullptr, a, cells, w.keys, (const uint32_t*)idx, idx_sorted, (int)n, 0,
                                          cell_bits, s));
  STRY(hipcub::DeviceReduce::ReduceByKey(nullptr, b, (const uint32_t*)w.keys, w.bcell,
                                         GatherIt(idx_sorted, Gather{call}), w.bcall, w.d_count, hipcub::Sum(),
                                         (int)n, s));
  STRY(scratch(w, std::max(a, b)));
  size_t bytes = w.tmp_bytes;
  STRY(hipcub::DeviceRadixSort::SortPairs(w.tmp, bytes, cells, w.keys, (const uint32_t*)idx, idx_sorted, (int)n, 0,
                                          cell_bits, s));
  // the unique cells land in bcell[0..U) (U <= n), ahead of the iota scratch in bcell[n..)
  bytes = w.tmp_bytes;
  STRY(hipcub::DeviceReduce::ReduceByKey(w.tmp, bytes, (const uint32_t*)w.keys, w.bcell,
                                         GatherIt(idx_sorted, Gather{call}), w.bcall, w.d_count, hipcub::Sum(),
                                         (int)n, s));
  bytes = w.tmp_bytes;
  STRY(hipcub::DeviceReduce::ReduceByKey(w.tmp, bytes, (const uint32_t*)w.keys, w.bcell,
                                         GatherIt(idx_sorted, Gather{err}), w.berr, w.d_count, hipcub::Sum(),
                                         (int)n, s));
  uint64_t U = 0;
  STRY(read_count(w, s, &U));
  return merge_into(w, t, w.bcell, w.bcall, w.berr, U, s);
}

}  // namespace zdl
