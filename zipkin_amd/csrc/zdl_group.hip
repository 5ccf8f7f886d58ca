// zdl_group.hip — on-device grouping of ungrouped spans by low trace id (zdl_group.h).
#include "zdl_group.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>

namespace zdl {
namespace {

__global__ void k_iota(uint32_t* __restrict__ idx, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) idx[i] = (uint32_t)i;
}

__global__ void k_take_keys(const uint64_t* __restrict__ trace_lo, const uint32_t* __restrict__ idx,
                            uint64_t* __restrict__ keys, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) keys[i] = trace_lo[idx[i]];
}

// flag[i] = 1 where a new trace starts in the sorted keys
__global__ void k_heads(const uint64_t* __restrict__ keys, uint64_t n, uint8_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flag[i] = i == 0 || keys[i] != keys[i - 1];
}

__global__ void k_close(uint64_t* __restrict__ off, const uint64_t* __restrict__ count, uint64_t n) {
  if (threadIdx.x == 0) off[*count] = n;
}

template <class T>
hipError_t grow(T*& p, size_t n) {
  if (p) (void)hipFree(p);
  p = nullptr;
  return hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T));
}

inline dim3 blocks(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace

void GroupWork::release() {
  for (auto*& p : keys) { if (p) (void)hipFree(p); p = nullptr; }
  for (auto*& p : idx) { if (p) (void)hipFree(p); p = nullptr; }
  for (auto*& p : ord_keys) { if (p) (void)hipFree(p); p = nullptr; }
  if (off) (void)hipFree(off);
  if (count) (void)hipFree(count);
  if (tmp) (void)hipFree(tmp);
  off = nullptr;
  count = nullptr;
  tmp = nullptr;
  tmp_bytes = 0;
  perm = nullptr;
  cap = 0;
}

#define GTRY(expr)                          \
  do {                                      \
    hipError_t _e = (expr);                 \
    if (_e != hipSuccess) return _e;        \
  } while (0)

hipError_t group_spans(GroupWork& g, const uint64_t* trace_lo, const uint32_t* ord, uint64_t n,
                       hipStream_t s) {
  if (n == 0 || n >= (1ull << 32)) return hipErrorInvalidValue;
  if (n > g.cap) {
    for (int b = 0; b < 2; ++b) {
      GTRY(grow(g.keys[b], n));
      GTRY(grow(g.idx[b], n));
      GTRY(grow(g.ord_keys[b], n));
    }
    GTRY(grow(g.off, n + 1));
    if (!g.count) GTRY(hipMalloc((void**)&g.count, sizeof(uint64_t)));
    // scratch: the larger of the two sorts and the run-head selection (flags live in ord_keys[1])
    size_t a = 0, b = 0, c = 0;
    GTRY(hipcub::DeviceRadixSort::SortPairs(nullptr, a, g.keys[0], g.keys[1], g.idx[0], g.idx[1], (int)n, 0, 64, s));
    GTRY(hipcub::DeviceRadixSort::SortPairs(nullptr, b, g.ord_keys[0], g.ord_keys[1], g.idx[0], g.idx[1], (int)n, 0,
                                            32, s));
    GTRY(hipcub::DeviceSelect::Flagged(nullptr, c, hipcub::CountingInputIterator<uint64_t>(0),
                                       reinterpret_cast<uint8_t*>(g.ord_keys[1]), g.off, g.count, (int)n, s));
    const size_t need = std::max(a, std::max(b, c));
    if (need > g.tmp_bytes) {
      if (g.tmp) (void)hipFree(g.tmp);
      g.tmp = nullptr;
      g.tmp_bytes = 0;
      GTRY(hipMalloc(&g.tmp, need));
      g.tmp_bytes = need;
    }
    g.cap = n;
  }
  hipLaunchKernelGGL(k_iota, blocks(n), dim3(256), 0, s, g.idx[0], n);
  GTRY(hipGetLastError());
  size_t bytes = g.tmp_bytes;
  const uint32_t* idx_in = g.idx[0];
  if (ord) {  // storage order first (stable), then the trace key (stable) keeps it
    GTRY(hipcub::DeviceRadixSort::SortPairs(g.tmp, bytes, ord, g.ord_keys[0], g.idx[0], g.idx[1], (int)n, 0, 32, s));
    idx_in = g.idx[1];
  }
  hipLaunchKernelGGL(k_take_keys, blocks(n), dim3(256), 0, s, trace_lo, idx_in, g.keys[0], n);
  GTRY(hipGetLastError());
  uint32_t* idx_out = ord ? g.idx[0] : g.idx[1];
  bytes = g.tmp_bytes;
  GTRY(hipcub::DeviceRadixSort::SortPairs(g.tmp, bytes, g.keys[0], g.keys[1], idx_in, idx_out, (int)n, 0, 64, s));
  g.perm = idx_out;
  uint8_t* flag = reinterpret_cast<uint8_t*>(g.ord_keys[1]);
  hipLaunchKernelGGL(k_heads, blocks(n), dim3(256), 0, s, g.keys[1], n, flag);
  GTRY(hipGetLastError());
  bytes = g.tmp_bytes;
  GTRY(hipcub::DeviceSelect::Flagged(g.tmp, bytes, hipcub::CountingInputIterator<uint64_t>(0), flag, g.off, g.count,
                                     (int)n, s));
  hipLaunchKernelGGL(k_close, dim3(1), dim3(64), 0, s, g.off, g.count, n);
  return hipGetLastError();
}

namespace {
struct NonZeroCell {
  const unsigned long long* call;
  __host__ __device__ bool operator()(const uint32_t& i) const { return call[i] != 0; }
};

__device__ __forceinline__ uint32_t rank16(int32_t id, const int32_t* rank, uint32_t nrank) {
  return (uint32_t)((uint32_t)id < nrank ? rank[id] : id) & 0xFFFFu;
}

__global__ void k_link_keys(const uint32_t* __restrict__ sel, const uint64_t* __restrict__ count, uint32_t S,
                            const int32_t* __restrict__ rank, uint32_t nrank, uint32_t* __restrict__ keys) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= *count) return;
  const uint32_t i = sel[j];
  keys[j] = (rank16((int32_t)(i / S), rank, nrank) << 16) | rank16((int32_t)(i % S), rank, nrank);
}

__global__ void k_link_records(const uint32_t* __restrict__ sel, const uint64_t* __restrict__ count, uint32_t S,
                               const unsigned long long* __restrict__ call, const unsigned long long* __restrict__ err,
                               int32_t* __restrict__ p, int32_t* __restrict__ c, int64_t* __restrict__ n,
                               int64_t* __restrict__ e) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= *count) return;
  const uint32_t i = sel[j];
  p[j] = (int32_t)(i / S);
  c[j] = (int32_t)(i % S);
  n[j] = (int64_t)call[i];
  e[j] = (int64_t)err[i];
}
}  // namespace

void LinkWork::release() {
  for (auto*& q : sel) { if (q) (void)hipFree(q); q = nullptr; }
  for (auto*& q : keys) { if (q) (void)hipFree(q); q = nullptr; }
  if (count) (void)hipFree(count);
  if (h_count) (void)hipHostFree(h_count);
  if (tmp) (void)hipFree(tmp);
  count = nullptr;
  h_count = nullptr;
  tmp = nullptr;
  tmp_bytes = 0;
  cap = 0;
}

namespace {
// The non-zero cells of a table up to SEL_MAX cells (LOG mode's S x S <= 2^20), in cell order,
// by two launches (round 5; hipCUB's DeviceSelect::If took three kernels, ~18 us at C3's 250 000
// cells): k_sel_count counts each tile's non-zero cells; k_sel_write sums the counts of the tiles
// before its own (at most SEL_MAX / SEL_TILE of them), scans its tile in the workgroup and writes
// the indices; the last tile writes the total.
constexpr int SEL_T = 256, SEL_PER = 16, SEL_TILE = SEL_T * SEL_PER;
constexpr uint64_t SEL_MAX = 1ull << 22;

__device__ __forceinline__ uint32_t sel_block_sum(uint32_t v, uint32_t* sh) {
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
  for (int k = 0; k < SEL_T / 64; ++k) t += sh[k];
  __syncthreads();
  return t;
}

__global__ void __launch_bounds__(SEL_T) k_sel_count(const unsigned long long* __restrict__ call, uint32_t SS,
                                                     uint32_t* __restrict__ tc) {
  __shared__ uint32_t sh[SEL_T / 64];
  const uint32_t b0 = blockIdx.x * SEL_TILE;
  uint32_t n = 0;
#pragma unroll
  for (int q = 0; q < SEL_PER; ++q) {
    const uint32_t i = b0 + q * SEL_T + threadIdx.x;
    n += (i < SS && call[i] != 0) ? 1u : 0u;
  }
  const uint32_t t = sel_block_sum(n, sh);
  if (threadIdx.x == 0) tc[blockIdx.x] = t;
}

__global__ void __launch_bounds__(SEL_T) k_sel_write(const unsigned long long* __restrict__ call, uint32_t SS,
                                                     const uint32_t* __restrict__ tc, uint32_t* __restrict__ sel,
                                                     uint64_t* __restrict__ count) {
  __shared__ uint32_t sh[SEL_T / 64];
  __shared__ uint32_t wsum[SEL_T / 64 + 1];
  uint32_t before = 0;
  for (uint32_t k = threadIdx.x; k < blockIdx.x; k += SEL_T) before += tc[k];
  const uint32_t base = sel_block_sum(before, sh);
  // thread t takes the SEL_PER consecutive cells [b0 + t * SEL_PER, ...): cell order is thread order
  const uint32_t c0 = blockIdx.x * SEL_TILE + threadIdx.x * SEL_PER;
  uint32_t flags = 0;
#pragma unroll
  for (int q = 0; q < SEL_PER; ++q) {
    const uint32_t i = c0 + q;
    flags |= (i < SS && call[i] != 0) ? (1u << q) : 0u;
  }
  const uint32_t mine = (uint32_t)__popc(flags);
  uint32_t incl = mine;  // inclusive scan over the workgroup
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint32_t wbase = 0;
  for (int k = 0; k < wv; ++k) wbase += wsum[k];
  uint32_t at = base + wbase + incl - mine;
  for (uint32_t f = flags; f; f &= f - 1) sel[at++] = c0 + (uint32_t)__ffs(f) - 1;
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == SEL_T - 1) *count = (uint64_t)(base + wbase + incl);
}
}  // namespace

hipError_t compact_select(LinkWork& w, const unsigned long long* call, uint64_t SS, uint64_t* n_out, hipStream_t s) {
  if (SS == 0 || SS >= (1ull << 32)) return hipErrorInvalidValue;
  if (SS <= SEL_MAX) {
    const uint32_t nt = (uint32_t)((SS + SEL_TILE - 1) / SEL_TILE);
    if (SS > w.cap) {
      for (int b = 0; b < 2; ++b) {
        GTRY(grow(w.sel[b], SS));
        GTRY(grow(w.keys[b], SS));
      }
      if (!w.count) GTRY(hipMalloc((void**)&w.count, sizeof(uint64_t)));
      if (!w.h_count) GTRY(hipHostMalloc((void**)&w.h_count, sizeof(uint64_t), hipHostMallocDefault));
      size_t b = 0;
      GTRY(hipcub::DeviceRadixSort::SortPairs(nullptr, b, w.keys[0], w.keys[1], w.sel[0], w.sel[1], (int)SS, 0, 32, s));
      if (b > w.tmp_bytes) {
        if (w.tmp) (void)hipFree(w.tmp);
        w.tmp = nullptr;
        w.tmp_bytes = 0;
        GTRY(hipMalloc(&w.tmp, b));
        w.tmp_bytes = b;
      }
      w.cap = SS;
    }
    uint32_t* tc = w.keys[1];  // the tile counts (the keys' second buffer is free until the rank sort)
    hipLaunchKernelGGL(k_sel_count, dim3(nt), dim3(SEL_T), 0, s, call, (uint32_t)SS, tc);
    GTRY(hipGetLastError());
    hipLaunchKernelGGL(k_sel_write, dim3(nt), dim3(SEL_T), 0, s, call, (uint32_t)SS, (const uint32_t*)tc, w.sel[0],
                       w.count);
    GTRY(hipGetLastError());
    GTRY(hipMemcpyAsync(w.h_count, w.count, 8, hipMemcpyDeviceToHost, s));
    GTRY(hipStreamSynchronize(s));
    *n_out = *w.h_count;
    return hipSuccess;
  }
  if (SS > w.cap) {
    for (int b = 0; b < 2; ++b) {
      GTRY(grow(w.sel[b], SS));
      GTRY(grow(w.keys[b], SS));
    }
    if (!w.count) GTRY(hipMalloc((void**)&w.count, sizeof(uint64_t)));
    if (!w.h_count) GTRY(hipHostMalloc((void**)&w.h_count, sizeof(uint64_t), hipHostMallocDefault));
    size_t a = 0, b = 0;
    GTRY(hipcub::DeviceSelect::If(nullptr, a, hipcub::CountingInputIterator<uint32_t>(0), w.sel[0], w.count, (int)SS,
                                  NonZeroCell{call}, s));
    GTRY(hipcub::DeviceRadixSort::SortPairs(nullptr, b, w.keys[0], w.keys[1], w.sel[0], w.sel[1], (int)SS, 0, 32, s));
    const size_t need = std::max(a, b);
    if (need > w.tmp_bytes) {
      if (w.tmp) (void)hipFree(w.tmp);
      w.tmp = nullptr;
      w.tmp_bytes = 0;
      GTRY(hipMalloc(&w.tmp, need));
      w.tmp_bytes = need;
    }
    w.cap = SS;
  }
  size_t bytes = w.tmp_bytes;
  GTRY(hipcub::DeviceSelect::If(w.tmp, bytes, hipcub::CountingInputIterator<uint32_t>(0), w.sel[0], w.count, (int)SS,
                                NonZeroCell{call}, s));
  GTRY(hipMemcpyAsync(w.h_count, w.count, 8, hipMemcpyDeviceToHost, s));  // pinned: a DMA, no staging
  GTRY(hipStreamSynchronize(s));
  *n_out = *w.h_count;
  return hipSuccess;
}

hipError_t compact_records(LinkWork& w, const unsigned long long* call, const unsigned long long* err, uint64_t m,
                           uint32_t S, const int32_t* rank, uint32_t nrank, int32_t* parent, int32_t* child,
                           int64_t* call_out, int64_t* err_out, hipStream_t s) {
  if (m == 0) return hipSuccess;
  const uint32_t* sel = w.sel[0];
  if (rank) {
    hipLaunchKernelGGL(k_link_keys, blocks(m), dim3(256), 0, s, w.sel[0], w.count, S, rank, nrank, w.keys[0]);
    GTRY(hipGetLastError());
    size_t bytes = w.tmp_bytes;
    GTRY(hipcub::DeviceRadixSort::SortPairs(w.tmp, bytes, w.keys[0], w.keys[1], w.sel[0], w.sel[1], (int)m, 0, 32, s));
    sel = w.sel[1];
  }
  hipLaunchKernelGGL(k_link_records, blocks(m), dim3(256), 0, s, sel, w.count, S, call, err, parent, child,
                     call_out, err_out);
  return hipGetLastError();
}

namespace {
__global__ void k_sparse_keys(const uint32_t* __restrict__ cell, uint64_t m, uint32_t S,
                              const int32_t* __restrict__ rank, uint32_t nrank, uint32_t* __restrict__ keys,
                              uint32_t* __restrict__ idx) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint32_t i = cell[j];
  keys[j] = (rank16((int32_t)(i / S), rank, nrank) << 16) | rank16((int32_t)(i % S), rank, nrank);
  idx[j] = (uint32_t)j;
}

__global__ void k_sparse_records(const uint32_t* __restrict__ sel, uint64_t m, uint32_t S,
                                 const uint32_t* __restrict__ cell, const unsigned long long* __restrict__ call,
                                 const unsigned long long* __restrict__ err, int32_t* __restrict__ p,
                                 int32_t* __restrict__ c, int64_t* __restrict__ n, int64_t* __restrict__ e) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint32_t k = sel ? sel[j] : (uint32_t)j;
  const uint32_t i = cell[k];
  p[j] = (int32_t)(i / S);
  c[j] = (int32_t)(i % S);
  n[j] = (int64_t)call[k];
  e[j] = (int64_t)err[k];
}
}  // namespace

hipError_t compact_sparse(LinkWork& w, const uint32_t* cell, const unsigned long long* call,
                          const unsigned long long* err, uint64_t m, uint32_t S, const int32_t* rank, uint32_t nrank,
                          int32_t* parent, int32_t* child, int64_t* call_out, int64_t* err_out, hipStream_t s) {
  if (m == 0) return hipSuccess;
  if (m >= (1ull << 31)) return hipErrorInvalidValue;
  const uint32_t* sel = nullptr;
  if (rank) {  // the list is in cell (id) order; names order: a stable sort by the ranks
    if (m > w.cap) {
      for (int b = 0; b < 2; ++b) {
        GTRY(grow(w.sel[b], m));
        GTRY(grow(w.keys[b], m));
      }
      w.cap = m;
      size_t need = 0;
      GTRY(hipcub::DeviceRadixSort::SortPairs(nullptr, need, w.keys[0], w.keys[1], w.sel[0], w.sel[1], (int)m, 0, 32,
                                              s));
      if (need > w.tmp_bytes) {
        if (w.tmp) (void)hipFree(w.tmp);
        w.tmp = nullptr;
        w.tmp_bytes = 0;
        GTRY(hipMalloc(&w.tmp, need));
        w.tmp_bytes = need;
      }
    }
    hipLaunchKernelGGL(k_sparse_keys, blocks(m), dim3(256), 0, s, cell, m, S, rank, nrank, w.keys[0], w.sel[0]);
    GTRY(hipGetLastError());
    size_t bytes = w.tmp_bytes;
    GTRY(hipcub::DeviceRadixSort::SortPairs(w.tmp, bytes, w.keys[0], w.keys[1], w.sel[0], w.sel[1], (int)m, 0, 32, s));
    sel = w.sel[1];
  }
  hipLaunchKernelGGL(k_sparse_records, blocks(m), dim3(256), 0, s, sel, m, S, cell, call, err, parent, child,
                     call_out, err_out);
  return hipGetLastError();
}

hipError_t compact_links(LinkWork& w, const unsigned long long* call, const unsigned long long* err, uint64_t SS,
                         uint32_t S, const int32_t* rank, uint32_t nrank, int32_t* parent, int32_t* child,
                         int64_t* call_out, int64_t* err_out, uint64_t* n_out, hipStream_t s) {
  GTRY(compact_select(w, call, SS, n_out, s));
  return compact_records(w, call, err, *n_out, S, rank, nrank, parent, child, call_out, err_out, s);
}

}  // namespace zdl
