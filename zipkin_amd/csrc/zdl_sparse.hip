// zdl_sparse.hip — sorted-list link table for large service dictionaries (zdl_sparse.h).
#include "zdl_sparse.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
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

struct Gather {
  const unsigned long long* v;
  __host__ __device__ unsigned long long operator()(uint32_t i) const { return v[i]; }
};

using GatherIt = hipcub::TransformInputIterator<unsigned long long, Gather, const uint32_t*>;
using IdxIt = hipcub::CountingInputIterator<uint32_t>;

__global__ void k_iota32(uint32_t* p, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (uint32_t)i;
}

// ---- run-length reduction of the sorted log (replaces a hipcub ReduceByKey over a transform
// iterator: 356 us for C5's 34 M entries). Keys are cell << 1 | error, sorted, so each cell's
// entries are one run of its even key (no error) followed by one run of its odd key (error).
// Pass 1 lists the key runs (start position, key) in order; pass 2 folds each cell's one or two
// key runs into (cell, call = entries, err = odd entries). Each pass counts per tile, scans the
// tile counts, then emits at the scanned offsets.
constexpr int RL_T = 256;
constexpr int RL_PK = 16, RL_TK = RL_T * RL_PK;  // key-run pass: 4096 entries a tile
constexpr int RL_PC = 8, RL_TC = RL_T * RL_PC;   // cell pass: 2048 runs a tile
// one pad word per 32: a thread's consecutive entries sit on distinct LDS banks
__device__ __forceinline__ int rlx(int i) { return i + (i >> 5); }
template <int TILE>
constexpr int rl_lds() { return TILE + TILE / 32 + 2; }

// block-wide exclusive scan of one value per thread (RL_T threads); returns the total in *tot
__device__ __forceinline__ uint32_t rl_scan(uint32_t v, uint32_t* sh, uint32_t* tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(x, d, 64);
    if (lane >= d) x += u;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t base = 0, all = 0;
#pragma unroll
  for (int k = 0; k < RL_T / 64; ++k) {
    base += k < w ? sh[k] : 0u;
    all += sh[k];
  }
  __syncthreads();
  *tot = all;
  return base + x - v;
}

// Tile t of a[0, n) (TILE entries + `extra` after it) into LDS, coalesced, padded; the entry
// before it into *prev (~0 for the first); ~0 past n
template <int TILE>
__device__ __forceinline__ void rl_load(const uint32_t* __restrict__ a, uint64_t n, uint64_t t, uint32_t* tile,
                                        uint32_t* prev, int extra = 0) {
  const uint64_t t0 = t * TILE;
  for (int k = threadIdx.x; k < TILE + extra; k += RL_T) tile[rlx(k)] = t0 + k < n ? a[t0 + k] : ~0u;
  if (prev && threadIdx.x == 0) *prev = t0 ? a[t0 - 1] : ~0u;
  __syncthreads();
}

// heads in a thread's PER consecutive entries, as a bit mask. MODE 0: key changes; 1: cell
// (key >> 1) changes
template <int MODE, int PER>
__device__ __forceinline__ uint32_t rl_heads(const uint32_t* tile, uint32_t prev, uint64_t g0, uint64_t n) {
  uint32_t h = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = threadIdx.x * PER + j;
    const uint32_t k = tile[rlx(i)], p = i ? tile[rlx(i - 1)] : prev;
    const bool head = MODE == 0 ? k != p : (k >> 1) != (p >> 1);
    h |= (g0 + j < n && (g0 + j == 0 || head)) ? (1u << j) : 0u;
  }
  return h;
}

// per tile: how many heads
template <int MODE, int PER>
__global__ void __launch_bounds__(RL_T) k_rl_count(const uint32_t* __restrict__ a, const uint64_t* n_dev, uint64_t n_host,
                                                   uint32_t* __restrict__ cnt) {
  constexpr int TILE = RL_T * PER;
  __shared__ uint32_t tile[rl_lds<TILE>()];
  __shared__ uint32_t prev, sh[RL_T / 64];
  const uint64_t n = n_dev ? *n_dev : n_host;
  if ((uint64_t)blockIdx.x * TILE >= n) {
    if (threadIdx.x == 0) cnt[blockIdx.x] = 0;
    return;
  }
  rl_load<TILE>(a, n, blockIdx.x, tile, &prev);
  const uint32_t h = rl_heads<MODE, PER>(tile, prev, (uint64_t)blockIdx.x * TILE + threadIdx.x * PER, n);
  uint32_t tot;
  (void)rl_scan((uint32_t)__popc(h), sh, &tot);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// Key runs -> (kp = start position, kv = key) at the scanned offsets, staged in LDS so that the
// stores are coalesced; *n_out = the run count R
__global__ void __launch_bounds__(RL_T) k_rl_keys(const uint32_t* __restrict__ keys, uint64_t n, const uint32_t* __restrict__ off,
                                                  const uint32_t* __restrict__ cnt, uint32_t ntiles,
                                                  uint32_t* __restrict__ kp, uint32_t* __restrict__ kv,
                                                  uint64_t* __restrict__ n_out) {
  __shared__ uint32_t tile[rl_lds<RL_TK>()];
  __shared__ uint32_t sp[RL_TK], sv[RL_TK];
  __shared__ uint32_t prev, sh[RL_T / 64];
  if (blockIdx.x == 0 && threadIdx.x == 0) *n_out = (uint64_t)off[ntiles - 1] + cnt[ntiles - 1];
  rl_load<RL_TK>(keys, n, blockIdx.x, tile, &prev);
  const uint64_t g0 = (uint64_t)blockIdx.x * RL_TK + threadIdx.x * RL_PK;
  const uint32_t h = rl_heads<0, RL_PK>(tile, prev, g0, n);
  uint32_t tot;
  uint32_t o = rl_scan((uint32_t)__popc(h), sh, &tot);
  for (int j = 0; j < RL_PK; ++j)
    if ((h >> j) & 1u) {
      sp[o] = (uint32_t)(g0 + j);
      sv[o] = tile[rlx(threadIdx.x * RL_PK + j)];
      ++o;
    }
  __syncthreads();
  const uint32_t base = off[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < tot; i += RL_T) {
    kp[base + i] = sp[i];
    kv[base + i] = sv[i];
  }
}

// Over the R key runs: each cell head folds its one or two runs (the error run follows) into
// (cell, call, err), staged in LDS, stored coalesced; *U = the cell count
__global__ void __launch_bounds__(RL_T) k_rl_cells(const uint32_t* __restrict__ kv, const uint32_t* __restrict__ kp,
                                                   const uint64_t* __restrict__ R_dev, uint64_t E,
                                                   const uint32_t* __restrict__ off, uint32_t* __restrict__ cell,
                                                   unsigned long long* __restrict__ call,
                                                   unsigned long long* __restrict__ err, uint64_t* __restrict__ U) {
  __shared__ uint32_t tv[rl_lds<RL_TC>()], tp[rl_lds<RL_TC>()];
  __shared__ uint32_t sc[RL_TC], sn[RL_TC], se[RL_TC];
  __shared__ uint32_t prev, sh[RL_T / 64];
  const uint64_t R = *R_dev;
  if ((uint64_t)blockIdx.x * RL_TC >= R) return;
  rl_load<RL_TC>(kv, R, blockIdx.x, tv, &prev, 1);
  rl_load<RL_TC>(kp, R, blockIdx.x, tp, nullptr, 2);
  const uint64_t t0 = (uint64_t)blockIdx.x * RL_TC, g0 = t0 + threadIdx.x * RL_PC;
  const uint32_t h = rl_heads<1, RL_PC>(tv, prev, g0, R);
  uint32_t tot;
  uint32_t o = rl_scan((uint32_t)__popc(h), sh, &tot);
  // a run's end: the next run's start (E past the last run)
  auto end_of = [&](uint64_t k) -> uint64_t { return k + 1 < R ? (uint64_t)tp[rlx((int)(k + 1 - t0))] : E; };
  for (int j = 0; j < RL_PC; ++j)
    if ((h >> j) & 1u) {
      const uint64_t k = g0 + j;
      const int i = (int)(k - t0);
      const uint32_t v = tv[rlx(i)];
      const uint64_t e0 = end_of(k), len = e0 - tp[rlx(i)];
      uint64_t c = len, x = (v & 1u) ? len : 0;
      if (!(v & 1u) && k + 1 < R && tv[rlx(i + 1)] == (v | 1u)) {  // the cell's error run follows
        const uint64_t e1 = end_of(k + 1);
        c += e1 - e0;
        x = e1 - e0;
      }
      sc[o] = v >> 1;
      sn[o] = (uint32_t)c;  // a put logs < 2^31 entries
      se[o] = (uint32_t)x;
      ++o;
    }
  __syncthreads();
  const uint32_t base = off[blockIdx.x];
  if (t0 + RL_TC >= R && threadIdx.x == 0) *U = (uint64_t)base + tot;
  for (uint32_t i = threadIdx.x; i < tot; i += RL_T) {
    cell[base + i] = sc[i];
    call[base + i] = sn[i];
    err[base + i] = se[i];
  }
}

// The log's sort: hipcub's radix sort (onesweep, 8-bit digits: four passes over C5's 28-bit keys;
// rocprim onesweep configs with 10- and 11-bit digits, three passes, were measured and not kept)
hipError_t sort_log(void* tmp, size_t& bytes, const uint32_t* in, uint32_t* out, uint64_t E, int key_bits,
                    hipStream_t s) {
  return hipcub::DeviceRadixSort::SortKeys(tmp, bytes, in, out, (int)E, 0, key_bits, s);
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
  if (!w.d_count) STRY(hipMalloc((void**)&w.d_count, 16));  // [0]: output counts, [1]: sparse_accumulate's R
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
  // the sorted log, then its key runs: the run starts in bcell's space is reused as kp (the
  // reduced cells land in bcell only in the last pass, from kv / kp held in keys' partner)
  const uint32_t nt = (uint32_t)((E + RL_TK - 1) / RL_TK), nc = (uint32_t)((E + RL_TC - 1) / RL_TC);
  size_t k2 = w.idx_cap;
  STRY(grow(w.idx_sorted, k2, 2 * E + 2 * (size_t)nc + 8));  // kp, kv, tile counts, offsets
  w.idx_cap = k2;
  uint32_t* const kp = w.idx_sorted;
  uint32_t* const kv = kp + E;
  uint32_t* const tc = kv + E;
  uint32_t* const to = tc + nc;
  uint64_t* const Rd = w.d_count + 1;
  size_t a = 0, b = 0;
  STRY(sort_log(nullptr, a, log, w.keys, E, key_bits, s));
  STRY(hipcub::DeviceScan::ExclusiveSum(nullptr, b, tc, to, (int)nc, s));
  STRY(scratch(w, std::max(a, b)));
  size_t bytes = w.tmp_bytes;
  STRY(sort_log(w.tmp, bytes, log, w.keys, E, key_bits, s));
  hipLaunchKernelGGL((k_rl_count<0, RL_PK>), dim3(nt), dim3(RL_T), 0, s, (const uint32_t*)w.keys,
                     (const uint64_t*)nullptr, E, tc);
  STRY(hipGetLastError());
  bytes = w.tmp_bytes;
  STRY(hipcub::DeviceScan::ExclusiveSum(w.tmp, bytes, tc, to, (int)nt, s));
  hipLaunchKernelGGL(k_rl_keys, dim3(nt), dim3(RL_T), 0, s, (const uint32_t*)w.keys, E, (const uint32_t*)to,
                     (const uint32_t*)tc, nt, kp, kv, Rd);
  STRY(hipGetLastError());
  hipLaunchKernelGGL((k_rl_count<1, RL_PC>), dim3(nc), dim3(RL_T), 0, s, (const uint32_t*)kv, (const uint64_t*)Rd, E, tc);
  STRY(hipGetLastError());
  bytes = w.tmp_bytes;
  STRY(hipcub::DeviceScan::ExclusiveSum(w.tmp, bytes, tc, to, (int)nc, s));
  hipLaunchKernelGGL(k_rl_cells, dim3(nc), dim3(RL_T), 0, s, (const uint32_t*)kv, (const uint32_t*)kp,
                     (const uint64_t*)Rd, E, (const uint32_t*)to, w.bcell, w.bcall, w.berr, w.d_count);
  STRY(hipGetLastError());
  uint64_t U = 0;
  STRY(read_count(w, s, &U));
  return merge_into(w, t, w.bcell, w.bcall, w.berr, U, s);
}

hipError_t sparse_reserve(SparseTable& t, size_t n) { return ensure_table(t, n); }

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
