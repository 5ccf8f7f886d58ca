// zdl_store.hip — InMemoryStorage's trace index on the device (zdl_store_index.h).
//
// All passes are HBM-bound gathers, flag/scan kernels, stable LSD radix sorts and merges
// (hipCUB). accept keeps the resident index current: the batch is sorted twice by (low id,
// timestamp, arrival) and (low id, first arrival of its key, arrival) and merged into the two
// resident orders. A getDependencies selection then filters the alive spans of the resident
// order and sorts one key per trace; an eviction sorts one key per trace. Counts (alive spans,
// traces, the eviction result) are the only values that come back to the host.
#include "zdl_store_index.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace zdl {
namespace {

constexpr uint64_t kSign = 1ull << 63;  // int64 -> order-preserving uint64

inline dim3 grid_of(uint64_t n) { return dim3((unsigned)std::max<uint64_t>((n + 255) / 256, 1)); }

#define ITRY(expr)                   \
  do {                               \
    hipError_t _e = (expr);          \
    if (_e != hipSuccess) return _e; \
  } while (0)

// ZDL_INDEX_TRACE=1: synchronise after every step and name the one that fails (diagnostics)
bool trace_steps() {
  static const bool on = getenv("ZDL_INDEX_TRACE") != nullptr;
  return on;
}
hipError_t step_done(hipStream_t s, int line) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && trace_steps()) e = hipStreamSynchronize(s);
  if (e != hipSuccess && trace_steps()) fprintf(stderr, "zdl_store.hip:%d: %s\n", line, hipGetErrorString(e));
  return e;
}

#define LAUNCH(kernel, n, ...)                                                    \
  do {                                                                            \
    hipLaunchKernelGGL(kernel, grid_of(n), dim3(256), 0, s, __VA_ARGS__);          \
    ITRY(step_done(s, __LINE__));                                                 \
  } while (0)

// key[i] = src[idx[i]] ^ x  (x = kSign turns a timestamp into an unsigned key)
__global__ void k_take(const uint64_t* __restrict__ src, const uint32_t* __restrict__ idx, uint64_t x,
                       uint64_t* __restrict__ key, uint64_t m) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) key[i] = src[idx[i]] ^ x;
}

// key[i] = src[outer[inner[i]]]
__global__ void k_take2(const uint64_t* __restrict__ src, const uint32_t* __restrict__ outer,
                        const uint32_t* __restrict__ inner, uint64_t* __restrict__ key, uint64_t m) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) key[i] = src[outer[inner[i]]];
}

// key[i] = the 128-bit-id bit of span idx[i] (alive bit 1)
__global__ void k_wide_key(const uint8_t* __restrict__ alive, const uint32_t* __restrict__ idx,
                           uint32_t* __restrict__ key, uint64_t m) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) key[i] = (alive[idx[i]] >> 1) & 1u;
}

__global__ void k_iota32(uint32_t* __restrict__ out, uint64_t m) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) out[i] = (uint32_t)i;
}

__global__ void k_iota_from(uint32_t* __restrict__ out, uint64_t base, uint64_t m) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) out[i] = (uint32_t)(base + i);
}

// key[i] = src[idx[i]] (32-bit)
__global__ void k_take32(const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx, uint32_t* __restrict__ key,
                         uint64_t m) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) key[i] = src[idx[i]];
}

// fs[bk[i]] = bk[head[i]]: a span's first arrival among the spans of its (low id, timestamp) key
__global__ void k_first_arrival(const uint32_t* __restrict__ bk, const uint32_t* __restrict__ head, uint64_t m,
                                uint32_t* __restrict__ fs) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) fs[bk[i]] = bk[head[i]];
}

// the resident orders' comparators (positions compared through the columns; the position last)
struct LoTsLess {
  const uint64_t* lo;
  const int64_t* ts;
  __device__ bool operator()(uint32_t a, uint32_t b) const {
    if (lo[a] != lo[b]) return lo[a] < lo[b];
    if (ts[a] != ts[b]) return ts[a] < ts[b];
    return a < b;
  }
};
struct LoFsLess {
  const uint64_t* lo;
  const uint32_t* fs;
  __device__ bool operator()(uint32_t a, uint32_t b) const {
    if (lo[a] != lo[b]) return lo[a] < lo[b];
    if (fs[a] != fs[b]) return fs[a] < fs[b];
    return a < b;
  }
};
struct AliveOf {
  const uint8_t* alive;
  __device__ bool operator()(uint32_t p) const { return alive[p] != 0; }
};

// flag[i] = a new run of equal keys starts at i (keys sorted)
__global__ void k_runs(const uint64_t* __restrict__ key, uint64_t m, uint8_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) flag[i] = i == 0 || key[i] != key[i - 1];
}

// flag[i] = the low id of span v[i] differs from v[i - 1]'s (v sorted by low id): k_take into a
// key array and k_runs over it in one pass
__global__ void k_runs_of(const uint64_t* __restrict__ lo, const uint32_t* __restrict__ v, uint64_t m,
                          uint8_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) flag[i] = i == 0 || lo[v[i]] != lo[v[i - 1]];
}

// ---- the set positions of flag[0..m) in order (offsets_of): a count pass and a write pass of
// CF_TILE flags per workgroup (16 per thread, one 16-B load), the workgroups' starts from an
// exclusive scan of the counts in between. (hipCUB's DeviceSelect::Flagged took 229 us for 10M
// flags; these two passes read the flags twice, 20 MB.)
constexpr int CF_WG = 256, CF_PER = 16, CF_TILE = CF_WG * CF_PER;

// bit k: flag[i0 + k] != 0, k < 16
__device__ __forceinline__ uint32_t flag_bits16(const uint8_t* __restrict__ flag, uint64_t i0, uint64_t m) {
  uint32_t b = 0;
  if (i0 + CF_PER <= m) {
    const uint4 v = *reinterpret_cast<const uint4*>(flag + i0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if ((w[q] >> (8 * k)) & 0xFFu) b |= 1u << (4 * q + k);
  } else {
    for (int k = 0; k < CF_PER; ++k)
      if (i0 + (uint64_t)k < m && flag[i0 + k]) b |= 1u << k;
  }
  return b;
}

// exclusive prefix of x over the CF_WG threads; *total = the sum (call once per kernel)
__device__ __forceinline__ uint32_t cf_scan(uint32_t x, uint32_t* total) {
  __shared__ uint32_t ws[CF_WG / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) ws[w] = incl;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < CF_WG / 64; ++k) {
    before += k < w ? ws[k] : 0u;
    tot += ws[k];
  }
  *total = tot;
  return before + incl - x;
}

__global__ void __launch_bounds__(CF_WG) k_flag_count(const uint8_t* __restrict__ flag, uint64_t m,
                                                      uint32_t* __restrict__ cnt) {
  const uint64_t i0 = ((uint64_t)blockIdx.x * CF_WG + threadIdx.x) * CF_PER;
  uint32_t tot;
  (void)cf_scan((uint32_t)__popc(flag_bits16(flag, i0, m)), &tot);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// start: the exclusive prefix of the workgroups' counts. The last workgroup also writes the
// total into d[0] and m as the closing offset.
__global__ void __launch_bounds__(CF_WG) k_flag_write(const uint8_t* __restrict__ flag, uint64_t m,
                                                      const uint32_t* __restrict__ start, uint64_t* __restrict__ off,
                                                      uint64_t* __restrict__ d) {
  const uint64_t i0 = ((uint64_t)blockIdx.x * CF_WG + threadIdx.x) * CF_PER;
  uint32_t bits = flag_bits16(flag, i0, m), tot;
  uint64_t at = (uint64_t)start[blockIdx.x] + cf_scan((uint32_t)__popc(bits), &tot);
  while (bits) {
    off[at++] = i0 + (uint64_t)(__ffs(bits) - 1);
    bits &= bits - 1u;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    const uint64_t T = (uint64_t)start[blockIdx.x] + tot;
    d[0] = T;
    off[T] = m;
  }
}

// flag[i] = a trace starts at position i of perm (low id changes; or high id, when given)
// (alive: bit 1 = the trace id is 128-bit, normalized to 32 hex characters; with hi, the strict
// grouping's key)
__global__ void k_trace_heads(const uint64_t* __restrict__ lo, const uint64_t* __restrict__ hi,
                              const uint8_t* __restrict__ alive, const uint32_t* __restrict__ perm, uint64_t m,
                              uint8_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  bool h = i == 0;
  if (!h) {
    const uint32_t a = perm[i - 1], b = perm[i];
    h = lo[a] != lo[b] || (hi && (hi[a] != hi[b] || ((alive[a] ^ alive[b]) & 2)));
  }
  flag[i] = h;
}


__global__ void k_widen(const uint8_t* __restrict__ flag, uint64_t m, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) out[i] = flag[i];
}

// (lowTraceId, timestamp) key runs over v (sorted by low id, timestamp, position):
// out[i] = i where a key starts, else 0 (a max-scan then names each span's key head)
__global__ void k_key_heads(const uint64_t* __restrict__ lo, const int64_t* __restrict__ ts,
                            const uint32_t* __restrict__ v, uint64_t m, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  bool h = i == 0;
  if (!h) {
    const uint32_t a = v[i - 1], b = v[i];
    h = lo[a] != lo[b] || ts[a] != ts[b];
  }
  out[i] = h ? (uint32_t)i : 0u;
}



// The keys' smallest and largest value: each workgroup's pair into part[blockIdx.x] and
// part[nb + blockIdx.x], then k_minmax_final into d[2], d[3] (one atomic per wave on two
// addresses serialised at the memory side: 368 us for 1M keys)
__device__ __forceinline__ void key_minmax(uint64_t k, bool on, uint64_t* __restrict__ part) {
  __shared__ unsigned long long wmn[4], wmx[4];
  unsigned long long mn = on ? k : ~0ull, mx = on ? k : 0ull;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    wmn[w] = mn;
    wmx[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
      mn = wmn[i] < mn ? wmn[i] : mn;
      mx = wmx[i] > mx ? wmx[i] : mx;
    }
    part[blockIdx.x] = mn;
    part[gridDim.x + blockIdx.x] = mx;
  }
}

__global__ void __launch_bounds__(1024) k_minmax_final(const uint64_t* __restrict__ part, uint64_t nb,
                                                       uint64_t* __restrict__ d) {
  __shared__ unsigned long long wmn[16], wmx[16];
  unsigned long long mn = ~0ull, mx = 0ull;
  for (uint64_t i = threadIdx.x; i < nb; i += blockDim.x) {
    mn = part[i] < mn ? part[i] : mn;
    mx = part[nb + i] > mx ? part[nb + i] : mx;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if ((threadIdx.x & 63) == 0) {
    wmn[threadIdx.x >> 6] = mn;
    wmx[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 16; ++i) {
      mn = wmn[i] < mn ? wmn[i] : mn;
      mx = wmx[i] > mx ? wmx[i] : mx;
    }
    d[1] = 0;  // k_place_seg's long-trace count
    d[2] = mn;
    d[3] = mx;
  }
}

// segment j's newest timestamp (the last span of j in v, sorted by timestamp inside a low id),
// as a descending key; segments fed in reverse (descending low id) so a stable sort breaks
// newest-timestamp ties by descending low id. Each workgroup's key range into part.
__global__ void __launch_bounds__(256) k_seg_newest_mm(const uint64_t* __restrict__ seg, uint64_t T,
                                                       const uint32_t* __restrict__ v, const int64_t* __restrict__ ts,
                                                       uint64_t* __restrict__ key, uint32_t* __restrict__ val,
                                                       uint64_t* __restrict__ part) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t k = 0;
  if (j < T) {
    k = ~((uint64_t)ts[v[seg[j + 1] - 1]] ^ kSign);
    key[T - 1 - j] = k;
    val[T - 1 - j] = (uint32_t)j;
  }
  key_minmax(k, j < T, part);
}

// key - lo, as 32 bits (the range fits) or 64
__global__ void k_key_rebase32(const uint64_t* __restrict__ key, uint64_t lo, uint64_t T, uint32_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < T) out[j] = (uint32_t)(key[j] - lo);
}
__global__ void k_key_rebase64(uint64_t* __restrict__ key, uint64_t lo, uint64_t T) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < T) key[j] -= lo;
}

// The traces of ranks [256 b, 256 b + 256) (order[r] = its segment j) copied to their new places
// start[r] of perm: each thread claims its trace's slots of the workgroup's span run in an LDS
// owner map, then the run is copied span-parallel (writes coalesced, reads in the traces'
// runs). A trace longer than PLACE_SMALL spans is listed (d[1] counts) for k_place_big. (A
// thread per trace copying its own spans took 115 us for C2's 1M traces: every lane of an
// access in another line.)
constexpr int PL_WG = 256;
constexpr uint32_t PLACE_SMALL = 64;
__global__ void __launch_bounds__(PL_WG) k_place_seg(const uint32_t* __restrict__ v, const uint64_t* __restrict__ seg,
                                                     const uint32_t* __restrict__ order,
                                                     const uint32_t* __restrict__ start, uint64_t T,
                                                     uint32_t* __restrict__ perm, uint32_t* __restrict__ big,
                                                     uint64_t* __restrict__ d) {
  __shared__ uint32_t pre[PL_WG], src[PL_WG], dst[PL_WG], ws[PL_WG / 64];
  __shared__ uint8_t owner[PL_WG * PLACE_SMALL];
  const uint64_t r = (uint64_t)blockIdx.x * PL_WG + threadIdx.x;
  uint32_t sz = 0;
  if (r < T) {
    const uint32_t j = order[r];
    const uint64_t b = seg[j], e = seg[j + 1];
    if (e - b > PLACE_SMALL) {
      big[atomicAdd(reinterpret_cast<unsigned long long*>(d + 1), 1ull)] = (uint32_t)r;
    } else {
      sz = (uint32_t)(e - b);
      src[threadIdx.x] = (uint32_t)b;
      dst[threadIdx.x] = start[r];
    }
  }
  // exclusive prefix of the sizes over the workgroup
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = sz;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) ws[w] = incl;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (int k = 0; k < PL_WG / 64; ++k) {
    before += k < w ? ws[k] : 0u;
    total += ws[k];
  }
  const uint32_t p0 = before + incl - sz;
  pre[threadIdx.x] = p0;
  for (uint32_t k = 0; k < sz; ++k) owner[p0 + k] = (uint8_t)threadIdx.x;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < total; i += PL_WG) {
    const uint32_t q = owner[i], k = i - pre[q];
    perm[dst[q] + k] = v[src[q] + k];
  }
}

// the listed long traces, a workgroup each (grid-stride over the list)
__global__ void k_place_big(const uint32_t* __restrict__ v, const uint64_t* __restrict__ seg,
                            const uint32_t* __restrict__ order, const uint32_t* __restrict__ start,
                            uint32_t* __restrict__ perm, const uint32_t* __restrict__ big, const uint64_t* __restrict__ d) {
  const uint64_t nb = d[1];
  for (uint64_t q = blockIdx.x; q < nb; q += gridDim.x) {
    const uint32_t r = big[q], j = order[r];
    const uint64_t b = seg[j], e = seg[j + 1];
    uint32_t* out = perm + start[r];
    for (uint64_t k = b + threadIdx.x; k < e; k += blockDim.x) out[k - b] = v[k];
  }
}

// segment j's smallest timestamp (eviction order key); segments come in ascending low id
__global__ void k_seg_oldest(const uint64_t* __restrict__ seg, uint64_t T, const uint32_t* __restrict__ v,
                             const int64_t* __restrict__ ts, uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= T) return;
  uint64_t best = ~0ull;
  for (uint64_t e = seg[j]; e < seg[j + 1]; ++e) best = std::min(best, (uint64_t)ts[v[e]] ^ kSign);
  key[j] = best;
  val[j] = (uint32_t)j;
}

__global__ void k_seg_sizes(const uint64_t* __restrict__ seg, const uint32_t* __restrict__ order, uint64_t T,
                            uint32_t* __restrict__ size) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < T) size[r] = (uint32_t)(seg[order[r] + 1] - seg[order[r]]);
}

__global__ void k_rank_of(const uint32_t* __restrict__ order, uint64_t T, uint32_t* __restrict__ rank) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < T) rank[order[r]] = (uint32_t)r;
}


__global__ void k_new_off(const uint32_t* __restrict__ start, uint64_t T, uint64_t m, uint64_t* __restrict__ off) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < T) off[r] = start[r];
  if (r == T) off[T] = m;
}

// (lowTraceId, traceId) group heads over u (span indexes into v, grouped, ascending inside)
__global__ void k_group_heads(const uint64_t* __restrict__ lo, const uint64_t* __restrict__ hi,
                              const uint8_t* __restrict__ alive, const uint32_t* __restrict__ v,
                              const uint32_t* __restrict__ u, uint64_t m, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  bool h = i == 0;
  if (!h) {
    const uint32_t a = v[u[i - 1]], b = v[u[i]];
    h = lo[a] != lo[b] || hi[a] != hi[b] || ((alive[a] ^ alive[b]) & 2);
  }
  out[i] = h ? (uint32_t)i : 0u;
}

__global__ void k_group_first(const uint32_t* __restrict__ u, const uint32_t* __restrict__ head, uint64_t m,
                              uint32_t* __restrict__ first) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) first[u[i]] = u[head[i]];
}

__global__ void k_evict_init(uint64_t T, uint64_t m, uint64_t* __restrict__ d) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    d[1] = T - 1;  // not found: every trace goes (the store runs empty)
    d[2] = m;
    d[3] = 1;
  }
}

// the first rank whose cumulative span count reaches R
__global__ void k_evict_find(const uint32_t* __restrict__ cum, uint64_t T, uint64_t R, uint64_t* __restrict__ d) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= T) return;
  const uint64_t c = cum[r], p = r ? cum[r - 1] : 0;
  if (c >= R && p < R) {
    d[1] = r;
    d[2] = c;
    d[3] = 0;
  }
}

__global__ void k_evict_mark(const uint32_t* __restrict__ v, const uint32_t* __restrict__ segid1,
                             const uint32_t* __restrict__ rank, const uint64_t* __restrict__ d, uint64_t m,
                             uint8_t* __restrict__ alive) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m && rank[segid1[i] - 1] <= d[1]) alive[v[i]] = 0;
}

template <class T>
hipError_t grow(T*& p, size_t n) {
  if (p) (void)hipFree(p);
  p = nullptr;
  return hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T));
}

hipError_t reserve(IndexWork& w, uint64_t n) {
  if (!w.d) {
    ITRY(hipMalloc((void**)&w.d, 4 * sizeof(uint64_t)));
    ITRY(hipHostMalloc((void**)&w.h, 4 * sizeof(uint64_t), hipHostMallocDefault));
  }
  if (n <= w.cap) return hipSuccess;
  for (auto*& p : w.k) ITRY(grow(p, n));
  for (auto*& p : w.v) ITRY(grow(p, n));
  for (auto*& p : w.u) ITRY(grow(p, n));
  // sk[1] also holds k_seg_newest_mm's per-workgroup min / max partials (2 per 256 traces)
  for (auto*& p : w.sk) ITRY(grow(p, std::max<uint64_t>(n, 2 * grid_of(n).x)));
  for (auto*& p : w.sv) ITRY(grow(p, n));
  ITRY(grow(w.seg, n + 1));
  ITRY(grow(w.flag, n));
  ITRY(grow(w.bc, 2 * (n / CF_TILE + 2)));
  w.cap = n;
  return hipSuccess;
}

// runs a hipCUB call twice: size query, then with (grown) scratch
template <class F>
hipError_t cub_at(IndexWork& w, hipStream_t s, int line, F f) {
  size_t need = 0;
  ITRY(f(nullptr, need));
  if (need > w.tmp_bytes) {
    if (w.tmp) (void)hipFree(w.tmp);
    w.tmp = nullptr;
    w.tmp_bytes = 0;
    ITRY(hipMalloc(&w.tmp, need));
    w.tmp_bytes = need;
  }
  size_t b = w.tmp_bytes;
  ITRY(f(w.tmp, b));
  return step_done(s, line);
}

hipError_t fetch(IndexWork& w, int k, hipStream_t s) {
  ITRY(hipMemcpyAsync(w.h, w.d, k * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  return hipStreamSynchronize(s);
}

// rocprim's radix sort, onesweep at every size above one block: its default config switches to
// a merge sort up to 2^20 items (block sort + 20 merge passes: 190 us for 1M trace keys, against
// tens of us for a few radix passes)
using StoreSortCfg = ::rocprim::radix_sort_config<::rocprim::default_config, ::rocprim::default_config,
                                                  ::rocprim::default_config, 0>;

hipError_t sort64(IndexWork& w, const uint64_t* kin, uint64_t* kout, const uint32_t* vin, uint32_t* vout,
                  uint64_t m, hipStream_t s, int end_bit = 64) {
  return cub_at(w, s, __LINE__, [&](void* t, size_t& b) {
    return ::rocprim::radix_sort_pairs<StoreSortCfg>(t, b, kin, kout, vin, vout, (size_t)m, 0u, (unsigned)end_bit, s);
  });
}

hipError_t sort32(IndexWork& w, const uint32_t* kin, uint32_t* kout, const uint32_t* vin, uint32_t* vout,
                  uint64_t m, hipStream_t s, int end_bit = 32) {
  return cub_at(w, s, __LINE__ * 64 + end_bit, [&](void* t, size_t& b) {
    return ::rocprim::radix_sort_pairs<StoreSortCfg>(t, b, kin, kout, vin, vout, (size_t)m, 0u, (unsigned)end_bit, s);
  });
}

hipError_t max_scan(IndexWork& w, const uint32_t* in, uint32_t* out, uint64_t m, hipStream_t s) {
  return cub_at(w, s, __LINE__, [&](void* t, size_t& b) {
    return hipcub::DeviceScan::InclusiveScan(t, b, in, out, hipcub::Max(), (int)m, s);
  });
}

hipError_t sum_scan(IndexWork& w, const uint32_t* in, uint32_t* out, uint64_t m, bool inclusive, hipStream_t s) {
  return cub_at(w, s, __LINE__, [&](void* t, size_t& b) {
    return inclusive ? hipcub::DeviceScan::InclusiveSum(t, b, in, out, (int)m, s)
                     : hipcub::DeviceScan::ExclusiveSum(t, b, in, out, (int)m, s);
  });
}

// the run heads of flag[0..m) as CSR offsets (off[0..T], T into w.d[0]); returns T
hipError_t offsets_of(IndexWork& w, const uint8_t* flag, uint64_t m, uint64_t* off, uint64_t* T, hipStream_t s) {
  const uint64_t nb = (m + CF_TILE - 1) / CF_TILE;  // m >= 1
  hipLaunchKernelGGL(k_flag_count, dim3((unsigned)nb), dim3(CF_WG), 0, s, flag, m, w.bc);
  ITRY(step_done(s, __LINE__));
  ITRY(cub_at(w, s, __LINE__, [&](void* t, size_t& b) {
    return hipcub::DeviceScan::ExclusiveSum(t, b, w.bc, w.bc + nb, (int)nb, s);
  }));
  hipLaunchKernelGGL(k_flag_write, dim3((unsigned)nb), dim3(CF_WG), 0, s, flag, m, w.bc + nb, off, w.d);
  ITRY(step_done(s, __LINE__));
  ITRY(fetch(w, 1, s));
  *T = w.h[0];
  return hipSuccess;
}

}  // namespace

void IndexWork::release() {
  for (auto*& p : k) { if (p) (void)hipFree(p); p = nullptr; }
  for (auto*& p : v) { if (p) (void)hipFree(p); p = nullptr; }
  for (auto*& p : u) { if (p) (void)hipFree(p); p = nullptr; }
  for (auto*& p : sk) { if (p) (void)hipFree(p); p = nullptr; }
  for (auto*& p : sv) { if (p) (void)hipFree(p); p = nullptr; }
  if (seg) (void)hipFree(seg);
  if (flag) (void)hipFree(flag);
  if (bc) (void)hipFree(bc);
  if (tmp) (void)hipFree(tmp);
  if (d) (void)hipFree(d);
  if (h) (void)hipHostFree(h);
  for (auto* p : {bk, st, fs, mo})
    if (p) (void)hipFree(p);
  bk = st = fs = mo = nullptr;
  rcap = 0;
  ni = 0;
  seg = nullptr;
  flag = nullptr;
  bc = nullptr;
  tmp = nullptr;
  d = nullptr;
  h = nullptr;
  tmp_bytes = 0;
  cap = 0;
}

hipError_t index_alive(IndexWork& w, const uint8_t* alive, uint64_t n, uint32_t* out, uint64_t* m, hipStream_t s) {
  if (n >= (1ull << 31)) return hipErrorInvalidValue;
  ITRY(reserve(w, n));
  *m = 0;
  if (n == 0) return hipSuccess;
  ITRY(cub_at(w, s, __LINE__, [&](void* t, size_t& b) {
    // a predicate, not Flagged: the alive byte also carries the id-width bit (value 3), and the
    // flags of a flagged select may be summed as integers
    return hipcub::DeviceSelect::If(t, b, hipcub::CountingInputIterator<uint32_t>(0), out, w.d, (int)n, AliveOf{alive}, s);
  }));
  ITRY(fetch(w, 1, s));
  *m = w.h[0];
  return hipSuccess;
}

namespace {
// grows the resident arrays keeping positions [0, ni)
hipError_t reserve_resident(IndexWork& w, uint64_t n, hipStream_t s) {
  if (n <= w.rcap) return hipSuccess;
  const size_t cap = std::max<size_t>(n + n / 2, 1 << 16);
  uint32_t* nb[4] = {};
  for (auto*& p : nb) ITRY(hipMalloc((void**)&p, cap * sizeof(uint32_t)));
  if (w.ni) {
    ITRY(hipMemcpyAsync(nb[0], w.bk, w.ni * 4, hipMemcpyDeviceToDevice, s));
    ITRY(hipMemcpyAsync(nb[1], w.st, w.ni * 4, hipMemcpyDeviceToDevice, s));
    ITRY(hipMemcpyAsync(nb[2], w.fs, w.ni * 4, hipMemcpyDeviceToDevice, s));
    ITRY(hipStreamSynchronize(s));
  }
  for (auto* p : {w.bk, w.st, w.fs, w.mo})
    if (p) (void)hipFree(p);
  w.bk = nb[0];
  w.st = nb[1];
  w.fs = nb[2];
  w.mo = nb[3];
  w.rcap = cap;
  return hipSuccess;
}

template <class Cmp>
hipError_t merge_into(IndexWork& w, uint32_t*& res, const uint32_t* batch, uint64_t n0, uint64_t b, Cmp cmp,
                      hipStream_t s) {
  if (n0 == 0) {
    ITRY(hipMemcpyAsync(res, batch, b * 4, hipMemcpyDeviceToDevice, s));
    return step_done(s, __LINE__);
  }
  ITRY(cub_at(w, s, __LINE__, [&](void* t, size_t& bytes) {
    return hipcub::DeviceMerge::MergeKeys(t, bytes, res, (int)n0, batch, (int)b, w.mo, cmp, s);
  }));
  std::swap(res, w.mo);
  return hipSuccess;
}

// the alive positions of a resident order (stable): into out, their number into *m (a sync);
// every position when nothing is evicted
hipError_t alive_of(IndexWork& w, const uint32_t* order, const uint8_t* alive, uint64_t n, uint64_t n_alive,
                    uint32_t* out, uint64_t* m, hipStream_t s) {
  if (n_alive == n) {
    ITRY(hipMemcpyAsync(out, order, n * 4, hipMemcpyDeviceToDevice, s));
    *m = n;
    return step_done(s, __LINE__);
  }
  ITRY(cub_at(w, s, __LINE__, [&](void* t, size_t& b) {
    return hipcub::DeviceSelect::If(t, b, order, out, w.d, (int)n, AliveOf{alive}, s);
  }));
  ITRY(fetch(w, 1, s));
  *m = w.h[0];
  return hipSuccess;
}
}  // namespace

hipError_t index_update(IndexWork& w, const uint64_t* lo, const int64_t* ts, uint64_t n, hipStream_t s) {
  if (n >= (1ull << 31)) return hipErrorInvalidValue;
  if (w.ni > n) w.ni = 0;  // renumbered (compaction) or cleared: rebuild
  if (w.ni == n) return hipSuccess;
  ITRY(reserve(w, n));  // before any w buffer is named: reserve reallocates them
  ITRY(reserve_resident(w, n, s));
  const uint64_t n0 = w.ni, b = n - n0;
  const uint64_t* ts64 = reinterpret_cast<const uint64_t*>(ts);
  // the batch by (low id, timestamp, arrival): stable sorts by timestamp, then by low id
  LAUNCH(k_iota_from, b, w.v[0], n0, b);
  LAUNCH(k_take, b, ts64, w.v[0], kSign, w.k[0], b);
  ITRY(sort64(w, w.k[0], w.k[1], w.v[0], w.v[1], b, s));
  LAUNCH(k_take, b, lo, w.v[1], 0ull, w.k[0], b);
  ITRY(sort64(w, w.k[0], w.k[1], w.v[1], w.v[0], b, s));
  ITRY(merge_into(w, w.bk, w.v[0], n0, b, LoTsLess{lo, ts}, s));
  // every span's first arrival among its (low id, timestamp) key (the old ones' do not change:
  // a new span arrives after every indexed one)
  LAUNCH(k_key_heads, n, lo, ts, w.bk, n, w.u[0]);
  ITRY(max_scan(w, w.u[0], w.u[1], n, s));
  LAUNCH(k_first_arrival, n, w.bk, w.u[1], n, w.fs);
  // the batch by (low id, first arrival, arrival)
  LAUNCH(k_iota_from, b, w.v[0], n0, b);
  LAUNCH(k_take32, b, w.fs, w.v[0], w.u[2], b);
  ITRY(sort32(w, w.u[2], w.u[3], w.v[0], w.v[1], b, s));
  LAUNCH(k_take, b, lo, w.v[1], 0ull, w.k[0], b);
  ITRY(sort64(w, w.k[0], w.k[1], w.v[1], w.v[0], b, s));
  ITRY(merge_into(w, w.st, w.v[0], n0, b, LoFsLess{lo, w.fs}, s));
  w.ni = n;
  return hipSuccess;
}

hipError_t index_select(IndexWork& w, const uint64_t* lo, const uint64_t* hi, const int64_t* ts,
                        const uint8_t* alive, uint64_t n, uint64_t n_alive, int mode, uint32_t* perm,
                        uint64_t* off, uint64_t* n_sel, uint64_t* n_traces, hipStream_t s) {
  uint64_t m = 0;
  *n_sel = *n_traces = 0;
  if (n >= (1ull << 31)) return hipErrorInvalidValue;
  ITRY(index_update(w, lo, ts, n, s));  // accept keeps it current: normally nothing to do
  ITRY(reserve(w, n));  // before any w buffer is named: reserve reallocates them
  if (n == 0 || n_alive == 0) return hipSuccess;
  // low ids ascending, storage order inside (IMS:448-454); (low id, timestamp, arrival) for the
  // newest timestamps below. Nothing evicted: the resident orders themselves (no copy).
  const uint32_t* stored = w.st;
  const uint32_t* by_key = w.bk;
  if (n_alive != n) {
    ITRY(alive_of(w, w.st, alive, n, n_alive, w.v[1], &m, s));
    stored = w.v[1];
  } else {
    m = n;
  }
  if (m == 0) return hipSuccess;
  if (mode == SEL_NEWEST && n_alive != n) {
    uint64_t m2 = 0;
    ITRY(alive_of(w, w.bk, alive, n, n_alive, w.u[3], &m2, s));
    if (m2 != m) return hipErrorUnknown;
    by_key = w.u[3];
  }
  uint64_t T = 0;
  if (mode == SEL_ALL) {
    ITRY(hipMemcpyAsync(perm, stored, m * 4, hipMemcpyDeviceToDevice, s));
    LAUNCH(k_runs_of, m, lo, stored, m, w.flag);
    ITRY(offsets_of(w, w.flag, m, off, &T, s));
  } else if (mode == SEL_NEWEST) {
    LAUNCH(k_runs_of, m, lo, stored, m, w.flag);
    ITRY(offsets_of(w, w.flag, m, w.seg, &T, s));  // the same low-id segments in by_key and stored
    // one key per trace (its newest timestamp, descending), sorted over the bits in which the
    // keys differ: 32-bit keys when their range fits (a selection of under ~71 minutes of
    // microsecond timestamps), the 64-bit ones from that range's top bit down otherwise
    LAUNCH(k_seg_newest_mm, T, w.seg, T, by_key, ts, w.sk[0], w.sv[0], w.sk[1]);
    hipLaunchKernelGGL(k_minmax_final, dim3(1), dim3(1024), 0, s, w.sk[1], (uint64_t)grid_of(T).x, w.d);
    ITRY(fetch(w, 4, s));
    const uint64_t klo = w.h[2], span = w.h[3] - w.h[2];
    const int bits = span == 0 ? 0 : 64 - __builtin_clzll(span);
    if (bits == 0) {  // one key: the stable order is the input order
      ITRY(hipMemcpyAsync(w.sv[1], w.sv[0], T * 4, hipMemcpyDeviceToDevice, s));
    } else if (bits <= 32) {
      LAUNCH(k_key_rebase32, T, w.sk[0], klo, T, w.u[0]);
      ITRY(sort32(w, w.u[0], w.u[1], w.sv[0], w.sv[1], T, s, bits));
    } else {
      LAUNCH(k_key_rebase64, T, w.sk[0], klo, T);
      ITRY(sort64(w, w.sk[0], w.sk[1], w.sv[0], w.sv[1], T, s, bits));
    }
    // the traces' new starts, then each trace's span run copied there (k_minmax_final zeroed
    // the long-trace count d[1])
    LAUNCH(k_seg_sizes, T, w.seg, w.sv[1], T, w.u[0]);
    ITRY(sum_scan(w, w.u[0], w.u[1], T, false, s));
    hipLaunchKernelGGL(k_place_seg, dim3((unsigned)((T + PL_WG - 1) / PL_WG)), dim3(PL_WG), 0, s, stored, w.seg, w.sv[1],
                       w.u[1], T, perm, w.u[2], w.d);
    ITRY(step_done(s, __LINE__));
    hipLaunchKernelGGL(k_place_big, dim3(256), dim3(256), 0, s, stored, w.seg, w.sv[1], w.u[1], perm, w.u[2], w.d);
    ITRY(step_done(s, __LINE__));
    LAUNCH(k_new_off, T + 1, w.u[1], T, m, off);
  } else if (mode == SEL_ALL_STRICT) {
    // group by (low id, trace id) - the normalized id string: its high 64 bits and its width,
    // since a 17-31 digit id padded to 32 characters keeps a zero high half - indexes into
    // `stored` ascending inside; a group goes where its first span is (first-seen order inside
    // the low id)
    LAUNCH(k_iota32, m, w.u[1], m);
    LAUNCH(k_wide_key, m, alive, stored, w.u[2], m);
    ITRY(sort32(w, w.u[2], w.u[3], w.u[1], w.u[0], m, s, 1));
    LAUNCH(k_take2, m, hi, stored, w.u[0], w.k[0], m);
    ITRY(sort64(w, w.k[0], w.k[1], w.u[0], w.u[1], m, s));
    LAUNCH(k_take2, m, lo, stored, w.u[1], w.k[0], m);
    ITRY(sort64(w, w.k[0], w.k[1], w.u[1], w.u[0], m, s));
    LAUNCH(k_group_heads, m, lo, hi, alive, stored, w.u[0], m, w.u[2]);
    ITRY(max_scan(w, w.u[2], w.u[1], m, s));
    LAUNCH(k_group_first, m, w.u[0], w.u[1], m, w.u[2]);
    ITRY(sort32(w, w.u[2], w.u[1], stored, perm, m, s));
    LAUNCH(k_trace_heads, m, lo, hi, alive, perm, m, w.flag);
    ITRY(offsets_of(w, w.flag, m, off, &T, s));
  } else {
    return hipErrorInvalidValue;
  }
  ITRY(hipStreamSynchronize(s));
  *n_sel = m;
  *n_traces = T;
  return hipSuccess;
}

hipError_t index_evict(IndexWork& w, const uint64_t* lo, const int64_t* ts, uint8_t* alive, uint64_t n,
                       uint64_t n_alive, uint64_t to_recover, uint64_t* evicted, bool* exhausted, hipStream_t s) {
  uint64_t m = 0;
  *evicted = 0;
  *exhausted = false;
  if (to_recover == 0) return hipSuccess;
  if (n >= (1ull << 31)) return hipErrorInvalidValue;
  ITRY(index_update(w, lo, ts, n, s));
  ITRY(reserve(w, n));  // before any w buffer is named: reserve reallocates them
  if (n_alive) ITRY(alive_of(w, w.bk, alive, n, n_alive, w.v[1], &m, s));  // by (low id, timestamp)
  if (m == 0) {
    *exhausted = true;
    return hipSuccess;
  }
  LAUNCH(k_take, m, lo, w.v[1], 0ull, w.k[1], m);
  LAUNCH(k_runs, m, w.k[1], m, w.flag);
  uint64_t T = 0;
  ITRY(offsets_of(w, w.flag, m, w.seg, &T, s));
  // traces by (smallest timestamp, low id) ascending: the order deleteOldestTrace takes them
  LAUNCH(k_seg_oldest, T, w.seg, T, w.v[1], ts, w.sk[0], w.sv[0]);
  ITRY(sort64(w, w.sk[0], w.sk[1], w.sv[0], w.sv[1], T, s));
  LAUNCH(k_seg_sizes, T, w.seg, w.sv[1], T, w.u[0]);
  ITRY(sum_scan(w, w.u[0], w.u[1], T, true, s));
  hipLaunchKernelGGL(k_evict_init, dim3(1), dim3(64), 0, s, T, m, w.d);
  ITRY(hipGetLastError());
  LAUNCH(k_evict_find, T, w.u[1], T, to_recover, w.d);
  LAUNCH(k_rank_of, T, w.sv[1], T, w.sv[0]);
  LAUNCH(k_widen, m, w.flag, m, w.u[2]);
  ITRY(sum_scan(w, w.u[2], w.u[0], m, true, s));
  LAUNCH(k_evict_mark, m, w.v[1], w.u[0], w.sv[0], w.d, m, alive);
  ITRY(fetch(w, 4, s));
  *evicted = w.h[2];
  *exhausted = w.h[3] != 0;
  return hipSuccess;
}

}  // namespace zdl
