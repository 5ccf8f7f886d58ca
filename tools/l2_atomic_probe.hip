// l2_atomic_probe.hip — does a workgroup-scope global atomic add execute in the XCD's L2, and is
// a per-XCD table counted exactly when every workgroup adds into the copy of its own XCD
// (s_getreg HW_REG_XCC_ID)? Compared with agent-scope atomics into one table and with the
// LOG mode's coalesced 4-B log stores. Cells are drawn like C3's links (Zipf-ish over S x S
// with S = 500). Prints the times and whether the summed copies equal the agent-scope table.
//   hipcc --offload-arch=gfx950 -O3 tools/l2_atomic_probe.hip -o tools/l2_atomic_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

constexpr int S = 500;
constexpr uint32_t CELLS = S * S;

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xFu;
}

__device__ __forceinline__ uint32_t cell_of(uint64_t i) {
  uint64_t z = i * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  // a skewed service: floor(S^u) - 1 for u uniform (Zipf-like head)
  const float u1 = (float)(z & 0xFFFFFF) / 16777216.0f, u2 = (float)((z >> 24) & 0xFFFFFF) / 16777216.0f;
  const uint32_t p = (uint32_t)(__powf((float)S, u1)) - 1u, c = (uint32_t)(__powf((float)S, u2)) - 1u;
  return (p < S ? p : S - 1) * S + (c < S ? c : S - 1);
}

// mode 0: per-XCD copy, workgroup-scope atomics; 1: one table, agent-scope atomics; 2: log store
template <int MODE>
__global__ void __launch_bounds__(1024) k_add(unsigned long long* tab, uint32_t* log, uint64_t n, uint32_t* xccs) {
  const uint32_t x = xcc_id();
  if (MODE == 0 && threadIdx.x == 0) atomicOr(&xccs[blockIdx.x & 1023], 1u << x);
  unsigned long long* t = MODE == 0 ? tab + (size_t)x * CELLS : tab;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = cell_of(i);
    const unsigned long long v = 1ull | ((unsigned long long)(i % 17 == 0) << 32);
    if (MODE == 0) __hip_atomic_fetch_add(&t[c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if (MODE == 1) __hip_atomic_fetch_add(&t[c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else log[i] = c << 1 | (uint32_t)(i % 17 == 0);
  }
}

__global__ void k_sum8(const unsigned long long* copies, unsigned long long* out) {
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < CELLS; c += gridDim.x * blockDim.x) {
    unsigned long long s = 0;
    for (int x = 0; x < 8; ++x) s += copies[(size_t)x * CELLS + c];
    out[c] = s;
  }
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 30000000ull;
  unsigned long long *copies, *one, *sum;
  uint32_t *log, *xccs;
  CK(hipMalloc(&copies, 8ull * CELLS * 8));
  CK(hipMalloc(&one, CELLS * 8ull));
  CK(hipMalloc(&sum, CELLS * 8ull));
  CK(hipMalloc(&log, n * 4));
  CK(hipMalloc(&xccs, 1024 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = 512;
  float ms[3] = {0, 0, 0};
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipMemset(copies, 0, 8ull * CELLS * 8));
    CK(hipMemset(one, 0, CELLS * 8ull));
    CK(hipMemset(xccs, 0, 1024 * 4));
    CK(hipDeviceSynchronize());
    float t;
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_add<0>, dim3(grid), dim3(1024), 0, 0, copies, log, n, xccs);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&t, a, b));
    if (rep) ms[0] += t / 3;
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_add<1>, dim3(grid), dim3(1024), 0, 0, one, log, n, xccs);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&t, a, b));
    if (rep) ms[1] += t / 3;
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_add<2>, dim3(grid), dim3(1024), 0, 0, one + 0, log, n, xccs);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&t, a, b));
    if (rep) ms[2] += t / 3;
  }
  // last rep: copies and `one` hold one pass each
  CK(hipMemset(copies, 0, 8ull * CELLS * 8));
  CK(hipMemset(one, 0, CELLS * 8ull));
  hipLaunchKernelGGL(k_add<0>, dim3(grid), dim3(1024), 0, 0, copies, log, n, xccs);
  hipLaunchKernelGGL(k_add<1>, dim3(grid), dim3(1024), 0, 0, one, log, n, xccs);
  hipLaunchKernelGGL(k_sum8, dim3(256), dim3(256), 0, 0, copies, sum);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> hs(CELLS), ho(CELLS), hc(8ull * CELLS);
  std::vector<uint32_t> hx(1024);
  CK(hipMemcpy(hs.data(), sum, CELLS * 8ull, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ho.data(), one, CELLS * 8ull, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hc.data(), copies, 8ull * CELLS * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hx.data(), xccs, 1024 * 4, hipMemcpyDeviceToHost));
  uint64_t bad = 0, tot = 0, used = 0;
  for (uint32_t c = 0; c < CELLS; ++c) {
    bad += hs[c] != ho[c];
    tot += ho[c] & 0xFFFFFFFFull;
  }
  for (int x = 0; x < 8; ++x) {
    uint64_t s = 0;
    for (uint32_t c = 0; c < CELLS; ++c) s += hc[(size_t)x * CELLS + c] & 0xFFFFFFFFull;
    used += s ? 1 : 0;
    std::printf("xcc %d copy: %llu adds\n", x, (unsigned long long)s);
  }
  int multi = 0;
  for (int g = 0; g < grid; ++g) multi += __builtin_popcount(hx[g]) != 1;
  std::printf("n %llu: per-XCD wg-scope %.3f ms, agent-scope one table %.3f ms, log stores %.3f ms\n",
              (unsigned long long)n, ms[0], ms[1], ms[2]);
  std::printf("total adds %llu (want %llu), cells differing %llu, copies used %llu, blocks seen on >1 XCD %d\n",
              (unsigned long long)tot, (unsigned long long)n, (unsigned long long)bad, (unsigned long long)used, multi);
  std::printf(bad == 0 && tot == n ? "EXACT\n" : "MISMATCH\n");
  return 0;
}
