// calib_fetch.hip — calibrates rocprofv3's FETCH_SIZE on gfx950 for the load widths k_link
// issues (MI355X_MICROARCH.md §HBM: FETCH_SIZE is calibrated there only for 16 B/lane).
// Each kernel streams a known byte count once (1 GiB, far beyond L2 + Infinity Cache),
// lanes on consecutive elements like k_link's window loads, with the window base shifted
// by an odd element count per wave so loads straddle 128-B lines as k_link's do.
//
//   hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/calib_fetch
//   rocprofv3 --pmc FETCH_SIZE -d OUT -o run --output-format csv -- tools/calib_fetch
// then FETCH_SIZE (KiB) * 1024 / bytes per kernel = the factor to apply.
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ unsigned long long val(uint32_t x) { return x; }
__device__ __forceinline__ unsigned long long val(uint64_t x) { return x; }
__device__ __forceinline__ unsigned long long val(uint4 x) { return (unsigned long long)x.x + x.y + x.z + x.w; }

template <class T>
__global__ void __launch_bounds__(256) k_stream(const T* __restrict__ p, size_t n, unsigned long long* out) {
  // wave w reads windows of 64 elements starting at w * 64 * iters + odd shift, tiled
  const size_t waves = (size_t)gridDim.x * 4, w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const size_t per = n / waves;
  const size_t b = w * per, e = b + per;
  unsigned long long acc = 0;
  for (size_t i = b + 37; i + 64 <= e; i += 57) {  // windows of 57 elements tile the chunk
    if (lane < 57) acc += val(p[i + lane]);
  }
  if (acc == 0x1234567ull) out[w] = acc;
}

int main() {
  const size_t bytes = 1ull << 30;
  void* buf = nullptr;
  unsigned long long* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc((void**)&out, 1 << 20) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, bytes);
  (void)hipDeviceSynchronize();
  const int grid = 256 * 8;
  hipLaunchKernelGGL(k_stream<uint32_t>, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, bytes / 4, out);
  hipLaunchKernelGGL(k_stream<uint64_t>, dim3(grid), dim3(256), 0, 0, (const uint64_t*)buf, bytes / 8, out);
  hipLaunchKernelGGL(k_stream<uint4>, dim3(grid), dim3(256), 0, 0, (const uint4*)buf, bytes / 16, out);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("each kernel reads ~%zu bytes once (57-element windows from an odd base)\n", bytes);
  return 0;
}
