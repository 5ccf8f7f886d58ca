// stream_probe.hip — how fast can k_link's access pattern stream at all? Seven C2-shaped columns
// (two 8-B, five 4-B, 10M spans) read in 58-span windows, one window's loads in flight while the
// previous one is consumed (k_link's pipeline), by 8192 waves (2 x 16-wave workgroups per CU),
// with the windows handed to the waves in different orders:
//   0  chunked      wave w: windows [w N / W, (w + 1) N / W)   (k_link today: concurrent reads
//                   of one column sit ~10 KB apart, one DRAM row per wave)
//   B  blocks of B  wave w: blocks w, w + W, ... of B consecutive windows
//   1  interleaved  wave w: windows w, w + W, w + 2W, ...    (a sweeping front: neighbouring
//                   waves read neighbouring windows at the same time)
// SPIN adds k cycles of dependent VALU per window (k_link's compute between waits).
//   hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o tools/stream_probe && tools/stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

struct Cols {
  const uint64_t *id, *pid;
  const uint32_t *a, *b, *c, *d, *e;
};

struct Win {
  uint64_t id, pid;
  uint32_t a, b, c, d, e;
};

__device__ __forceinline__ void load(Win& w, const Cols& q, uint64_t base, int lane, uint64_t n) {
  const uint64_t g = lane < 58 && base + lane < n ? base + lane : n - 1;
  w.id = q.id[g];
  w.pid = q.pid[g];
  w.a = q.a[g];
  w.b = q.b[g];
  w.c = q.c[g];
  w.d = q.d[g];
  w.e = q.e[g];
}

__global__ void __launch_bounds__(1024, 2) k_probe(Cols q, uint64_t n, int block, int spin, unsigned long long* out) {
  const int lane = threadIdx.x & 63;
  const uint64_t W = (uint64_t)gridDim.x * 16, w = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t NWIN = (n + 57) / 58;
  // the k-th window of this wave, or ~0 past its share
  auto win = [&](uint64_t k) -> uint64_t {
    if (block == 0) {
      const uint64_t b = NWIN * w / W, e = NWIN * (w + 1) / W;
      return b + k < e ? b + k : ~0ull;
    }
    const uint64_t B = (uint64_t)block, blk = k / B, r = k % B;
    const uint64_t x = (blk * W + w) * B + r;
    return x < NWIN ? x : ~0ull;
  };
  unsigned long long acc = 0;
  uint64_t k = 0, cur = win(0);
  Win sp, nsp;
  if (cur != ~0ull) load(sp, q, cur * 58, lane, n);
  while (cur != ~0ull) {
    const uint64_t nx = win(++k);
    if (nx != ~0ull) load(nsp, q, nx * 58, lane, n);
    uint32_t x = (uint32_t)(sp.id ^ sp.pid) + sp.a + sp.b + sp.c + sp.d + sp.e;
    for (int i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;
    acc += x;
    cur = nx;
    if (cur != ~0ull) sp = nsp;
  }
  if (acc == 0x12345678ull) out[w] = acc;
}

int main(int argc, char** argv) {
  const uint64_t n = 10001749;
  std::vector<void*> bufs;
  auto alloc = [&](size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) std::exit(1);
    (void)hipMemset(p, 1, bytes);
    bufs.push_back(p);
    return p;
  };
  Cols q;
  q.id = (const uint64_t*)alloc(n * 8);
  q.pid = (const uint64_t*)alloc(n * 8);
  q.a = (const uint32_t*)alloc(n * 4);
  q.b = (const uint32_t*)alloc(n * 4);
  q.c = (const uint32_t*)alloc(n * 4);
  q.d = (const uint32_t*)alloc(n * 4);
  q.e = (const uint32_t*)alloc(n * 4);
  // a second copy, read alternately, so no launch finds the previous one's bytes in the 256 MiB
  // Infinity Cache
  Cols q2 = q;
  q2.id = (const uint64_t*)alloc(n * 8);
  q2.pid = (const uint64_t*)alloc(n * 8);
  q2.a = (const uint32_t*)alloc(n * 4);
  q2.b = (const uint32_t*)alloc(n * 4);
  q2.c = (const uint32_t*)alloc(n * 4);
  q2.d = (const uint32_t*)alloc(n * 4);
  q2.e = (const uint32_t*)alloc(n * 4);
  unsigned long long* out = (unsigned long long*)alloc(1 << 20);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double bytes = 36.0 * n;
  const int blocks[] = {0, 1, 2, 4, 11, 32};
  const int spins[] = {0, 64, 256};
  for (int spin : spins)
    for (int b : blocks) {
      float best = 1e9f, sum = 0.f;
      const int reps = 10;
      for (int r = 0; r < reps + 2; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_probe, dim3(512), dim3(1024), 0, 0, (r & 1) ? q2 : q, n, b, spin, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r >= 2) {
          best = ms < best ? ms : best;
          sum += ms;
        }
      }
      printf("spin %3d order %-12s%2d  mean %7.1f us  best %7.1f us  %6.2f TB/s (algorithmic 36 B/span)\n", spin,
             b == 0 ? "chunked" : (b == 1 ? "interleaved" : "blocks of"), b, 1e3f * sum / reps, 1e3f * best,
             bytes / (best * 1e-3) / 1e12);
      fflush(stdout);
    }
  for (void* p : bufs) (void)hipFree(p);
  return 0;
}
