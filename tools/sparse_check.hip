// sparse_check.hip — sparse_accumulate (zdl_sparse.hip) against a CPU reduce on random logs of 12-32
// key bits, and hipcub's radix sort on key bits [b, key_bits) alone: tools/sparse_check [E] (links libzdl.so).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <vector>

#include "../zipkin_amd/csrc/zdl_sparse.h"

static int check(uint64_t E, int key_bits, bool skew) {
  std::mt19937_64 g(key_bits * 1000 + E);
  std::vector<uint32_t> log(E);
  const uint64_t cells = 1ull << (key_bits - 1);
  for (auto& x : log) {
    uint64_t c = skew && (g() & 1) ? g() % std::min<uint64_t>(3000, cells) : g() % cells;
    x = (uint32_t)((c << 1) | (g() & 1));
  }
  std::map<uint32_t, std::pair<uint64_t, uint64_t>> want;
  for (uint32_t x : log) {
    auto& w = want[x >> 1];
    ++w.first;
    w.second += x & 1;
  }
  uint32_t* d;
  hipMalloc(&d, E * 4);
  hipMemcpy(d, log.data(), E * 4, hipMemcpyHostToDevice);
  // the sort alone: sorted by key >> 14?
  uint32_t* o;
  hipMalloc(&o, E * 4);
  size_t tb = 0;
  const int b0 = key_bits >= 32 ? 0 : 14;
  hipcub::DeviceRadixSort::SortKeys(nullptr, tb, d, o, (int)E, b0, key_bits);
  void* tmp;
  hipMalloc(&tmp, tb);
  hipcub::DeviceRadixSort::SortKeys(tmp, tb, d, o, (int)E, b0, key_bits);
  std::vector<uint32_t> so(E);
  hipMemcpy(so.data(), o, E * 4, hipMemcpyDeviceToHost);
  uint64_t bad = 0;
  for (uint64_t i = 1; i < E; ++i) bad += (so[i] >> 14) < (so[i - 1] >> 14);
  zdl::SparseWork w;
  zdl::SparseTable t;
  hipError_t e = zdl::sparse_accumulate(w, t, d, E, key_bits, 0);
  hipDeviceSynchronize();
  std::vector<uint32_t> c(t.n);
  std::vector<unsigned long long> call(t.n), err(t.n);
  hipMemcpy(c.data(), t.cell, t.n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(call.data(), t.call, t.n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(err.data(), t.err, t.n * 8, hipMemcpyDeviceToHost);
  uint64_t miss = t.n != want.size();
  size_t i = 0;
  for (auto& kv : want) {
    if (i >= t.n) break;
    miss += c[i] != kv.first || call[i] != kv.second.first || err[i] != kv.second.second;
    ++i;
  }
  printf("E %llu key_bits %d skew %d: hip %d, sort inversions %llu, list %zu / %zu, mismatches %llu\n",
         (unsigned long long)E, key_bits, (int)skew, (int)e, (unsigned long long)bad, t.n, want.size(),
         (unsigned long long)miss);
  hipFree(d);
  hipFree(o);
  hipFree(tmp);
  return bad || miss || e != hipSuccess;
}

int main(int argc, char** argv) {
  const uint64_t E = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000;
  int fails = 0;
  for (int kb : {12, 20, 28, 31, 32})
    for (bool sk : {false, true}) fails += check(E, kb, sk);
  printf("%s\n", fails ? "FAIL" : "ok");
  return fails != 0;
}
