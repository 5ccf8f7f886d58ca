// zdl_shard.h — the host side of a device group's put: a batch of
// span columns split into N shards by splitmix64(trace_lo) % N, whole traces, storage order
// kept inside every shard. Host-only C++ (no HIP), shared by libzdl's group_put and by
// libzdl_synth (the CPU tests check it against zipkin_amd/shard.py's partition_columns, and
// bench.py times it over the 1B-span C3 batch).
//
// Two parallel passes over contiguous chunks of traces (or spans, for ungrouped input):
//   count    per (chunk, shard): spans and traces; then an exclusive scan over the chunks
//            gives every chunk its base in every shard, and the shards' sizes;
//   scatter  every chunk copies its traces' column slices to their shard at its bases, and
//            writes the shard's CSR offsets.
// The shard of a trace is that of its first span's trace_lo (the low 64 bits, as
// InMemoryStorage groups them, InMemoryStorage.java:163, 330, 465-467). Algorithmic bytes: every
// column read once and written once (44 B a span each way without timestamps), offsets likewise.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace zdl_shard {

inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct In {  // any of ts / ord may be null
  const uint64_t *lo, *id, *pid;
  const int32_t *ls, *rs, *i4, *i6;
  const uint32_t* pf;
  const int64_t* ts;
  const uint32_t* ord;
};
struct Out {  // one shard's columns (sized by the plan); off: its CSR offsets (grouped input)
  uint64_t *lo, *id, *pid;
  int32_t *ls, *rs, *i4, *i6;
  uint32_t* pf;
  int64_t* ts;
  uint32_t* ord;
  uint64_t* off;
};

struct Plan {
  uint32_t N = 0, chunks = 0;
  uint64_t units = 0;                 // traces (grouped) or spans (ungrouped)
  std::vector<uint64_t> spans, traces;  // per shard
  std::vector<uint64_t> sbase, tbase;   // per (chunk, shard): the chunk's first span / trace there
};

template <class F>
inline void parallel_chunks(uint32_t chunks, int threads, F f) {
  if (threads <= 1 || chunks <= 1) {
    for (uint32_t c = 0; c < chunks; ++c) f(c);
    return;
  }
  std::vector<std::thread> th;
  const uint32_t nt = std::min<uint32_t>((uint32_t)threads, chunks);
  for (uint32_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (uint32_t c = t; c < chunks; c += nt) f(c);
    });
  for (auto& x : th) x.join();
}

// units [b, e) of chunk c (chunks of about equal units)
inline void chunk_range(const Plan& p, uint32_t c, uint64_t& b, uint64_t& e) {
  b = p.units * c / p.chunks;
  e = p.units * (c + 1) / p.chunks;
}

// off == nullptr: ungrouped input, every span by its own trace_lo (input order kept)
inline Plan plan(const In& in, uint64_t n_spans, const uint64_t* off, uint64_t n_traces, uint32_t N, int threads) {
  Plan p;
  p.N = N;
  p.units = off ? n_traces : n_spans;
  p.chunks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(p.units / 4096 + 1, (uint64_t)std::max(threads, 1) * 8));
  std::vector<uint64_t> cs((size_t)p.chunks * N, 0), ct((size_t)p.chunks * N, 0);
  parallel_chunks(p.chunks, threads, [&](uint32_t c) {
    uint64_t b, e;
    chunk_range(p, c, b, e);
    uint64_t* s = &cs[(size_t)c * N];
    uint64_t* t = &ct[(size_t)c * N];
    if (off) {
      for (uint64_t x = b; x < e; ++x) {
        const uint64_t sb = off[x], se = off[x + 1];
        if (se == sb) continue;  // an empty trace goes nowhere
        const uint32_t d = (uint32_t)(splitmix64(in.lo[sb]) % N);
        s[d] += se - sb;
        t[d] += 1;
      }
    } else {
      for (uint64_t x = b; x < e; ++x) s[(uint32_t)(splitmix64(in.lo[x]) % N)] += 1;
    }
  });
  p.spans.assign(N, 0);
  p.traces.assign(N, 0);
  p.sbase.resize((size_t)p.chunks * N);
  p.tbase.resize((size_t)p.chunks * N);
  for (uint32_t c = 0; c < p.chunks; ++c)
    for (uint32_t d = 0; d < N; ++d) {
      const size_t k = (size_t)c * N + d;
      p.sbase[k] = p.spans[d];
      p.tbase[k] = p.traces[d];
      p.spans[d] += cs[k];
      p.traces[d] += ct[k];
    }
  return p;
}

// Every shard's columns (and, grouped, offsets: traces[d] + 1 entries, off[0] = 0) written.
inline void scatter(const In& in, const uint64_t* off, const Plan& p, const Out* out, int threads) {
  const uint32_t N = p.N;
  if (off)
    for (uint32_t d = 0; d < N; ++d)
      if (out[d].off) out[d].off[0] = 0;
  parallel_chunks(p.chunks, threads, [&](uint32_t c) {
    uint64_t b, e;
    chunk_range(p, c, b, e);
    std::vector<uint64_t> sp(p.sbase.begin() + (size_t)c * N, p.sbase.begin() + (size_t)(c + 1) * N);
    std::vector<uint64_t> tr(p.tbase.begin() + (size_t)c * N, p.tbase.begin() + (size_t)(c + 1) * N);
    auto copy = [&](const Out& o, uint64_t at, uint64_t sb, uint64_t n) {
      std::memcpy(o.lo + at, in.lo + sb, n * 8);
      std::memcpy(o.id + at, in.id + sb, n * 8);
      std::memcpy(o.pid + at, in.pid + sb, n * 8);
      std::memcpy(o.ls + at, in.ls + sb, n * 4);
      std::memcpy(o.rs + at, in.rs + sb, n * 4);
      std::memcpy(o.i4 + at, in.i4 + sb, n * 4);
      std::memcpy(o.i6 + at, in.i6 + sb, n * 4);
      std::memcpy(o.pf + at, in.pf + sb, n * 4);
      if (in.ts && o.ts) std::memcpy(o.ts + at, in.ts + sb, n * 8);
      if (in.ord && o.ord) std::memcpy(o.ord + at, in.ord + sb, n * 4);
    };
    if (off) {
      for (uint64_t x = b; x < e; ++x) {
        const uint64_t sb = off[x], se = off[x + 1];
        if (se == sb) continue;
        const uint32_t d = (uint32_t)(splitmix64(in.lo[sb]) % N);
        copy(out[d], sp[d], sb, se - sb);
        sp[d] += se - sb;
        if (out[d].off) out[d].off[++tr[d]] = sp[d];
      }
    } else {
      for (uint64_t x = b; x < e; ++x) {
        const uint32_t d = (uint32_t)(splitmix64(in.lo[x]) % N);
        copy(out[d], sp[d], x, 1);
        ++sp[d];
      }
    }
  });
}

// The host threads a split uses: ZDL_HOST_THREADS, else the hardware's, at most 16 (a box's
// CPU share; nproc there counts the whole machine)
inline int host_threads(const char* env) {
  if (env && *env) return std::max(1, atoi(env));
  const unsigned h = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(h ? h : 1u, 16u));
}

}  // namespace zdl_shard
