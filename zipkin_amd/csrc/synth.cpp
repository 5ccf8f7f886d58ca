// synth.cpp — deterministic synthetic Zipkin traces written straight to columns
// (libzdl_synth.so). Generates the BASELINE.json workloads:
//   C2  10M spans / 1M traces / 50 services, depth <= 8, 1+Poisson(9) spans per trace
//   C3  the same shape sharded by splitmix64(trace_lo) % n_shards
//   C4  messaging stress: PRODUCER/CONSUMER hops, missing brokers, deleted spans,
//       extra roots, uninstrumented clients, dropped shared parent ids, fragments
//   C5  10k services, depth 64, Pareto(1.2) trace sizes, fan-out up to 1000
// Every trace t is generated from its own splitmix64 stream, so sizes (pass 1) and
// contents (pass 2) agree and any thread count gives identical output.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

extern "C" {

typedef struct zdl_synth_params {
  uint64_t seed;
  uint64_t n_traces;
  uint32_t n_services;     // regular services: ids [0, n_services)
  uint32_t n_brokers;      // broker services: ids [n_services, n_services + n_brokers)
  uint32_t max_depth;
  uint32_t size_dist;      // 0: 1 + Poisson(lambda); 1: Pareto(alpha) clipped to [1, max_size]
  double lambda;
  double pareto_alpha;
  uint32_t max_size;
  uint32_t max_fanout;     // 0 = unlimited
  double zipf_s;
  double p_shared;
  double p_local;
  double p_error;
  double p_messaging;
  double p_missing_broker;
  double p_delete;
  double p_extra_root;
  double p_uninstrumented;
  double p_drop_shared_parent;
  double p_split;
  double p_root_remote;    // root SERVER span names its (uninstrumented) caller
  uint32_t shard, n_shards;
  uint32_t instances;      // ip4 instances per service
  uint32_t reserved;
  int64_t base_ts_us;
} zdl_synth_params;

}  // extern "C"

namespace {

constexpr uint32_t KIND_CLIENT = 0, KIND_SERVER = 1, KIND_PRODUCER = 2, KIND_CONSUMER = 3, KIND_NULL = 7;

inline uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

inline uint64_t mix(uint64_t x) { return splitmix64(x); }

struct Rng {
  uint64_t s;
  uint64_t next() { return splitmix64(s); }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint64_t nonzero() {
    uint64_t v;
    do v = next(); while (v == 0);
    return v;
  }
  uint32_t below(uint32_t n) { return (uint32_t)(uni() * n) % n; }
  bool coin(double p) { return p > 0 && uni() < p; }
  uint32_t poisson(double lam) {  // Knuth; lam is small
    const double L = std::exp(-lam);
    uint32_t k = 0;
    double p = 1.0;
    do {
      ++k;
      p *= uni();
    } while (p > L);
    return k - 1;
  }
};

struct Rec {
  uint64_t id, pid;
  int32_t lsvc, rsvc, ip4, ip6;
  uint32_t pf;
  int64_t ts;
};

struct Zipf {
  std::vector<double> cdf;
  void init(uint32_t n, double s) {
    cdf.resize(n);
    double acc = 0;
    for (uint32_t i = 0; i < n; ++i) {
      acc += 1.0 / std::pow((double)(i + 1), s);
      cdf[i] = acc;
    }
    for (auto& c : cdf) c /= acc;
  }
  uint32_t draw(Rng& r) const {
    const double u = r.uni();
    return (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin()) % cdf.size();
  }
};

struct Node {
  uint64_t id;
  uint32_t svc, depth, fanout;
};

inline uint32_t pf_of(uint32_t port, uint32_t kind, uint32_t shared, bool err, bool rip4) {
  return (port & 0xFFFFu) | (kind << 16) | (shared << 19) | (err ? (1u << 21) : 0u) | (rip4 ? (1u << 22) : 0u);
}

struct Gen {
  const zdl_synth_params& P;
  Zipf zipf;
  explicit Gen(const zdl_synth_params& p) : P(p) { zipf.init(std::max<uint32_t>(p.n_services, 1), p.zipf_s); }

  uint32_t trace_size(Rng& r) const {
    if (P.size_dist == 2) return std::max<uint32_t>(1, P.max_size);  // every trace exactly max_size spans
    if (P.size_dist == 1) {
      const double u = 1.0 - r.uni();
      double x = std::pow(u, -1.0 / P.pareto_alpha);
      if (x > P.max_size) x = P.max_size;
      return std::max<uint32_t>(1, (uint32_t)x);
    }
    uint32_t n = 1 + r.poisson(P.lambda);
    if (P.max_size && n > P.max_size) n = P.max_size;
    return n;
  }

  int32_t ip_of(uint32_t svc, Rng& r) const {
    const uint32_t inst = std::max<uint32_t>(P.instances, 1);
    return (int32_t)(svc * inst + r.below(inst));
  }
  static uint32_t port_of(uint32_t svc) { return 8000 + (svc % 1000); }

  // Generates trace t into out; returns its trace_lo.
  uint64_t trace(uint64_t t, std::vector<Rec>& out) const {
    out.clear();
    uint64_t st = P.seed ^ mix(t * 0xD1B54A32D192ED03ull + 0x5EED);
    Rng r{st};
    uint64_t lo = r.nonzero();
    if (P.n_shards > 1)
      while (mix(lo) % P.n_shards != P.shard) lo = r.nonzero();
    const uint32_t size = trace_size(r);
    const int64_t t0 = P.base_ts_us + (int64_t)(t % 86400000ull) * 1000;
    std::vector<Node> open;
    open.reserve(size);
    const uint32_t root_svc = zipf.draw(r);
    const uint64_t root_id = r.nonzero();
    {
      Rec s{};
      s.id = root_id;
      s.pid = 0;
      s.lsvc = (int32_t)root_svc;
      s.rsvc = r.coin(P.p_root_remote) ? (int32_t)zipf.draw(r) : -1;
      s.ip4 = ip_of(root_svc, r);
      s.ip6 = -1;
      s.pf = pf_of(port_of(root_svc), KIND_SERVER, 0, r.coin(P.p_error), false);
      s.ts = t0;
      out.push_back(s);
      open.push_back(Node{root_id, root_svc, 0, 0});
    }
    while (out.size() < size) {
      // prefer the newest node half of the time: deeper, chain-like traces
      size_t oi = r.coin(0.5) ? open.size() - 1 : r.below((uint32_t)open.size());
      for (int tries = 0; tries < 8; ++tries) {
        const Node& o = open[oi];
        if (o.depth + 1 < P.max_depth && (P.max_fanout == 0 || o.fanout < P.max_fanout)) break;
        oi = r.below((uint32_t)open.size());
      }
      Node& o = open[oi];
      o.fanout++;
      const uint32_t depth = std::min(o.depth + 1, P.max_depth ? P.max_depth - 1 : o.depth + 1);
      const uint64_t parent_id = o.id;
      const uint32_t caller = o.svc;
      const int64_t ts = t0 + (int64_t)out.size() * 10;
      const double u = r.uni();
      const uint32_t budget = size - (uint32_t)out.size();
      if (u < P.p_local) {
        Rec s{};
        s.id = r.nonzero();
        s.pid = parent_id;
        s.lsvc = (int32_t)caller;
        s.rsvc = -1;
        s.ip4 = ip_of(caller, r);
        s.ip6 = -1;
        s.pf = pf_of(0, KIND_NULL, 0, false, false);
        s.ts = ts;
        out.push_back(s);
        open.push_back(Node{s.id, caller, depth, 0});
      } else if (u < P.p_local + P.p_messaging && P.n_brokers > 0) {
        const int32_t broker = (int32_t)(P.n_services + r.below(P.n_brokers));
        Rec pr{};
        pr.id = r.nonzero();
        pr.pid = parent_id;
        pr.lsvc = (int32_t)caller;
        pr.rsvc = r.coin(P.p_missing_broker) ? -1 : broker;
        pr.ip4 = ip_of(caller, r);
        pr.ip6 = -1;
        pr.pf = pf_of(0, KIND_PRODUCER, 0, r.coin(P.p_error), false);
        pr.ts = ts;
        out.push_back(pr);
        if (budget >= 2) {
          const uint32_t callee = zipf.draw(r);
          Rec co{};
          co.id = r.nonzero();
          co.pid = pr.id;
          co.lsvc = (int32_t)callee;
          co.rsvc = r.coin(P.p_missing_broker) ? -1 : broker;
          co.ip4 = ip_of(callee, r);
          co.ip6 = -1;
          co.pf = pf_of(port_of(callee), KIND_CONSUMER, 0, r.coin(P.p_error), false);
          co.ts = ts + 5;
          out.push_back(co);
          open.push_back(Node{co.id, callee, depth, 0});
        }
      } else {
        uint32_t callee = zipf.draw(r);
        if (callee == caller) callee = zipf.draw(r);
        Rec cl{};
        cl.id = r.nonzero();
        cl.pid = parent_id;
        cl.lsvc = (int32_t)caller;
        cl.rsvc = (int32_t)callee;
        cl.ip4 = ip_of(caller, r);
        cl.ip6 = -1;
        cl.pf = pf_of(0, KIND_CLIENT, 0, r.coin(P.p_error), true);
        cl.ts = ts;
        out.push_back(cl);
        if (budget >= 2 && !r.coin(P.p_uninstrumented)) {
          Rec sv{};
          sv.lsvc = (int32_t)callee;
          sv.rsvc = (int32_t)caller;
          sv.ip4 = ip_of(callee, r);
          sv.ip6 = -1;
          sv.ts = ts + 2;
          if (r.coin(P.p_shared)) {
            sv.id = cl.id;
            sv.pid = r.coin(P.p_drop_shared_parent) ? 0 : parent_id;
            sv.pf = pf_of(port_of(callee), KIND_SERVER, 2, r.coin(P.p_error), false);
          } else {
            sv.id = r.nonzero();
            sv.pid = cl.id;
            sv.pf = pf_of(port_of(callee), KIND_SERVER, 0, r.coin(P.p_error), false);
          }
          out.push_back(sv);
          open.push_back(Node{sv.id, callee, depth, 0});
        }
      }
    }
    if (r.coin(P.p_extra_root)) {
      const uint32_t svc = zipf.draw(r);
      Rec s{};
      s.id = r.nonzero();
      s.pid = 0;
      s.lsvc = (int32_t)svc;
      s.rsvc = -1;
      s.ip4 = ip_of(svc, r);
      s.ip6 = -1;
      s.pf = pf_of(port_of(svc), KIND_SERVER, 0, false, false);
      s.ts = t0 + 1;
      out.push_back(s);
    }
    if (P.p_delete > 0) {
      size_t w = 0;
      for (size_t i = 0; i < out.size(); ++i)
        if (!r.coin(P.p_delete)) out[w++] = out[i];
      out.resize(w);
    }
    if (P.p_split > 0) {
      // a second fragment with the same id/shared/local endpoint and the same remote
      // endpoint (so Span.Builder.merge cannot NPE), kind unset, no error tag
      const size_t n = out.size();
      for (size_t i = 0; i < n; ++i) {
        if (!r.coin(P.p_split)) continue;
        Rec f = out[i];
        f.pf = (f.pf & ~((7u << 16) | (1u << 21))) | (KIND_NULL << 16);
        if (r.coin(0.5)) f.pid = 0;
        f.ts = 0;
        out.push_back(f);
      }
    }
    for (size_t i = out.size(); i > 1; --i) std::swap(out[i - 1], out[r.below((uint32_t)i)]);
    return lo;
  }
};

template <class F>
void parallel_for(uint64_t n, int threads, F&& f) {
  threads = std::max(1, threads);
  if (threads == 1 || n < 1024) {
    f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  const uint64_t chunk = (n + threads - 1) / threads;
  for (int i = 0; i < threads; ++i) {
    const uint64_t b = i * chunk, e = std::min(n, b + chunk);
    if (b >= e) break;
    ts.emplace_back([&, b, e] { f(b, e); });
  }
  for (auto& t : ts) t.join();
}

}  // namespace

extern "C" {

// Pass 1: offsets[t+1] - offsets[t] = size of trace t; returns the span count.
uint64_t zdl_synth_sizes(const zdl_synth_params* p, uint64_t* offsets, int threads) {
  Gen g(*p);
  offsets[0] = 0;
  parallel_for(p->n_traces, threads, [&](uint64_t b, uint64_t e) {
    std::vector<Rec> buf;
    for (uint64_t t = b; t < e; ++t) {
      g.trace(t, buf);
      offsets[t + 1] = buf.size();
    }
  });
  for (uint64_t t = 0; t < p->n_traces; ++t) offsets[t + 1] += offsets[t];
  return offsets[p->n_traces];
}

// Pass 2: fills the columns (each n_spans long). Any pointer may be NULL.
void zdl_synth_fill(const zdl_synth_params* p, const uint64_t* offsets, uint64_t* trace_lo, uint64_t* id,
                    uint64_t* parent_id, int32_t* local_svc, int32_t* remote_svc, int32_t* local_ip4,
                    int32_t* local_ip6, uint32_t* port_flags, int64_t* timestamp, int threads) {
  Gen g(*p);
  parallel_for(p->n_traces, threads, [&](uint64_t b, uint64_t e) {
    std::vector<Rec> buf;
    for (uint64_t t = b; t < e; ++t) {
      const uint64_t lo = g.trace(t, buf);
      uint64_t o = offsets[t];
      for (const Rec& s : buf) {
        if (trace_lo) trace_lo[o] = lo;
        if (id) id[o] = s.id;
        if (parent_id) parent_id[o] = s.pid;
        if (local_svc) local_svc[o] = s.lsvc;
        if (remote_svc) remote_svc[o] = s.rsvc;
        if (local_ip4) local_ip4[o] = s.ip4;
        if (local_ip6) local_ip6[o] = s.ip6;
        if (port_flags) port_flags[o] = s.pf;
        if (timestamp) timestamp[o] = s.ts;
        ++o;
      }
    }
  });
}

}  // extern "C"

// ---- proto3 encoding of synthetic columns (bench / test input for zdl_decode_proto3) ----
// Writes a ListOfSpans (Proto3ZipkinFields.java:246-302 field order) for spans [0, n) of the
// columns: trace_id (8 bytes), parent_id, id, kind, timestamp, local endpoint {service name,
// ipv4 10.a.b.c from the ipv4 id, port}, remote endpoint {service name, port 80 when RPORT},
// tag error="" when the error flag is set, shared when shared == true. Service id i is
// names[name_off[i], name_off[i+1]). Returns the byte count; out == NULL only measures.
namespace {
inline size_t put_varint(uint8_t* o, uint64_t v) {
  size_t k = 0;
  while (v >= 0x80) {
    if (o) o[k] = (uint8_t)(v | 0x80);
    v >>= 7;
    ++k;
  }
  if (o) o[k] = (uint8_t)v;
  return k + 1;
}
inline size_t varint_len(uint64_t v) { return put_varint(nullptr, v); }
inline void put_be64(uint8_t* o, uint64_t v) {
  for (int i = 7; i >= 0; --i) o[7 - i] = (uint8_t)(v >> (8 * i));
}
}  // namespace

extern "C" uint64_t zdl_synth_proto3(uint64_t n, const uint64_t* trace_lo, const uint64_t* id,
                                     const uint64_t* parent_id, const int32_t* local_svc,
                                     const int32_t* remote_svc, const int32_t* local_ip4,
                                     const uint32_t* port_flags, const int64_t* timestamp,
                                     const char* names, const uint32_t* name_off, uint8_t* out) {
  uint64_t pos = 0;
  uint8_t span[512];
  for (uint64_t i = 0; i < n; ++i) {
    size_t k = 0;
    span[k++] = 1 << 3 | 2, span[k++] = 8, put_be64(span + k, trace_lo[i]), k += 8;
    if (parent_id[i]) span[k++] = 2 << 3 | 2, span[k++] = 8, put_be64(span + k, parent_id[i]), k += 8;
    span[k++] = 3 << 3 | 2, span[k++] = 8, put_be64(span + k, id[i]), k += 8;
    const uint32_t pf = port_flags[i];
    const uint32_t kind = (pf >> 16) & 7;
    if (kind != 7) span[k++] = 4 << 3, span[k++] = (uint8_t)(kind + 1);
    if (timestamp[i] > 0) {
      span[k++] = 6 << 3 | 1;
      for (int b = 0; b < 8; ++b) span[k++] = (uint8_t)((uint64_t)timestamp[i] >> (8 * b));
    }
    for (int side = 0; side < 2; ++side) {
      const int32_t svc = side ? remote_svc[i] : local_svc[i];
      const int32_t ip = side ? -1 : local_ip4[i];
      const uint32_t port = side ? ((pf >> 24 & 1) ? 80u : 0u) : (pf & 0xFFFF);
      uint8_t ep[256];
      size_t e = 0;
      if (svc >= 0) {
        const uint32_t l = name_off[svc + 1] - name_off[svc];
        ep[e++] = 1 << 3 | 2;
        e += put_varint(ep + e, l);
        memcpy(ep + e, names + name_off[svc], l);
        e += l;
      }
      if (ip >= 0) {
        ep[e++] = 2 << 3 | 2, ep[e++] = 4, ep[e++] = 10;
        ep[e++] = (uint8_t)(ip >> 16), ep[e++] = (uint8_t)(ip >> 8), ep[e++] = (uint8_t)ip;
      }
      if (port) ep[e++] = 4 << 3, e += put_varint(ep + e, port);
      if (!e) continue;
      span[k++] = (uint8_t)((8 + side) << 3 | 2);
      k += put_varint(span + k, e);
      memcpy(span + k, ep, e);
      k += e;
    }
    if (pf & (1u << 21)) {  // tags {"error": ""}: the map entry carries only its key
      const uint8_t tag[] = {11 << 3 | 2, 7, 1 << 3 | 2, 5, 'e', 'r', 'r', 'o', 'r'};
      memcpy(span + k, tag, sizeof(tag));
      k += sizeof(tag);
    }
    if (((pf >> 19) & 3) == 2) span[k++] = 13 << 3, span[k++] = 1;
    const size_t hdr = 1 + varint_len(k);
    if (out) {
      out[pos] = 1 << 3 | 2;
      put_varint(out + pos + 1, k);
      memcpy(out + pos + hdr, span, k);
    }
    pos += hdr + k;
  }
  return pos;
}

// ---- JSON v2 encoding of synthetic columns (bench / test input for zdl_decode_json_v2) ----
// V2SpanWriter's member order (internal/V2SpanWriter.java:88-160) for spans [0, n): traceId,
// parentId, id, kind, name "get", timestamp, duration, localEndpoint {serviceName, ipv4 10.a.b.c
// from the ipv4 id, port}, remoteEndpoint {serviceName, port 80 when RPORT}, tags {"error":""}
// when the error flag is set, shared. Returns the byte count; out == NULL only measures.
namespace {
struct JW {
  uint8_t* o;
  uint64_t pos;
  void raw(const char* s, size_t n) {
    if (o) memcpy(o + pos, s, n);
    pos += n;
  }
  void str(const char* s) { raw(s, strlen(s)); }
  void hex16(uint64_t v) {
    char b[16];
    for (int i = 15; i >= 0; --i, v >>= 4) b[i] = "0123456789abcdef"[v & 15];
    raw(b, 16);
  }
  void dec(uint64_t v) {
    char b[24];
    int k = 24;
    do b[--k] = (char)('0' + v % 10), v /= 10;
    while (v);
    raw(b + k, 24 - k);
  }
};
}  // namespace

extern "C" uint64_t zdl_synth_json_v2(uint64_t n, const uint64_t* trace_lo, const uint64_t* id,
                                      const uint64_t* parent_id, const int32_t* local_svc,
                                      const int32_t* remote_svc, const int32_t* local_ip4,
                                      const uint32_t* port_flags, const int64_t* timestamp,
                                      const char* names, const uint32_t* name_off, uint8_t* out) {
  static const char* kinds[4] = {"CLIENT", "SERVER", "PRODUCER", "CONSUMER"};
  JW w{out, 0};
  w.str("[");
  for (uint64_t i = 0; i < n; ++i) {
    if (i) w.str(",");
    w.str("{\"traceId\":\"");
    w.hex16(trace_lo[i]);
    w.str("\"");
    if (parent_id[i] && parent_id[i] != id[i]) {
      w.str(",\"parentId\":\"");
      w.hex16(parent_id[i]);
      w.str("\"");
    }
    w.str(",\"id\":\"");
    w.hex16(id[i]);
    w.str("\"");
    const uint32_t pf = port_flags[i];
    const uint32_t kind = (pf >> 16) & 7;
    if (kind < 4) {
      w.str(",\"kind\":\"");
      w.str(kinds[kind]);
      w.str("\"");
    }
    w.str(",\"name\":\"get\"");
    if (timestamp[i] > 0) {
      w.str(",\"timestamp\":");
      w.dec((uint64_t)timestamp[i]);
      w.str(",\"duration\":");
      w.dec(100 + (id[i] % 100000));
    }
    for (int side = 0; side < 2; ++side) {
      const int32_t svc = side ? remote_svc[i] : local_svc[i];
      const int32_t ip = side ? -1 : local_ip4[i];
      const uint32_t port = side ? ((pf >> 24 & 1) ? 80u : 0u) : (pf & 0xFFFF);
      if (svc < 0 && ip < 0 && !port) continue;
      w.str(side ? ",\"remoteEndpoint\":{" : ",\"localEndpoint\":{");
      bool any = false;
      if (svc >= 0) {
        w.str("\"serviceName\":\"");
        w.raw(names + name_off[svc], name_off[svc + 1] - name_off[svc]);
        w.str("\"");
        any = true;
      }
      if (ip >= 0) {
        w.str(any ? ",\"ipv4\":\"10." : "\"ipv4\":\"10.");
        w.dec((uint32_t)(ip >> 16) & 255);
        w.str(".");
        w.dec((uint32_t)(ip >> 8) & 255);
        w.str(".");
        w.dec((uint32_t)ip & 255);
        w.str("\"");
        any = true;
      }
      if (port) {
        w.str(any ? ",\"port\":" : "\"port\":");
        w.dec(port);
      }
      w.str("}");
    }
    if (pf & (1u << 21)) w.str(",\"tags\":{\"error\":\"\"}");
    if (((pf >> 19) & 3) == 2) w.str(",\"shared\":true");
    w.str("}");
  }
  w.str("]");
  return w.pos;
}

#include "../../include/zdl.h"

extern "C" {

// The caller side of zdl_put_trace as the reference's callers drive putTrace - one call per
// trace, in order (InMemoryStorage.java:340 linkDependencies, mysql-v1
// AggregateDependencies.java:81) - what a JNI shim does after packing each trace: the column
// slices of trace t are handed over, nothing else. `put` is zdl_put_trace (passed in so this
// host helper does not link libzdl). Returns the first non-zero status (and its trace in *at).
int zdl_synth_put_trace_loop(int (*put)(zdl_ctx*, const zdl_span_cols*, uint64_t), zdl_ctx* ctx,
                             const zdl_span_cols* cols, const uint64_t* off, uint64_t n_traces, uint64_t* at) {
  for (uint64_t t = 0; t < n_traces; ++t) {
    const uint64_t b = off[t];
    zdl_span_cols c{};
    c.trace_lo = cols->trace_lo ? cols->trace_lo + b : nullptr;
    c.id = cols->id + b;
    c.parent_id = cols->parent_id + b;
    c.local_svc = cols->local_svc + b;
    c.remote_svc = cols->remote_svc + b;
    c.local_ip4 = cols->local_ip4 + b;
    c.local_ip6 = cols->local_ip6 + b;
    c.port_flags = cols->port_flags + b;
    c.timestamp = cols->timestamp ? cols->timestamp + b : nullptr;
    const int rc = put(ctx, &c, off[t + 1] - b);
    if (rc != 0) {
      if (at) *at = t;
      return rc;
    }
  }
  return 0;
}

}  // extern "C"

#include <chrono>

#include "zdl_shard.h"

extern "C" {

// A device group's host split (zdl_shard.h, the code libzdl's group_put runs) on host columns:
// zdl_synth_shard_plan sizes the shards (spans, traces per shard), zdl_synth_shard plans and
// scatters into the caller's columns - out[d] (columns of spans[d] entries; off: traces[d] + 1
// entries, or NULL for ungrouped input) - and returns its wall-clock seconds (plan + scatter).
void zdl_synth_shard_plan(const zdl_span_cols* in, uint64_t n_spans, const uint64_t* off, uint64_t n_traces,
                          uint32_t n_shards, int threads, uint64_t* spans, uint64_t* traces) {
  const zdl_shard::In x{in->trace_lo,  in->id,        in->parent_id,  in->local_svc, in->remote_svc,
                        in->local_ip4, in->local_ip6, in->port_flags, in->timestamp, in->ord};
  const zdl_shard::Plan p = zdl_shard::plan(x, n_spans, off, n_traces, n_shards, threads);
  for (uint32_t d = 0; d < n_shards; ++d) {
    spans[d] = p.spans[d];
    traces[d] = p.traces[d];
  }
}

double zdl_synth_shard(const zdl_span_cols* in, uint64_t n_spans, const uint64_t* off, uint64_t n_traces,
                       uint32_t n_shards, int threads, const zdl_span_cols* out, uint64_t* const* out_off) {
  const auto t0 = std::chrono::steady_clock::now();
  const zdl_shard::In x{in->trace_lo,  in->id,        in->parent_id,  in->local_svc, in->remote_svc,
                        in->local_ip4, in->local_ip6, in->port_flags, in->timestamp, in->ord};
  const zdl_shard::Plan p = zdl_shard::plan(x, n_spans, off, n_traces, n_shards, threads);
  std::vector<zdl_shard::Out> o(n_shards);
  for (uint32_t d = 0; d < n_shards; ++d)
    o[d] = zdl_shard::Out{const_cast<uint64_t*>(out[d].trace_lo), const_cast<uint64_t*>(out[d].id),
                          const_cast<uint64_t*>(out[d].parent_id), const_cast<int32_t*>(out[d].local_svc),
                          const_cast<int32_t*>(out[d].remote_svc), const_cast<int32_t*>(out[d].local_ip4),
                          const_cast<int32_t*>(out[d].local_ip6), const_cast<uint32_t*>(out[d].port_flags),
                          const_cast<int64_t*>(out[d].timestamp), const_cast<uint32_t*>(out[d].ord),
                          off ? out_off[d] : nullptr};
  zdl_shard::scatter(x, off, p, o.data(), threads);
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // extern "C"

