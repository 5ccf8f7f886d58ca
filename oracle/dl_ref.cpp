// ORACLE — TEST INFRASTRUCTURE ONLY, NEVER A PRODUCT PATH.
//
// C++ restatement of the reference's dependency-link algorithm over the
// columnar input of include/zdl.h, written from the Java sources (paths below
// relative to /root/reference/zipkin/src/main/java/zipkin2/), with the same
// data structures: a stable sort + ArrayList-style merge (internal/Trace.java),
// LinkedHashMap-ordered spanToParent and a node tree (internal/SpanNode.java),
// breadth-first rule pass and insertion-ordered pair counts
// (internal/DependencyLinker.java). It does not share code or formulation with
// the HIP engine (zipkin_amd/csrc), which is what makes it a checker.
//
// Used by tests/ (large-scale parity: same synthetic columns, bit-exact links)
// and by bench.py's cpu_baseline leg (timed on the GPU box's host cores).
// Cross-checked against the Python oracle (oracle/dl_oracle.py), which is pinned
// by the reference's own test vectors (tests/golden/).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <optional>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

struct NPE {};  // java.lang.NullPointerException
struct IAE {};  // java.lang.IllegalArgumentException

struct Ep {  // zipkin2.Endpoint restricted to its identity (Endpoint.java:554-563)
  int32_t svc = -1, ip4 = -1, ip6 = -1;
  uint32_t port = 0;
  bool is_null() const { return svc < 0 && ip4 < 0 && ip6 < 0 && port == 0; }
  bool operator==(const Ep& o) const { return svc == o.svc && ip4 == o.ip4 && ip6 == o.ip6 && port == o.port; }
};

struct REp {  // remote endpoint: service name + which other fields are set
  int32_t svc = -1;
  uint32_t bits = 0;  // 1 ipv4, 2 ipv6, 4 port
  bool is_null() const { return svc < 0 && bits == 0; }
};

struct Span {
  uint64_t id = 0, pid = 0;  // pid 0 = null
  int kind = -1;             // -1 null, 0 CLIENT 1 SERVER 2 PRODUCER 3 CONSUMER
  int shared_set = 0, shared_val = 0;
  Ep local;
  REp remote;
  bool err = false;
  bool shared_true() const { return shared_set && shared_val; }
};

struct Ranks {
  const int32_t* r[3];
  uint32_t n[3];
  int64_t rank(int which, int32_t id) const {
    if (r[which] && (uint32_t)id < n[which]) return r[which][id];
    return id;
  }
};

// Trace.nullSafeCompareTo for dictionary-encoded strings (Trace.java:118-126)
int cmp_str(const Ranks& R, int which, int32_t a, int32_t b, bool null_first) {
  if (a < 0) return b < 0 ? 0 : (null_first ? -1 : 1);
  if (b < 0) return null_first ? 1 : -1;
  const int64_t ra = R.rank(which, a), rb = R.rank(which, b);
  return ra < rb ? -1 : (ra > rb ? 1 : 0);
}

// Trace.compareEndpoint (Trace.java:105-116)
int cmp_endpoint(const Ranks& R, const Ep& l, const Ep& r) {
  if (l.is_null()) return r.is_null() ? 0 : -1;
  if (r.is_null()) return 1;
  int c = cmp_str(R, 0, l.svc, r.svc, false);
  if (c) return c;
  c = cmp_str(R, 1, l.ip4, r.ip4, false);
  if (c) return c;
  return cmp_str(R, 2, l.ip6, r.ip6, false);
}

// Trace.CLEANUP_COMPARATOR (Trace.java:89-98)
int cleanup_compare(const Ranks& R, const Span& l, const Span& r) {
  if (l.id != r.id) return l.id < r.id ? -1 : 1;
  // nullSafeCompareTo(shared, shared, nullFirst = true); Boolean false < true
  const int ls = l.shared_set ? 1 + l.shared_val : 0, rs = r.shared_set ? 1 + r.shared_val : 0;
  if (ls != rs) return ls < rs ? -1 : 1;
  return cmp_endpoint(R, l.local, r.local);
}

struct EndpointTracker {  // Trace.java:132-157
  int32_t svc = -1, ip4 = -1, ip6 = -1;
  uint32_t port = 0;
  bool try_merge(const Ep& e) {
    if (e.is_null()) return true;
    if (svc >= 0 && e.svc >= 0 && svc != e.svc) return false;
    if (ip4 >= 0 && e.ip4 >= 0 && ip4 != e.ip4) return false;
    if (ip6 >= 0 && e.ip6 >= 0 && ip6 != e.ip6) return false;
    if (port != 0 && e.port != 0 && port != e.port) return false;
    if (svc < 0) svc = e.svc;
    if (ip4 < 0) ip4 = e.ip4;
    if (ip6 < 0) ip6 = e.ip6;
    if (port == 0) port = e.port;
    return true;
  }
};

// Endpoint.Builder.merge (Endpoint.java:121-129): dereferences a null source at the
// first field the accumulator lacks.
Ep merge_local(const Ep& acc, const Ep& src) {
  Ep r = acc;
  const bool src_null = src.is_null();
  if (r.svc < 0) { if (src_null) throw NPE(); r.svc = src.svc; }
  if (r.ip4 < 0) { if (src_null) throw NPE(); r.ip4 = src.ip4; }
  if (r.ip6 < 0) { if (src_null) throw NPE(); r.ip6 = src.ip6; }
  if (r.port == 0) { if (src_null) throw NPE(); r.port = src.port; }
  return r;
}

REp merge_remote(const REp& acc, const REp& src) {
  REp r = acc;
  const bool src_null = src.is_null();
  if (r.svc < 0) { if (src_null) throw NPE(); r.svc = src.svc; }
  for (uint32_t bit : {1u, 2u, 4u})
    if (!(r.bits & bit)) { if (src_null) throw NPE(); r.bits |= (src.bits & bit); }
  return r;
}

// Span.Builder.merge (Span.java:358-388)
void builder_merge(Span& b, const Span& src) {
  if (b.pid == 0) b.pid = src.pid;
  if (b.kind < 0) b.kind = src.kind;
  if (b.local.is_null()) b.local = src.local; else b.local = merge_local(b.local, src.local);
  if (b.remote.is_null()) b.remote = src.remote; else b.remote = merge_remote(b.remote, src.remote);
  b.err = b.err || src.err;
  if (src.shared_set) { b.shared_set = 1; b.shared_val = b.shared_val || src.shared_val; }  // flags OR
}

// Trace.merge (Trace.java:28-87)
std::vector<Span> trace_merge(const Ranks& R, const std::vector<Span>& spans) {
  int length = (int)spans.size();
  if (length <= 1) return spans;
  std::vector<Span> result = spans;
  std::stable_sort(result.begin(), result.end(),
                   [&](const Span& a, const Span& b) { return cleanup_compare(R, a, b) < 0; });
  for (int i = 0; i < length; i++) {
    Span previous = result[i];
    const uint64_t previous_id = previous.id;
    const bool previous_shared = previous.shared_true();
    std::optional<Span> replacement;
    std::optional<EndpointTracker> tracker;
    while (i + 1 < length) {
      const Span next = result[i + 1];
      if (next.id != previous_id) break;
      if (!tracker) {
        tracker.emplace();
        tracker->try_merge(previous.local);
      }
      const bool next_shared = next.shared_true();
      if (previous_shared == next_shared && tracker->try_merge(next.local)) {
        if (!replacement) replacement = previous;
        builder_merge(*replacement, next);
        previous = next;
        length--;
        result.erase(result.begin() + i + 1);
        continue;
      }
      if (next_shared && next.pid == 0 && previous.pid != 0) result[i + 1].pid = previous.pid;
      break;
    }
    if (replacement) {
      if (replacement->pid == replacement->id) replacement->pid = 0;  // Span.build
      result[i] = *replacement;
    }
  }
  return result;
}

// SpanNode.Key (SpanNode.java:256-293)
struct Key {
  uint64_t id;
  bool shared;
  bool has_ep;
  Ep ep;
  bool operator==(const Key& o) const {
    return id == o.id && shared == o.shared && has_ep == o.has_ep && (!has_ep || ep == o.ep);
  }
};
struct KeyHash {
  size_t operator()(const Key& k) const {
    uint64_t h = k.id * 0x9E3779B97F4A7C15ull ^ (k.shared ? 1231 : 1237);
    if (k.has_ep) {
      h = h * 1000003 ^ (uint32_t)k.ep.svc;
      h = h * 1000003 ^ (uint32_t)k.ep.ip4;
      h = h * 1000003 ^ (uint32_t)k.ep.ip6;
      h = h * 1000003 ^ k.ep.port;
    }
    return (size_t)(h ^ (h >> 29));
  }
};

Key make_key(uint64_t id, bool shared, const Ep* ep) {
  Key k{id, shared, ep != nullptr && !ep->is_null(), Ep()};
  if (k.has_ep) k.ep = *ep;
  return k;
}

// java.util.LinkedHashMap: put on an existing key keeps its position; remove + put
// appends at the end.
template <class K, class V, class H>
struct LinkedMap {
  struct E {
    K k;
    V v;
    bool live;
  };
  std::vector<E> entries;
  std::unordered_map<K, size_t, H> idx;
  void put(const K& k, const V& v) {
    auto it = idx.find(k);
    if (it != idx.end()) {
      entries[it->second].v = v;
      return;
    }
    idx.emplace(k, entries.size());
    entries.push_back(E{k, v, true});
  }
  bool contains(const K& k) const { return idx.count(k) != 0; }
  V* get(const K& k) {
    auto it = idx.find(k);
    return it == idx.end() ? nullptr : &entries[it->second].v;
  }
  void remove(const K& k) {
    auto it = idx.find(k);
    if (it == idx.end()) return;
    entries[it->second].live = false;
    idx.erase(it);
  }
};

struct Node {
  int span = -1;  // -1 = synthetic root
  int parent = -1;
  std::vector<int> children;
};

struct Tree {
  std::vector<Node> nodes;
  int root = -1;
  void add_child(int self, int child) {  // SpanNode.addChild (SpanNode.java:92-103)
    if (child < 0) throw NPE();
    if (child == self) throw IAE();
    auto& ch = nodes[self].children;
    if (std::find(ch.begin(), ch.end(), child) != ch.end()) throw IAE();
    ch.push_back(child);
    nodes[child].parent = self;
  }
};

// SpanNode.Builder.build (SpanNode.java:122-249)
Tree build_tree(const std::vector<Span>& cleaned) {
  Tree t;
  std::unordered_map<Key, int, KeyHash> key_to_node;
  LinkedMap<Key, std::optional<Key>, KeyHash> span_to_parent;
  for (const Span& s : cleaned) {  // index (SpanNode.java:179-192)
    if (s.shared_true()) {
      span_to_parent.put(make_key(s.id, true, &s.local), make_key(s.id, false, nullptr));
    } else {
      std::optional<Key> pk;
      if (s.pid) pk = make_key(s.pid, false, nullptr);
      span_to_parent.put(make_key(s.id, false, nullptr), pk);
    }
  }
  for (size_t i = 0; i < cleaned.size(); ++i) {  // process (SpanNode.java:203-249)
    const Span& s = cleaned[i];
    const bool shared = s.shared_true();
    const Key key = make_key(s.id, shared, &s.local);
    const Key nek = make_key(s.id, shared, nullptr);
    std::optional<Key> parent;
    if (shared) {
      parent = make_key(s.id, false, nullptr);
    } else if (s.pid) {
      Key p = make_key(s.pid, true, &s.local);
      if (span_to_parent.contains(p)) {
        span_to_parent.put(nek, p);
        parent = p;
      } else {
        parent = make_key(s.pid, false, nullptr);
      }
    }
    t.nodes.push_back(Node{(int)i, -1, {}});
    const int node = (int)t.nodes.size() - 1;
    if (!parent && t.root < 0) {
      t.root = node;
      span_to_parent.remove(nek);
    } else if (shared) {
      key_to_node[key] = node;
      key_to_node[nek] = node;
    } else {
      key_to_node[nek] = node;
    }
  }
  if (t.root < 0) {
    t.nodes.push_back(Node{-1, -1, {}});
    t.root = (int)t.nodes.size() - 1;
  }
  for (const auto& e : span_to_parent.entries) {
    if (!e.live) continue;
    auto c = key_to_node.find(e.k);
    const int child = c == key_to_node.end() ? -1 : c->second;
    int parent = -1;
    if (e.v) {
      auto p = key_to_node.find(*e.v);
      if (p != key_to_node.end()) parent = p->second;
    }
    t.add_child(parent < 0 ? t.root : parent, child);
  }
  return t;
}

struct PairHash {
  size_t operator()(const std::pair<int32_t, int32_t>& p) const {
    return (size_t)((uint64_t)(uint32_t)p.first * 1000003ull ^ (uint32_t)p.second);
  }
};

struct Linker {  // DependencyLinker.java:37-247
  LinkedMap<std::pair<int32_t, int32_t>, std::pair<int64_t, int64_t>, PairHash> counts;

  void add_link(int32_t parent, int32_t child, bool is_error) {  // :166-182
    const auto k = std::make_pair(parent, child);
    auto* v = counts.get(k);
    if (!v) {
      counts.put(k, {0, 0});
      v = counts.get(k);
    }
    v->first += 1;
    if (is_error) v->second += 1;
  }

  void put_trace(const Ranks& R, const std::vector<Span>& spans) {  // :53-151
    if (spans.empty()) return;
    const std::vector<Span> cleaned = trace_merge(R, spans);
    const Tree tree = build_tree(cleaned);
    std::deque<int> q{tree.root};
    while (!q.empty()) {
      const int cur = q.front();
      q.pop_front();
      const Node& n = tree.nodes[cur];
      for (int c : n.children) q.push_back(c);
      if (n.span < 0) continue;  // skipping fake root node
      const Span& s = cleaned[n.span];
      int kind = s.kind;
      if (kind == 0 && !n.children.empty()) continue;
      const int32_t service = s.local.svc, remote = s.remote.svc;
      if (kind < 0) {
        if (service >= 0 && remote >= 0) kind = 0; else continue;
      }
      int32_t child, parent;
      if (kind == 1 || kind == 3) {
        child = service;
        parent = remote;
        if (cur == tree.root && parent < 0) continue;
      } else {
        parent = service;
        child = remote;
      }
      bool is_error = s.err;
      if (kind == 2 || kind == 3) {
        if (parent >= 0 && child >= 0) add_link(parent, child, is_error);
        continue;
      }
      // firstRemoteAncestor (:153-164)
      const Span* ra = nullptr;
      for (int a = n.parent; a >= 0; a = tree.nodes[a].parent) {
        const int si = tree.nodes[a].span;
        if (si >= 0 && cleaned[si].kind >= 0) { ra = &cleaned[si]; break; }
      }
      if (ra && ra->local.svc >= 0) {
        const int32_t ran = ra->local.svc;
        if (kind == 0 && service >= 0 && ran != service) add_link(ran, service, false);
        if (kind == 1 || parent < 0) parent = ran;
        if (!is_error && ra->kind == 0 && s.pid != 0 && s.pid == ra->id) is_error = ra->err;
      }
      if (parent < 0 || child < 0) continue;
      add_link(parent, child, is_error);
    }
  }
};

struct Cols {
  const uint64_t* id;
  const uint64_t* pid;
  const int32_t* lsvc;
  const int32_t* rsvc;
  const int32_t* ip4;
  const int32_t* ip6;
  const uint32_t* pf;
  const int64_t* ts;
};

Span span_at(const Cols& c, uint64_t g) {
  Span s;
  s.id = c.id[g];
  s.pid = c.pid[g] == s.id ? 0 : c.pid[g];
  const uint32_t pf = c.pf[g];
  const uint32_t k = (pf >> 16) & 7u;
  s.kind = k == 7u ? -1 : (int)k;
  const uint32_t sh = (pf >> 19) & 3u;
  s.shared_set = sh != 0;
  s.shared_val = sh == 2;
  s.local = Ep{c.lsvc[g], c.ip4[g], c.ip6[g], pf & 0xFFFFu};
  s.remote = REp{c.rsvc[g], (pf >> 22) & 7u};
  s.err = (pf >> 21) & 1u;
  return s;
}

// QueryRequest.test time rule (storage/QueryRequest.java:262-279)
bool window_pass(const Cols& c, uint64_t b, uint64_t e, int64_t lo, int64_t hi) {
  int64_t ts = 0;
  for (uint64_t g = b; g < e; ++g) {
    const int64_t x = c.ts[g];
    if (x == 0) continue;
    const uint64_t pid = c.pid[g] == c.id[g] ? 0 : c.pid[g];
    if (pid == 0) { ts = x; break; }
    if (ts == 0 || ts > x) ts = x;
  }
  return !(ts == 0 || ts < lo || ts > hi);
}

struct Result {
  int status = 0;
  std::vector<int32_t> p, c;
  std::vector<int64_t> call, err;
};

}  // namespace

extern "C" {

typedef struct oracle_cols {
  const uint64_t* id;
  const uint64_t* parent_id;
  const int32_t* local_svc;
  const int32_t* remote_svc;
  const int32_t* local_ip4;
  const int32_t* local_ip6;
  const uint32_t* port_flags;
  const int64_t* timestamp;
} oracle_cols;

// Runs DependencyLinker over CSR-grouped traces. threads > 1 shards contiguous trace
// ranges over DependencyLinker instances and combines them with DependencyLinker.merge
// semantics in range order (first-seen order is preserved). Result in insertion order.
void* oracle_link(const oracle_cols* cols, uint64_t n_spans, const uint64_t* off, uint64_t n_traces,
                  const int32_t* svc_rank, uint32_t nsvc, const int32_t* ip4_rank, uint32_t nip4,
                  const int32_t* ip6_rank, uint32_t nip6, int window, int64_t win_lo, int64_t win_hi,
                  int threads) {
  (void)n_spans;
  const Cols c{cols->id, cols->parent_id, cols->local_svc, cols->remote_svc, cols->local_ip4,
               cols->local_ip6, cols->port_flags, cols->timestamp};
  const Ranks R{{svc_rank, ip4_rank, ip6_rank}, {nsvc, nip4, nip6}};
  threads = std::max(1, threads);
  if ((uint64_t)threads > n_traces) threads = (int)std::max<uint64_t>(1, n_traces);
  std::vector<Linker> linkers(threads);
  std::vector<int> status(threads, 0);
  auto work = [&](int w) {
    const uint64_t b = n_traces * w / threads, e = n_traces * (w + 1) / threads;
    std::vector<Span> trace;
    try {
      for (uint64_t t = b; t < e; ++t) {
        if (window && !window_pass(c, off[t], off[t + 1], win_lo, win_hi)) continue;
        trace.clear();
        for (uint64_t g = off[t]; g < off[t + 1]; ++g) trace.push_back(span_at(c, g));
        linkers[w].put_trace(R, trace);
      }
    } catch (const NPE&) {
      status[w] = -4;
    } catch (const IAE&) {
      status[w] = -5;
    }
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> ts;
    for (int w = 0; w < threads; ++w) ts.emplace_back(work, w);
    for (auto& t : ts) t.join();
  }
  Result* r = new Result();
  for (int s : status)
    if (s && !r->status) r->status = s;
  // DependencyLinker.merge over the shard results, in shard order (:189-204)
  LinkedMap<std::pair<int32_t, int32_t>, std::pair<int64_t, int64_t>, PairHash> merged;
  for (auto& l : linkers)
    for (auto& e : l.counts.entries) {
      if (!e.live) continue;
      auto* v = merged.get(e.k);
      if (!v) {
        merged.put(e.k, {0, 0});
        v = merged.get(e.k);
      }
      v->first += e.v.first;
      v->second += e.v.second;
    }
  for (auto& e : merged.entries) {
    r->p.push_back(e.k.first);
    r->c.push_back(e.k.second);
    r->call.push_back(e.v.first);
    r->err.push_back(e.v.second);
  }
  return r;
}

int oracle_status(void* h) { return ((Result*)h)->status; }
uint64_t oracle_count(void* h) { return ((Result*)h)->p.size(); }
void oracle_copy(void* h, int32_t* p, int32_t* c, int64_t* call, int64_t* err) {
  Result* r = (Result*)h;
  const size_t n = r->p.size();
  if (n == 0) return;
  std::memcpy(p, r->p.data(), n * 4);
  std::memcpy(c, r->c.data(), n * 4);
  std::memcpy(call, r->call.data(), n * 8);
  std::memcpy(err, r->err.data(), n * 8);
}
void oracle_free(void* h) { delete (Result*)h; }

}  // extern "C"
