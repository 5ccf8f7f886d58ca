// zdl_algo.h — per-trace dependency-link algorithm as device functions.
//
// The reference builds a tree per trace with hash maps and walks it
// (internal/Trace.java, internal/SpanNode.java, internal/DependencyLinker.java).
// Here the same result is computed from flat arrays that a workgroup holds in
// LDS (tile kernel) or in HBM scratch (big-trace kernel):
//
//   slot      a span's index in the input order of its trace (storage order)
//   position  its index after the Trace.merge sort; positions of one trace
//             occupy the same range as its slots
//
// Field arrays are indexed by slot; perm/parent/live/haschild by position.
// The LinkedHashMap semantics of SpanNode.Builder reduce to "last cleaned span
// in sorted order with property P" rules, derived in DESIGN.md §3 and
// restated at each function below. Everything is integer; results are exact.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zdl.h"

namespace zdl {

enum : uint32_t { ST_NPE = 1u, ST_BADSVC = 2u, ST_BADOFF = 4u, ST_IAE = 8u, ST_INTERNAL = 16u, ST_DAYS = 64u };  // (32: unused)
enum : int32_t { PAR_TERMINAL = -1, PAR_NONMEMBER = -3 };

template <class PermT, class ParT>
struct ViewT {
  uint64_t* id;
  uint64_t* pid;
  int32_t* lsvc;
  int32_t* rsvc;
  int32_t* ip4;
  int32_t* ip6;
  uint32_t* pf;
  PermT* perm;        // position -> slot
  ParT* parent;       // position -> parent position | PAR_TERMINAL | PAR_NONMEMBER
  uint8_t* live;      // position -> 1 if it heads a cleaned span (Trace.merge output)
  uint8_t* haschild;  // position -> 1 if some node's tree parent is this position
};
using View = ViewT<uint32_t, int32_t>;   // HBM scratch (big traces)
using WView = ViewT<uint8_t, int16_t>;   // one wave's 128 LDS slots

struct Ranks {
  const int32_t* svc;
  const int32_t* ip4;
  const int32_t* ip6;
  uint32_t nsvc, nip4, nip6;
};

__device__ __forceinline__ uint32_t kind_of(uint32_t pf) { return (pf >> ZDL_PF_KIND_SHIFT) & 7u; }
__device__ __forceinline__ uint32_t shared_of(uint32_t pf) { return (pf >> ZDL_PF_SHARED_SHIFT) & 3u; }
__device__ __forceinline__ uint32_t port_of(uint32_t pf) { return pf & ZDL_PF_PORT_MASK; }
__device__ __forceinline__ bool err_of(uint32_t pf) { return (pf & ZDL_PF_ERROR) != 0; }
__device__ __forceinline__ uint32_t rbits_of(uint32_t pf) { return (pf >> 22) & 7u; }
__device__ __forceinline__ bool is_shared(uint32_t pf) { return shared_of(pf) == 2u; }

template <class V>
__device__ __forceinline__ bool local_null(const V& v, uint32_t s) {
  return v.lsvc[s] < 0 && v.ip4[s] < 0 && v.ip6[s] < 0 && port_of(v.pf[s]) == 0;
}

// Endpoint.equals on (serviceName, ipv4, ipv6, port), Endpoint.java:554-563; null == null.
template <class V>
__device__ __forceinline__ bool local_eq(const V& v, uint32_t a, uint32_t b) {
  return v.lsvc[a] == v.lsvc[b] && v.ip4[a] == v.ip4[b] && v.ip6[a] == v.ip6[b] &&
         port_of(v.pf[a]) == port_of(v.pf[b]);
}

__device__ __forceinline__ int32_t rank_of(int32_t id, const int32_t* rank, uint32_t n) {
  if (id < 0) return 0x7fffffff;  // nulls last (Trace.nullSafeCompareTo(.., false))
  if (rank != nullptr && (uint32_t)id < n) return rank[id];
  return id;
}

// Trace.CLEANUP_COMPARATOR (Trace.java:89-98) made total with the slot as the final key,
// which reproduces Collections.sort's stability: (id, shared tri-state null<false<true,
// local endpoint: null first, then serviceName/ipv4/ipv6 by String order, nulls last;
// port ignored), then storage order.
template <class V>
__device__ __forceinline__ bool span_less(const V& v, const Ranks& R, uint32_t a, uint32_t b) {
  const uint64_t ia = v.id[a], ib = v.id[b];
  if (ia != ib) return ia < ib;
  const uint32_t sa = shared_of(v.pf[a]), sb = shared_of(v.pf[b]);
  if (sa != sb) return sa < sb;
  const bool na = local_null(v, a), nb = local_null(v, b);
  if (na != nb) return na;
  if (!na) {
    int32_t ra = rank_of(v.lsvc[a], R.svc, R.nsvc), rb = rank_of(v.lsvc[b], R.svc, R.nsvc);
    if (ra != rb) return ra < rb;
    ra = rank_of(v.ip4[a], R.ip4, R.nip4);
    rb = rank_of(v.ip4[b], R.ip4, R.nip4);
    if (ra != rb) return ra < rb;
    ra = rank_of(v.ip6[a], R.ip6, R.nip6);
    rb = rank_of(v.ip6[b], R.ip6, R.nip6);
    if (ra != rb) return ra < rb;
  }
  return a < b;
}

// Span.Builder accumulating a merge run (Span.java:358-388, Endpoint.java:121-129).
struct Acc {
  uint64_t pid;
  int32_t lsvc, ip4, ip6, rsvc;
  uint32_t port, kind, shared, rbits;
  bool err;
};

template <class V>
__device__ __forceinline__ Acc acc_load(const V& v, uint32_t s) {
  const uint32_t pf = v.pf[s];
  Acc a;
  a.pid = v.pid[s];
  a.lsvc = v.lsvc[s];
  a.ip4 = v.ip4[s];
  a.ip6 = v.ip6[s];
  a.rsvc = v.rsvc[s];
  a.port = port_of(pf);
  a.kind = kind_of(pf);
  a.shared = shared_of(pf);
  a.rbits = rbits_of(pf);
  a.err = err_of(pf);
  return a;
}

template <class V>
__device__ __forceinline__ void acc_store(const V& v, uint32_t s, const Acc& a) {
  v.pid[s] = a.pid;
  v.lsvc[s] = a.lsvc;
  v.ip4[s] = a.ip4;
  v.ip6[s] = a.ip6;
  v.rsvc[s] = a.rsvc;
  v.pf[s] = a.port | (a.kind << ZDL_PF_KIND_SHIFT) | (a.shared << ZDL_PF_SHARED_SHIFT) |
            (a.err ? ZDL_PF_ERROR : 0u) | (a.rbits << 22);
}

// Builder.merge(source): first non-null wins per field; an endpoint merge with a null
// source dereferences it at the first field the accumulator lacks (quirk Q1 -> NPE).
template <class V>
__device__ __forceinline__ bool acc_merge(Acc& a, const V& v, uint32_t s) {
  bool npe = false;
  const uint32_t pf = v.pf[s];
  if (a.pid == 0) a.pid = v.pid[s];
  if (a.kind == ZDL_KIND_NULL) a.kind = kind_of(pf);
  const int32_t sl = v.lsvc[s], s4 = v.ip4[s], s6 = v.ip6[s];
  const uint32_t sp = port_of(pf);
  const bool acc_lnull = a.lsvc < 0 && a.ip4 < 0 && a.ip6 < 0 && a.port == 0;
  const bool src_lnull = sl < 0 && s4 < 0 && s6 < 0 && sp == 0;
  if (acc_lnull) {
    a.lsvc = sl; a.ip4 = s4; a.ip6 = s6; a.port = sp;
  } else if (src_lnull) {
    if (a.lsvc < 0 || a.ip4 < 0 || a.ip6 < 0 || a.port == 0) npe = true;
  } else {
    if (a.lsvc < 0) a.lsvc = sl;
    if (a.ip4 < 0) a.ip4 = s4;
    if (a.ip6 < 0) a.ip6 = s6;
    if (a.port == 0) a.port = sp;
  }
  const int32_t sr = v.rsvc[s];
  const uint32_t sb = rbits_of(pf);
  const bool acc_rnull = a.rsvc < 0 && a.rbits == 0;
  const bool src_rnull = sr < 0 && sb == 0;
  if (acc_rnull) {
    a.rsvc = sr; a.rbits = sb;
  } else if (src_rnull) {
    if (a.rsvc < 0 || a.rbits != 7u) npe = true;
  } else {
    if (a.rsvc < 0) a.rsvc = sr;
    a.rbits |= sb;
  }
  a.err = a.err || err_of(pf);
  if (shared_of(pf) > a.shared) a.shared = shared_of(pf);  // flags OR (Span.java:387)
  return npe;
}

// Trace.merge's greedy scan over one id group [gb, ge) of sorted positions
// (Trace.java:42-84). Run by one lane. Heads of merge runs become live; the merged
// span is written over the head's slot. Returns true if the reference would NPE.
template <class V>
__device__ __forceinline__ bool merge_group(const V& v, int gb, int ge) {
  bool npe = false;
  int i = gb;
  while (i < ge) {
    const uint32_t head = v.perm[i];
    const bool prev_shared = is_shared(v.pf[head]);
    uint32_t prev = head;  // Q7: `previous` is the last raw fragment absorbed
    v.live[i] = 1;
    int j = i + 1;
    if (j < ge) {
      // EndpointTracker seeded with previous.localEndpoint (Trace.java:58-61)
      int32_t tsv = v.lsvc[head], t4 = v.ip4[head], t6 = v.ip6[head];
      uint32_t tp = port_of(v.pf[head]);
      Acc acc = acc_load(v, head);
      bool merged = false;
      for (; j < ge; ++j) {
        const uint32_t nx = v.perm[j];
        const uint32_t npf = v.pf[nx];
        bool ok = is_shared(npf) == prev_shared;
        if (ok) {  // EndpointTracker.tryMerge (Trace.java:136-156)
          const int32_t esv = v.lsvc[nx], e4 = v.ip4[nx], e6 = v.ip6[nx];
          const uint32_t ep = port_of(npf);
          if (!(esv < 0 && e4 < 0 && e6 < 0 && ep == 0)) {
            if ((tsv >= 0 && esv >= 0 && tsv != esv) || (t4 >= 0 && e4 >= 0 && t4 != e4) ||
                (t6 >= 0 && e6 >= 0 && t6 != e6) || (tp != 0 && ep != 0 && tp != ep)) {
              ok = false;
            } else {
              if (tsv < 0) tsv = esv;
              if (t4 < 0) t4 = e4;
              if (t6 < 0) t6 = e6;
              if (tp == 0) tp = ep;
            }
          }
        }
        if (ok) {
          npe |= acc_merge(acc, v, nx);
          merged = true;
          prev = nx;
          v.live[j] = 0;
          continue;
        }
        // backfill a shared server's missing parent id (Trace.java:76-79)
        if (is_shared(npf) && v.pid[nx] == 0 && v.pid[prev] != 0) v.pid[nx] = v.pid[prev];
        break;
      }
      if (merged) acc_store(v, head, acc);
    }
    i = j;
  }
  return npe;
}

// lower_bound of span id P over positions [tb, te) (ids are sorted by position).
template <class V>
__device__ __forceinline__ void find_group(const V& v, int tb, int te, uint64_t P, int& gb, int& ge) {
  int lo = tb, hi = te;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (v.id[v.perm[mid]] < P) lo = mid + 1; else hi = mid;
  }
  gb = lo;
  int e = lo;
  while (e < te && v.id[v.perm[e]] == P) ++e;
  ge = e;
}

// K2N[Key(P, true, ep)] (SpanNode.java:244-245): the last shared cleaned span with id P
// whose local endpoint equals the slot `es`'s; -1 when SpanNode.Builder holds no such key.
template <class V>
__device__ __forceinline__ int last_shared_with_ep(const V& v, int tb, int te, uint64_t P, uint32_t es) {
  int gb, ge;
  find_group(v, tb, te, P, gb, ge);
  int r = -1;
  for (int q = gb; q < ge; ++q)
    if (v.live[q] && is_shared(v.pf[v.perm[q]]) && local_eq(v, v.perm[q], es)) r = q;
  return r;
}

// K2N[Key(P, false, null)] (SpanNode.java:247): the last non-shared cleaned span with id
// P that is not the root (the root is never put in keyToNode, SpanNode.java:238-240).
template <class V>
__device__ __forceinline__ int last_nonshared(const V& v, int tb, int te, uint64_t P, int rp) {
  int gb, ge;
  find_group(v, tb, te, P, gb, ge);
  int r = -1;
  for (int q = gb; q < ge; ++q)
    if (v.live[q] && q != rp && !is_shared(v.pf[v.perm[q]])) r = q;
  return r;
}

// Tree edges of one id group [gb, ge) — the final state of SpanNode.Builder's
// spanToParent/keyToNode maps after index() and process() (SpanNode.java:122-249):
//  * a shared span is a node iff it is the last shared one with its (id, endpoint);
//    its parent is K2N[Key(id,false,null)], else the root;
//  * Key(id,false,null) is attached iff it survives the root's removal: when the root
//    has this id, only a later process() write (a child of a same-endpoint shared
//    span) re-inserts it. Its node is the last non-root non-shared span; its parent is
//    the value of the last write: Key(pid,true,ep) from process(), else index()'s
//    Key(pid,false,null) of the last non-shared span, else none (-> root).
template <class V>
__device__ __forceinline__ void resolve_group(const V& v, int tb, int te, int gb, int ge, int rp) {
  const int root_attach = rp >= 0 ? rp : PAR_TERMINAL;
  int last_ns = -1, last_ns_any = -1, last_w = -1;
  for (int p = gb; p < ge; ++p) {
    if (!v.live[p]) { v.parent[p] = PAR_NONMEMBER; continue; }
    const uint32_t s = v.perm[p];
    if (is_shared(v.pf[s])) continue;
    v.parent[p] = PAR_NONMEMBER;
    last_ns_any = p;
    if (p != rp) last_ns = p;
    const uint64_t P = v.pid[s];
    if (P != 0 && last_shared_with_ep(v, tb, te, P, s) >= 0) last_w = p;
  }
  for (int p = gb; p < ge; ++p) {
    if (!v.live[p]) continue;
    const uint32_t s = v.perm[p];
    if (!is_shared(v.pf[s])) continue;
    bool last = true;
    for (int q = p + 1; q < ge; ++q)
      if (v.live[q] && is_shared(v.pf[v.perm[q]]) && local_eq(v, s, v.perm[q])) { last = false; break; }
    v.parent[p] = last ? (last_ns >= 0 ? last_ns : root_attach) : PAR_NONMEMBER;
  }
  const bool root_here = rp >= gb && rp < ge;
  if (root_here) v.parent[rp] = PAR_TERMINAL;
  const bool w_after = last_w >= 0 && (!root_here || last_w > rp);
  const bool present = root_here ? w_after : (last_ns_any >= 0);
  if (!present) return;
  int par;
  if (w_after) {
    const uint32_t ws = v.perm[last_w];
    par = last_shared_with_ep(v, tb, te, v.pid[ws], ws);
  } else {
    const uint64_t P = v.pid[v.perm[last_ns_any]];
    if (P == 0) {
      par = root_attach;
    } else {
      const int q = last_nonshared(v, tb, te, P, rp);
      par = q >= 0 ? q : root_attach;
    }
  }
  v.parent[last_ns] = (decltype(+v.parent[0]))par;
}

// DependencyLinker.putTrace's per-node rules (DependencyLinker.java:58-148) for the node
// at position p; `emit(parent_svc, child_svc, is_error, k)` is addLink, k its order within
// the node (0: the missing-link backfill, DependencyLinker.java:126-129; 1: the node's link).
template <class V, class Emit>
__device__ __forceinline__ void link_node(const V& v, int p, int rp, int n, Emit&& emit) {
  // reachability from the root and firstRemoteAncestor (DependencyLinker.java:153-164)
  int q = v.parent[p];
  int ra = -1;
  int steps = 0;
  bool reach = false;
  while (true) {
    if (q == PAR_TERMINAL) { reach = true; break; }
    if (q < 0) break;                  // under a node that is not in the tree
    if (ra < 0 && kind_of(v.pf[v.perm[q]]) != ZDL_KIND_NULL) ra = q;
    q = v.parent[q];
    if (++steps > n) break;            // cycle not through the root: never visited
  }
  if (!reach) return;
  const uint32_t s = v.perm[p];
  const uint32_t pf = v.pf[s];
  uint32_t kind = kind_of(pf);
  if (kind == ZDL_KIND_CLIENT && v.haschild[p]) return;
  const int32_t svc = v.lsvc[s], rsvc = v.rsvc[s];
  if (kind == ZDL_KIND_NULL) {
    if (svc >= 0 && rsvc >= 0) kind = ZDL_KIND_CLIENT; else return;
  }
  int32_t parent, child;
  if (kind == ZDL_KIND_SERVER || kind == ZDL_KIND_CONSUMER) {
    child = svc;
    parent = rsvc;
    if (p == rp && parent < 0) return;  // root's client is unknown
  } else {
    parent = svc;
    child = rsvc;
  }
  bool is_error = err_of(pf);
  if (kind == ZDL_KIND_PRODUCER || kind == ZDL_KIND_CONSUMER) {
    if (parent >= 0 && child >= 0) emit(parent, child, is_error, 1);
    return;
  }
  if (ra >= 0) {
    const uint32_t as = v.perm[ra];
    const int32_t ran = v.lsvc[as];
    if (ran >= 0) {
      if (kind == ZDL_KIND_CLIENT && svc >= 0 && ran != svc) emit(ran, svc, false, 0);  // missing link
      if (kind == ZDL_KIND_SERVER || parent < 0) parent = ran;
      const uint64_t mypid = v.pid[s];
      if (!is_error && kind_of(v.pf[as]) == ZDL_KIND_CLIENT && mypid != 0 && mypid == v.id[as])
        is_error = err_of(v.pf[as]);
    }
  }
  if (parent >= 0 && child >= 0) emit(parent, child, is_error, 1);
}

// ZDL_FLAG_TREE_EXPORT's reason codes (ZDL_RSN_*): the branch DependencyLinker.putTrace takes
// for one visited node (DependencyLinker.java:58-148), from which the host renders the FINE
// messages. Restates link_node's decisions without emitting; pid_match = the node's parent id
// is the ancestor's id (the split-RPC error check, :136-139).
struct Rsn {
  uint32_t code;
  int32_t pa, ch, xpa, xch;
};
__device__ __forceinline__ Rsn node_reason(uint32_t pf, bool haschild, int32_t svc, int32_t rsvc, bool is_root,
                                           bool has_anc, int32_t ran, uint32_t apf, bool pid_match) {
  Rsn r{0u, -1, -1, -1, -1};
  uint32_t kind = kind_of(pf);
  if (kind == ZDL_KIND_CLIENT && haschild) { r.code = ZDL_RSN_CLIENT_PARENT; return r; }
  if (kind == ZDL_KIND_NULL) {
    if (svc >= 0 && rsvc >= 0) kind = ZDL_KIND_CLIENT;
    else { r.code = ZDL_RSN_NON_REMOTE; return r; }
  }
  int32_t parent, child;
  if (kind == ZDL_KIND_SERVER || kind == ZDL_KIND_CONSUMER) {
    child = svc;
    parent = rsvc;
    if (is_root && parent < 0) { r.code = ZDL_RSN_ROOT_CLIENT_UNKNOWN; return r; }
  } else {
    parent = svc;
    child = rsvc;
  }
  bool is_error = err_of(pf);
  if (kind == ZDL_KIND_PRODUCER || kind == ZDL_KIND_CONSUMER) {
    if (parent >= 0 && child >= 0) {
      r.code = ZDL_RSN_MESSAGING | (is_error ? ZDL_RSN_ERROR : 0u);
      r.pa = parent;
      r.ch = child;
    } else {
      r.code = ZDL_RSN_MESSAGING_NO_BROKER;
    }
    return r;
  }
  uint32_t fl = 0;
  if (has_anc) {
    fl |= ZDL_RSN_ANCESTOR;
    if (ran >= 0) {
      if (kind == ZDL_KIND_CLIENT && svc >= 0 && ran != svc) {
        fl |= ZDL_RSN_MISSING_LINK;
        r.xpa = ran;
        r.xch = svc;
      }
      if (kind == ZDL_KIND_SERVER || parent < 0) parent = ran;
      if (!is_error && kind_of(apf) == ZDL_KIND_CLIENT && pid_match) is_error = err_of(apf);
    }
  }
  if (parent >= 0 && child >= 0) {
    r.code = ZDL_RSN_LINK | fl | (is_error ? ZDL_RSN_ERROR : 0u);
    r.pa = parent;
    r.ch = child;
  } else {
    r.code = ZDL_RSN_NO_REMOTE_ANCESTOR | fl;
  }
  return r;
}

// Insertion order (ZDL_FLAG_INSERTION_ORDER): first[cell] keeps the smallest rank of an
// addLink of that (parent, child): (put-global position of the trace's first span + the
// node's breadth-first index) << 1 | k. A trace of n spans has fewer than n nodes, so its
// ranks lie below the next trace's first position: the order is (trace, breadth-first
// index, k) with no bit field to outgrow - any trace size, positions below 2^62. The plain
// load skips the atomic once a smaller rank is in (ranks only decrease; a stale read only
// costs the atomic).
__device__ __forceinline__ void ord_min(unsigned long long* f, unsigned long long rank) {
  if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > rank) atomicMin(f, rank);
}
__device__ __forceinline__ unsigned long long ord_rank(uint64_t trace_pos, uint32_t bfs, int k) {
  return (((unsigned long long)trace_pos + bfs) << 1) | (unsigned long long)k;
}

// Daily buckets (ITDependencies.aggregateLinks, ITDependencies.java:666-700): a trace's day
// is flooredTraceTimestamp's, restated literally over its spans in storage order: the first
// span with a timestamp sets m = midnightUTC(ts / 1000) (Java long division, then
// DateUtil.midnightUTC's floor, DateUtil.java:27-35); a later one replaces it only if its
// microseconds compare below m's milliseconds (the reference's unit mix; never for real
// clocks). INT64_MAX: no timestamp (the reference's assertion fails).
constexpr int64_t DAY_MS = 86400000ll;
__device__ __forceinline__ int64_t midnight_utc(int64_t ms) {
  const int64_t q = ms / DAY_MS;
  return (q - ((ms % DAY_MS) < 0 ? 1 : 0)) * DAY_MS;
}
__device__ __forceinline__ int64_t floored_step(int64_t m, int64_t ts) {
  return (ts != 0 && ts < m) ? midnight_utc(ts / 1000) : m;
}

// QueryRequest.test's time rule over a trace in storage order (QueryRequest.java:262-279):
// the timestamp of the first span without a parent, else the smallest one.
__device__ __forceinline__ bool window_pass(int64_t ts, int64_t lo, int64_t hi) {
  return ts != 0 && ts >= lo && ts <= hi;
}

}  // namespace zdl
