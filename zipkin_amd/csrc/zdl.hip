// zdl.hip — MI355X (gfx950) kernels and the C ABI of libzdl.so.
//
// Pipeline for one zdl_put_spans over CSR-grouped traces:
//   k_link       persistent waves, each streams a contiguous chunk of traces: windows of
//                whole traces <= 64 spans, planned from the trace offsets, are linked in
//                registers + a small LDS hash; traces longer than WSMALL are listed;
//                (parent, child) counts accumulate in the workgroup's LDS table, added
//                to the S x S table by atomics when the workgroup ends
//   k_tail       one 1024-thread workgroup per CU: the windows k_link queued (fragments /
//                duplicate ids: full Trace.merge + SpanNode.Builder emulation, one wave
//                per window), then one workgroup per trace longer than WSMALL (HBM
//                scratch, bitonic sort), then the last workgroup compacts a small table
//                into mapped host memory
// zdl_link reads that (or compacts the non-zero cells itself: k_compact_ordered /
// k_compact) and sorts by service rank when ranks are set.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <rccl/rccl.h>

#include "zdl_group.h"
#include "zdl_store_index.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zdl.h"
#include "zdl_algo.h"
#include "zdl_sparse.h"
#include "zdl_xplan.h"
#include "zdl_shard.h"

namespace zdl {

constexpr int BIG_WG = 1024;        // threads per big-trace workgroup
constexpr int HCAP = 2048;          // LDS hash slots of the (parent, child) table when S*S is large
constexpr int HPROBE = 4;   // LDS hash probes before an add goes straight to HBM
constexpr int WSMALL = 64;          // traces up to this many spans are k_link's
constexpr uint32_t ORD_RANK_ONLY = 1u << 15;  // Args::skip: wave_link ranks addLinks, counts nothing
constexpr int TAIL_WG = 1024;       // threads per k_tail workgroup (= BIG_WG)
constexpr int WDENSE_MAX = 4544;    // S*S <= this -> dense u64 LDS cells (call | err << 32): S <= 67
constexpr int WTABLE_BYTES = 36864; // max(8 * (WDENSE_MAX + 64 dummy cells), 12 * HCAP); two k_link
                                    // workgroups (table + 16 wave carves) fill a CU's 160 KB
static_assert(8 * (WDENSE_MAX + 64) <= WTABLE_BYTES && 12 * HCAP <= WTABLE_BYTES, "LDS table carve");
// k_link with a time window carries 512 B more per wave (per-trace minima): its table stays at
// the round-1 size so that the workgroups still share a CU
constexpr int WDENSE_MAX_WINDOW = 2560;
constexpr int WTABLE_BYTES_WINDOW = 24576;
static_assert(8 * (WDENSE_MAX_WINDOW + 64) <= WTABLE_BYTES_WINDOW && 12 * HCAP <= WTABLE_BYTES_WINDOW, "LDS table carve");
constexpr int wdense_max(int window) { return window ? WDENSE_MAX_WINDOW : WDENSE_MAX; }
constexpr int wtable_bytes(int window) { return window ? WTABLE_BYTES_WINDOW : WTABLE_BYTES; }
// LOG mode (WDENSE_MAX < S*S <= PMAX << PSHIFT, e.g. C3's 500 services): k_link appends every
// link to a per-wave log in HBM and counts it per partition of 2^PSHIFT cells; k_pscan /
// k_scatter2 group the log by partition, k_hist2 counts each partition in dense LDS tables.
constexpr int PSHIFT = 12;          // cells per partition: 4096 u32 call + error cells in k_hist2
constexpr int PMAX = 256;           // partitions (k_link's LDS counters per row): S <= 1024
constexpr uint32_t LBLK = 1024;     // entries per block of LOG mode's block pool
// Rows (round 5): k_link's waves count their log entries per partition in one LDS counter
// array per row of ZDL_LOG_ROW_WAVES waves (round 6: shared by the row's waves, which leaves
// the hot corner 12-14 KB more), k_scatter2 takes one row's segments in order - so a
// partition's entries of consecutive segments land in ONE contiguous run - and k_hist2 runs
// one 1024-thread workgroup per CU (fewer flushes of each partition's cells).
constexpr int ZDL_LOG_ROW_WAVES = 4;  // a divisor of 12 and 16
// k_link's table modes (template parameter DENSE): hash, dense, log
constexpr int TM_HASH = 0, TM_DENSE = 1, TM_LOG = 2;
// SORT (sparse contexts, zdl_sparse.h): k_link logs every link like LOG, without partition
// counts; the put's log is sorted and merged into the context's sorted link list
constexpr int TM_SORT = 3;

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

struct Args {
  Cols c;
  const uint64_t* n_traces_dev;  // device-side trace count (grouped on the device), else null
  const uint64_t* off;
  uint64_t n_traces;
  uint64_t n_spans;
  Ranks R;
  uint32_t S;
  int dense;
  int window;
  int64_t win_lo, win_hi;
  unsigned long long* call;
  unsigned long long* err;
  uint32_t* big_list;   // k_link -> k_tail: the traces longer than WSMALL
  uint32_t* big_count;
  uint32_t* status;
  uint32_t small_max;    // traces longer than this are k_tail's (big_one, wave_big)
  uint32_t* cx_count;
  unsigned long long* map;  // mapped pinned host buffer: k_tail's last workgroup writes the
                             // ordered link records there (S*S <= 8192), else nullptr
  uint32_t* done;            // k_tail workgroups finished (the last one compacts; resets it)
  unsigned long long* flag;  // mapped pinned: k_tail's last workgroup stores `seq` after the
  unsigned long long seq;    // records (system-scope release), so zdl_link can spin on it
  int lazy;                  // k_link's last workgroup compacts when nothing is left for k_mid /
                             // k_tail (which the put then does not launch), else stores seq | FLAG_TAIL
  unsigned long long* prof;  // ZDL_PROF=1: k_link phase cycles (12 counters)
  uint64_t* cx_win;      // k_link -> k_tail: (base | P << 48, starts mask) per window
  uint32_t cx_slots;     // cx_win holds a slot per trace (k_link mode 3), not a queue of cx_count
  uint32_t skip;         // timing-only ablation of k_link (ZDL_SKIP): 32 stream only, 64 fields,
                         // 128 +hash, 256 +parents, 512 +jumping, 2048 no table adds, 4096 cache-resident;
                         // k_tail insertion order: 8192 no breadth-first ranks, 16384 no ord_min;
                         // ORD_RANK_ONLY (zdl_ord.inc's pass): ranks without counts
  // big-trace scratch (HBM), indexed by global span index
  uint64_t* b_id;
  uint64_t* b_pid;
  int32_t* b_lsvc;
  int32_t* b_rsvc;
  int32_t* b_ip4;
  int32_t* b_ip6;
  uint32_t* b_pf;
  uint32_t* b_perm;
  int32_t* b_parent;
  uint8_t* b_live;
  uint8_t* b_haschild;
  int skip_simple;            // ZDL_BIG_EXACT=1 (tests): every big trace takes the exact path
  int32_t* b_nm;              // big_simple in HBM: nearest-kinded-ancestor pointers
  unsigned long long* b_hk;   // big_simple in HBM: 2 hash slots per span (keys, then two u32 values)
  uint32_t* b_hv;
  // insertion order (ZDL_FLAG_INSERTION_ORDER): first-addLink ranks per cell (ord_min),
  // the put-global position of this put's span 0, and big-trace breadth-first scratch
  unsigned long long* first;
  unsigned long long* ord_w;  // insertion order, mode 6: per cell the put's first simple trace
                              // adding it, (start << 8 | length), put-relative (zdl_ord.inc)
  unsigned long long* ord_log;  // ... each wave's records (cell << 40 | start << 8 | length),
  uint64_t* ord_start;          // its segment's start in ord_log and its record count
  uint32_t* ord_cnt;
  uint64_t ord_stride;          // segments at wave * ord_stride (0: at 2 x the chunk's first span)
  uint64_t span_base;
  // daily buckets (zdl_set_days): rows = days * S (else S), day 0 = midnight day0 (ms);
  // day_first[d] = put-global position of day d's first trace
  uint32_t rows;
  uint32_t days;
  uint32_t days_skip;  // ZDL_DAYS_SKIP_OUTSIDE: a trace outside the days is skipped, not an error
  int64_t day0;
  unsigned long long* day_first;
  unsigned long long* o_key;
  uint32_t* o_fa;
  uint32_t* o_fb;
  uint32_t* o_bfs;
  uint32_t* o_pay;  // big_bfs's payload for traces of 2^21 - 1 spans and more (null when none)
  // LOG / SORT modes: wave gw's log segment starts at lg + lg_start[gw] (= 2 * its first span)
  // and holds lg_n[gw] entries (cell << 1 | error); lg_P partitions (cell >> PSHIFT), lg_W =
  // k_link's waves. LOG mode's block pool (round 6, zdl_log.inc): every k_link workgroup
  // reserves, per partition p it logged into, ceil(c_p / LBLK) consecutive blocks of lg_pool
  // (lg_set[PMAX]: the pool cursor) and as many places in p's directory (lg_dir[p * lg_bcap +
  // r], lg_set[p]: p's blocks so far), and moves its waves' entries there itself; lg_bn[b] =
  // block b's entries, lg_set[PMAX + 1] = the put's entries
  uint32_t* lg;
  uint64_t* lg_start;
  uint32_t* lg_n;
  uint32_t* lg_pool;
  uint32_t* lg_dir;
  uint32_t* lg_bn;
  uint32_t* lg_set;
  uint32_t lg_bcap;
  uint32_t lg_P, lg_W;
  // ZDL_FLAG_TREE_EXPORT (insertion-order contexts): per span of the put, its node's head
  // slot, its parent's head slot (-1 synthetic root, -2 root, -3 no node) and BFS index
  int32_t* tr_node;
  int32_t* tr_parent;
  int32_t* tr_bfs;
  uint8_t* tr_reason;  // zdl_tree_reasons
  int32_t* tr_anc;
  int32_t* tr_link;
  int32_t* tr_sorted;
  // sparse contexts (zdl_sparse.h): k_tail's links go to log segments in tlg (2 entries per
  // span: at 2 * the trace's / window's first span); tseg_big[bi] / tseg_win[k] = their counts
  int sparse;
  uint32_t* tlg;
  uint32_t* tseg_big;
  uint32_t* tseg_win;
  // k_tail's big traces: k_link lists those of at most wb_max spans (wave_big: one wave each)
  // from the front of big_list (big_count), the others from its back (big_list[big_cap - 1 - j],
  // large_count: one workgroup each); k_tail takes them by tickets, the workgroup ones first.
  // A wave_big trace that is not simple is retried by k_tail's last workgroup (retry list).
  uint32_t wb_max;
  uint32_t big_cap;
  uint32_t* large_count;
  uint32_t* tick_large;
  uint32_t* tick_mid;
  uint32_t* retry_count;
  uint32_t* retry;
  uint32_t* ctr_next;  // the next put's counter block, zeroed by this put's k_tail (CTR_* slots)
  // the device-wide big-trace tier (zdl_giant.inc): per back-list index, 1 = linked there,
  // 2 = k_tail's exact path, 0 = k_tail as usual; null when the tier did not run
  const uint8_t* gstat;
  const uint32_t* grest;    // and then the back-list indexes k_tail links instead of the whole back
  const uint32_t* grest_n;  // list (the giant ones dropped; the ones the tier rejected appended)
  uint8_t* bstat;           // k_big's verdict per back-list index (1 linked, 2 exact path), or null
  uint32_t* exact;          // with bstat: the back-list indexes k_big left to k_tail's exact path,
  uint32_t* exact_n;        // appended as found (k_tail walks this list, not the whole back list)
  uint32_t* tick_big;       // k_big's trace tickets
  uint32_t kb_small;        // k_big<256> takes the traces of at most this many spans (<= KB_SMALL)
};
// The counter block of one put (two alternate by put, so no put issues a memset)
enum : int { CTR_MID = 0, CTR_CX = 1, CTR_LARGE = 2, CTR_TICK_LARGE = 3, CTR_TICK_MID = 4, CTR_RETRY = 5,
             CTR_TICK_BIG = 6, CTR_EXACT = 8, CTR_N = 10 };  // (CTR_TICK_BIG + 1: k_big<256>'s tickets)
constexpr int CTR_DONE = 2 * CTR_N;  // k_tail's finished-workgroup count (after both blocks)

#include "zdl_full.inc"  // the full per-window emulation (k_tail's first part)
constexpr unsigned long long FLAG_TAIL = 1ull << 62;  // lazy put: k_mid / k_tail still have work
__device__ void lk_lazy_end(const Args& A, uint32_t* scratch);  // k_link's end in a lazy put (below)
__device__ void lk_lazy_end_log(const Args& A, uint32_t* scratch);  // ... of a LOG-mode put
#include "zdl_link.inc"  // k_link, full_windows (need zdl_full.inc's helpers)
#include "zdl_log.inc"   // LOG mode reduce: k_pscan, k_pbase, k_scatter2, k_hist2

// ---------------------------------------------------------- big traces (k_tail)
// k_tail's second part: one workgroup per trace longer than WSMALL; arrays live in HBM
// scratch at the trace's global span offset. zdl_algo.h's phases, bitonic sort instead of
// ranks.
__device__ __forceinline__ void big_sync() { __syncthreads(); }

// Exclusive scan of one value per thread over the workgroup (BIG_WG threads); *total gets
// the sum. Every thread must call.
__device__ __forceinline__ uint32_t big_scan(uint32_t x, uint32_t* total) {
  __shared__ uint32_t ws[BIG_WG / 64 + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) ws[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < BIG_WG / 64; ++i) {
      const uint32_t t = ws[i];
      ws[i] = acc;
      acc += t;
    }
    ws[BIG_WG / 64] = acc;
  }
  __syncthreads();
  const uint32_t r = ws[w] + incl - x;
  *total = ws[BIG_WG / 64];
  __syncthreads();
  return r;
}

// First position >= `from` whose sorted key is >= k (keys ascending over [0, n)).
__device__ __forceinline__ uint32_t big_lower(const unsigned long long* key, uint32_t n, unsigned long long k) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (key[mid] < k) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Insertion order for one big trace: the breadth-first index of every node reachable
// from the root (SpanNode.traverse, SpanNode.java:64-89) into bfs[]. Children lists are the
// nodes sorted by (parent, spanToParent entry position) - see wave_bfs for the entry
// rule; the synthetic root is position n. Then level by level: a frontier in
// breadth-first order, each node's children appended at a scanned offset.
// Sort keys: (parent, entry, node) in 21 bits each while n < 2^21 - 1; a longer trace sorts
// (parent << 32 | entry) keys with the node as a payload in pay[] (a live node's (parent,
// entry) is unique, so the payload needs no ordering of its own).
__device__ __forceinline__ void big_bfs(const View& v, int n, int rp, unsigned long long* key, uint32_t* fa,
                                        uint32_t* fb, uint32_t* bfs, uint32_t* pay) {
  constexpr unsigned long long M21 = (1ull << 21) - 1;
  const bool wide = n >= (1 << 21) - 1;
  const int psh = wide ? 32 : 42;
  for (int p = threadIdx.x; p < n; p += BIG_WG) {
    unsigned long long k = ~0ull;
    const int par = v.parent[p];
    if (v.live[p] && par != PAR_NONMEMBER) {
      const uint32_t s = v.perm[p];
      const uint64_t my = v.id[s];
      int gb = p;
      while (gb > 0 && v.id[v.perm[gb - 1]] == my) --gb;
      int ge = p + 1;
      while (ge < n && v.id[v.perm[ge]] == my) ++ge;
      int ek = p;
      if (is_shared(v.pf[s])) {
        for (int q = gb; q < p; ++q)
          if (v.live[q] && is_shared(v.pf[v.perm[q]]) && local_eq(v, v.perm[q], s)) { ek = q; break; }
      } else if (rp >= gb && rp < ge) {
        ek = n;
      } else {
        for (int q = gb; q < p; ++q)
          if (v.live[q] && !is_shared(v.pf[v.perm[q]])) { ek = q; break; }
      }
      const unsigned long long pp = par >= 0 ? (unsigned long long)par : (unsigned long long)n;
      k = wide ? (pp << 32) | (unsigned long long)ek : (pp << 42) | ((unsigned long long)ek << 21) | (unsigned long long)p;
    }
    key[p] = k;
    if (wide) pay[p] = (uint32_t)p;
  }
  big_sync();
  int npad = 1;
  while (npad < n) npad <<= 1;
  for (int kk = 2; kk <= npad; kk <<= 1) {  // ascending bitonic (any n: absent partners are +inf)
    for (int jj = kk - 1; jj > 0; jj = (jj == kk - 1 ? kk >> 2 : jj >> 1)) {
      for (int i = threadIdx.x; i < n; i += BIG_WG) {
        const int l = i ^ jj;
        if (l > i && l < n) {
          const unsigned long long a = key[i], b = key[l];
          if (b < a) {
            key[i] = b;
            key[l] = a;
            if (wide) {
              const uint32_t t = pay[i];
              pay[i] = pay[l];
              pay[l] = t;
            }
          }
        }
      }
      big_sync();
    }
  }
  __shared__ uint32_t sh_f;
  if (threadIdx.x == 0) {
    fa[0] = rp >= 0 ? (uint32_t)rp : (uint32_t)n;
    if (rp >= 0) bfs[rp] = 0;
    sh_f = 1;
  }
  big_sync();
  uint32_t fsz = sh_f, next = rp >= 0 ? 1u : 0u;
  while (fsz != 0) {
    uint32_t gsz = 0;
    for (uint32_t i0 = 0; i0 < fsz; i0 += BIG_WG) {
      const uint32_t i = i0 + threadIdx.x;
      uint32_t lo = 0, cnt = 0;
      if (i < fsz) {
        const unsigned long long u = fa[i];
        lo = big_lower(key, (uint32_t)n, u << psh);
        cnt = big_lower(key, (uint32_t)n, (u + 1) << psh) - lo;
      }
      uint32_t tot;
      const uint32_t o = gsz + big_scan(cnt, &tot);
      for (uint32_t j = 0; j < cnt; ++j) {
        const uint32_t node = wide ? pay[lo + j] : (uint32_t)(key[lo + j] & M21);
        fb[o + j] = node;
        bfs[node] = next + o + j;
      }
      gsz += tot;
    }
    big_sync();
    next += gsz;
    fsz = gsz;
    uint32_t* t = fa;
    fa = fb;
    fb = t;
  }
}

// ------------------------------------------------- big traces, simple ids (k_tail)
// A trace longer than WSMALL whose ids are "simple" (per id at most one non-shared and one
// shared span, the condition under which k_link's windows skip Trace.merge) is linked without
// sorting: k_link's algorithm at workgroup scale, every phase one parallel loop and a barrier.
//   1. (id) -> {non-shared, shared} index in a hash of exact 64-bit keys (2n slots, CAS);
//      a second span with the same (id, shared) aborts to the exact (sorting) path;
//   2. root = the non-shared parentless span with the smallest id (SpanNode.java:203-249 via
//      DESIGN.md §3); tree parents by lookup of the parent id, the shared candidate first when
//      its endpoint equals (SpanNode.Builder.process); Trace.merge's backfill of a shared span's
//      parent id (Trace.java:76-79);
//   3. reachability and firstRemoteAncestor (DependencyLinker.java:153-164) by pointer jumping
//      (O(log depth) rounds; a cycle never reaches the root, as in SpanNode.traverse);
//   4. DependencyLinker.java:58-148 per node, straight into the global tables.
// The arrays live in the workgroup's LDS when the trace fits, else in HBM scratch at the
// trace's span offset. Returns false (nothing counted) when the trace is not simple.
struct BSView {
  uint64_t* id;
  uint64_t* pid;
  int32_t* ls;
  int32_t* rs;
  int32_t* i4;
  int32_t* i6;
  uint32_t* pf;
  int32_t* par;
  int32_t* a;
  int32_t* nm;
  unsigned long long* hk;
  uint32_t* hns;
  uint32_t* hsh;
  uint8_t* hasc;
};
constexpr size_t bs_bytes(int n) { return (size_t)n * (8 + 8 + 4 * 5 + 4 * 3 + 1) + (size_t)2 * n * (8 + 4 + 4) + 16 * 15; }  // + alignment of 14 arrays

__device__ __forceinline__ int bs_slot(uint64_t key, int n) {
  const uint32_t h = ((uint32_t)key ^ (uint32_t)(key >> 32)) * 0x9E3779B1u;
  return (int)__umulhi(h, 2u * (uint32_t)n);
}
// The slot holding key (or the empty slot where it would go).
__device__ __forceinline__ int bs_find(const BSView& v, uint64_t key, int n) {
  int q = bs_slot(key, n);
  while (true) {
    const unsigned long long k = v.hk[q];
    if (k == key || k == 0ull) return q;
    q = q + 1 == 2 * n ? 0 : q + 1;
  }
}

template <int NT = BIG_WG>  // threads of the workgroup
__device__ __forceinline__ bool big_simple(const Args& A, unsigned char* lds, size_t lds_bytes, uint64_t b, int n, uint32_t day,
                           uint32_t* scnt) {
  __shared__ int sh_bad, sh_more[3];
  __shared__ unsigned long long sh_rootid;
  __shared__ int sh_rp;
  BSView v;
  if (bs_bytes(n) <= lds_bytes) {  // LDS
    unsigned char* p = lds;
    auto take = [&](size_t bytes) { unsigned char* r = p; p += (bytes + 15) & ~(size_t)15; return r; };
    v.hk = (unsigned long long*)take((size_t)16 * n);
    v.id = (uint64_t*)take((size_t)8 * n);
    v.pid = (uint64_t*)take((size_t)8 * n);
    v.hns = (uint32_t*)take((size_t)8 * n);
    v.hsh = (uint32_t*)take((size_t)8 * n);
    v.ls = (int32_t*)take((size_t)4 * n);
    v.rs = (int32_t*)take((size_t)4 * n);
    v.i4 = (int32_t*)take((size_t)4 * n);
    v.i6 = (int32_t*)take((size_t)4 * n);
    v.pf = (uint32_t*)take((size_t)4 * n);
    v.par = (int32_t*)take((size_t)4 * n);
    v.a = (int32_t*)take((size_t)4 * n);
    v.nm = (int32_t*)take((size_t)4 * n);
    v.hasc = (uint8_t*)take((size_t)n);
  } else {  // HBM scratch at the trace's span offset (2 hash slots per span)
    v.id = A.b_id + b;
    v.pid = A.b_pid + b;
    v.ls = A.b_lsvc + b;
    v.rs = A.b_rsvc + b;
    v.i4 = A.b_ip4 + b;
    v.i6 = A.b_ip6 + b;
    v.pf = A.b_pf + b;
    v.par = A.b_parent + b;
    v.a = (int32_t*)(A.b_perm + b);
    v.nm = A.b_nm + b;
    v.hasc = A.b_haschild + b;
    v.hk = A.b_hk + 2 * b;
    v.hns = A.b_hv + 4 * b;
    v.hsh = A.b_hv + 4 * b + 2 * n;
  }
  if (threadIdx.x == 0) {
    sh_bad = 0;
    sh_rootid = ~0ull;
    sh_rp = PAR_TERMINAL;
  }
  for (int i = threadIdx.x; i < 2 * n; i += NT) {
    v.hk[i] = 0ull;
    v.hns[i] = 0u;
    v.hsh[i] = 0u;
  }
  for (int i = threadIdx.x; i < n; i += NT) {
    const uint64_t g = b + i;
    const uint64_t id = A.c.id[g];
    const uint64_t pid = A.c.pid[g];
    v.id[i] = id;
    v.pid[i] = pid == id ? 0 : pid;  // Span.build drops a self parent (Span.java:611-617)
    v.ls[i] = A.c.lsvc[g];
    v.rs[i] = A.c.rsvc[g];
    v.i4[i] = A.c.ip4[g];
    v.i6[i] = A.c.ip6[g];
    v.pf[i] = A.c.pf[g];
    v.hasc[i] = 0;
  }
  __syncthreads();
  // 1. the id hash; a second span with one (id, shared) -> not simple
  for (int i = threadIdx.x; i < n; i += NT) {
    const uint64_t id = v.id[i];
    int q = bs_slot(id, n);
    while (true) {
      const unsigned long long old = atomicCAS(&v.hk[q], 0ull, (unsigned long long)id);
      if (old == 0ull || old == id) break;
      q = q + 1 == 2 * n ? 0 : q + 1;
    }
    const bool sh = is_shared(v.pf[i]);
    if (atomicCAS(sh ? &v.hsh[q] : &v.hns[q], 0u, (uint32_t)i + 1u) != 0u) sh_bad = 1;
    if ((uint32_t)v.ls[i] >= A.S && v.ls[i] >= 0) sh_bad = 2;
    if ((uint32_t)v.rs[i] >= A.S && v.rs[i] >= 0) sh_bad = 2;
    if (!sh && v.pid[i] == 0) atomicMin(&sh_rootid, (unsigned long long)id);
  }
  __syncthreads();
  if (sh_bad == 2 && threadIdx.x == 0) atomicOr(A.status, ST_BADSVC);
  if (sh_bad) {
    __syncthreads();
    return sh_bad == 2;  // bad service ids: counted nowhere, the put fails
  }
  if (threadIdx.x == 0 && sh_rootid != ~0ull) sh_rp = (int)v.hns[bs_find(v, sh_rootid, n)] - 1;
  __syncthreads();
  const int rp = sh_rp, root_attach = rp >= 0 ? rp : PAR_TERMINAL;
  // 2. tree parents (+ the shared spans' parent-id backfill) and has-children
  for (int i = threadIdx.x; i < n; i += NT) {
    const uint32_t pf = v.pf[i];
    int par;
    if (is_shared(pf)) {
      const int ns_own = (int)v.hns[bs_find(v, v.id[i], n)] - 1;
      par = ns_own >= 0 ? ns_own : root_attach;
      if (ns_own >= 0 && v.pid[i] == 0) v.pid[i] = v.pid[ns_own];  // Trace.java:76-79 (only shared pids change)
    } else if (i == rp) {
      par = PAR_TERMINAL;
    } else if (v.pid[i] != 0) {
      const uint64_t P = v.pid[i];
      const int q = bs_find(v, P, n);
      int nss = -1, shs = -1;
      if (v.hk[q] == P) {
        nss = (int)v.hns[q] - 1;
        shs = (int)v.hsh[q] - 1;
      }
      const bool same_ep = shs >= 0 && v.ls[shs] == v.ls[i] && v.i4[shs] == v.i4[i] && v.i6[shs] == v.i6[i] &&
                           port_of(v.pf[shs]) == port_of(pf);
      par = same_ep ? shs : (nss >= 0 ? nss : root_attach);
    } else {
      par = root_attach;
    }
    v.par[i] = par;
    v.a[i] = par;
    v.nm[i] = par;
    if (par >= 0) v.hasc[par] = 1;
    if (A.tr_parent) {  // ZDL_FLAG_TREE_STREAM
      A.tr_node[b + i] = (int32_t)(b + i);
      A.tr_parent[b + i] = i == rp ? -2 : (par >= 0 ? (int32_t)(b + par) : -1);
    }
  }
  __syncthreads();
  // 3. pointer jumping: a -> PAR_TERMINAL iff reachable, nm -> nearest ancestor with a kind
  // Round r's "anything moved" flag is sh_more[r % 3], cleared by thread 0 in round r - 1 before
  // that round's barrier (so before any round-r writer) and after every reader of round r - 3
  // has passed round r - 2's barrier. (One flag cleared at the top of each round let a fast
  // wave clear it while a slow one had still to read the previous round's value: the slow
  // wave left the loop early, the barriers paired up across phases and traces, and LDS was
  // overwritten under it - garbage cells or a faulting access once four workgroups shared a CU.)
  int rounds = 4;
  for (int m = n; m > 1; m >>= 1) rounds += 2;
  if (threadIdx.x == 0) sh_more[0] = 0;
  __syncthreads();
  for (int r = 0; r < rounds; ++r) {
    if (threadIdx.x == 0) sh_more[(r + 1) % 3] = 0;
    bool more = false;
    for (int i = threadIdx.x; i < n; i += NT) {
      const int x = v.a[i];
      if (x >= 0) {
        v.a[i] = v.a[x];
        more = true;
      }
      const int y = v.nm[i];
      if (y >= 0 && kind_of(v.pf[y]) == ZDL_KIND_NULL) {
        v.nm[i] = v.nm[y];
        more = true;
      }
    }
    if (more) sh_more[r % 3] = 1;
    __syncthreads();
    if (!sh_more[r % 3]) break;
  }
  if (A.tr_parent)
    for (int i = threadIdx.x; i < n; i += NT) {
      const bool rch = v.a[i] == PAR_TERMINAL;
      A.tr_bfs[b + i] = rch ? 0 : -1;
      A.tr_anc[b + i] = rch && v.nm[i] >= 0 ? (int32_t)(b + v.nm[i]) : -1;
    }
  // 4. DependencyLinker's rules per node (every span of a simple trace is a node)
  for (int i = threadIdx.x; i < n; i += NT) {
    if (v.a[i] != PAR_TERMINAL) continue;  // unreachable (a cycle not through the root)
    const uint32_t pf = v.pf[i];
    const uint32_t kind0 = kind_of(pf);
    if (kind0 == ZDL_KIND_CLIENT && v.hasc[i]) continue;
    const int32_t svc = v.ls[i], rsvc = v.rs[i];
    uint32_t kind = kind0;
    if (kind == ZDL_KIND_NULL) {
      if (svc >= 0 && rsvc >= 0) kind = ZDL_KIND_CLIENT; else continue;
    }
    const bool srv = kind == ZDL_KIND_SERVER || kind == ZDL_KIND_CONSUMER;
    int32_t pa = srv ? rsvc : svc;
    const int32_t ch = srv ? svc : rsvc;
    if (srv && i == rp && pa < 0) continue;
    bool err = err_of(pf);
    auto emit = [&](int32_t x, int32_t y, bool e) {
      const size_t idx = ((size_t)day * A.S + (size_t)x) * A.S + y;
      if (A.sparse) {  // the trace's log segment
        A.tlg[2 * b + atomicAdd(scnt, 1u)] = ((uint32_t)idx << 1) | (e ? 1u : 0u);
        return;
      }
      atomicAdd(&A.call[idx], 1ull);
      if (e) atomicAdd(&A.err[idx], 1ull);
    };
    if (kind == ZDL_KIND_PRODUCER || kind == ZDL_KIND_CONSUMER) {
      if (pa >= 0 && ch >= 0) emit(pa, ch, err);
      continue;
    }
    const int ra = v.nm[i];
    if (ra >= 0) {
      const int32_t ran = v.ls[ra];
      if (ran >= 0) {
        if (kind == ZDL_KIND_CLIENT && svc >= 0 && ran != svc) emit(ran, svc, false);
        if (kind == ZDL_KIND_SERVER || pa < 0) pa = ran;
        const uint32_t apf = v.pf[ra];
        if (!err && kind_of(apf) == ZDL_KIND_CLIENT && v.pid[i] != 0 && v.pid[i] == v.id[ra]) err = err_of(apf);
      }
    }
    if (pa >= 0 && ch >= 0) emit(pa, ch, err);
  }
  __syncthreads();
  return true;
}

// ---------------------------------------------------------------- wave_big
// Traces of WSMALL < n <= WB_MAX spans with simple ids, one wave each: big_simple's algorithm
// at wave scale (wave_sync instead of workgroup barriers), so a CU links 16 such traces at
// once instead of one. Lane l owns spans l, l + 64, ... (at most WB_K). The wave's LDS carve
// holds id, parent id, services, local endpoint and flags, the id hash (2 slots per span: u32
// words of non-shared | shared span index + 1, keys compared through the id array), the
// pointer-jumping arrays (i16) and has-children bytes: 49 B per span.
constexpr int WB_CARVE = 9600;              // bytes per wave (16 waves: 150 KB of k_tail's LDS)
constexpr int WB_SCR = WB_CARVE - 32;       // 4 u64 scratch words: root id, window index / min, count
constexpr int WB_MAX = 192;
constexpr int WB_K = (WB_MAX + 63) / 64;
static_assert(49 * WB_MAX <= WB_SCR && WB_MAX % 8 == 0 && WB_MAX < 32767, "wave_big carve");
struct WBv {
  uint64_t* id;
  uint64_t* pid;
  int32_t* ls;
  int32_t* rs;
  int32_t* i4;
  int32_t* i6;
  uint32_t* pf;
  uint32_t* slot;
  int16_t* a;
  int16_t* nm;
  uint8_t* hasc;
};
__device__ __forceinline__ WBv wb_view(unsigned char* p, int n) {
  const int m = (n + 7) & ~7;
  WBv v;
  v.id = reinterpret_cast<uint64_t*>(p);
  v.pid = v.id + m;
  v.ls = reinterpret_cast<int32_t*>(v.pid + m);
  v.rs = v.ls + m;
  v.i4 = v.rs + m;
  v.i6 = v.i4 + m;
  v.pf = reinterpret_cast<uint32_t*>(v.i6 + m);
  v.slot = v.pf + m;
  v.a = reinterpret_cast<int16_t*>(v.slot + 2 * m);
  v.nm = v.a + m;
  v.hasc = reinterpret_cast<uint8_t*>(v.nm + m);
  return v;
}
__device__ __forceinline__ int wb_home(uint64_t key, int H) {
  const uint32_t h = ((uint32_t)key ^ (uint32_t)(key >> 32)) * 0x9E3779B1u;
  return (int)__umulhi(h, (uint32_t)H);
}
__device__ __forceinline__ uint32_t wb_word_idx(uint32_t w) { return ((w & 0xFFFFu) ? (w & 0xFFFFu) : (w >> 16)) - 1u; }
// The slot word of key (0 if absent)
__device__ __forceinline__ uint32_t wb_find(const WBv& v, uint64_t key, int H) {
  int q = wb_home(key, H);
  while (true) {
    const uint32_t w = v.slot[q];
    if (w == 0u || v.id[wb_word_idx(w)] == key) return w;
    q = q + 1 == H ? 0 : q + 1;
  }
}

// Links trace big_list[bi] (n <= WB_MAX spans) with the calling wave (every lane calls).
// Returns false when its ids are not simple: nothing was counted, the caller retries it on the
// exact path. A bad service id fails the put like big_simple; a trace outside the time window
// counts nothing (big_one's rule: its first parentless timestamp, else its minimum).
__device__ __forceinline__ bool wave_big(const Args& A, unsigned char* p, uint32_t bi, int lane) {
  const uint32_t t = A.big_list[bi];
  const uint64_t b = A.off[t], e = A.off[t + 1];
  if (e < b || e > A.n_spans || e - b > (uint64_t)WB_MAX) {  // k_link flagged it
    if (A.sparse && lane == 0) A.tseg_big[bi] = 0;
    return true;
  }
  const int n = (int)(e - b), H = 2 * ((n + 7) & ~7);
  const WBv v = wb_view(p, n);
  unsigned long long* scr = reinterpret_cast<unsigned long long*>(p + WB_SCR);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(scr + 3);
  if (lane < 3) scr[lane] = ~0ull;
  if (lane == 3) scr[3] = 0ull;
  for (int q = lane; q < H; q += 64) v.slot[q] = 0u;
  bool bad = false;
  // the spans into the carve (every column's loads first: one round trip for the trace)
  uint64_t id[WB_K], pid[WB_K];
  int32_t ls[WB_K], rs[WB_K], i4[WB_K], i6[WB_K];
  uint32_t pf[WB_K];
#pragma unroll
  for (int k = 0; k < WB_K; ++k) {
    const int i = lane + 64 * k;
    if (i >= n) continue;
    const uint64_t g = b + i;
    id[k] = A.c.id[g];
    pid[k] = A.c.pid[g];
    ls[k] = A.c.lsvc[g];
    rs[k] = A.c.rsvc[g];
    i4[k] = A.c.ip4[g];
    i6[k] = A.c.ip6[g];
    pf[k] = A.c.pf[g];
  }
#pragma unroll
  for (int k = 0; k < WB_K; ++k) {
    const int i = lane + 64 * k;
    if (i >= n) continue;
    v.id[i] = id[k];
    v.pid[i] = pid[k] == id[k] ? 0 : pid[k];  // Span.build drops a self parent (Span.java:611-617)
    v.ls[i] = ls[k];
    v.rs[i] = rs[k];
    v.i4[i] = i4[k];
    v.i6[i] = i6[k];
    v.pf[i] = pf[k];
    v.hasc[i] = 0;
    bad |= ((uint32_t)ls[k] >= A.S && ls[k] >= 0) || ((uint32_t)rs[k] >= A.S && rs[k] >= 0);
  }
  wave_sync();
  if (A.window) {
#pragma unroll
    for (int k = 0; k < WB_K; ++k) {
      const int i = lane + 64 * k;
      if (i >= n) continue;
      const int64_t x = A.c.ts[b + i];
      if (x == 0) continue;
      if (v.pid[i] == 0) atomicMin(&scr[1], (unsigned long long)i);
      atomicMin(&scr[2], (unsigned long long)x);
    }
    wave_sync();
    const unsigned long long fi = scr[1], mn = scr[2];
    const int64_t ts = fi != ~0ull ? A.c.ts[b + fi] : (mn == ~0ull ? 0 : (int64_t)mn);
    if (!window_pass(ts, A.win_lo, A.win_hi)) {
      if (A.sparse && lane == 0) A.tseg_big[bi] = 0;
      return true;
    }
  }
  if (ballot(bad)) {  // counted nowhere: the put fails
    if (lane == 0) {
      atomicOr(A.status, ST_BADSVC);
      if (A.sparse) A.tseg_big[bi] = 0;
    }
    return true;
  }
  // 1. the id hash; a second span with one (id, shared) -> not simple
  bool dup = false;
#pragma unroll
  for (int k = 0; k < WB_K; ++k) {
    const int i = lane + 64 * k;
    if (i >= n) continue;
    const uint64_t my = v.id[i];
    const bool sh = is_shared(v.pf[i]);
    const uint32_t mine = sh ? (uint32_t)(i + 1) << 16 : (uint32_t)(i + 1);
    int q = wb_home(my, H);
    while (true) {
      uint32_t w = v.slot[q];
      if (w == 0u) {
        w = atomicCAS(&v.slot[q], 0u, mine);
        if (w == 0u) break;
      }
      if (v.id[wb_word_idx(w)] == my) {
        dup |= (atomicOr(&v.slot[q], mine) & (sh ? 0xFFFF0000u : 0xFFFFu)) != 0u;
        break;
      }
      q = q + 1 == H ? 0 : q + 1;
    }
    if (!sh && v.pid[i] == 0) atomicMin(&scr[0], (unsigned long long)my);
  }
  wave_sync();
  if (ballot(dup)) return false;
  const unsigned long long rootid = scr[0];
  const int rp = rootid != ~0ull ? (int)(wb_find(v, rootid, H) & 0xFFFFu) - 1 : -1;
  const int root_attach = rp >= 0 ? rp : PAR_TERMINAL;
  // 2. tree parents (+ the shared spans' parent-id backfill, Trace.java:76-79: only shared
  // spans' entries change, and only their own lane reads them again) and has-children
#pragma unroll
  for (int k = 0; k < WB_K; ++k) {
    const int i = lane + 64 * k;
    if (i >= n) continue;
    const uint32_t pfi = v.pf[i];
    const uint64_t pidi = v.pid[i];
    int par;
    if (is_shared(pfi)) {
      const int ns_own = (int)(wb_find(v, v.id[i], H) & 0xFFFFu) - 1;
      par = ns_own >= 0 ? ns_own : root_attach;
      if (ns_own >= 0 && pidi == 0) v.pid[i] = v.pid[ns_own];
    } else if (i == rp) {
      par = PAR_TERMINAL;
    } else if (pidi != 0) {
      const uint32_t w = wb_find(v, pidi, H);
      const int nss = (int)(w & 0xFFFFu) - 1, shs = (int)(w >> 16) - 1;
      const bool same_ep = shs >= 0 && v.ls[shs] == v.ls[i] && v.i4[shs] == v.i4[i] && v.i6[shs] == v.i6[i] &&
                           port_of(v.pf[shs]) == port_of(pfi);
      par = same_ep ? shs : (nss >= 0 ? nss : root_attach);
    } else {
      par = root_attach;
    }
    v.a[i] = (int16_t)par;
    v.nm[i] = (int16_t)par;
    if (par >= 0) v.hasc[par] = 1;
    if (A.tr_parent) {  // ZDL_FLAG_TREE_STREAM
      A.tr_node[b + i] = (int32_t)(b + i);
      A.tr_parent[b + i] = i == rp ? -2 : (par >= 0 ? (int32_t)(b + par) : -1);
    }
  }
  wave_sync();
  // 3. pointer jumping: a -> PAR_TERMINAL iff reachable, nm -> nearest ancestor with a kind
  int rounds = 4;
  for (int m = n; m > 1; m >>= 1) rounds += 2;
  for (int r = 0; r < rounds; ++r) {
    bool more = false;
#pragma unroll
    for (int k = 0; k < WB_K; ++k) {
      const int i = lane + 64 * k;
      if (i >= n) continue;
      const int x = v.a[i];
      if (x >= 0) {
        v.a[i] = v.a[x];
        more = true;
      }
      const int y = v.nm[i];
      if (y >= 0 && kind_of(v.pf[y]) == ZDL_KIND_NULL) {
        v.nm[i] = v.nm[y];
        more = true;
      }
    }
    wave_sync();
    if (!ballot(more)) break;
  }
  if (A.tr_parent) {
#pragma unroll
    for (int k = 0; k < WB_K; ++k) {
      const int i = lane + 64 * k;
      if (i >= n) continue;
      const bool rch = v.a[i] == PAR_TERMINAL;
      A.tr_bfs[b + i] = rch ? 0 : -1;
      A.tr_anc[b + i] = rch && v.nm[i] >= 0 ? (int32_t)(b + v.nm[i]) : -1;
    }
  }
  // 4. DependencyLinker's rules per node (DependencyLinker.java:58-148)
  auto emit = [&](int32_t x, int32_t y, bool er) {
    const uint32_t idx = (uint32_t)x * A.S + (uint32_t)y;
    if (A.sparse) {  // the trace's log segment
      A.tlg[2 * b + atomicAdd(cnt, 1u)] = (idx << 1) | (er ? 1u : 0u);
      return;
    }
    atomicAdd(&A.call[idx], 1ull);
    if (er) atomicAdd(&A.err[idx], 1ull);
  };
#pragma unroll
  for (int k = 0; k < WB_K; ++k) {
    const int i = lane + 64 * k;
    if (i >= n || v.a[i] != PAR_TERMINAL) continue;  // unreachable: a cycle not through the root
    const uint32_t pfi = v.pf[i];
    const uint32_t kind0 = kind_of(pfi);
    if (kind0 == ZDL_KIND_CLIENT && v.hasc[i]) continue;
    const int32_t svc = v.ls[i], rsvc = v.rs[i];
    uint32_t kind = kind0;
    if (kind == ZDL_KIND_NULL) {
      if (svc >= 0 && rsvc >= 0) kind = ZDL_KIND_CLIENT; else continue;
    }
    const bool srv = kind == ZDL_KIND_SERVER || kind == ZDL_KIND_CONSUMER;
    int32_t pa = srv ? rsvc : svc;
    const int32_t ch = srv ? svc : rsvc;
    if (srv && i == rp && pa < 0) continue;
    bool er = err_of(pfi);
    if (kind == ZDL_KIND_PRODUCER || kind == ZDL_KIND_CONSUMER) {
      if (pa >= 0 && ch >= 0) emit(pa, ch, er);
      continue;
    }
    const int ra = v.nm[i];
    if (ra >= 0) {
      const int32_t ran = v.ls[ra];
      if (ran >= 0) {
        if (kind == ZDL_KIND_CLIENT && svc >= 0 && ran != svc) emit(ran, svc, false);
        if (kind == ZDL_KIND_SERVER || pa < 0) pa = ran;
        const uint32_t apf = v.pf[ra];
        const uint64_t pidi = v.pid[i];
        if (!er && kind_of(apf) == ZDL_KIND_CLIENT && pidi != 0 && pidi == v.id[ra]) er = err_of(apf);
      }
    }
    if (pa >= 0 && ch >= 0) emit(pa, ch, er);
  }
  wave_sync();
  if (A.sparse && lane == 0) A.tseg_big[bi] = *cnt;
  return true;
}

// k_mid, between k_link and k_tail: every wave takes front-list traces by ticket, WB_CHUNK per
// ticket (the next ticket fetched while the current ones are linked); a trace that is not
// simple goes to the retry list, which k_tail's workgroups take after the back list. A
// kernel of its own: wave_big's registers then never meet k_tail's (one kernel spilled both).
constexpr uint32_t WB_CHUNK = 8;
constexpr int MID_WG = 256;  // 4 waves: 4 workgroups (16 carves, 150 KB of LDS) per CU
__global__ void __launch_bounds__(MID_WG) k_mid(Args A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned char* p = lds + (size_t)w * WB_CARVE;
  const uint32_t nmid = *A.big_count;
  if (nmid == 0) return;  // no ticket traffic when there is nothing (every wave on one address)
  uint32_t c = 0;
  if (lane == 0) c = atomicAdd(A.tick_mid, 1u);
  c = __builtin_amdgcn_readfirstlane(c);
  while (c * WB_CHUNK < nmid) {
    uint32_t nx = 0;
    if (lane == 0) nx = atomicAdd(A.tick_mid, 1u);
    const uint32_t j1 = min(nmid, (c + 1) * WB_CHUNK);
    for (uint32_t j = c * WB_CHUNK; j < j1; ++j) {
      if (!wave_big(A, p, j, lane) && lane == 0)
        __hip_atomic_store(&A.retry[atomicAdd(A.retry_count, 1u)], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      wave_sync();  // the carve is reused
    }
    c = __builtin_amdgcn_readfirstlane(nx);
  }
}

// The exact path for one big trace (every thread of the workgroup calls): the spans copied to
// HBM scratch at the trace's offset, bitonic-sorted by Trace.merge's comparator, merged,
// the SpanNode tree and DependencyLinker's rules (zdl_algo.h). Runs for non-simple traces
// (and every big trace in insertion order) only.
template <int ORD>
__device__ __forceinline__ void big_exact(const Args& A, uint64_t b, int n, uint32_t day, uint32_t bi) {
  __shared__ uint32_t sh_cnt;  // sparse: links logged for the trace
  __shared__ int32_t sh_root;
  View v;
  v.id = A.b_id + b;
  v.pid = A.b_pid + b;
  v.lsvc = A.b_lsvc + b;
  v.rsvc = A.b_rsvc + b;
  v.ip4 = A.b_ip4 + b;
  v.ip6 = A.b_ip6 + b;
  v.pf = A.b_pf + b;
  v.perm = A.b_perm + b;
  v.parent = A.b_parent + b;
  v.live = A.b_live + b;
  v.haschild = A.b_haschild + b;
  if (threadIdx.x == 0) {
    sh_cnt = 0;
    sh_root = 0x7fffffff;
  }
  for (int s = threadIdx.x; s < n; s += BIG_WG) {
    const uint64_t g = b + s;
    const uint64_t id = A.c.id[g];
    uint64_t pid = A.c.pid[g];
    if (pid == id) pid = 0;  // Span.build drops a self parent (Span.java:611-617)
    v.id[s] = id;
    v.pid[s] = pid;
    v.lsvc[s] = A.c.lsvc[g];
    v.rsvc[s] = A.c.rsvc[g];
    v.ip4[s] = A.c.ip4[g];
    v.ip6[s] = A.c.ip6[g];
    v.pf[s] = A.c.pf[g];
    v.perm[s] = s;
    v.haschild[s] = 0;
  }
  big_sync();
  // bitonic sort of perm by span_less (any n: out-of-range partners are +inf)
  int npad = 1;
  while (npad < n) npad <<= 1;
  for (int kk = 2; kk <= npad; kk <<= 1) {
    for (int i = threadIdx.x; i < n; i += BIG_WG) {
      const int l = i ^ (kk - 1);
      if (l > i && l < n) {
        const uint32_t a = v.perm[i], c = v.perm[l];
        if (span_less(v, A.R, c, a)) { v.perm[i] = c; v.perm[l] = a; }
      }
    }
    big_sync();
    for (int jj = kk >> 2; jj > 0; jj >>= 1) {
      for (int i = threadIdx.x; i < n; i += BIG_WG) {
        const int l = i ^ jj;
        if (l > i && l < n) {
          const uint32_t a = v.perm[i], c = v.perm[l];
          if (span_less(v, A.R, c, a)) { v.perm[i] = c; v.perm[l] = a; }
        }
      }
      big_sync();
    }
  }
  bool npe = false;
  for (int p = threadIdx.x; p < n; p += BIG_WG) {
    const uint64_t my = v.id[v.perm[p]];
    if (p != 0 && v.id[v.perm[p - 1]] == my) continue;
    int ge = p + 1;
    while (ge < n && v.id[v.perm[ge]] == my) ++ge;
    if (ge == p + 1) { v.live[p] = 1; continue; }
    npe |= merge_group(v, p, ge);
  }
  if (npe) atomicOr(A.status, ST_NPE);
  if (__syncthreads_or(npe ? 1 : 0)) {  // Trace.merge threw: putTrace adds nothing for the trace
    if (A.sparse && threadIdx.x == 0) A.tseg_big[bi] = 0;
    return;
  }
  for (int p = threadIdx.x; p < n; p += BIG_WG) {
    const uint32_t s = v.perm[p];
    if (v.live[p] && !is_shared(v.pf[s]) && v.pid[s] == 0) atomicMin(&sh_root, p);
  }
  big_sync();
  const int rp = sh_root == 0x7fffffff ? -1 : sh_root;
  for (int p = threadIdx.x; p < n; p += BIG_WG) {
    const uint64_t my = v.id[v.perm[p]];
    if (p != 0 && v.id[v.perm[p - 1]] == my) continue;
    int ge = p + 1;
    while (ge < n && v.id[v.perm[ge]] == my) ++ge;
    resolve_group(v, 0, n, p, ge, rp);
  }
  big_sync();
  for (int p = threadIdx.x; p < n; p += BIG_WG) {
    const int32_t q = v.parent[p];
    if (q >= 0) v.haschild[q] = 1;
  }
  big_sync();
  uint32_t* bfs = nullptr;
  if (ORD) {
    bfs = A.o_bfs + b;
    big_bfs(v, n, rp, A.o_key + b, A.o_fa + b, A.o_fb + b, bfs, A.o_pay ? A.o_pay + b : nullptr);
    big_sync();
  }
  if (A.tr_parent) {  // ZDL_FLAG_TREE_EXPORT / _STREAM (wave_tree_export's encoding)
    for (int p = threadIdx.x; p < n; p += BIG_WG) {
      int head = p;
      while (!v.live[head] && head > 0 && v.id[v.perm[head - 1]] == v.id[v.perm[p]]) --head;
      const uint64_t slot = b + v.perm[p];
      A.tr_node[slot] = (int32_t)(b + v.perm[head]);
      const int par = v.parent[p];
      int32_t pr = -3, bf = -1;
      if (v.live[p] && par != PAR_NONMEMBER) {
        pr = p == rp ? -2 : (par == PAR_TERMINAL ? -1 : (int32_t)(b + v.perm[par]));
        int q = par, steps = 0;
        while (q >= 0 && steps++ <= n) q = v.parent[q];
        if (q == PAR_TERMINAL) bf = ORD ? (int32_t)bfs[p] : 0;
      }
      A.tr_parent[slot] = pr;
      A.tr_bfs[slot] = bf;
      // reason codes (wave_tree_reasons' encoding): firstRemoteAncestor by walking up
      const uint32_t sp = v.perm[p];
      Rsn r{0u, -1, -1, -1, -1};
      int32_t anc = -1;
      if (bf >= 0) {
        int ra = -1;
        for (int q2 = v.parent[p], st2 = 0; q2 >= 0 && st2 <= n; q2 = v.parent[q2], ++st2)
          if (kind_of(v.pf[v.perm[q2]]) != ZDL_KIND_NULL) { ra = q2; break; }
        const bool has = ra >= 0;
        const uint32_t as = has ? v.perm[ra] : 0u;
        r = node_reason(v.pf[sp], v.haschild[p] != 0, v.lsvc[sp], v.rsvc[sp], p == rp, has, has ? v.lsvc[as] : -1,
                        has ? v.pf[as] : 0u, has && v.pid[sp] != 0 && v.pid[sp] == v.id[as]);
        if (has) anc = (int32_t)(b + as);
      }
      if (v.live[p] && !is_shared(v.pf[sp]) && v.pid[sp] == 0 && rp >= 0 && p != rp) r.code |= ZDL_RSN_ATTRIBUTED;
      A.tr_reason[slot] = (uint8_t)r.code;
      A.tr_anc[slot] = anc;
      A.tr_link[4 * slot] = r.pa;
      A.tr_link[4 * slot + 1] = r.ch;
      A.tr_link[4 * slot + 2] = r.xpa;
      A.tr_link[4 * slot + 3] = r.xch;
      A.tr_sorted[slot] = p;
    }
  }
  for (int p = threadIdx.x; p < n; p += BIG_WG) {
    if (v.parent[p] == PAR_NONMEMBER) continue;
    link_node(v, p, rp, n, [&](int32_t a, int32_t c, bool e, int k) {
      if ((uint32_t)a >= A.S || (uint32_t)c >= A.S) { atomicOr(A.status, ST_BADSVC); return; }
      const size_t idx = ((size_t)day * A.S + (size_t)a) * A.S + c;  // row day * S + parent
      if (A.sparse) {
        A.tlg[2 * b + atomicAdd(&sh_cnt, 1u)] = ((uint32_t)idx << 1) | (e ? 1u : 0u);
        return;
      }
      atomicAdd(&A.call[idx], 1ull);
      if (e) atomicAdd(&A.err[idx], 1ull);
      if (ORD) ord_min(&A.first[idx], ord_rank(A.span_base + b, bfs[p], k));
    });
  }
  big_sync();
  if (A.sparse && threadIdx.x == 0) A.tseg_big[bi] = sh_cnt;
}

// One big trace with the workgroup (every thread calls): the time-window / day filters, then
// big_simple, else (or with try_simple false) the exact path.
// SIMPLE_ONLY (k_big): no exact path; returns false when the trace needs it (not simple).
template <int ORD, bool SIMPLE_ONLY = false, int NT = BIG_WG>
__device__ __forceinline__ bool big_one(const Args& A, unsigned char* lds, size_t lds_bytes, uint32_t bi, bool try_simple) {
  __shared__ uint32_t sh_cnt;  // sparse: links logged for the current trace (big_simple)
  __shared__ int sh_act;
  __shared__ int64_t sh_ts_root_idx, sh_ts_min;
  bool handled = true;
  do {
    const uint32_t t = A.big_list[bi];
    const uint64_t b = A.off[t];
    if (A.off[t + 1] < b || A.off[t + 1] > A.n_spans) {  // k_link flagged it
      if (A.sparse && threadIdx.x == 0) A.tseg_big[bi] = 0;
      break;
    }
    const int n = (int)(A.off[t + 1] - b);
    if (threadIdx.x == 0) {
      sh_cnt = 0;
      if (A.sparse) A.tseg_big[bi] = 0;  // a trace skipped below logs nothing
      sh_act = 1;
      sh_ts_root_idx = 0x7fffffffffffffffll;
      sh_ts_min = 0;
    }
    big_sync();
    if (A.window) {
      // first parentless span with a timestamp (storage order), else the minimum one
      for (int s = threadIdx.x; s < n; s += NT) {
        const int64_t x = A.c.ts[b + s];
        if (x == 0) continue;
        const uint64_t pid = A.c.pid[b + s];
        if (pid == 0 || pid == A.c.id[b + s]) atomicMin((long long*)&sh_ts_root_idx, (long long)s);
      }
      big_sync();
      if (threadIdx.x == 0 && sh_ts_root_idx != 0x7fffffffffffffffll)
        sh_ts_min = A.c.ts[b + sh_ts_root_idx];
      big_sync();
      if (sh_ts_root_idx == 0x7fffffffffffffffll) {
        for (int s = threadIdx.x; s < n; s += NT) {
          const int64_t x = A.c.ts[b + s];
          if (x != 0) {
            // atomicMin over positive micros; 0 stays "unset"
            unsigned long long* m = (unsigned long long*)&sh_ts_min;
            unsigned long long cur = *m;
            while ((cur == 0 || (unsigned long long)x < cur)) {
              const unsigned long long prev = atomicCAS(m, cur, (unsigned long long)x);
              if (prev == cur) break;
              cur = prev;
            }
          }
        }
        big_sync();
      }
      if (threadIdx.x == 0) sh_act = window_pass(sh_ts_min, A.win_lo, A.win_hi) ? 1 : 0;
      big_sync();
      if (!sh_act) { big_sync(); continue; }
    }
    if (A.days) {  // daily buckets: flooredTraceTimestamp over the trace in storage order
      if (threadIdx.x == 0) sh_ts_root_idx = 0x7fffffffffffffffll;
      big_sync();
      for (int s = threadIdx.x; s < n; s += NT)  // the first span with a timestamp
        if (A.c.ts[b + s] != 0) atomicMin((long long*)&sh_ts_root_idx, (long long)s);
      big_sync();
      const int f0 = sh_ts_root_idx == 0x7fffffffffffffffll ? n : (int)sh_ts_root_idx;
      const int64_t m1 = f0 < n ? floored_step(INT64_MAX, A.c.ts[b + f0]) : INT64_MAX;
      if (threadIdx.x == 0) sh_act = 0;
      big_sync();
      // a later span changes m only if its micros compare below m's millis: find any
      for (int s = f0 + 1 + threadIdx.x; s < n; s += NT)
        if (A.c.ts[b + s] != 0 && A.c.ts[b + s] < m1) sh_act = 1;
      big_sync();
      if (threadIdx.x == 0) {
        int64_t m = m1;
        if (sh_act)  // the literal walk (never for real clocks)
          for (int s = f0 + 1; s < n; ++s) m = floored_step(m, A.c.ts[b + s]);
        sh_act = 1;
        const int64_t d = m == INT64_MAX ? -1 : (m - A.day0) / DAY_MS;
        const bool ok = m != INT64_MAX && m >= A.day0 && d < (int64_t)A.days;
        if (!ok && (m == INT64_MAX || !A.days_skip)) atomicOr(A.status, ST_DAYS);
        else if (ok) ord_min(&A.day_first[d], A.span_base + b);
        sh_ts_min = ok ? d : -1;
      }
      big_sync();
      if (sh_ts_min < 0) { big_sync(); continue; }
    }
    const uint32_t day = A.days ? (uint32_t)sh_ts_min : 0u;
    if (!ORD && try_simple && !A.skip_simple && big_simple<NT>(A, lds, lds_bytes, b, n, day, &sh_cnt)) {
      if (A.sparse && threadIdx.x == 0) A.tseg_big[bi] = sh_cnt;
      continue;
    }
    if (SIMPLE_ONLY) handled = false;
    else big_exact<ORD>(A, b, n, day, bi);
  } while (false);
  big_sync();
  return handled;
}

#include "zdl_giant.inc"  // the device-wide tier for big traces (sparse contexts)

// ---------------------------------------------------------------- k_compact
// zdl_link's output record (24 B), copied to the host in one transfer.
struct ZLink {
  int32_t parent, child;
  int64_t call, err;
};

// Non-zero cells -> records, in cell order (= (parent id, child id) order): one workgroup,
// a block-wide exclusive scan of the per-thread non-zero counts. For S*S <= 1024 * 8.
constexpr int COMPACT_WG = 1024;
constexpr size_t MAP_CAP = (size_t)COMPACT_WG * 8;  // records of the mapped output
// The mapped output, columns (lanes store consecutive 4 / 8 B: few host-bus transactions):
// u64 meta[2] = {status word, record count}, i32 parent[MAP_CAP], i32 child[MAP_CAP],
// i64 call[MAP_CAP], i64 err[MAP_CAP].
constexpr size_t MAP_BYTES = 16 + MAP_CAP * 24;
struct MapCols {
  int32_t* parent;
  int32_t* child;
  int64_t* call;
  int64_t* err;
};
__host__ __device__ inline MapCols map_cols(unsigned long long* meta) {
  unsigned char* b = reinterpret_cast<unsigned char*>(meta) + 16;
  return MapCols{reinterpret_cast<int32_t*>(b), reinterpret_cast<int32_t*>(b + 4 * MAP_CAP),
                 reinterpret_cast<int64_t*>(b + 8 * MAP_CAP), reinterpret_cast<int64_t*>(b + 16 * MAP_CAP)};
}
// Writes into mapped pinned host memory: meta[0] = the status word, meta[1] = the record
// count, then the records (the host reads them after one sync). One workgroup of
// COMPACT_WG threads; every thread of it must call.
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {  // device-coherent read
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wsum: COMPACT_WG / 64 + 1 words of LDS scratch.
__device__ __forceinline__ void compact_ordered(const unsigned long long* __restrict__ call,
                                                const unsigned long long* __restrict__ err, uint32_t SS,
                                                uint32_t S, const uint32_t* __restrict__ status,
                                                unsigned long long* __restrict__ meta, uint32_t* wsum) {
  constexpr int KMAX = 8;  // cells per thread: SS <= COMPACT_WG * KMAX
  const MapCols out = map_cols(meta);
  const uint32_t K = (SS + COMPACT_WG - 1) / COMPACT_WG, c0 = threadIdx.x * K;
  unsigned long long cv[KMAX];
  uint32_t nz = 0;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    cv[k] = (uint32_t)k < K && c0 + k < SS ? ld_agent(&call[c0 + k]) : 0ull;
    nz += cv[k] != 0 ? 1u : 0u;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = nz;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < COMPACT_WG / 64; ++i) {
      const uint32_t t = wsum[i];
      wsum[i] = acc;
      acc += t;
    }
    wsum[COMPACT_WG / 64] = acc;
    meta[0] = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    meta[1] = acc;
  }
  __syncthreads();
  uint32_t o = wsum[w] + incl - nz;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (cv[k] == 0) continue;
    const uint32_t i = c0 + k;
    out.parent[o] = (int32_t)(i / S);
    out.child[o] = (int32_t)(i % S);
    out.call[o] = (int64_t)cv[k];
    out.err[o] = (int64_t)ld_agent(&err[i]);
    ++o;
  }
}

// A lazy put's end, in k_link (every thread of every workgroup calls): the hand-off of k_tail's
// compaction (MI355X_MICROARCH.md, "Valid forms", first row): each wave waits for its table
// atomics, one lane per workgroup adds to `done`, and the workgroup whose add returns the last
// ticket sees every count. If k_link left nothing for k_mid / k_tail (no listed big trace, no
// queued window) it compacts the table into the mapped buffer, zeroes the next put's counter
// slots and releases `seq` - the put is complete without launching them; otherwise it stores
// seq | FLAG_TAIL and the host launches them (zdl_link, or the context's next call).
__device__ void lk_lazy_end(const Args& A0, uint32_t* scratch) {
  KArgs& A = rare(A0);  // read here from the argument segment, not held across k_link's loop
  // scratch (LDS, after the table flush): [0] last, [1] tail, [4..] compact_ordered's sums
  uint32_t& last = scratch[0];
  uint32_t& tail = scratch[1];
  __syncthreads();  // every wave is past its flush's LDS reads
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(A.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    const uint32_t b = __hip_atomic_load(A.big_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t l = __hip_atomic_load(A.large_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t x = __hip_atomic_load(A.cx_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tail = (b | l | x) != 0;
  }
  __syncthreads();
  if (!tail) compact_ordered(A.call, A.err, A.rows * A.S, A.S, A.status, A.map, scratch + 4);
  __syncthreads();
  if (!tail && threadIdx.x < CTR_N) A.ctr_next[threadIdx.x] = 0;  // k_tail's job when it runs
  if (threadIdx.x == 0) {
    *A.done = 0;
    __threadfence_system();  // the records and counts are visible to the host before the flag
    __hip_atomic_store(A.flag, tail ? (A.seq | FLAG_TAIL) : A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// A lazy LOG-mode put's k_link end (round 5): the same ticket as lk_lazy_end, but nothing to
// compact (large tables are compacted on the device at zdl_link, after the LOG reduce). If k_link
// left nothing for k_mid / k_big / k_tail, the last workgroup zeroes the next put's counter
// slots and stores `seq`: the put is k_link and the LOG reduce (its kernels already queued), and
// the tail kernels, five near-empty launches a step, are never launched.
__device__ void lk_lazy_end_log(const Args& A0, uint32_t* scratch) {
  KArgs& A = rare(A0);
  uint32_t& last = scratch[0];
  uint32_t& tail = scratch[1];
  __syncthreads();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(A.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    const uint32_t b = __hip_atomic_load(A.big_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t l = __hip_atomic_load(A.large_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t x = __hip_atomic_load(A.cx_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tail = (b | l | x) != 0;
  }
  __syncthreads();
  if (!tail && threadIdx.x < CTR_N) A.ctr_next[threadIdx.x] = 0;  // k_tail's job when it runs
  if (threadIdx.x == 0) {
    *A.done = 0;
    __threadfence_system();
    __hip_atomic_store(A.flag, tail ? (A.seq | FLAG_TAIL) : A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void __launch_bounds__(COMPACT_WG) k_compact_ordered(const unsigned long long* __restrict__ call,
                                                                const unsigned long long* __restrict__ err,
                                                                uint32_t SS, uint32_t S,
                                                                const uint32_t* __restrict__ status,
                                                                unsigned long long* __restrict__ meta) {
  __shared__ uint32_t wsum[COMPACT_WG / 64 + 1];
  compact_ordered(call, err, SS, S, status, meta, wsum);
}

// ------------------------------------------------------------------- k_tail
// The put's last kernel, one 1024-thread workgroup per CU: the windows k_link queued (one
// wave each), then the traces longer than WSMALL (one workgroup each), then - when the
// table is small enough for ordered output - the last workgroup to finish compacts the
// table into the mapped host buffer, so zdl_link needs no kernel. Also zeroes the next
// put's counters.
static_assert(TAIL_WG == BIG_WG && TAIL_WG == COMPACT_WG, "k_tail runs all three parts");
constexpr size_t tail_block_bytes(int window) {  // full_windows' table + carves; at least 150 KB (big_simple)
  return WTABLE_BYTES + (TAIL_WG / 64) * wl::bytes(window) > (size_t)(TAIL_WG / 64) * WB_CARVE
             ? WTABLE_BYTES + (TAIL_WG / 64) * wl::bytes(window)
             : (size_t)(TAIL_WG / 64) * WB_CARVE;
}

template <int DENSE, int WINDOW, int ORD>
__global__ void __launch_bounds__(TAIL_WG, 1) k_tail(Args A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  __shared__ bool last;
  if (blockIdx.x == 0 && threadIdx.x < CTR_N) A.ctr_next[threadIdx.x] = 0;
  full_windows<DENSE, WINDOW, TAIL_WG / 64, ORD>(A, lds);
  __syncthreads();
  // big_list's back (traces longer than wb_max), then the traces k_mid could not link (not
  // simple), one workgroup each, by ticket (the next one fetched while this trace is linked),
  // so that a giant trace delays only its own workgroup
  __shared__ uint32_t sh_j;
  // when k_big ran, only the back-list traces it left for the exact path (its compacted list;
  // walking the whole back list by ticket cost a returning atomic per entry: ~0.3 ms at C5)
  const uint32_t nlarge = A.bstat ? *A.exact_n : A.grest ? *A.grest_n : *A.large_count;
  const uint32_t nbig = nlarge + (A.wb_max ? *A.retry_count : 0u);
  if (nbig) {
    if (threadIdx.x == 0) sh_j = atomicAdd(A.tick_large, 1u);
    while (true) {
      __syncthreads();
      const uint32_t j = sh_j;
      __syncthreads();
      if (j >= nbig) break;
      if (threadIdx.x == 0) sh_j = atomicAdd(A.tick_large, 1u);
      const bool back = j < nlarge;
      const uint32_t bi = !back ? A.retry[j - nlarge]
                                : A.bstat ? A.exact[j] : A.grest ? A.grest[j] : A.big_cap - 1u - j;
      // the giant tier's verdict when k_big did not run: 1 linked, 2 the exact path
      const uint8_t gs = !back ? 0 : A.bstat ? 2 : A.gstat ? A.gstat[bi] : 0;  // (uniform)
      if (gs != 1) big_one<ORD>(A, lds, tail_block_bytes(WINDOW), bi, back && gs == 0);
    }
  }
  if (!A.map) return;
  // Hand-off to the last workgroup (MI355X_MICROARCH.md, "Valid forms", first table row):
  // the table and status updates are agent-scope atomics, performed at the memory side;
  // every wave waits for its own to be acknowledged (vmcnt(0), written as inline asm: a
  // workgroup-scope fence lowers to no wait outside TgSplit mode), then one lane per
  // workgroup adds to `done`, and the workgroup whose add returns the last ticket reads
  // the cells with sc1 (agent-scope) loads only. No agent-scope fence: that would write
  // back the XCD's L2 per workgroup (37 us measured) and protects nothing here.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(A.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __shared__ uint32_t wsum[COMPACT_WG / 64 + 1];
  compact_ordered(A.call, A.err, A.rows * A.S, A.S, A.status, A.map, wsum);
  __syncthreads();
  if (threadIdx.x == 0) {
    *A.done = 0;
    __threadfence_system();  // the records and counts are visible to the host before the flag
    __hip_atomic_store(A.flag, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// k_big: the back list's big traces by big_simple alone (the time-window / day filters
// included), before k_tail; what is not simple is left to k_tail's exact path. Its own kernel so
// that big_simple's registers never meet full_windows' and big_exact's: together they spilled
// k_tail at 1024 threads (52 VGPRs, 244 B of scratch per lane: 1.9 GB of scratch writes per C5
// put, profiles/r03e_hbm_c2_c5.json). Two launches by trace size: k_big<256> takes the traces of
// at most KB_SMALL spans, four 256-thread workgroups per CU in 37.5 KB of LDS each (a trace's
// phases are barrier-latency-bound, so four traces in flight beat one 1024-thread workgroup),
// k_big<1024> the longer ones in 150 KB. The back list is taken 16 entries per ticket; each
// launch links the entries of its size class. bstat[bi] = 1 linked (or outside the window),
// 2 for k_tail's exact path.
constexpr int KB_SMALL_LDS = 38400;
constexpr int KB_SMALL = (KB_SMALL_LDS - 240) / 81;  // bs_bytes(n) <= KB_SMALL_LDS
constexpr int KB_BATCH = 16;
template <int NT>
__global__ void __launch_bounds__(NT, NT == 256 ? 4 : 1) k_big(Args A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  __shared__ uint32_t sh_j;
  constexpr bool SMALL = NT == 256;
  const uint32_t nlarge = A.grest ? *A.grest_n : *A.large_count;
  if (nlarge == 0) return;
  const size_t lds_bytes = SMALL ? (size_t)KB_SMALL_LDS : tail_block_bytes(A.days ? 2 : A.window);
  uint32_t* const tick = SMALL ? A.tick_big + 1 : A.tick_big;
  while (true) {
    __syncthreads();
    if (threadIdx.x == 0) sh_j = atomicAdd(tick, (uint32_t)KB_BATCH);
    __syncthreads();
    const uint32_t j0 = sh_j;
    if (j0 >= nlarge) break;
    for (uint32_t j = j0; j < j0 + KB_BATCH && j < nlarge; ++j) {
      const uint32_t bi = A.grest ? A.grest[j] : A.big_cap - 1u - j;
      const uint32_t t = A.big_list[bi];
      const uint64_t n = A.off[t + 1] - A.off[t];  // (k_link checked the offsets; a flagged trace
      if (SMALL != (n <= (uint64_t)A.kb_small)) continue;  // has n out of range: the large launch's)
      const uint8_t gs = A.gstat ? A.gstat[bi] : 0;  // the giant tier's verdict (uniform)
      uint8_t st = gs;
      if (gs == 0) st = big_one<0, true, NT>(A, lds, lds_bytes, bi, true) ? 1 : 2;
      if (threadIdx.x == 0) {
        A.bstat[bi] = st;
        if (st == 2) A.exact[atomicAdd(A.exact_n, 1u)] = bi;  // rare: not simple, or the tier rejected it
      }
    }
  }
}

inline const void* k_tail_fn(int dense, int window, int ord = 0) {  // dense: 0 hash, 1 dense, 2 sparse sink
  if (dense == 2)  // (daily buckets on a sparse context: the day rides in the logged cell)
    return window == 2 ? (const void*)k_tail<2, 2, 0> : window ? (const void*)k_tail<2, 1, 0> : (const void*)k_tail<2, 0, 0>;
  if (window == 2) {  // daily buckets
    if (ord) return dense ? (const void*)k_tail<1, 2, 1> : (const void*)k_tail<0, 2, 1>;
    return dense ? (const void*)k_tail<1, 2, 0> : (const void*)k_tail<0, 2, 0>;
  }
  if (ord) {
    if (dense) return window ? (const void*)k_tail<1, 1, 1> : (const void*)k_tail<1, 0, 1>;
    return window ? (const void*)k_tail<0, 1, 1> : (const void*)k_tail<0, 0, 1>;
  }
  if (dense) return window ? (const void*)k_tail<1, 1, 0> : (const void*)k_tail<1, 0, 0>;
  return window ? (const void*)k_tail<0, 1, 0> : (const void*)k_tail<0, 0, 0>;
}

#include "zdl_ord.inc"  // insertion order's second pass after a mode 6 put

// Any S: non-zero cells -> records in arbitrary order (the host sorts them).
__global__ void k_compact(const unsigned long long* __restrict__ call, const unsigned long long* __restrict__ err,
                          uint64_t SS, uint32_t S, unsigned long long* __restrict__ count, ZLink* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= SS) return;
  const unsigned long long n = call[i];
  if (n == 0) return;
  const unsigned long long w = atomicAdd(count, 1ull);
  out[w] = ZLink{(int32_t)(i / S), (int32_t)(i % S), (int64_t)n, (int64_t)err[i]};
}

// ---------------------------------------------------------- merge (DL.merge)
// Sums input links per (parent, child) and records the first index each pair was seen
// at, reproducing LinkedHashMap first-seen order (DependencyLinker.java:189-204).
__global__ void k_merge_accum(const int32_t* __restrict__ p, const int32_t* __restrict__ c,
                              const int64_t* __restrict__ call, const int64_t* __restrict__ err, uint64_t n,
                              uint32_t S, unsigned long long* __restrict__ tcall,
                              unsigned long long* __restrict__ terr, unsigned long long* __restrict__ tfirst,
                              uint32_t* __restrict__ status, uint64_t first_base, int first_shift) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if ((uint32_t)p[i] >= S || (uint32_t)c[i] >= S) { atomicOr(status, ST_BADSVC); return; }
  const size_t idx = (size_t)p[i] * S + c[i];
  atomicAdd(&tcall[idx], (unsigned long long)call[i]);
  atomicAdd(&terr[idx], (unsigned long long)err[i]);
  atomicMin(&tfirst[idx], (unsigned long long)(first_base + i) << first_shift);
}

__global__ void k_merge_compact(const unsigned long long* __restrict__ tcall, const unsigned long long* __restrict__ terr,
                                const unsigned long long* __restrict__ tfirst, uint64_t SS, uint32_t S,
                                unsigned long long* __restrict__ count, int32_t* __restrict__ op,
                                int32_t* __restrict__ oc, int64_t* __restrict__ ocall, int64_t* __restrict__ oerr,
                                uint64_t* __restrict__ ofirst) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= SS) return;
  if (tfirst[i] == ~0ull) return;
  const unsigned long long w = atomicAdd(count, 1ull);
  op[w] = (int32_t)(i / S);
  oc[w] = (int32_t)(i % S);
  ocall[w] = (int64_t)tcall[i];
  oerr[w] = (int64_t)terr[i];
  ofirst[w] = tfirst[i];
}

// Insertion order, tables of at most MAP_CAP cells: the non-empty cells (first rank set) with
// their counts and first ranks written straight into mapped pinned host memory (meta[0] the
// status, meta[1] the count, then parent, child, call, err, first columns of MAP_CAP each) IN
// RANK ORDER (DependencyLinker.link()'s list order), so link() costs one kernel, one wait and no
// host sort. Wave w of the grid takes cells w + k NW (k < OC_KEYS): a non-empty cell's place is
// the number of smaller first ranks in the table (ranks are distinct: one addLink, one cell;
// empty cells hold all ones). The wave sweeps the L2-resident table once, OC_BATCH x 64 cells a
// batch (their loads in flight together), comparing each batch against all its cells' ranks
// (a ballot and a popcount per 64), then stores each (rank, cell) at its place. No LDS and
// 256-thread workgroups, so the kernel fits beside the other in-flight context's k_link. The
// workgroup whose ticket comes last (MI355X_MICROARCH.md "Valid forms": every storing wave waits
// vmcnt(0), a barrier, an agent release, the ticket; the last one acquires) writes the columns.
// Round 6 first sorted on the host (std::sort, ~20-30 us of the step's host time at C2's 2 500
// links), then in one workgroup's LDS (a bitonic sort: 50-150 us), then in 96 KB of LDS per
// workgroup (which waited for the other context's k_link to leave a CU: 79 us in flight), then
// a sweep of the table per record (latency-bound: 195 us).
constexpr int OC_WG = 256, ORD_SORT_G = 256, OC_KEYS = 8, OC_BATCH = 16;
static_assert((size_t)ORD_SORT_G * (OC_WG / 64) * OC_KEYS >= MAP_CAP, "k_ord_compact covers every cell");
__global__ void __launch_bounds__(OC_WG) k_ord_compact(const unsigned long long* __restrict__ tcall,
                                                       const unsigned long long* __restrict__ terr,
                                                       const unsigned long long* __restrict__ tfirst, uint32_t SS,
                                                       uint32_t S, const uint32_t* __restrict__ status,
                                                       unsigned long long* __restrict__ meta,
                                                       unsigned long long* __restrict__ srank,
                                                       uint32_t* __restrict__ scell, uint32_t* __restrict__ done) {
  __shared__ uint32_t last, wcnt[OC_WG / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * (OC_WG / 64), gw = blockIdx.x * (OC_WG / 64) + (uint32_t)w;
  unsigned long long key[OC_KEYS];
  uint32_t below[OC_KEYS];
#pragma unroll
  for (int k = 0; k < OC_KEYS; ++k) {
    const uint32_t c = gw + (uint32_t)k * nw;
    key[k] = c < SS ? tfirst[c] : ~0ull;
    below[k] = 0;
  }
  for (uint32_t j0 = 0; j0 < SS; j0 += 64 * OC_BATCH) {
    unsigned long long v[OC_BATCH];
#pragma unroll
    for (int q = 0; q < OC_BATCH; ++q) {
      const uint32_t j = j0 + (uint32_t)(q * 64 + lane);
      v[q] = j < SS ? tfirst[j] : ~0ull;
    }
#pragma unroll
    for (int k = 0; k < OC_KEYS; ++k) {
      if (key[k] == ~0ull) continue;  // (uniform)
      uint32_t n = 0;
#pragma unroll
      for (int q = 0; q < OC_BATCH; ++q) n += (uint32_t)__popcll(__ballot(v[q] < key[k]));
      below[k] += n;
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < OC_KEYS; ++k) {
      if (key[k] == ~0ull) continue;
      srank[below[k]] = key[k];
      scell[below[k]] = gw + (uint32_t)k * nw;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t n = 0;  // the record count: the non-empty cells
  for (uint32_t c = threadIdx.x; c < SS; c += OC_WG) n += tfirst[c] != ~0ull ? 1u : 0u;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) n += __shfl_xor(n, d, 64);
  if (lane == 0) wcnt[w] = n;
  __syncthreads();
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < OC_WG / 64; ++k) m += wcnt[k];
  if (threadIdx.x == 0) {
    *done = 0;  // for the next launch (stream-ordered)
    meta[0] = *status;
    meta[1] = m;
  }
  unsigned char* b = reinterpret_cast<unsigned char*>(meta) + 16;
  int32_t* op = reinterpret_cast<int32_t*>(b);
  int32_t* oc = reinterpret_cast<int32_t*>(b + 4 * MAP_CAP);
  int64_t* ocall = reinterpret_cast<int64_t*>(b + 8 * MAP_CAP);
  int64_t* oerr = reinterpret_cast<int64_t*>(b + 16 * MAP_CAP);
  uint64_t* ofirst = reinterpret_cast<uint64_t*>(b + 24 * MAP_CAP);
  for (uint32_t i = threadIdx.x; i < m; i += OC_WG) {  // consecutive records a wave: coalesced
    const uint32_t cell = scell[i];
    op[i] = (int32_t)(cell / S);
    oc[i] = (int32_t)(cell % S);
    ocall[i] = (int64_t)tcall[cell];
    oerr[i] = (int64_t)terr[cell];
    ofirst[i] = srank[i];
  }
}

}  // namespace zdl

// ====================================================================== host
using namespace zdl;

namespace {

thread_local std::string g_create_error;

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t want) {
    if (want <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    const size_t alloc = std::max<size_t>(want, 1);
    hipError_t e = hipMalloc((void**)&p, alloc * sizeof(T));
    if (e == hipSuccess) n = alloc;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// zdl_put_trace's host staging: the traces of consecutive putTrace calls packed as one CSR
// batch in pinned memory (two slots: one filling while the other's upload runs), put as one
// launch when a slot fills or the context is used otherwise (zdl_stage.inc)
struct StageSlot {
  unsigned char* mem = nullptr;  // one pinned block: the columns, then the offsets
  uint64_t *lo = nullptr, *id = nullptr, *pid = nullptr, *off = nullptr;
  int32_t *ls = nullptr, *rs = nullptr, *i4 = nullptr, *i6 = nullptr;
  uint32_t* pf = nullptr;
  int64_t* ts = nullptr;
  uint64_t n = 0, nt = 0;        // spans and traces staged
  bool has_lo = false, has_ts = false;
  hipEvent_t done = nullptr;     // recorded after the slot's uploads
  bool inflight = false;
};
struct Stage {
  StageSlot slot[2];
  int cur = 0;
  uint64_t cap = 0;  // spans (and traces) per slot
};

}  // namespace

struct zdl_ctx {
  int device = 0;
  uint32_t S = 0;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;
  std::string err;
  int grid = 0;
  int cus = 0;
  uint32_t skip = 0;  // ZDL_SKIP: k_link timing-only ablation bits
  // ranks
  DevBuf<int32_t> rank[3];
  uint32_t nrank[3] = {0, 0, 0};
  // S x S counters
  DevBuf<unsigned long long> call, errc;
  DevBuf<uint32_t> status;
  // insertion order (ZDL_FLAG_INSERTION_ORDER): first-addLink rank per cell, the put-global
  // position of the next put's span 0, big-trace breadth-first scratch
  bool ord = false;
  // daily buckets (zdl_set_days): the tables hold rows = days * S parent rows
  uint32_t days = 0, rows = 0;
  bool days_skip = false;
  int64_t day0 = 0;
  DevBuf<unsigned long long> day_first;
  std::vector<unsigned long long> h_day_first;
  std::vector<int64_t> out_day, out_days;
  DevBuf<unsigned long long> first, o_key;
  DevBuf<uint64_t> ord_n;  // insertion order, mode 6: the traces zdl_ord.inc's pass ranks
  DevBuf<unsigned long long> ord_w;  // ... and the first simple trace of each pair (Args::ord_w),
  DevBuf<unsigned long long> ord_log;  // the waves' records
  DevBuf<uint64_t> ord_start;
  DevBuf<uint32_t> ord_cnt;

  uint64_t span_base = 0;
  DevBuf<uint32_t> o_fa, o_fb, o_bfs, o_pay;
  // per-put scratch
  DevBuf<uint32_t> big_list, counters;
  DevBuf<uint32_t> big_exact_list;  // k_big -> k_tail: the back-list traces for the exact path
  DevBuf<uint8_t> big_stat;  // k_big's verdicts  // counters: two CTR_N blocks alternating by put, then done
  DevBuf<uint32_t> retry;  // k_tail: wave_big traces for the exact path
  uint32_t epoch = 0;
  DevBuf<uint64_t> cx_win;
  // LOG mode (zdl_log.inc): the emit log, its grouped copy, per-wave segments and counts
  DevBuf<uint32_t> lg, lg_pool, lg_n, lg_dir, lg_bn, lg_sets;
  uint32_t lg_par = 0;  // the LOG put's counter set (lg_sets: two of PMAX + 2 words, alternating)
  DevBuf<uint64_t> lg_start;
  int force_tm = -1;  // ZDL_TM=hash|dense|log (tests / ablation): k_link's table mode when it fits
  DevBuf<int32_t> tr_node, tr_parent, tr_bfs;  // ZDL_FLAG_TREE_EXPORT: the last put's tree
  DevBuf<int32_t> tr_anc, tr_link, tr_sorted;  // and its reason codes (zdl_tree_reasons)
  DevBuf<uint8_t> tr_reason;
  // sparse contexts (zdl_sparse.h): the accumulated links as one list sorted by cell; per put
  // the log segments of k_link and k_tail are gathered (seg_*) into lin and merged
  bool sparse = false;
  SparseTable acc;
  SparseWork sw;
  DevBuf<uint64_t> seg_src;
  DevBuf<uint32_t> seg_n, seg_off, tseg_big, tseg_win, lin;
  DevBuf<unsigned char> seg_tmp;
  uint64_t tr_n = 0;
  // Multi-GPU. A device group (zdl_config.device_ids): one context per device,
  // traces sharded by splitmix64(trace_lo) % n, the tables summed by RCCL (ncclReduce to the
  // first device) at zdl_link. A rank of a multi-process job (zdl_comm_init): the tables
  // summed over the ranks (ncclAllReduce) at zdl_link / zdl_table_export.
  std::vector<zdl_ctx*> sub;
  std::vector<ncclComm_t> comms;
  ncclComm_t comm = nullptr;
  struct LocalWorld* lworld = nullptr;  // zdl_comm_init_local: ranks are contexts of this process (zdl_xport.inc)
  int comm_rank = 0, comm_world = 1;
  DevBuf<unsigned long long> xs[3];  // the local transport's reduce scratch
  SparseTable gslice;                // sparse combine: this rank's cell range of the job's list
  DevBuf<unsigned long long> red_call, red_err;  // the summed tables
  DevBuf<unsigned long long> red_first;          // insertion order: the job's first ranks (MIN)
  DevBuf<unsigned long long> ord_lk;             // (the local-order combine: sorted first ranks,
  DevBuf<uint32_t> ord_lv, ord_lv2;              //  their cells before and after the sort,
  DevBuf<unsigned char> ord_ltmp;                //  the sort's scratch)
  // sparse combine (device groups / jobs above 1024 services): every device's or rank's sorted
  // list gathered here (cell, call, err), summed into gacc (sparse_add: DependencyLinker.merge)
  DevBuf<uint32_t> gx_cell;
  DevBuf<unsigned long long> gx_call, gx_err;
  DevBuf<uint64_t> gx_n;  // ranks' list lengths (ncclAllGather)
  SparseTable gacc;
  DevBuf<unsigned long long> prof;
  int prof_on = 0;
  DevBuf<uint64_t> b_id, b_pid;
  DevBuf<int32_t> b_lsvc, b_rsvc, b_ip4, b_ip6, b_parent;
  DevBuf<uint32_t> b_pf, b_perm;
  DevBuf<uint8_t> b_live, b_hasc;
  DevBuf<int32_t> b_nm;
  DevBuf<unsigned long long> b_hk;
  DevBuf<uint32_t> b_hv;
  // the device-wide big-trace tier (zdl_giant.inc, sparse contexts): per-put lists and scratch
  int giant_min = 2048;  // traces longer than this (ZDL_GIANT_MIN; 0: off, k_tail's workgroups)
  DevBuf<uint32_t> gg_bi, gg_n, gg_tile0, gg_bad, gg_tile_g, gg_bstart, gg_blen, gg_meta, gg_H, gg_rest;
  DevBuf<unsigned long long> gg_jl0, gg_jl1;  // k_g_jump's live lists
  DevBuf<uint32_t> gg_jc;                     // and their segments' lengths
  DevBuf<unsigned char> gg_tmp;
  DevBuf<uint32_t> gg_part32;  // k_g_prep_*'s block sums, then carries
  DevBuf<unsigned long long> gg_part64;
  DevBuf<uint64_t> gg_base, gg_h0;
  DevBuf<unsigned long long> gg_root, gg_tsroot, gg_tsmin;
  DevBuf<int32_t> gg_rootidx;
  DevBuf<uint8_t> gg_stat;
  GArgs gg_args{};            // the tier's arguments, from giant_prep to giant_run
  hipEvent_t gg_ev = nullptr;  // k_g_prep's totals copied to h_gmeta
  uint64_t gg_ntmax = 0;
  uint32_t* h_gmeta = nullptr;  // pinned: the tier's GM_* words
  int big_exact = 0;
  bool wave_big = true;  // ZDL_WAVE_BIG=0: every big trace takes a workgroup (tests compare both)  // ZDL_BIG_EXACT=1: big traces skip big_simple (tests compare both paths)
  // host-API staging
  DevBuf<uint64_t> h_id, h_pid, h_off;
  DevBuf<int32_t> h_lsvc, h_rsvc, h_ip4, h_ip6;
  DevBuf<uint32_t> h_pf, h_ord;
  DevBuf<int64_t> h_ts;
  DevBuf<uint64_t> h_lo;
  // ungrouped input: zdl_group's sort + the columns in grouped order
  GroupWork grp;
  LinkWork lw;  // zdl_link's device compaction for S * S > 8192
  DevBuf<uint64_t> g_id, g_pid;
  DevBuf<int32_t> g_lsvc, g_rsvc, g_ip4, g_ip6;
  DevBuf<uint32_t> g_pf;
  DevBuf<int64_t> g_ts;
  // link output
  DevBuf<unsigned long long> count, m_call, m_err, m_first;
  DevBuf<int32_t> o_p, o_c;
  DevBuf<int64_t> o_call, o_err;
  DevBuf<ZLink> o_links;
  uint64_t* h_meta = nullptr;  // pinned (8 words): link count, status; sparse_finish's counts
  unsigned long long* h_map = nullptr;  // mapped pinned: status, count, ordered records
  unsigned long long* h_ordmap = nullptr;  // mapped pinned: insertion order's records (k_ord_compact)
  unsigned long long* d_ordmap = nullptr;
  unsigned long long* d_map = nullptr;  // its device address
  bool map_fresh = false;               // h_map holds the compaction of the current table
  bool ordmap_fresh = false;            // h_ordmap holds the insertion-order compaction of the current table
  bool poisoned = false;                // a put stopped between its kernels: zdl_reset required
  unsigned long long* h_flag = nullptr;  // mapped pinned: the last put's k_tail stores its seq
  unsigned long long* d_flag = nullptr;
  unsigned long long seq = 0;            // puts that compacted into h_map
  // zdl_link's large-table output: mapped pinned host columns (parent, child i32; call, err
  // i64) that k_link_records writes over PCIe directly, no staging copy
  unsigned char* h_rec = nullptr;
  unsigned char* d_rec = nullptr;
  size_t h_rec_cap = 0;
  // ... staged in HBM first (same column layout) and copied by the DMA engine: a compaction
  // kernel storing over PCIe held its CUs for the whole transfer (1.9 ms at C5), so the other
  // step in flight could not run beside it
  DevBuf<unsigned char> rec_dev;
  // ZDL_REC_SDMA=1: the staged records go to the host on an SDMA engine (hsa_amd_memory_async_copy
  // from a helper thread once the compaction's event fired) instead of k_pcie_copy's workgroups
  std::thread rec_th;
  int rec_th_rc = 0;
  hipEvent_t rec_ev = nullptr;
  bool rec_job = false;  // a record copy is pending (run by rec_wait, or by rec_th once launched)
  size_t rec_off[4] = {}, rec_len[4] = {};
  DevBuf<uint64_t> o_first;
  DevBuf<unsigned long long> oc_rank;  // k_ord_compact: (rank, cell) by place, and its ticket
  DevBuf<uint32_t> oc_cell, oc_done;
  DevBuf<int32_t> mi_p, mi_c;
  DevBuf<int64_t> mi_call, mi_err;
  std::vector<int32_t> out_p, out_c;
  std::vector<int64_t> out_call, out_err;
  std::vector<int32_t> host_rank[3];
  // window
  int window = 0;
  int64_t win_lo = 0, win_hi = 0;
  // timing
  hipEvent_t ev[12] = {};
  // ZDL_FLAG_TIMING: a ring of (start, end) event pairs around k_link, one pair per put,
  // averaged by zdl_get_kernel_times (no per-put host query)
  static constexpr int LK_RING = 64;
  hipEvent_t lk_ev[2][LK_RING] = {};
  uint32_t lk_n = 0;
  uint32_t lk_stride = 1, lk_puts = 0;  // time every lk_stride-th put
  zdl_kernel_times times = {};
  uint32_t last_log_lP = 0;    // the last put's LOG partitions (0: not LOG mode), for log_entries
  uint32_t* last_log_set = nullptr;  // ... and its counter set
  uint64_t last_sparse_E = 0;  // the last put's sparse link-log entries
  // a lazy put (Args::lazy): launched k_link only; k_mid / k_tail follow only if its flag says
  // so (resolve_lazy), with the put's arguments kept here
  bool lazy_pending = false;
  Args lazy_A{};
  int lazy_wmode = 0, lazy_dense = 0;
  int link_pending = -1;  // zdl_link_start's order until zdl_link_finish (-1: none)
  bool link_async = false;  // the started link is a sparse compaction in flight
  Stage stg;                // zdl_put_trace's staged traces
};

// a rank of a job: RCCL (zdl_comm_init) or a local world (zdl_comm_init_local)
static inline bool in_job(const zdl_ctx* c) { return c->comm != nullptr || c->lworld != nullptr; }
static void lw_release(zdl_ctx* c);  // zdl_xport.inc

namespace {

int fail(zdl_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hip_fail(zdl_ctx* c, hipError_t e, const char* what) {
  return fail(c, e == hipErrorOutOfMemory ? ZDL_ENOMEM : ZDL_EDEVICE,
              std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(c, expr)                                   \
  do {                                                     \
    hipError_t _e = (expr);                                \
    if (_e != hipSuccess) return hip_fail((c), _e, #expr); \
  } while (0)

// Every API entry: select the context's device and drop a stale error another call left
// (hipGetLastError after a launch would otherwise report it as the launch's).
hipError_t enter(zdl_ctx* c) {
  (void)hipGetLastError();
  return hipSetDevice(c->device);
}

int status_code(zdl_ctx* c, uint32_t st) {
  if (st & ST_NPE) return fail(c, ZDL_EREF_NPE, "reference throws NullPointerException (Span.Builder.merge of a null endpoint)");
  if (st & ST_IAE) return fail(c, ZDL_EREF_IAE, "reference throws IllegalArgumentException");
  if (st & ST_BADSVC) return fail(c, ZDL_EINVAL, "service id >= n_services");
  if (st & ST_BADOFF) return fail(c, ZDL_EINVAL, "trace offsets are not non-decreasing");
  if (st & ST_INTERNAL) return fail(c, ZDL_EDEVICE, "internal consistency check failed on the device");
  if (st & ST_DAYS) return fail(c, ZDL_EINVAL, "daily buckets: a trace has no timestamp or its day is outside the range");
  return ZDL_OK;
}

// Events: 1 / 7 bracket k_link (ZDL_FLAG_TIMING); the others every kernel of the put and
// the link (ZDL_FLAG_TIMING_ALL). Each event is a packet in the stream, so the light mode
// keeps the timed step close to an untimed one.
bool ev_on(const zdl_ctx* c, int i) {
  (void)i;
  return (c->flags & ZDL_FLAG_TIMING_ALL) != 0;
}

void ev_record(zdl_ctx* c, int i) {
  if (ev_on(c, i)) (void)hipEventRecord(c->ev[i], c->stream);
  if ((c->flags & ZDL_FLAG_TIMING) && (i == 1 || i == 7) && c->lk_puts % c->lk_stride == 0)
    (void)hipEventRecord(c->lk_ev[i == 1 ? 0 : 1][(i == 1 ? c->lk_n : c->lk_n++) % zdl_ctx::LK_RING], c->stream);
  if (i == 7) ++c->lk_puts;
}

float ev_ms(zdl_ctx* c, int a, int b) {
  float ms = -1.f;
  if (!ev_on(c, a) || !ev_on(c, b)) return -1.f;
  if (hipEventElapsedTime(&ms, c->ev[a], c->ev[b]) != hipSuccess) ms = -1.f;
  (void)hipGetLastError();  // an unrecorded event is not an error of the next call
  return ms;
}

void put_times(zdl_ctx* c) {
  if (!(c->flags & ZDL_FLAG_TIMING_ALL)) return;
  // events: 1 | k_link | 7 | LOG reduce | 2 | k_mid | 3 | giant tier | 8 | k_tail | 4 | sparse | 9
  c->times.plan_ms = 0.f;
  c->times.full_ms = 0.f;
  c->times.tiles_ms = ev_ms(c, 1, 7);
  c->times.reduce_ms = ev_ms(c, 7, 2);
  c->times.mid_ms = ev_ms(c, 2, 3);
  c->times.giant_ms = ev_ms(c, 3, 8);
  c->times.big_ms = ev_ms(c, 8, 4);
  c->times.sparse_ms = ev_ms(c, 4, 9);
  c->times.sparse_entries = c->last_sparse_E;
  c->times.log_entries = 0;
  if (c->last_log_lP && c->last_log_set) {  // the put's entry count (its work is complete here)
    uint32_t v = 0;
    if (hipMemcpyAsync(&v, c->last_log_set + PMAX + 1, 4, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
        hipStreamSynchronize(c->stream) == hipSuccess)
      c->times.log_entries = v;
    (void)hipGetLastError();
  }
}

}  // namespace

// ---- device groups (zdl_config.device_ids) ----
// Runs f on every device's context; the first failure's message becomes the group's.
template <class F>
int group_each(zdl_ctx* g, F&& f) {
  for (zdl_ctx* s : g->sub) {
    const int rc = f(s);
    if (rc != ZDL_OK) {
      g->err = s->err;
      return rc;
    }
  }
  return ZDL_OK;
}
int group_first(zdl_ctx* g, int rc, zdl_ctx* s = nullptr) {
  if (rc != ZDL_OK) g->err = (s ? s : g->sub[0])->err;
  return rc;
}
int group_put(zdl_ctx* g, const zdl_span_cols* col, uint64_t n_spans, const uint64_t* off, uint64_t n_traces);
int group_export(zdl_ctx* g, void* dev_call, void* dev_err);
static int resolve_lazy(zdl_ctx* c, bool wait);  // a lazy put's k_mid / k_tail (below)
static int stage_flush(zdl_ctx* c);                // zdl_put_trace's staged traces as one put
static void stage_drop(zdl_ctx* c);                // ... discarded (zdl_reset)
static void stage_free(zdl_ctx* c);
static int rec_wait(zdl_ctx* c);  // the SDMA record copy of the last link (ZDL_REC_SDMA)
static int x_failed(zdl_ctx* c, int rc);  // a failed combine breaks a local world (zdl_xport.inc)
static int ord_compact(zdl_ctx* c, const unsigned long long* call, const unsigned long long* errc,
                       const unsigned long long* first_rank);  // insertion order into h_ordmap

// splitmix64 finaliser (shard.py's): trace t goes to device splitmix64(trace_lo) % n
inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

extern "C" {

int zdl_abi_version(void) { return ZDL_ABI_VERSION; }

int zdl_link_occupancy(int device, int table_mode, int window) {
  if (table_mode < TM_HASH || table_mode > TM_SORT || window < 0 || window > 1) return -1;
  if (hipSetDevice(device) != hipSuccess) return -1;
  const void* f = k_link_fn(table_mode, window);
  if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)link_block_bytes(window, table_mode)) !=
      hipSuccess)
    return -1;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, lk::waves(window) * 64, link_block_bytes(window, table_mode)) !=
      hipSuccess)
    return -1;
  return n;
}

const char* zdl_create_error(void) { return g_create_error.c_str(); }

static zdl_ctx* create_group(const zdl_config* cfg);

zdl_ctx* zdl_create(const zdl_config* cfg) {
  g_create_error.clear();
  if (!cfg || cfg->n_services == 0 || cfg->n_services > 65535u) {
    g_create_error = "n_services must be in [1, 65535]";
    return nullptr;
  }
  if (cfg->device_ids) return create_group(cfg);
  zdl_ctx* c = new zdl_ctx();
  c->device = cfg->device;
  c->S = cfg->n_services;
  c->flags = cfg->flags;
  c->ord = (cfg->flags & ZDL_FLAG_INSERTION_ORDER) != 0;
  // a sorted link list instead of the S x S table above 1024 services (zdl_sparse.h); cells
  // and keys are u32 (cell << 1 | error), so S <= 46340. ZDL_SPARSE=1/0 forces it (tests).
  {
    const char* sp = getenv("ZDL_SPARSE");
    const bool want = sp ? sp[0] == '1' : cfg->n_services > 1024;
    c->sparse = want && cfg->n_services <= 46340u &&
                !(cfg->flags & (ZDL_FLAG_INSERTION_ORDER | ZDL_FLAG_DENSE_TABLE));
  }
  if ((cfg->flags & ZDL_FLAG_TREE_EXPORT) && (cfg->flags & ZDL_FLAG_TREE_STREAM)) {
    delete c;
    g_create_error = "ZDL_FLAG_TREE_EXPORT and ZDL_FLAG_TREE_STREAM exclude each other";
    return nullptr;
  }
  if ((cfg->flags & ZDL_FLAG_TREE_EXPORT) && !c->ord) {
    delete c;
    g_create_error = "ZDL_FLAG_TREE_EXPORT needs ZDL_FLAG_INSERTION_ORDER (the exact per-trace path)";
    return nullptr;
  }
  c->rows = cfg->n_services;
  c->lk_stride = std::max<uint32_t>(1u, cfg->timing_stride);
  hipError_t e = hipSetDevice(c->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  const size_t SS = c->sparse ? 0 : (size_t)c->S * c->S;  // sparse: no S x S table
  if (e == hipSuccess && SS) e = c->call.ensure(SS);
  if (e == hipSuccess && SS) e = c->errc.ensure(SS);
  if (e == hipSuccess) e = c->status.ensure(4);
  if (e == hipSuccess) e = c->count.ensure(1);
  if (e == hipSuccess && SS) e = hipMemsetAsync(c->call.p, 0, SS * 8, c->stream);
  if (e == hipSuccess && SS) e = hipMemsetAsync(c->errc.p, 0, SS * 8, c->stream);
  if (e == hipSuccess) e = hipMemsetAsync(c->status.p, 0, 16, c->stream);
  if (e == hipSuccess && c->ord) e = c->first.ensure(SS);
  if (e == hipSuccess && c->ord) e = hipMemsetAsync(c->first.p, 0xff, SS * 8, c->stream);
  if (e == hipSuccess) e = c->counters.ensure(CTR_DONE + 1);  // + k_tail's finished-workgroup count
  if (e == hipSuccess) e = hipMemsetAsync(c->counters.p, 0, (CTR_DONE + 1) * 4, c->stream);
  if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_meta, 64, hipHostMallocDefault);
  // timing-only events: no system-scope fence (cache writeback) between the kernels they bracket
  for (int i = 0; i < 12 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->ev[i], hipEventDisableSystemFence);
  for (int i = 0; i < 2 * zdl_ctx::LK_RING && e == hipSuccess && (cfg->flags & ZDL_FLAG_TIMING); ++i)
    e = hipEventCreateWithFlags(&c->lk_ev[i & 1][i >> 1], hipEventDisableSystemFence);
  if (e == hipSuccess) {
    int cus = 0;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    c->cus = std::max(1, cus);
    c->grid = c->cus;  // k_tail: one 1024-thread workgroup per CU
  }
  for (int w = 0; w < 2 && e == hipSuccess; ++w) {
    for (int tm = 0; tm < 3 && e == hipSuccess; ++tm)
      e = hipFuncSetAttribute(k_link_fn(tm, w), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)link_block_bytes(w, tm));
    for (int m = 1; m <= 5 && e == hipSuccess; ++m)
      for (int tm = 0; tm < (m == 5 ? 4 : (m == 4 || m == 2) ? 3 : 2) && e == hipSuccess; ++tm)
        e = hipFuncSetAttribute(k_link_fn(tm, w, m), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)link_block_bytes(m == 3 ? 0 : w, tm, m));
  }
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_g_join, hipFuncAttributeMaxDynamicSharedMemorySize, GHCAP * 16);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_big<TAIL_WG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)std::max(tail_block_bytes(0), std::max(tail_block_bytes(1), tail_block_bytes(2))));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_big<256>, hipFuncAttributeMaxDynamicSharedMemorySize, KB_SMALL_LDS);
  for (int d = 0; d < 3 && e == hipSuccess; ++d)
    for (int w = 0; w < 3 && e == hipSuccess; ++w)
      for (int o = 0; o < (d == 2 ? 1 : 2) && e == hipSuccess; ++o)
        e = hipFuncSetAttribute(k_tail_fn(d, w, o), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)tail_block_bytes(w));
  for (int w = 0; w < 2 && e == hipSuccess; ++w) {
    e = hipFuncSetAttribute(k_link_fn(TM_DENSE, w, 6), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)link_block_bytes(w, TM_DENSE, 6));
    if (e == hipSuccess)
      e = hipFuncSetAttribute(k_ord_rank_fn(w), hipFuncAttributeMaxDynamicSharedMemorySize, (int)tail_block_bytes(w));
  }

  if (e == hipSuccess) {
    const char* pe = getenv("ZDL_PROF");
    c->prof_on = pe && pe[0] == '1';
    if (c->prof_on) {  // 12 phase counters, then (start, end, hardware id) of every k_link wave
      const size_t words = 12 + 3 * (size_t)c->cus * lk::wgs_per_cu * lk::waves(0);
      e = c->prof.ensure(words);
      if (e == hipSuccess) e = hipMemsetAsync(c->prof.p, 0, words * 8, c->stream);
    }
    const char* sk = getenv("ZDL_SKIP");
    c->skip = sk ? (uint32_t)strtoul(sk, nullptr, 0) : 0u;
    const char* be = getenv("ZDL_BIG_EXACT");
    c->big_exact = be && be[0] == '1';
    const char* wb = getenv("ZDL_WAVE_BIG");
    c->wave_big = !(wb && wb[0] == '0');
    const char* gm = getenv("ZDL_GIANT_MIN");
    if (gm) c->giant_min = (int)strtol(gm, nullptr, 0);
    if (c->giant_min > 0 && c->giant_min < WB_MAX) c->giant_min = WB_MAX;  // k_mid keeps its traces
    const char* ft = getenv("ZDL_TM");
    if (ft) c->force_tm = !strcmp(ft, "hash") ? TM_HASH : (!strcmp(ft, "log") ? TM_LOG : -1);
  }
  // the initial memsets run on the context's (non-blocking) stream and are waited for
  // here: a null-stream hipMemset is not ordered before the first put's kernels on a
  // non-blocking stream, and could land after k_link had counted (lost big-trace lists)
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    g_create_error = std::string("device init failed: ") + hipGetErrorString(e);
    zdl_destroy(c);
    return nullptr;
  }
  return c;
}

void zdl_destroy(zdl_ctx* c) {
  if (!c) return;
  if (!c->sub.empty() || !c->comms.empty()) {  // a device group
    for (auto& cm : c->comms)
      if (cm) (void)ncclCommDestroy(cm);
    for (auto* s : c->sub) zdl_destroy(s);
    stage_free(c);
    delete c;
    return;
  }
  if (c->comm) (void)ncclCommDestroy(c->comm);
  lw_release(c);
  (void)hipSetDevice(c->device);
  (void)resolve_lazy(c, false);
  stage_free(c);
  if (c->rec_th.joinable()) c->rec_th.join();  // a started link's copy; a pending one is dropped
  c->rec_job = false;
  if (c->rec_ev) (void)hipEventDestroy(c->rec_ev);
  c->red_call.release();
  c->red_err.release();
  c->red_first.release();
  c->ord_lk.release(); c->ord_lv.release(); c->ord_lv2.release(); c->ord_ltmp.release();
  for (auto& x : c->xs) x.release();
  c->gslice.release();
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& r : c->rank) r.release();
  c->call.release(); c->errc.release(); c->status.release();
  c->first.release(); c->ord_n.release(); c->ord_w.release(); c->ord_log.release();
  c->ord_start.release(); c->ord_cnt.release(); c->day_first.release(); c->o_key.release(); c->o_fa.release(); c->o_fb.release(); c->o_bfs.release(); c->o_pay.release();
  c->big_list.release(); c->big_stat.release(); c->big_exact_list.release(); c->counters.release(); c->retry.release();
  c->cx_win.release();
  if (c->prof_on && c->prof.p) {
    unsigned long long h[12] = {};
    if (hipMemcpy(h, c->prof.p, sizeof h, hipMemcpyDeviceToHost) == hipSuccess) {
      double tot = 0;
      for (int k = 0; k < 12; ++k) tot += (double)h[k];
      fprintf(stderr, "[zdl prof] k_link cycles per phase (all waves, all puts):");
      for (int k = 0; k < 12; ++k) fprintf(stderr, " %d:%.1f%%", k, tot > 0 ? 100.0 * (double)h[k] / tot : 0.0);
      fprintf(stderr, " total %.3e\n", tot);
    }
    // the last put's k_link waves: when each finished after the first one started (100 MHz clock)
    const size_t W = (size_t)c->cus * lk::wgs_per_cu * lk::waves(0);
    std::vector<unsigned long long> w(3 * W);
    if (hipMemcpy(w.data(), c->prof.p + 12, 3 * W * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      if (const char* dp = getenv("ZDL_PROF_DUMP")) {  // (start, end, hardware id) per wave, raw u64
        if (FILE* f = fopen(dp, "wb")) {
          fwrite(w.data(), 8, w.size(), f);
          fclose(f);
        }
      }
      unsigned long long t0 = ~0ull;
      for (size_t i = 0; i < W; ++i)
        if (w[3 * i]) t0 = std::min(t0, w[3 * i]);
      std::vector<double> end, busy;
      for (size_t i = 0; i < W; ++i)
        if (w[3 * i] && w[3 * i + 1]) {
          end.push_back((double)(w[3 * i + 1] - t0) * 0.01);
          busy.push_back((double)(w[3 * i + 1] - w[3 * i]) * 0.01);
        }
      std::sort(end.begin(), end.end());
      std::sort(busy.begin(), busy.end());
      if (!end.empty()) {
        auto q = [&](const std::vector<double>& v, double f) { return v[std::min(v.size() - 1, (size_t)(f * v.size()))]; };
        fprintf(stderr, "[zdl prof] k_link waves %zu: end us min %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f; "
                        "busy us p10 %.1f p50 %.1f p90 %.1f max %.1f\n",
                end.size(), end.front(), q(end, 0.1), q(end, 0.5), q(end, 0.9), q(end, 0.99), end.back(), q(busy, 0.1),
                q(busy, 0.5), q(busy, 0.9), busy.back());
      }
    }
  }
  c->prof.release();
  c->lg.release(); c->lg_pool.release(); c->lg_n.release(); c->lg_dir.release(); c->lg_bn.release(); c->lg_sets.release();
  c->lg_start.release();
  c->tr_node.release(); c->tr_parent.release(); c->tr_bfs.release();
  c->tr_anc.release(); c->tr_link.release(); c->tr_sorted.release(); c->tr_reason.release();
  c->acc.release(); c->sw.release(); c->seg_src.release(); c->seg_n.release(); c->seg_off.release();
  c->gx_cell.release(); c->gx_call.release(); c->gx_err.release(); c->gx_n.release(); c->gacc.release();
  c->tseg_big.release(); c->tseg_win.release(); c->lin.release(); c->seg_tmp.release();
  c->b_id.release(); c->b_pid.release(); c->b_lsvc.release(); c->b_rsvc.release(); c->b_ip4.release();
  c->b_ip6.release(); c->b_parent.release(); c->b_pf.release(); c->b_perm.release(); c->b_live.release();
  c->b_hasc.release(); c->b_nm.release(); c->b_hk.release(); c->b_hv.release();
  for (auto* b : {&c->gg_bi, &c->gg_n, &c->gg_tile0, &c->gg_bad, &c->gg_tile_g, &c->gg_bstart, &c->gg_blen,
                  &c->gg_meta, &c->gg_H, &c->gg_rest})
    b->release();
  c->gg_jl0.release();
  c->gg_jl1.release();
  c->gg_jc.release();
  c->gg_tmp.release();
  c->gg_part32.release();
  c->gg_part64.release();
  if (c->gg_ev) (void)hipEventDestroy(c->gg_ev);
  c->gg_base.release(); c->gg_h0.release(); c->gg_root.release(); c->gg_tsroot.release(); c->gg_tsmin.release();
  c->gg_rootidx.release(); c->gg_stat.release();
  if (c->h_gmeta) (void)hipHostFree(c->h_gmeta);
  c->h_id.release(); c->h_pid.release(); c->h_off.release(); c->h_lsvc.release(); c->h_rsvc.release();
  c->h_ip4.release(); c->h_ip6.release(); c->h_pf.release(); c->h_ts.release();
  c->h_lo.release(); c->h_ord.release(); c->grp.release(); c->lw.release();
  c->g_id.release(); c->g_pid.release(); c->g_lsvc.release(); c->g_rsvc.release(); c->g_ip4.release();
  c->g_ip6.release(); c->g_pf.release(); c->g_ts.release();
  c->count.release(); c->m_call.release(); c->m_err.release(); c->m_first.release();
  c->o_p.release(); c->o_c.release(); c->o_call.release(); c->o_err.release(); c->o_first.release();
  c->oc_rank.release(); c->oc_cell.release(); c->oc_done.release();
  c->o_links.release();
  if (c->h_meta) (void)hipHostFree(c->h_meta);
  if (c->h_map) (void)hipHostFree(c->h_map);
  if (c->h_ordmap) (void)hipHostFree(c->h_ordmap);
  if (c->h_flag) (void)hipHostFree(c->h_flag);
  if (c->h_rec) (void)hipHostFree(c->h_rec);
  c->rec_dev.release();
  c->mi_p.release(); c->mi_c.release(); c->mi_call.release(); c->mi_err.release();
  for (auto& ev : c->ev)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& row : c->lk_ev)
    for (auto& ev : row)
      if (ev) (void)hipEventDestroy(ev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* zdl_last_error(const zdl_ctx* c) { return c ? c->err.c_str() : "null context"; }

void* zdl_stream(zdl_ctx* c) {
  if (c && !c->sub.empty()) return zdl_stream(c->sub[0]);
  return c ? (void*)c->stream : nullptr;
}

int zdl_set_ranks(zdl_ctx* c, int dict, const int32_t* rank, uint32_t n) {
  if (!c || dict < 0 || dict > 2) return fail(c, ZDL_EINVAL, "bad dictionary");
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_set_ranks: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) return group_each(c, [&](zdl_ctx* s) { return zdl_set_ranks(s, dict, rank, n); });
  HIP_TRY(c, enter(c));
  c->host_rank[dict].assign(rank, rank + n);
  if (n == 0) {
    c->nrank[dict] = 0;
    return ZDL_OK;
  }
  HIP_TRY(c, c->rank[dict].ensure(n));
  HIP_TRY(c, hipMemcpyAsync(c->rank[dict].p, rank, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->nrank[dict] = n;
  return ZDL_OK;
}

int zdl_set_days(zdl_ctx* c, int64_t day0_ms, uint32_t n_days) {
  if (!c) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_set_days: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty() || in_job(c)) return fail(c, ZDL_EINVAL, "zdl_set_days: one device, one process");
  const bool skip = (n_days & ZDL_DAYS_SKIP_OUTSIDE) != 0;
  n_days &= ~ZDL_DAYS_SKIP_OUTSIDE;
  if (n_days > 255) return fail(c, ZDL_EINVAL, "zdl_set_days: at most 255 days");
  if (n_days && (day0_ms % DAY_MS) != 0) return fail(c, ZDL_EINVAL, "zdl_set_days: day0 must be a UTC midnight");
  if (n_days && c->window) return fail(c, ZDL_EINVAL, "zdl_set_days: not with a time window");
  // a sparse context's cells are u32 log entries (cell << 1 | error): the day rides in the cell
  const uint64_t cells = (uint64_t)(n_days ? n_days : 1) * c->S * c->S;
  if (c->sparse && cells >= (1ull << 31))
    return fail(c, ZDL_EINVAL, "zdl_set_days: a sparse context needs days * S * S below 2^31");
  if (cells >= (1ull << 32)) return fail(c, ZDL_EINVAL, "zdl_set_days: days * S * S must stay below 2^32");
  HIP_TRY(c, enter(c));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->days = n_days;
  c->days_skip = n_days && skip;
  c->day0 = n_days ? day0_ms : 0;
  c->rows = (n_days ? n_days : 1) * c->S;
  const size_t SS = c->sparse ? 0 : (size_t)c->rows * c->S;  // sparse: one list, no table
  if (SS) HIP_TRY(c, c->call.ensure(SS));
  if (SS) HIP_TRY(c, c->errc.ensure(SS));
  if (c->ord) HIP_TRY(c, c->first.ensure(SS));
  if (n_days) HIP_TRY(c, c->day_first.ensure(n_days));
  c->map_fresh = false;
  c->ordmap_fresh = false;
  return zdl_reset(c);
}

int zdl_set_window(zdl_ctx* c, int64_t end_ts_ms, int64_t lookback_ms) {
  if (!c) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_set_window: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) return group_each(c, [&](zdl_ctx* s) { return zdl_set_window(s, end_ts_ms, lookback_ms); });
  if (c->days && lookback_ms > 0) return fail(c, ZDL_EINVAL, "zdl_set_window: not with daily buckets");
  if (lookback_ms <= 0) {
    c->window = 0;
    return ZDL_OK;
  }
  c->window = 1;
  c->win_hi = end_ts_ms * 1000;
  c->win_lo = (end_ts_ms - lookback_ms) * 1000;
  return ZDL_OK;
}

// Ungrouped input: the columns in grouped order (perm = zdl_group's sorted positions).
__global__ void k_gather(Cols in, const uint32_t* __restrict__ perm, uint64_t n, uint64_t* __restrict__ id,
                         uint64_t* __restrict__ pid, int32_t* __restrict__ lsvc, int32_t* __restrict__ rsvc,
                         int32_t* __restrict__ ip4, int32_t* __restrict__ ip6, uint32_t* __restrict__ pf,
                         int64_t* __restrict__ ts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = perm[i];
  id[i] = in.id[j];
  pid[i] = in.pid[j];
  lsvc[i] = in.lsvc[j];
  rsvc[i] = in.rsvc[j];
  ip4[i] = in.ip4[j];
  ip6[i] = in.ip6[j];
  pf[i] = in.pf[j];
  if (ts) ts[i] = in.ts[j];
}

// The mapped pinned buffer of ordered link output (S*S <= COMPACT_WG * 8).
static hipError_t ensure_map(zdl_ctx* c) {
  if (c->h_map) return hipSuccess;
  hipError_t e = hipHostMalloc((void**)&c->h_map, MAP_BYTES, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&c->d_map, c->h_map, 0);
  if (e == hipSuccess) e = hipHostMalloc((void**)&c->h_flag, 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&c->d_flag, c->h_flag, 0);
  if (e == hipSuccess) *c->h_flag = 0;
  return e;
}

// Insertion order and daily buckets: k_link only plans (mode 3), k_tail counts every window.
// k_link mode 3 (every window through k_tail's exact path): daily buckets, tree export, or
// ZDL_ORD_EXACT=1 (insertion order the PR-1 way, for A/B); mode 4 otherwise on an
// insertion-order context (simple windows ranked in k_link)
static bool plan_only_mode(const zdl_ctx* c) {
  static const bool ord_exact = getenv("ZDL_ORD_EXACT") != nullptr;
  return c->days || (c->ord && ((c->flags & ZDL_FLAG_TREE_EXPORT) || ord_exact));
}

// Sparse contexts: the segments (k_link's waves, then k_tail's big traces and queued windows)
// listed with their start in lg and their link count.
__global__ void k_seg_build(const uint64_t* __restrict__ lg_start, const uint32_t* __restrict__ lg_n, uint32_t W,
                            const uint32_t* __restrict__ big_list, const uint64_t* __restrict__ off,
                            const uint32_t* __restrict__ tseg_big, uint32_t nb, uint32_t nl, uint32_t cap,
                            const uint64_t* __restrict__ cx_win, const uint32_t* __restrict__ tseg_win, uint32_t nw,
                            uint64_t tbase, uint64_t* __restrict__ src, uint32_t* __restrict__ cnt,
                            uint32_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nbl = (uint64_t)nb + nl;
  if (i < W) {
    src[i] = lg_start[i];
    cnt[i] = lg_n[i];
  } else if (i < (uint64_t)W + nbl) {  // big_list's front (wave_big), then its back
    const uint32_t j = (uint32_t)(i - W);
    const uint32_t bi = j < nb ? j : cap - 1u - (j - nb);
    const uint32_t t = big_list[bi];
    src[i] = tbase + 2 * off[t];
    uint32_t c = tseg_big[bi];
    if ((uint64_t)c > 2 * (off[t + 1] - off[t])) {  // more links than the segment holds: a bug, not data
      atomicOr(status, ST_INTERNAL);
      c = 0;
    }
    cnt[i] = c;
  } else if (i < (uint64_t)W + nbl + nw) {
    const uint64_t k = i - W - nbl;
    src[i] = tbase + 2 * (cx_win[2 * k] & ((1ull << 48) - 1));
    uint32_t c = tseg_win[k];
    if (c > 2 * (uint32_t)(cx_win[2 * k] >> 48)) {
      atomicOr(status, ST_INTERNAL);
      c = 0;
    }
    cnt[i] = c;
  }
}

// The segments gathered into one array, by output tiles of SEG_TILE entries (one workgroup
// each: the first segment found by a binary search of the offsets, then walked): a segment
// per workgroup left a 400 k-entry giant trace to one workgroup (243 us at C5).
constexpr uint32_t SEG_TILE = 4096;
__global__ void __launch_bounds__(256) k_seg_copy(const uint32_t* __restrict__ lg, const uint64_t* __restrict__ src,
                                                  const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ at,
                                                  uint64_t nseg, uint64_t E, uint32_t* __restrict__ lin) {
  __shared__ uint64_t sh_s;
  const uint64_t t0 = (uint64_t)blockIdx.x * SEG_TILE, t1 = t0 + SEG_TILE < E ? t0 + SEG_TILE : E;
  if (threadIdx.x == 0) {  // the last segment starting at or before t0
    uint64_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) / 2;
      if (at[mid] <= t0) lo = mid;
      else hi = mid;
    }
    sh_s = lo;
  }
  __syncthreads();
  for (uint64_t sg = sh_s; sg < nseg; ++sg) {
    const uint64_t a = at[sg];
    if (a >= t1) break;
    const uint64_t b0 = a > t0 ? a : t0, e = a + cnt[sg], b1 = e < t1 ? e : t1;
    const uint32_t* in = lg + src[sg];
    for (uint64_t j = b0 + threadIdx.x; j < b1; j += 256) lin[j] = in[j - a];
  }
}

static int sparse_finish(zdl_ctx* c, uint32_t ep, uint32_t lW, uint64_t n_spans, uint64_t n_traces,
                         const uint64_t* off, const uint64_t* n_traces_dev, bool slots) {
  const hipStream_t s = c->stream;
  // how many big traces and queued windows k_tail logged (this put's counter slots)
  HIP_TRY(c, hipMemcpyAsync(c->h_meta, c->counters.p + ep * CTR_N, 4 * (CTR_LARGE + 1), hipMemcpyDeviceToHost, s));
  if (n_traces_dev) HIP_TRY(c, hipMemcpyAsync(c->h_meta + 2, n_traces_dev, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  // (grouped on the device: n_traces is an upper bound - big_list's capacity - and the count is
  // the device's)
  const uint64_t n_dev = n_traces_dev ? std::min<uint64_t>(n_traces, c->h_meta[2]) : n_traces;
  const uint32_t nb = ((uint32_t*)c->h_meta)[CTR_MID], nl = ((uint32_t*)c->h_meta)[CTR_LARGE];
  // k_link mode 3 (plan only: daily buckets) queues a slot per trace, not a counted queue
  const uint32_t nw = slots ? (uint32_t)n_dev : ((uint32_t*)c->h_meta)[CTR_CX];
  if ((uint64_t)nb + nl > n_traces || nw > n_traces) return fail(c, ZDL_EDEVICE, "sparse: inconsistent tail counters");
  const uint64_t nseg = (uint64_t)lW + nb + nl + nw;
  if (nseg == 0) return ZDL_OK;
  HIP_TRY(c, c->seg_src.ensure(nseg));
  HIP_TRY(c, c->seg_n.ensure(nseg));
  HIP_TRY(c, c->seg_off.ensure(nseg));
  hipLaunchKernelGGL(k_seg_build, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s, c->lg_start.p, c->lg_n.p, lW,
                     c->big_list.p, off, c->tseg_big.p, nb, nl, (uint32_t)n_traces, c->cx_win.p, c->tseg_win.p, nw,
                     (uint64_t)2 * n_spans,
                     c->seg_src.p, c->seg_n.p, c->status.p);
  HIP_TRY(c, hipGetLastError());
  size_t need = 0;
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, need, c->seg_n.p, c->seg_off.p, (int)nseg, s));
  HIP_TRY(c, c->seg_tmp.ensure(need));
  HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(c->seg_tmp.p, need, c->seg_n.p, c->seg_off.p, (int)nseg, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_meta, c->seg_off.p + (nseg - 1), 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipMemcpyAsync((uint32_t*)c->h_meta + 1, c->seg_n.p + (nseg - 1), 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  const uint64_t E = (uint64_t)((uint32_t*)c->h_meta)[0] + ((uint32_t*)c->h_meta)[1];
  if (E > 4 * n_spans) return fail(c, ZDL_EDEVICE, "sparse: more links than the log holds");
  c->last_sparse_E = E;
  if (E == 0) return ZDL_OK;
  HIP_TRY(c, c->lin.ensure(E));
  hipLaunchKernelGGL(k_seg_copy, dim3((unsigned)((E + SEG_TILE - 1) / SEG_TILE)), dim3(256), 0, s, c->lg.p,
                     c->seg_src.p, c->seg_n.p, c->seg_off.p, nseg, E, c->lin.p);
  HIP_TRY(c, hipGetLastError());
  int kb = 1;
  while ((1ull << kb) < (uint64_t)c->rows * c->S) ++kb;  // daily buckets: the day rides in the cell
  HIP_TRY(c, sparse_accumulate(c->sw, c->acc, c->lin.p, E, kb + 1, s));
  return ZDL_OK;
}

// The device-wide big-trace tier (zdl_giant.inc), sparse contexts only. giant_prep runs right
// after k_link, before k_mid: k_g_prep_* split k_link's back list on the device's own count of it
// and its totals are copied to pinned memory behind an event; giant_run (after k_mid's launch)
// waits for that event only - k_mid keeps running meanwhile - and launches the tier's kernels,
// which queue behind k_mid. Arrays indexed by back-list entry are sized by the bound on the
// back list (every entry is longer than the wave tier's limit). Sets A.gstat / A.grest when the
// tier has giant traces; k_big / k_tail then skip the traces it linked.
static uint64_t giant_nl_bound(const Args& A, uint64_t n_spans, uint64_t n_traces) {
  const uint64_t lim = std::max<uint64_t>(A.wb_max, (uint64_t)WSMALL) + 1;  // back-list traces are longer
  return std::min<uint64_t>(n_traces, n_spans / lim + 1);
}
static int giant_prep(zdl_ctx* c, Args& A, uint64_t n_spans, uint64_t n_traces) {
  const hipStream_t s = c->stream;
  if (!c->h_gmeta) HIP_TRY(c, hipHostMalloc((void**)&c->h_gmeta, GM_WORDS * 4, hipHostMallocDefault));
  if (!c->gg_ev) HIP_TRY(c, hipEventCreateWithFlags(&c->gg_ev, hipEventDisableTiming));
  const uint64_t nl = giant_nl_bound(A, n_spans, n_traces);
  const uint64_t ntmax = n_spans / GT + nl + 1;
  HIP_TRY(c, c->gg_bi.ensure(nl));
  HIP_TRY(c, c->gg_n.ensure(nl));
  HIP_TRY(c, c->gg_tile0.ensure(nl));
  HIP_TRY(c, c->gg_bad.ensure(nl));
  HIP_TRY(c, c->gg_base.ensure(nl));
  HIP_TRY(c, c->gg_h0.ensure(nl));
  HIP_TRY(c, c->gg_root.ensure(nl));
  HIP_TRY(c, c->gg_tsroot.ensure(nl));
  HIP_TRY(c, c->gg_tsmin.ensure(nl));
  HIP_TRY(c, c->gg_rootidx.ensure(nl));
  HIP_TRY(c, c->gg_stat.ensure(n_traces));
  HIP_TRY(c, c->gg_tile_g.ensure(ntmax));
  HIP_TRY(c, c->gg_bstart.ensure(ntmax));
  HIP_TRY(c, c->gg_blen.ensure(ntmax));
  HIP_TRY(c, c->gg_meta.ensure(GM_WORDS));
  HIP_TRY(c, c->gg_rest.ensure(nl));
  GArgs& G = c->gg_args;
  G = GArgs{};
  G.bi = c->gg_bi.p;
  G.base = c->gg_base.p;
  G.n = c->gg_n.p;
  G.tile0 = c->gg_tile0.p;
  G.h0 = c->gg_h0.p;
  G.root = c->gg_root.p;
  G.rootidx = c->gg_rootidx.p;
  G.bad = c->gg_bad.p;
  G.tsroot = c->gg_tsroot.p;
  G.tsmin = c->gg_tsmin.p;
  G.tile_g = c->gg_tile_g.p;
  G.bstart = c->gg_bstart.p;
  G.blen = c->gg_blen.p;
  G.meta = c->gg_meta.p;
  G.gstat = c->gg_stat.p;
  G.gmin = (uint32_t)c->giant_min;
  G.rest = c->gg_rest.p;
  G.nl = (uint32_t)nl;
  HIP_TRY(c, hipMemsetAsync(c->gg_meta.p, 0, GM_WORDS * 4, s));
  const uint32_t nb = (uint32_t)((nl + GT - 1) / GT);
  HIP_TRY(c, c->gg_part32.ensure(4 * (size_t)nb));
  HIP_TRY(c, c->gg_part64.ensure(nb));
  hipLaunchKernelGGL(k_g_prep_count, dim3(nb), dim3(GT), 0, s, A, G, c->gg_part32.p, c->gg_part64.p);
  hipLaunchKernelGGL(k_g_prep_scan, dim3(1), dim3(GT), 0, s, A, G, nb, c->gg_part32.p, c->gg_part64.p);
  hipLaunchKernelGGL(k_g_prep_write, dim3(nb), dim3(GT), 0, s, A, G, (const uint32_t*)c->gg_part32.p,
                     (const unsigned long long*)c->gg_part64.p);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipMemcpyAsync(c->h_gmeta, c->gg_meta.p, GM_WORDS * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipEventRecord(c->gg_ev, s));
  c->gg_ntmax = ntmax;
  // every back-list entry has its verdict (giant or not) and the rest list is final: k_big and
  // k_tail take the rest list (k_g_par hands the traces the join rejects to k_tail's exact list
  // itself), so k_big need not wait for the tier
  A.gstat = c->gg_stat.p;
  A.grest = c->gg_rest.p;
  A.grest_n = c->gg_meta.p + GM_REST;
  return ZDL_OK;
}

static int giant_run(zdl_ctx* c, Args& A) {
  const hipStream_t s = c->stream;
  HIP_TRY(c, hipEventSynchronize(c->gg_ev));  // k_link and k_g_prep (k_mid may still run)
  GArgs& G = c->gg_args;
  const uint32_t ng = c->h_gmeta[GM_G], nt = c->h_gmeta[GM_NT], maxn = c->h_gmeta[GM_MAXN], nh = c->h_gmeta[GM_NH];
  if (ng == 0) return ZDL_OK;  // the rest list is the whole back list
  if (nt > c->gg_ntmax || maxn > (uint32_t)GMAXN || nh == 0xFFFFFFFFu)
    return fail(c, ZDL_EDEVICE, "giant tier: inconsistent sizes");
  HIP_TRY(c, c->gg_H.ensure(nh));
  G.H = c->gg_H.p;
  const uint32_t jgrid = std::min<uint32_t>(8 * ((nt + 7) / 8), (uint32_t)c->cus * 2);  // k_g_jump's grid
  const size_t jcap = (size_t)((8 * ((nt + 7) / 8) + jgrid - 1) / jgrid) * GT;           // (g_jump_cap)
  HIP_TRY(c, c->gg_jl0.ensure(jcap * jgrid));  // a block's segment holds its round-0 spans
  HIP_TRY(c, c->gg_jl1.ensure(jcap * jgrid));
  HIP_TRY(c, c->gg_jc.ensure(2 * (size_t)jgrid));
  G.jl[0] = c->gg_jl0.p;
  G.jl[1] = c->gg_jl1.p;
  G.jc[0] = c->gg_jc.p;
  G.jc[1] = c->gg_jc.p + jgrid;
  G.nt = nt;
  G.per = (nt + 7) / 8;
  const dim3 tg(8 * G.per), tb(GT);
  hipLaunchKernelGGL(k_g_hist, tg, tb, 0, s, A, G);
  hipLaunchKernelGGL(k_g_scan, dim3(std::min<uint32_t>(ng, (uint32_t)c->cus * 4)), dim3(BIG_WG), 0, s, A, G);
  hipLaunchKernelGGL(k_g_scatter, tg, tb, 0, s, A, G);
  hipLaunchKernelGGL(k_g_join, tg, tb, GHCAP * 16, s, A, G);
  hipLaunchKernelGGL(k_g_par, tg, tb, 0, s, A, G);
  // after r rounds of two hops a points at least 3^r generations up: enough once 3^r >= the
  // depth (<= n); rounds after convergence return at once (the flag)
  int rounds = 1;
  for (uint64_t reach = 3; reach < (uint64_t)maxn && rounds < GROUNDS_MAX; reach *= 3) ++rounds;
  const dim3 jg(jgrid);  // persistent; a multiple of 8 (8 * G.per = 8 * ceil(nt / 8))
  for (int r = 0; r < rounds; ++r) hipLaunchKernelGGL(k_g_jump, jg, tb, 0, s, A, G, r);
  hipLaunchKernelGGL(k_g_rules, tg, tb, 0, s, A, G);
  HIP_TRY(c, hipGetLastError());
  return ZDL_OK;
}

// A lazy put's k_mid / k_tail, when its k_link left them work (flag seq | FLAG_TAIL) or has not
// finished yet (then they run after it in stream order and find what there is; k_tail compacts
// and releases seq again). wait: spin for k_link first (zdl_link); otherwise never waits.
// k_big's two launches (small traces, four workgroups per CU; then the longer ones)
static int launch_big(zdl_ctx* c, void** kargs, int wmode) {
  hipError_t be = hipLaunchKernel((const void*)k_big<256>, dim3((unsigned)c->cus * 4), dim3(256), kargs,
                                  (size_t)KB_SMALL_LDS, c->stream);
  if (be == hipSuccess)
    be = hipLaunchKernel((const void*)k_big<TAIL_WG>, dim3(c->grid), dim3(TAIL_WG), kargs, tail_block_bytes(wmode),
                         c->stream);
  if (be != hipSuccess) {
    c->poisoned = true;
    return hip_fail(c, be, "k_big launch");
  }
  return ZDL_OK;
}

static int resolve_lazy(zdl_ctx* c, bool wait) {
  if (!c->lazy_pending) return ZDL_OK;
  c->lazy_pending = false;
  const volatile unsigned long long* f = c->h_flag;
  unsigned long long v = *f;
  for (uint32_t i = 1; wait && (v & ~FLAG_TAIL) != c->seq; ++i) {
    if ((i & 255) == 0 && hipStreamQuery(c->stream) != hipErrorNotReady) {
      v = *f;
      break;
    }
    __builtin_ia32_pause();
    v = *f;
  }
  if (v == c->seq) return ZDL_OK;  // complete: k_link's last workgroup compacted
  Args A = c->lazy_A;
  A.lazy = 0;
  void* kargs[] = {&A};
  if (A.wb_max) {
    hipLaunchKernelGGL(k_mid, dim3((unsigned)c->cus * 4), dim3(MID_WG), 4 * WB_CARVE, c->stream, A);
    const hipError_t me = hipGetLastError();
    if (me != hipSuccess) {
      c->poisoned = true;
      return hip_fail(c, me, "k_mid launch");
    }
  }
  if (A.bstat) {
    const int brc = launch_big(c, kargs, c->lazy_wmode);
    if (brc != ZDL_OK) return brc;
  }
  const hipError_t le = hipLaunchKernel(k_tail_fn(c->lazy_dense, c->lazy_wmode, 0), dim3(c->grid), dim3(TAIL_WG), kargs,
                                        tail_block_bytes(c->lazy_wmode), c->stream);
  if (le != hipSuccess) {
    c->poisoned = true;
    return hip_fail(c, le, "k_tail launch");
  }
  return ZDL_OK;
}

// Default pipeline: k_link streams every trace of <= WSMALL spans; k_tail re-runs the
// windows it queued, takes the traces it listed as longer than WSMALL and (small tables)
// compacts the table into the mapped buffer zdl_link reads.
static int put_spans_link(zdl_ctx* c, const zdl_span_cols* col, uint64_t n_spans, const uint64_t* off,
                          uint64_t n_traces, const uint64_t* n_traces_dev = nullptr) {
  {
    const int lrc = resolve_lazy(c, false);  // the previous lazy put's k_mid / k_tail first
    if (lrc != ZDL_OK) return lrc;
  }
  if (c->poisoned) return fail(c, ZDL_EDEVICE, "an earlier put failed between its kernels: call zdl_reset");
  const size_t SS = (size_t)c->rows * c->S;  // table cells (days * S * S with daily buckets)
  const int dense = SS <= (size_t)wdense_max(plan_only_mode(c) ? 0 : c->window);
  // k_link's table mode: dense LDS cells; else the emit log when the partitions fit (S <= 1024,
  // n_spans < 2^31: u32 positions); else the LDS hash with HBM spill
  int tm = dense ? TM_DENSE : (SS <= ((size_t)PMAX << PSHIFT) && n_spans < (1ull << 31) ? TM_LOG : TM_HASH);
  if (c->force_tm == TM_HASH && !dense) tm = TM_HASH;
  if (c->force_tm == TM_LOG && SS <= ((size_t)PMAX << PSHIFT) && n_spans < (1ull << 31)) tm = TM_LOG;
  const bool plan_only = plan_only_mode(c);  // k_link mode 3: k_tail counts every window
  // plan-only puts count in k_tail (table modes); insertion-order puts rank every addLink in the
  // global first-rank table by themselves, so they count in any mode k_link has (LOG included)
  if (plan_only || (c->ord && tm != TM_LOG)) tm = dense ? TM_DENSE : TM_HASH;
  if (c->sparse) {  // every link to a log, sorted and merged after k_tail (zdl_sparse.h)
    if (n_spans >= (1ull << 30)) return fail(c, ZDL_EINVAL, "sparse context: a put holds at most 2^30 spans");
    tm = TM_SORT;
  }
  const int grid = c->grid, lgrid = c->cus * lk::wgs_per_cu;  // k_link: two 16-wave workgroups per CU
  HIP_TRY(c, c->big_list.ensure(n_traces));
  HIP_TRY(c, c->big_stat.ensure(n_traces));
  HIP_TRY(c, c->big_exact_list.ensure(n_traces));
  // queued windows: at most one per trace; mode 3 (insertion order) uses one slot per trace
  HIP_TRY(c, c->cx_win.ensure(2 * ((c->ord || c->days) ? n_traces : std::min<uint64_t>(n_traces, n_spans))));
  Args A{};
  A.c = Cols{col->id, col->parent_id, col->local_svc, col->remote_svc, col->local_ip4, col->local_ip6,
             col->port_flags, col->timestamp};
  A.off = off;
  A.n_traces = n_traces;  // with n_traces_dev: an upper bound (sizes the queues)
  A.n_traces_dev = n_traces_dev;
  A.n_spans = n_spans;
  A.R = Ranks{c->nrank[0] ? c->rank[0].p : nullptr, c->nrank[1] ? c->rank[1].p : nullptr,
              c->nrank[2] ? c->rank[2].p : nullptr, c->nrank[0], c->nrank[1], c->nrank[2]};
  A.S = c->S;
  A.dense = dense;
  A.window = c->window;
  A.rows = c->rows;
  A.days = c->days;
  A.days_skip = c->days_skip ? 1u : 0u;
  A.day0 = c->day0;
  A.day_first = c->day_first.p;
  const int wmode = c->days ? 2 : c->window;  // k_tail's timestamp mode
  A.win_lo = c->win_lo;
  A.win_hi = c->win_hi;
  A.call = c->call.p;
  A.err = c->errc.p;
  A.big_list = c->big_list.p;
  A.bstat = c->ord ? nullptr : c->big_stat.p;  // k_big runs (insertion order: every big trace exact)
  A.exact = c->big_exact_list.p;
  const uint32_t ep = c->epoch & 1u;
  uint32_t* ctr = c->counters.p + ep * CTR_N;
  A.big_count = ctr + CTR_MID;
  A.large_count = ctr + CTR_LARGE;
  A.tick_large = ctr + CTR_TICK_LARGE;
  A.tick_mid = ctr + CTR_TICK_MID;
  A.retry_count = ctr + CTR_RETRY;
  A.tick_big = ctr + CTR_TICK_BIG;
  A.exact_n = ctr + CTR_EXACT;
  {
    static const uint32_t kbs = [] {
      const char* e = getenv("ZDL_KB_SMALL");  // A/B and tests: 0 = every trace in k_big<1024>
      return e ? (uint32_t)std::min<long>(std::max<long>(atol(e), 0), KB_SMALL) : (uint32_t)KB_SMALL;
    }();
    A.kb_small = kbs;
  }
  A.ctr_next = c->counters.p + (ep ^ 1u) * CTR_N;
  A.big_cap = (uint32_t)n_traces;
  A.status = c->status.p;
  A.small_max = WSMALL;
  A.cx_count = ctr + CTR_CX;
  A.cx_win = c->cx_win.p;
  A.cx_slots = plan_only ? 1u : 0u;
  A.skip = c->skip;
  A.prof = c->prof.p;
  // insertion order: mode 6 (first traces, then zdl_ord.inc's pass) on dense tables, mode 4
  // (every simple window ranked in k_link) otherwise: other tables, ZDL_FLAG_TREE_STREAM (its
  // breadth-first indexes come from mode 4's), or ZDL_ORD_MODE4=1 (A/B)
  static const bool ord_mode4 = getenv("ZDL_ORD_MODE4") != nullptr;
  const int omode = tm == TM_DENSE && !ord_mode4 && !(c->flags & ZDL_FLAG_TREE_STREAM) ? 6 : 4;
  const int lmode = plan_only ? 3 : c->ord ? omode : (c->flags & ZDL_FLAG_TREE_STREAM) ? 5 : (c->prof_on ? 1 : (c->skip ? 2 : 0));
  const uint32_t lW = (uint32_t)lgrid * (uint32_t)lk::waves(c->window, lmode);  // k_link's waves
  const uint32_t lP = (uint32_t)((SS + (1u << PSHIFT) - 1) >> PSHIFT);
  if (tm == TM_SORT) {  // k_link's segments in [0, 2n), k_tail's in [2n, 4n)
    HIP_TRY(c, c->lg.ensure(4 * n_spans));
    HIP_TRY(c, c->lg_start.ensure(lW));
    HIP_TRY(c, c->lg_n.ensure(lW));
    HIP_TRY(c, c->tseg_big.ensure(n_traces));
    HIP_TRY(c, c->tseg_win.ensure(std::min<uint64_t>(n_traces, n_spans)));
    A.lg = c->lg.p;
    A.lg_start = c->lg_start.p;
    A.lg_n = c->lg_n.p;
    A.sparse = 1;
    A.tlg = c->lg.p + 2 * n_spans;
    A.tseg_big = c->tseg_big.p;
    A.tseg_win = c->tseg_win.p;
  }
  if (tm == TM_LOG) {
    // the pool: every entry (at most 2 a span) plus one partial block per workgroup and partition
    const uint64_t bcap = (2 * n_spans + LBLK - 1) / LBLK + (uint64_t)lgrid * lP + 1;
    if (bcap * LBLK >= (1ull << 40) || bcap >= (1ull << 32)) return fail(c, ZDL_EINVAL, "LOG mode: put too large");
    HIP_TRY(c, c->lg.ensure(2 * n_spans));
    HIP_TRY(c, c->lg_pool.ensure(bcap * LBLK));
    HIP_TRY(c, c->lg_dir.ensure((size_t)lP * bcap));
    HIP_TRY(c, c->lg_bn.ensure(bcap));
    HIP_TRY(c, c->lg_start.ensure(lW));
    HIP_TRY(c, c->lg_n.ensure(lW));
    if (!c->lg_sets.p) {  // both counter sets start at zero; each put's k_hist3 clears the next one's
      HIP_TRY(c, c->lg_sets.ensure(2 * (PMAX + 2)));
      HIP_TRY(c, hipMemsetAsync(c->lg_sets.p, 0, 2 * (PMAX + 2) * 4, c->stream));
    }
    A.lg = c->lg.p;
    A.lg_start = c->lg_start.p;
    A.lg_n = c->lg_n.p;
    A.lg_pool = c->lg_pool.p;
    A.lg_dir = c->lg_dir.p;
    A.lg_bn = c->lg_bn.p;
    A.lg_set = c->lg_sets.p + (size_t)c->lg_par * (PMAX + 2);
    A.lg_bcap = (uint32_t)bcap;
    A.lg_P = lP;
    A.lg_W = lW;
  }
  // Every buffer of the put is allocated before its first kernel is launched: a failed
  // allocation then leaves the tables, the counter slots and the epoch untouched.
  HIP_TRY(c, c->b_id.ensure(n_spans));
  HIP_TRY(c, c->b_pid.ensure(n_spans));
  HIP_TRY(c, c->b_lsvc.ensure(n_spans));
  HIP_TRY(c, c->b_rsvc.ensure(n_spans));
  HIP_TRY(c, c->b_ip4.ensure(n_spans));
  HIP_TRY(c, c->b_ip6.ensure(n_spans));
  HIP_TRY(c, c->b_pf.ensure(n_spans));
  HIP_TRY(c, c->b_perm.ensure(n_spans));
  HIP_TRY(c, c->b_parent.ensure(n_spans));
  HIP_TRY(c, c->b_live.ensure(n_spans));
  HIP_TRY(c, c->b_hasc.ensure(n_spans));
  HIP_TRY(c, c->b_nm.ensure(n_spans));
  HIP_TRY(c, c->b_hk.ensure(2 * n_spans));
  HIP_TRY(c, c->b_hv.ensure(4 * n_spans));
  A.b_id = c->b_id.p;
  A.b_pid = c->b_pid.p;
  A.b_lsvc = c->b_lsvc.p;
  A.b_rsvc = c->b_rsvc.p;
  A.b_ip4 = c->b_ip4.p;
  A.b_ip6 = c->b_ip6.p;
  A.b_pf = c->b_pf.p;
  A.b_perm = c->b_perm.p;
  A.b_parent = c->b_parent.p;
  A.b_live = c->b_live.p;
  A.b_haschild = c->b_hasc.p;
  A.b_nm = c->b_nm.p;
  A.b_hk = c->b_hk.p;
  A.b_hv = c->b_hv.p;
  A.skip_simple = c->big_exact;
  // wave_big: not with insertion order / daily buckets (their big traces take the exact path)
  A.wb_max = (c->wave_big && !c->big_exact && !c->ord && !c->days) ? (uint32_t)WB_MAX : 0u;
  if (A.wb_max) {
    HIP_TRY(c, c->retry.ensure(n_traces));
    A.retry = c->retry.p;
  }
  if (c->flags & (ZDL_FLAG_TREE_EXPORT | ZDL_FLAG_TREE_STREAM)) {  // the last put's tree
    if ((c->flags & ZDL_FLAG_TREE_STREAM) && c->window)
      return fail(c, ZDL_EINVAL, "ZDL_FLAG_TREE_STREAM: no time window");
    HIP_TRY(c, c->tr_node.ensure(n_spans));
    HIP_TRY(c, c->tr_parent.ensure(n_spans));
    HIP_TRY(c, c->tr_bfs.ensure(n_spans));
    HIP_TRY(c, hipMemsetAsync(c->tr_node.p, 0xFF, n_spans * 4, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->tr_parent.p, 0xFF, n_spans * 4, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->tr_bfs.p, 0xFF, n_spans * 4, c->stream));
    HIP_TRY(c, c->tr_reason.ensure(n_spans));
    HIP_TRY(c, c->tr_anc.ensure(n_spans));
    HIP_TRY(c, c->tr_link.ensure(4 * n_spans));
    HIP_TRY(c, c->tr_sorted.ensure(n_spans));
    HIP_TRY(c, hipMemsetAsync(c->tr_reason.p, 0, n_spans, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->tr_anc.p, 0xFF, n_spans * 4, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->tr_link.p, 0xFF, n_spans * 16, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->tr_sorted.p, 0xFF, n_spans * 4, c->stream));
    A.tr_node = c->tr_node.p;
    A.tr_parent = c->tr_parent.p;
    A.tr_bfs = c->tr_bfs.p;
    A.tr_reason = c->tr_reason.p;
    A.tr_anc = c->tr_anc.p;
    A.tr_link = c->tr_link.p;
    A.tr_sorted = c->tr_sorted.p;
    c->tr_n = n_spans;
  }
  if (c->ord) {
    HIP_TRY(c, c->ord_n.ensure(1));
    const bool fresh_w = c->ord_w.n < SS;
    HIP_TRY(c, c->ord_w.ensure(SS));
    if (fresh_w) HIP_TRY(c, hipMemsetAsync(c->ord_w.p, 0xFF, SS * 8, c->stream));  // (k_ord_reduce's atomicMin)
    if (lmode == 6) {
      if ((lW + ORD_RED_G - 1) / ORD_RED_G > (uint32_t)ORD_RED_MAXW)
        return fail(c, ZDL_EINVAL, "insertion order: too many k_link waves for k_ord_reduce");
      // a wave records at most two pairs a span, and with its bitset of the cells seen at most
      // every cell once
      const uint64_t full = LK_ORD6_SEEN ? (uint64_t)lW * SS : ~0ull;
      A.ord_stride = 2 * n_spans <= full ? 0 : SS;
      HIP_TRY(c, c->ord_log.ensure(std::max<uint64_t>(1, std::min<uint64_t>(2 * n_spans, full))));
      HIP_TRY(c, c->ord_start.ensure(lW));
      HIP_TRY(c, c->ord_cnt.ensure(lW));
      A.ord_log = c->ord_log.p;
      A.ord_start = c->ord_start.p;
      A.ord_cnt = c->ord_cnt.p;
    }
    HIP_TRY(c, c->o_key.ensure(n_spans));
    HIP_TRY(c, c->o_fa.ensure(n_spans));
    HIP_TRY(c, c->o_fb.ensure(n_spans));
    HIP_TRY(c, c->o_bfs.ensure(n_spans));
    if (n_spans >= (1u << 21) - 1) HIP_TRY(c, c->o_pay.ensure(n_spans));  // a trace may need big_bfs's wide keys
    A.first = c->first.p;
    A.ord_w = c->ord_w.p;
    A.span_base = c->span_base;
    A.o_key = c->o_key.p;
    A.o_fa = c->o_fa.p;
    A.o_fb = c->o_fb.p;
    A.o_bfs = c->o_bfs.p;
    A.o_pay = n_spans >= (1u << 21) - 1 ? c->o_pay.p : nullptr;
  }
  const bool ordered = SS <= (size_t)COMPACT_WG * 8 && !c->ord && !c->days && !c->sparse;
  static const bool nolazy = getenv("ZDL_NOLAZY") != nullptr;
  // a lazy LOG put (round 5): k_mid / k_big / k_tail only when k_link's flag asks for them
  const bool lazy_log = tm == TM_LOG && lmode == 0 && !c->ord && !c->days && !nolazy &&
                        !(c->flags & ZDL_FLAG_TIMING_ALL);
  if (ordered || lazy_log) HIP_TRY(c, ensure_map(c));
  A.map = ordered && !getenv("ZDL_NOTAILMAP") ? c->d_map : nullptr;
  A.done = c->counters.p + CTR_DONE;
  if (A.map || lazy_log) {
    A.flag = c->d_flag;
    A.seq = c->seq + 1;
  }
  // lazy put (small dense tables, the production k_link): k_link's last workgroup compacts when
  // nothing is left for k_mid / k_tail, which then are not launched (resolve_lazy launches them
  // when its flag says so)
  A.lazy = (A.map && tm == TM_DENSE && lmode == 0 && !nolazy && !(c->flags & ZDL_FLAG_TIMING_ALL)) || lazy_log ? 1 : 0;
  void* kargs[] = {&A};
  ev_record(c, 0);
  ev_record(c, 1);
  // A failed launch poisons nothing yet either: no kernel of this put ran
  // (mode 3 on a sparse context runs the hash instantiation, k_link_fn: its LDS holds the table)
  HIP_TRY(c, hipLaunchKernel(k_link_fn(tm, c->window, lmode), dim3(lgrid), dim3(lk::waves(c->window, lmode) * 64), kargs,
                             link_block_bytes(lmode == 3 ? 0 : c->window, lmode == 3 && tm == TM_SORT ? TM_HASH : tm,
                                              lmode),
                             c->stream));
  ev_record(c, 7);
  c->last_log_lP = tm == TM_LOG ? lP : 0u;
  c->last_sparse_E = 0;
  if (tm == TM_LOG) {  // group the log by partition, count each partition in LDS (zdl_log.inc)
    // k_link's workgroups moved their entries into the block pool: one kernel counts them
    uint32_t* const set = A.lg_set;
    uint32_t* const next = c->lg_sets.p + (size_t)(c->lg_par ^ 1u) * (PMAX + 2);
    c->last_log_set = set;
    c->lg_par ^= 1u;
    hipLaunchKernelGGL(k_hist3, dim3((unsigned)c->cus), dim3(HIST2_WG), 0, c->stream, c->lg_pool.p, c->lg_dir.p,
                       c->lg_bn.p, (const uint32_t*)set, next, lP, A.lg_bcap, (uint64_t)SS, c->call.p, c->errc.p);
    const hipError_t ke = hipGetLastError();
    if (ke != hipSuccess) {
      c->poisoned = true;
      return hip_fail(c, ke, "LOG mode reduce launch");
    }
  }
  ev_record(c, 2);
  c->map_fresh = false;  // k_link has changed the table
  c->ordmap_fresh = false;
  if (A.lazy) {
    c->lazy_A = A;
    c->lazy_wmode = wmode;
    c->lazy_dense = dense;
    c->lazy_pending = true;
    c->seq = A.seq;
    c->span_base += n_spans;
    ++c->epoch;  // k_link's last workgroup (or k_tail) zeroes the other counter slots
    c->map_fresh = tm == TM_DENSE;  // (a LOG put compacts nothing into the mapped buffer)
    c->times.grid = (uint32_t)grid;
    return ZDL_OK;
  }
  const bool giant = c->sparse && c->giant_min > 0 && !c->ord && !c->days;
  if (giant) {  // the giant tier's split of the back list, before k_mid (giant_prep)
    const int grc = giant_prep(c, A, n_spans, n_traces);
    if (grc != ZDL_OK) {
      c->poisoned = true;  // k_link ran: the counter slots hold this put's counts
      return grc;
    }
  }
  if (A.wb_max) {  // big_list's front (WSMALL < n <= WB_MAX spans): one wave per trace
    hipLaunchKernelGGL(k_mid, dim3((unsigned)c->cus * 4), dim3(MID_WG), 4 * WB_CARVE, c->stream, A);
    const hipError_t me = hipGetLastError();
    if (me != hipSuccess) {
      c->poisoned = true;
      return hip_fail(c, me, "k_mid launch");
    }
  }
  ev_record(c, 3);
  if (giant) {  // the device-wide big-trace tier (its prep ran before k_mid)
    const int grc = giant_run(c, A);
    if (grc != ZDL_OK) {
      c->poisoned = true;  // k_link ran: the counter slots hold this put's counts
      return grc;
    }
  }
  ev_record(c, 8);
  if (A.bstat) {
    const int brc = launch_big(c, kargs, wmode);
    if (brc != ZDL_OK) return brc;
  }
  const hipError_t le = hipLaunchKernel(k_tail_fn(c->sparse ? 2 : dense, wmode, c->ord ? 1 : 0), dim3(grid),
                                        dim3(TAIL_WG), kargs, tail_block_bytes(wmode), c->stream);
  if (le != hipSuccess) {
    // k_link ran but k_tail did not: the counter slots are not re-zeroed and the table
    // holds part of the put. Mark the context: every put and link fails until zdl_reset.
    c->poisoned = true;
    return hip_fail(c, le, "k_tail launch");
  }
  if (A.map) c->seq = A.seq;
  if (lmode == 6) {  // the pairs' first simple traces ranked exactly (zdl_ord.inc); cx_win is free again
    hipLaunchKernelGGL(k_ord_reduce, dim3(ORD_RED_G), dim3(ORD_RED_WG), (size_t)SS * 8, c->stream, c->ord_log.p,
                       c->ord_start.p, c->ord_cnt.p, lW, (uint32_t)SS, c->ord_w.p);
    hipLaunchKernelGGL(k_ord_winners, dim3(1), dim3(OW_WG), 0, c->stream, c->ord_w.p, (uint32_t)SS, n_spans,
                       c->cx_win.p, c->ord_n.p, c->status.p);
    Args R = A;
    R.n_traces_dev = c->ord_n.p;
    R.cx_slots = 1;
    R.skip = A.skip | ORD_RANK_ONLY;
    void* rargs[] = {&R};
    hipError_t oe = hipGetLastError();
    if (oe == hipSuccess)
      oe = hipLaunchKernel(k_ord_rank_fn(c->window), dim3(grid), dim3(TAIL_WG), rargs, tail_block_bytes(c->window),
                           c->stream);
    if (oe != hipSuccess) {
      c->poisoned = true;  // the counts are in, the ranks are not
      return hip_fail(c, oe, "insertion order pass launch");
    }
  }
  ev_record(c, 4);
  if (c->sparse) {  // gather the put's log segments, sort, reduce and merge into the list
    // (plan only, k_link mode 3, logs nothing: its k_link instantiation keeps no segments)
    const int rc = sparse_finish(c, ep, plan_only ? 0u : lW, n_spans, n_traces, off, n_traces_dev, plan_only);
    if (rc != ZDL_OK) {
      c->span_base += n_spans;
      ++c->epoch;
      c->map_fresh = false;
  c->ordmap_fresh = false;
      return rc;
    }
  }
  c->span_base += n_spans;  // the next put's traces come after this one's
  if (c->ord && !c->days && SS <= MAP_CAP && !in_job(c)) {  // zdl_link's compaction, queued behind the put
    const int orc = ord_compact(c, c->call.p, c->errc.p, c->first.p);
    if (orc != ZDL_OK) return orc;
    c->ordmap_fresh = true;
  }
  ev_record(c, 9);
  ++c->epoch;  // k_tail zeroed the other counter slots
  c->map_fresh = A.map != nullptr;
  c->times.grid = (uint32_t)grid;
  return ZDL_OK;
}

// Ungrouped device columns: group by trace_lo (zdl_group.hip), gather the columns into
// grouped order, link with the device-side trace count.
static int put_spans_ungrouped(zdl_ctx* c, const zdl_span_cols* col, uint64_t n) {
  if (!col->trace_lo) return fail(c, ZDL_EINVAL, "ungrouped input needs the trace_lo column");
  if (n >= (1ull << 32)) return fail(c, ZDL_EINVAL, "ungrouped input too large (n_spans >= 2^32)");
  HIP_TRY(c, group_spans(c->grp, col->trace_lo, col->ord, n, c->stream));
  HIP_TRY(c, c->g_id.ensure(n));
  HIP_TRY(c, c->g_pid.ensure(n));
  HIP_TRY(c, c->g_lsvc.ensure(n));
  HIP_TRY(c, c->g_rsvc.ensure(n));
  HIP_TRY(c, c->g_ip4.ensure(n));
  HIP_TRY(c, c->g_ip6.ensure(n));
  HIP_TRY(c, c->g_pf.ensure(n));
  const bool with_ts = c->window || c->days;
  if (with_ts) HIP_TRY(c, c->g_ts.ensure(n));
  const Cols in{col->id, col->parent_id, col->local_svc, col->remote_svc, col->local_ip4, col->local_ip6,
                col->port_flags, with_ts ? col->timestamp : nullptr};
  hipLaunchKernelGGL(k_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, in, c->grp.perm, n,
                     c->g_id.p, c->g_pid.p, c->g_lsvc.p, c->g_rsvc.p, c->g_ip4.p, c->g_ip6.p, c->g_pf.p,
                     with_ts ? c->g_ts.p : nullptr);
  HIP_TRY(c, hipGetLastError());
  zdl_span_cols g{};
  g.id = c->g_id.p;
  g.parent_id = c->g_pid.p;
  g.local_svc = c->g_lsvc.p;
  g.remote_svc = c->g_rsvc.p;
  g.local_ip4 = c->g_ip4.p;
  g.local_ip6 = c->g_ip6.p;
  g.port_flags = c->g_pf.p;
  g.timestamp = with_ts ? c->g_ts.p : nullptr;
  return put_spans_link(c, &g, n, c->grp.off, n, c->grp.count);
}

// ------------------------------------------------------------------ span store
// A device-resident column store (the ingest side of InMemoryStorage):
// accepted spans are appended to HBM columns once, with their trace ids, timestamps and an
// alive byte; eviction and a query's trace selection run on the device (zdl_store.hip) and the
// selection is gathered and linked without leaving HBM.
struct zdl_store {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t cstream = nullptr;  // zdl_store_append: the columns the index does not read
  hipEvent_t cev = nullptr;
  std::string err;
  uint64_t n = 0, cap = 0, n_alive = 0;
  DevBuf<uint64_t> id, pid, lo, hi;
  DevBuf<int32_t> lsvc, rsvc, ip4, ip6;
  DevBuf<uint32_t> pf;
  DevBuf<int64_t> ts;
  DevBuf<uint8_t> alive;
  zdl::IndexWork iw;
  DevBuf<uint32_t> sel;  // the last zdl_store_select: positions in trace order
  DevBuf<uint64_t> sel_off;  // and its CSR trace offsets
  uint64_t sel_n = 0, sel_traces = 0;
  bool sel_valid = false;
};

}  // extern "C"
namespace {
template <class T>
hipError_t store_grow(DevBuf<T>& b, uint64_t keep, uint64_t cap, hipStream_t s) {
  DevBuf<T> nb;
  hipError_t e = nb.ensure(cap);
  if (e == hipSuccess && keep) e = hipMemcpyAsync(nb.p, b.p, keep * sizeof(T), hipMemcpyDeviceToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    nb.release();
    return e;
  }
  b.release();
  b = nb;
  return hipSuccess;
}
int store_fail(zdl_store* st, int code, const std::string& msg) {
  if (st) st->err = msg;
  return code;
}
int store_hip_fail(zdl_store* st, hipError_t e, const char* where) {
  return store_fail(st, e == hipErrorOutOfMemory ? ZDL_ENOMEM : ZDL_EDEVICE,
                    std::string(where) + ": " + hipGetErrorString(e));
}

__global__ void k_gather_index(const uint64_t* __restrict__ lo, const uint64_t* __restrict__ hi,
                               const uint8_t* __restrict__ alive, const uint32_t* __restrict__ idx, uint64_t n,
                               uint64_t* __restrict__ lo_o, uint64_t* __restrict__ hi_o, uint8_t* __restrict__ alive_o) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = idx[i];
  lo_o[i] = lo[j];
  hi_o[i] = hi[j];
  alive_o[i] = alive[j];
}

// The alive bytes of appended spans: 1, | 2 when the trace id is 128-bit (normalized to 32 hex
// characters) - from the caller's width bytes (already copied here) or else from hi != 0
__global__ void k_alive_init(uint8_t* __restrict__ alive, const uint64_t* __restrict__ hi, int from_wide, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool w = from_wide ? alive[i] != 0 : (hi != nullptr && hi[i] != 0);
  alive[i] = (uint8_t)(w ? 3u : 1u);
}

// Keeps the stored spans idx[0..n_keep) (device, ascending) and frees the rest.
hipError_t store_compact_dev(zdl_store* st, const uint32_t* idx, uint64_t n_keep) {
  const hipStream_t s = st->stream;
  const uint64_t cap = std::max<uint64_t>(2 * n_keep, 1 << 16);
  DevBuf<uint64_t> id, pid, lo, hi;
  DevBuf<int32_t> lsvc, rsvc, ip4, ip6;
  DevBuf<uint32_t> pf;
  DevBuf<int64_t> ts;
  DevBuf<uint8_t> alive;
  hipError_t e = id.ensure(cap);
  if (e == hipSuccess) e = pid.ensure(cap);
  if (e == hipSuccess) e = lo.ensure(cap);
  if (e == hipSuccess) e = hi.ensure(cap);
  if (e == hipSuccess) e = lsvc.ensure(cap);
  if (e == hipSuccess) e = rsvc.ensure(cap);
  if (e == hipSuccess) e = ip4.ensure(cap);
  if (e == hipSuccess) e = ip6.ensure(cap);
  if (e == hipSuccess) e = pf.ensure(cap);
  if (e == hipSuccess) e = ts.ensure(cap);
  if (e == hipSuccess) e = alive.ensure(cap);
  if (e == hipSuccess && n_keep) {
    const Cols in{st->id.p, st->pid.p, st->lsvc.p, st->rsvc.p, st->ip4.p, st->ip6.p, st->pf.p, st->ts.p};
    const dim3 g((unsigned)((n_keep + 255) / 256));
    hipLaunchKernelGGL(k_gather, g, dim3(256), 0, s, in, idx, n_keep, id.p, pid.p, lsvc.p, rsvc.p, ip4.p, ip6.p,
                       pf.p, ts.p);
    e = hipGetLastError();
    if (e == hipSuccess) {
      hipLaunchKernelGGL(k_gather_index, g, dim3(256), 0, s, st->lo.p, st->hi.p, st->alive.p, idx, n_keep, lo.p,
                         hi.p, alive.p);
      e = hipGetLastError();
    }
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    id.release(); pid.release(); lo.release(); hi.release(); lsvc.release(); rsvc.release(); ip4.release();
    ip6.release(); pf.release(); ts.release(); alive.release();
    return e;
  }
  st->id.release(); st->pid.release(); st->lo.release(); st->hi.release(); st->lsvc.release(); st->rsvc.release();
  st->ip4.release(); st->ip6.release(); st->pf.release(); st->ts.release(); st->alive.release();
  st->id = id; st->pid = pid; st->lo = lo; st->hi = hi; st->lsvc = lsvc; st->rsvc = rsvc; st->ip4 = ip4;
  st->ip6 = ip6; st->pf = pf; st->ts = ts; st->alive = alive;
  st->n = n_keep;
  st->cap = cap;
  st->sel_valid = false;
  st->iw.ni = 0;  // positions renumbered: the resident index is rebuilt by the next update
  return hipSuccess;
}

// Gathers the selection perm[0..n_sel) (device) of the store and links it as the CSR traces
// off[0..n_traces] (device), like zdl_put_spans on the gathered columns.
int put_stored_dev(zdl_ctx* c, const zdl_store* st, const uint32_t* perm, uint64_t n_sel, const uint64_t* off,
                   uint64_t n_traces) {
  const hipStream_t s = c->stream;
  HIP_TRY(c, c->g_id.ensure(n_sel));
  HIP_TRY(c, c->g_pid.ensure(n_sel));
  HIP_TRY(c, c->g_lsvc.ensure(n_sel));
  HIP_TRY(c, c->g_rsvc.ensure(n_sel));
  HIP_TRY(c, c->g_ip4.ensure(n_sel));
  HIP_TRY(c, c->g_ip6.ensure(n_sel));
  HIP_TRY(c, c->g_pf.ensure(n_sel));
  const bool with_ts = c->window || c->days;
  if (with_ts) HIP_TRY(c, c->g_ts.ensure(n_sel));
  const Cols in{st->id.p, st->pid.p, st->lsvc.p, st->rsvc.p, st->ip4.p, st->ip6.p, st->pf.p,
                with_ts ? st->ts.p : nullptr};
  hipLaunchKernelGGL(k_gather, dim3((unsigned)((n_sel + 255) / 256)), dim3(256), 0, s, in, perm, n_sel,
                     c->g_id.p, c->g_pid.p, c->g_lsvc.p, c->g_rsvc.p, c->g_ip4.p, c->g_ip6.p, c->g_pf.p,
                     with_ts ? c->g_ts.p : nullptr);
  HIP_TRY(c, hipGetLastError());
  zdl_span_cols g{};
  g.id = c->g_id.p;
  g.parent_id = c->g_pid.p;
  g.local_svc = c->g_lsvc.p;
  g.remote_svc = c->g_rsvc.p;
  g.local_ip4 = c->g_ip4.p;
  g.local_ip6 = c->g_ip6.p;
  g.port_flags = c->g_pf.p;
  g.timestamp = with_ts ? c->g_ts.p : nullptr;
  const int rc = put_spans_link(c, &g, n_sel, off, n_traces);
  if (rc != ZDL_OK) return rc;
  return zdl_sync(c);
}
}  // namespace
extern "C" {

zdl_store* zdl_store_create(int device) {
  zdl_store* st = new zdl_store();
  st->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&st->cstream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&st->cev, hipEventDisableTiming) != hipSuccess) {
    if (st->cstream) (void)hipStreamDestroy(st->cstream);
    if (st->stream) (void)hipStreamDestroy(st->stream);
    g_create_error = "zdl_store_create: device init failed";
    delete st;
    return nullptr;
  }
  return st;
}

void zdl_store_destroy(zdl_store* st) {
  if (!st) return;
  (void)hipSetDevice(st->device);
  (void)hipStreamSynchronize(st->stream);
  st->id.release(); st->pid.release(); st->lo.release(); st->hi.release(); st->lsvc.release(); st->rsvc.release();
  st->ip4.release(); st->ip6.release(); st->pf.release(); st->ts.release(); st->alive.release();
  st->sel.release(); st->sel_off.release();
  st->iw.release();
  (void)hipStreamSynchronize(st->cstream);
  (void)hipEventDestroy(st->cev);
  (void)hipStreamDestroy(st->cstream);
  (void)hipStreamDestroy(st->stream);
  delete st;
}

const char* zdl_store_last_error(const zdl_store* st) { return st ? st->err.c_str() : "null store"; }

uint64_t zdl_store_size(const zdl_store* st) { return st ? st->n : 0; }

uint64_t zdl_store_alive(const zdl_store* st) { return st ? st->n_alive : 0; }

int zdl_store_clear(zdl_store* st) {
  if (!st) return ZDL_EINVAL;
  st->n = st->n_alive = 0;
  st->sel_valid = false;
  st->iw.ni = 0;
  return ZDL_OK;
}

int zdl_store_append_ids(zdl_store* st, const zdl_span_cols* col, const uint64_t* trace_hi, const uint8_t* trace_wide,
                         uint64_t n) {
  if (!st || !col) return ZDL_EINVAL;
  if (n == 0) return ZDL_OK;
  if (!col->id || !col->parent_id || !col->local_svc || !col->remote_svc || !col->local_ip4 || !col->local_ip6 ||
      !col->port_flags)
    return store_fail(st, ZDL_EINVAL, "zdl_store_append: missing column");
  if (st->n + n >= (1ull << 31)) return store_fail(st, ZDL_EINVAL, "zdl_store_append: store limited to 2^31 spans");
  (void)hipGetLastError();
  hipError_t e = hipSetDevice(st->device);
  const hipStream_t s = st->stream;
  if (e == hipSuccess && st->n + n > st->cap) {  // grow by doubling (HBM is large; appends stay O(1))
    const uint64_t cap = std::max<uint64_t>(st->n + n, std::max<uint64_t>(2 * st->cap, 1 << 16));
    if (e == hipSuccess) e = store_grow(st->id, st->n, cap, s);
    if (e == hipSuccess) e = store_grow(st->pid, st->n, cap, s);
    if (e == hipSuccess) e = store_grow(st->lo, st->n, cap, s);
    if (e == hipSuccess) e = store_grow(st->hi, st->n, cap, s);
    if (e == hipSuccess) e = store_grow(st->lsvc, st->n, cap, s);
    if (e == hipSuccess) e = store_grow(st->rsvc, st->n, cap, s);
    if (e == hipSuccess) e = store_grow(st->ip4, st->n, cap, s);
    if (e == hipSuccess) e = store_grow(st->ip6, st->n, cap, s);
    if (e == hipSuccess) e = store_grow(st->pf, st->n, cap, s);
    if (e == hipSuccess) e = store_grow(st->ts, st->n, cap, s);
    if (e == hipSuccess) e = store_grow(st->alive, st->n, cap, s);
    if (e == hipSuccess) st->cap = cap;
  }
  const uint64_t o = st->n;
  // The trace index reads trace_lo and the timestamps only: they cross PCIe first, the index
  // update (sort + merge) runs on the stream while the other columns cross on cstream.
  if (e == hipSuccess)
    e = col->trace_lo ? hipMemcpyAsync(st->lo.p + o, col->trace_lo, n * 8, hipMemcpyDefault, s)
                      : hipMemsetAsync(st->lo.p + o, 0, n * 8, s);
  if (e == hipSuccess)
    e = col->timestamp ? hipMemcpyAsync(st->ts.p + o, col->timestamp, n * 8, hipMemcpyDefault, s)
                       : hipMemsetAsync(st->ts.p + o, 0, n * 8, s);
  if (e == hipSuccess) e = hipEventRecord(st->cev, s);  // (and the growth's copies before it)
  // the resident trace index takes the batch in (sorted, merged: the TreeMap inserts of
  // InMemoryStorage.accept, IMS:156-181), so a query only filters and orders traces
  if (e == hipSuccess) e = zdl::index_update(st->iw, st->lo.p, st->ts.p, st->n + n, s);
  const hipStream_t cs = st->cstream;
  if (e == hipSuccess) e = hipStreamWaitEvent(cs, st->cev, 0);
  if (e == hipSuccess) e = hipMemcpyAsync(st->id.p + o, col->id, n * 8, hipMemcpyDefault, cs);
  if (e == hipSuccess) e = hipMemcpyAsync(st->pid.p + o, col->parent_id, n * 8, hipMemcpyDefault, cs);
  if (e == hipSuccess)
    e = trace_hi ? hipMemcpyAsync(st->hi.p + o, trace_hi, n * 8, hipMemcpyDefault, cs)
                 : hipMemsetAsync(st->hi.p + o, 0, n * 8, cs);
  if (e == hipSuccess) e = hipMemcpyAsync(st->lsvc.p + o, col->local_svc, n * 4, hipMemcpyDefault, cs);
  if (e == hipSuccess) e = hipMemcpyAsync(st->rsvc.p + o, col->remote_svc, n * 4, hipMemcpyDefault, cs);
  if (e == hipSuccess) e = hipMemcpyAsync(st->ip4.p + o, col->local_ip4, n * 4, hipMemcpyDefault, cs);
  if (e == hipSuccess) e = hipMemcpyAsync(st->ip6.p + o, col->local_ip6, n * 4, hipMemcpyDefault, cs);
  if (e == hipSuccess) e = hipMemcpyAsync(st->pf.p + o, col->port_flags, n * 4, hipMemcpyDefault, cs);
  // alive bytes: 1, | 2 for a 128-bit trace id (the strict grouping's width bit)
  if (e == hipSuccess && trace_wide) e = hipMemcpyAsync(st->alive.p + o, trace_wide, n, hipMemcpyDefault, cs);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_alive_init, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, cs, st->alive.p + o,
                       trace_hi ? st->hi.p + o : nullptr, trace_wide ? 1 : 0, n);
    e = hipGetLastError();
  }
  {  // the columns are borrowed for the call only: both streams finish before it returns
    const hipError_t e1 = hipStreamSynchronize(cs);
    const hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e1 != hipSuccess ? e1 : e2;
  }
  if (e != hipSuccess) return store_hip_fail(st, e, "zdl_store_append");
  st->n += n;
  st->n_alive += n;
  st->sel_valid = false;
  return ZDL_OK;
}

int zdl_store_append_traced(zdl_store* st, const zdl_span_cols* col, const uint64_t* trace_hi, uint64_t n) {
  return zdl_store_append_ids(st, col, trace_hi, nullptr, n);
}

int zdl_store_append(zdl_store* st, const zdl_span_cols* col, uint64_t n) {
  return zdl_store_append_ids(st, col, nullptr, nullptr, n);
}

int zdl_store_compact(zdl_store* st, const uint32_t* keep, uint64_t n_keep) {
  if (!st || (n_keep && !keep)) return ZDL_EINVAL;
  if (n_keep > st->n) return store_fail(st, ZDL_EINVAL, "zdl_store_compact: more positions than stored spans");
  for (uint64_t i = 0; i < n_keep; ++i)
    if (keep[i] >= st->n || (i && keep[i] <= keep[i - 1]))
      return store_fail(st, ZDL_EINVAL, "zdl_store_compact: positions must ascend inside the store");
  (void)hipGetLastError();
  hipError_t e = hipSetDevice(st->device);
  DevBuf<uint32_t> idx;
  if (e == hipSuccess) e = idx.ensure(std::max<uint64_t>(n_keep, 1));
  if (e == hipSuccess && n_keep) e = hipMemcpyAsync(idx.p, keep, n_keep * 4, hipMemcpyHostToDevice, st->stream);
  if (e == hipSuccess) e = store_compact_dev(st, idx.p, n_keep);
  uint64_t alive = 0;
  if (e == hipSuccess) e = zdl::index_alive(st->iw, st->alive.p, st->n, idx.p, &alive, st->stream);
  idx.release();
  if (e != hipSuccess) return store_hip_fail(st, e, "zdl_store_compact");
  st->n_alive = alive;
  return ZDL_OK;
}

int zdl_store_compact_evicted(zdl_store* st) {
  if (!st) return ZDL_EINVAL;
  if (st->n_alive == st->n) return ZDL_OK;
  (void)hipGetLastError();
  hipError_t e = hipSetDevice(st->device);
  DevBuf<uint32_t> idx;
  uint64_t m = 0;
  if (e == hipSuccess) e = idx.ensure(std::max<uint64_t>(st->n, 1));
  if (e == hipSuccess) e = zdl::index_alive(st->iw, st->alive.p, st->n, idx.p, &m, st->stream);
  if (e == hipSuccess) e = store_compact_dev(st, idx.p, m);
  idx.release();
  if (e != hipSuccess) return store_hip_fail(st, e, "zdl_store_compact_evicted");
  st->n_alive = m;
  return ZDL_OK;
}

int zdl_store_evict(zdl_store* st, uint64_t to_recover, uint64_t* evicted) {
  if (!st) return ZDL_EINVAL;
  if (evicted) *evicted = 0;
  if (to_recover == 0) return ZDL_OK;
  (void)hipGetLastError();
  hipError_t e = hipSetDevice(st->device);
  uint64_t ev = 0;
  bool exhausted = false;
  if (e == hipSuccess)
    e = zdl::index_evict(st->iw, st->lo.p, st->ts.p, st->alive.p, st->n, st->n_alive, to_recover, &ev, &exhausted,
                         st->stream);
  if (e != hipSuccess) return store_hip_fail(st, e, "zdl_store_evict");
  st->n_alive -= ev;
  st->sel_valid = false;
  if (evicted) *evicted = ev;
  if (exhausted)
    return store_fail(st, ZDL_EREF_NSE, "zdl_store_evict: the store ran empty (TreeMap.lastKey of an empty map)");
  return ZDL_OK;
}

int zdl_store_select(zdl_store* st, int mode, uint64_t* n_sel, uint64_t* n_traces) {
  if (!st) return ZDL_EINVAL;
  if (mode != ZDL_SELECT_NEWEST && mode != ZDL_SELECT_ALL && mode != ZDL_SELECT_ALL_STRICT)
    return store_fail(st, ZDL_EINVAL, "zdl_store_select: unknown mode");
  (void)hipGetLastError();
  st->sel_valid = false;
  hipError_t e = hipSetDevice(st->device);
  if (e == hipSuccess) e = st->sel.ensure(std::max<uint64_t>(st->n, 1));
  if (e == hipSuccess) e = st->sel_off.ensure(st->n + 1);
  const int m = mode == ZDL_SELECT_NEWEST ? zdl::SEL_NEWEST : mode == ZDL_SELECT_ALL ? zdl::SEL_ALL : zdl::SEL_ALL_STRICT;
  if (e == hipSuccess)
    e = zdl::index_select(st->iw, st->lo.p, st->hi.p, st->ts.p, st->alive.p, st->n, st->n_alive, m, st->sel.p,
                          st->sel_off.p,
                          &st->sel_n, &st->sel_traces, st->stream);
  if (e != hipSuccess) return store_hip_fail(st, e, "zdl_store_select");
  st->sel_valid = true;
  if (n_sel) *n_sel = st->sel_n;
  if (n_traces) *n_traces = st->sel_traces;
  return ZDL_OK;
}

int zdl_store_selection(const zdl_store* cst, uint32_t* perm, uint64_t* trace_offsets) {
  zdl_store* st = const_cast<zdl_store*>(cst);
  if (!st) return ZDL_EINVAL;
  if (!st->sel_valid) return store_fail(st, ZDL_EINVAL, "zdl_store_selection: no current selection");
  hipError_t e = hipSetDevice(st->device);
  if (e == hipSuccess && perm && st->sel_n)
    e = hipMemcpyAsync(perm, st->sel.p, st->sel_n * 4, hipMemcpyDeviceToHost, st->stream);
  if (e == hipSuccess && trace_offsets && st->sel_traces)
    e = hipMemcpyAsync(trace_offsets, st->sel_off.p, (st->sel_traces + 1) * 8, hipMemcpyDeviceToHost, st->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(st->stream);
  if (e != hipSuccess) return store_hip_fail(st, e, "zdl_store_selection");
  if (trace_offsets && !st->sel_traces) trace_offsets[0] = 0;
  return ZDL_OK;
}

int zdl_put_selection(zdl_ctx* c, const zdl_store* st) {
  if (!c || !st) return fail(c, ZDL_EINVAL, "null argument");
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_put_selection: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) return fail(c, ZDL_EINVAL, "zdl_put_selection: a store lives on one device");
  if (st->device != c->device) return fail(c, ZDL_EINVAL, "zdl_put_selection: store and context on different devices");
  if (!st->sel_valid) return fail(c, ZDL_EINVAL, "zdl_put_selection: no current selection (zdl_store_select)");
  if (st->sel_traces == 0) return ZDL_OK;
  HIP_TRY(c, enter(c));
  {  // a lazy put's k_mid / k_tail read the previous put's columns and scratch: launched first
    const int lrc = resolve_lazy(c, false);
    if (lrc != ZDL_OK) return lrc;
  }
  HIP_TRY(c, hipStreamSynchronize(st->stream));
  return put_stored_dev(c, st, st->sel.p, st->sel_n, st->sel_off.p, st->sel_traces);
}

int zdl_put_stored(zdl_ctx* c, const zdl_store* st, const uint32_t* perm, uint64_t n_sel, const uint64_t* off,
                   uint64_t n_traces) {
  if (!c || !st || (n_sel && !perm) || !off) return fail(c, ZDL_EINVAL, "null argument");
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_put_stored: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) return fail(c, ZDL_EINVAL, "zdl_put_stored: a store lives on one device");
  if (st->device != c->device) return fail(c, ZDL_EINVAL, "zdl_put_stored: store and context on different devices");
  if (n_traces == 0 || n_sel == 0) return ZDL_OK;
  if (off[0] != 0 || off[n_traces] != n_sel) return fail(c, ZDL_EINVAL, "trace offsets must span [0, n_sel]");
  for (uint64_t t = 0; t < n_traces; ++t)
    if (off[t + 1] < off[t]) return fail(c, ZDL_EINVAL, "trace offsets are not non-decreasing");
  for (uint64_t i = 0; i < n_sel; ++i)
    if (perm[i] >= st->n) return fail(c, ZDL_EINVAL, "zdl_put_stored: selection outside the store");
  HIP_TRY(c, enter(c));
  {  // a lazy put's k_mid / k_tail read h_off / h_ord: launched before they are regrown or refilled
    const int lrc = resolve_lazy(c, false);
    if (lrc != ZDL_OK) return lrc;
  }
  HIP_TRY(c, hipStreamSynchronize(st->stream));
  HIP_TRY(c, c->h_ord.ensure(n_sel));
  HIP_TRY(c, c->h_off.ensure(n_traces + 1));
  HIP_TRY(c, hipMemcpyAsync(c->h_ord.p, perm, n_sel * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->h_off.p, off, (n_traces + 1) * 8, hipMemcpyHostToDevice, c->stream));
  return put_stored_dev(c, st, c->h_ord.p, n_sel, c->h_off.p, n_traces);
}

int zdl_put_spans_device(zdl_ctx* c, const zdl_span_cols* col, uint64_t n_spans, const uint64_t* off,
                         uint64_t n_traces) {
  if (!c || !col) return fail(c, ZDL_EINVAL, "null argument");
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_put_spans_device: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty())
    return fail(c, ZDL_EINVAL, "zdl_put_spans_device: a device group takes zdl_put_spans or zdl_put_spans_device_multi");
  if (n_spans == 0 || (off && n_traces == 0)) return ZDL_OK;
  if (!col->id || !col->parent_id || !col->local_svc || !col->remote_svc || !col->local_ip4 ||
      !col->local_ip6 || !col->port_flags)
    return fail(c, ZDL_EINVAL, "missing column");
  if ((c->window || c->days) && !col->timestamp)
    return fail(c, ZDL_EINVAL, "window or days set but no timestamp column");
  // k_link plans its windows in 32-bit positions: a put holds at most 2^32 - 129 spans (split a
  // larger input into several puts; the counts accumulate)
  if (n_traces >= 0xffffffffull || n_spans > (1ull << 32) - 129) return fail(c, ZDL_EINVAL, "input too large");
  HIP_TRY(c, enter(c));
  {  // a lazy put's k_mid / k_tail read the previous put's columns and scratch: launched first
    const int lrc = resolve_lazy(c, false);
    if (lrc != ZDL_OK) return lrc;
  }
  if (!off) return put_spans_ungrouped(c, col, n_spans);
  return put_spans_link(c, col, n_spans, off, n_traces);
}

int zdl_sync(zdl_ctx* c) {
  if (!c) return ZDL_EINVAL;
  if (c->link_pending < 0)
    if (const int frc = stage_flush(c)) return frc;
  if (!c->sub.empty()) return group_each(c, [&](zdl_ctx* s) { return zdl_sync(s); });
  HIP_TRY(c, enter(c));
  {
    const int lrc = resolve_lazy(c, false);
    if (lrc != ZDL_OK) return lrc;
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  uint32_t st = 0;
  HIP_TRY(c, hipMemcpy(&st, c->status.p, 4, hipMemcpyDeviceToHost));
  put_times(c);
  return status_code(c, st);
}

int zdl_put_spans(zdl_ctx* c, const zdl_span_cols* col, uint64_t n_spans, const uint64_t* off,
                  uint64_t n_traces) {
  if (!c || !col) return fail(c, ZDL_EINVAL, "null argument");
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_put_spans: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) return group_put(c, col, n_spans, off, n_traces);
  if (off) {
    if (n_traces == 0) return ZDL_OK;
    if (off[0] != 0 || off[n_traces] != n_spans) return fail(c, ZDL_EINVAL, "trace offsets must span [0, n_spans]");
    for (uint64_t t = 0; t < n_traces; ++t)
      if (off[t + 1] < off[t]) return fail(c, ZDL_EINVAL, "trace offsets are not non-decreasing");
  } else if (!col->trace_lo) {
    return fail(c, ZDL_EINVAL, "ungrouped input needs the trace_lo column");
  }
  if (n_spans == 0) return ZDL_OK;
  HIP_TRY(c, enter(c));
  {  // a lazy put's k_mid / k_tail read the h_* columns: launched before they are regrown or refilled
    const int lrc = resolve_lazy(c, false);
    if (lrc != ZDL_OK) return lrc;
  }
  HIP_TRY(c, c->h_id.ensure(n_spans));
  HIP_TRY(c, c->h_pid.ensure(n_spans));
  HIP_TRY(c, c->h_lsvc.ensure(n_spans));
  HIP_TRY(c, c->h_rsvc.ensure(n_spans));
  HIP_TRY(c, c->h_ip4.ensure(n_spans));
  HIP_TRY(c, c->h_ip6.ensure(n_spans));
  HIP_TRY(c, c->h_pf.ensure(n_spans));
  if (off) HIP_TRY(c, c->h_off.ensure(n_traces + 1));
  hipStream_t s = c->stream;
  HIP_TRY(c, hipMemcpyAsync(c->h_id.p, col->id, n_spans * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_pid.p, col->parent_id, n_spans * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_lsvc.p, col->local_svc, n_spans * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_rsvc.p, col->remote_svc, n_spans * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_ip4.p, col->local_ip4, n_spans * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_ip6.p, col->local_ip6, n_spans * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->h_pf.p, col->port_flags, n_spans * 4, hipMemcpyHostToDevice, s));
  zdl_span_cols d{};
  if (off) {
    HIP_TRY(c, hipMemcpyAsync(c->h_off.p, off, (n_traces + 1) * 8, hipMemcpyHostToDevice, s));
  } else {  // grouped on the device
    HIP_TRY(c, c->h_lo.ensure(n_spans));
    HIP_TRY(c, hipMemcpyAsync(c->h_lo.p, col->trace_lo, n_spans * 8, hipMemcpyHostToDevice, s));
    d.trace_lo = c->h_lo.p;
    if (col->ord) {
      HIP_TRY(c, c->h_ord.ensure(n_spans));
      HIP_TRY(c, hipMemcpyAsync(c->h_ord.p, col->ord, n_spans * 4, hipMemcpyHostToDevice, s));
      d.ord = c->h_ord.p;
    }
  }
  d.id = c->h_id.p;
  d.parent_id = c->h_pid.p;
  d.local_svc = c->h_lsvc.p;
  d.remote_svc = c->h_rsvc.p;
  d.local_ip4 = c->h_ip4.p;
  d.local_ip6 = c->h_ip6.p;
  d.port_flags = c->h_pf.p;
  if (c->window || c->days) {
    if (!col->timestamp) return fail(c, ZDL_EINVAL, "window or days set but no timestamp column");
    HIP_TRY(c, c->h_ts.ensure(n_spans));
    HIP_TRY(c, hipMemcpyAsync(c->h_ts.p, col->timestamp, n_spans * 8, hipMemcpyHostToDevice, s));
    d.timestamp = c->h_ts.p;
  }
  int rc = zdl_put_spans_device(c, &d, n_spans, off ? c->h_off.p : nullptr, n_traces);
  if (rc != ZDL_OK) return rc;
  return zdl_sync(c);
}

int zdl_reset(zdl_ctx* c) {
  if (!c) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_reset: a started link is not finished (zdl_link_finish)");
  stage_drop(c);  // traces staged by zdl_put_trace before the reset are dropped with the counts
  if (!c->sub.empty()) return group_each(c, [&](zdl_ctx* s) { return zdl_reset(s); });
  HIP_TRY(c, enter(c));
  {
    const int lrc = resolve_lazy(c, false);  // its counter slots must be left as k_tail leaves them
    if (lrc != ZDL_OK) return lrc;
  }
  if (c->poisoned) {  // the counter slots may hold a half-finished put's counts
    HIP_TRY(c, hipMemsetAsync(c->counters.p, 0, (CTR_DONE + 1) * 4, c->stream));
    if (c->lg_sets.p) HIP_TRY(c, hipMemsetAsync(c->lg_sets.p, 0, 2 * (PMAX + 2) * 4, c->stream));
    if (c->ord_w.p) HIP_TRY(c, hipMemsetAsync(c->ord_w.p, 0xFF, c->ord_w.n * 8, c->stream));  // all ones between puts
    c->poisoned = false;
  }
  const size_t SS = c->sparse ? 0 : (size_t)c->rows * c->S;  // sparse: only the status word
  c->acc.n = 0;
  hipLaunchKernelGGL(k_zero_tables, dim3((unsigned)std::max<size_t>((SS + 255) / 256, 1)), dim3(256), 0, c->stream,
                     c->call.p, c->errc.p, (uint64_t)SS, c->status.p, c->ord ? c->first.p : nullptr);
  c->span_base = 0;
  if (c->days) HIP_TRY(c, hipMemsetAsync(c->day_first.p, 0xff, (size_t)c->days * 8, c->stream));
  HIP_TRY(c, hipGetLastError());
  c->map_fresh = false;
  c->ordmap_fresh = false;
  return ZDL_OK;  // stream-ordered: no host wait
}

static void sort_output(zdl_ctx* c, size_t n) {
  const std::vector<int32_t>& r = c->host_rank[0];
  auto rk = [&](int32_t id) -> int64_t { return (size_t)id < r.size() ? r[id] : id; };
  std::vector<uint32_t> idx(n);
  for (size_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
  std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
    const int64_t pa = rk(c->out_p[a]), pb = rk(c->out_p[b]);
    if (pa != pb) return pa < pb;
    return rk(c->out_c[a]) < rk(c->out_c[b]);
  });
  std::vector<int32_t> p(n), ch(n);
  std::vector<int64_t> ca(n), er(n);
  for (size_t i = 0; i < n; ++i) {
    p[i] = c->out_p[idx[i]];
    ch[i] = c->out_c[idx[i]];
    ca[i] = c->out_call[idx[i]];
    er[i] = c->out_err[idx[i]];
  }
  c->out_p.swap(p);
  c->out_c.swap(ch);
  c->out_call.swap(ca);
  c->out_err.swap(er);
}

// zdl_link in ZDL_ORDER_INSERTION: the non-zero cells with their first-addLink ranks
// (k_merge_compact over the context's tables), ordered by rank.
// k_ord_compact of (call, errc, first_rank) into the mapped buffer h_ordmap (tables of at most
// MAP_CAP cells), queued on the context's stream
static int ord_compact(zdl_ctx* c, const unsigned long long* call, const unsigned long long* errc,
                       const unsigned long long* first_rank) {
  const uint64_t SS = (uint64_t)c->rows * c->S;
  if (!c->h_ordmap) {
    HIP_TRY(c, hipHostMalloc((void**)&c->h_ordmap, 16 + 32 * MAP_CAP, hipHostMallocMapped | hipHostMallocCoherent));
    HIP_TRY(c, hipHostGetDevicePointer((void**)&c->d_ordmap, c->h_ordmap, 0));
  }
  if (!c->oc_done.p) {
    HIP_TRY(c, c->oc_done.ensure(1));
    HIP_TRY(c, hipMemsetAsync(c->oc_done.p, 0, 4, c->stream));
  }
  HIP_TRY(c, c->oc_rank.ensure(MAP_CAP));
  HIP_TRY(c, c->oc_cell.ensure(MAP_CAP));
  hipLaunchKernelGGL(k_ord_compact, dim3(ORD_SORT_G), dim3(OC_WG), 0, c->stream, call, errc, first_rank,
                     (uint32_t)SS, c->S, c->status.p, c->d_ordmap, c->oc_rank.p, c->oc_cell.p, c->oc_done.p);
  HIP_TRY(c, hipGetLastError());
  return ZDL_OK;
}

static int link_insertion(zdl_ctx* c, zdl_links* out, const unsigned long long* call,
                          const unsigned long long* errc, const unsigned long long* first_rank) {
  const uint64_t SS = (uint64_t)c->rows * c->S;
  if (SS <= MAP_CAP) {  // one kernel into mapped memory (queued by the put already when fresh), one wait
    if (!(c->ordmap_fresh && call == c->call.p)) {
      const int orc = ord_compact(c, call, errc, first_rank);
      if (orc != ZDL_OK) return orc;
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    put_times(c);
    const int rc = status_code(c, (uint32_t)c->h_ordmap[0]);
    if (rc != ZDL_OK) return rc;
    const size_t m = (size_t)c->h_ordmap[1];
    const unsigned char* b = reinterpret_cast<const unsigned char*>(c->h_ordmap) + 16;
    const int32_t* p = reinterpret_cast<const int32_t*>(b);
    const int32_t* ch = reinterpret_cast<const int32_t*>(b + 4 * MAP_CAP);
    const int64_t* ca = reinterpret_cast<const int64_t*>(b + 8 * MAP_CAP);
    const int64_t* er = reinterpret_cast<const int64_t*>(b + 16 * MAP_CAP);
    c->out_p.assign(p, p + m);  // already in rank order (k_ord_compact)
    c->out_c.assign(ch, ch + m);
    c->out_call.assign(ca, ca + m);
    c->out_err.assign(er, er + m);
    out->n = m;
    out->parent = c->out_p.data();
    out->child = c->out_c.data();
    out->call_count = c->out_call.data();
    out->error_count = c->out_err.data();
    return ZDL_OK;
  }
  HIP_TRY(c, c->o_p.ensure(SS));
  HIP_TRY(c, c->o_c.ensure(SS));
  HIP_TRY(c, c->o_call.ensure(SS));
  HIP_TRY(c, c->o_err.ensure(SS));
  HIP_TRY(c, c->o_first.ensure(SS));
  HIP_TRY(c, hipMemsetAsync(c->count.p, 0, 8, c->stream));
  hipLaunchKernelGGL(k_merge_compact, dim3((unsigned)((SS + 255) / 256)), dim3(256), 0, c->stream, call,
                     errc, first_rank, SS, c->S, c->count.p, c->o_p.p, c->o_c.p, c->o_call.p, c->o_err.p,
                     c->o_first.p);
  HIP_TRY(c, hipGetLastError());
  unsigned long long m = 0;
  HIP_TRY(c, hipMemcpyAsync(&m, c->count.p, 8, hipMemcpyDeviceToHost, c->stream));
  const int rc = zdl_sync(c);
  if (rc != ZDL_OK) return rc;
  std::vector<uint64_t> first(m);
  std::vector<int32_t> p(m), ch(m);
  std::vector<int64_t> ca(m), er(m);
  if (m) {
    HIP_TRY(c, hipMemcpy(p.data(), c->o_p.p, m * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(ch.data(), c->o_c.p, m * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(ca.data(), c->o_call.p, m * 8, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(er.data(), c->o_err.p, m * 8, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(first.data(), c->o_first.p, m * 8, hipMemcpyDeviceToHost));
  }
  std::vector<uint32_t> idx(m);
  for (size_t i = 0; i < m; ++i) idx[i] = (uint32_t)i;
  std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return first[a] < first[b]; });
  c->out_p.resize(m);
  c->out_c.resize(m);
  c->out_call.resize(m);
  c->out_err.resize(m);
  for (size_t i = 0; i < m; ++i) {
    c->out_p[i] = p[idx[i]];
    c->out_c[i] = ch[idx[i]];
    c->out_call[i] = ca[idx[i]];
    c->out_err[i] = er[idx[i]];
  }
  out->n = m;
  out->parent = c->out_p.data();
  out->child = c->out_c.data();
  out->call_count = c->out_call.data();
  out->error_count = c->out_err.data();
  return ZDL_OK;
}

}  // extern "C"

static int rec_download(zdl_ctx* c, uint64_t m);
static int ensure_rec(zdl_ctx* c, uint64_t m);

// zdl_link's sorted output from the S x S tables (call, err) on c's device: c's own tables
// (own: k_tail may already have compacted them into the mapped buffer) or summed ones (a
// device group's or a multi-process job's reduction).
static int link_sorted(zdl_ctx* c, const unsigned long long* call, const unsigned long long* err, bool own,
                       zdl_links* out) {
  const uint64_t SS = (uint64_t)c->S * c->S;
  const bool ordered = SS <= (uint64_t)COMPACT_WG * 8;
  ev_record(c, 5);
  size_t n = 0;
  c->out_p.clear();
  if (ordered) {
    // status, count and records land in mapped pinned memory: written by the last put's
    // k_tail, or here when the table changed since
    HIP_TRY(c, ensure_map(c));
    const bool tail_compacted = own && c->map_fresh;
    if (!tail_compacted) {
      hipLaunchKernelGGL(k_compact_ordered, dim3(1), dim3(COMPACT_WG), 0, c->stream, call, err, (uint32_t)SS, c->S,
                         c->status.p, c->d_map);
      HIP_TRY(c, hipGetLastError());
      c->map_fresh = own;  // h_map now holds the compaction of c's own table, or of a sum
    }
    ev_record(c, 6);
    // the last put's k_tail compacted: spin on its flag in mapped memory (a blocking
    // stream sync costs ~10 us of host wake-up), checking the stream now and then so a
    // failed kernel still surfaces; otherwise (or with every-kernel timing) a plain sync
    bool seen = false;
    if (!tail_compacted || ev_on(c, 6)) {
      HIP_TRY(c, hipStreamSynchronize(c->stream));
    } else {
      const volatile unsigned long long* f = c->h_flag;
      for (uint32_t i = 1;; ++i) {
        if (*f == c->seq) { seen = true; break; }
        if ((i & 255) == 0 && hipStreamQuery(c->stream) != hipErrorNotReady) break;
        __builtin_ia32_pause();
      }
      if (!seen || *f != c->seq) HIP_TRY(c, hipStreamSynchronize(c->stream));  // surfaces a failure
    }
    put_times(c);
    c->times.compact_ms = ev_ms(c, 5, 6);
    const int rc = status_code(c, (uint32_t)c->h_map[0]);
    if (rc != ZDL_OK) return rc;
    n = (size_t)c->h_map[1];
    const MapCols m = map_cols(c->h_map);
    c->out_p.assign(m.parent, m.parent + n);
    c->out_c.assign(m.child, m.child + n);
    c->out_call.assign(m.call, m.call + n);
    c->out_err.assign(m.err, m.err + n);
  } else {
    // non-zero cells selected and (with ranks) radix-sorted on the device, in output order,
    // written straight into mapped pinned host columns sized by the link count
    uint64_t m = 0;
    HIP_TRY(c, compact_select(c->lw, call, SS, &m, c->stream));
    const int erc = ensure_rec(c, m);
    if (erc != ZDL_OK) return erc;
    const size_t cap = c->h_rec_cap;
    unsigned char* const d = c->rec_dev.p;
    HIP_TRY(c, compact_records(c->lw, call, err, m, c->S, c->nrank[0] ? c->rank[0].p : nullptr, c->nrank[0],
                               (int32_t*)d, (int32_t*)(d + 4 * cap), (int64_t*)(d + 8 * cap),
                               (int64_t*)(d + 16 * cap), c->stream));
    ev_record(c, 6);
    const int drc = rec_download(c, m);
    if (drc != ZDL_OK) return drc;
    HIP_TRY(c, hipMemcpyAsync(c->h_meta, c->status.p, 16, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (const int wrc = rec_wait(c)) return wrc;
    put_times(c);
    c->times.compact_ms = ev_ms(c, 5, 6);
    const int rc = status_code(c, (uint32_t)c->h_meta[0]);
    if (rc != ZDL_OK) return rc;
    out->n = m;
    out->parent = (const int32_t*)c->h_rec;
    out->child = (const int32_t*)(c->h_rec + 4 * cap);
    out->call_count = (const int64_t*)(c->h_rec + 8 * cap);
    out->error_count = (const int64_t*)(c->h_rec + 16 * cap);
    return ZDL_OK;
  }
  // cell order is (parent id, child id) order; names order needs the service rank table
  if (ordered && c->nrank[0] != 0) sort_output(c, n);  // the large path came sorted
  out->n = n;
  out->parent = c->out_p.data();
  out->child = c->out_c.data();
  out->call_count = c->out_call.data();
  out->error_count = c->out_err.data();
  return ZDL_OK;
}

static int comm_sum_tables(zdl_ctx* c);  // multi-process job: every rank's tables summed (below)
static int comm_sum_ord(zdl_ctx* c);     // ... and, insertion order, the rank-tagged first ranks' MIN

// Four byte ranges [off, off + len) copied from HBM to mapped pinned host memory (same offsets
// on both sides; offsets multiples of 8, lengths multiples of 4), 8 bytes a lane, grid-stride.
struct PcieSegs {
  size_t off[4], len[4];
};
__global__ void __launch_bounds__(256) k_pcie_copy(unsigned char* __restrict__ dst, const unsigned char* __restrict__ src,
                                                   PcieSegs g) {
  // top issue priority: its waves only issue stores and share CUs with the next put's kernels,
  // which would otherwise starve them (the copy then stretched 2.6 -> 5.6 ms beside a C5 put)
  __builtin_amdgcn_s_setprio(3);
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, T = (size_t)gridDim.x * blockDim.x;
  for (int k = 0; k < 4; ++k) {
    const size_t n8 = g.len[k] / 8;
    const uint64_t* s = reinterpret_cast<const uint64_t*>(src + g.off[k]);
    uint64_t* d = reinterpret_cast<uint64_t*>(dst + g.off[k]);
    for (size_t i = t; i < n8; i += T) __builtin_nontemporal_store(s[i], d + i);
    if (t == 0 && (g.len[k] & 7))
      *reinterpret_cast<uint32_t*>(dst + g.off[k] + 8 * n8) = *reinterpret_cast<const uint32_t*>(src + g.off[k] + 8 * n8);
  }
}

// The mapped pinned output columns (parent, child i32; call, err i64) for m links, and their
// HBM staging copy.
static bool rec_dma() {
  static const bool on = [] {
    const char* e = getenv("ZDL_REC_DMA");
    return e && e[0] == '1';
  }();
  return on;
}

static int ensure_rec(zdl_ctx* c, uint64_t m) {
  if (const int wrc = rec_wait(c)) return wrc;
  if (m <= c->h_rec_cap) return ZDL_OK;
  c->rec_dev.release();
  if (c->h_rec) (void)hipHostFree(c->h_rec);
  c->h_rec = nullptr;
  c->d_rec = nullptr;
  c->h_rec_cap = 0;
  const size_t cap = std::max<size_t>((size_t)(m + m / 2 + 1) & ~(size_t)1, 1024);
  if (rec_dma()) {  // coarse-grained pinned memory: the copy engine can take it
    HIP_TRY(c, hipHostMalloc((void**)&c->h_rec, cap * 24, hipHostMallocNonCoherent));
  } else {
    HIP_TRY(c, hipHostMalloc((void**)&c->h_rec, cap * 24, hipHostMallocMapped | hipHostMallocCoherent));
    HIP_TRY(c, hipHostGetDevicePointer((void**)&c->d_rec, c->h_rec, 0));
  }
  HIP_TRY(c, c->rec_dev.ensure(cap * 24));
  c->h_rec_cap = cap;
  return ZDL_OK;
}

// The first m records of each staged column to the pinned host columns, by a narrow copy kernel
// (k_pcie_copy: PCIe-bound at any width, so it leaves the other CUs to the next put's kernels;
// hipMemcpyAsync ran rocclr's copyBuffer blit kernels across the whole GPU and slowed the
// concurrent k_link from 0.66 to 2.1 ms, profiles/r03g_c5_timeline.txt).
static bool rec_sdma() {  // default on; ZDL_REC_SDMA=0 (A/B): k_pcie_copy's workgroups instead
  static const bool on = [] {
    const char* e = getenv("ZDL_REC_SDMA");
    return !(e && e[0] == '0');
  }();
  return on && !rec_dma();
}

// The four record columns [off, off + len) from HBM to the pinned host columns by SDMA copies
// (ROCr's hsa_amd_memory_async_copy: a copy engine, no workgroups), waited for here.
static int sdma_copy(unsigned char* dst, const unsigned char* src, const size_t* off, const size_t* len) {
  hsa_amd_pointer_info_t ps{}, pd{};
  ps.size = sizeof ps;
  pd.size = sizeof pd;
  if (hsa_amd_pointer_info(src, &ps, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
      hsa_amd_pointer_info(dst, &pd, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS)
    return ZDL_EDEVICE;
  hsa_signal_t sig;
  if (hsa_signal_create(4, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return ZDL_EDEVICE;
  int rc = ZDL_OK;
  int issued = 0;
  for (int k = 0; k < 4; ++k) {
    if (len[k] == 0) {
      hsa_signal_subtract_screlease(sig, 1);
      continue;
    }
    if (hsa_amd_memory_async_copy(dst + off[k], pd.agentOwner, src + off[k], ps.agentOwner, len[k], 0, nullptr, sig) !=
        HSA_STATUS_SUCCESS) {
      rc = ZDL_EDEVICE;
      hsa_signal_subtract_screlease(sig, 4 - k);  // the copies not issued
      break;
    }
    ++issued;
  }
  (void)issued;
  while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) >= 1) {
  }
  hsa_signal_destroy(sig);
  return rc;
}

// The pending record copy: waited for (its helper thread) or, when no thread took it (a
// synchronous zdl_link), run here - the compaction's event, then the SDMA copies.
static int rec_wait(zdl_ctx* c) {
  int rc = ZDL_OK;
  if (c->rec_th.joinable()) {
    c->rec_th.join();
    rc = c->rec_th_rc;
    c->rec_th_rc = ZDL_OK;
  } else if (c->rec_job) {
    rc = hipEventSynchronize(c->rec_ev) != hipSuccess ? ZDL_EDEVICE
                                                      : sdma_copy(c->h_rec, c->rec_dev.p, c->rec_off, c->rec_len);
  }
  c->rec_job = false;
  return rc == ZDL_OK ? ZDL_OK : fail(c, rc, "SDMA copy of the link records failed");
}

// zdl_link_start: the pending record copy goes to a helper thread, so that it crosses PCIe
// while the caller goes on (the next put); zdl_link_finish joins it.
static int rec_launch(zdl_ctx* c) {
  if (!c->rec_job || c->rec_th.joinable()) return ZDL_OK;
  unsigned char* const dst = c->h_rec;
  const unsigned char* const src = c->rec_dev.p;
  hipEvent_t ev = c->rec_ev;
  size_t off[4], len[4];
  for (int k = 0; k < 4; ++k) {
    off[k] = c->rec_off[k];
    len[k] = c->rec_len[k];
  }
  c->rec_th = std::thread([c, dst, src, ev, off, len] {
    c->rec_th_rc = hipEventSynchronize(ev) != hipSuccess ? ZDL_EDEVICE : sdma_copy(dst, src, off, len);
  });
  return ZDL_OK;
}

static int rec_download(zdl_ctx* c, uint64_t m) {
  const size_t cap = c->h_rec_cap;
  if (m == 0) return ZDL_OK;
  if (rec_sdma()) {  // SDMA: the copy job behind the compaction's event (rec_wait / rec_launch)
    if (const int wrc = rec_wait(c)) return wrc;
    if (!c->rec_ev) HIP_TRY(c, hipEventCreateWithFlags(&c->rec_ev, hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(c->rec_ev, c->stream));
    const size_t off[4] = {0, 4 * cap, 8 * cap, 16 * cap}, len[4] = {4 * m, 4 * m, 8 * m, 8 * m};
    for (int k = 0; k < 4; ++k) {
      c->rec_off[k] = off[k];
      c->rec_len[k] = len[k];
    }
    c->rec_job = true;
    return ZDL_OK;
  }
  if (rec_dma()) {  // ZDL_REC_DMA=1 (A/B): hipMemcpyAsync into coarse-grained pinned memory
    for (size_t off : {(size_t)0, 4 * cap})
      HIP_TRY(c, hipMemcpyAsync(c->h_rec + off, c->rec_dev.p + off, m * 4, hipMemcpyDeviceToHost, c->stream));
    for (size_t off : {8 * cap, 16 * cap})
      HIP_TRY(c, hipMemcpyAsync(c->h_rec + off, c->rec_dev.p + off, m * 8, hipMemcpyDeviceToHost, c->stream));
    return ZDL_OK;
  }
  static const int wgs = [] {
    const char* e = getenv("ZDL_PCIE_WGS");
    return e ? std::max(1, atoi(e)) : 8;  // 8 / 32 / 64: C5 two in flight 6.73 / 7.08 / 7.17 ms
  }();
  PcieSegs g{};
  const size_t off[4] = {0, 4 * cap, 8 * cap, 16 * cap}, len[4] = {4 * m, 4 * m, 8 * m, 8 * m};
  for (int k = 0; k < 4; ++k) {
    g.off[k] = off[k];
    g.len[k] = len[k];
  }
  // a small list (C3's 250 k links, 6 MB) crosses faster from many workgroups; a large one (C5's
  // 4.5 M, 107 MB) is left to few, beside the next put
  const unsigned grid = m * 24 <= ((size_t)16 << 20) ? 128u : (unsigned)wgs;
  hipLaunchKernelGGL(k_pcie_copy, dim3(grid), dim3(256), 0, c->stream, c->d_rec, c->rec_dev.p, g);
  HIP_TRY(c, hipGetLastError());
  return ZDL_OK;
}

// A sparse context's links: its sorted list (cell = id order), rank-sorted when ranks are set.
// The first half enqueues the compaction into the mapped host columns (zdl_link_start stops
// there), the second waits and fills out.
static int link_sparse_start(zdl_ctx* c, const SparseTable& t) {
  const uint64_t m = t.n;
  int rc = ensure_rec(c, m);
  if (rc != ZDL_OK) return rc;
  const size_t cap = c->h_rec_cap;
  ev_record(c, 5);
  unsigned char* const d = c->rec_dev.p;
  HIP_TRY(c, compact_sparse(c->lw, t.cell, t.call, t.err, m, c->S,
                            c->nrank[0] ? c->rank[0].p : nullptr, c->nrank[0], (int32_t*)d,
                            (int32_t*)(d + 4 * cap), (int64_t*)(d + 8 * cap),
                            (int64_t*)(d + 16 * cap), c->stream));
  ev_record(c, 6);
  rc = rec_download(c, m);
  if (rc != ZDL_OK) return rc;
  HIP_TRY(c, hipMemcpyAsync(c->h_meta, c->status.p, 16, hipMemcpyDeviceToHost, c->stream));
  return ZDL_OK;
}
static int link_sparse(zdl_ctx* c, zdl_links* out, const SparseTable* tab = nullptr, bool started = false) {
  const SparseTable& t = tab ? *tab : c->acc;
  const uint64_t m = t.n;
  int rc = started ? ZDL_OK : link_sparse_start(c, t);
  if (rc != ZDL_OK) return rc;
  const size_t cap = c->h_rec_cap;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (const int wrc = rec_wait(c)) return wrc;
  rc = status_code(c, (uint32_t)c->h_meta[0]);
  if (rc != ZDL_OK) return rc;
  out->n = m;
  out->parent = (const int32_t*)c->h_rec;
  out->child = (const int32_t*)(c->h_rec + 4 * cap);
  out->call_count = (const int64_t*)(c->h_rec + 8 * cap);
  out->error_count = (const int64_t*)(c->h_rec + 16 * cap);
  return ZDL_OK;
}
static int group_link(zdl_ctx* g, int order, zdl_links* out);
static int comm_sum_sparse(zdl_ctx* c);  // multi-process job, sparse lists (below)

extern "C" {

int zdl_link(zdl_ctx* c, int order, zdl_links* out) {
  if (!c || !out) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_link: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) return group_link(c, order, out);
  if (c->lazy_pending) {
    HIP_TRY(c, enter(c));
    const int lrc = resolve_lazy(c, true);
    if (lrc != ZDL_OK) return lrc;
  }
  if (c->days) return fail(c, ZDL_EINVAL, "daily buckets are set: use zdl_link_days");
  if (c->poisoned) return fail(c, ZDL_EDEVICE, "an earlier put failed between its kernels: call zdl_reset");
  if (order == ZDL_ORDER_INSERTION) {
    if (!c->ord) return fail(c, ZDL_EINVAL, "ZDL_ORDER_INSERTION needs a ZDL_FLAG_INSERTION_ORDER context");
    HIP_TRY(c, enter(c));
    if (in_job(c)) {  // a rank of a job: DependencyLinker.merge over the ranks' lists in rank order
      const int rc = comm_sum_ord(c);
      if (rc != ZDL_OK) return x_failed(c, rc);
      return link_insertion(c, out, c->red_call.p, c->red_err.p, c->red_first.p);
    }
    return link_insertion(c, out, c->call.p, c->errc.p, c->first.p);
  }
  if (order != ZDL_ORDER_SORTED) return fail(c, ZDL_EINVAL, "zdl_link: order must be ZDL_ORDER_SORTED or ZDL_ORDER_INSERTION");
  HIP_TRY(c, enter(c));
  if (c->sparse && in_job(c)) {  // a rank of a job: every rank's list, summed
    const int rc = comm_sum_sparse(c);
    if (rc != ZDL_OK) return x_failed(c, rc);
    return link_sparse(c, out, &c->gacc);
  }
  if (c->sparse) return link_sparse(c, out);
  if (in_job(c)) {  // a rank of a job: the links of every rank's tables
    const int rc = comm_sum_tables(c);
    if (rc != ZDL_OK) return x_failed(c, rc);
    return link_sorted(c, c->red_call.p, c->red_err.p, false, out);
  }
  return link_sorted(c, c->call.p, c->errc.p, true, out);
}

int zdl_link_start(zdl_ctx* c, int order) {
  if (!c) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_link_start: a started link is not finished");
  if (const int frc = stage_flush(c)) return frc;
  c->link_pending = order;
  c->link_async = false;
  if (c->sparse && !in_job(c) && c->sub.empty() && order == ZDL_ORDER_SORTED && !c->poisoned) {
    HIP_TRY(c, enter(c));
    int rc = link_sparse_start(c, c->acc);
    if (rc == ZDL_OK) rc = rec_launch(c);  // the records cross PCIe on an SDMA engine meanwhile
    if (rc != ZDL_OK) {
      c->link_pending = -1;
      return rc;
    }
    c->link_async = true;
  }
  return ZDL_OK;
}

int zdl_link_finish(zdl_ctx* c, zdl_links* out) {
  if (!c || !out) return ZDL_EINVAL;
  if (c->link_pending < 0) return fail(c, ZDL_EINVAL, "zdl_link_finish: no started link");
  const int order = c->link_pending;
  const bool started = c->link_async;
  c->link_pending = -1;
  c->link_async = false;
  if (started) {
    HIP_TRY(c, enter(c));
    return link_sparse(c, out, nullptr, true);
  }
  return zdl_link(c, order, out);
}

// Daily buckets: the cells as (day, parent, child, counts), ordered like
// ITDependencies.aggregateLinks' map of per-day DependencyLinker.link() lists.
}  // extern "C"

// The per-day output from (row = day * S + parent, child, counts[, first ranks]) records:
// sorted by (day, parent, child) in the rank tables' order, or (insertion order) days by their
// first trace and each day's links by first rank; and the days that hold a trace.
static int days_out(zdl_ctx* c, int order, std::vector<int32_t>& row, std::vector<int32_t>& ch,
                    std::vector<int64_t>& ca, std::vector<int64_t>& er, const std::vector<uint64_t>& first,
                    zdl_day_links* out) {
  const size_t m = row.size();
  const std::vector<int32_t>& r = c->host_rank[0];
  auto rk = [&](int32_t id) -> int64_t { return (size_t)id < r.size() ? r[id] : id; };
  const uint32_t S = c->S;
  std::vector<uint32_t> idx(m);
  for (size_t i = 0; i < m; ++i) idx[i] = (uint32_t)i;
  if (order == ZDL_ORDER_INSERTION) {  // days by first trace, then the day's linker order
    std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
      const uint64_t fa = c->h_day_first[(uint32_t)row[a] / S], fb = c->h_day_first[(uint32_t)row[b] / S];
      if (fa != fb) return fa < fb;
      return first[a] < first[b];
    });
  } else {  // (day, parent, child) with names in String order
    std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
      const uint32_t da = (uint32_t)row[a] / S, db = (uint32_t)row[b] / S;
      if (da != db) return da < db;
      const int64_t pa = rk(row[a] % (int32_t)S), pb = rk(row[b] % (int32_t)S);
      if (pa != pb) return pa < pb;
      return rk(ch[a]) < rk(ch[b]);
    });
  }
  c->out_day.resize(m);
  c->out_p.resize(m);
  c->out_c.resize(m);
  c->out_call.resize(m);
  c->out_err.resize(m);
  for (size_t i = 0; i < m; ++i) {
    const uint32_t j = idx[i];
    c->out_day[i] = c->day0 + (int64_t)((uint32_t)row[j] / S) * DAY_MS;
    c->out_p[i] = (int32_t)((uint32_t)row[j] % S);
    c->out_c[i] = ch[j];
    c->out_call[i] = ca[j];
    c->out_err[i] = er[j];
  }
  std::vector<uint32_t> dl;  // the days that hold a trace (links or not)
  for (uint32_t d = 0; d < c->days; ++d)
    if (c->h_day_first[d] != ~0ull) dl.push_back(d);
  if (order == ZDL_ORDER_INSERTION)
    std::sort(dl.begin(), dl.end(), [&](uint32_t a, uint32_t b) { return c->h_day_first[a] < c->h_day_first[b]; });
  c->out_days.resize(dl.size());
  for (size_t i = 0; i < dl.size(); ++i) c->out_days[i] = c->day0 + (int64_t)dl[i] * DAY_MS;
  out->n_days = dl.size();
  out->day_ms = c->out_days.data();
  out->n = m;
  out->day = c->out_day.data();
  out->parent = c->out_p.data();
  out->child = c->out_c.data();
  out->call_count = c->out_call.data();
  out->error_count = c->out_err.data();
  return ZDL_OK;
}

// A sparse context's daily buckets: its sorted list, cells (day * S + parent) * S + child
static int link_days_sparse(zdl_ctx* c, int order, zdl_day_links* out) {
  if (order != ZDL_ORDER_SORTED) return fail(c, ZDL_EINVAL, "zdl_link_days: a sparse context links in ZDL_ORDER_SORTED only");
  c->h_day_first.assign(c->days, 0);
  HIP_TRY(c, hipMemcpyAsync(c->h_day_first.data(), c->day_first.p, (size_t)c->days * 8, hipMemcpyDeviceToHost,
                            c->stream));
  const int rc = zdl_sync(c);
  if (rc != ZDL_OK) return rc;
  const size_t m = c->acc.n;
  std::vector<uint32_t> cell(m);
  std::vector<int32_t> row(m), ch(m);
  std::vector<int64_t> ca(m), er(m);
  if (m) {
    HIP_TRY(c, hipMemcpy(cell.data(), c->acc.cell, m * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(ca.data(), c->acc.call, m * 8, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(er.data(), c->acc.err, m * 8, hipMemcpyDeviceToHost));
  }
  for (size_t i = 0; i < m; ++i) {
    row[i] = (int32_t)(cell[i] / c->S);
    ch[i] = (int32_t)(cell[i] % c->S);
  }
  return days_out(c, order, row, ch, ca, er, std::vector<uint64_t>(), out);
}

extern "C" {

int zdl_link_days(zdl_ctx* c, int order, zdl_day_links* out) {
  if (!c || !out) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_link_days: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty() || in_job(c)) return fail(c, ZDL_EINVAL, "zdl_link_days: one device, one process");
  if (!c->days) return fail(c, ZDL_EINVAL, "zdl_link_days: no daily buckets (zdl_set_days)");
  if (order == ZDL_ORDER_INSERTION && !c->ord)
    return fail(c, ZDL_EINVAL, "ZDL_ORDER_INSERTION needs a ZDL_FLAG_INSERTION_ORDER context");
  if (order != ZDL_ORDER_INSERTION && order != ZDL_ORDER_SORTED)
    return fail(c, ZDL_EINVAL, "zdl_link_days: order must be ZDL_ORDER_SORTED or ZDL_ORDER_INSERTION");
  HIP_TRY(c, enter(c));
  if (c->sparse) return link_days_sparse(c, order, out);
  const uint64_t SS = (uint64_t)c->rows * c->S;
  HIP_TRY(c, c->o_p.ensure(SS));
  HIP_TRY(c, c->o_c.ensure(SS));
  HIP_TRY(c, c->o_call.ensure(SS));
  HIP_TRY(c, c->o_err.ensure(SS));
  HIP_TRY(c, c->o_first.ensure(SS));
  HIP_TRY(c, hipMemsetAsync(c->count.p, 0, 8, c->stream));
  if (c->ord) {  // non-zero cells with their first-addLink ranks
    hipLaunchKernelGGL(k_merge_compact, dim3((unsigned)((SS + 255) / 256)), dim3(256), 0, c->stream, c->call.p,
                       c->errc.p, c->first.p, SS, c->S, c->count.p, c->o_p.p, c->o_c.p, c->o_call.p, c->o_err.p,
                       c->o_first.p);
  } else {
    HIP_TRY(c, c->o_links.ensure(SS));
    hipLaunchKernelGGL(k_compact, dim3((unsigned)((SS + 255) / 256)), dim3(256), 0, c->stream, c->call.p, c->errc.p,
                       SS, c->S, c->count.p, c->o_links.p);
  }
  HIP_TRY(c, hipGetLastError());
  unsigned long long m = 0;
  HIP_TRY(c, hipMemcpyAsync(&m, c->count.p, 8, hipMemcpyDeviceToHost, c->stream));
  c->h_day_first.assign(c->days, 0);
  HIP_TRY(c, hipMemcpyAsync(c->h_day_first.data(), c->day_first.p, (size_t)c->days * 8, hipMemcpyDeviceToHost,
                            c->stream));
  const int rc = zdl_sync(c);
  if (rc != ZDL_OK) return rc;
  std::vector<int32_t> row(m), ch(m);
  std::vector<int64_t> ca(m), er(m);
  std::vector<uint64_t> first(m, 0);
  if (m && c->ord) {
    HIP_TRY(c, hipMemcpy(row.data(), c->o_p.p, m * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(ch.data(), c->o_c.p, m * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(ca.data(), c->o_call.p, m * 8, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(er.data(), c->o_err.p, m * 8, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(first.data(), c->o_first.p, m * 8, hipMemcpyDeviceToHost));
  } else if (m) {
    std::vector<ZLink> recs(m);
    HIP_TRY(c, hipMemcpy(recs.data(), c->o_links.p, m * sizeof(ZLink), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < m; ++i) {
      row[i] = recs[i].parent;
      ch[i] = recs[i].child;
      ca[i] = recs[i].call;
      er[i] = recs[i].err;
    }
  }
  return days_out(c, order, row, ch, ca, er, first, out);
}

int zdl_merge_links(zdl_ctx* c, const int32_t* parent, const int32_t* child, const int64_t* call_count,
                    const int64_t* error_count, uint64_t n, zdl_links* out) {
  if (!c || !out) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_merge_links: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) return group_first(c, zdl_merge_links(c->sub[0], parent, child, call_count, error_count, n, out));
  HIP_TRY(c, enter(c));
  const uint64_t SS = (uint64_t)c->S * c->S;
  HIP_TRY(c, c->m_call.ensure(SS));
  HIP_TRY(c, c->m_err.ensure(SS));
  HIP_TRY(c, c->m_first.ensure(SS));
  HIP_TRY(c, c->o_p.ensure(SS));
  HIP_TRY(c, c->o_c.ensure(SS));
  HIP_TRY(c, c->o_call.ensure(SS));
  HIP_TRY(c, c->o_err.ensure(SS));
  HIP_TRY(c, c->o_first.ensure(SS));
  HIP_TRY(c, c->mi_p.ensure(n));
  HIP_TRY(c, c->mi_c.ensure(n));
  HIP_TRY(c, c->mi_call.ensure(n));
  HIP_TRY(c, c->mi_err.ensure(n));
  hipStream_t s = c->stream;
  HIP_TRY(c, hipMemsetAsync(c->m_call.p, 0, SS * 8, s));
  HIP_TRY(c, hipMemsetAsync(c->m_err.p, 0, SS * 8, s));
  HIP_TRY(c, hipMemsetAsync(c->m_first.p, 0xff, SS * 8, s));
  HIP_TRY(c, hipMemsetAsync(c->count.p, 0, 8, s));
  HIP_TRY(c, hipMemsetAsync(c->status.p, 0, 16, s));
  if (n) {
    HIP_TRY(c, hipMemcpyAsync(c->mi_p.p, parent, n * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(c->mi_c.p, child, n * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(c->mi_call.p, call_count, n * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(c->mi_err.p, error_count, n * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_merge_accum, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c->mi_p.p, c->mi_c.p,
                       c->mi_call.p, c->mi_err.p, n, c->S, c->m_call.p, c->m_err.p, c->m_first.p, c->status.p,
                       (uint64_t)0, 0);
    HIP_TRY(c, hipGetLastError());
  }
  hipLaunchKernelGGL(k_merge_compact, dim3((unsigned)((SS + 255) / 256)), dim3(256), 0, s, c->m_call.p, c->m_err.p,
                     c->m_first.p, SS, c->S, c->count.p, c->o_p.p, c->o_c.p, c->o_call.p, c->o_err.p, c->o_first.p);
  HIP_TRY(c, hipGetLastError());
  unsigned long long m = 0;
  HIP_TRY(c, hipMemcpyAsync(&m, c->count.p, 8, hipMemcpyDeviceToHost, s));
  int rc = zdl_sync(c);
  if (rc != ZDL_OK) return rc;
  std::vector<uint64_t> first(m);
  c->out_p.resize(m);
  c->out_c.resize(m);
  c->out_call.resize(m);
  c->out_err.resize(m);
  if (m) {
    HIP_TRY(c, hipMemcpy(c->out_p.data(), c->o_p.p, m * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(c->out_c.data(), c->o_c.p, m * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(c->out_call.data(), c->o_call.p, m * 8, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(c->out_err.data(), c->o_err.p, m * 8, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(first.data(), c->o_first.p, m * 8, hipMemcpyDeviceToHost));
  }
  std::vector<uint32_t> idx(m);
  for (size_t i = 0; i < m; ++i) idx[i] = (uint32_t)i;
  std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return first[a] < first[b]; });
  std::vector<int32_t> p(m), ch(m);
  std::vector<int64_t> ca(m), er(m);
  for (size_t i = 0; i < m; ++i) {
    p[i] = c->out_p[idx[i]];
    ch[i] = c->out_c[idx[i]];
    ca[i] = c->out_call[idx[i]];
    er[i] = c->out_err[idx[i]];
  }
  c->out_p.swap(p);
  c->out_c.swap(ch);
  c->out_call.swap(ca);
  c->out_err.swap(er);
  out->n = m;
  out->parent = c->out_p.data();
  out->child = c->out_c.data();
  out->call_count = c->out_call.data();
  out->error_count = c->out_err.data();
  return ZDL_OK;
}

int zdl_add_links(zdl_ctx* c, const int32_t* parent, const int32_t* child, const int64_t* call_count,
                  const int64_t* error_count, uint64_t n) {
  if (!c) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_add_links: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) return group_first(c, zdl_add_links(c->sub[0], parent, child, call_count, error_count, n));
  if (c->days) return fail(c, ZDL_EINVAL, "zdl_add_links: not with daily buckets");
  if (n == 0) return ZDL_OK;
  HIP_TRY(c, enter(c));
  {
    const int lrc = resolve_lazy(c, false);  // a lazy put's k_mid / k_tail before the table is used
    if (lrc != ZDL_OK) return lrc;
  }
  if (c->sparse) {  // merged into the sorted list (DependencyLinker.merge's sum per pair)
    std::vector<uint32_t> cells(n);
    for (uint64_t i = 0; i < n; ++i) {
      if ((uint32_t)parent[i] >= c->S || (uint32_t)child[i] >= c->S) return fail(c, ZDL_EINVAL, "service id >= n_services");
      cells[i] = (uint32_t)parent[i] * c->S + (uint32_t)child[i];
    }
    hipStream_t s = c->stream;
    HIP_TRY(c, c->lin.ensure(n));
    HIP_TRY(c, c->mi_call.ensure(n));
    HIP_TRY(c, c->mi_err.ensure(n));
    HIP_TRY(c, hipMemcpyAsync(c->lin.p, cells.data(), n * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(c->mi_call.p, call_count, n * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(c->mi_err.p, error_count, n * 8, hipMemcpyHostToDevice, s));
    int kb = 1;
    while ((1ull << kb) < (uint64_t)c->S * c->S) ++kb;
    HIP_TRY(c, sparse_add(c->sw, c->acc, c->lin.p, (const unsigned long long*)c->mi_call.p,
                          (const unsigned long long*)c->mi_err.p, n, kb, s));
    return zdl_sync(c);
  }
  const uint64_t SS = (uint64_t)c->S * c->S;
  HIP_TRY(c, c->m_first.ensure(SS));
  HIP_TRY(c, c->mi_p.ensure(n));
  HIP_TRY(c, c->mi_c.ensure(n));
  HIP_TRY(c, c->mi_call.ensure(n));
  HIP_TRY(c, c->mi_err.ensure(n));
  hipStream_t s = c->stream;
  HIP_TRY(c, hipMemcpyAsync(c->mi_p.p, parent, n * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->mi_c.p, child, n * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->mi_call.p, call_count, n * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipMemcpyAsync(c->mi_err.p, error_count, n * 8, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_merge_accum, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c->mi_p.p, c->mi_c.p,
                     c->mi_call.p, c->mi_err.p, n, c->S, c->call.p, c->errc.p,
                     c->ord ? c->first.p : c->m_first.p, c->status.p, c->ord ? c->span_base : 0, c->ord ? 1 : 0);
  HIP_TRY(c, hipGetLastError());
  if (c->ord) c->span_base += n;  // the links rank before anything put afterwards (ord_rank's layout)
  c->map_fresh = false;
  c->ordmap_fresh = false;
  return zdl_sync(c);
}

int zdl_table_export(zdl_ctx* c, void* dev_call, void* dev_err) {
  if (!c || !dev_call || !dev_err) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_table_export: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) return group_export(c, dev_call, dev_err);
  if (c->sparse) return fail(c, ZDL_EINVAL, "zdl_table_export: a sparse context has no S x S table");
  HIP_TRY(c, enter(c));
  {
    const int lrc = resolve_lazy(c, false);  // a lazy put's k_mid / k_tail before the table is used
    if (lrc != ZDL_OK) return lrc;
  }
  if (in_job(c)) {  // every rank's tables, summed
    const int rc = comm_sum_tables(c);
    if (rc != ZDL_OK) return x_failed(c, rc);
    const size_t bytes = (size_t)c->rows * c->S * 8;
    HIP_TRY(c, hipMemcpyAsync(dev_call, c->red_call.p, bytes, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(dev_err, c->red_err.p, bytes, hipMemcpyDeviceToDevice, c->stream));
    return ZDL_OK;
  }
  const size_t bytes = (size_t)c->rows * c->S * 8;
  HIP_TRY(c, hipMemcpyAsync(dev_call, c->call.p, bytes, hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(dev_err, c->errc.p, bytes, hipMemcpyDeviceToDevice, c->stream));
  return ZDL_OK;
}

int zdl_table_import(zdl_ctx* c, const void* dev_call, const void* dev_err) {
  if (!c || !dev_call || !dev_err) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_table_import: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) {  // the first device holds the imported counts, the others none
    for (size_t d = 1; d < c->sub.size(); ++d) {
      const int rc = zdl_reset(c->sub[d]);
      if (rc != ZDL_OK) return group_first(c, rc, c->sub[d]);
    }
    return group_first(c, zdl_table_import(c->sub[0], dev_call, dev_err));
  }
  if (c->ord) return fail(c, ZDL_EINVAL, "zdl_table_import: the table carries no insertion-order ranks");
  if (c->sparse) return fail(c, ZDL_EINVAL, "zdl_table_import: a sparse context has no S x S table");
  HIP_TRY(c, enter(c));
  {
    const int lrc = resolve_lazy(c, false);  // a lazy put's k_mid / k_tail before the table is used
    if (lrc != ZDL_OK) return lrc;
  }
  const size_t bytes = (size_t)c->rows * c->S * 8;
  HIP_TRY(c, hipMemcpyAsync(c->call.p, dev_call, bytes, hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->errc.p, dev_err, bytes, hipMemcpyDeviceToDevice, c->stream));
  c->map_fresh = false;
  c->ordmap_fresh = false;
  return ZDL_OK;
}

int zdl_get_kernel_times(zdl_ctx* c, zdl_kernel_times* out) {
  if (!c || !out) return ZDL_EINVAL;
  if (!c->sub.empty()) return group_first(c, zdl_get_kernel_times(c->sub[0], out));
  if ((c->flags & ZDL_FLAG_TIMING) && c->lk_n) {  // mean k_link time of the last <= 64 puts
    HIP_TRY(c, enter(c));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const uint32_t k = std::min<uint32_t>(c->lk_n, zdl_ctx::LK_RING);
    double sum = 0;
    for (uint32_t j = 0; j < k; ++j) {
      const uint32_t i = (c->lk_n - 1 - j) % zdl_ctx::LK_RING;
      float ms = 0.f;
      HIP_TRY(c, hipEventElapsedTime(&ms, c->lk_ev[0][i], c->lk_ev[1][i]));
      sum += ms;
    }
    c->times.tiles_ms = (float)(sum / k);
    c->times.n_tiles = k;  // the puts averaged
    c->lk_n = 0;
  }
  if (c->flags & ZDL_FLAG_TIMING_ALL) {  // the last put's and link's phases
    HIP_TRY(c, enter(c));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    put_times(c);
    c->times.compact_ms = ev_ms(c, 5, 6);
  }
  *out = c->times;
  return ZDL_OK;
}

}  // extern "C"

// ====================================================================== multi-GPU
// traces are independent, so whole traces go to one device each by
// splitmix64(trace_lo) % n (the LOW 64 bits: getDependencies groups by lowTraceId,
// InMemoryStorage.java:163, 330, 465-467) and the per-device tables are summed once - the
// additive reduce of DependencyLinker.merge (DependencyLinker.java:189-204) - by RCCL over xGMI.

static zdl_ctx* create_group(const zdl_config* cfg) {
  const uint32_t n = cfg->n_devices;
  if (n == 0 || n > 64) {
    g_create_error = "device group: n_devices must be in [1, 64]";
    return nullptr;
  }
  for (uint32_t i = 0; i < n; ++i)
    for (uint32_t j = i + 1; j < n; ++j)
      if (cfg->device_ids[i] == cfg->device_ids[j]) {
        g_create_error = "device group: a device appears twice (RCCL takes one rank per device)";
        return nullptr;
      }
  if (cfg->flags & ZDL_FLAG_INSERTION_ORDER) {
    g_create_error = "device group: ZDL_FLAG_INSERTION_ORDER needs one device (first-addLink ranks are per device)";
    return nullptr;
  }
  zdl_ctx* g = new zdl_ctx();
  g->S = cfg->n_services;
  g->rows = cfg->n_services;
  g->flags = cfg->flags;
  g->device = cfg->device_ids[0];
  for (uint32_t d = 0; d < n; ++d) {
    zdl_config one = *cfg;
    one.device = cfg->device_ids[d];
    one.n_devices = 0;
    one.device_ids = nullptr;
    // above 1024 services every device keeps a sparse list (ZDL_FLAG_DENSE_TABLE keeps tables):
    // zdl_link gathers the lists onto the first device and sums them (group_link_sparse)
    zdl_ctx* s = zdl_create(&one);
    if (!s) {
      const std::string e = g_create_error;
      zdl_destroy(g);
      g_create_error = "device " + std::to_string(cfg->device_ids[d]) + ": " + e;
      return nullptr;
    }
    g->sub.push_back(s);
  }
  g->comms.assign(n, nullptr);
  const ncclResult_t r = ncclCommInitAll(g->comms.data(), (int)n, cfg->device_ids);
  if (r != ncclSuccess) {
    g->comms.clear();
    zdl_destroy(g);
    g_create_error = std::string("device group: ncclCommInitAll: ") + ncclGetErrorString(r);
    return nullptr;
  }
  return g;
}

// The host split (zdl_shard.h): two parallel passes over the batch (count, scatter) into one
// column set per device, then one host thread per device uploads and launches its shard.
int group_put(zdl_ctx* g, const zdl_span_cols* col, uint64_t n_spans, const uint64_t* off, uint64_t n_traces) {
  if (!col->trace_lo) return fail(g, ZDL_EINVAL, "device group: traces are sharded by trace_lo, which is missing");
  if (!col->id || !col->parent_id || !col->local_svc || !col->remote_svc || !col->local_ip4 || !col->local_ip6 ||
      !col->port_flags)
    return fail(g, ZDL_EINVAL, "missing column");
  if (off) {
    if (n_traces == 0) return ZDL_OK;
    if (off[0] != 0 || off[n_traces] != n_spans) return fail(g, ZDL_EINVAL, "trace offsets must span [0, n_spans]");
    for (uint64_t t = 0; t < n_traces; ++t)
      if (off[t + 1] < off[t]) return fail(g, ZDL_EINVAL, "trace offsets are not non-decreasing");
  }
  if (n_spans == 0) return ZDL_OK;
  const uint32_t N = (uint32_t)g->sub.size();
  const int threads = zdl_shard::host_threads(getenv("ZDL_HOST_THREADS"));
  const zdl_shard::In in{col->trace_lo, col->id,        col->parent_id,  col->local_svc, col->remote_svc,
                         col->local_ip4, col->local_ip6, col->port_flags, col->timestamp, col->ord};
  const zdl_shard::Plan plan = zdl_shard::plan(in, n_spans, off, n_traces, N, threads);
  struct Shard {  // uninitialized host columns (new T[n]: the scatter writes every element)
    std::unique_ptr<uint64_t[]> lo, id, pid, off;
    std::unique_ptr<int32_t[]> ls, rs, i4, i6;
    std::unique_ptr<uint32_t[]> pf, ord;
    std::unique_ptr<int64_t[]> ts;
  };
  std::vector<Shard> sh(N);
  std::vector<zdl_shard::Out> outs(N);
  for (uint32_t d = 0; d < N; ++d) {
    const uint64_t n = std::max<uint64_t>(plan.spans[d], 1);
    Shard& s = sh[d];
    s.lo.reset(new uint64_t[n]);
    s.id.reset(new uint64_t[n]);
    s.pid.reset(new uint64_t[n]);
    s.ls.reset(new int32_t[n]);
    s.rs.reset(new int32_t[n]);
    s.i4.reset(new int32_t[n]);
    s.i6.reset(new int32_t[n]);
    s.pf.reset(new uint32_t[n]);
    if (col->timestamp) s.ts.reset(new int64_t[n]);
    if (col->ord) s.ord.reset(new uint32_t[n]);
    if (off) s.off.reset(new uint64_t[plan.traces[d] + 1]);
    outs[d] = zdl_shard::Out{s.lo.get(), s.id.get(), s.pid.get(), s.ls.get(), s.rs.get(), s.i4.get(),
                             s.i6.get(), s.pf.get(), s.ts.get(), s.ord.get(), s.off.get()};
  }
  zdl_shard::scatter(in, off, plan, outs.data(), threads);
  std::vector<int> rc(N, ZDL_OK);
  auto run = [&](uint32_t d) {
    if (plan.spans[d] == 0) return;
    const zdl_shard::Out& o = outs[d];
    zdl_span_cols sc{o.lo, o.id, o.pid, o.ls, o.rs, o.i4, o.i6, o.pf, o.ts, o.ord};
    rc[d] = zdl_put_spans(g->sub[d], &sc, plan.spans[d], off ? o.off : nullptr, off ? plan.traces[d] : 0);
  };
  std::vector<std::thread> th;  // one host thread per device: upload + launch overlap
  for (uint32_t d = 0; d < N; ++d) th.emplace_back(run, d);
  for (auto& t : th) t.join();
  for (uint32_t d = 0; d < N; ++d)
    if (rc[d] != ZDL_OK) return group_first(g, rc[d], g->sub[d]);
  return ZDL_OK;
}

// The per-device tables summed onto the first device (root of the reduce), into recv.
static int group_reduce(zdl_ctx* g, unsigned long long* rcall, unsigned long long* rerr) {
  const size_t SS = (size_t)g->S * g->S;
  for (zdl_ctx* s : g->sub)
    if (s->poisoned) return fail(g, ZDL_EDEVICE, "an earlier put failed between its kernels: call zdl_reset");
  ncclResult_t r = ncclGroupStart();
  for (size_t d = 0; d < g->sub.size() && r == ncclSuccess; ++d) {
    zdl_ctx* s = g->sub[d];
    (void)hipSetDevice(s->device);
    r = ncclReduce(s->call.p, d == 0 ? (void*)rcall : (void*)s->call.p, SS, ncclUint64, ncclSum, 0, g->comms[d],
                   s->stream);
    if (r == ncclSuccess)
      r = ncclReduce(s->errc.p, d == 0 ? (void*)rerr : (void*)s->errc.p, SS, ncclUint64, ncclSum, 0, g->comms[d],
                     s->stream);
  }
  const ncclResult_t r2 = ncclGroupEnd();
  (void)hipSetDevice(g->sub[0]->device);
  if (r != ncclSuccess || r2 != ncclSuccess)
    return fail(g, ZDL_EDEVICE, std::string("device group: ncclReduce: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
  return ZDL_OK;
}

// Device groups above 1024 services: every device's sorted list sent to the first device
// (ncclSend / ncclRecv over xGMI, exact lengths), concatenated and summed per cell there
// (sparse_add: radix sort, reduce by key - DependencyLinker.merge, DependencyLinker.java:189-204).
// an allgather of compacted (pair, call, err) instead of S x S tables.
static int group_link_sparse(zdl_ctx* g, zdl_links* out) {
  zdl_ctx* s0 = g->sub[0];
  const int N = (int)g->sub.size();
  std::vector<uint64_t> n((size_t)N);
  for (int d = 0; d < N; ++d) n[d] = g->sub[d]->acc.n;
  const zdl_xplan::Plan plan = zdl_xplan::gather_plan(n.data(), N, false);  // every list to device 0
  const uint64_t total = plan.total();
  HIP_TRY(g, enter(s0));
  HIP_TRY(g, s0->gx_cell.ensure(total));
  HIP_TRY(g, s0->gx_call.ensure(total));
  HIP_TRY(g, s0->gx_err.ensure(total));
  ncclResult_t r = ncclGroupStart();
  for (const zdl_xplan::Xfer& x : plan.ops) {
    if (x.src == x.dst || r != ncclSuccess) continue;  // device 0's own list: a copy below
    zdl_ctx* s = g->sub[x.src];
    zdl_ctx* t = g->sub[x.dst];
    (void)hipSetDevice(s->device);
    r = ncclSend(s->acc.cell, x.n, ncclUint32, x.dst, g->comms[x.src], s->stream);
    if (r == ncclSuccess) r = ncclSend(s->acc.call, x.n, ncclUint64, x.dst, g->comms[x.src], s->stream);
    if (r == ncclSuccess) r = ncclSend(s->acc.err, x.n, ncclUint64, x.dst, g->comms[x.src], s->stream);
    (void)hipSetDevice(t->device);
    if (r == ncclSuccess) r = ncclRecv(t->gx_cell.p + x.at, x.n, ncclUint32, x.src, g->comms[x.dst], t->stream);
    if (r == ncclSuccess) r = ncclRecv(t->gx_call.p + x.at, x.n, ncclUint64, x.src, g->comms[x.dst], t->stream);
    if (r == ncclSuccess) r = ncclRecv(t->gx_err.p + x.at, x.n, ncclUint64, x.src, g->comms[x.dst], t->stream);
  }
  const ncclResult_t r2 = ncclGroupEnd();
  (void)hipSetDevice(s0->device);
  if (r != ncclSuccess || r2 != ncclSuccess)
    return fail(g, ZDL_EDEVICE, std::string("device group: ncclSend/Recv: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
  hipStream_t st = s0->stream;
  for (const zdl_xplan::Xfer& x : plan.ops) {
    if (x.src != x.dst) continue;
    HIP_TRY(g, hipMemcpyAsync(s0->gx_cell.p + x.at, s0->acc.cell, x.n * 4, hipMemcpyDeviceToDevice, st));
    HIP_TRY(g, hipMemcpyAsync(s0->gx_call.p + x.at, s0->acc.call, x.n * 8, hipMemcpyDeviceToDevice, st));
    HIP_TRY(g, hipMemcpyAsync(s0->gx_err.p + x.at, s0->acc.err, x.n * 8, hipMemcpyDeviceToDevice, st));
  }
  s0->gacc.n = 0;
  int kb = 1;
  while ((1ull << kb) < (uint64_t)g->S * g->S) ++kb;
  HIP_TRY(g, sparse_add(s0->sw, s0->gacc, s0->gx_cell.p, s0->gx_call.p, s0->gx_err.p, total, kb, st));
  return group_first(g, link_sparse(s0, out, &s0->gacc));
}

static int group_link(zdl_ctx* g, int order, zdl_links* out) {
  if (order != ZDL_ORDER_SORTED) return fail(g, ZDL_EINVAL, "device group: zdl_link returns ZDL_ORDER_SORTED");
  for (zdl_ctx* s : g->sub) {  // lazy puts: their k_mid / k_tail before the tables are reduced
    (void)hipSetDevice(s->device);
    const int lrc = resolve_lazy(s, false);
    if (lrc != ZDL_OK) return group_first(g, lrc, s);
  }
  zdl_ctx* s0 = g->sub[0];
  for (size_t d = 1; d < g->sub.size(); ++d) {  // surfaces the other devices' status (NPE, bad ids)
    const int rc = zdl_sync(g->sub[d]);
    if (rc != ZDL_OK) return group_first(g, rc, g->sub[d]);
  }
  if (s0->sparse) return group_link_sparse(g, out);
  HIP_TRY(g, enter(s0));
  const size_t SS = (size_t)g->S * g->S;
  HIP_TRY(g, s0->red_call.ensure(SS));
  HIP_TRY(g, s0->red_err.ensure(SS));
  const int rc = group_reduce(g, s0->red_call.p, s0->red_err.p);
  if (rc != ZDL_OK) return rc;
  return group_first(g, link_sorted(s0, s0->red_call.p, s0->red_err.p, false, out));
}

int group_export(zdl_ctx* g, void* dev_call, void* dev_err) {
  if (g->sub[0]->sparse) return fail(g, ZDL_EINVAL, "zdl_table_export: a sparse device group has no S x S table");
  for (zdl_ctx* s : g->sub) {
    (void)hipSetDevice(s->device);
    const int lrc = resolve_lazy(s, false);
    if (lrc != ZDL_OK) return group_first(g, lrc, s);
  }
  HIP_TRY(g, enter(g->sub[0]));
  return group_reduce(g, (unsigned long long*)dev_call, (unsigned long long*)dev_err);
}

#include "zdl_xport.inc"  // the transport under the combines: RCCL or a local world

// Every rank's tables, summed (DependencyLinker.merge over the ranks' maps, DependencyLinker.java:189-204)
static int comm_sum_tables(zdl_ctx* c) {
  const size_t SS = (size_t)c->rows * c->S;
  HIP_TRY(c, c->red_call.ensure(SS));
  HIP_TRY(c, c->red_err.ensure(SS));
  const XRed ops[2] = {{c->call.p, c->red_call.p, SS, 0}, {c->errc.p, c->red_err.p, SS, 0}};
  return x_allreduce(c, ops, 2);
}

// Each rank's first-seen ranks tagged with the job rank above them (zdl_xplan::ord_tag)
__global__ void k_ord_tag(const unsigned long long* __restrict__ first, unsigned long long* __restrict__ out,
                          uint64_t n, int rank) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = zdl_xplan::ord_tag(first[i], rank);
}

__global__ void k_iota32(uint32_t* __restrict__ v, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    v[i] = (uint32_t)i;
}
// The local-order tags: the cell at sorted position j (its rank's j-th first-seen pair) gets
// rank << 32 | j; a pair the rank never saw stays ~0
__global__ void k_ord_local(const unsigned long long* __restrict__ key, const uint32_t* __restrict__ cell,
                            unsigned long long* __restrict__ out, uint64_t n, int rank) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x)
    out[cell[j]] = key[j] == ~0ull ? ~0ull : (((unsigned long long)(uint32_t)rank << 32) | j);
}

// Insertion order across a job (zdl_xplan.h): the sums as comm_sum_tables, and one MIN of the
// rank-tagged first ranks, so a pair sits where DependencyLinker.merge over the ranks' link()
// lists, concatenated in rank order, first sees it (DependencyLinker.java:189-204). Only the order
// of the tags matters (link_insertion sorts by them), so beyond 64 ranks each rank replaces its
// first ranks by their order among its own pairs (a local sort of its S x S cells) and tags that
// index with its rank in the upper 32 bits: any world size, no limit on the spans put.
static int comm_sum_ord(zdl_ctx* c) {
  const size_t SS = (size_t)c->rows * c->S;
  HIP_TRY(c, c->red_call.ensure(SS));
  HIP_TRY(c, c->red_err.ensure(SS));
  HIP_TRY(c, c->red_first.ensure(SS));
  const int world = c->comm_world;
  const char* lo = getenv("ZDL_ORD_LOCAL_ORDER");  // (tests: the local-order tags at any size)
  const unsigned g = (unsigned)std::min<size_t>((SS + 255) / 256, 4096);
  // (the choice is the job's: every rank sees the same world size)
  if (world > zdl_xplan::ORD_MAX_WORLD || (lo && lo[0] == '1')) {
    // (hipcub's item count is an int)
    if (SS >= (1ull << 31)) return fail(c, ZDL_EINVAL, "insertion order across ranks: a table of 2^31 cells or more");
    HIP_TRY(c, c->ord_lk.ensure(SS));
    HIP_TRY(c, c->ord_lv.ensure(SS));
    HIP_TRY(c, c->ord_lv2.ensure(SS));
    hipLaunchKernelGGL(k_iota32, dim3(g), dim3(256), 0, c->stream, c->ord_lv.p, (uint64_t)SS);
    size_t tb = 0;
    HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tb, c->first.p, c->ord_lk.p, c->ord_lv.p, c->ord_lv2.p,
                                                   (int)SS, 0, 64, c->stream));
    HIP_TRY(c, c->ord_ltmp.ensure(tb));
    HIP_TRY(c, hipcub::DeviceRadixSort::SortPairs(c->ord_ltmp.p, tb, c->first.p, c->ord_lk.p, c->ord_lv.p,
                                                   c->ord_lv2.p, (int)SS, 0, 64, c->stream));
    hipLaunchKernelGGL(k_ord_local, dim3(g), dim3(256), 0, c->stream, c->ord_lk.p, c->ord_lv2.p, c->red_first.p,
                       (uint64_t)SS, c->comm_rank);
  } else {
    if (c->span_base >= zdl_xplan::ORD_POS_LIMIT)
      return fail(c, ZDL_EINVAL, "insertion order across ranks: more than 2^56 spans put on this rank");
    hipLaunchKernelGGL(k_ord_tag, dim3(g), dim3(256), 0, c->stream, c->first.p, c->red_first.p, (uint64_t)SS,
                       c->comm_rank);
  }
  HIP_TRY(c, hipGetLastError());
  const XRed ops[3] = {{c->call.p, c->red_call.p, SS, 0}, {c->errc.p, c->red_err.p, SS, 0},
                       {c->red_first.p, c->red_first.p, SS, 1}};
  return x_allreduce(c, ops, 3);
}

// The sampled cells of a rank's sorted list: meta[0] = n, meta[1 + i] = cell at the middle of the
// i-th of q equal parts (zdl_xplan::range_split)
__global__ void k_x_samples(const uint32_t* __restrict__ cell, uint64_t n, uint32_t q, uint64_t* __restrict__ meta) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) meta[0] = n;
  if (i < q) meta[1 + i] = n ? cell[((2 * (uint64_t)i + 1) * n) / (2 * (uint64_t)q)] : 0;
}

// cnt[k] = entries of the sorted list in [split[k], split[k + 1]) (lower bounds; split[W] = 2^32)
__global__ void k_x_slices(const uint32_t* __restrict__ cell, uint64_t n, const uint64_t* __restrict__ split, int W,
                           uint64_t* __restrict__ cnt) {
  __shared__ uint64_t lb[zdl_xplan::MAX_WORLD + 1];
  for (int k = threadIdx.x; k <= W; k += blockDim.x) {
    const uint64_t v = split[k];
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if ((uint64_t)cell[mid] < v) lo = mid + 1; else hi = mid;
    }
    lb[k] = lo;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < W; k += blockDim.x) cnt[k] = lb[k + 1] - lb[k];
}

// Multi-rank jobs above 1024 services: a reduce-scatter by cell range,
// then an all-gather of the reduced ranges. Every rank's list is sorted by cell, so
//  1. each rank samples its list (q cells, and its length), one all-gather of the samples, and
//     every rank picks the same W - 1 splitters from them (zdl_xplan::range_split);
//  2. each rank's list falls into W contiguous slices, slice k to rank k: one all-gather of the
//     W x W slice lengths, then every slice to its rank (point to point, exact lengths);
//  3. each rank sums the W runs it received per cell (sparse_add: DependencyLinker.merge's sum)
//     - only its cell range, about 1/W of all entries;
//  4. one all-gather of the reduced ranges' lengths, then every range to every rank: ranges are
//     disjoint and ascending with the rank, so the rank-order concatenation is the job's list,
//     sorted, each cell once - no second sort.
// Per rank that moves ~(own list + job list) entries and sorts ~1/W of the job's entries, where
// gathering every list to every rank moved and sorted W lists (DESIGN §6 prices both at C5).
static int comm_sum_sparse(zdl_ctx* c) {
  const int W = c->comm_world, me = c->comm_rank;
  const hipStream_t st = c->stream;
  const uint32_t q = zdl_xplan::SPLIT_SAMPLES;
  const size_t mrow = 1 + (size_t)q;                 // one rank's sample block (u64)
  const size_t mw = (size_t)W * mrow;                // the gathered samples
  const size_t sw_off = 2 * mw, cnt_off = sw_off + (size_t)W + 1, cntg_off = cnt_off + (size_t)W;
  HIP_TRY(c, c->gx_n.ensure(cntg_off + (size_t)W * W + 2 * (size_t)W));
  uint64_t* meta = c->gx_n.p;
  // 1. samples -> splitters
  hipLaunchKernelGGL(k_x_samples, dim3((q + 255) / 256), dim3(256), 0, st, (const uint32_t*)c->acc.cell,
                     (uint64_t)c->acc.n, q, meta + mw);
  HIP_TRY(c, hipGetLastError());
  if (const int rc = x_allgather(c, meta + mw, meta, mrow * 8)) return rc;
  std::vector<uint64_t> hm(mw);
  HIP_TRY(c, hipMemcpyAsync(hm.data(), meta, mw * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  const std::vector<uint64_t> split = zdl_xplan::range_split(hm.data(), W, q);
  HIP_TRY(c, hipMemcpyAsync(meta + sw_off, split.data(), ((size_t)W + 1) * 8, hipMemcpyHostToDevice, st));
  // 2. slice lengths, the W x W matrix, the all-to-all of the slices
  hipLaunchKernelGGL(k_x_slices, dim3(1), dim3(64), 0, st, (const uint32_t*)c->acc.cell, (uint64_t)c->acc.n,
                     (const uint64_t*)(meta + sw_off), W, meta + cnt_off);
  HIP_TRY(c, hipGetLastError());
  if (const int rc = x_allgather(c, meta + cnt_off, meta + cntg_off, (size_t)W * 8)) return rc;
  std::vector<uint64_t> cnt((size_t)W * W);
  HIP_TRY(c, hipMemcpyAsync(cnt.data(), meta + cntg_off, cnt.size() * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  const zdl_xplan::Plan a2a = zdl_xplan::slice_plan(cnt.data(), W, me);
  const uint64_t rtot = a2a.total();
  HIP_TRY(c, c->gx_cell.ensure(std::max<uint64_t>(rtot, 1)));
  HIP_TRY(c, c->gx_call.ensure(std::max<uint64_t>(rtot, 1)));
  HIP_TRY(c, c->gx_err.ensure(std::max<uint64_t>(rtot, 1)));
  std::vector<XSend> sends;
  std::vector<XRecv> recvs;
  for (const zdl_xplan::Xfer& x : a2a.ops) {
    if (x.src == me && x.dst == me) {  // my own slice: a device copy
      HIP_TRY(c, hipMemcpyAsync(c->gx_cell.p + x.at, c->acc.cell + x.from, x.n * 4, hipMemcpyDeviceToDevice, st));
      HIP_TRY(c, hipMemcpyAsync(c->gx_call.p + x.at, c->acc.call + x.from, x.n * 8, hipMemcpyDeviceToDevice, st));
      HIP_TRY(c, hipMemcpyAsync(c->gx_err.p + x.at, c->acc.err + x.from, x.n * 8, hipMemcpyDeviceToDevice, st));
    } else if (x.src == me) {
      sends.push_back({x.dst, c->acc.cell + x.from, x.n * 4});
      sends.push_back({x.dst, c->acc.call + x.from, x.n * 8});
      sends.push_back({x.dst, c->acc.err + x.from, x.n * 8});
    } else {
      recvs.push_back({x.src, c->gx_cell.p + x.at, x.n * 4});
      recvs.push_back({x.src, c->gx_call.p + x.at, x.n * 8});
      recvs.push_back({x.src, c->gx_err.p + x.at, x.n * 8});
    }
  }
  if (const int rc = x_exchange(c, sends, recvs)) return rc;
  // 3. this rank's range, summed per cell
  c->gslice.n = 0;
  int kb = 1;
  while ((1ull << kb) < (uint64_t)c->S * c->S) ++kb;
  HIP_TRY(c, sparse_add(c->sw, c->gslice, c->gx_cell.p, c->gx_call.p, c->gx_err.p, rtot, kb, st));
  // 4. every reduced range to every rank, in rank order
  uint64_t* rn = meta + cntg_off + (size_t)W * W;
  HIP_TRY(c, hipMemcpyAsync(rn + W, &c->gslice.n, 8, hipMemcpyHostToDevice, st));
  if (const int rc = x_allgather(c, rn + W, rn, 8)) return rc;
  std::vector<uint64_t> n((size_t)W);
  HIP_TRY(c, hipMemcpyAsync(n.data(), rn, 8 * (size_t)W, hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  const zdl_xplan::Plan plan = zdl_xplan::gather_plan(n.data(), W, true);  // every range to every rank
  const uint64_t total = plan.total();
  HIP_TRY(c, sparse_reserve(c->gacc, total));
  sends.clear();
  recvs.clear();
  for (const zdl_xplan::Xfer& x : plan.ops) {
    if (x.src == me && x.dst == me) {
      HIP_TRY(c, hipMemcpyAsync(c->gacc.cell + x.at, c->gslice.cell, x.n * 4, hipMemcpyDeviceToDevice, st));
      HIP_TRY(c, hipMemcpyAsync(c->gacc.call + x.at, c->gslice.call, x.n * 8, hipMemcpyDeviceToDevice, st));
      HIP_TRY(c, hipMemcpyAsync(c->gacc.err + x.at, c->gslice.err, x.n * 8, hipMemcpyDeviceToDevice, st));
    } else if (x.src == me) {
      sends.push_back({x.dst, c->gslice.cell, x.n * 4});
      sends.push_back({x.dst, c->gslice.call, x.n * 8});
      sends.push_back({x.dst, c->gslice.err, x.n * 8});
    } else if (x.dst == me) {
      recvs.push_back({x.src, c->gacc.cell + x.at, x.n * 4});
      recvs.push_back({x.src, c->gacc.call + x.at, x.n * 8});
      recvs.push_back({x.src, c->gacc.err + x.at, x.n * 8});
    }
  }
  if (const int rc = x_exchange(c, sends, recvs)) return rc;
  c->gacc.n = total;
  return ZDL_OK;
}

extern "C" {

int zdl_comm_unique_id(uint8_t* out) {
  if (!out) return ZDL_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return ZDL_EDEVICE;
  memcpy(out, &id, sizeof id);
  return ZDL_OK;
}

int zdl_comm_init(zdl_ctx* c, const uint8_t* id, int rank, int world) {
  if (!c || !id || world < 1 || rank < 0 || rank >= world) return fail(c, ZDL_EINVAL, "zdl_comm_init: bad rank / world");
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_comm_init: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!c->sub.empty()) return fail(c, ZDL_EINVAL, "zdl_comm_init: a device group has its own communicator");
  if (c->days) return fail(c, ZDL_EINVAL, "zdl_comm_init: daily buckets are per process");
  if (in_job(c)) return fail(c, ZDL_EINVAL, "zdl_comm_init: already joined");
  if (c->sparse && world > zdl_xplan::MAX_WORLD) return fail(c, ZDL_EINVAL, "zdl_comm_init: a sparse job has at most 1024 ranks");
  HIP_TRY(c, enter(c));
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  const ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
  if (r != ncclSuccess) {
    c->comm = nullptr;
    return fail(c, ZDL_EDEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  c->comm_rank = rank;
  c->comm_world = world;
  return ZDL_OK;
}

int zdl_comm_init_local(zdl_ctx* const* ctxs, int world) {
  if (!ctxs || world < 1 || world > zdl_xplan::MAX_WORLD) return ZDL_EINVAL;
  for (int k = 0; k < world; ++k) {
    zdl_ctx* c = ctxs[k];
    if (!c) return ZDL_EINVAL;
    for (int j = 0; j < k; ++j)
      if (ctxs[j] == c) return fail(c, ZDL_EINVAL, "zdl_comm_init_local: a context listed twice");
    if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_comm_init_local: a started link is not finished (zdl_link_finish)");
    if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
    if (!c->sub.empty()) return fail(c, ZDL_EINVAL, "zdl_comm_init_local: a device group has its own communicator");
    if (c->days) return fail(c, ZDL_EINVAL, "zdl_comm_init_local: daily buckets are per process");
    if (in_job(c)) return fail(c, ZDL_EINVAL, "zdl_comm_init_local: already joined");
    const zdl_ctx* c0 = ctxs[0];
    if (c->device != c0->device || c->S != c0->S || c->rows != c0->rows || c->sparse != c0->sparse || c->ord != c0->ord)
      return fail(c, ZDL_EINVAL, "zdl_comm_init_local: the ranks need one device, one service count and one mode");
  }
  LocalWorld* w = new LocalWorld;
  w->W = world;
  w->device = ctxs[0]->device;
  w->refs = world;
  w->board.resize((size_t)world);
  if (const char* e = getenv("ZDL_LOCAL_WORLD_TIMEOUT_S")) {
    const double t = atof(e);
    if (t > 0) w->timeout_s = t;
  }
  for (int k = 0; k < world; ++k) {
    ctxs[k]->lworld = w;
    ctxs[k]->comm_rank = k;
    ctxs[k]->comm_world = world;
  }
  return ZDL_OK;
}

int zdl_put_spans_device_multi(zdl_ctx* c, const zdl_span_cols* cols, const uint64_t* n_spans,
                               const uint64_t* const* offsets, const uint64_t* n_traces) {
  if (!c || !cols || !n_spans || !offsets || !n_traces) return fail(c, ZDL_EINVAL, "null argument");
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_put_spans_device_multi: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (c->sub.empty()) return zdl_put_spans_device(c, &cols[0], n_spans[0], offsets[0], n_traces[0]);
  for (size_t d = 0; d < c->sub.size(); ++d) {
    const int rc = zdl_put_spans_device(c->sub[d], &cols[d], n_spans[d], offsets[d], n_traces[d]);
    if (rc != ZDL_OK) return group_first(c, rc, c->sub[d]);
  }
  return ZDL_OK;
}

int zdl_device_count(const zdl_ctx* c) { return !c ? 0 : (c->sub.empty() ? 1 : (int)c->sub.size()); }

void zdl_shard_of(const uint64_t* trace_lo, uint64_t n, uint32_t n_shards, uint32_t* out) {
  for (uint64_t i = 0; i < n; ++i) out[i] = n_shards ? (uint32_t)(splitmix64(trace_lo[i]) % n_shards) : 0u;
}

}  // extern "C"

extern "C" {

int zdl_tree_export(zdl_ctx* c, int32_t* node_of, int32_t* parent, int32_t* bfs, uint64_t n) {
  if (!c || !node_of || !parent || !bfs) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_tree_export: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!(c->flags & (ZDL_FLAG_TREE_EXPORT | ZDL_FLAG_TREE_STREAM)) || !c->sub.empty())
    return fail(c, ZDL_EINVAL, "context without ZDL_FLAG_TREE_EXPORT / ZDL_FLAG_TREE_STREAM");
  if (n != c->tr_n) return fail(c, ZDL_EINVAL, "zdl_tree_export: n must be the last put's span count");
  const int rc = zdl_sync(c);
  if (rc != ZDL_OK) return rc;
  if (n == 0) return ZDL_OK;
  HIP_TRY(c, hipMemcpy(node_of, c->tr_node.p, n * 4, hipMemcpyDeviceToHost));
  HIP_TRY(c, hipMemcpy(parent, c->tr_parent.p, n * 4, hipMemcpyDeviceToHost));
  HIP_TRY(c, hipMemcpy(bfs, c->tr_bfs.p, n * 4, hipMemcpyDeviceToHost));
  return ZDL_OK;
}

int zdl_tree_reasons(zdl_ctx* c, uint8_t* reason, int32_t* ancestor, int32_t* link, int32_t* sorted, uint64_t n) {
  if (!c || !reason || !ancestor || !link || !sorted) return ZDL_EINVAL;
  if (c->link_pending >= 0) return fail(c, ZDL_EINVAL, "zdl_tree_reasons: a started link is not finished (zdl_link_finish)");
  if (const int frc = stage_flush(c)) return frc;  // staged putTrace calls come first
  if (!(c->flags & (ZDL_FLAG_TREE_EXPORT | ZDL_FLAG_TREE_STREAM)) || !c->sub.empty())
    return fail(c, ZDL_EINVAL, "context without ZDL_FLAG_TREE_EXPORT / ZDL_FLAG_TREE_STREAM");
  if (n != c->tr_n) return fail(c, ZDL_EINVAL, "zdl_tree_reasons: n must be the last put's span count");
  const int rc = zdl_sync(c);
  if (rc != ZDL_OK) return rc;
  if (n == 0) return ZDL_OK;
  HIP_TRY(c, hipMemcpy(reason, c->tr_reason.p, n, hipMemcpyDeviceToHost));
  HIP_TRY(c, hipMemcpy(ancestor, c->tr_anc.p, n * 4, hipMemcpyDeviceToHost));
  HIP_TRY(c, hipMemcpy(link, c->tr_link.p, n * 16, hipMemcpyDeviceToHost));
  HIP_TRY(c, hipMemcpy(sorted, c->tr_sorted.p, n * 4, hipMemcpyDeviceToHost));
  return ZDL_OK;
}

}  // extern "C"

#include "zdl_stage.inc"  // zdl_put_trace: putTrace call by call, staged into batches
