/*
 * zdl.h — C ABI of the MI355X dependency-link engine (libzdl.so).
 *
 * This is the drop-in boundary for Zipkin's dependency-link hot path. The
 * reference has no native code; each entry point below replaces one Java
 * method of the path, and the JNI shim a maintainer would add calls exactly
 * these functions. Paths are relative to
 * /root/reference/zipkin/src/main/java/zipkin2/.
 *
 *   zdl_create / zdl_destroy  <- new DependencyLinker()          internal/DependencyLinker.java:42-48
 *   zdl_put_spans             <- DependencyLinker.putTrace(List)  internal/DependencyLinker.java:53-151
 *                                (one call = many putTrace calls: CSR-grouped traces)
 *   zdl_link                  <- DependencyLinker.link()          internal/DependencyLinker.java:184-186,206-219
 *   zdl_merge_links           <- DependencyLinker.merge(Iterable) internal/DependencyLinker.java:189-204
 *   zdl_set_window            <- the QueryRequest.test time rule  storage/QueryRequest.java:262-279
 *                                used by InMemoryStorage.getDependencies(endTs, lookback)
 *                                storage/InMemoryStorage.java:323-348
 *   status ZDL_EREF_NPE       <- the NullPointerException Span.Builder.merge throws
 *                                (Span.java:375-379 -> Endpoint.java:121-129)
 *
 * Conventions: plain C, plain pointers and sizes. Return 0 (ZDL_OK) or a
 * negative status; zdl_last_error() has the message. A context is used by one
 * thread at a time (DependencyLinker is not thread-safe either); separate
 * contexts may run concurrently. Every context owns one HIP stream on its
 * device. Strings never cross this boundary: services, ipv4 and ipv6
 * addresses are dictionary ids assigned by the caller, with optional rank
 * tables giving each id's position in java.lang.String.compareTo order
 * (needed because Trace.merge sorts endpoints by string, Trace.java:105-116).
 */
#ifndef ZDL_H
#define ZDL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZDL_ABI_VERSION 7  /* 2: zdl_config.n_devices / device_ids, RCCL combine; 3: zdl_kernel_times
                              per phase of a put (mid_ms, giant_ms, sparse_ms); 4: trace id widths
                              (zdl_store_append_ids, zdl_decoded.dev_trace_wide); 5: zdl_put_trace,
                              a trace whose Trace.merge throws adds nothing, a started link locks
                              the context until zdl_link_finish; 6: zdl_comm_init_local (a job of
                              contexts of one process), a sparse job sums by reduce-scatter; 7: zdl_kernel_times
                              log_entries / sparse_entries (the reduce's and the merge's inputs) */

/* ---- status codes ---- */
#define ZDL_OK          0
#define ZDL_EINVAL     (-1)  /* bad argument (offsets not monotone, service id >= n_services, ...) */
#define ZDL_ENOMEM     (-2)  /* device or host allocation failed */
#define ZDL_EDEVICE    (-3)  /* HIP runtime error */
#define ZDL_EREF_NPE   (-4)  /* the reference throws NullPointerException for this input (quirk Q1) */
#define ZDL_EREF_IAE   (-5)  /* the reference throws IllegalArgumentException for this input */
#define ZDL_EREF_NSE   (-6)  /* the reference throws NoSuchElementException (an eviction that
                                empties the store, InMemoryStorage.java:184-196) */

/* ---- port_flags column bit layout (one u32 per span) ---- */
#define ZDL_PF_PORT_MASK     0x0000FFFFu /* local endpoint port, 0 = null (Endpoint.java:245-260) */
#define ZDL_PF_KIND_SHIFT    16          /* 3 bits: Span.Kind ordinal, 7 = null */
#define ZDL_KIND_CLIENT      0u
#define ZDL_KIND_SERVER      1u
#define ZDL_KIND_PRODUCER    2u
#define ZDL_KIND_CONSUMER    3u
#define ZDL_KIND_NULL        7u
#define ZDL_PF_SHARED_SHIFT  19          /* 2 bits: 0 = shared null, 1 = false, 2 = true */
#define ZDL_PF_ERROR         (1u << 21)  /* tags contain the key "error" */
#define ZDL_PF_RIP4          (1u << 22)  /* remote endpoint carries an ipv4 */
#define ZDL_PF_RIP6          (1u << 23)  /* remote endpoint carries an ipv6 */
#define ZDL_PF_RPORT         (1u << 24)  /* remote endpoint carries a port */

/* ---- dictionaries whose ranks can be set ---- */
#define ZDL_DICT_SERVICE 0
#define ZDL_DICT_IPV4    1
#define ZDL_DICT_IPV6    2
/* JSON v2 decoder keys (zdl_decode_json_v2): the raw JSON text of a service-name token (string
 * content with its escapes, or a number's text: the binder unescapes and lower-cases it), an
 * ipv4 address text as Endpoint keeps it (Endpoint.java:222-227), and - in the missing-key list
 * only - an ipv6 address text, to be bound as its 16 bytes under ZDL_DICT_IPV6. */
#define ZDL_DICT_JSON_SERVICE  3
#define ZDL_DICT_JSON_IPV4     4
#define ZDL_DICT_JSON_IPV6TEXT 5

/* ---- output order for zdl_link ---- */
#define ZDL_ORDER_SORTED      0  /* by (rank[parent], rank[child]) */
#define ZDL_ORDER_FIRST_SEEN  1  /* only for zdl_merge_links output: DependencyLinker.merge order */
#define ZDL_ORDER_INSERTION   2  /* DependencyLinker.link() order: the LinkedHashMap insertion order of
                                    addLink (DependencyLinker.java:166-186) over the puts' traces in
                                    order, each tree breadth-first (SpanNode.java:64-89). Needs a
                                    context created with ZDL_FLAG_INSERTION_ORDER. */

/* ---- context flags ---- */
#define ZDL_FLAG_TIMING  1u      /* HIP events around k_link only: zdl_kernel_times.tiles_ms = mean of the
                                    puts since the previous zdl_get_kernel_times (last <= 64) */
#define ZDL_FLAG_TIMING_ALL 2u   /* record HIP events around every kernel (all zdl_kernel_times fields) */
#define ZDL_FLAG_INSERTION_ORDER 4u  /* keep, per (parent, child), the rank of its first addLink so that
                                        zdl_link can return ZDL_ORDER_INSERTION; puts take the exact
                                        per-trace path (slower than the default streaming path); any
                                        trace size */
#define ZDL_FLAG_DENSE_TABLE 16u     /* keep the S x S count table above 1024 services (a device group's
                                        and a multi-process job's RCCL reduce sums those tables); without
                                        it such a context keeps its links as one sorted list instead
                                        (a sparse context: no 16 * S^2 bytes of tables, S <= 46340) */
#define ZDL_FLAG_TREE_STREAM 32u     /* every put records, per span, the tree the path that linked it
                                        built - k_link's windows, k_mid, k_tail's big traces, the
                                        giant tier, the exact paths - without sending anything to the
                                        exact path: zdl_tree_export's node / parent, bfs = the traverse
                                        index on an insertion-order context, 0 for a visited node on a
                                        sorted one (-1 not visited), zdl_tree_reasons' ancestor =
                                        firstRemoteAncestor's slot (parity tests of the benchmarked
                                        kernels' trees; no time window) */
#define ZDL_FLAG_TREE_EXPORT 8u      /* with ZDL_FLAG_INSERTION_ORDER: every put also records the tree
                                        SpanNode.Builder builds (SpanNode.java:122-249), read back by
                                        zdl_tree_export (parity tests of the tree itself, not only its
                                        links) */

/*
 * Span columns, structure of arrays, n_spans entries each. A local endpoint is
 * null iff local_svc, local_ip4, local_ip6 are -1 and the port is 0; a remote
 * endpoint is null iff remote_svc is -1 and none of RIP4/RIP6/RPORT is set
 * (Span.Builder coerces empty endpoints to null, Span.java:527-536).
 */
typedef struct zdl_span_cols {
  const uint64_t* trace_lo;   /* low 64 bits of the trace id: read only to group ungrouped input
                                 (trace_offsets == NULL), like InMemoryStorage.getDependencies */
  const uint64_t* id;         /* span id, != 0 */
  const uint64_t* parent_id;  /* 0 = null; parent_id == id is treated as null (Span.java:611-617) */
  const int32_t*  local_svc;  /* service dictionary id, -1 = null */
  const int32_t*  remote_svc; /* service dictionary id, -1 = null */
  const int32_t*  local_ip4;  /* ipv4 dictionary id, -1 = null */
  const int32_t*  local_ip6;  /* ipv6 dictionary id, -1 = null */
  const uint32_t* port_flags; /* see ZDL_PF_* */
  const int64_t*  timestamp;  /* epoch micros, 0 = absent; read only when a window is set */
  const uint32_t* ord;        /* optional storage order within a trace (ungrouped input only);
                                 NULL = the input order is the storage order */
} zdl_span_cols;

typedef struct zdl_config {
  int32_t  device;      /* HIP device ordinal (device_ids == NULL) */
  uint32_t n_services;  /* service dictionary size S; links are counted in an S x S table */
  uint32_t flags;       /* ZDL_FLAG_* */
  uint32_t timing_stride; /* ZDL_FLAG_TIMING: time k_link on every stride-th put (0, 1: every put) */
  /* Device group: device_ids != NULL makes one context drive n_devices GPUs of
   * this process. zdl_put_spans shards whole traces by splitmix64(trace_lo) % n_devices (the
   * low 64 bits, as InMemoryStorage groups them, InMemoryStorage.java:163, 330, 465-467; the
   * trace_lo column is then required), every device links its shard, and zdl_link sums the
   * per-device tables on device_ids[0] with one RCCL reduce over xGMI (DependencyLinker.merge
   * semantics, DependencyLinker.java:189-204) before compacting. Sorted output only: not with
   * ZDL_FLAG_INSERTION_ORDER, zdl_set_days, the span store or mysql rows. n_devices = 1 with
   * device_ids set runs the same path on one device. */
  uint32_t n_devices;
  const int32_t* device_ids;
} zdl_config;

/* Links owned by the context; valid until the next zdl_link/zdl_merge_links/zdl_destroy. */
typedef struct zdl_links {
  uint64_t       n;
  const int32_t* parent;       /* service dictionary ids */
  const int32_t* child;
  const int64_t* call_count;
  const int64_t* error_count;
} zdl_links;

typedef struct zdl_kernel_times {  /* the last put's phases (ZDL_FLAG_TIMING_ALL) unless noted */
  float plan_ms;     /* unused (0): k_link plans its windows from the offsets itself */
  float tiles_ms;    /* k_link: every trace of <= 64 spans (ZDL_FLAG_TIMING: mean of the puts) */
  float big_ms;      /* k_tail: queued windows, traces > 64 spans k_mid and the giant tier left,
                        ordered compaction */
  float reduce_ms;   /* LOG mode's reduce of k_link's emit log (k_pscan .. k_hist) */
  float compact_ms;  /* zdl_link's compaction */
  uint32_t n_tiles, n_big, grid;  /* n_tiles: puts averaged into tiles_ms (ZDL_FLAG_TIMING) */
  float full_ms;     /* unused (0): k_tail runs the queued windows */
  float mid_ms;      /* k_mid: traces of 65..192 spans, one wave each */
  float giant_ms;    /* the device-wide big-trace tier (sparse contexts), host syncs included */
  float sparse_ms;   /* sparse contexts: gathering, sorting and merging the put's link log */
  uint64_t log_entries;     /* LOG mode: the entries k_link logged for the reduce (the hot corner's
                               links not included) */
  uint64_t sparse_entries;  /* sparse contexts: the link-log entries the merge sorted */
} zdl_kernel_times;

/* Context lifecycle. zdl_create returns NULL on failure (zdl_create_error() says why). */
typedef struct zdl_ctx zdl_ctx;
zdl_ctx*    zdl_create(const zdl_config* cfg);
const char* zdl_create_error(void);
void        zdl_destroy(zdl_ctx* ctx);
const char* zdl_last_error(const zdl_ctx* ctx);
int         zdl_abi_version(void);
/* Diagnostic: workgroups of the production k_link (table mode 0 hash, 1 dense, 2 LOG, 3 sorted
 * log; window 0/1) resident per CU on `device` (the design needs 2: 80 KB of LDS each); -1 on
 * error. */
int         zdl_link_occupancy(int device, int table_mode, int window);

/* rank[id] = position of dictionary string `id` in java.lang.String order. Without a
 * table the id itself is the rank. n must cover every id the columns use. */
int zdl_set_ranks(zdl_ctx* ctx, int dict, const int32_t* rank, uint32_t n);

/* Restrict subsequent puts to traces whose timestamp (QueryRequest.test rule) lies in
 * [(end_ts_ms - lookback_ms) * 1000, end_ts_ms * 1000]; lookback_ms <= 0 clears it. */
int zdl_set_window(zdl_ctx* ctx, int64_t end_ts_ms, int64_t lookback_ms);

/* putTrace over n_traces CSR-grouped traces from HOST buffers: trace t is spans
 * [trace_offsets[t], trace_offsets[t+1]) in storage order; trace_offsets has n_traces+1
 * entries, starts at 0 and ends at n_spans (at most 2^32 - 129 spans a put: split larger
 * inputs, the counts accumulate). Synchronous. Counts accumulate in the context across
 * calls. On ZDL_EREF_NPE the traces whose Trace.merge throws add nothing; the others of the
 * batch are counted (the status stays NPE until zdl_reset; zdl_put_trace clears it).
 * trace_offsets == NULL: the spans are ungrouped; they are grouped on the device by
 * trace_lo (stable in `ord`, else input order; n_traces is ignored, n_spans < 2^32),
 * as InMemoryStorage.getDependencies groups by lowTraceId (InMemoryStorage.java:323-332,
 * 448-467). */
int zdl_put_spans(zdl_ctx* ctx, const zdl_span_cols* cols, uint64_t n_spans,
                  const uint64_t* trace_offsets, uint64_t n_traces);

/* Same, with every pointer (columns and offsets) in device memory of the context's
 * device. Asynchronous on the context stream; errors surface at zdl_sync/zdl_link.
 * Lifetime: the put may still read the columns and offsets after this call returns - on a
 * small dense table its last kernels (k_mid / k_tail, only when some trace needs them) are
 * launched at the context's NEXT call (zdl_sync, zdl_link, zdl_link_start, zdl_reset, a put,
 * zdl_table_export, zdl_destroy). Keep them valid and unchanged until one of those has
 * returned; a device-wide synchronize (hipDeviceSynchronize) does not complete the put. */
int zdl_put_spans_device(zdl_ctx* ctx, const zdl_span_cols* dev_cols, uint64_t n_spans,
                         const uint64_t* dev_trace_offsets, uint64_t n_traces);

/* DependencyLinker.putTrace (internal/DependencyLinker.java:53) called once per trace, as the
 * reference's callers loop (storage/InMemoryStorage.java:340; mysql-v1
 * AggregateDependencies.java:81): `cols` holds ONE trace's n_spans spans (host memory, read
 * during the call only; trace_lo needed by device groups, timestamp when a window or days are
 * set). The trace is appended to a pinned staging batch that is put as one launch when it
 * fills (ZDL_STAGE_SPANS, default 2^20 spans) or when the context is next used for anything
 * else (zdl_link, zdl_sync, another put, a setting...), so traces are linked in call order.
 * A trace with two spans of one (id, shared) - the only input on which Trace.merge can throw -
 * is put alone and waited for: ZDL_EREF_NPE is returned by THIS call (quirk Q1), the trace adds
 * nothing, and the context stays usable, as the Java linker does after a caught throw. Errors
 * of a staged batch (ZDL_EINVAL: a service id >= n_services) are returned by the call that
 * flushes it or by the next zdl_sync / zdl_link. n_spans = 0 is a no-op (putTrace of an empty
 * list). zdl_reset drops staged traces with the counts. */
int zdl_put_trace(zdl_ctx* ctx, const zdl_span_cols* cols, uint64_t n_spans);

/* ---- device-resident span store (the ingest side of InMemoryStorage,
 * storage/InMemoryStorage.java:156-181 accept) ----
 * Spans are appended to HBM columns once (zdl_store_append copies the borrowed columns, host
 * or device memory, e.g. a zdl_decoded's; `timestamp` may be NULL = absent, `trace_lo` NULL =
 * 0). Each stored span also keeps its trace id (low and high 64 bits; high 0 for a 64-bit id)
 * and an alive byte, from which the store answers InMemoryStorage's questions on the device:
 * eviction (zdl_store_evict) and the trace selection of a query (zdl_store_select), which
 * zdl_put_selection gathers and links without leaving HBM. Positions count appends (0..size);
 * evicted spans keep theirs until zdl_store_compact_evicted / zdl_store_compact renumber. */
typedef struct zdl_store zdl_store;
zdl_store*  zdl_store_create(int device);
void        zdl_store_destroy(zdl_store* store);
const char* zdl_store_last_error(const zdl_store* store);
int         zdl_store_append(zdl_store* store, const zdl_span_cols* cols, uint64_t n_spans);
/* zdl_store_append with the high 64 bits of each span's trace id (NULL = all 0). */
int         zdl_store_append_traced(zdl_store* store, const zdl_span_cols* cols, const uint64_t* trace_hi,
                                    uint64_t n_spans);
/* ... and each trace id's width (1 = 128-bit: Span.normalizeTraceId gave 32 hex characters, which
 * a 17-31 character id does even when its high half is zero; 0 = 64-bit). trace_wide NULL:
 * 128-bit exactly when trace_hi != 0 (true for every id a proto3 decoder reads). The strict
 * no-argument getDependencies() groups by (low, high, width): the reference's strictByTraceId
 * compares the normalized strings (InMemoryStorage.java:241-262). */
int         zdl_store_append_ids(zdl_store* store, const zdl_span_cols* cols, const uint64_t* trace_hi,
                                 const uint8_t* trace_wide, uint64_t n_spans);
int         zdl_store_clear(zdl_store* store);
/* Keeps the stored spans keep[0..n_keep) (ascending positions), in that order, and frees the
 * rest, in one device gather. Positions are renumbered 0..n_keep). */
int         zdl_store_compact(zdl_store* store, const uint32_t* keep, uint64_t n_keep);
/* Frees the evicted spans (what deleteOldestTrace releases, InMemoryStorage.java:193-211) in
 * one device gather; the alive spans keep their order and are renumbered. */
int         zdl_store_compact_evicted(zdl_store* store);
uint64_t    zdl_store_size(const zdl_store* store);   /* stored positions, evicted included */
uint64_t    zdl_store_alive(const zdl_store* store);  /* spans not evicted */
/* evictToRecoverSpans(to_recover) (InMemoryStorage.java:184-211): deleteOldestTrace - every
 * span of the low trace id whose smallest (timestamp, lowTraceId) key is the smallest - until
 * at least to_recover spans are gone; *evicted = their number. ZDL_EREF_NSE when the store
 * runs empty first (everything is evicted, as the reference's loop does before it throws). */
int         zdl_store_evict(zdl_store* store, uint64_t to_recover, uint64_t* evicted);
/* Trace selections of the alive spans, each trace in IMS storage order (spansByTraceId,
 * InMemoryStorage.java:448-454: distinct (lowTraceId, timestamp) keys in first-seen order,
 * then arrival): */
#define ZDL_SELECT_NEWEST     0  /* getDependencies(endTs, lookback) / getTraces(request): low
                                    trace ids by their newest timestamp, then lowTraceId, both
                                    descending (TIMESTAMP_DESCENDING, :272-291, 356-366) */
#define ZDL_SELECT_ALL        1  /* getTraces() (:251-262): low trace ids ascending */
#define ZDL_SELECT_ALL_STRICT 2  /* getTraces() with strictTraceId: each low trace id split by
                                    the full trace id, first-seen order (:241-249) */
/* Computes the selection on the device (kept by the store until the next change);
 * *n_sel spans in *n_traces traces. */
int         zdl_store_select(zdl_store* store, int mode, uint64_t* n_sel, uint64_t* n_traces);
/* Copies the current selection out: perm[0..n_sel) positions, trace_offsets[0..n_traces]. */
int         zdl_store_selection(const zdl_store* store, uint32_t* perm, uint64_t* trace_offsets);
/* Links the store's current selection (zdl_put_stored without the upload). Synchronous. */
int         zdl_put_selection(zdl_ctx* ctx, const zdl_store* store);
/* Links the stored spans perm[0..n_sel) (host) as CSR-grouped traces (trace t = positions
 * [trace_offsets[t], trace_offsets[t+1]) of perm, storage order), like zdl_put_spans would on
 * the gathered columns. Synchronous. The store may serve any context of its device. */
int zdl_put_stored(zdl_ctx* ctx, const zdl_store* store, const uint32_t* perm, uint64_t n_sel,
                   const uint64_t* trace_offsets, uint64_t n_traces);

/* ZDL_FLAG_TREE_EXPORT: the last put's trees, per input span i (its column index in the put):
 * node_of[i] = column index of the head fragment of the cleaned span i belongs to (Trace.merge,
 * Trace.java:28-87: the first fragment of its merge run in sorted order); parent[i] = the
 * parent node's head index, -1 the synthetic root (SpanNode.java:145-147), -2 i is the root,
 * -3 i is not a tree node (an absorbed fragment or a span SpanNode.Builder leaves out);
 * bfs[i] = the node's index in SpanNode.traverse order (SpanNode.java:64-89; the synthetic root
 * not counted), -1 unreachable. n = the last put's span count. Synchronous. */
int zdl_tree_export(zdl_ctx* ctx, int32_t* node_of, int32_t* parent, int32_t* bfs, uint64_t n);

/* ZDL_FLAG_TREE_EXPORT, the FINE log of DependencyLinker / SpanNode.Builder
 * (DependencyLinker.java:57-169, SpanNode.java:130, 145-147, 227-231) as codes, per input span i
 * of the last put (meaningful for node heads, node_of[i] == i): reason[i] = the branch putTrace
 * took for the node (low 3 bits, ZDL_RSN_NONE for a node the traversal never visits) | flags;
 * ancestor[i] = head slot of firstRemoteAncestor's span (ZDL_RSN_ANCESTOR), else -1;
 * link[4i..4i+3] = (parent, child) service ids of the node's link and (parent, child) of the
 * missing-link backfill (ZDL_RSN_MISSING_LINK), -1 when absent; sorted[i] = the span's position
 * in its trace after Trace.merge's sort (CLEANUP_COMPARATOR, Trace.java:88-97). Synchronous. */
#define ZDL_RSN_NONE                0
#define ZDL_RSN_CLIENT_PARENT       1  /* client span with children: skipped without a message */
#define ZDL_RSN_NON_REMOTE          2  /* "non remote span; skipping" */
#define ZDL_RSN_ROOT_CLIENT_UNKNOWN 3  /* "root's client is unknown; skipping" */
#define ZDL_RSN_MESSAGING           4  /* producer/consumer link */
#define ZDL_RSN_MESSAGING_NO_BROKER 5  /* "cannot link messaging span to its broker; skipping" */
#define ZDL_RSN_LINK                6  /* link (after firstRemoteAncestor) */
#define ZDL_RSN_NO_REMOTE_ANCESTOR  7  /* "cannot find remote ancestor; skipping" */
#define ZDL_RSN_ANCESTOR            8  /* flag: "found remote ancestor <span>" */
#define ZDL_RSN_MISSING_LINK       16  /* flag: "detected missing link to client span" + its link */
#define ZDL_RSN_ERROR              32  /* flag: the node's link is an error link */
#define ZDL_RSN_ATTRIBUTED         64  /* flag: "attributing span missing parent to root" */
int zdl_tree_reasons(zdl_ctx* ctx, uint8_t* reason, int32_t* ancestor, int32_t* link, int32_t* sorted, uint64_t n);

/* Waits for the context stream and reports device-side status (e.g. ZDL_EREF_NPE). */
int zdl_sync(zdl_ctx* ctx);

/* DependencyLinker.link(): materialise the accumulated counts. The context keeps
 * them (link() may be called again, like the reference). order: ZDL_ORDER_SORTED, or
 * ZDL_ORDER_INSERTION on a ZDL_FLAG_INSERTION_ORDER context (the reference's list order). */
int zdl_link(zdl_ctx* ctx, int order, zdl_links* out);

/* zdl_link in two halves, so that the link list's trip over PCIe into the context's pinned
 * host columns overlaps other work (e.g. the next put on another context): zdl_link_start
 * enqueues the compaction and returns; zdl_link_finish waits for it and fills out exactly as
 * zdl_link would. A sparse context's sorted list is compacted asynchronously; every other case
 * computes in zdl_link_finish. Nothing else may use the context in between. */
int zdl_link_start(zdl_ctx* ctx, int order);
int zdl_link_finish(zdl_ctx* ctx, zdl_links* out);

/* DependencyLinker.merge(links): sums call/error counts per (parent, child) of the n
 * input links, on the device; output in first-seen order (ZDL_ORDER_FIRST_SEEN).
 * Does not touch the context's accumulated counts. */
int zdl_merge_links(zdl_ctx* ctx, const int32_t* parent, const int32_t* child,
                    const int64_t* call_count, const int64_t* error_count, uint64_t n,
                    zdl_links* out);

/* Adds n pre-aggregated links to the context's accumulated counts (what
 * DependencyLinker.merge does for stores that keep daily links, e.g.
 * cassandra SelectDependencies.java:75-91); used when a context is re-created with a
 * larger service dictionary. On a ZDL_FLAG_INSERTION_ORDER context the n links count as
 * first seen in their input order, before anything put afterwards. Synchronous. */
int zdl_add_links(zdl_ctx* ctx, const int32_t* parent, const int32_t* child,
                  const int64_t* call_count, const int64_t* error_count, uint64_t n);

/* Clears the accumulated counts and the sticky device status. */
int zdl_reset(zdl_ctx* ctx);

/* Multi-GPU combine support: copy the S x S int64 call and error tables to/from device
 * buffers of the same device (e.g. for an RCCL all-reduce), ordered on the ctx stream.
 * zdl_table_import is refused on a ZDL_FLAG_INSERTION_ORDER context (no first-seen ranks).
 * A device group exports the sum over its devices into buffers on device_ids[0] and imports
 * into device_ids[0] (the other devices are reset); a rank that joined a job (zdl_comm_init)
 * exports the sum over the ranks. */
int zdl_table_export(zdl_ctx* ctx, void* dev_call, void* dev_err);
int zdl_table_import(zdl_ctx* ctx, const void* dev_call, const void* dev_err);

/* ---- multi-process jobs (one process per GPU, e.g. torch.distributed.run): each process
 * makes a one-device context and joins one RCCL communicator; from then on zdl_link and
 * zdl_table_export of every rank sum the tables of all ranks (ncclAllReduce over xGMI) and
 * return the job's links (ZDL_ORDER_INSERTION: DependencyLinker.merge over the ranks' lists in
 * rank order). Rank 0 makes the id and sends its 128 bytes to the others. Not with daily
 * buckets. ---- */
#define ZDL_COMM_ID_BYTES 128
int zdl_comm_unique_id(uint8_t* out /* ZDL_COMM_ID_BYTES */);
int zdl_comm_init(zdl_ctx* ctx, const uint8_t* id, int rank, int world);

/* A job of `world` contexts of THIS process (ctxs[k] becomes rank k), all on one device, with
 * one service count and mode: the same combines as an RCCL job (zdl_link / zdl_table_export of
 * every rank return the job's links, insertion order included), the transport being device
 * copies and an element-wise reduce kernel instead of RCCL (zipkin_amd/csrc/zdl_xport.inc).
 * Like the processes of an RCCL job, the ranks' zdl_link (or zdl_table_export) calls must run
 * concurrently, one thread per context; a rank that never arrives makes the others fail after
 * ZDL_LOCAL_WORLD_TIMEOUT_S seconds (default 120). For shards that share a GPU, and for testing
 * a job's combines on one GPU. Destroying any rank's context ends the job for all. */
int zdl_comm_init_local(zdl_ctx* const* ctxs, int world);

/* Device-resident, already sharded input of a device group: cols[d] / n_spans[d] /
 * offsets[d] / n_traces[d] live on device_ids[d] (zdl_put_spans_device per device,
 * asynchronous). On a one-device context, entry 0 only. */
int zdl_put_spans_device_multi(zdl_ctx* ctx, const zdl_span_cols* cols, const uint64_t* n_spans,
                               const uint64_t* const* offsets, const uint64_t* n_traces);
int zdl_device_count(const zdl_ctx* ctx);
/* out[i] = splitmix64(trace_lo[i]) % n_shards: the device (or rank) of a trace. Host only. */
void zdl_shard_of(const uint64_t* trace_lo, uint64_t n, uint32_t n_shards, uint32_t* out);

/* ---- daily buckets (the zipkin-dependencies job; ITDependencies.aggregateLinks,
 * zipkin/src/test/java/zipkin2/storage/ITDependencies.java:666-700) ----
 * zdl_set_days: from now on every trace is linked into the bucket of its day - the
 * flooredTraceTimestamp rule over its spans in storage order (:680-690), with `timestamp`
 * holding guessTimestamp (Span.timestamp, else the first annotation's, :692-700) - for the
 * n_days (<= 255) UTC days from day0_ms (a midnight). A trace without a timestamp or
 * outside the range fails the put (ZDL_EINVAL); with ZDL_DAYS_SKIP_OUTSIDE or-ed into n_days
 * a trace whose day lies outside the range is skipped instead (a caller covers a long span
 * of days by putting the same batch once per range of days). Resets the counts; n_days = 0
 * turns it off. Not with a time window. Dense and hash tables hold n_days * S * S cells
 * (< 2^32); zdl_table_export/import move all of them. A sparse context (above 1024 services)
 * keeps its one sorted list with the day in the cell - (day * S + parent) * S + child, below
 * 2^31 - so no table is allocated per day; it links in ZDL_ORDER_SORTED only. zdl_link is
 * refused while days are set: */
#define ZDL_DAYS_SKIP_OUTSIDE 0x80000000u
int zdl_set_days(zdl_ctx* ctx, int64_t day0_ms, uint32_t n_days);

typedef struct zdl_day_links {
  uint64_t       n_days;
  const int64_t* day_ms;       /* the days that hold a trace (with or without links):
                                  ZDL_ORDER_INSERTION first-seen order, else ascending */
  uint64_t       n;
  const int64_t* day;          /* per link: its midnight (ms) */
  const int32_t* parent;
  const int32_t* child;
  const int64_t* call_count;
  const int64_t* error_count;
} zdl_day_links;

/* The per-day link lists: ZDL_ORDER_INSERTION = aggregateLinks' LinkedHashMap (days in
 * the order their first trace was put, each day's links in DependencyLinker.link() order;
 * needs ZDL_FLAG_INSERTION_ORDER), ZDL_ORDER_SORTED = by (day, parent, child). Owned by the
 * context until the next link call. */
int zdl_link_days(zdl_ctx* ctx, int order, zdl_day_links* out);

/* ---- proto3 ingest: SpanBytesDecoder.PROTO3.decodeList(bytes)
 * (codec/SpanBytesDecoder.java:144-152, internal/Proto3Codec.java readList,
 * internal/Proto3ZipkinFields.java:309-369) decoded on the device straight to span columns.
 * Strings map to dictionary ids by the decoder's table of RAW keys: service names as the
 * field's UTF-8 bytes before toLowerCase, ipv4 as 4 bytes, ipv6 as 16 bytes (after
 * Endpoint.Builder.parseIp(byte[]), Endpoint.java:179-198). A decode that meets keys the
 * table lacks returns ZDL_OK with n_missing > 0 and no columns: the caller assigns ids
 * (lower-cased name -> its dictionary, first-seen order; zdl_decoder_missing lists the keys
 * in (span, slot) order: local service, local ipv4, local ipv6, remote service), binds them
 * and calls zdl_decode_proto3_retry, which re-runs on the resident batch.
 * Status: ZDL_EREF_IAE where the reference throws IllegalArgumentException; ZDL_EINVAL for
 * input the reference reads leniently across a message end (not supported). An empty
 * input or a zero-length span message gives n_spans = 0 (the reference's empty list). */
typedef struct zdl_decoder zdl_decoder;
typedef struct zdl_decoded {
  uint64_t        n_spans;
  zdl_span_cols   dev;        /* device columns owned by the decoder (ord NULL), valid until
                                 the next decode; feed zdl_put_spans_device / zdl_store_append */
  const uint64_t* trace_lo;   /* NULL (ABI 3): nothing is copied to the host; zdl_decoder_download */
  const int64_t*  timestamp;  /* copies the columns a caller needs */
  uint64_t        n_missing;  /* > 0: bind the keys, then zdl_decode_proto3_retry */
  const uint64_t* dev_trace_hi; /* device: each span's trace id high 64 bits (0 = 64-bit id), for
                                   zdl_store_append_traced */
  const uint8_t*  dev_trace_wide; /* device: each trace id's width (1 = 128-bit), for
                                     zdl_store_append_ids; NULL: 128-bit iff dev_trace_hi != 0 */
} zdl_decoded;
zdl_decoder* zdl_decoder_create(int device);
void         zdl_decoder_destroy(zdl_decoder* dec);
const char*  zdl_decoder_last_error(const zdl_decoder* dec);
int          zdl_decoder_bind(zdl_decoder* dec, int dict, const uint8_t* key, uint32_t len, int32_t id);
uint64_t     zdl_decoder_dict_size(const zdl_decoder* dec);
float        zdl_decoder_kernel_ms(const zdl_decoder* dec);  /* HIP-event time of the last decode kernel */
int          zdl_decoder_missing(const zdl_decoder* dec, uint64_t i, int* dict, const uint8_t** key,
                                 uint32_t* len);
int          zdl_decode_proto3(zdl_decoder* dec, const uint8_t* bytes, uint64_t len, zdl_decoded* out);
int          zdl_decode_proto3_retry(zdl_decoder* dec, zdl_decoded* out);  /* = zdl_decode_retry */
/* Re-runs the last decode (proto3 or JSON v2) on the resident batch after binds. */
int          zdl_decode_retry(zdl_decoder* dec, zdl_decoded* out);
/* ---- JSON v2 ingest: SpanBytesDecoder.JSON_V2.decodeList(bytes)
 * (codec/SpanBytesDecoder.java:94-120, internal/JsonCodec.java:142-155, internal/V2SpanReader.java
 * over gson 2.8.5's strict JsonReader) decoded on the device to span columns. The same
 * dictionary protocol as proto3 with the ZDL_DICT_JSON_* keys. Empty input or an empty array
 * gives n_spans = 0 (the reference's empty list); ZDL_EREF_IAE where the reference throws
 * IllegalArgumentException (the first failing span decides, as in the sequential read);
 * ZDL_EINVAL for what the decoder does not restate: a timestamp / duration / port written as a
 * fraction, exponent or out-of-range integer (the reference's Double.parseDouble fallback), an
 * ip string with an escape, nesting deeper than 64 inside a span; batches up to 4 GiB. */
int          zdl_decode_json_v2(zdl_decoder* dec, const uint8_t* bytes, uint64_t len, zdl_decoded* out);
float        zdl_decoder_struct_ms(const zdl_decoder* dec);  /* HIP-event time of the last JSON structure passes */
/* Spans of the last JSON decode read by the exact reader (the rest took the fast path: compact,
 * unescaped, no annotations; see zdl_json.inc). Every span when ZDL_JS_EXACT=1 was set at
 * zdl_decoder_create. Diagnostic. */
uint64_t     zdl_decoder_exact_spans(const zdl_decoder* dec);
/* copies the last decode's device columns into the non-NULL host columns of dst */
int          zdl_decoder_download(zdl_decoder* dec, const zdl_span_cols* dst);

/* ---- mysql-v1 rows: AggregateDependencies.apply's loop
 * (zipkin-storage/mysql-v1/.../AggregateDependencies.java:71-84) over its cursor: rows grouped by
 * trace then span id (the query's groupBy), each span's rows projected to a minimal span by
 * DependencyLinkV2SpanIterator.next (DependencyLinkV2SpanIterator.java:88-159) on the device, the
 * spans put trace by trace (traces = runs of equal trace_lo, as ByTraceId compares only the low
 * 64 bits). Row columns may be host or device memory; synchronous.
 * `service` = raw dictionary id of ENDPOINT_SERVICE_NAME (-1 = SQL null or ""): raw strings, since
 * the "sa".equals("ca") check compares them before lower-casing; lower[raw] = the service id of
 * the lower-cased name (Endpoint.Builder.serviceName), which the counts use. */
#define ZDL_AKEY_NONE  0  /* a_key null or another key */
#define ZDL_AKEY_LC    1
#define ZDL_AKEY_CA    2
#define ZDL_AKEY_CS    3
#define ZDL_AKEY_SA    4
#define ZDL_AKEY_SR    5
#define ZDL_AKEY_ERROR 6
typedef struct zdl_mysql_rows {
  const uint64_t* trace_lo;   /* ZIPKIN_SPANS.TRACE_ID */
  const uint64_t* trace_hi;   /* TRACE_ID_HIGH, may be NULL (only checked for the all-zero id) */
  const uint64_t* span_id;    /* ZIPKIN_SPANS.ID */
  const uint64_t* parent_id;  /* 0 = SQL null */
  const uint8_t*  a_key;      /* ZDL_AKEY_* of ZIPKIN_ANNOTATIONS.A_KEY */
  const int32_t*  a_type;     /* A_TYPE (V1BinaryAnnotation.TYPE_STRING = 6 marks an error tag) */
  const int32_t*  service;    /* raw ENDPOINT_SERVICE_NAME id, -1 = null / empty */
} zdl_mysql_rows;
int         zdl_put_mysql_rows(zdl_ctx* ctx, const zdl_mysql_rows* rows, uint64_t n_rows,
                               const int32_t* lower, uint32_t n_raw);
const char* zdl_rows_last_error(void);  /* this thread's last zdl_put_mysql_rows failure */

/* Kernel durations of the most recent put (+ link) when ZDL_FLAG_TIMING is set. */
int zdl_get_kernel_times(zdl_ctx* ctx, zdl_kernel_times* out);

/* The hipStream_t of the context, as an opaque pointer. */
void* zdl_stream(zdl_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* ZDL_H */
