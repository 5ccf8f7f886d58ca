// zdl_rows.hip — mysql-v1 dependency rows straight to linked traces.
//
// Replaces AggregateDependencies.apply's loop (zipkin-storage/mysql-v1/src/main/java/zipkin2/
// storage/mysql/v1/AggregateDependencies.java:71-84): the cursor's rows (span columns left-joined
// with the lc/cs/ca/sr/sa/error annotations, grouped by trace then span) are projected to minimal
// spans by DependencyLinkV2SpanIterator (DependencyLinkV2SpanIterator.java:88-159) and put trace
// by trace into a DependencyLinker. Here one lane per span run does the projection and writes the
// span columns and the trace CSR offsets in HBM; the spans are then linked like any other put.
//
//   k_row_heads   : trace head = trace id (low 64 bits) differs from the previous row's
//                   (ByTraceId / hasNext compare the low bits only); span head = trace head or a
//                   span id change (next()'s run of rows for one span id)
//   exclusive scan: (trace heads << 32 | span heads) -> each head's trace and span index
//   k_row_project : the span's rows in order: last value per key wins, "error" sets
//                   error = (a_type == TYPE_STRING) each time; then the ca/cs/sa fallbacks and the
//                   sr / sa / cs cases of next()

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <string>

#include "../../include/zdl.h"

namespace zrows {

constexpr int32_t kTypeString = 6;  // V1BinaryAnnotation.TYPE_STRING (zipkin2/v1/V1BinaryAnnotation.java:33)

struct Rows {
  const uint64_t *lo, *hi, *id, *pid;
  const uint8_t* key;
  const int32_t *type, *svc;
  const int32_t* lower;  // raw service id -> service id of the lower-cased name (ep(..) lower-cases)
  uint32_t n_raw;
};

struct Cols {
  uint64_t *lo, *id, *pid;
  int32_t *lsvc, *rsvc, *ip4, *ip6;
  uint32_t* pf;
  int64_t* ts;
  uint64_t* off;
  uint32_t* status;  // bit 0: the reference throws IllegalArgumentException; bit 1: bad service id
};

__device__ __forceinline__ bool span_head(const Rows& r, uint64_t i, bool* trace_head) {
  const bool th = i == 0 || r.lo[i] != r.lo[i - 1];
  *trace_head = th;
  return th || r.id[i] != r.id[i - 1];
}

__global__ void k_row_heads(Rows r, uint64_t n, unsigned long long* heads) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool th;
  const bool sh = span_head(r, i, &th);
  heads[i] = (unsigned long long)th << 32 | (unsigned long long)sh;
}

__global__ void k_row_project(Rows r, uint64_t n, const unsigned long long* pos, Cols c) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool th;
  if (!span_head(r, i, &th)) return;
  const uint32_t s = (uint32_t)pos[i], t = (uint32_t)(pos[i] >> 32);
  if (th) c.off[t] = s;
  int32_t lc = -1, ca = -1, cs = -1, sa = -1, sr = -1;
  bool error = false;
  uint64_t j = i;
  do {
    const int32_t v = r.svc[j];
    const uint8_t k = r.key[j];
    if (v >= 0 && k != ZDL_AKEY_NONE) {  // key == null || value == null: neither client nor server
      if (v >= (int32_t)r.n_raw) atomicOr(c.status, 2u);
      switch (k) {
        case ZDL_AKEY_LC: lc = v; break;
        case ZDL_AKEY_CA: ca = v; break;
        case ZDL_AKEY_CS: cs = v; break;
        case ZDL_AKEY_SA: sa = v; break;
        case ZDL_AKEY_SR: sr = v; break;
        case ZDL_AKEY_ERROR: error = r.type[j] == kTypeString; break;
        default: break;
      }
    }
    ++j;
  } while (j < n && r.lo[j] == r.lo[i] && r.id[j] == r.id[i]);
  if (ca < 0) ca = cs;              // the client address is more authoritative than "cs"
  if (sa >= 0 && sa == ca) ca = -1;  // Finagle labels both socket sides alike: raw-string equality
  int32_t local = -1, remote = -1;
  uint32_t kind = ZDL_KIND_NULL;
  if (sr >= 0) {
    kind = ZDL_KIND_SERVER, local = sr, remote = ca;
  } else if (sa >= 0) {
    local = ca >= 0 ? ca : lc;
    kind = cs >= 0 ? ZDL_KIND_CLIENT : ZDL_KIND_NULL;
    remote = sa;
  } else if (cs >= 0) {
    kind = ZDL_KIND_SERVER, local = ca;
  }
  auto lower = [&](int32_t raw) { return raw >= 0 && raw < (int32_t)r.n_raw ? r.lower[raw] : -1; };
  const uint64_t id = r.id[i];
  const uint64_t hi = r.hi ? r.hi[i] : 0;
  if (id == 0 || (r.lo[i] == 0 && hi == 0)) atomicOr(c.status, 1u);  // Span.Builder.id / traceId throw
  const uint64_t pid = r.pid[i];
  c.lo[s] = r.lo[i];
  c.id[s] = id;
  c.pid[s] = pid == id ? 0 : pid;
  c.lsvc[s] = lower(local);
  c.rsvc[s] = lower(remote);
  c.ip4[s] = -1;
  c.ip6[s] = -1;
  c.pf[s] = kind << ZDL_PF_KIND_SHIFT | (error ? ZDL_PF_ERROR : 0u);
  c.ts[s] = 0;
  // the last span run closes the offsets; t counts the trace heads before row i, so a run that
  // is not itself a trace head belongs to trace t - 1
  if (j == n) c.off[(th ? t : t - 1) + 1] = s + 1;
}

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t want) {
    if (want <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc((void**)&p, std::max<size_t>(want, 1) * sizeof(T));
    if (e == hipSuccess) n = std::max<size_t>(want, 1);
    return e;
  }
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace zrows

using namespace zrows;

struct zdl_rows_buf {
  DBuf<uint64_t> lo, hi, id, pid;
  DBuf<uint8_t> key;
  DBuf<int32_t> type, svc, lower;
  DBuf<unsigned long long> heads, pos;
  DBuf<uint8_t> tmp;
  DBuf<uint64_t> c_lo, c_id, c_pid, c_off;
  DBuf<int32_t> c_lsvc, c_rsvc, c_ip4, c_ip6;
  DBuf<uint32_t> c_pf, status;
  DBuf<int64_t> c_ts;
};

namespace {
thread_local std::string g_rows_err;

#define ROWS_TRY(expr)                                                             \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      g_rows_err = std::string(#expr) + ": " + hipGetErrorString(_e);              \
      return _e == hipErrorOutOfMemory ? ZDL_ENOMEM : ZDL_EDEVICE;                 \
    }                                                                              \
  } while (0)
}  // namespace

extern "C" {

const char* zdl_rows_last_error(void) { return g_rows_err.c_str(); }

int zdl_put_mysql_rows(zdl_ctx* ctx, const zdl_mysql_rows* rows, uint64_t n_rows, const int32_t* lower,
                       uint32_t n_raw) {
  g_rows_err.clear();
  if (!ctx || !rows || (n_raw && !lower)) {
    g_rows_err = "null argument";
    return ZDL_EINVAL;
  }
  if (n_rows == 0) return ZDL_OK;
  if (!rows->trace_lo || !rows->span_id || !rows->parent_id || !rows->a_key || !rows->a_type || !rows->service) {
    g_rows_err = "missing row column";
    return ZDL_EINVAL;
  }
  if (n_rows >= (1ull << 32)) {
    g_rows_err = "at most 2^32 - 1 rows per call";
    return ZDL_EINVAL;
  }
  const hipStream_t s = (hipStream_t)zdl_stream(ctx);
  int dev = 0;
  ROWS_TRY(hipStreamGetDevice(s, &dev));
  ROWS_TRY(hipSetDevice(dev));
  // staging grows to the largest call of this thread; deliberately not freed at thread exit
  // (the HIP runtime may be gone by then); dropped when the thread moves to another device
  static thread_local zdl_rows_buf* bp = nullptr;
  static thread_local int bp_dev = -1;
  if (bp && bp_dev != dev) {
    delete bp;
    bp = nullptr;
  }
  if (!bp) {
    bp = new zdl_rows_buf();
    bp_dev = dev;
  }
  zdl_rows_buf& b = *bp;
  const uint64_t n = n_rows;
  ROWS_TRY(b.lo.ensure(n));
  ROWS_TRY(b.id.ensure(n));
  ROWS_TRY(b.pid.ensure(n));
  ROWS_TRY(b.key.ensure(n));
  ROWS_TRY(b.type.ensure(n));
  ROWS_TRY(b.svc.ensure(n));
  ROWS_TRY(b.lower.ensure(n_raw));
  if (rows->trace_hi) ROWS_TRY(b.hi.ensure(n));
  ROWS_TRY(hipMemcpyAsync(b.lo.p, rows->trace_lo, n * 8, hipMemcpyDefault, s));
  if (rows->trace_hi) ROWS_TRY(hipMemcpyAsync(b.hi.p, rows->trace_hi, n * 8, hipMemcpyDefault, s));
  ROWS_TRY(hipMemcpyAsync(b.id.p, rows->span_id, n * 8, hipMemcpyDefault, s));
  ROWS_TRY(hipMemcpyAsync(b.pid.p, rows->parent_id, n * 8, hipMemcpyDefault, s));
  ROWS_TRY(hipMemcpyAsync(b.key.p, rows->a_key, n, hipMemcpyDefault, s));
  ROWS_TRY(hipMemcpyAsync(b.type.p, rows->a_type, n * 4, hipMemcpyDefault, s));
  ROWS_TRY(hipMemcpyAsync(b.svc.p, rows->service, n * 4, hipMemcpyDefault, s));
  if (n_raw) ROWS_TRY(hipMemcpyAsync(b.lower.p, lower, n_raw * 4ull, hipMemcpyDefault, s));
  ROWS_TRY(b.heads.ensure(n));
  ROWS_TRY(b.pos.ensure(n));
  Rows r{b.lo.p, rows->trace_hi ? b.hi.p : nullptr, b.id.p, b.pid.p, b.key.p, b.type.p, b.svc.p, b.lower.p, n_raw};
  const unsigned grid = (unsigned)((n + 255) / 256);
  k_row_heads<<<grid, 256, 0, s>>>(r, n, b.heads.p);
  ROWS_TRY(hipGetLastError());
  size_t tb = 0;
  ROWS_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, b.heads.p, b.pos.p, (int)n, s));
  ROWS_TRY(b.tmp.ensure(tb));
  ROWS_TRY(hipcub::DeviceScan::ExclusiveSum(b.tmp.p, tb, b.heads.p, b.pos.p, (int)n, s));
  unsigned long long last[2];
  ROWS_TRY(hipMemcpyAsync(&last[0], b.pos.p + n - 1, 8, hipMemcpyDeviceToHost, s));
  ROWS_TRY(hipMemcpyAsync(&last[1], b.heads.p + n - 1, 8, hipMemcpyDeviceToHost, s));
  ROWS_TRY(hipStreamSynchronize(s));
  const unsigned long long tot = last[0] + last[1];
  const uint64_t n_spans = (uint32_t)tot, n_traces = (uint32_t)(tot >> 32);
  ROWS_TRY(b.c_lo.ensure(n_spans));
  ROWS_TRY(b.c_id.ensure(n_spans));
  ROWS_TRY(b.c_pid.ensure(n_spans));
  ROWS_TRY(b.c_lsvc.ensure(n_spans));
  ROWS_TRY(b.c_rsvc.ensure(n_spans));
  ROWS_TRY(b.c_ip4.ensure(n_spans));
  ROWS_TRY(b.c_ip6.ensure(n_spans));
  ROWS_TRY(b.c_pf.ensure(n_spans));
  ROWS_TRY(b.c_ts.ensure(n_spans));
  ROWS_TRY(b.c_off.ensure(n_traces + 1));
  ROWS_TRY(b.status.ensure(1));
  ROWS_TRY(hipMemsetAsync(b.status.p, 0, 4, s));
  Cols c{b.c_lo.p,  b.c_id.p,  b.c_pid.p, b.c_lsvc.p, b.c_rsvc.p, b.c_ip4.p,
         b.c_ip6.p, b.c_pf.p,  b.c_ts.p,  b.c_off.p,  b.status.p};
  k_row_project<<<grid, 256, 0, s>>>(r, n, b.pos.p, c);
  ROWS_TRY(hipGetLastError());
  uint32_t st = 0;
  ROWS_TRY(hipMemcpyAsync(&st, b.status.p, 4, hipMemcpyDeviceToHost, s));
  ROWS_TRY(hipStreamSynchronize(s));
  if (st & 1u) {
    g_rows_err = "reference throws IllegalArgumentException (span id 0 or trace id 0)";
    return ZDL_EREF_IAE;
  }
  if (st & 2u) {
    g_rows_err = "service id >= n_raw";
    return ZDL_EINVAL;
  }
  const zdl_span_cols cols{b.c_lo.p,  b.c_id.p, b.c_pid.p, b.c_lsvc.p, b.c_rsvc.p, b.c_ip4.p,
                           b.c_ip6.p, b.c_pf.p, b.c_ts.p,  nullptr};
  const int rc = zdl_put_spans_device(ctx, &cols, n_spans, b.c_off.p, n_traces);
  if (rc != ZDL_OK) {
    g_rows_err = zdl_last_error(ctx);
    return rc;
  }
  const int sr = zdl_sync(ctx);  // the row buffers are reused by the next call
  if (sr != ZDL_OK) g_rows_err = zdl_last_error(ctx);
  return sr;
}

}  // extern "C"
