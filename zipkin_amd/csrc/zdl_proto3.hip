// zdl_proto3.hip — proto3 ListOfSpans straight to zdl span columns on the device
// (the wire-format decoder in front of the dependency-link path).
//
// Replaces SpanBytesDecoder.PROTO3.decodeList(bytes) (codec/SpanBytesDecoder.java:144-152 ->
// internal/Proto3Codec.java readList) followed by the facade's Span -> column projection, for
// the fields the linker reads. Paths relative to /root/reference/zipkin/src/main/java/zipkin2/.
//
//   host  : top-level scan of the ListOfSpans (key, length prefix, ensureLength; a zero-length
//           span makes the whole result empty, Proto3Codec.readList -> emptyList) — O(1) work per
//           span, it only records where each span message lies;
//   device: k_proto3_spans, one lane per span message: SpanField.readValue
//           (Proto3ZipkinFields.java:314-369) with EndpointField / AnnotationField / TagField,
//           Buffer.readVarint32/64 (Buffer.java:300-365, incl. the 5th byte of a varint32 read
//           without advancing), skipValue and ensureLength (Proto3Fields.java), Span.Builder's id
//           rules (Span.java:402-484) and Endpoint.Builder.parseIp(byte[]) (Endpoint.java:179-198,
//           269-285). Strings become dictionary ids by an exact-key device hash table.
//
// Dictionary keys are the RAW field bytes (service names before toLowerCase; ipv4 as its 4
// normalised bytes, ipv6 as its 16 bytes). Keys the table does not hold are reported per span
// and slot; the caller assigns ids (lower-casing, first-seen order) with zdl_decoder_bind and
// re-runs the kernel on the resident buffer (zdl_decode_proto3_retry).
//
// Errors: the first failing span decides (lowest index, like the sequential reader):
// ZDL_EREF_IAE where the reference throws IllegalArgumentException; ZDL_EINVAL where a field
// read ends beyond its enclosing message (the reference then reads on leniently from a
// misaligned position; not supported here).

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/zdl.h"

namespace zp3 {

constexpr uint32_t kNoKey = 0xFFFFFFFFu;
constexpr uint64_t kNoErr = ~0ull;

// exact-key dictionary, open addressing; key bytes in an arena as [u32 len][bytes]
struct Slot {
  uint64_t h;
  uint32_t koff;  // kNoKey = empty
  int32_t id;
  uint32_t len, kind;
  uint64_t k0, k1;  // the key's first 16 bytes (little-endian, zero-padded): keys up to 16 bytes
                    // compare here, without the arena
};

struct Dict {
  const Slot* slot;
  const uint8_t* arena;
  uint32_t mask;  // capacity - 1
};

// Key hash (FNV-1a over the kind and the bytes): the host and both decoders use this function
template <class Get>
__host__ __device__ __forceinline__ uint64_t key_hash(int kind, Get get, uint32_t n) {
  uint64_t h = 1469598103934665603ull ^ (uint64_t)(kind + 1);
  h *= 1099511628211ull;
  for (uint32_t i = 0; i < n; ++i) {
    h ^= get(i);
    h *= 1099511628211ull;
  }
  return h ^ (h >> 29);
}

constexpr int kBlock = 256;
constexpr uint32_t kWin = 24 * 1024;  // LDS window per block: the block's span messages (C2: ~19 KB)

struct Out {
  uint64_t *trace_lo, *id, *pid;
  int32_t *lsvc, *rsvc, *ip4, *ip6;
  uint32_t* pf;
  int64_t* ts;
  uint8_t* miss;       // per span: bit s = slot s's key is not in the table
  uint64_t* miss_off;  // [4 n]: key offset in the batch (ip4: the 4 normalised bytes)
  uint32_t* miss_len;  // [4 n]
  unsigned long long* first_err;  // min over failing spans of (span << 1 | (iae ? 1 : 0))
  uint32_t* any_miss;
  uint64_t* trace_hi;  // the trace id's high 64 bits (0 for a 64-bit id)
  uint8_t* trace_wide;  // JSON: 1 when Span.normalizeTraceId gives 32 characters (null for proto3)
};

enum : int { SLOT_LSVC = 0, SLOT_LIP4 = 1, SLOT_LIP6 = 2, SLOT_RSVC = 3 };
enum : int { F_OK = 0, F_IAE = 1, F_OVERRUN = 2 };

// Buffer over the whole batch (bounds = the batch, as in Buffer.java); fail is sticky. Bytes
// inside the block's LDS window [w0, w0 + wn) are read from LDS, the rest from HBM.
typedef __attribute__((address_space(3))) const uint8_t lds_u8;  // ds_read, not flat loads

struct Rd {
  const uint8_t* b;
  uint64_t n, pos;
  int fail;
  lds_u8* w;
  uint64_t w0, wn;

  __device__ __forceinline__ uint8_t at(uint64_t p) const {
    const uint64_t q = p - w0;
    if (q < wn) return w[(uint32_t)q];
    return b[p];
  }
  __device__ __forceinline__ uint8_t byte() {
    if (pos >= n) {
      fail = fail ? fail : F_IAE;  // "Truncated reading position"
      return 0;
    }
    return at(pos++);
  }
  __device__ __forceinline__ int32_t varint32() {  // Buffer.readVarint32
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
      const uint8_t x = byte();
      if (fail) return 0;
      if (x < 0x80) return (int32_t)(r | (uint32_t)x << (7 * i));
      r |= (uint32_t)(x & 0x7F) << (7 * i);
    }
    if (pos >= n) {
      fail = F_IAE;
      return 0;
    }
    const uint8_t x = at(pos);  // not advanced (Buffer.java:328-333)
    if (x & 0xF0) {
      fail = F_IAE;
      return 0;
    }
    return (int32_t)(r | (uint32_t)x << 28);
  }
  __device__ __forceinline__ void varint64() {  // Buffer.readVarint64, value unused
    uint8_t x = byte();
    for (int i = 1; !fail && x >= 0x80 && i < 10; ++i) {
      x = byte();
      if (!fail && i == 9 && (x & 0xF0)) fail = F_IAE;
    }
  }
  __device__ __forceinline__ int64_t remaining() const { return (int64_t)(n - pos); }
  __device__ __forceinline__ int32_t length_prefix() {  // readLengthPrefix + ensureLength
    const int32_t len = varint32();
    if (!fail && (int64_t)len > remaining()) fail = F_IAE;
    return len;
  }
  __device__ __forceinline__ int64_t fixed64() {  // Fixed64Field.readValue
    if (remaining() < 8) {
      fail = F_IAE;
      return 0;
    }
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v |= (uint64_t)at(pos + i) << (8 * i);
    pos += 8;
    return (int64_t)v;
  }
  __device__ __forceinline__ void clamp_skip(int64_t k) {  // Buffer.skip
    pos = (pos + (uint64_t)k > n) ? n : pos + (uint64_t)k;
  }
  __device__ __forceinline__ void skip_value(int32_t key) {  // logAndSkip -> skipValue
    switch (key & 7) {
      case 0: {
        const int64_t rem = remaining();
        for (int64_t i = 0; i < rem; ++i)
          if (at(pos++) < 0x80) return;
        return;
      }
      case 1: clamp_skip(8); return;
      case 2: {
        const int32_t len = varint32();
        if (fail) return;
        if (len < 0) fail = F_OVERRUN;  // the reference would move backwards: unsupported
        else clamp_skip(len);
        return;
      }
      case 5: clamp_skip(4); return;
      default: fail = F_IAE; return;  // "Malformed: invalid wireType"
    }
  }
  // a nested loop over [pos, end) finished: reading past `end` is the lenient case
  __device__ __forceinline__ void close(int64_t end) {
    if (!fail && (int64_t)pos > end) fail = F_OVERRUN;
  }
  // a string / bytes field of length len (0 = null): positive lengths are skipped
  __device__ __forceinline__ bool take(int32_t len, uint64_t* off) {
    if (fail) return false;
    if (len < 0) {  // new byte[negative] / new String(.., negative)
      fail = F_IAE;
      return false;
    }
    *off = pos;
    pos += (uint64_t)len;
    return len > 0;
  }
};

struct Ep {  // Endpoint.Builder state for the columns
  uint64_t svc_off = 0;
  uint32_t svc_len = 0;  // 0 = null
  uint32_t ip4 = 0;      // bytes, big-endian order in a u32
  bool has4 = false, has6 = false;
  uint64_t ip6_off = 0;
  int32_t port = 0;
  __device__ __forceinline__ bool empty() const { return !svc_len && !has4 && !has6 && !port; }
};

__device__ __forceinline__ void parse_ip(Rd& r, uint64_t off, int32_t len, Ep& e) {  // Endpoint.Builder.parseIp(byte[])
  auto p = [&](int i) { return (uint32_t)r.at(off + i); };
  if (len == 4) {
    e.ip4 = p(0) << 24 | p(1) << 16 | p(2) << 8 | p(3);
    e.has4 = true;
  } else if (len == 16) {
    bool z = true;
    for (int i = 0; i < 12; ++i) z &= p(i) == 0;  // 80 zero bits and flag == 0 (flag == -1 never holds)
    const bool loop = z && p(12) == 0 && p(13) == 0 && p(14) == 0 && p(15) == 1;  // ::1
    if (z && !loop) {
      e.ip4 = p(12) << 24 | p(13) << 16 | p(14) << 8 | p(15);
      e.has4 = true;
    } else {
      e.ip6_off = off;
      e.has6 = true;
    }
  }
}

__device__ __forceinline__ void read_endpoint(Rd& r, int32_t len, Ep& e) {  // EndpointField.readValue
  e = Ep();
  const int64_t end = (int64_t)r.pos + len;  // before pos when len < 0: nothing read, then close()
  while (!r.fail && (int64_t)r.pos < end) {
    const int32_t key = r.varint32();
    if (r.fail) return;
    uint64_t off = 0;
    if (key == (1 << 3 | 2)) {
      const int32_t n = r.length_prefix();
      e.svc_len = r.take(n, &off) ? (uint32_t)n : 0;
      e.svc_off = off;
    } else if (key == (2 << 3 | 2) || key == (3 << 3 | 2)) {
      const int32_t n = r.length_prefix();
      if (r.take(n, &off)) parse_ip(r, off, n, e);
    } else if (key == (4 << 3 | 0)) {
      const int32_t p = r.varint32();
      if (!r.fail && p > 0xFFFF) r.fail = F_IAE;  // "invalid port"
      e.port = p < 0 ? 0 : p;
    } else {
      r.skip_value(key);
    }
  }
  r.close(end);
}

__device__ __forceinline__ bool bytes_are_error(const Rd& r, uint64_t o) {
  return r.at(o) == 'e' && r.at(o + 1) == 'r' && r.at(o + 2) == 'r' && r.at(o + 3) == 'o' && r.at(o + 4) == 'r';
}

// hex id of L bytes -> value; rules of Span.Builder.traceId / id / parentId
__device__ __forceinline__ uint64_t be_tail(const Rd& r, uint64_t off, int32_t n) {
  uint64_t v = 0;
  for (int32_t i = n > 8 ? n - 8 : 0; i < n; ++i) v = v << 8 | r.at(off + i);
  return v;
}

template <class Get>
__device__ __forceinline__ int32_t lookup(const Dict& d, int kind, Get p, uint32_t n) {
  if (d.mask == 0) return -2;
  const uint64_t h = key_hash(kind, p, n);
  for (uint32_t i = (uint32_t)h & d.mask, probes = 0; probes <= d.mask; i = (i + 1) & d.mask, ++probes) {
    const Slot s = d.slot[i];
    if (s.koff == kNoKey) return -2;
    if (s.h != h) continue;
    const uint8_t* k = d.arena + s.koff;
    const uint32_t kl = (uint32_t)k[0] | (uint32_t)k[1] << 8 | (uint32_t)k[2] << 16 | (uint32_t)k[3] << 24;
    if (kl != n || k[4] != (uint8_t)kind) continue;
    bool eq = true;
    if (n <= 24) {  // every byte at once: one memory round trip, not one per byte
#pragma unroll
      for (uint32_t j = 0; j < 24; ++j)
        if (j < n) eq &= k[5 + j] == p(j);
    } else {
      for (uint32_t j = 0; j < n && eq; ++j) eq = k[5 + j] == p(j);
    }
    if (eq) return s.id;
  }
  return -2;
}

// A key of n <= 16 bytes given as two little-endian words (zero past n): its hash
__device__ __forceinline__ uint64_t key_hash16(int kind, uint64_t w0, uint64_t w1, uint32_t n) {
  return key_hash(kind, [&](uint32_t j) { return (uint32_t)((j < 8 ? w0 >> (8 * j) : w1 >> (8 * (j - 8))) & 0xFFu); },
                  n);
}
// ... and its id from the slot at (h & mask) when that slot is the key's (nearly always): the
// first probe is issued by the caller for several keys at once; -3 = probe on (lookup())
__device__ __forceinline__ int32_t slot_match(const Slot& s, uint64_t h, int kind, uint64_t w0, uint64_t w1,
                                              uint32_t n) {
  if (s.koff == kNoKey) return -2;
  if (s.h == h && s.len == n && s.kind == (uint32_t)kind && s.k0 == w0 && s.k1 == w1) return s.id;
  return -3;
}

__global__ void __launch_bounds__(kBlock) k_proto3_spans(const uint8_t* __restrict__ buf, uint64_t len,
                                                           const uint64_t* __restrict__ start,
                                                           const uint32_t* __restrict__ slen, uint32_t n, Dict dict,
                                                           Out o) {
  // The block's span messages are contiguous in the batch: stage them in LDS with coalesced
  // 16-byte loads (from a 16-byte aligned base), so the byte-serial parsing below reads LDS.
  __shared__ __attribute__((aligned(16))) uint8_t win[kWin];
  const uint32_t first = blockIdx.x * kBlock;
  const uint32_t last = min(first + kBlock, n) - 1;
  const uint64_t w0 = start[first] & ~15ull;
  const uint64_t wn = min<uint64_t>(start[last] + slen[last] - w0, kWin);
  for (uint64_t q = (uint64_t)threadIdx.x * 16; q < wn; q += kBlock * 16) {
    if (w0 + q + 16 <= len) {
      *(uint4*)(win + q) = *(const uint4*)(buf + w0 + q);
    } else {
      for (uint64_t t = q; t < q + 16 && w0 + t < len; ++t) win[t] = buf[w0 + t];
    }
  }
  __syncthreads();
  const uint32_t i = first + threadIdx.x;
  if (i >= n) return;
  Rd r{buf, len, start[i], F_OK, (lds_u8*)win, w0, wn};
  const int64_t end = (int64_t)(r.pos + slen[i]);
  bool has_trace = false, has_id = false, shared = false, error = false;
  uint64_t lo = 0, hi = 0, id = 0, pid = 0;
  int64_t ts = 0;
  uint32_t kind = ZDL_KIND_NULL;
  Ep le, re;
  while (!r.fail && (int64_t)r.pos < end) {
    const int32_t key = r.varint32();
    if (r.fail) break;
    uint64_t off = 0;
    switch (key) {
      case 1 << 3 | 2: {  // trace_id
        const int32_t m = r.length_prefix();
        if (!r.take(m, &off) && !r.fail) r.fail = F_IAE;  // traceId == null
        if (r.fail) break;
        bool zero = true;
        for (int32_t j = 0; j < m; ++j) zero &= r.at(off + j) == 0;
        if (m > 16 || zero) r.fail = F_IAE;  // length > 32 hex / all zeros
        lo = be_tail(r, off, m);
        hi = m > 8 ? be_tail(r, off, m - 8) : 0;
        has_trace = true;
        break;
      }
      case 2 << 3 | 2: {  // parent_id
        const int32_t m = r.length_prefix();
        if (!r.take(m, &off)) {
          pid = 0;
          break;
        }
        if (m > 8) r.fail = F_IAE;
        pid = be_tail(r, off, m);  // all zeros -> null (0)
        break;
      }
      case 3 << 3 | 2: {  // id
        const int32_t m = r.length_prefix();
        if (!r.take(m, &off) && !r.fail) r.fail = F_IAE;  // id == null
        if (r.fail) break;
        if (m > 8) r.fail = F_IAE;
        id = be_tail(r, off, m);
        if (m == 8 && id == 0) r.fail = F_IAE;  // "id is all zeros" (16 zero hex digits only)
        has_id = true;
        break;
      }
      case 4 << 3 | 0: {  // kind: 0 and > 4 ignored, negative -> Kind.values()[-n] throws
        const int32_t k = r.varint32();
        if (r.fail || k == 0 || k > 4) break;
        if (k < 0) r.fail = F_IAE;
        else kind = (uint32_t)(k - 1);
        break;
      }
      case 5 << 3 | 2: r.take(r.length_prefix(), &off); break;  // name
      case 6 << 3 | 1: {
        const int64_t t = r.fixed64();
        ts = t < 0 ? 0 : t;
        break;
      }
      case 7 << 3 | 0: r.varint64(); break;  // duration
      case 8 << 3 | 2:
      case 9 << 3 | 2: {
        const int32_t m = r.length_prefix();
        if (r.fail) break;
        Ep e;  // m == 0: readLengthPrefixAndValue -> null endpoint
        if (m != 0) read_endpoint(r, m, e);
        if (key == (8 << 3 | 2)) le = e;  // no reference select: both stay in registers
        else re = e;
        break;
      }
      case 10 << 3 | 2: {  // annotation: validated, not kept
        const int32_t m = r.length_prefix();
        if (r.fail || m == 0) break;
        const int64_t ae = (int64_t)r.pos + m;
        while (!r.fail && (int64_t)r.pos < ae) {
          const int32_t k = r.varint32();
          if (r.fail) break;
          if (k == (1 << 3 | 1)) r.fixed64();
          else if (k == (2 << 3 | 2)) r.take(r.length_prefix(), &off);
          else r.skip_value(k);
        }
        r.close(ae);
        break;
      }
      case 11 << 3 | 2: {  // tag: only whether the key "error" is present matters
        const int32_t m = r.length_prefix();
        if (r.fail || m == 0) break;
        const int64_t te = (int64_t)r.pos + m;
        int32_t klen = 0;  // 0 = key null
        uint64_t koff = 0;
        while (!r.fail && (int64_t)r.pos < te) {
          const int32_t k = r.varint32();
          if (r.fail) break;
          if (k == (1 << 3 | 2)) {
            const int32_t kl = r.length_prefix();
            klen = r.take(kl, &koff) ? kl : 0;
          } else if (k == (2 << 3 | 2)) {
            r.take(r.length_prefix(), &off);
          } else {
            r.skip_value(k);
          }
        }
        r.close(te);
        if (!r.fail && klen == 5 && bytes_are_error(r, koff)) error = true;
        break;
      }
      case 12 << 3 | 0:
      case 13 << 3 | 0: {  // BooleanField.read: one byte, 0 or 1
        const uint8_t v = r.byte();
        if (r.fail) break;
        if (v > 1) r.fail = F_IAE;
        else if (v == 1 && key == (13 << 3 | 0)) shared = true;
        break;
      }
      default: r.skip_value(key);
    }
  }
  r.close(end);
  if (!r.fail && (!has_trace || !has_id)) r.fail = F_IAE;  // Span.Builder.build: "Missing :"
  if (r.fail) {
    atomicMin(o.first_err, (unsigned long long)i << 1 | (r.fail == F_IAE ? 1ull : 0ull));
    return;
  }
  if (pid == id) pid = 0;  // Span.Builder.build undoes the circular dependency
  const bool lnull = le.empty(), rnull = re.empty();
  int32_t ls = -1, l4 = -1, l6 = -1, rs = -1;
  uint8_t miss = 0;
  uint64_t moff[4] = {0, 0, 0, 0};
  uint32_t mlen[4] = {0, 0, 0, 0};
  if (!lnull && le.svc_len) {
    ls = lookup(dict, ZDL_DICT_SERVICE, [&](uint32_t j) { return r.at(le.svc_off + j); }, le.svc_len);
    moff[SLOT_LSVC] = le.svc_off, mlen[SLOT_LSVC] = le.svc_len;
  }
  if (!lnull && le.has4) {
    const uint8_t k[4] = {(uint8_t)(le.ip4 >> 24), (uint8_t)(le.ip4 >> 16), (uint8_t)(le.ip4 >> 8), (uint8_t)le.ip4};
    l4 = lookup(dict, ZDL_DICT_IPV4, [&](uint32_t j) { return k[j]; }, 4);
    moff[SLOT_LIP4] = le.ip4, mlen[SLOT_LIP4] = 4;
  }
  if (!lnull && le.has6) {
    l6 = lookup(dict, ZDL_DICT_IPV6, [&](uint32_t j) { return r.at(le.ip6_off + j); }, 16);
    moff[SLOT_LIP6] = le.ip6_off, mlen[SLOT_LIP6] = 16;
  }
  if (!rnull && re.svc_len) {
    rs = lookup(dict, ZDL_DICT_SERVICE, [&](uint32_t j) { return r.at(re.svc_off + j); }, re.svc_len);
    moff[SLOT_RSVC] = re.svc_off, mlen[SLOT_RSVC] = re.svc_len;
  }
  miss = (ls == -2) | (l4 == -2) << 1 | (l6 == -2) << 2 | (rs == -2) << 3;
  o.miss[i] = miss;
  if (miss) {
    for (int s = 0; s < 4; ++s)
      if (miss >> s & 1) o.miss_off[4ull * i + s] = moff[s], o.miss_len[4ull * i + s] = mlen[s];
    atomicOr(o.any_miss, 1u);
    return;
  }
  uint32_t pf = (uint32_t)(lnull ? 0 : le.port) & ZDL_PF_PORT_MASK;
  pf |= kind << ZDL_PF_KIND_SHIFT;
  pf |= (shared ? 2u : 0u) << ZDL_PF_SHARED_SHIFT;  // proto3 only ever sets shared(true)
  if (error) pf |= ZDL_PF_ERROR;
  if (!rnull) {
    if (re.has4) pf |= ZDL_PF_RIP4;
    if (re.has6) pf |= ZDL_PF_RIP6;
    if (re.port) pf |= ZDL_PF_RPORT;
  }
  o.trace_lo[i] = lo;
  o.trace_hi[i] = hi;
  o.id[i] = id;
  o.pid[i] = pid;
  o.lsvc[i] = ls;
  o.rsvc[i] = rs;
  o.ip4[i] = l4;
  o.ip6[i] = l6;
  o.pf[i] = pf;
  o.ts[i] = ts;
}

#include "zdl_json.inc"

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

template <class T>
struct HBuf {  // pinned host
  T* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t want) {
    if (want <= n) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipHostMalloc((void**)&p, std::max<size_t>(want, 1) * sizeof(T), hipHostMallocDefault);
    if (e == hipSuccess) n = std::max<size_t>(want, 1);
    return e;
  }
  ~HBuf() {
    if (p) (void)hipHostFree(p);
  }
};

// host-side Buffer.readVarint32 for the top-level scan; false = IllegalArgumentException
inline bool host_varint32(const uint8_t* b, uint64_t n, uint64_t& pos, int32_t& v) {
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) {
    if (pos >= n) return false;
    const uint8_t x = b[pos++];
    if (x < 0x80) {
      v = (int32_t)(r | (uint32_t)x << (7 * i));
      return true;
    }
    r |= (uint32_t)(x & 0x7F) << (7 * i);
  }
  if (pos >= n || (b[pos] & 0xF0)) return false;
  v = (int32_t)(r | (uint32_t)b[pos] << 28);
  return true;
}

}  // namespace zp3

using namespace zp3;

struct zdl_decoder {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // dictionary: host mirror (kind byte + raw key -> id) and the device table built from it
  std::unordered_map<std::string, int32_t> keys;
  std::vector<uint8_t> arena_h;
  bool dirty = false;
  DBuf<Slot> slots;
  DBuf<uint8_t> arena;
  uint32_t cap = 0;
  // the resident batch
  DBuf<uint8_t> buf;
  DBuf<uint64_t> start;
  DBuf<uint32_t> slen;
  std::vector<uint64_t> start_h;
  std::vector<uint32_t> slen_h;
  uint64_t len = 0, n = 0;
  int scan_rc = ZDL_OK;  // result of the top-level scan beyond span n (IAE or empty)
  // outputs
  DBuf<uint64_t> lo, hi, id, pid;
  DBuf<int32_t> lsvc, rsvc, ip4, ip6;
  DBuf<uint32_t> pf;
  DBuf<int64_t> ts;
  DBuf<uint8_t> miss;
  DBuf<uint8_t> wide;  // JSON: trace id widths (zdl_decoded.dev_trace_wide)
  DBuf<uint64_t> miss_off;
  DBuf<uint32_t> miss_len;
  DBuf<unsigned long long> status;  // [0] first_err, [1] any_miss (u32 in the low half)
  HBuf<unsigned long long> status_h;
  std::vector<std::string> missing;  // kind byte + key bytes, first-seen order
  hipEvent_t ev[2] = {nullptr, nullptr};  // around the last k_proto3_spans / k_js_spans
  float kernel_ms = 0.f;
  int fmt = 0;  // the resident batch: 0 proto3, 1 JSON v2
  // JSON v2 structure (zdl_json.inc)
  DBuf<int4> js_fn, js_gfn, js_lpre;  // block functions / prefixes, group functions, lane prefixes
  DBuf<uint16_t> js_slots;           // per block: its objects' block-relative positions
  DBuf<unsigned long long> js_gst, js_misc;  // misc: [0] E (the array's closing bracket), [1] spans before E, [2] lane overflow
  DBuf<uint32_t> js_cnt;
  DBuf<uint64_t> js_off, js_starts;
  DBuf<uint8_t> js_tmp;  // hipCUB scan scratch
  DBuf<uint32_t> js_list;  // spans k_js_fast hands to the exact reader (their count: status[2])
  uint64_t js_n_exact = 0;  // that count for the last JSON decode
  bool js_exact = false;             // ZDL_JS_EXACT=1: every span through the exact reader (A/B, tests)
  int js_global = 2;  // the fast path reads its objects from HBM / the caches at 4 waves per SIMD
                      // (ZDL_JS_GLOBAL=2, default; 3 / 4: 5 / 6 waves), at the registers' 3 (1), or from the block's LDS
                      // window (0: 2 waves per SIMD); A/B in profiles/r03t_js_fast_variants.log
  HBuf<unsigned long long> js_h;
  uint64_t js_open = 0;  // the opening '['
  float struct_ms = 0.f;  // HIP-event time of the structural passes of the last JSON decode
  hipEvent_t ev_s[2] = {nullptr, nullptr};
};

namespace {

int dfail(zdl_decoder* d, int code, const std::string& msg) {
  if (d) d->err = msg;
  return code;
}

#define DEC_TRY(d, expr)                                                                                  \
  do {                                                                                                    \
    hipError_t _e = (expr);                                                                               \
    if (_e != hipSuccess)                                                                                 \
      return dfail((d), _e == hipErrorOutOfMemory ? ZDL_ENOMEM : ZDL_EDEVICE,                             \
                   std::string(#expr) + ": " + hipGetErrorString(_e));                                    \
  } while (0)

// rebuild the device table from the host mirror (only after binds)
int upload_dict(zdl_decoder* d) {
  if (!d->dirty) return ZDL_OK;
  uint32_t cap = 16;
  while (cap < 2 * d->keys.size() + 2) cap <<= 1;
  std::vector<Slot> sl(cap, Slot{0, kNoKey, -1, 0, 0, 0, 0});
  for (const auto& kv : d->keys) {
    const std::string& k = kv.first;  // k[0] = kind, then the key bytes
    const uint32_t koff = (uint32_t)d->arena_h.size();
    const uint32_t kl = (uint32_t)(k.size() - 1);
    for (int b = 0; b < 4; ++b) d->arena_h.push_back((uint8_t)(kl >> (8 * b)));
    d->arena_h.insert(d->arena_h.end(), k.begin(), k.end());
    const uint8_t* kb = (const uint8_t*)k.data() + 1;
    const uint64_t h = key_hash((uint8_t)k[0], [kb](uint32_t j) { return kb[j]; }, kl);
    uint32_t i = (uint32_t)h & (cap - 1);
    while (sl[i].koff != kNoKey) i = (i + 1) & (cap - 1);
    uint64_t kw[2] = {0, 0};
    for (uint32_t j = 0; j < kl && j < 16; ++j) kw[j >> 3] |= (uint64_t)kb[j] << (8 * (j & 7));
    sl[i] = Slot{h, koff, kv.second, kl, (uint32_t)(uint8_t)k[0], kw[0], kw[1]};
  }
  DEC_TRY(d, d->slots.ensure(cap));
  DEC_TRY(d, d->arena.ensure(d->arena_h.size()));
  DEC_TRY(d, hipMemcpyAsync(d->slots.p, sl.data(), cap * sizeof(Slot), hipMemcpyHostToDevice, d->stream));
  DEC_TRY(d, hipMemcpyAsync(d->arena.p, d->arena_h.data(), d->arena_h.size(), hipMemcpyHostToDevice, d->stream));
  DEC_TRY(d, hipStreamSynchronize(d->stream));  // sl and arena_h are reused
  d->arena_h.clear();
  d->cap = cap;
  d->dirty = false;
  return ZDL_OK;
}

int run_kernel(zdl_decoder* d, zdl_decoded* out) {
  std::memset(out, 0, sizeof(*out));
  int rc = upload_dict(d);
  if (rc != ZDL_OK) return rc;
  const hipStream_t s = d->stream;
  const uint64_t n = d->n;
  if (n) {
    DEC_TRY(d, hipMemsetAsync(d->status.p, 0xFF, 8, s));
    DEC_TRY(d, hipMemsetAsync(d->status.p + 1, 0, 16, s));
    Dict dict{d->slots.p, d->arena.p, d->cap ? d->cap - 1 : 0};
    Out o{d->lo.p,   d->id.p, d->pid.p, d->lsvc.p,     d->rsvc.p,     d->ip4.p,    d->ip6.p,
          d->pf.p,   d->ts.p, d->miss.p, d->miss_off.p, d->miss_len.p, d->status.p, (uint32_t*)(d->status.p + 1),
          d->hi.p, d->fmt == 1 ? d->wide.p : nullptr};
    DEC_TRY(d, hipEventRecord(d->ev[0], s));
    const unsigned nb = (unsigned)((n + zjs::kSpanWG - 1) / zjs::kSpanWG);
    if (d->fmt == 1 && d->js_exact) {
      zjs::k_js_spans<<<nb, zjs::kSpanWG, 0, s>>>(d->buf.p, d->len, d->js_starts.p, (uint32_t)n, d->js_open,
                                                  d->js_misc.p, dict, o);
    } else if (d->fmt == 1) {  // the common shape fast, the rest exact
      DEC_TRY(d, d->js_list.ensure(n));
      if (d->js_global == 2)
        zjs::k_js_fast_g<4><<<nb, zjs::kSpanWG, 0, s>>>(d->buf.p, d->len, d->js_starts.p, (uint32_t)n, d->js_open,
                                                        d->js_misc.p, dict, o, d->js_list.p, (uint32_t*)(d->status.p + 2));
      else if (d->js_global == 3)
        zjs::k_js_fast_g<5><<<nb, zjs::kSpanWG, 0, s>>>(d->buf.p, d->len, d->js_starts.p, (uint32_t)n, d->js_open,
                                                        d->js_misc.p, dict, o, d->js_list.p, (uint32_t*)(d->status.p + 2));
      else if (d->js_global == 4)
        zjs::k_js_fast_g<6><<<nb, zjs::kSpanWG, 0, s>>>(d->buf.p, d->len, d->js_starts.p, (uint32_t)n, d->js_open,
                                                        d->js_misc.p, dict, o, d->js_list.p, (uint32_t*)(d->status.p + 2));
      else if (d->js_global)
        zjs::k_js_fast_g<1><<<nb, zjs::kSpanWG, 0, s>>>(d->buf.p, d->len, d->js_starts.p, (uint32_t)n, d->js_open,
                                                     d->js_misc.p, dict, o, d->js_list.p, (uint32_t*)(d->status.p + 2));
      else
        zjs::k_js_fast<<<nb, zjs::kSpanWG, 0, s>>>(d->buf.p, d->len, d->js_starts.p, (uint32_t)n, d->js_open,
                                                   d->js_misc.p, dict, o, d->js_list.p, (uint32_t*)(d->status.p + 2));
      DEC_TRY(d, hipGetLastError());
      zjs::k_js_spans_list<<<nb < 1024u ? nb : 1024u, zjs::kSpanWG, 0, s>>>(
          d->buf.p, d->len, d->js_starts.p, (uint32_t)n, d->js_open, d->js_misc.p, dict, o, d->js_list.p,
          (const uint32_t*)(d->status.p + 2));
    } else
      k_proto3_spans<<<(unsigned)((n + kBlock - 1) / kBlock), kBlock, 0, s>>>(d->buf.p, d->len, d->start.p, d->slen.p,
                                                                              (uint32_t)n, dict, o);
    DEC_TRY(d, hipGetLastError());
    DEC_TRY(d, hipEventRecord(d->ev[1], s));
    DEC_TRY(d, hipMemcpyAsync(d->status_h.p, d->status.p, 24, hipMemcpyDeviceToHost, s));
    DEC_TRY(d, hipStreamSynchronize(s));
    DEC_TRY(d, hipEventElapsedTime(&d->kernel_ms, d->ev[0], d->ev[1]));
    if (d->fmt == 1) d->js_n_exact = d->js_exact ? n : (uint32_t)d->status_h.p[2];
    const unsigned long long fe = d->status_h.p[0];
    if (fe != kNoErr && d->fmt == 1)  // (span << 2 | after-the-span << 1 | iae): the lowest decides
      return (fe & 1) ? dfail(d, ZDL_EREF_IAE, "reference throws IllegalArgumentException reading List<Span> from json (span " +
                                                   std::to_string(fe >> 2) + ((fe & 2) ? ", after it)" : ")"))
                      : dfail(d, ZDL_EINVAL, "json v2: span " + std::to_string(fe >> 2) +
                                                 " nests objects or arrays deeper than 64 (not supported)");
    if (fe != kNoErr)  // the first failing span decides, before the scan's own verdict
      return (fe & 1) ? dfail(d, ZDL_EREF_IAE, "reference throws IllegalArgumentException reading List<Span> from proto3 (span " +
                                                   std::to_string(fe >> 1) + ")")
                      : dfail(d, ZDL_EINVAL, "proto3: a field of span " + std::to_string(fe >> 1) +
                                                 " ends beyond its enclosing message (the reference reads on leniently; not supported)");
  }
  if (d->scan_rc == ZDL_EREF_IAE) return dfail(d, ZDL_EREF_IAE, "reference throws IllegalArgumentException reading List<Span> from proto3 (truncated list)");
  if (d->scan_rc == ZDL_EINVAL) return dfail(d, ZDL_EINVAL, "proto3: negative span length (the reference reads on leniently; not supported)");
  if (d->scan_rc == 1) return ZDL_OK;  // a zero-length span: readList -> false -> empty list
  if (n && (uint32_t)d->status_h.p[1]) {  // keys to bind, first-seen order (span, slot)
    std::vector<uint8_t> m(n);
    std::vector<uint64_t> mo(4 * n);
    std::vector<uint32_t> ml(4 * n);
    DEC_TRY(d, hipMemcpyAsync(m.data(), d->miss.p, n, hipMemcpyDeviceToHost, s));
    DEC_TRY(d, hipMemcpyAsync(mo.data(), d->miss_off.p, 4 * n * 8, hipMemcpyDeviceToHost, s));
    DEC_TRY(d, hipMemcpyAsync(ml.data(), d->miss_len.p, 4 * n * 4, hipMemcpyDeviceToHost, s));
    // the raw key bytes: the batch back from HBM (only on a pass with misses, i.e. new keys)
    std::vector<uint8_t> raw(d->len);
    DEC_TRY(d, hipMemcpyAsync(raw.data(), d->buf.p, d->len, hipMemcpyDeviceToHost, s));
    DEC_TRY(d, hipStreamSynchronize(s));
    d->missing.clear();
    std::unordered_map<std::string, bool> seen;
    static const int kind_of[2][4] = {{ZDL_DICT_SERVICE, ZDL_DICT_IPV4, ZDL_DICT_IPV6, ZDL_DICT_SERVICE},
                                      {ZDL_DICT_JSON_SERVICE, ZDL_DICT_JSON_IPV4, ZDL_DICT_JSON_IPV6TEXT,
                                       ZDL_DICT_JSON_SERVICE}};
    for (uint64_t i = 0; i < n; ++i) {
      for (int sl = 0; m[i] && sl < 4; ++sl) {
        if (!(m[i] >> sl & 1)) continue;
        std::string k(1, (char)kind_of[d->fmt][sl]);
        const uint64_t off = mo[4 * i + sl];
        if (sl == SLOT_LIP4 && d->fmt == 0) {
          for (int b = 3; b >= 0; --b) k.push_back((char)(uint8_t)(off >> (8 * b)));
        } else {
          k.append((const char*)raw.data() + off, ml[4 * i + sl]);
        }
        if (seen.emplace(k, true).second) d->missing.push_back(k);
      }
    }
    out->n_missing = d->missing.size();
    return ZDL_OK;
  }
  out->n_spans = n;
  // device columns only: nothing crosses PCIe (zdl_decoder_download copies what a caller needs)
  out->dev = zdl_span_cols{d->lo.p, d->id.p, d->pid.p, d->lsvc.p, d->rsvc.p, d->ip4.p, d->ip6.p, d->pf.p, d->ts.p, nullptr};
  out->trace_lo = nullptr;
  out->dev_trace_hi = d->hi.p;
  out->dev_trace_wide = d->fmt == 1 ? d->wide.p : nullptr;  // proto3: 128-bit iff the high half is non-zero
  out->timestamp = nullptr;
  return ZDL_OK;
}

}  // namespace

extern "C" {

zdl_decoder* zdl_decoder_create(int device) {
  zdl_decoder* d = new (std::nothrow) zdl_decoder();
  if (!d) return nullptr;
  d->device = device;
  const char* ex = std::getenv("ZDL_JS_EXACT");
  d->js_exact = ex && ex[0] == '1';
  const char* jg = std::getenv("ZDL_JS_GLOBAL");
  if (jg && jg[0] >= '0' && jg[0] <= '4') d->js_global = jg[0] - '0';
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess ||
      d->status.ensure(3) != hipSuccess || d->status_h.ensure(3) != hipSuccess ||
      hipEventCreate(&d->ev[0]) != hipSuccess || hipEventCreate(&d->ev[1]) != hipSuccess ||
      hipEventCreate(&d->ev_s[0]) != hipSuccess || hipEventCreate(&d->ev_s[1]) != hipSuccess) {
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
    return nullptr;
  }
  return d;
}

void zdl_decoder_destroy(zdl_decoder* d) {
  if (!d) return;
  (void)hipSetDevice(d->device);
  if (d->stream) (void)hipStreamSynchronize(d->stream);
  hipStream_t s = d->stream;
  for (hipEvent_t e : d->ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : d->ev_s)
    if (e) (void)hipEventDestroy(e);
  delete d;  // buffers free themselves
  if (s) (void)hipStreamDestroy(s);
}

const char* zdl_decoder_last_error(const zdl_decoder* d) { return d ? d->err.c_str() : "null decoder"; }

int zdl_decoder_bind(zdl_decoder* d, int kind, const uint8_t* key, uint32_t len, int32_t id) {
  if (!d || (len && !key) || id < 0 || kind < ZDL_DICT_SERVICE || kind > ZDL_DICT_JSON_IPV4)
    return dfail(d, ZDL_EINVAL, "zdl_decoder_bind: bad argument");
  if ((kind == ZDL_DICT_IPV4 && len != 4) || (kind == ZDL_DICT_IPV6 && len != 16) || len == 0)
    return dfail(d, ZDL_EINVAL, "zdl_decoder_bind: key length");
  std::string k(1, (char)kind);
  k.append((const char*)key, len);
  d->keys[k] = id;
  d->dirty = true;
  return ZDL_OK;
}

uint64_t zdl_decoder_dict_size(const zdl_decoder* d) { return d ? d->keys.size() : 0; }

float zdl_decoder_kernel_ms(const zdl_decoder* d) { return d ? d->kernel_ms : 0.f; }

float zdl_decoder_struct_ms(const zdl_decoder* d) { return d ? d->struct_ms : 0.f; }
uint64_t zdl_decoder_exact_spans(const zdl_decoder* d) { return d ? d->js_n_exact : 0; }

int zdl_decoder_missing(const zdl_decoder* d, uint64_t i, int* kind, const uint8_t** key, uint32_t* len) {
  if (!d || i >= d->missing.size() || !kind || !key || !len) return ZDL_EINVAL;
  const std::string& k = d->missing[i];
  *kind = (uint8_t)k[0];
  *key = (const uint8_t*)k.data() + 1;
  *len = (uint32_t)(k.size() - 1);
  return ZDL_OK;
}

int zdl_decode_proto3(zdl_decoder* d, const uint8_t* data, uint64_t len, zdl_decoded* out) {
  if (!d || !out || (len && !data)) return dfail(d, ZDL_EINVAL, "zdl_decode_proto3: null argument");
  if (len >= (1ull << 40)) return dfail(d, ZDL_EINVAL, "zdl_decode_proto3: batch limited to 2^40 bytes");
  (void)hipGetLastError();
  DEC_TRY(d, hipSetDevice(d->device));
  d->missing.clear();
  d->fmt = 0;
  const hipStream_t s = d->stream;
  // the batch goes up straight from the caller's bytes while a host thread runs the top-level
  // scan (Proto3Codec.readList / SpanField.read: key tossed / readLengthPrefix) over them
  d->start_h.clear();
  d->slen_h.clear();
  d->scan_rc = len == 0 ? 1 : ZDL_OK;  // empty input -> false -> emptyList
  std::thread scan([d, data, len] {
    uint64_t pos = 0;
    while (d->scan_rc == ZDL_OK && pos < len) {
      int32_t key, n;
      if (!host_varint32(data, len, pos, key) || !host_varint32(data, len, pos, n) ||
          (int64_t)n > (int64_t)(len - pos)) {
        d->scan_rc = ZDL_EREF_IAE;
        break;
      }
      if (n == 0) {
        d->scan_rc = 1;
        break;
      }
      if (n < 0) {  // readValue(negative) ends before it starts: the lenient case (unsupported)
        d->scan_rc = ZDL_EINVAL;
        break;
      }
      d->start_h.push_back(pos);
      d->slen_h.push_back((uint32_t)n);
      pos += (uint64_t)n;
    }
  });
  hipError_t up = d->buf.ensure(len);
  if (up == hipSuccess && len) up = hipMemcpyAsync(d->buf.p, data, len, hipMemcpyHostToDevice, s);
  if (up == hipSuccess) up = hipStreamSynchronize(s);  // `data` is borrowed for this call only
  scan.join();
  DEC_TRY(d, up);
  if (d->start_h.size() >= (1ull << 31)) return dfail(d, ZDL_EINVAL, "zdl_decode_proto3: at most 2^31 spans per batch");
  const uint64_t n = d->start_h.size();
  d->n = n;
  d->len = len;
  if (n) {
    DEC_TRY(d, d->start.ensure(n));
    DEC_TRY(d, d->slen.ensure(n));
    DEC_TRY(d, hipMemcpyAsync(d->start.p, d->start_h.data(), n * 8, hipMemcpyHostToDevice, s));
    DEC_TRY(d, hipMemcpyAsync(d->slen.p, d->slen_h.data(), n * 4, hipMemcpyHostToDevice, s));
    DEC_TRY(d, d->lo.ensure(n));
    DEC_TRY(d, d->hi.ensure(n));
    DEC_TRY(d, d->id.ensure(n));
    DEC_TRY(d, d->pid.ensure(n));
    DEC_TRY(d, d->lsvc.ensure(n));
    DEC_TRY(d, d->rsvc.ensure(n));
    DEC_TRY(d, d->ip4.ensure(n));
    DEC_TRY(d, d->ip6.ensure(n));
    DEC_TRY(d, d->pf.ensure(n));
    DEC_TRY(d, d->ts.ensure(n));
    DEC_TRY(d, d->miss.ensure(n));
    DEC_TRY(d, d->miss_off.ensure(4 * n));
    DEC_TRY(d, d->miss_len.ensure(4 * n));
  }
  return run_kernel(d, out);
}

int zdl_decode_retry(zdl_decoder* d, zdl_decoded* out) {
  if (!d || !out) return dfail(d, ZDL_EINVAL, "zdl_decode_retry: null argument");
  (void)hipGetLastError();
  DEC_TRY(d, hipSetDevice(d->device));
  d->missing.clear();
  return run_kernel(d, out);
}

int zdl_decode_json_v2(zdl_decoder* d, const uint8_t* data, uint64_t len, zdl_decoded* out) {
  using namespace zjs;
  if (!d || !out || (len && !data)) return dfail(d, ZDL_EINVAL, "zdl_decode_json_v2: null argument");
  if (len > (uint64_t)kBlk * kGroup * 1024) return dfail(d, ZDL_EINVAL, "zdl_decode_json_v2: batch limited to 4 GiB");
  (void)hipGetLastError();
  DEC_TRY(d, hipSetDevice(d->device));
  std::memset(out, 0, sizeof(*out));
  d->missing.clear();
  d->fmt = 1;
  d->n = 0;
  d->len = len;
  d->scan_rc = ZDL_OK;
  d->struct_ms = 0.f;
  if (len == 0) return ZDL_OK;  // JsonCodec.readList: empty input -> false -> emptyList
  // beginArray: the first token must be '[' (whitespace before it; comments are lenient-only)
  uint64_t p0 = 0;
  while (p0 < len && (data[p0] == ' ' || data[p0] == '\n' || data[p0] == '\t' || data[p0] == '\r')) ++p0;
  if (p0 == len || data[p0] != '[')
    return dfail(d, ZDL_EREF_IAE, "reference throws IllegalArgumentException reading List<Span> from json (no array)");
  d->js_open = p0;
  const hipStream_t s = d->stream;
  const uint32_t nblk = (uint32_t)((len + kBlk - 1) / kBlk);
  const uint32_t ngroup = (nblk + kGroup - 1) / kGroup;
  DEC_TRY(d, d->buf.ensure(len + 64));  // k_js_spans reads whole aligned 16-byte chunks
  DEC_TRY(d, hipMemcpyAsync(d->buf.p, data, len, hipMemcpyHostToDevice, s));
  DEC_TRY(d, d->js_fn.ensure(nblk));
  DEC_TRY(d, d->js_lpre.ensure((size_t)nblk * 64));
  DEC_TRY(d, d->js_gfn.ensure(ngroup));
  DEC_TRY(d, d->js_gst.ensure(ngroup));
  DEC_TRY(d, d->js_cnt.ensure(nblk));
  DEC_TRY(d, d->js_off.ensure(nblk));
  DEC_TRY(d, d->js_slots.ensure((size_t)nblk * kBlockCap));
  DEC_TRY(d, d->js_misc.ensure(3));
  DEC_TRY(d, d->js_h.ensure(3));
  size_t tmp = 0;
  DEC_TRY(d, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, d->js_cnt.p, d->js_off.p, (int)nblk, s));
  DEC_TRY(d, d->js_tmp.ensure(tmp));
  DEC_TRY(d, hipEventRecord(d->ev_s[0], s));
  DEC_TRY(d, hipMemsetAsync(d->js_misc.p, 0xFF, 8, s));     // E
  DEC_TRY(d, hipMemsetAsync(d->js_misc.p + 1, 0, 16, s));   // spans before E, lane overflow
  const unsigned g4 = (unsigned)((nblk + 3) / 4);
  k_js_fn<<<g4, 256, 0, s>>>(d->buf.p, len, nblk, d->js_fn.p, d->js_lpre.p);
  k_js_group<<<ngroup, 1024, 0, s>>>(d->js_fn.p, nblk, d->js_gfn.p);
  k_js_top<<<1, 1024, 0, s>>>(d->js_gfn.p, ngroup, d->js_gst.p);
  uint32_t* over = (uint32_t*)(d->js_misc.p + 2);
  k_js_starts<<<g4, 256, 0, s>>>(d->buf.p, len, nblk, d->js_fn.p, d->js_lpre.p, d->js_gst.p, d->js_cnt.p,
                                  d->js_slots.p, over, d->js_misc.p);
  DEC_TRY(d, hipGetLastError());
  DEC_TRY(d, hipcub::DeviceScan::ExclusiveSum(d->js_tmp.p, tmp, d->js_cnt.p, d->js_off.p, (int)nblk, s));
  uint64_t last_off = 0;
  uint32_t last_cnt = 0, over_h = 0;
  DEC_TRY(d, hipMemcpyAsync(&last_off, d->js_off.p + nblk - 1, 8, hipMemcpyDeviceToHost, s));
  DEC_TRY(d, hipMemcpyAsync(&last_cnt, d->js_cnt.p + nblk - 1, 4, hipMemcpyDeviceToHost, s));
  DEC_TRY(d, hipMemcpyAsync(&over_h, over, 4, hipMemcpyDeviceToHost, s));
  DEC_TRY(d, hipStreamSynchronize(s));
  if (over_h) {  // some lane held more than kLaneCap objects: the exact two-pass path
    k_js_starts_exact<0><<<g4, 256, 0, s>>>(d->buf.p, len, nblk, d->js_fn.p, d->js_lpre.p, d->js_gst.p, d->js_cnt.p,
                                             nullptr, nullptr);
    DEC_TRY(d, hipGetLastError());
    DEC_TRY(d, hipcub::DeviceScan::ExclusiveSum(d->js_tmp.p, tmp, d->js_cnt.p, d->js_off.p, (int)nblk, s));
    DEC_TRY(d, hipMemcpyAsync(&last_off, d->js_off.p + nblk - 1, 8, hipMemcpyDeviceToHost, s));
    DEC_TRY(d, hipMemcpyAsync(&last_cnt, d->js_cnt.p + nblk - 1, 4, hipMemcpyDeviceToHost, s));
    DEC_TRY(d, hipStreamSynchronize(s));
  }
  const uint64_t total = last_off + last_cnt;
  if (total) {
    DEC_TRY(d, d->js_starts.ensure(total));
    if (over_h)
      k_js_starts_exact<1><<<g4, 256, 0, s>>>(d->buf.p, len, nblk, d->js_fn.p, d->js_lpre.p, d->js_gst.p, nullptr,
                                               d->js_off.p, d->js_starts.p);
    else
      k_js_gather<<<(nblk + 15) / 16, 256, 0, s>>>(d->js_slots.p, d->js_cnt.p, d->js_off.p, nblk, d->js_starts.p);
    k_js_before<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(d->js_starts.p, total, d->js_misc.p, d->js_misc.p + 1);
    DEC_TRY(d, hipGetLastError());
  }
  DEC_TRY(d, hipEventRecord(d->ev_s[1], s));
  DEC_TRY(d, hipMemcpyAsync(d->js_h.p, d->js_misc.p, 16, hipMemcpyDeviceToHost, s));
  DEC_TRY(d, hipStreamSynchronize(s));
  DEC_TRY(d, hipEventElapsedTime(&d->struct_ms, d->ev_s[0], d->ev_s[1]));
  const uint64_t E = d->js_h.p[0], n = d->js_h.p[1];
  if (n == 0) {  // "[ ]" (hasNext false) is the empty list; anything else in it is not a span object
    if (E == ~0ull)
      return dfail(d, ZDL_EREF_IAE, "reference throws IllegalArgumentException reading List<Span> from json (End of input)");
    for (uint64_t p = p0 + 1; p < E; ++p)
      if (!(data[p] == ' ' || data[p] == '\n' || data[p] == '\t' || data[p] == '\r'))
        return dfail(d, ZDL_EREF_IAE, "reference throws IllegalArgumentException reading List<Span> from json (element 0)");
    return ZDL_OK;
  }
  if (n >= (1ull << 31)) return dfail(d, ZDL_EINVAL, "zdl_decode_json_v2: at most 2^31 spans per batch");
  d->n = n;
  DEC_TRY(d, d->lo.ensure(n));
  DEC_TRY(d, d->hi.ensure(n));
  DEC_TRY(d, d->wide.ensure(n));
  DEC_TRY(d, d->id.ensure(n));
  DEC_TRY(d, d->pid.ensure(n));
  DEC_TRY(d, d->lsvc.ensure(n));
  DEC_TRY(d, d->rsvc.ensure(n));
  DEC_TRY(d, d->ip4.ensure(n));
  DEC_TRY(d, d->ip6.ensure(n));
  DEC_TRY(d, d->pf.ensure(n));
  DEC_TRY(d, d->ts.ensure(n));
  DEC_TRY(d, d->miss.ensure(n));
  DEC_TRY(d, d->miss_off.ensure(4 * n));
  DEC_TRY(d, d->miss_len.ensure(4 * n));
  return run_kernel(d, out);
}

int zdl_decode_proto3_retry(zdl_decoder* d, zdl_decoded* out) {
  if (!d || !out) return dfail(d, ZDL_EINVAL, "zdl_decode_proto3_retry: null argument");
  (void)hipGetLastError();
  DEC_TRY(d, hipSetDevice(d->device));
  d->missing.clear();
  return run_kernel(d, out);
}

int zdl_decoder_download(zdl_decoder* d, const zdl_span_cols* dst) {
  if (!d || !dst) return dfail(d, ZDL_EINVAL, "zdl_decoder_download: null argument");
  const uint64_t n = d->n;
  const hipStream_t s = d->stream;
  DEC_TRY(d, hipSetDevice(d->device));
  auto cp = [&](const void* dp, const void* src, size_t bytes) {
    return dp ? hipMemcpyAsync(const_cast<void*>(dp), src, bytes, hipMemcpyDeviceToHost, s) : hipSuccess;
  };
  if (n) {
    DEC_TRY(d, cp(dst->trace_lo, d->lo.p, n * 8));
    DEC_TRY(d, cp(dst->id, d->id.p, n * 8));
    DEC_TRY(d, cp(dst->parent_id, d->pid.p, n * 8));
    DEC_TRY(d, cp(dst->local_svc, d->lsvc.p, n * 4));
    DEC_TRY(d, cp(dst->remote_svc, d->rsvc.p, n * 4));
    DEC_TRY(d, cp(dst->local_ip4, d->ip4.p, n * 4));
    DEC_TRY(d, cp(dst->local_ip6, d->ip6.p, n * 4));
    DEC_TRY(d, cp(dst->port_flags, d->pf.p, n * 4));
    DEC_TRY(d, cp(dst->timestamp, d->ts.p, n * 8));
    DEC_TRY(d, hipStreamSynchronize(s));
  }
  return ZDL_OK;
}

}  // extern "C"
