"""ctypes binding of libzdl.so (include/zdl.h). The engine has no CPU fallback:
if the library is missing or no device can be opened, calls raise."""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ZDL_LIB_PATH") or os.path.join(HERE, "libzdl.so")  # override: A/B builds

ZDL_OK, ZDL_EINVAL, ZDL_ENOMEM, ZDL_EDEVICE, ZDL_EREF_NPE, ZDL_EREF_IAE, ZDL_EREF_NSE = 0, -1, -2, -3, -4, -5, -6
ZDL_SELECT_NEWEST, ZDL_SELECT_ALL, ZDL_SELECT_ALL_STRICT = 0, 1, 2
(ZDL_RSN_NONE, ZDL_RSN_CLIENT_PARENT, ZDL_RSN_NON_REMOTE, ZDL_RSN_ROOT_CLIENT_UNKNOWN, ZDL_RSN_MESSAGING,
 ZDL_RSN_MESSAGING_NO_BROKER, ZDL_RSN_LINK, ZDL_RSN_NO_REMOTE_ANCESTOR) = range(8)
ZDL_RSN_ANCESTOR, ZDL_RSN_MISSING_LINK, ZDL_RSN_ERROR, ZDL_RSN_ATTRIBUTED = 8, 16, 32, 64
ZDL_DICT_SERVICE, ZDL_DICT_IPV4, ZDL_DICT_IPV6 = 0, 1, 2
# JSON v2 keys (include/zdl.h): raw service token text, ipv4 text, ipv6 text (missing list only)
ZDL_DICT_JSON_SERVICE, ZDL_DICT_JSON_IPV4, ZDL_DICT_JSON_IPV6TEXT = 3, 4, 5
ZDL_ORDER_SORTED, ZDL_ORDER_FIRST_SEEN, ZDL_ORDER_INSERTION = 0, 1, 2
ZDL_DAYS_SKIP_OUTSIDE = 0x80000000
ZDL_FLAG_TIMING = 1
ZDL_FLAG_TIMING_ALL = 2
ZDL_FLAG_INSERTION_ORDER = 4
ZDL_FLAG_TREE_EXPORT = 8
ZDL_FLAG_TREE_STREAM = 32
ZDL_FLAG_DENSE_TABLE = 16
ZDL_AKEY_NONE, ZDL_AKEY_LC, ZDL_AKEY_CA, ZDL_AKEY_CS, ZDL_AKEY_SA, ZDL_AKEY_SR, ZDL_AKEY_ERROR = range(7)

PF_KIND_SHIFT = 16
PF_SHARED_SHIFT = 19
PF_ERROR = 1 << 21
PF_RIP4 = 1 << 22
PF_RIP6 = 1 << 23
PF_RPORT = 1 << 24
KIND_NULL = 7

EXPORTS = (
    "zdl_abi_version", "zdl_link_occupancy", "zdl_create", "zdl_create_error", "zdl_destroy", "zdl_last_error",
    "zdl_set_ranks", "zdl_set_window", "zdl_put_spans", "zdl_put_spans_device", "zdl_sync",
    "zdl_link", "zdl_merge_links", "zdl_add_links", "zdl_reset", "zdl_table_export",
    "zdl_table_import", "zdl_get_kernel_times", "zdl_stream", "zdl_set_days", "zdl_link_days",
    "zdl_store_create", "zdl_store_destroy", "zdl_store_last_error", "zdl_store_append", "zdl_store_clear",
    "zdl_store_size", "zdl_put_stored", "zdl_store_compact", "zdl_store_append_traced", "zdl_store_append_ids", "zdl_store_alive",
    "zdl_store_evict", "zdl_store_compact_evicted", "zdl_store_select", "zdl_store_selection", "zdl_put_selection",
    "zdl_decoder_create", "zdl_decoder_destroy", "zdl_decoder_last_error", "zdl_decoder_bind",
    "zdl_decoder_dict_size", "zdl_decoder_missing", "zdl_decode_proto3", "zdl_decode_proto3_retry",
    "zdl_decoder_download", "zdl_decoder_kernel_ms", "zdl_put_mysql_rows", "zdl_rows_last_error",
    "zdl_comm_unique_id", "zdl_comm_init", "zdl_put_spans_device_multi", "zdl_device_count", "zdl_shard_of",
    "zdl_tree_export", "zdl_tree_reasons", "zdl_decode_json_v2", "zdl_decode_retry", "zdl_decoder_struct_ms", "zdl_decoder_exact_spans",
    "zdl_link_start", "zdl_link_finish", "zdl_put_trace", "zdl_comm_init_local",
)
ZDL_ABI_VERSION = 7
ZDL_COMM_ID_BYTES = 128


class SpanCols(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in (
        "trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6",
        "port_flags", "timestamp", "ord")]


class Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("n_services", C.c_uint32), ("flags", C.c_uint32),
                ("timing_stride", C.c_uint32), ("n_devices", C.c_uint32), ("device_ids", C.POINTER(C.c_int32))]


class Links(C.Structure):
    _fields_ = [("n", C.c_uint64), ("parent", C.POINTER(C.c_int32)), ("child", C.POINTER(C.c_int32)),
                ("call_count", C.POINTER(C.c_int64)), ("error_count", C.POINTER(C.c_int64))]


class DayLinks(C.Structure):
    _fields_ = [("n_days", C.c_uint64), ("day_ms", C.POINTER(C.c_int64)), ("n", C.c_uint64),
                ("day", C.POINTER(C.c_int64)), ("parent", C.POINTER(C.c_int32)), ("child", C.POINTER(C.c_int32)),
                ("call_count", C.POINTER(C.c_int64)), ("error_count", C.POINTER(C.c_int64))]


class MysqlRows(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("trace_lo", "trace_hi", "span_id", "parent_id", "a_key", "a_type",
                                          "service")]

    @staticmethod
    def arrays(hi, lo, pid, sid, key, typ, svc) -> dict:
        return dict(trace_hi=np.asarray(hi, np.uint64), trace_lo=np.asarray(lo, np.uint64),
                    parent_id=np.asarray(pid, np.uint64), span_id=np.asarray(sid, np.uint64),
                    a_key=np.asarray(key, np.uint8), a_type=np.asarray(typ, np.int32),
                    service=np.asarray(svc, np.int32))


class Decoded(C.Structure):
    _fields_ = [("n_spans", C.c_uint64), ("dev", SpanCols), ("trace_lo", C.POINTER(C.c_uint64)),
                ("timestamp", C.POINTER(C.c_int64)), ("n_missing", C.c_uint64), ("dev_trace_hi", C.c_void_p),
                ("dev_trace_wide", C.c_void_p)]


class KernelTimes(C.Structure):
    _fields_ = [("plan_ms", C.c_float), ("tiles_ms", C.c_float), ("big_ms", C.c_float),
                ("reduce_ms", C.c_float), ("compact_ms", C.c_float), ("n_tiles", C.c_uint32),
                ("n_big", C.c_uint32), ("grid", C.c_uint32), ("full_ms", C.c_float), ("mid_ms", C.c_float),
                ("giant_ms", C.c_float), ("sparse_ms", C.c_float), ("log_entries", C.c_uint64),
                ("sparse_entries", C.c_uint64)]


class ZdlError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"zdl error {code}: {msg}")
        self.code = code


class ReferenceNullPointerException(ZdlError):
    """The reference throws java.lang.NullPointerException for this input (quirk Q1)."""


class ReferenceIllegalArgumentException(ZdlError):
    """The reference throws java.lang.IllegalArgumentException for this input."""


_lib: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    vp, i32, u32, u64, i64 = C.c_void_p, C.c_int32, C.c_uint32, C.c_uint64, C.c_int64
    L.zdl_abi_version.restype = C.c_int
    L.zdl_link_occupancy.restype = C.c_int
    L.zdl_link_occupancy.argtypes = [C.c_int, C.c_int, C.c_int]
    L.zdl_create.restype = vp
    L.zdl_create.argtypes = [C.POINTER(Config)]
    L.zdl_create_error.restype = C.c_char_p
    L.zdl_destroy.argtypes = [vp]
    L.zdl_last_error.restype = C.c_char_p
    L.zdl_last_error.argtypes = [vp]
    L.zdl_set_ranks.argtypes = [vp, C.c_int, vp, u32]
    L.zdl_set_window.argtypes = [vp, i64, i64]
    L.zdl_put_spans.argtypes = [vp, C.POINTER(SpanCols), u64, vp, u64]
    L.zdl_put_spans_device.argtypes = [vp, C.POINTER(SpanCols), u64, vp, u64]
    L.zdl_put_trace.argtypes = [vp, C.POINTER(SpanCols), u64]
    L.zdl_sync.argtypes = [vp]
    L.zdl_link.argtypes = [vp, C.c_int, C.POINTER(Links)]
    L.zdl_link_start.argtypes = [vp, C.c_int]
    L.zdl_link_finish.argtypes = [vp, C.POINTER(Links)]
    L.zdl_merge_links.argtypes = [vp, vp, vp, vp, vp, u64, C.POINTER(Links)]
    L.zdl_add_links.argtypes = [vp, vp, vp, vp, vp, u64]
    L.zdl_reset.argtypes = [vp]
    L.zdl_table_export.argtypes = [vp, vp, vp]
    L.zdl_table_import.argtypes = [vp, vp, vp]
    L.zdl_get_kernel_times.argtypes = [vp, C.POINTER(KernelTimes)]
    L.zdl_set_days.argtypes = [vp, i64, u32]
    L.zdl_link_days.argtypes = [vp, C.c_int, C.POINTER(DayLinks)]
    L.zdl_store_create.restype = vp
    L.zdl_store_create.argtypes = [C.c_int]
    L.zdl_store_destroy.argtypes = [vp]
    L.zdl_store_last_error.restype = C.c_char_p
    L.zdl_store_last_error.argtypes = [vp]
    L.zdl_store_append.argtypes = [vp, C.POINTER(SpanCols), u64]
    L.zdl_store_append.restype = C.c_int
    L.zdl_store_clear.argtypes = [vp]
    L.zdl_store_clear.restype = C.c_int
    L.zdl_store_compact.argtypes = [vp, vp, u64]
    L.zdl_store_compact.restype = C.c_int
    L.zdl_store_size.argtypes = [vp]
    L.zdl_store_size.restype = u64
    L.zdl_store_append_traced.argtypes = [vp, C.POINTER(SpanCols), vp, u64]
    L.zdl_store_append_traced.restype = C.c_int
    L.zdl_store_append_ids.argtypes = [vp, C.POINTER(SpanCols), vp, vp, u64]
    L.zdl_store_append_ids.restype = C.c_int
    L.zdl_store_alive.argtypes = [vp]
    L.zdl_store_alive.restype = u64
    L.zdl_store_evict.argtypes = [vp, u64, C.POINTER(u64)]
    L.zdl_store_evict.restype = C.c_int
    L.zdl_store_compact_evicted.argtypes = [vp]
    L.zdl_store_compact_evicted.restype = C.c_int
    L.zdl_store_select.argtypes = [vp, C.c_int, C.POINTER(u64), C.POINTER(u64)]
    L.zdl_store_select.restype = C.c_int
    L.zdl_store_selection.argtypes = [vp, vp, vp]
    L.zdl_store_selection.restype = C.c_int
    L.zdl_put_selection.argtypes = [vp, vp]
    L.zdl_put_selection.restype = C.c_int
    L.zdl_put_stored.argtypes = [vp, vp, vp, u64, vp, u64]
    L.zdl_put_stored.restype = C.c_int
    L.zdl_stream.restype = vp
    L.zdl_stream.argtypes = [vp]
    L.zdl_decoder_create.restype = vp
    L.zdl_decoder_create.argtypes = [C.c_int]
    L.zdl_decoder_destroy.argtypes = [vp]
    L.zdl_decoder_last_error.restype = C.c_char_p
    L.zdl_decoder_last_error.argtypes = [vp]
    L.zdl_decoder_bind.argtypes = [vp, C.c_int, C.c_char_p, u32, i32]
    L.zdl_decoder_dict_size.restype = u64
    L.zdl_decoder_dict_size.argtypes = [vp]
    L.zdl_decoder_missing.argtypes = [vp, u64, C.POINTER(C.c_int), C.POINTER(C.POINTER(C.c_uint8)),
                                      C.POINTER(u32)]
    L.zdl_decode_proto3.argtypes = [vp, C.c_char_p, u64, C.POINTER(Decoded)]
    L.zdl_decode_proto3_retry.argtypes = [vp, C.POINTER(Decoded)]
    L.zdl_decode_json_v2.argtypes = [vp, C.c_char_p, u64, C.POINTER(Decoded)]
    L.zdl_decode_retry.argtypes = [vp, C.POINTER(Decoded)]
    L.zdl_decoder_struct_ms.restype = C.c_float
    L.zdl_decoder_struct_ms.argtypes = [vp]
    L.zdl_decoder_exact_spans.restype = C.c_uint64
    L.zdl_decoder_exact_spans.argtypes = [vp]
    L.zdl_decoder_download.argtypes = [vp, C.POINTER(SpanCols)]
    L.zdl_put_mysql_rows.argtypes = [vp, C.POINTER(MysqlRows), u64, vp, u32]
    L.zdl_put_mysql_rows.restype = C.c_int
    L.zdl_rows_last_error.restype = C.c_char_p
    L.zdl_comm_unique_id.argtypes = [vp]
    L.zdl_comm_unique_id.restype = C.c_int
    L.zdl_comm_init.argtypes = [vp, vp, C.c_int, C.c_int]
    L.zdl_comm_init.restype = C.c_int
    L.zdl_comm_init_local.argtypes = [vp, C.c_int]
    L.zdl_comm_init_local.restype = C.c_int
    L.zdl_put_spans_device_multi.argtypes = [vp, C.POINTER(SpanCols), vp, vp, vp]
    L.zdl_put_spans_device_multi.restype = C.c_int
    L.zdl_device_count.argtypes = [vp]
    L.zdl_device_count.restype = C.c_int
    L.zdl_shard_of.argtypes = [vp, u64, u32, vp]
    L.zdl_shard_of.restype = None
    L.zdl_tree_export.argtypes = [vp, vp, vp, vp, u64]
    L.zdl_tree_export.restype = C.c_int
    L.zdl_tree_reasons.argtypes = [vp, vp, vp, vp, vp, u64]
    L.zdl_tree_reasons.restype = C.c_int
    if L.zdl_abi_version() != ZDL_ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI {L.zdl_abi_version()}, this binding {ZDL_ABI_VERSION}: rebuild")
    L.zdl_decoder_kernel_ms.restype = C.c_float
    L.zdl_decoder_kernel_ms.argtypes = [vp]
    for name in ("zdl_decoder_bind", "zdl_decoder_missing", "zdl_decode_proto3", "zdl_decode_proto3_retry",
                 "zdl_decoder_download", "zdl_decode_json_v2", "zdl_decode_retry"):
        getattr(L, name).restype = C.c_int
    for name in ("zdl_set_ranks", "zdl_set_window", "zdl_put_spans", "zdl_put_spans_device", "zdl_sync",
                 "zdl_link", "zdl_merge_links", "zdl_add_links", "zdl_reset", "zdl_table_export",
                 "zdl_table_import", "zdl_get_kernel_times", "zdl_set_days", "zdl_link_days"):
        getattr(L, name).restype = C.c_int
    _lib = L
    return L


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Context:
    """One zdl_ctx: a device-resident link-count table for S services."""

    def __init__(self, n_services: int, device: int = 0, timing: bool = False, timing_all: bool = False,
                 timing_stride: int = 1, insertion_order: bool = False, device_ids=None,
                 tree_export: bool = False, dense_table: bool = False, tree_stream: bool = False):
        """device_ids: a device group (zdl_config.device_ids): traces sharded over these GPUs,
        the tables summed by RCCL at link()."""
        L = lib()
        flags = (ZDL_FLAG_TIMING if timing else 0) | (ZDL_FLAG_TIMING_ALL if timing_all else 0)
        flags |= ZDL_FLAG_INSERTION_ORDER if insertion_order else 0
        flags |= ZDL_FLAG_TREE_EXPORT if tree_export else 0
        flags |= ZDL_FLAG_TREE_STREAM if tree_stream else 0
        flags |= ZDL_FLAG_DENSE_TABLE if dense_table else 0
        ids = None
        if device_ids is not None:
            ids = (C.c_int32 * len(device_ids))(*[int(d) for d in device_ids])
        cfg = Config(device, int(n_services), flags, int(timing_stride), len(device_ids) if ids else 0,
                     C.cast(ids, C.POINTER(C.c_int32)) if ids else None)
        h = L.zdl_create(C.byref(cfg))
        if not h:
            raise ZdlError(ZDL_EDEVICE, L.zdl_create_error().decode())
        self.h = C.c_void_p(h)
        self.n_services = int(n_services)
        self.insertion_order = bool(insertion_order)
        self._group = device_ids is not None
        self._L = L

    def close(self):
        if getattr(self, "h", None):
            self._L.zdl_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int):
        if rc == ZDL_OK:
            return
        msg = self._L.zdl_last_error(self.h).decode()
        if rc == ZDL_EREF_NPE:
            raise ReferenceNullPointerException(rc, msg)
        if rc == ZDL_EREF_IAE:
            raise ReferenceIllegalArgumentException(rc, msg)
        raise ZdlError(rc, msg)

    def set_ranks(self, dict_id: int, ranks: np.ndarray):
        r = np.ascontiguousarray(ranks, dtype=np.int32)
        self.check(self._L.zdl_set_ranks(self.h, dict_id, _ptr(r), len(r)))

    def set_window(self, end_ts_ms: int, lookback_ms: int):
        self.check(self._L.zdl_set_window(self.h, int(end_ts_ms), int(lookback_ms)))

    def comm_init(self, uid: bytes, rank: int, world: int) -> None:
        """Joins a multi-process job (zdl_comm_init): link() then returns every rank's links."""
        b = C.create_string_buffer(bytes(uid), ZDL_COMM_ID_BYTES)
        self.check(self._L.zdl_comm_init(self.h, b, int(rank), int(world)))

    @staticmethod
    def comm_init_local(ctxs) -> None:
        """zdl_comm_init_local: contexts of this process (one device) become ranks 0..W-1 of one
        job; each rank's link() must then run on its own thread, concurrently with the others'."""
        hs = (C.c_void_p * len(ctxs))(*[c.h.value for c in ctxs])
        rc = lib().zdl_comm_init_local(hs, len(ctxs))
        if rc != ZDL_OK:
            msg = next((c._L.zdl_last_error(c.h).decode() for c in ctxs if c._L.zdl_last_error(c.h)), "")
            raise ZdlError(rc, msg or "zdl_comm_init_local failed")

    @staticmethod
    def comm_unique_id() -> bytes:
        b = C.create_string_buffer(ZDL_COMM_ID_BYTES)
        rc = lib().zdl_comm_unique_id(b)
        if rc != ZDL_OK:
            raise ZdlError(rc, "zdl_comm_unique_id failed")
        return b.raw

    def tree_export(self, n_spans: int):
        """ZDL_FLAG_TREE_EXPORT: (node_of, parent, bfs) int32 arrays of the last put (zdl.h)."""
        out = [np.empty(n_spans, np.int32) for _ in range(3)]
        self.check(self._L.zdl_tree_export(self.h, *(_ptr(a) for a in out), int(n_spans)))
        return tuple(out)

    def tree_reasons(self, n_spans: int):
        """ZDL_FLAG_TREE_EXPORT: (reason u8, ancestor i32, link i32 [n, 4], sorted i32) of the last
        put (zdl_tree_reasons, ZDL_RSN_*)."""
        reason = np.empty(n_spans, np.uint8)
        anc = np.empty(n_spans, np.int32)
        link = np.empty((n_spans, 4), np.int32)
        srt = np.empty(n_spans, np.int32)
        self.check(self._L.zdl_tree_reasons(self.h, _ptr(reason), _ptr(anc), _ptr(link), _ptr(srt), int(n_spans)))
        return reason, anc, link, srt

    def device_count(self) -> int:
        return int(self._L.zdl_device_count(self.h))

    def put_spans(self, cols) -> None:
        """cols: columnar.Columns (host numpy arrays)."""
        if self.device_count() > 1 or self._group:
            sc = SpanCols(_ptr(cols.trace_lo), _ptr(cols.id), _ptr(cols.parent_id), _ptr(cols.local_svc),
                          _ptr(cols.remote_svc), _ptr(cols.local_ip4), _ptr(cols.local_ip6), _ptr(cols.port_flags),
                          _ptr(cols.timestamp))
            self.check(self._L.zdl_put_spans(self.h, C.byref(sc), cols.n_spans, _ptr(cols.offsets), cols.n_traces))
            return
        sc = SpanCols(None, _ptr(cols.id), _ptr(cols.parent_id), _ptr(cols.local_svc), _ptr(cols.remote_svc),
                      _ptr(cols.local_ip4), _ptr(cols.local_ip6), _ptr(cols.port_flags), _ptr(cols.timestamp))
        self.check(self._L.zdl_put_spans(self.h, C.byref(sc), cols.n_spans, _ptr(cols.offsets), cols.n_traces))

    def put_trace(self, cols) -> None:
        """zdl_put_trace: ONE trace's host columns (columnar.Columns with one trace), staged;
        raises ReferenceNullPointerException from this call when its Trace.merge throws."""
        sc = SpanCols(_ptr(cols.trace_lo), _ptr(cols.id), _ptr(cols.parent_id), _ptr(cols.local_svc),
                      _ptr(cols.remote_svc), _ptr(cols.local_ip4), _ptr(cols.local_ip6), _ptr(cols.port_flags),
                      _ptr(cols.timestamp))
        self.check(self._L.zdl_put_trace(self.h, C.byref(sc), cols.n_spans))

    def put_spans_ungrouped(self, cols, ord=None) -> None:
        """Host columns in any trace order (cols.trace_lo read, cols.offsets ignored): the
        device groups them by trace_lo, stable in `ord` (u32 storage order) or input order."""
        o = None if ord is None else np.ascontiguousarray(ord, np.uint32)
        sc = SpanCols(_ptr(cols.trace_lo), _ptr(cols.id), _ptr(cols.parent_id), _ptr(cols.local_svc),
                      _ptr(cols.remote_svc), _ptr(cols.local_ip4), _ptr(cols.local_ip6), _ptr(cols.port_flags),
                      _ptr(cols.timestamp), _ptr(o) if o is not None else None)
        self.check(self._L.zdl_put_spans(self.h, C.byref(sc), cols.n_spans, None, 0))

    def put_spans_device(self, ptrs: dict, n_spans: int, offsets_ptr: int, n_traces: int) -> None:
        sc = SpanCols(ptrs.get("trace_lo"), *(ptrs.get(k) for k in ("id", "parent_id", "local_svc", "remote_svc",
                                                                   "local_ip4", "local_ip6", "port_flags",
                                                                   "timestamp", "ord")))
        self.check(self._L.zdl_put_spans_device(self.h, C.byref(sc), n_spans, offsets_ptr, n_traces))

    def sync(self):
        self.check(self._L.zdl_sync(self.h))

    def put_mysql_rows(self, a: dict, lower: np.ndarray) -> None:
        """zdl_put_mysql_rows over host row columns (MysqlRows.arrays)."""
        a = {k: np.ascontiguousarray(v) for k, v in a.items()}
        lw = np.ascontiguousarray(lower, np.int32)
        r = MysqlRows(*(_ptr(a[k]) for k in ("trace_lo", "trace_hi", "span_id", "parent_id", "a_key", "a_type",
                                             "service")))
        rc = self._L.zdl_put_mysql_rows(self.h, C.byref(r), len(a["trace_lo"]), _ptr(lw), len(lw))
        if rc != ZDL_OK:
            msg = self._L.zdl_rows_last_error().decode()
            if rc == ZDL_EREF_IAE:
                raise ReferenceIllegalArgumentException(rc, msg)
            raise ZdlError(rc, msg)

    @staticmethod
    def _links_to_numpy(out: Links, copy: bool = True):
        n = int(out.n)
        if n == 0:
            z32, z64 = np.zeros(0, np.int32), np.zeros(0, np.int64)
            return z32, z32.copy(), z64, z64.copy()
        cols = (np.ctypeslib.as_array(out.parent, (n,)), np.ctypeslib.as_array(out.child, (n,)),
                np.ctypeslib.as_array(out.call_count, (n,)), np.ctypeslib.as_array(out.error_count, (n,)))
        return tuple(a.copy() for a in cols) if copy else cols

    def link(self, order: int = ZDL_ORDER_SORTED, copy: bool = True):
        """(parent, child, call, err) arrays; order ZDL_ORDER_SORTED or, on an
        insertion_order context, ZDL_ORDER_INSERTION (DependencyLinker.link()'s order).
        copy=False returns views of the library's output columns (zdl_links: pinned host memory
        owned by the context), valid until the context's next link/put/close - what a JNI caller
        reads without a copy."""
        out = Links()
        self.check(self._L.zdl_link(self.h, int(order), C.byref(out)))
        return self._links_to_numpy(out, copy)

    def link_start(self, order: int = ZDL_ORDER_SORTED) -> None:
        """zdl_link_start: enqueue the link list's compaction (finish with link_finish)."""
        self.check(self._L.zdl_link_start(self.h, int(order)))

    def link_finish(self, copy: bool = True):
        """zdl_link_finish: the started link's (parent, child, call, err), as link() returns them."""
        out = Links()
        self.check(self._L.zdl_link_finish(self.h, C.byref(out)))
        return self._links_to_numpy(out, copy)

    def set_days(self, day0_ms: int, n_days: int, skip_outside: bool = False):
        """Daily buckets (zdl_set_days): the timestamp column then holds guessTimestamp.
        skip_outside: traces whose day lies outside the range are skipped (ZDL_DAYS_SKIP_OUTSIDE)."""
        self.check(self._L.zdl_set_days(self.h, int(day0_ms), int(n_days) | (ZDL_DAYS_SKIP_OUTSIDE if skip_outside
                                                                                 else 0)))

    def link_days(self, order: int = ZDL_ORDER_SORTED):
        """(days, day, parent, child, call, err): the days holding a trace, then per link."""
        out = DayLinks()
        self.check(self._L.zdl_link_days(self.h, int(order), C.byref(out)))
        nd, n = int(out.n_days), int(out.n)
        days = np.ctypeslib.as_array(out.day_ms, (nd,)).copy() if nd else np.zeros(0, np.int64)
        if n == 0:
            z32, z64 = np.zeros(0, np.int32), np.zeros(0, np.int64)
            return days, z64, z32, z32.copy(), z64.copy(), z64.copy()
        arr = lambda p: np.ctypeslib.as_array(p, (n,)).copy()  # noqa: E731
        return days, arr(out.day), arr(out.parent), arr(out.child), arr(out.call_count), arr(out.error_count)

    def put_stored(self, store: "Store", perm: np.ndarray, offsets: np.ndarray) -> None:
        """zdl_put_stored: link stored spans perm[...] as CSR traces (offsets over perm)."""
        pm = np.ascontiguousarray(perm, np.uint32)
        off = np.ascontiguousarray(offsets, np.uint64)
        self.check(self._L.zdl_put_stored(self.h, store.h, _ptr(pm), len(pm), _ptr(off), len(off) - 1))

    def put_selection(self, store: "Store") -> None:
        """zdl_put_selection: link the store's current selection (Store.select), device-resident."""
        self.check(self._L.zdl_put_selection(self.h, store.h))

    def merge_links(self, parent, child, call, err):
        p, c = np.ascontiguousarray(parent, np.int32), np.ascontiguousarray(child, np.int32)
        n, e = np.ascontiguousarray(call, np.int64), np.ascontiguousarray(err, np.int64)
        out = Links()
        self.check(self._L.zdl_merge_links(self.h, _ptr(p), _ptr(c), _ptr(n), _ptr(e), len(p), C.byref(out)))
        return self._links_to_numpy(out)

    def add_links(self, parent, child, call, err):
        p, c = np.ascontiguousarray(parent, np.int32), np.ascontiguousarray(child, np.int32)
        n, e = np.ascontiguousarray(call, np.int64), np.ascontiguousarray(err, np.int64)
        self.check(self._L.zdl_add_links(self.h, _ptr(p), _ptr(c), _ptr(n), _ptr(e), len(p)))

    def reset(self):
        self.check(self._L.zdl_reset(self.h))

    def table_export(self, dev_call: int, dev_err: int):
        self.check(self._L.zdl_table_export(self.h, dev_call, dev_err))

    def table_import(self, dev_call: int, dev_err: int):
        self.check(self._L.zdl_table_import(self.h, dev_call, dev_err))

    def kernel_times(self) -> KernelTimes:
        t = KernelTimes()
        self.check(self._L.zdl_get_kernel_times(self.h, C.byref(t)))
        return t

    def stream(self) -> int:
        return self._L.zdl_stream(self.h) or 0


class Store:
    """zdl_store: span columns resident in HBM, appended once per accept."""

    def __init__(self, device: int = 0):
        L = lib()
        h = L.zdl_store_create(int(device))
        if not h:
            raise ZdlError(ZDL_EDEVICE, L.zdl_create_error().decode())
        self.h = C.c_void_p(h)
        self._L = L

    def _check(self, rc: int) -> None:
        if rc != ZDL_OK:
            raise ZdlError(rc, self._L.zdl_store_last_error(self.h).decode())

    def append_device(self, dev: SpanCols, n: int, trace_hi: Optional[int] = None,
                      trace_wide: Optional[int] = None) -> None:
        """Appends device columns (e.g. a Decoder's output, trace_lo included) without a host
        round trip; trace_hi / trace_wide: device pointers to the high trace ids (None = all 0)
        and the ids' widths (None = 128-bit iff the high half is non-zero)."""
        self._check(self._L.zdl_store_append_ids(self.h, C.byref(dev), trace_hi, trace_wide, int(n)))

    def append(self, cols, trace_hi: Optional[np.ndarray] = None, trace_wide: Optional[np.ndarray] = None) -> None:
        """Appends host columns with their trace ids (trace_hi: high 64 bits, None = 0;
        trace_wide: 1 for an id normalized to 32 hex characters, None = where trace_hi != 0)."""
        hi = None if trace_hi is None else np.ascontiguousarray(trace_hi, np.uint64)
        wd = None if trace_wide is None else np.ascontiguousarray(trace_wide, np.uint8)
        sc = SpanCols(_ptr(cols.trace_lo), _ptr(cols.id), _ptr(cols.parent_id), _ptr(cols.local_svc),
                      _ptr(cols.remote_svc), _ptr(cols.local_ip4), _ptr(cols.local_ip6), _ptr(cols.port_flags),
                      _ptr(cols.timestamp))
        self._check(self._L.zdl_store_append_ids(self.h, C.byref(sc), _ptr(hi), _ptr(wd), cols.n_spans))

    def clear(self) -> None:
        self._L.zdl_store_clear(self.h)

    def compact(self, keep: np.ndarray) -> None:
        """zdl_store_compact: keep the spans at these ascending positions, renumbered 0..n."""
        k = np.ascontiguousarray(keep, np.uint32)
        self._check(self._L.zdl_store_compact(self.h, _ptr(k), len(k)))

    def compact_evicted(self) -> None:
        """zdl_store_compact_evicted: free the evicted spans, renumbering the alive ones."""
        self._check(self._L.zdl_store_compact_evicted(self.h))

    def evict(self, to_recover: int) -> int:
        """zdl_store_evict (evictToRecoverSpans): returns the number of spans evicted. Raises
        ZdlError(ZDL_EREF_NSE) when the store runs empty first."""
        ev = C.c_uint64(0)
        self._check(self._L.zdl_store_evict(self.h, max(int(to_recover), 0), C.byref(ev)))
        return int(ev.value)

    @property
    def alive(self) -> int:
        return int(self._L.zdl_store_alive(self.h))

    def select(self, mode: int):
        """zdl_store_select: computes the selection on the device; returns (n_sel, n_traces)."""
        n, t = C.c_uint64(0), C.c_uint64(0)
        self._check(self._L.zdl_store_select(self.h, int(mode), C.byref(n), C.byref(t)))
        return int(n.value), int(t.value)

    def selection(self, mode: int):
        """The selection copied out: (u32 positions, u64 CSR trace offsets)."""
        n, t = self.select(mode)
        perm = np.empty(n, np.uint32)
        off = np.zeros(t + 1, np.uint64)
        self._check(self._L.zdl_store_selection(self.h, _ptr(perm), _ptr(off)))
        return perm, off

    def __len__(self) -> int:
        return int(self._L.zdl_store_size(self.h))

    def close(self):
        if getattr(self, "h", None):
            self._L.zdl_store_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Decoder:
    """zdl_decoder: proto3 ListOfSpans / JSON v2 span lists -> device span columns
    (zdl_decode_proto3, zdl_decode_json_v2)."""

    def __init__(self, device: int = 0):
        L = lib()
        h = L.zdl_decoder_create(int(device))
        if not h:
            raise ZdlError(ZDL_EDEVICE, "zdl_decoder_create failed")
        self.h = C.c_void_p(h)
        self._L = L
        self.gen = 0  # decodes so far: a batch's device columns belong to one generation

    def check(self, rc: int):
        if rc == ZDL_OK:
            return
        msg = self._L.zdl_decoder_last_error(self.h).decode()
        if rc == ZDL_EREF_IAE:
            raise ReferenceIllegalArgumentException(rc, msg)
        raise ZdlError(rc, msg)

    def decode(self, data: bytes) -> Decoded:
        out = Decoded()
        self.gen += 1
        self.check(self._L.zdl_decode_proto3(self.h, bytes(data), len(data), C.byref(out)))
        return out

    def decode_json(self, data: bytes) -> Decoded:
        out = Decoded()
        self.gen += 1
        self.check(self._L.zdl_decode_json_v2(self.h, bytes(data), len(data), C.byref(out)))
        return out

    def retry(self) -> Decoded:
        out = Decoded()
        self.check(self._L.zdl_decode_retry(self.h, C.byref(out)))
        return out

    def missing(self, n: int):
        """[(dict, raw key bytes)] in first-seen (span, slot) order."""
        res = []
        for i in range(n):
            k, p, ln = C.c_int(), C.POINTER(C.c_uint8)(), C.c_uint32()
            self.check(self._L.zdl_decoder_missing(self.h, i, C.byref(k), C.byref(p), C.byref(ln)))
            res.append((k.value, C.string_at(p, ln.value)))
        return res

    def bind(self, dict_id: int, key: bytes, id_: int):
        self.check(self._L.zdl_decoder_bind(self.h, int(dict_id), bytes(key), len(key), int(id_)))

    _COLS = (("trace_lo", np.uint64), ("id", np.uint64), ("parent_id", np.uint64), ("local_svc", np.int32),
             ("remote_svc", np.int32), ("local_ip4", np.int32), ("local_ip6", np.int32), ("port_flags", np.uint32),
             ("timestamp", np.int64))

    def download(self, n: int, names=None):
        """The last decode's columns (all, or `names`) as host numpy arrays (dict by column name)."""
        cols = {k: np.empty(n, t) for k, t in self._COLS if names is None or k in names}
        sc = SpanCols(*(_ptr(cols[k]) if k in cols else None for k, _ in self._COLS), None)
        self.check(self._L.zdl_decoder_download(self.h, C.byref(sc)))
        return cols

    def kernel_ms(self) -> float:
        return float(self._L.zdl_decoder_kernel_ms(self.h))

    def struct_ms(self) -> float:
        return float(self._L.zdl_decoder_struct_ms(self.h))

    def exact_spans(self) -> int:
        """Spans of the last JSON decode the exact reader took (the rest: the fast path)."""
        return int(self._L.zdl_decoder_exact_spans(self.h))

    def close(self):
        if getattr(self, "h", None):
            self._L.zdl_decoder_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_of(trace_lo: np.ndarray, n_shards: int) -> np.ndarray:
    """zdl_shard_of: the device / rank of each trace_lo (host only, no device needed)."""
    a = np.ascontiguousarray(trace_lo, np.uint64)
    out = np.empty(len(a), np.uint32)
    lib().zdl_shard_of(_ptr(a), len(a), int(n_shards), _ptr(out))
    return out
