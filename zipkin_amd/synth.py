"""Synthetic workloads of BASELINE.json via libzdl_synth.so.

Deterministic: splitmix64 streams seeded per trace from ``0x5EED0000 + config``.
Service ids are their own String-order ranks (names ``svc-00000``...; brokers
``kafka-0``... sort after them), so rank tables are the identity.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, fields, replace
from typing import Optional

import numpy as np

from .columnar import Columns
from ._native import PF_ERROR as _PF_ERROR, PF_KIND_SHIFT as _PF_KIND_SHIFT, PF_RIP4 as _PF_RIP4, PF_RIP6 as _PF_RIP6
from ._native import PF_RPORT as _PF_RPORT, PF_SHARED_SHIFT as _PF_SHARED_SHIFT

HERE = os.path.dirname(os.path.abspath(__file__))
SYNTH_PATH = os.path.join(HERE, "libzdl_synth.so")


class Params(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64), ("n_traces", C.c_uint64), ("n_services", C.c_uint32), ("n_brokers", C.c_uint32),
        ("max_depth", C.c_uint32), ("size_dist", C.c_uint32), ("lam", C.c_double), ("pareto_alpha", C.c_double),
        ("max_size", C.c_uint32), ("max_fanout", C.c_uint32), ("zipf_s", C.c_double), ("p_shared", C.c_double),
        ("p_local", C.c_double), ("p_error", C.c_double), ("p_messaging", C.c_double),
        ("p_missing_broker", C.c_double), ("p_delete", C.c_double), ("p_extra_root", C.c_double),
        ("p_uninstrumented", C.c_double), ("p_drop_shared_parent", C.c_double), ("p_split", C.c_double),
        ("p_root_remote", C.c_double), ("shard", C.c_uint32), ("n_shards", C.c_uint32),
        ("instances", C.c_uint32), ("reserved", C.c_uint32), ("base_ts_us", C.c_int64),
    ]


@dataclass(frozen=True)
class Workload:
    name: str
    seed: int
    n_traces: int
    n_services: int
    n_brokers: int = 0
    max_depth: int = 8
    size_dist: int = 0
    lam: float = 9.0
    pareto_alpha: float = 1.2
    max_size: int = 0
    max_fanout: int = 0
    zipf_s: float = 1.0
    p_shared: float = 0.7
    p_local: float = 0.15
    p_error: float = 0.02
    p_messaging: float = 0.0
    p_missing_broker: float = 0.0
    p_delete: float = 0.0
    p_extra_root: float = 0.0
    p_uninstrumented: float = 0.0
    p_drop_shared_parent: float = 0.0
    p_split: float = 0.0
    p_root_remote: float = 0.1
    shard: int = 0
    n_shards: int = 1
    instances: int = 2
    base_ts_us: int = 1704067200000000  # 2024-01-01T00:00:00Z

    @property
    def total_services(self) -> int:
        return self.n_services + self.n_brokers

    def scaled(self, n_traces: int) -> "Workload":
        return replace(self, n_traces=n_traces)

    def sharded(self, shard: int, n_shards: int) -> "Workload":
        return replace(self, shard=shard, n_shards=n_shards)

    def params(self) -> Params:
        p = Params()
        for f in fields(self):
            if f.name == "name":
                continue
            setattr(p, f.name, getattr(self, f.name))
        return p


# BASELINE.json configs; seeds 0x5EED0000 + config number
C2 = Workload("c2_10M_spans_1M_traces_50_services", 0x5EED0002, 1_000_000, 50)
C3 = Workload("c3_1B_spans_100M_traces_500_services", 0x5EED0003, 100_000_000, 500)
C4 = Workload("c4_messaging_stress", 0x5EED0004, 1_000_000, 50, n_brokers=4, p_error=0.05,
              p_messaging=0.4, p_missing_broker=0.1, p_delete=0.05, p_extra_root=0.03, p_uninstrumented=0.1,
              p_drop_shared_parent=0.1, p_split=0.05)
C5 = Workload("c5_high_cardinality_10k_services", 0x5EED0005, 16_000_000, 10_000, max_depth=64, size_dist=1,
              pareto_alpha=1.2, max_size=200_000, max_fanout=1000, zipf_s=1.1)
CONFIGS = {"c2": C2, "c3": C3, "c4": C4, "c5": C5}

_lib: Optional[C.CDLL] = None


def _synth() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(SYNTH_PATH):
            raise ImportError(f"{SYNTH_PATH} missing: run __graft_entry__.build()")
        L = C.CDLL(SYNTH_PATH)
        L.zdl_synth_sizes.restype = C.c_uint64
        L.zdl_synth_sizes.argtypes = [C.POINTER(Params), C.c_void_p, C.c_int]
        L.zdl_synth_fill.restype = None
        L.zdl_synth_fill.argtypes = [C.POINTER(Params), C.c_void_p] + [C.c_void_p] * 9 + [C.c_int]
        L.zdl_synth_shard_plan.restype = None
        L.zdl_synth_shard_plan.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_uint32, C.c_int,
                                           C.c_void_p, C.c_void_p]
        L.zdl_synth_shard.restype = C.c_double
        L.zdl_synth_shard.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_uint32, C.c_int,
                                      C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


def generate(w: Workload, threads: int = 0) -> Columns:
    threads = threads or min(16, os.cpu_count() or 1)
    L = _synth()
    p = w.params()
    off = np.empty(w.n_traces + 1, np.uint64)
    n = int(L.zdl_synth_sizes(C.byref(p), off.ctypes.data, threads))
    cols = Columns(np.empty(n, np.uint64), np.empty(n, np.uint64), np.empty(n, np.uint64),
                   np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int32),
                   np.empty(n, np.uint32), np.empty(n, np.int64), off)
    ptr = lambda a: a.ctypes.data  # noqa: E731
    L.zdl_synth_fill(C.byref(p), off.ctypes.data, ptr(cols.trace_lo), ptr(cols.id), ptr(cols.parent_id),
                     ptr(cols.local_svc), ptr(cols.remote_svc), ptr(cols.local_ip4), ptr(cols.local_ip6),
                     ptr(cols.port_flags), ptr(cols.timestamp), threads)
    return cols


def service_names(w: Workload):
    return [f"svc-{i:05d}" for i in range(w.n_services)] + [f"zkafka-{i}" for i in range(w.n_brokers)]


def encode_proto3(cols: Columns, names) -> np.ndarray:
    """The spans of `cols` (in column order) as one proto3 ListOfSpans (zdl_synth_proto3 in
    csrc/synth.cpp): what a collector would receive for the same batch. `names[i]` is service i."""
    L = _synth()
    if not hasattr(L, "_p3"):
        L.zdl_synth_proto3.restype = C.c_uint64
        L.zdl_synth_proto3.argtypes = [C.c_uint64] + [C.c_void_p] * 11
        L._p3 = True
    blob = "".join(names).encode()
    off = np.zeros(len(names) + 1, np.uint32)
    off[1:] = np.cumsum([len(x.encode()) for x in names])
    args = [cols.trace_lo, cols.id, cols.parent_id, cols.local_svc, cols.remote_svc, cols.local_ip4,
            cols.port_flags, cols.timestamp]
    ptrs = [a.ctypes.data for a in args] + [C.c_char_p(blob), off.ctypes.data]
    n = L.zdl_synth_proto3(cols.n_spans, *ptrs, None)
    out = np.empty(n, np.uint8)
    L.zdl_synth_proto3(cols.n_spans, *ptrs, out.ctypes.data)
    return out


def encode_json_v2(cols: Columns, names) -> np.ndarray:
    """The spans of `cols` (in column order) as one JSON v2 list (zdl_synth_json_v2 in
    csrc/synth.cpp, V2SpanWriter's member order). `names[i]` is service i."""
    L = _synth()
    if not hasattr(L, "_js"):
        L.zdl_synth_json_v2.restype = C.c_uint64
        L.zdl_synth_json_v2.argtypes = [C.c_uint64] + [C.c_void_p] * 11
        L._js = True
    blob = "".join(names).encode()
    off = np.zeros(len(names) + 1, np.uint32)
    off[1:] = np.cumsum([len(x.encode()) for x in names])
    args = [cols.trace_lo, cols.id, cols.parent_id, cols.local_svc, cols.remote_svc, cols.local_ip4,
            cols.port_flags, cols.timestamp]
    ptrs = [a.ctypes.data for a in args] + [C.c_char_p(blob), off.ctypes.data]
    n = L.zdl_synth_json_v2(cols.n_spans, *ptrs, None)
    out = np.empty(n, np.uint8)
    L.zdl_synth_json_v2(cols.n_spans, *ptrs, out.ctypes.data)
    return out


def put_trace_loop(ctx, cols: Columns, timestamps: bool = False) -> None:
    """One zdl_put_trace per trace of `cols`, in order, from native code (libzdl_synth's
    zdl_synth_put_trace_loop): the call pattern of the reference's putTrace callers
    (InMemoryStorage.java:340, AggregateDependencies.java:81) as a JNI shim would drive it."""
    from . import _native as N
    L = _synth()
    if not hasattr(L, "_ptl"):
        L.zdl_synth_put_trace_loop.restype = C.c_int
        L.zdl_synth_put_trace_loop.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(N.SpanCols), C.c_void_p,
                                               C.c_uint64, C.POINTER(C.c_uint64)]
        L._ptl = True
    p = N._ptr
    sc = N.SpanCols(p(cols.trace_lo), p(cols.id), p(cols.parent_id), p(cols.local_svc), p(cols.remote_svc),
                    p(cols.local_ip4), p(cols.local_ip6), p(cols.port_flags),
                    p(cols.timestamp) if timestamps else None)
    at = C.c_uint64(0)
    fn = C.cast(N.lib().zdl_put_trace, C.c_void_p)
    rc = L.zdl_synth_put_trace_loop(fn, ctx.h, C.byref(sc), cols.offsets.ctypes.data, cols.n_traces, C.byref(at))
    if rc != 0:
        ctx.check(rc)


def spans_of(cols: Columns, w: "Workload", n_traces: int):
    """The first n_traces traces of `cols` as zipkin2 Span objects (one list per trace), for
    timing the Python facade's putTrace path: service ids become service_names(w), local ip ids
    dotted quads / v6 literals, a remote endpoint's flagged ip or port a fixed value (the linker
    reads only their presence)."""
    from .model import Endpoint, Kind, Span
    names = service_names(w)
    kinds = {0: Kind.CLIENT, 1: Kind.SERVER, 2: Kind.PRODUCER, 3: Kind.CONSUMER}
    off = cols.offsets
    out = []
    for t in range(min(n_traces, cols.n_traces)):
        tr = []
        for i in range(int(off[t]), int(off[t + 1])):
            pf = int(cols.port_flags[i])
            ls, rs = int(cols.local_svc[i]), int(cols.remote_svc[i])
            l4, l6 = int(cols.local_ip4[i]), int(cols.local_ip6[i])
            le = None
            if ls >= 0 or l4 >= 0 or l6 >= 0 or (pf & 0xFFFF):
                le = Endpoint(names[ls] if ls >= 0 else None,
                              f"10.{(l4 >> 16) & 255}.{(l4 >> 8) & 255}.{l4 & 255}" if l4 >= 0 else None,
                              f"2001:db8::{l6:x}" if l6 >= 0 else None, pf & 0xFFFF)
            re = None
            if rs >= 0 or pf & (_PF_RIP4 | _PF_RIP6 | _PF_RPORT):
                re = Endpoint(names[rs] if rs >= 0 else None, "10.9.9.9" if pf & _PF_RIP4 else None,
                              "2001:db8::99" if pf & _PF_RIP6 else None, 9000 if pf & _PF_RPORT else 0)
            sh = (pf >> _PF_SHARED_SHIFT) & 3
            pid = int(cols.parent_id[i])
            tr.append(Span(f"{int(cols.trace_lo[i]):016x}", f"{int(cols.id[i]):016x}",
                           f"{pid:016x}" if pid else None, kinds.get((pf >> _PF_KIND_SHIFT) & 7),
                           None, int(cols.timestamp[i]), 0, le, re, (),
                           (("error", ""),) if pf & _PF_ERROR else (), None if sh == 0 else sh == 2, None))
        out.append(tr)
    return out


def shard_host(cols: Columns, n_shards: int, threads: int = 0, grouped: bool = True, timestamps: bool = True):
    """A device group's host split (zipkin_amd/csrc/zdl_shard.h, the code libzdl's group_put
    runs) over host columns: (shards as Columns, seconds of plan + scatter). grouped=False
    shards span by span (ungrouped input; the shards' offsets are then empty). timestamps=False
    splits the 44 B/span a put without a time window passes (the shards' timestamp columns are
    then empty)."""
    from ._native import SpanCols
    threads = threads or min(16, os.cpu_count() or 1)
    L = _synth()
    ptr = lambda a: a.ctypes.data if a is not None else None  # noqa: E731
    src = SpanCols(ptr(cols.trace_lo), ptr(cols.id), ptr(cols.parent_id), ptr(cols.local_svc), ptr(cols.remote_svc),
                   ptr(cols.local_ip4), ptr(cols.local_ip6), ptr(cols.port_flags),
                   ptr(cols.timestamp) if timestamps else None, None)
    off = cols.offsets if grouped else None
    nt = cols.n_traces if grouped else 0
    spans = np.zeros(n_shards, np.uint64)
    traces = np.zeros(n_shards, np.uint64)
    L.zdl_synth_shard_plan(C.addressof(src), cols.n_spans, ptr(off), nt, n_shards, threads, ptr(spans), ptr(traces))
    out = []
    for d in range(n_shards):
        n = int(spans[d])
        out.append(Columns(np.empty(n, np.uint64), np.empty(n, np.uint64), np.empty(n, np.uint64),
                           np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int32),
                           np.empty(n, np.uint32), np.empty(n if timestamps else 0, np.int64),
                           np.zeros(int(traces[d]) + 1 if grouped else 1, np.uint64)))
    dst = (SpanCols * n_shards)(*[SpanCols(ptr(o.trace_lo), ptr(o.id), ptr(o.parent_id), ptr(o.local_svc),
                                           ptr(o.remote_svc), ptr(o.local_ip4), ptr(o.local_ip6), ptr(o.port_flags),
                                           ptr(o.timestamp) if timestamps else None, None) for o in out])
    offp = (C.c_void_p * n_shards)(*[ptr(o.offsets) for o in out])
    sec = float(L.zdl_synth_shard(C.addressof(src), cols.n_spans, ptr(off), nt, n_shards, threads,
                                  C.addressof(dst), C.addressof(offp)))
    return out, sec

