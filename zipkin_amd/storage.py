"""InMemoryStorage with getDependencies on the MI355X engine.

Drop-in for the parts of zipkin2.storage.InMemoryStorage
(zipkin/src/main/java/zipkin2/storage/InMemoryStorage.java) that
SpanStore.getDependencies(endTs, lookback) exercises:

* builder flags strictTraceId / searchEnabled / maxSpanCount (IMS:72-100);
* ``accept(spans)`` appends in arrival order and evicts the oldest traces past
  maxSpanCount (IMS:156-211); spans are packed to columns on arrival and appended to a
  device-resident store (zdl_store, HBM) once;
* ``getDependencies(endTs, lookback)`` groups by the low 64 bits of the trace id
  (IMS:323-332, 448-467; strictTraceId is ignored here like the reference), keeps
  the storage order inside a trace (distinct (lowTraceId, timestamp) keys in
  first-seen order, then insertion order); eviction, that trace order and the
  selection are computed on the device (zdl_store_evict / zdl_store_select) and linked
  there (zdl_put_selection), with the QueryRequest.test time window
  (QueryRequest.java:262-279) evaluated on the device. Returns a single-use Call
  (Call.java:370-381).
"""
from __future__ import annotations

from typing import Callable, Generic, List, Optional, Sequence, TypeVar

import numpy as np

from . import _native as N
from .columnar import pack_traces
from .linker import DependencyLinker
from .model import DependencyLink, Span

T = TypeVar("T")


class IllegalStateException(RuntimeError):
    pass


class NoSuchElementException(LookupError):
    """What IMS.deleteOldestTrace throws when a batch alone exceeds maxSpanCount
    (TreeMap.lastKey on an empty map, IMS:193-195)."""


class Call(Generic[T]):
    """zipkin2.Call: execute() once (Call.java:156, Base.execute :370-381)."""

    def __init__(self, fn: Callable[[], T]):
        self._fn = fn
        self._executed = False

    def execute(self) -> T:
        if self._executed:
            raise IllegalStateException("Already Executed")
        self._executed = True
        return self._fn()

    def map(self, mapper: Callable[[T], "U"]) -> "Call":
        return Call(lambda: mapper(self.execute()))


class InMemoryStorage:
    """The span columns live in HBM (a zdl_store, appended once per accept) with each span's
    trace id, timestamp and alive byte; the host keeps no per-span state. Eviction
    (zdl_store_evict) and a query's trace selection (zdl_store_select) run on the device and
    the selection is gathered and linked there (zdl_put_selection): only counts cross PCIe.
    Evicted spans are released by a device compaction (zdl_store_compact_evicted) once they
    outnumber the live ones, so maxSpanCount bounds the footprint like the reference's."""

    def __init__(self, strict_trace_id: bool = True, search_enabled: bool = True,
                 max_span_count: int = 500000, device: int = 0, compact_min: int = 1 << 16,
                 insertion_order: bool = True):
        """compact_min: evicted spans are released once they number more than
        max(live spans, compact_min). insertion_order=False links the selection on the streaming
        path and returns the links sorted by (parent, child) instead of DependencyLinker's order."""
        if max_span_count <= 0:
            raise ValueError("maxSpanCount <= 0")
        self.insertion_order = insertion_order
        self.strict_trace_id = strict_trace_id
        self.search_enabled = search_enabled
        self.max_span_count = max_span_count
        self.device = device
        self.compact_min = compact_min
        self._linker = DependencyLinker(device)  # owns the dictionaries
        # the queries' linkers (no window / a time window), kept between queries: a context is
        # created once and reset per query (creating one per query cost more than the link)
        self._qlinker = {}
        self._store: Optional[N.Store] = None
        self._decoder = None  # proto3.Proto3Decoder, created on the first accept_proto3
        self._json_decoder = None  # jsonv2.JsonV2Decoder, created on the first accept_json_v2

    @staticmethod
    def new_builder():
        return _Builder()

    newBuilder = new_builder

    def _st(self) -> N.Store:
        if self._store is None:
            self._store = N.Store(self.device)
        return self._store

    def _evict(self, incoming: int):
        """evictToRecoverSpans((stored + incoming) - maxSpanCount) (IMS:156-211) on the device;
        NoSuchElementException where the reference's TreeMap.lastKey throws (the store ran
        empty: everything is evicted first, like the reference's loop)."""
        st = self._st()
        to_recover = st.alive + incoming - self.max_span_count
        if to_recover <= 0:
            return
        try:
            st.evict(to_recover)
        except N.ZdlError as e:
            if e.code == N.ZDL_EREF_NSE:
                raise NoSuchElementException("evicting from an empty store") from None
            raise
        if len(st) - st.alive > max(st.alive, self.compact_min):
            st.compact_evicted()

    def accept(self, spans: Sequence[Span]) -> Call[None]:
        spans = list(spans)
        if spans:  # the reference accepts synchronously inside accept() (IMS:156-181)
            self._evict(len(spans))
            # one "trace" per span: grouping happens at query time
            cols = pack_traces([[s] for s in spans], self._linker.svc, self._linker.ip4, self._linker.ip6)
            # the normalized id's high half and width (a 17-31 digit id pads to 32 characters, high
            # half zero: strictByTraceId still tells it from the 16-character id)
            hi = np.array([int(s.trace_id[:16], 16) if len(s.trace_id) == 32 else 0 for s in spans], np.uint64)
            wide = np.array([len(s.trace_id) == 32 for s in spans], np.uint8)
            self._st().append(cols, hi, wide)
        return Call(lambda: None)

    def accept_proto3(self, data: bytes) -> Call[None]:
        """``accept(SpanBytesDecoder.PROTO3.decodeList(data))`` with the decoding on the device
        (zdl_decode_proto3): the decoded columns go from the decoder's HBM
        buffers into the store without a host round trip, high trace ids included (the strict
        no-argument getDependencies() splits by them). Raises ReferenceIllegalArgumentException
        where the reference's decoder throws."""
        if self._decoder is None:
            from .proto3 import Proto3Decoder
            self._decoder = Proto3Decoder(self._linker.svc, self._linker.ip4, self._linker.ip6, self.device)
        b = self._decoder.decode(data)
        if b.n_spans:
            self._evict(b.n_spans)
            self._st().append_device(b.dev, b.n_spans, b.dev_trace_hi, b.dev_trace_wide)
        return Call(lambda: None)

    acceptProto3 = accept_proto3

    def accept_json_v2(self, data: bytes) -> Call[None]:
        """``accept(SpanBytesDecoder.JSON_V2.decodeList(data))`` with the decoding on the device
        (zdl_decode_json_v2), the decoded HBM columns appended to the store as
        ``accept_proto3`` does. Raises ReferenceIllegalArgumentException where the reference's
        decoder throws."""
        if self._json_decoder is None:
            from .jsonv2 import JsonV2Decoder
            self._json_decoder = JsonV2Decoder(self._linker.svc, self._linker.ip4, self._linker.ip6, self.device)
        b = self._json_decoder.decode(data)
        if b.n_spans:
            self._evict(b.n_spans)
            self._st().append_device(b.dev, b.n_spans, b.dev_trace_hi, b.dev_trace_wide)
        return Call(lambda: None)

    acceptJsonV2 = accept_json_v2

    def _link_selection(self, mode: int, window=None) -> List[DependencyLink]:
        """Selects on the device (zdl_store_select: getDependencies' trace order for
        ZDL_SELECT_NEWEST, IMS:272-291, 356-366; getTraces()' for ZDL_SELECT_ALL[_STRICT],
        IMS:241-262; IMS storage order inside a trace, IMS:448-454) and links the selection."""
        if self._store is None or self._store.alive == 0:
            return []
        _, n_traces = self._store.select(mode)
        if n_traces == 0:
            return []
        key = window is not None
        linker = self._qlinker.get(key)
        if linker is None:
            linker = DependencyLinker(self.device, insertion_order=self.insertion_order)
            linker.svc, linker.ip4, linker.ip6 = self._linker.svc, self._linker.ip4, self._linker.ip6
            self._qlinker[key] = linker
        # carry=False: a context too small for the grown dictionary is replaced, never linked, so
        # a previous query's NPE or device error cannot surface here; a kept one is reset
        old = linker._ctx
        ctx = linker._context(key, carry=False)
        if ctx is old:
            ctx.reset()
        if window is not None:
            ctx.set_window(*window)
        ctx.put_selection(self._store)
        return linker.link()

    def get_dependencies(self, end_ts: Optional[int] = None, lookback: Optional[int] = None):
        """SpanStore.getDependencies(endTs, lookback) (SpanStore.java:85; IMS:323-332), in
        milliseconds, as a single-use Call over the traces selected when it is called (the
        reference's getTraces(request, false) snapshot). With no arguments, the test-only
        getDependencies() (IMS:265-270, used by ZipkinRule): every trace, grouped strictly when
        strictTraceId, returned as a list."""
        if end_ts is None and lookback is None:
            return self._link_selection(N.ZDL_SELECT_ALL_STRICT if self.strict_trace_id else N.ZDL_SELECT_ALL)
        if end_ts is None or end_ts <= 0:
            raise ValueError("endTs <= 0")
        if lookback is None or lookback <= 0:
            raise ValueError("lookback <= 0")
        if not self.search_enabled:
            return Call(lambda: [])
        # the selection is the snapshot taken now (getTraces(request, false)); LinkDependencies
        # is a Call.map, so a reference exception (quirk Q1) comes out of execute() (IMS:331-348)
        try:
            links = self._link_selection(N.ZDL_SELECT_NEWEST, (end_ts, lookback))
        except (N.ReferenceNullPointerException, N.ReferenceIllegalArgumentException) as ex:
            err = ex

            def fail():
                raise err
            return Call(fail)
        return Call(lambda: links)

    getDependencies = get_dependencies

    def clear(self):
        if self._store is not None:
            self._store.clear()

    def close(self):
        self._linker.close()
        for q in self._qlinker.values():
            q.close()
        self._qlinker = {}
        for d in (self._decoder, self._json_decoder):
            if d is not None:
                d.close()
        self._decoder = self._json_decoder = None
        if self._store is not None:
            self._store.close()
            self._store = None


class _Builder:
    def __init__(self):
        self._kw = {}

    def strictTraceId(self, v: bool):
        self._kw["strict_trace_id"] = v
        return self

    def searchEnabled(self, v: bool):
        self._kw["search_enabled"] = v
        return self

    def maxSpanCount(self, v: int):
        if v <= 0:
            raise ValueError("maxSpanCount <= 0")
        self._kw["max_span_count"] = v
        return self

    def build(self) -> InMemoryStorage:
        return InMemoryStorage(**self._kw)
