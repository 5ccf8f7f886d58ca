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
  first-seen order, then insertion order), and hands the engine only the selection
  (a permutation of the stored spans + CSR offsets: zdl_put_stored gathers on the
  device) with the QueryRequest.test time window (QueryRequest.java:262-279)
  evaluated on the device. Returns a single-use Call (Call.java:370-381).
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
    """The span columns live in HBM (a zdl_store, appended once per accept); the host keeps
    only what eviction and trace order need (low and high trace id, timestamp, alive) in
    arrays that grow by doubling. A query uploads its selection - a u32 permutation in
    getDependencies' order + CSR offsets - and the device gathers and links (zdl_put_stored).
    Evicted spans are released by a device compaction (zdl_store_compact) once they outnumber
    the live ones, so maxSpanCount bounds the footprint like the reference's."""

    def __init__(self, strict_trace_id: bool = True, search_enabled: bool = True,
                 max_span_count: int = 500000, device: int = 0, compact_min: int = 1 << 16):
        """compact_min: evicted spans are released (zdl_store_compact) once they number more
        than max(live spans, compact_min)."""
        if max_span_count <= 0:
            raise ValueError("maxSpanCount <= 0")
        self.strict_trace_id = strict_trace_id
        self.search_enabled = search_enabled
        self.max_span_count = max_span_count
        self.device = device
        self.compact_min = compact_min
        self._linker = DependencyLinker(device)  # owns the dictionaries
        self._store: Optional[N.Store] = None
        self._n = 0  # stored spans (alive or evicted, not yet compacted away)
        self._n_alive = 0
        self._lo = np.zeros(0, np.uint64)
        self._hi = np.zeros(0, np.uint64)  # 0 for 64-bit trace ids (normalized 16-char)
        self._ts = np.zeros(0, np.int64)
        self._alive = np.zeros(0, bool)
        self._decoder = None  # proto3.Proto3Decoder, created on the first accept_proto3
        self._json_decoder = None  # jsonv2.JsonV2Decoder, created on the first accept_json_v2

    @staticmethod
    def new_builder():
        return _Builder()

    newBuilder = new_builder

    # -- host index: amortized growth, eviction, compaction ---------------------------------
    def _append_index(self, lo: np.ndarray, hi: np.ndarray, ts: np.ndarray) -> None:
        k = len(lo)
        if self._n + k > len(self._lo):
            cap = max(self._n + k, 2 * len(self._lo), 1024)
            for name in ("_lo", "_hi", "_ts", "_alive"):
                old = getattr(self, name)
                grown = np.zeros(cap, old.dtype)
                grown[:self._n] = old[:self._n]
                setattr(self, name, grown)
        self._lo[self._n:self._n + k] = lo
        self._hi[self._n:self._n + k] = hi
        self._ts[self._n:self._n + k] = ts
        self._alive[self._n:self._n + k] = True
        self._n += k
        self._n_alive += k

    def _evict(self, to_recover: int):
        """evictToRecoverSpans / deleteOldestTrace (IMS:184-211): repeatedly the last key of
        TIMESTAMP_DESCENDING - the smallest timestamp, ties by the smallest lowTraceId - and
        with it every span of its lowTraceId. One sort per accept: walking the live
        (timestamp, lowTraceId) keys upwards meets the traces in eviction order."""
        if to_recover <= 0:
            return
        if self._n_alive == 0:
            raise NoSuchElementException("evicting from an empty store")
        idx = np.nonzero(self._alive[:self._n])[0]
        lo, ts = self._lo[idx], self._ts[idx]
        order = np.lexsort((lo, ts))
        ulo, first_at, counts = np.unique(lo, return_index=True, return_counts=True)
        # traces in the order their smallest key comes up
        rank = np.empty(len(lo), np.int64)
        rank[order] = np.arange(len(order))
        t_first = np.full(len(ulo), np.iinfo(np.int64).max, np.int64)
        np.minimum.at(t_first, np.searchsorted(ulo, lo), rank)
        tord = np.argsort(t_first, kind="stable")
        cum = np.cumsum(counts[tord])
        k = int(np.searchsorted(cum, to_recover)) + 1  # traces to evict
        if k > len(ulo):
            raise NoSuchElementException("evicting from an empty store")
        victims = ulo[tord[:k]]
        dead = idx[np.isin(lo, victims)]
        self._alive[dead] = False
        self._n_alive -= len(dead)
        if self._store is not None and self._n - self._n_alive > max(self._n_alive, self.compact_min):
            self._compact()

    def _compact(self):
        keep = np.nonzero(self._alive[:self._n])[0]
        self._store.compact(keep.astype(np.uint32))
        for name in ("_lo", "_hi", "_ts", "_alive"):
            setattr(self, name, getattr(self, name)[keep].copy())
        self._n = self._n_alive = len(keep)

    def accept(self, spans: Sequence[Span]) -> Call[None]:
        spans = list(spans)
        if spans:  # the reference accepts synchronously inside accept() (IMS:156-181)
            self._evict((self._n_alive + len(spans)) - self.max_span_count)
            # one "trace" per span: grouping happens at query time
            cols = pack_traces([[s] for s in spans], self._linker.svc, self._linker.ip4, self._linker.ip6)
            if self._store is None:
                self._store = N.Store(self.device)
            self._store.append(cols)
            hi = np.array([int(s.trace_id[:16], 16) if len(s.trace_id) == 32 else 0 for s in spans], np.uint64)
            self._append_index(cols.trace_lo, hi, cols.timestamp)
        return Call(lambda: None)

    def accept_proto3(self, data: bytes) -> Call[None]:
        """``accept(SpanBytesDecoder.PROTO3.decodeList(data))`` with the decoding on the device
        (zdl_decode_proto3): the decoded columns go from the decoder's HBM
        buffers into the store without a host round trip; only the low trace ids and
        timestamps come back for eviction and trace order. Raises
        ReferenceIllegalArgumentException where the reference's decoder throws. (The
        strict no-argument getDependencies() needs high trace ids, which this path does not
        bring back: it groups these spans by their low trace id.)"""
        if self._decoder is None:
            from .proto3 import Proto3Decoder
            self._decoder = Proto3Decoder(self._linker.svc, self._linker.ip4, self._linker.ip6, self.device)
        b = self._decoder.decode(data)
        if b.n_spans:
            self._evict((self._n_alive + b.n_spans) - self.max_span_count)
            if self._store is None:
                self._store = N.Store(self.device)
            self._store.append_device(b.dev, b.n_spans)
            self._append_index(b.trace_lo, np.zeros(b.n_spans, np.uint64), b.timestamp)
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
            self._evict((self._n_alive + b.n_spans) - self.max_span_count)
            if self._store is None:
                self._store = N.Store(self.device)
            self._store.append_device(b.dev, b.n_spans)
            self._append_index(b.trace_lo, np.zeros(b.n_spans, np.uint64), b.timestamp)
        return Call(lambda: None)

    acceptJsonV2 = accept_json_v2

    # -- trace selections -------------------------------------------------------------------
    def _storage_order(self, idx):
        """IMS storage order inside a low trace id (spansByTraceId, IMS:448-454): distinct
        (lowTraceId, timestamp) keys in first-seen order, then arrival. Returns, per alive span,
        the first arrival of its key (the sort key before the arrival itself)."""
        low, ts = self._lo[idx], self._ts[idx]
        keys = np.stack([low, ts.view(np.uint64)], axis=1)
        _, inv = np.unique(keys, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        first = np.full(inv.max() + 1, np.iinfo(np.int64).max, np.int64)
        np.minimum.at(first, inv, np.arange(len(idx), dtype=np.int64))
        return first[inv]

    def _selection(self):
        """Alive spans grouped by trace_lo, in getDependencies' trace order: IMS iterates
        spansByTraceIdTimeStamp in TIMESTAMP_DESCENDING order (timestamp, then lowTraceId,
        both descending; IMS:272-291, 356-366), so a trace comes at its newest key. Inside a
        trace: IMS storage order. Returns (store positions, CSR offsets) or None."""
        idx = np.nonzero(self._alive[:self._n])[0]
        if len(idx) == 0:
            return None
        low = self._lo[idx]
        ts = self._ts[idx]
        key_first = self._storage_order(idx)
        ulow, tinv = np.unique(low, return_inverse=True)
        newest = np.full(len(ulow), np.iinfo(np.int64).min, np.int64)
        np.maximum.at(newest, tinv.reshape(-1), ts)
        newest = newest[tinv.reshape(-1)]
        order = np.lexsort((np.arange(len(idx)), key_first, ~low, -newest))
        sel = idx[order]
        low_sorted = self._lo[sel]
        starts = np.nonzero(np.concatenate([[True], low_sorted[1:] != low_sorted[:-1]]))[0]
        offsets = np.concatenate([starts, [len(sel)]]).astype(np.uint64)
        return sel.astype(np.uint32), offsets

    def _selection_all(self):
        """getTraces() (IMS:251-262): every alive trace, lowTraceId ascending (TreeMap with
        STRING_COMPARATOR over normalized 16-hex ids = numeric order), storage order inside;
        with strictTraceId each split by the full trace id in first-seen order
        (strictByTraceId, IMS:241-249)."""
        idx = np.nonzero(self._alive[:self._n])[0]
        if len(idx) == 0:
            return None
        low, hi = self._lo[idx], self._hi[idx]
        inner = np.lexsort((np.arange(len(idx)), self._storage_order(idx), low))  # storage order per low id
        rank = np.empty(len(idx), np.int64)
        rank[inner] = np.arange(len(idx))
        if self.strict_trace_id:
            keys = np.stack([low, hi], axis=1)
            _, ginv = np.unique(keys, axis=0, return_inverse=True)
            ginv = ginv.reshape(-1)
            gfirst = np.full(ginv.max() + 1, np.iinfo(np.int64).max, np.int64)
            np.minimum.at(gfirst, ginv, rank)
            order = np.lexsort((rank, gfirst[ginv], low))
        else:
            order = inner
        sel = idx[order]
        a, b = self._lo[sel], self._hi[sel]
        new = a[1:] != a[:-1]
        if self.strict_trace_id:
            new |= b[1:] != b[:-1]
        starts = np.nonzero(np.concatenate([[True], new]))[0]
        offsets = np.concatenate([starts, [len(sel)]]).astype(np.uint64)
        return sel.astype(np.uint32), offsets

    def _link_selection(self, picked, window=None) -> List[DependencyLink]:
        if picked is None:
            return []
        sel, offsets = picked
        linker = DependencyLinker(self.device)
        linker.svc, linker.ip4, linker.ip6 = self._linker.svc, self._linker.ip4, self._linker.ip6
        try:
            ctx = linker._context()
            if window is not None:
                ctx.set_window(*window)
            ctx.put_stored(self._store, sel, offsets)
            return linker.link()
        finally:
            linker.close()

    def get_dependencies(self, end_ts: Optional[int] = None, lookback: Optional[int] = None):
        """SpanStore.getDependencies(endTs, lookback) (SpanStore.java:85; IMS:323-332), in
        milliseconds, as a single-use Call over the traces selected when it is called (the
        reference's getTraces(request, false) snapshot). With no arguments, the test-only
        getDependencies() (IMS:265-270, used by ZipkinRule): every trace, grouped strictly when
        strictTraceId, returned as a list."""
        if end_ts is None and lookback is None:
            return self._link_selection(self._selection_all())
        if end_ts is None or end_ts <= 0:
            raise ValueError("endTs <= 0")
        if lookback is None or lookback <= 0:
            raise ValueError("lookback <= 0")
        if not self.search_enabled:
            return Call(lambda: [])
        links = self._link_selection(self._selection(), (end_ts, lookback))
        return Call(lambda: links)

    getDependencies = get_dependencies

    def clear(self):
        if self._store is not None:
            self._store.clear()
        self._n = self._n_alive = 0
        self._lo = np.zeros(0, np.uint64)
        self._hi = np.zeros(0, np.uint64)
        self._ts = np.zeros(0, np.int64)
        self._alive = np.zeros(0, bool)

    def close(self):
        self._linker.close()
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
