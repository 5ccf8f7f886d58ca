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
    only what eviction and trace order need (low trace id, timestamp, alive). A query
    uploads its selection - a u32 permutation in getDependencies' order + CSR offsets - and
    the device gathers and links (zdl_put_stored)."""

    def __init__(self, strict_trace_id: bool = True, search_enabled: bool = True,
                 max_span_count: int = 500000, device: int = 0):
        if max_span_count <= 0:
            raise ValueError("maxSpanCount <= 0")
        self.strict_trace_id = strict_trace_id
        self.search_enabled = search_enabled
        self.max_span_count = max_span_count
        self.device = device
        self._linker = DependencyLinker(device)  # owns the dictionaries
        self._store: Optional[N.Store] = None
        self._lo = np.zeros(0, np.uint64)
        self._ts = np.zeros(0, np.int64)
        self._alive = np.zeros(0, bool)
        self._decoder = None  # proto3.Proto3Decoder, created on the first accept_proto3

    @staticmethod
    def new_builder():
        return _Builder()

    newBuilder = new_builder

    def accept(self, spans: Sequence[Span]) -> Call[None]:
        spans = list(spans)

        def run():
            if not spans:
                return None
            n_now = int(self._alive.sum())
            self._evict((n_now + len(spans)) - self.max_span_count)
            # one "trace" per span: grouping happens at query time
            cols = pack_traces([[s] for s in spans], self._linker.svc, self._linker.ip4, self._linker.ip6)
            if self._store is None:
                self._store = N.Store(self.device)
            self._store.append(cols)
            self._lo = np.concatenate([self._lo, cols.trace_lo])
            self._ts = np.concatenate([self._ts, cols.timestamp])
            self._alive = np.concatenate([self._alive, np.ones(len(spans), bool)])
            return None

        # the reference accepts synchronously inside accept() (IMS:156-181)
        run()
        return Call(lambda: None)

    def accept_proto3(self, data: bytes) -> Call[None]:
        """``accept(SpanBytesDecoder.PROTO3.decodeList(data))`` with the decoding on the device
        (zdl_decode_proto3): the decoded columns go from the decoder's HBM
        buffers into the store without a host round trip; only the low trace ids and
        timestamps come back for eviction and trace order. Raises
        ReferenceIllegalArgumentException where the reference's decoder throws."""
        if self._decoder is None:
            from .proto3 import Proto3Decoder
            self._decoder = Proto3Decoder(self._linker.svc, self._linker.ip4, self._linker.ip6, self.device)
        b = self._decoder.decode(data)
        if b.n_spans:
            n_now = int(self._alive.sum())
            self._evict((n_now + b.n_spans) - self.max_span_count)
            if self._store is None:
                self._store = N.Store(self.device)
            self._store.append_device(b.dev, b.n_spans)
            self._lo = np.concatenate([self._lo, b.trace_lo])
            self._ts = np.concatenate([self._ts, b.timestamp])
            self._alive = np.concatenate([self._alive, np.ones(b.n_spans, bool)])
        return Call(lambda: None)

    acceptProto3 = accept_proto3

    def _evict(self, to_recover: int):
        """deleteOldestTrace (IMS:193-211): the last key of TIMESTAMP_DESCENDING is the
        smallest timestamp, ties broken by the smallest lowTraceId."""
        while to_recover > 0:
            if not self._alive.any():
                raise NoSuchElementException("evicting from an empty store")
            idx = np.nonzero(self._alive)[0]
            ts = self._ts[idx]
            m = ts.min()
            cand = idx[ts == m]
            low = self._lo[cand].min()
            victims = idx[self._lo[idx] == low]
            self._alive[victims] = False
            to_recover -= len(victims)

    def _selection(self):
        """Alive spans grouped by trace_lo, in getDependencies' trace order: IMS iterates
        spansByTraceIdTimeStamp in TIMESTAMP_DESCENDING order (timestamp, then lowTraceId,
        both descending; IMS:272-291, 356-366), so a trace comes at its newest key. Inside a
        trace: IMS storage order (spansByTraceId, IMS:448-454). Returns (store positions,
        CSR offsets) or None."""
        idx = np.nonzero(self._alive)[0]
        if len(idx) == 0:
            return None
        low = self._lo[idx]
        ts = self._ts[idx]
        # first arrival index of each distinct (lowTraceId, timestamp) key
        keys = np.stack([low, ts.view(np.uint64)], axis=1)
        _, inv = np.unique(keys, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        first = np.full(inv.max() + 1, np.iinfo(np.int64).max, np.int64)
        np.minimum.at(first, inv, np.arange(len(idx), dtype=np.int64))
        ulow, tinv = np.unique(low, return_inverse=True)
        newest = np.full(len(ulow), np.iinfo(np.int64).min, np.int64)
        np.maximum.at(newest, tinv.reshape(-1), ts)
        newest = newest[tinv.reshape(-1)]
        order = np.lexsort((np.arange(len(idx)), first[inv], ~low, -newest))
        sel = idx[order]
        low_sorted = self._lo[sel]
        starts = np.nonzero(np.concatenate([[True], low_sorted[1:] != low_sorted[:-1]]))[0]
        offsets = np.concatenate([starts, [len(sel)]]).astype(np.uint64)
        return sel.astype(np.uint32), offsets

    def get_dependencies(self, end_ts: int, lookback: int) -> Call[List[DependencyLink]]:
        """SpanStore.getDependencies (SpanStore.java:85; IMS:323-332). Milliseconds."""
        if end_ts <= 0:
            raise ValueError("endTs <= 0")
        if lookback <= 0:
            raise ValueError("lookback <= 0")

        def run():
            if not self.search_enabled:
                return []
            picked = self._selection()
            if picked is None:
                return []
            sel, offsets = picked
            linker = DependencyLinker(self.device)
            linker.svc, linker.ip4, linker.ip6 = self._linker.svc, self._linker.ip4, self._linker.ip6
            try:
                ctx = linker._context()
                ctx.set_window(end_ts, lookback)
                ctx.put_stored(self._store, sel, offsets)
                return linker.link()
            finally:
                linker.close()

        return Call(run)

    getDependencies = get_dependencies

    def clear(self):
        if self._store is not None:
            self._store.clear()
        self._lo = np.zeros(0, np.uint64)
        self._ts = np.zeros(0, np.int64)
        self._alive = np.zeros(0, bool)

    def close(self):
        self._linker.close()
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
