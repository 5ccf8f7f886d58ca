"""DependencyLinker on the MI355X engine.

Same surface as zipkin2.internal.DependencyLinker
(zipkin/src/main/java/zipkin2/internal/DependencyLinker.java:37-247):
``putTrace(spans)`` (one trace per call, returns self; empty list is a no-op),
``link()`` (a new list every call; the linker stays usable) and the static
``merge(links)``. Not thread-safe, like the reference. Where the reference
throws, this raises: ReferenceNullPointerException for quirk Q1
(Span.Builder.merge of a null endpoint), ReferenceIllegalArgumentException.

Work runs in libzdl (include/zdl.h) on the GPU; there is no CPU path.
Output order: like the reference, ``link()`` returns links in LinkedHashMap
insertion order (first addLink over the traces in put order, each tree
breadth-first; ZDL_FLAG_INSERTION_ORDER). With
``insertion_order=False`` the engine takes its streaming path and ``link()``
returns the same links sorted by (parent, child) in String order.
``merge`` keeps the reference's first-seen order.

``DependencyLinker(logger=...)`` is the package-private ``DependencyLinker(Logger)`` (:46): with
the logger enabled for DEBUG (java.util.logging FINE), every put takes the exact per-trace path
with ZDL_FLAG_TREE_EXPORT and the device's reason codes (zdl_tree_reasons) are rendered as the
reference's FINE messages, in its order (SpanNode.java:130, 145-147, 227-231;
DependencyLinker.java:57-169). "processing <span>" and "found remote ancestor <span>" quote the
node's span as Trace.merge leaves it (the fragments of its run merged, the trace id and a shared
span's missing parent id filled in): `_merged_spans` replays Trace.merge's merge loop over the
fragments in the device's sort order (zdl_tree_reasons), only to render that text.
"""
from __future__ import annotations

import functools
import logging
from typing import Iterable, List, Optional, Sequence

import numpy as np

from . import _native as N
from .columnar import Columns, Dictionary, pack_traces
from .model import DependencyLink, Span

_MAKE_LINK = functools.partial(tuple.__new__, DependencyLink)

DENSE_MAX = 67         # S*S <= 4544 (WDENSE_MAX): k_link counts in its dense LDS table
DENSE_MAX_WINDOW = 50  # S*S <= 2560 (WDENSE_MAX_WINDOW): the same with a time window


def _capacity(n: int, window: bool = False) -> int:
    """The context's service capacity for n services: the dense table while it fits, then
    powers of two (up to 1024: k_link's LOG mode, sorted and insertion order; above: a sparse
    list when sorted, the LDS hash when ranked)."""
    d = DENSE_MAX_WINDOW if window else DENSE_MAX
    if n <= d:
        return d
    cap = 128
    while cap < n:
        cap *= 2
    return cap


class _EndpointTracker:
    """Trace.EndpointTracker (Trace.java:131-155): whether fragments share one local endpoint."""
    __slots__ = ("svc", "ip4", "ip6", "port")

    def __init__(self):
        self.svc = self.ip4 = self.ip6 = None
        self.port = 0

    def try_merge(self, e) -> bool:
        if e is None:
            return True
        if self.svc is not None and e.service_name is not None and self.svc != e.service_name:
            return False
        if self.ip4 is not None and e.ipv4 is not None and self.ip4 != e.ipv4:
            return False
        if self.ip6 is not None and e.ipv6 is not None and self.ip6 != e.ipv6:
            return False
        if self.port != 0 and e.port != 0 and self.port != e.port:
            return False
        self.svc = self.svc if self.svc is not None else e.service_name
        self.ip4 = self.ip4 if self.ip4 is not None else e.ipv4
        self.ip6 = self.ip6 if self.ip6 is not None else e.ipv6
        self.port = self.port or e.port
        return True


def _endpoint_merge(acc, src):
    """Endpoint.Builder.merge (Endpoint.java:121-129); a put whose merge would dereference a null
    source threw before anything was logged, so src is never needed as null here."""
    if src is None:
        return acc
    return acc.__class__(acc.service_name if acc.service_name is not None else src.service_name,
                         acc.ipv4 if acc.ipv4 is not None else src.ipv4,
                         acc.ipv6 if acc.ipv6 is not None else src.ipv6, acc.port or src.port)


def _span_merge(frags, trace_id):
    """Span.Builder: frags[0].toBuilder() (trace id set), then merge(f) of every later fragment
    in order (Span.java:358-388): fields the builder lacks, endpoints merged, annotations and tags
    accumulated, the shared / debug flag bits OR-ed."""
    from dataclasses import replace
    first = frags[0]
    d = {f: getattr(first, f) for f in first.__dataclass_fields__}
    if len(first.trace_id) != len(trace_id):  # (Trace.java:47-49)
        d["trace_id"] = trace_id
    tags, anns = dict(first.tags), list(first.annotations)
    sh_set, sh, db_set, db = first.shared is not None, bool(first.shared), first.debug is not None, bool(first.debug)
    for src in frags[1:]:
        for k in ("parent_id", "kind", "name"):
            if d[k] is None:
                d[k] = getattr(src, k)
        for k in ("timestamp", "duration"):
            if not d[k]:
                d[k] = getattr(src, k)
        for k in ("local_endpoint", "remote_endpoint"):
            d[k] = getattr(src, k) if d[k] is None else _endpoint_merge(d[k], getattr(src, k))
        anns.extend(src.annotations)
        tags.update(dict(src.tags))
        if src.shared is not None:
            sh_set, sh = True, sh or bool(src.shared)
        if src.debug is not None:
            db_set, db = True, db or bool(src.debug)
    d.update(tags=tuple(sorted(tags.items())), annotations=tuple(sorted(set(anns))),
             shared=sh if sh_set else None, debug=db if db_set else None)
    if d["parent_id"] == d["id"]:
        d["parent_id"] = None
    return replace(first, **d)


def _merged_spans(spans, pos, trace_id):
    """Trace.merge's output spans (Trace.java:42-84) keyed by their first fragment's index in
    `spans`: the merge loop over the spans in the device's sort order `pos` (Trace.merge's
    CLEANUP_COMPARATOR order, from zdl_tree_reasons): a run of one id and sharedness whose local
    endpoints agree (EndpointTracker) is one span; a shared span without a parent id that
    follows a fragment with one takes that fragment's (:76-79); a span whose trace id is not
    the trace's longest takes it."""
    order = sorted(range(len(spans)), key=lambda i: pos[i])
    res = [spans[i] for i in order]
    out = {}
    n, k = len(order), 0
    while k < n:
        k0, prev = k, res[k]
        prev_shared = prev.shared is True
        frags = [prev]
        tracker = None
        while k + 1 < n:
            nxt = res[k + 1]
            if nxt.id != res[k0].id:
                break
            if tracker is None:
                tracker = _EndpointTracker()
                tracker.try_merge(prev.local_endpoint)
            if prev_shared == (nxt.shared is True) and tracker.try_merge(nxt.local_endpoint):
                frags.append(nxt)
                prev = nxt
                k += 1
                continue
            if nxt.shared is True and nxt.parent_id is None and prev.parent_id is not None:
                res[k + 1] = nxt.to_builder(parent_id=prev.parent_id)
            break
        out[order[k0]] = frags[0] if len(frags) == 1 and len(frags[0].trace_id) == len(trace_id) \
            else _span_merge(frags, trace_id)
        k += 1
    return out


class DependencyLinker:
    def __init__(self, device: int = 0, insertion_order: bool = True, logger: Optional[logging.Logger] = None):
        self.device = device
        self.logger = logger
        self._fine = logger is not None and logger.isEnabledFor(logging.DEBUG)
        # the FINE log needs the exact path's tree and reason codes (insertion-order contexts)
        self.insertion_order = insertion_order or self._fine
        self.svc = Dictionary()
        self.ip4 = Dictionary()
        self.ip6 = Dictionary()
        self._ctx: Optional[N.Context] = None
        self._ranked = (-1, -1, -1)

    # -- context management -------------------------------------------------
    def _context(self, window: bool = False, carry: bool = True) -> N.Context:
        """The engine context sized for the dictionary. carry=False (a query context that is
        reset before use): a context too small is closed, not linked - its counts and status
        word (a previous query's NPE or device error included) are dropped with it."""
        need = _capacity(max(len(self.svc), 1), window)
        if self._ctx is not None and not carry and self._ctx.n_services < need:
            self._ctx.close()
            self._ctx = None
        if self._ctx is None:
            self._ctx = N.Context(need, self.device, insertion_order=self.insertion_order, tree_export=self._fine)
            self._ranked = (-1, -1, -1)
        elif self._ctx.n_services < need:
            # grow the S x S table: carry the counts (in order) over on the device
            p, c, n, e = self._ctx.link(self._order())
            old = self._ctx
            self._ctx = N.Context(need, self.device, insertion_order=self.insertion_order, tree_export=self._fine)
            self._ranked = (-1, -1, -1)
            if len(p):
                self._ctx.add_links(p, c, n, e)
            old.close()
        sizes = (len(self.svc), len(self.ip4), len(self.ip6))
        if sizes != self._ranked:
            self._ctx.set_ranks(N.ZDL_DICT_SERVICE, self.svc.ranks())
            self._ctx.set_ranks(N.ZDL_DICT_IPV4, self.ip4.ranks())
            self._ctx.set_ranks(N.ZDL_DICT_IPV6, self.ip6.ranks())
            self._ranked = sizes
        return self._ctx

    def _order(self) -> int:
        return N.ZDL_ORDER_INSERTION if self.insertion_order else N.ZDL_ORDER_SORTED

    # -- reference API --------------------------------------------------------
    def put_trace(self, spans: Sequence[Span]) -> "DependencyLinker":
        """putTrace (DependencyLinker.java:53): spans of one trace. Staged by the engine
        (zdl_put_trace): consecutive calls are linked as one batch launch, in call order; an
        NPE (quirk Q1) is raised by the call whose trace throws, and the linker stays usable."""
        if not spans:
            return self
        if self._fine:  # the FINE log renders each put's tree: one put per call
            return self.put_traces([spans])
        cols = pack_traces([spans], self.svc, self.ip4, self.ip6)
        self._context().put_trace(cols)
        return self

    def put_traces(self, traces: Sequence[Sequence[Span]]) -> "DependencyLinker":
        """Batch of putTrace calls in one engine launch."""
        traces = [t for t in traces if t]
        if not traces:
            return self
        cols = pack_traces(traces, self.svc, self.ip4, self.ip6)
        self.put_columns(cols)
        if self._fine:
            self._log_put(traces, cols.n_spans)
        return self

    def _log_put(self, traces: Sequence[Sequence[Span]], n: int) -> None:
        """The last put's FINE messages from the device's tree and reason codes."""
        node_of, parent, bfs = self._ctx.tree_export(n)
        reason, anc, link, srt = self._ctx.tree_reasons(n)
        flat = [s for t in traces for s in t]
        names = self.svc.strings
        fine = self.logger.debug
        base = 0
        for t in traces:
            k = len(t)
            idx = range(base, base + k)
            by_sort = sorted(idx, key=lambda i: srt[i])
            # Trace.merge's trace id (Trace.java:34-38): the first input span's, then sorted spans'
            # while it is not 32 characters; a cleaned span of another length takes it
            tid = flat[base].trace_id
            for i in by_sort[1:]:
                if len(tid) != 32:
                    tid = flat[i].trace_id
            cleaned_tid = lambda i: tid if len(flat[i].trace_id) != len(tid) else flat[i].trace_id
            root_tid = cleaned_tid(by_sort[0])  # SpanNode.Builder's traceId: cleaned.get(0)'s
            fine(f"building trace tree: traceId={root_tid}")
            heads = [i for i in by_sort if node_of[i] == i]
            roots = [i for i in heads if parent[i] == -2]
            for i in heads:
                if reason[i] & N.ZDL_RSN_ATTRIBUTED and roots:
                    fine("attributing span missing parent to root: traceId=%s, rootSpanId=%s, spanId=%s"
                         % (cleaned_tid(i), flat[roots[0]].id, flat[i].id))
            if not roots:
                fine(f"substituting dummy node for missing root span: traceId={root_tid}")
            merged = _merged_spans(t, [srt[i] for i in idx], tid)  # by local index
            quote = lambda i: merged[i - base].to_json_v2()  # noqa: E731
            fine("traversing trace tree, breadth-first")
            if not roots:
                fine("skipping fake root node for broken span tree")
            for i in sorted((i for i in heads if bfs[i] >= 0), key=lambda i: bfs[i]):
                fine(f"processing {quote(i)}")
                r = int(reason[i])
                code = r & 7
                pa, ch, xpa, xch = (int(x) for x in link[i])
                err = "error " if r & N.ZDL_RSN_ERROR else ""
                if code == N.ZDL_RSN_NON_REMOTE:
                    fine("non remote span; skipping")
                elif code == N.ZDL_RSN_ROOT_CLIENT_UNKNOWN:
                    fine("root's client is unknown; skipping")
                elif code == N.ZDL_RSN_MESSAGING_NO_BROKER:
                    fine("cannot link messaging span to its broker; skipping")
                elif code == N.ZDL_RSN_MESSAGING:
                    fine(f"incrementing {err}link {names[pa]} -> {names[ch]}")
                elif code in (N.ZDL_RSN_LINK, N.ZDL_RSN_NO_REMOTE_ANCESTOR):
                    if r & N.ZDL_RSN_ANCESTOR:
                        fine(f"found remote ancestor {quote(int(anc[i]))}")
                    if r & N.ZDL_RSN_MISSING_LINK:
                        fine("detected missing link to client span")
                        fine(f"incrementing link {names[xpa]} -> {names[xch]}")
                    if code == N.ZDL_RSN_LINK:
                        fine(f"incrementing {err}link {names[pa]} -> {names[ch]}")
                    else:
                        fine("cannot find remote ancestor; skipping")
            base += k

    def put_columns(self, cols: Columns) -> "DependencyLinker":
        """Already-packed traces (dictionary ids must come from this linker's dictionaries)."""
        ctx = self._context()
        ctx.put_spans(cols)
        return self

    def put_mysql_rows(self, rows) -> "DependencyLinker":
        """AggregateDependencies.apply's putTrace loop over its cursor rows (mysql-v1
        AggregateDependencies.java:71-84) with DependencyLinkV2SpanIterator's projection
        (DependencyLinkV2SpanIterator.java:88-159) on the device (zdl_put_mysql_rows).

        rows: (trace_id_high, trace_id, parent_id, id, a_key, a_type, endpoint_service_name)
        tuples in the query's order (grouped by trace id, then span id); None = SQL null."""
        rows = list(rows)
        if not rows:
            return self
        m = (1 << 64) - 1
        raw = Dictionary()
        keys = {"lc": N.ZDL_AKEY_LC, "ca": N.ZDL_AKEY_CA, "cs": N.ZDL_AKEY_CS, "sa": N.ZDL_AKEY_SA,
                "sr": N.ZDL_AKEY_SR, "error": N.ZDL_AKEY_ERROR}
        cols = N.MysqlRows.arrays(
            [(r[0] or 0) & m for r in rows], [(r[1] or 0) & m for r in rows], [(r[2] or 0) & m for r in rows],
            [(r[3] or 0) & m for r in rows], [keys.get(r[4], N.ZDL_AKEY_NONE) for r in rows],
            [r[5] if r[5] is not None else -1 for r in rows],
            [raw.id(r[6]) if r[6] else -1 for r in rows])  # emptyToNull
        # ep(name) lower-cases (Endpoint.Builder.serviceName); the raw ids keep "sa".equals("ca")
        lower = np.array([self.svc.id(x.lower()) for x in raw.strings], np.int32)
        self._context().put_mysql_rows(cols, lower)
        return self

    def link(self) -> List[DependencyLink]:
        """link() (DependencyLinker.java:184)."""
        if self._ctx is None:
            return []
        p, c, n, e = self._ctx.link(self._order())
        low = self.svc.lowered()  # DependencyLink.Builder lower-cases (DependencyLink.java:72-82)
        # built without a Python frame per link (tuple.__new__ through a partial)
        return list(map(_MAKE_LINK, zip(map(low.__getitem__, p.tolist()), map(low.__getitem__, c.tolist()),
                                        n.tolist(), e.tolist())))

    @staticmethod
    def merge(links: Iterable[DependencyLink], device: int = 0) -> List[DependencyLink]:
        """merge(Iterable) (DependencyLinker.java:189-204), first-seen order, on the device."""
        links = list(links)
        if not links:
            return []
        d = Dictionary()
        p = np.array([d.id(l.parent) for l in links], np.int32)
        c = np.array([d.id(l.child) for l in links], np.int32)
        n = np.array([l.call_count for l in links], np.int64)
        e = np.array([l.error_count for l in links], np.int64)
        ctx = N.Context(_capacity(len(d)), device)
        try:
            mp, mc, mn, me = ctx.merge_links(p, c, n, e)
        finally:
            ctx.close()
        return [DependencyLink.create(d.strings[a], d.strings[b], int(x), int(y))
                for a, b, x, y in zip(mp, mc, mn, me)]

    # Java-style aliases
    putTrace = put_trace

    def close(self):
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None


def aggregate_dependencies(rows, device: int = 0) -> List[DependencyLink]:
    """mysql-v1's getDependencies after its query: AggregateDependencies.apply
    (zipkin-storage/mysql-v1/src/main/java/zipkin2/storage/mysql/v1/AggregateDependencies.java:55-84)
    over the SQL cursor's rows (spans left-joined with their lc/cs/ca/sr/sa/error annotations,
    grouped by trace then span id): DependencyLinkV2SpanIterator's projection and the linking
    on the device (zdl_put_mysql_rows), DependencyLinker.link()'s order.

    rows: (trace_id_high, trace_id, parent_id, id, a_key, a_type, endpoint_service_name)."""
    rows = list(rows)
    if not rows:  # !traces.hasNext() -> emptyList
        return []
    linker = DependencyLinker(device)
    try:
        return linker.put_mysql_rows(rows).link()
    finally:
        linker.close()
