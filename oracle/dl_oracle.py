"""ORACLE — TEST INFRASTRUCTURE ONLY, NEVER A PRODUCT PATH.

Literal CPU restatement of the reference's dependency-link algorithm, used by
``tests/`` (and ``__graft_entry__.smoke`` / ``bench.py``'s cpu_baseline leg via
the C++ restatement) as the checker for the HIP engine. Nothing under
``zipkin_amd/`` imports this module.

Every function follows the reference file:line it names, with the reference's
own data structures (ordered dicts stand in for ``LinkedHashMap``: assigning an
existing key keeps its position, ``pop`` + re-insert moves it to the end,
exactly like ``LinkedHashMap.put/remove``). Python's ``sorted`` is a stable
TimSort, like ``Collections.sort``.

Pinned by: the reference's own test vectors (DependencyLinkerTest,
SpanNodeTest, TraceTest, ITDependencies via InMemoryStorage,
InMemoryStorageTest.replayOverwrites), transcribed into ``tests/golden/`` by
``tests/golden/make_golden.py``; see ``tests/test_oracle_golden.py``.

Paths are relative to /root/reference/zipkin/src/main/java/zipkin2/.
"""
from __future__ import annotations

import functools
from collections import deque
from typing import Dict, Iterable, List, Optional, Tuple

from zipkin_amd.model import DependencyLink, Endpoint, Kind, Span, java_string_key


class ReferenceNPE(Exception):
    """Where the reference throws java.lang.NullPointerException."""


class ReferenceIAE(Exception):
    """Where the reference throws java.lang.IllegalArgumentException."""


# ---------------------------------------------------------------- Trace.merge
def _null_safe_compare(left, right, null_first: bool) -> int:
    """Trace.nullSafeCompareTo (internal/Trace.java:118-126)."""
    if left is None:
        return 0 if right is None else (-1 if null_first else 1)
    if right is None:
        return 1 if null_first else -1
    if isinstance(left, str):
        lk, rk = java_string_key(left), java_string_key(right)
    else:
        lk, rk = left, right
    return (lk > rk) - (lk < rk)


def compare_endpoint(left: Optional[Endpoint], right: Optional[Endpoint]) -> int:
    """Trace.compareEndpoint (internal/Trace.java:105-116). Port is ignored."""
    if left is None:
        return 0 if right is None else -1
    if right is None:
        return 1
    c = _null_safe_compare(left.service_name, right.service_name, False)
    if c:
        return c
    c = _null_safe_compare(left.ipv4, right.ipv4, False)
    if c:
        return c
    return _null_safe_compare(left.ipv6, right.ipv6, False)


def cleanup_compare(left: Span, right: Span) -> int:
    """Trace.CLEANUP_COMPARATOR (internal/Trace.java:89-98)."""
    if left == right:
        return 0
    if left.id != right.id:
        return -1 if left.id < right.id else 1  # 16 lower-hex chars: string order == u64 order
    c = _null_safe_compare(left.shared, right.shared, True)
    if c:
        return c
    return compare_endpoint(left.local_endpoint, right.local_endpoint)


class EndpointTracker:
    """Trace.EndpointTracker (internal/Trace.java:132-157)."""

    def __init__(self):
        self.service_name = self.ipv4 = self.ipv6 = None
        self.port = 0

    def try_merge(self, e: Optional[Endpoint]) -> bool:
        if e is None:
            return True
        if self.service_name is not None and e.service_name is not None and self.service_name != e.service_name:
            return False
        if self.ipv4 is not None and e.ipv4 is not None and self.ipv4 != e.ipv4:
            return False
        if self.ipv6 is not None and e.ipv6 is not None and self.ipv6 != e.ipv6:
            return False
        if self.port != 0 and e.port != 0 and self.port != e.port:
            return False
        if self.service_name is None:
            self.service_name = e.service_name
        if self.ipv4 is None:
            self.ipv4 = e.ipv4
        if self.ipv6 is None:
            self.ipv6 = e.ipv6
        if self.port == 0:
            self.port = e.port
        return True


def _endpoint_merge(acc: Endpoint, source: Optional[Endpoint]) -> Endpoint:
    """Endpoint.Builder.merge (Endpoint.java:121-129): dereferences ``source`` at
    the first field the accumulator lacks, so ``source == null`` throws NPE unless
    the accumulator already has serviceName, ipv4, ipv6 and port."""
    svc, ip4, ip6, port = acc.service_name, acc.ipv4, acc.ipv6, acc.port
    if svc is None:
        if source is None:
            raise ReferenceNPE("Endpoint.Builder.merge(null)")
        svc = source.service_name
    if ip4 is None:
        if source is None:
            raise ReferenceNPE("Endpoint.Builder.merge(null)")
        ip4 = source.ipv4
    if ip6 is None:
        if source is None:
            raise ReferenceNPE("Endpoint.Builder.merge(null)")
        ip6 = source.ipv6
    if port == 0:
        if source is None:
            raise ReferenceNPE("Endpoint.Builder.merge(null)")
        port = source.port
    return Endpoint(svc, ip4, ip6, port)


class _SpanBuilder:
    """The subset of Span.Builder that Trace.merge touches (Span.java:290-388)."""

    def __init__(self, s: Span):
        self.d = {f: getattr(s, f) for f in s.__dataclass_fields__}
        self.tags = dict(s.tags)
        self.annotations = list(s.annotations)
        # flags bit field: shared/debug "set" bits OR together (Span.java:387)
        self.shared_set = s.shared is not None
        self.shared_val = bool(s.shared)
        self.debug_set = s.debug is not None
        self.debug_val = bool(s.debug)

    def merge(self, src: Span) -> "_SpanBuilder":
        """Span.Builder.merge (Span.java:358-388)."""
        d = self.d
        if d["parent_id"] is None:
            d["parent_id"] = src.parent_id
        if d["kind"] is None:
            d["kind"] = src.kind
        if d["name"] is None:
            d["name"] = src.name
        if d["timestamp"] == 0:
            d["timestamp"] = src.timestamp
        if d["duration"] == 0:
            d["duration"] = src.duration
        if d["local_endpoint"] is None:
            d["local_endpoint"] = src.local_endpoint
        else:
            d["local_endpoint"] = _endpoint_merge(d["local_endpoint"], src.local_endpoint)
        if d["remote_endpoint"] is None:
            d["remote_endpoint"] = src.remote_endpoint
        else:
            d["remote_endpoint"] = _endpoint_merge(d["remote_endpoint"], src.remote_endpoint)
        self.annotations.extend(src.annotations)
        self.tags.update(dict(src.tags))
        if src.shared is not None:
            self.shared_set = True
            self.shared_val = self.shared_val or bool(src.shared)
        if src.debug is not None:
            self.debug_set = True
            self.debug_val = self.debug_val or bool(src.debug)
        return self

    def build(self) -> Span:
        d = dict(self.d)
        d["tags"] = tuple(sorted(self.tags.items()))
        d["annotations"] = tuple(sorted(set(self.annotations)))
        d["shared"] = self.shared_val if self.shared_set else None
        d["debug"] = self.debug_val if self.debug_set else None
        if d["parent_id"] == d["id"]:
            d["parent_id"] = None
        return Span(**d)


def trace_merge(spans: List[Span]) -> List[Span]:
    """Trace.merge (internal/Trace.java:28-87)."""
    return trace_merge_sources(spans)[0]


def trace_merge_sources(spans: List[Span]):
    """Trace.merge, also returning for every output span the input indices it was merged
    from, in Trace.merge's sorted order (the first is the head fragment). Test helper for the
    GPU tree export (zdl_tree_export); the merge itself is the same code path."""
    length = len(spans)
    if length <= 1:
        return spans, [[i] for i in range(length)]
    order = sorted(range(length), key=functools.cmp_to_key(lambda a, b: cleanup_compare(spans[a], spans[b])))
    result = [spans[k] for k in order]
    sources = [[k] for k in order]

    # longest trace id wins (Trace.java:34-39)
    trace_id = spans[0].trace_id
    for i in range(1, length):
        nxt = result[i].trace_id
        if len(trace_id) != 32:
            trace_id = nxt

    i = 0
    while i < length:
        previous = result[i]
        previous_id = previous.id
        previous_shared = previous.shared is True
        replacement = None
        if len(previous.trace_id) != len(trace_id):
            replacement = _SpanBuilder(previous)
            replacement.d["trace_id"] = trace_id
        tracker = None
        while i + 1 < length:
            nxt = result[i + 1]
            if nxt.id != previous_id:
                break
            if tracker is None:
                tracker = EndpointTracker()
                tracker.try_merge(previous.local_endpoint)
            next_shared = nxt.shared is True
            if previous_shared == next_shared and tracker.try_merge(nxt.local_endpoint):
                if replacement is None:
                    replacement = _SpanBuilder(previous)
                replacement.merge(nxt)
                previous = nxt  # Q7: the raw fragment, not the merged value (Trace.java:69)
                length -= 1
                del result[i + 1]
                sources[i].extend(sources.pop(i + 1))
                continue
            if next_shared and nxt.parent_id is None and previous.parent_id is not None:
                # shared RPC server span that wasn't propagated its parent (Trace.java:76-79)
                result[i + 1] = nxt.to_builder(parent_id=previous.parent_id)
            break
        if replacement is not None:
            result[i] = replacement.build()
        i += 1
    return result, sources


# ------------------------------------------------------------------- SpanNode
class SpanNode:
    """internal/SpanNode.java:37-103."""
    __slots__ = ("parent", "span", "children")

    def __init__(self, span: Optional[Span]):
        self.parent = None
        self.span = span
        self.children: List["SpanNode"] = []

    def add_child(self, child: Optional["SpanNode"]) -> "SpanNode":
        """SpanNode.addChild (SpanNode.java:92-103)."""
        if child is None:
            raise ReferenceNPE("child == null")
        if child is self:
            raise ReferenceIAE(f"circular dependency on {self}")
        if any(c is child for c in self.children):
            raise ReferenceIAE(f"children already contains {child}")
        self.children.append(child)
        child.parent = self
        return self

    def traverse(self):
        """Breadth-first (SpanNode.java:64-89)."""
        q = deque([self])
        while q:
            n = q.popleft()
            q.extend(n.children)
            yield n


def _key(id_: str, shared, endpoint: Optional[Endpoint]):
    """SpanNode.Key (SpanNode.java:256-293): (id, Boolean.TRUE.equals(shared), endpoint)."""
    return (id_, shared is True, endpoint)


class SpanNodeBuilder:
    """SpanNode.Builder (SpanNode.java:105-250)."""

    def __init__(self, log: Optional[List[str]] = None):
        self.log = log
        self.root_span: Optional[SpanNode] = None
        self.key_to_node: Dict = {}
        self.span_to_parent: Dict = {}

    def _fine(self, msg):
        if self.log is not None:
            self.log.append(msg)

    def build(self, spans: List[Span], cleaned: Optional[List[Span]] = None) -> SpanNode:
        """cleaned: Trace.merge(spans) already computed (tree_heads passes it to keep the
        merged span objects, whose identity maps nodes back to input fragments)."""
        if not spans:
            raise ReferenceIAE("spans were empty")
        if cleaned is None:
            cleaned = trace_merge(spans)
        trace_id = cleaned[0].trace_id
        self._fine(f"building trace tree: traceId={trace_id}")
        for s in cleaned:
            self._index(s)
        for s in cleaned:
            self._process(s)
        if self.root_span is None:
            self._fine(f"substituting dummy node for missing root span: traceId={trace_id}")
            self.root_span = SpanNode(None)
        for k, v in self.span_to_parent.items():
            child = self.key_to_node.get(k)
            parent = self.key_to_node.get(v) if v is not None else None
            if parent is None:  # headless: attach to root (SpanNode.java:157-158)
                self.root_span.add_child(child)
            else:
                parent.add_child(child)
        return self.root_span

    def _index(self, span: Span):
        """SpanNode.Builder.index (SpanNode.java:179-192)."""
        if span.shared is True:
            id_key = _key(span.id, True, span.local_endpoint)
            parent_key = _key(span.id, False, None)
        else:
            id_key = _key(span.id, span.shared, None)
            parent_key = _key(span.parent_id, False, None) if span.parent_id is not None else None
        self.span_to_parent[id_key] = parent_key

    def _process(self, span: Span):
        """SpanNode.Builder.process (SpanNode.java:203-249)."""
        endpoint = span.local_endpoint
        key = _key(span.id, span.shared, endpoint)
        no_endpoint_key = _key(span.id, span.shared, None) if endpoint is not None else key
        parent = None
        if key[1]:
            parent = _key(span.id, False, None)
        elif span.parent_id is not None:
            parent = _key(span.parent_id, True, endpoint)
            if parent in self.span_to_parent:
                self.span_to_parent[no_endpoint_key] = parent
            else:
                parent = _key(span.parent_id, False, None)
        else:
            if self.root_span is not None:
                self._fine("attributing span missing parent to root: traceId=%s, rootSpanId=%s, spanId=%s"
                           % (span.trace_id, self.root_span.span.id, key[0]))
        node = SpanNode(span)
        if parent is None and self.root_span is None:
            self.root_span = node
            self.span_to_parent.pop(no_endpoint_key, None)
        elif key[1]:
            self.key_to_node[key] = node
            self.key_to_node[no_endpoint_key] = node
        else:
            self.key_to_node[no_endpoint_key] = node


# ----------------------------------------------------------- DependencyLinker
class DependencyLinker:
    """internal/DependencyLinker.java:37-247."""

    def __init__(self, log: Optional[List[str]] = None):
        self.log = log
        self.call_counts: Dict[Tuple[str, str], int] = {}
        self.error_counts: Dict[Tuple[str, str], int] = {}

    def _fine(self, msg):
        if self.log is not None:
            self.log.append(msg)

    def put_trace(self, spans: List[Span]) -> "DependencyLinker":
        """DependencyLinker.putTrace (DependencyLinker.java:53-151)."""
        if not spans:
            return self
        trace_tree = SpanNodeBuilder(self.log).build(spans)
        self._fine("traversing trace tree, breadth-first")
        for current in trace_tree.traverse():
            cs = current.span
            if cs is None:
                self._fine("skipping fake root node for broken span tree")
                continue
            self._fine(f"processing {cs.to_json_v2()}")  # Span.toString(): JSON_V2 (Span.java:622-624)
            kind = cs.kind
            if kind == Kind.CLIENT and current.children:
                continue
            service_name = cs.local_service_name
            remote_service_name = cs.remote_service_name
            if kind is None:
                if service_name is not None and remote_service_name is not None:
                    kind = Kind.CLIENT
                else:
                    self._fine("non remote span; skipping")
                    continue
            if kind in (Kind.SERVER, Kind.CONSUMER):
                child, parent = service_name, remote_service_name
                if current is trace_tree and parent is None:
                    self._fine("root's client is unknown; skipping")
                    continue
            else:
                parent, child = service_name, remote_service_name
            is_error = cs.is_error
            if kind in (Kind.PRODUCER, Kind.CONSUMER):
                if parent is None or child is None:
                    self._fine("cannot link messaging span to its broker; skipping")
                else:
                    self.add_link(parent, child, is_error)
                continue
            remote_ancestor = self.first_remote_ancestor(current)
            if remote_ancestor is not None and remote_ancestor.local_service_name is not None:
                ra_name = remote_ancestor.local_service_name
                if kind == Kind.CLIENT and service_name is not None and ra_name != service_name:
                    self._fine("detected missing link to client span")
                    self.add_link(ra_name, service_name, False)
                if kind == Kind.SERVER or parent is None:
                    parent = ra_name
                if (not is_error and remote_ancestor.kind == Kind.CLIENT and cs.parent_id is not None
                        and cs.parent_id == remote_ancestor.id):
                    is_error = remote_ancestor.is_error
            if parent is None or child is None:
                self._fine("cannot find remote ancestor; skipping")
                continue
            self.add_link(parent, child, is_error)
        return self

    def first_remote_ancestor(self, current: SpanNode) -> Optional[Span]:
        """DependencyLinker.firstRemoteAncestor (DependencyLinker.java:153-164)."""
        a = current.parent
        while a is not None:
            s = a.span
            if s is not None and s.kind is not None:
                self._fine(f"found remote ancestor {s.to_json_v2()}")
                return s
            a = a.parent
        return None

    def add_link(self, parent: str, child: str, is_error: bool):
        """DependencyLinker.addLink (DependencyLinker.java:166-182)."""
        self._fine(f"incrementing {'error ' if is_error else ''}link {parent} -> {child}")
        key = (parent, child)
        self.call_counts[key] = self.call_counts.get(key, 0) + 1
        if is_error:
            self.error_counts[key] = self.error_counts.get(key, 0) + 1

    def link(self) -> List[DependencyLink]:
        """DependencyLinker.link() (DependencyLinker.java:184-186, 206-219)."""
        return _link(self.call_counts, self.error_counts)

    @staticmethod
    def merge(links: Iterable[DependencyLink]) -> List[DependencyLink]:
        """DependencyLinker.merge (DependencyLinker.java:189-204)."""
        calls: Dict[Tuple[str, str], int] = {}
        errs: Dict[Tuple[str, str], int] = {}
        for l in links:
            k = (l.parent, l.child)
            calls[k] = calls.get(k, 0) + l.call_count
            errs[k] = errs.get(k, 0) + l.error_count
        return _link(calls, errs)


def _link(calls, errs) -> List[DependencyLink]:
    return [DependencyLink.create(p, c, n, errs.get((p, c), 0)) for (p, c), n in calls.items()]


# ------------------------------------------------------------ InMemoryStorage
def query_test_time(spans: List[Span], end_ts_ms: int, lookback_ms: int) -> bool:
    """The time part of QueryRequest.test (storage/QueryRequest.java:262-279); the
    rest of test() is vacuous for getDependencies (no service/span/annotation/duration)."""
    ts = 0
    for s in spans:
        if s.timestamp == 0:
            continue
        if s.parent_id is None:
            ts = s.timestamp
            break
        if ts == 0 or ts > s.timestamp:
            ts = s.timestamp
    if ts == 0 or ts < (end_ts_ms - lookback_ms) * 1000 or ts > end_ts_ms * 1000:
        return False
    return True


class InMemoryStorage:
    """The slice of storage/InMemoryStorage.java that getDependencies(endTs, lookback)
    reads: accept ordering (:156-181), eviction (:184-211), traceIdsDescendingByTimestamp
    (:272-291), spansByTraceId (:448-454), getTraces(request, false) (:218-239) and
    getDependencies (:323-348)."""

    def __init__(self, strict_trace_id=True, search_enabled=True, max_span_count=500000):
        self.strict_trace_id = strict_trace_id
        self.search_enabled = search_enabled
        self.max_span_count = max_span_count
        self.by_key: Dict[Tuple[str, int], List[Span]] = {}     # spansByTraceIdTimeStamp
        self.trace_keys: Dict[str, Dict[Tuple[str, int], None]] = {}  # traceIdToTraceIdTimeStamps
        self.size = 0

    def _sorted_keys(self):
        # TIMESTAMP_DESCENDING (InMemoryStorage.java:364-378): ts desc, then lowTraceId desc
        return sorted(self.by_key, key=lambda k: (-k[1], _Desc(k[0])))

    def accept(self, spans: List[Span]) -> None:
        to_recover = (self.size + len(spans)) - self.max_span_count
        while to_recover > 0:
            to_recover -= self._delete_oldest_trace()
        for s in spans:
            low = s.trace_lo
            k = (low, s.timestamp)
            self.by_key.setdefault(k, []).append(s)
            self.size += 1
            self.trace_keys.setdefault(low, {})[k] = None

    def _delete_oldest_trace(self) -> int:
        last = self._sorted_keys()[-1]
        low = last[0]
        evicted = 0
        for k in self.trace_keys.pop(low, {}):
            evicted += len(self.by_key.pop(k, []))
        self.size -= evicted
        return evicted

    def spans_by_trace_id(self, low: str) -> List[Span]:
        out: List[Span] = []
        for k in self.trace_keys.get(low, {}):
            out.extend(self.by_key.get(k, []))
        return out

    def get_traces_for_dependencies(self, end_ts: int, lookback: int) -> List[List[Span]]:
        if end_ts <= 0:
            raise ReferenceIAE("endTs <= 0")
        if lookback <= 0:
            raise ReferenceIAE("lookback <= 0")
        if not self.search_enabled:
            return []
        ordered: Dict[str, None] = {}
        start = end_ts * 1000 - lookback * 1000
        for k in self._sorted_keys():
            if k[1] >= start or k[1] <= end_ts * 1000:  # Q4: '||' never filters (IMS:286)
                ordered[k[0]] = None
        result = []
        for low in ordered:
            nxt = self.spans_by_trace_id(low)
            if query_test_time(nxt, end_ts, lookback):
                result.append(nxt)
        return result

    def get_dependencies(self, end_ts: int, lookback: int) -> List[DependencyLink]:
        linker = DependencyLinker()
        for trace in self.get_traces_for_dependencies(end_ts, lookback):
            linker.put_trace(trace)
        return linker.link()

    def get_traces_all(self) -> List[List[Span]]:
        """getTraces() (InMemoryStorage.java:251-262): every trace unconditionally, lowTraceId
        in TreeMap(STRING_COMPARATOR) order, split by the full trace id (strictByTraceId,
        :241-249) when strictTraceId."""
        result: List[List[Span]] = []
        for low in sorted(self.trace_keys):
            same = self.spans_by_trace_id(low)
            if self.strict_trace_id:
                result.extend(strict_by_trace_id(same))
            else:
                result.append(same)
        return result

    def get_dependencies_all(self) -> List[DependencyLink]:
        """getDependencies() (InMemoryStorage.java:265-270, used by ZipkinRule): the links of
        getTraces(), through LinkDependencies (:334-348)."""
        linker = DependencyLinker()
        for trace in self.get_traces_all():
            linker.put_trace(trace)
        return linker.link()


def strict_by_trace_id(spans: List[Span]) -> List[List[Span]]:
    """InMemoryStorage.strictByTraceId (:241-249): LinkedHashMap by the full trace id."""
    groups: Dict[str, List[Span]] = {}
    for s in spans:
        groups.setdefault(s.trace_id, []).append(s)
    return list(groups.values())


# ------------------------------------------------- daily buckets (zipkin-dependencies)
# zipkin/src/test/java/zipkin2/storage/ITDependencies.java:666-700,
# storage/GroupByTraceId.java:41-54, internal/DateUtil.java:27-35.
DAY_MS = 86_400_000


def midnight_utc(epoch_millis: int) -> int:
    """DateUtil.midnightUTC: the Calendar fields below the day zeroed (a floor)."""
    return (epoch_millis // DAY_MS) * DAY_MS


def _java_div(a: int, b: int) -> int:
    """Java long division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def guess_timestamp(span: Span) -> int:
    """ITDependencies.guessTimestamp (:692-700)."""
    if span.timestamp != 0:
        return span.timestamp
    for ts, _ in span.annotations:
        if 0 < ts:
            return ts
    return 0


def floored_trace_timestamp(trace: List[Span]) -> int:
    """ITDependencies.flooredTraceTimestamp (:680-690), literally: micros are compared
    with the (already floored) millis of the current value."""
    m = 2 ** 63 - 1
    for span in trace:
        current = guess_timestamp(span)
        if current != 0 and current < m:
            m = midnight_utc(_java_div(current, 1000))
    assert m != 2 ** 63 - 1, "trace without a timestamp"
    return m


def group_by_trace_id(spans: Iterable[Span], strict: bool = False) -> List[List[Span]]:
    """GroupByTraceId.map (:41-54): LinkedHashMap by (low) trace id."""
    groups: Dict[str, List[Span]] = {}
    for s in spans:
        groups.setdefault(s.trace_id if strict else s.trace_lo, []).append(s)
    return list(groups.values())


def aggregate_links(spans: Iterable[Span]) -> Dict[int, List[DependencyLink]]:
    """ITDependencies.aggregateLinks (:666-677): midnight -> DependencyLinker.link()."""
    linkers: Dict[int, DependencyLinker] = {}
    for trace in group_by_trace_id(spans, False):
        midnight = floored_trace_timestamp(trace)
        linkers.setdefault(midnight, DependencyLinker()).put_trace(trace)
    return {m: l.link() for m, l in linkers.items()}


@functools.total_ordering
class _Desc:
    """Reverses java String order for the TIMESTAMP_DESCENDING tiebreak."""
    __slots__ = ("k",)

    def __init__(self, s):
        self.k = java_string_key(s)

    def __eq__(self, o):
        return self.k == o.k

    def __lt__(self, o):
        return self.k > o.k


# ------------------------------------------------------------- tree debugging
def tree_heads(spans: List[Span]):
    """Test helper: the tree SpanNode.Builder builds for one trace, as
    {head input index: (parent head index | -1 synthetic root | -2 the root itself, BFS index)}
    over the nodes SpanNode.traverse visits (the synthetic root not counted). A node's head is
    the first input fragment of its merged span in Trace.merge's sorted order."""
    cleaned, sources = trace_merge_sources(spans)
    head_of = {id(s): src[0] for s, src in zip(cleaned, sources)}
    root = SpanNodeBuilder().build(spans, cleaned)
    out, k = {}, 0
    for n in root.traverse():
        if n.span is None:
            continue
        if n.parent is None:
            par = -2
        elif n.parent.span is None:
            par = -1
        else:
            par = head_of[id(n.parent.span)]
        out[head_of[id(n.span)]] = (par, k)
        k += 1
    return out


def tree_parents(spans: List[Span]):
    """Builds the tree like SpanNode.Builder and returns, for the tree, a list of
    (node_span, parent_span_or_None, reachable) in BFS order. Test helper."""
    root = SpanNodeBuilder().build(spans)
    return [(n.span, n.parent.span if n.parent is not None else None) for n in root.traverse()]
