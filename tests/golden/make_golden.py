"""Transcribes the reference's own test vectors for the dependency-link path into
JSON fixtures (inputs + the expectations the reference tests assert).

Nothing here is computed by the oracle or the engine: every expected value is
copied from the assertion at the cited line. Sources (relative to
/root/reference/zipkin/src/test/java/zipkin2/):

* internal/DependencyLinkerTest.java  -> dependency_linker.json
* internal/SpanNodeTest.java          -> span_node.json
* internal/TraceTest.java             -> trace_merge.json
* storage/ITDependencies.java (+ TestObjects.java), storage/InMemoryStorageTest.java
                                      -> storage_dependencies.json

TestObjects.TODAY is wall-clock midnight in the reference; it is frozen here to
TODAY below. ITDependencies.subtractDay uses an unseeded random trace id; it is
frozen to SUBTRACT_DAY_TRACE_ID.

Run:  python tests/golden/make_golden.py   (rewrites the JSON files in place)
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from zipkin_amd.codec import span_to_json  # noqa: E402
from zipkin_amd.model import Endpoint, Kind, Span, span2  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
K = Kind
TODAY = 1704067200000  # 2024-01-01T00:00:00Z, frozen TestObjects.TODAY
DAY = 86400000
SUBTRACT_DAY_TRACE_ID = "5eed5eed5eed5eed"


def L(parent, child, call, err=0):
    return {"parent": parent, "child": child, "callCount": call, "errorCount": err}


def J(spans):
    return [span_to_json(s) for s in spans]


# ------------------------------------------------------------ DependencyLinkerTest
def dependency_linker_cases():
    TRACE = [  # DependencyLinkerTest.java:31-37
        span2("a", None, "a", K.SERVER, "web", None, False),
        span2("a", "a", "b", K.CLIENT, "web", "app", False),
        span2("a", "a", "b", K.SERVER, "app", "web", False).to_builder(shared=True),
        span2("a", "b", "c", K.CLIENT, "app", "db", True),
    ]
    cases = []

    def case(name, line, traces, expect, mode="only", log_contains=None):
        cases.append({"name": name, "ref": f"DependencyLinkerTest.java:{line}",
                      "traces": [J(t) for t in traces], "expect": expect, "mode": mode,
                      "log_contains": log_contains or []})

    case("baseCase", 53, [], [], "exact")
    case("linksSpans", 58, [TRACE], [L("web", "app", 1), L("app", "db", 1, 1)], "exact")
    t = [span2("a", None, "a", K.SERVER, "arn", None, False),
         span2("a", "a", "b", K.CLIENT, "arn", "link", False),
         span2("a", None, "b", K.SERVER, "link", "arn", False).to_builder(shared=True)]
    t.reverse()
    case("linksSpans_serverMissingParentId", 71, [t], [L("arn", "link", 1)], "exact")
    case("logsTraceId", 90, [TRACE], None, "log",
         ["building trace tree: traceId=000000000000000a"])
    case("messagingSpansDontLinkWithoutBroker_consumer", 98,
         [[span2("a", None, "a", K.PRODUCER, "producer", None, False),
           span2("a", "a", "b", K.CONSUMER, "consumer", "kafka", False)]],
         [L("kafka", "consumer", 1)])
    case("messagingSpansDontLinkWithoutBroker_producer", 110,
         [[span2("a", None, "a", K.PRODUCER, "producer", "kafka", False),
           span2("a", "a", "b", K.CONSUMER, "consumer", None, False)]],
         [L("producer", "kafka", 1)])
    case("messagingWithBroker_both_sides_same", 122,
         [[span2("a", None, "a", K.PRODUCER, "producer", "kafka", False),
           span2("a", "a", "b", K.CONSUMER, "consumer", "kafka", False)]],
         [L("producer", "kafka", 1), L("kafka", "consumer", 1)])
    case("messagingWithBroker_different", 135,
         [[span2("a", None, "a", K.PRODUCER, "producer", "kafka1", False),
           span2("a", "a", "b", K.CONSUMER, "consumer", "kafka2", False)]],
         [L("producer", "kafka1", 1), L("kafka2", "consumer", 1)])
    case("messagingWithoutBroker_noLinks", 149,
         [[span2("a", None, "a", K.PRODUCER, "producer", None, False),
           span2("a", "a", "b", K.CONSUMER, "consumer", None, False)]], [], "exact")
    case("producerLinksToServer_childSpan", 161,
         [[span2("a", None, "a", K.PRODUCER, "producer", None, False),
           span2("a", "a", "b", K.SERVER, "server", None, False)]],
         [L("producer", "server", 1)])
    case("producerLinksToServer_sameSpan", 177,
         [[span2("a", None, "a", K.PRODUCER, "producer", None, False),
           span2("a", None, "a", K.SERVER, "server", None, False).to_builder(shared=True)]],
         [L("producer", "server", 1)])
    case("clientDoesntLinkToConsumer_child", 194,
         [[span2("a", None, "a", K.CLIENT, "client", None, False),
           span2("a", "a", "b", K.CONSUMER, "consumer", None, False)]], [], "exact")
    for i, s in enumerate([span2("a", None, "a", K.SERVER, "server", "client", False),
                           span2("a", None, "a", K.CLIENT, "client", "server", False).to_builder(shared=True)]):
        case(f"linksSpansDirectedByKind[{i}]", 209, [[s]], [L("client", "server", 1)])
    case("callsAgainstTheSameLinkIncreasesCallCount_span", 224,
         [[span2("a", None, "a", K.SERVER, "client", None, False),
           span2("a", "a", "b", K.CLIENT, None, "server", False),
           span2("a", "a", "c", K.CLIENT, None, "server", False)]],
         [L("client", "server", 2)])
    t = [span2("a", None, "a", K.SERVER, "client", None, False),
         span2("a", "a", "b", K.CLIENT, None, "server", False)]
    case("callsAgainstTheSameLinkIncreasesCallCount_trace", 237, [t, t], [L("client", "server", 2)])
    case("singleHostSpansResultInASingleCallCount", 255,
         [[span2("a", None, "a", K.CLIENT, "client", None, False),
           span2("a", "a", "b", K.SERVER, "server", None, False)]],
         [L("client", "server", 1)])
    case("singleHostSpansResultInASingleErrorCount", 267,
         [[span2("a", None, "a", K.CLIENT, "client", None, True),
           span2("a", "a", "b", K.SERVER, "server", None, True)]],
         [L("client", "server", 1, 1)])
    case("singleHostSpansResultInASingleErrorCount_sameId", 284,
         [[span2("a", None, "a", K.CLIENT, "client", None, True),
           span2("a", None, "a", K.SERVER, "server", None, True).to_builder(shared=True)]],
         [L("client", "server", 1, 1)])
    case("singleHostSpansResultInASingleCallCount_defersNameToServer", 302,
         [[span2("a", None, "a", K.CLIENT, "client", "server", False),
           span2("a", "a", "b", K.SERVER, "server", None, False)]],
         [L("client", "server", 1)])
    case("singleHostSpans_multipleChildren", 314,
         [[span2("a", None, "a", K.CLIENT, "client", None, False),
           span2("a", "a", "b", K.SERVER, "server", "client", True),
           span2("a", "a", "c", K.SERVER, "server", "client", False)]],
         [L("client", "server", 2, 1)])
    case("singleHostSpans_multipleChildren_defersNameToServer", 332,
         [[span2("a", None, "a", K.CLIENT, "client", "server", False),
           span2("a", "a", "b", K.SERVER, "server", None, False),
           span2("a", "a", "c", K.SERVER, "server", None, False)]],
         [L("client", "server", 2)])
    case("intermediatedClientSpansMissingLocalServiceNameLinkToNearestServer", 349,
         [[span2("a", None, "a", K.SERVER, "client", None, False),
           span2("a", "a", "b", None, None, None, False),
           span2("a", "b", "c", K.CLIENT, "server", None, False),
           span2("a", "b", "d", K.CLIENT, "server", None, False)]],
         [L("client", "server", 2)])
    case("errorsOnUninstrumentedLinks", 364,
         [[span2("a", None, "a", K.SERVER, "client", None, False),
           span2("a", "a", "b", None, None, None, False),
           span2("a", "b", "c", K.CLIENT, "server", None, True),
           span2("a", "b", "d", K.CLIENT, "server", None, True)]],
         [L("client", "server", 2)])
    case("errorsOnInstrumentedLinks", 379,
         [[span2("a", None, "a", K.SERVER, "foo", None, False),
           span2("a", "a", "b", None, None, None, False),
           span2("a", "b", "c", K.CLIENT, "bar", "baz", True),
           span2("a", "b", "d", K.CLIENT, "bar", "baz", False)]],
         [L("foo", "bar", 2), L("bar", "baz", 2, 1)])
    case("linkWithErrorIsLogged", 394,
         [[span2("a", "b", "c", K.CLIENT, "foo", "bar", True)]], None, "log",
         ["incrementing error link foo -> bar"])
    case("annotationNamedErrorDoesntIncrementErrorCount", 407,
         [[span2("a", "b", "c", K.CLIENT, "foo", "bar", False, annotations=((1, "error"),))]],
         [L("foo", "bar", 1)])
    for i, s in enumerate([span2("a", None, "a", K.SERVER, "service", "service", False),
                           span2("b", None, "b", K.CLIENT, "service", "service", False)]):
        case(f"linksLoopbackSpans[{i}]", 420, [[s]], [L("service", "service", 1)])
    case("noSpanKindTreatedSameAsClient", 434,
         [[span2("a", None, "a", None, "some-client", "web", False),
           span2("a", "a", "b", None, "web", "app", False),
           span2("a", "b", "c", None, "app", "db", False)]],
         [L("some-client", "web", 1), L("web", "app", 1), L("app", "db", 1)])
    case("noSpanKindWithError", 449,
         [[span2("a", None, "a", None, "some-client", "web", False),
           span2("a", "a", "b", None, "web", "app", True),
           span2("a", "b", "c", None, "app", "db", False)]],
         [L("some-client", "web", 1), L("web", "app", 1, 1), L("app", "db", 1)])
    for i, s in enumerate([span2("a", None, "a", K.SERVER, None, None, False),
                           span2("a", None, "a", K.SERVER, "server", None, False),
                           span2("a", None, "a", K.SERVER, None, "client", False),
                           span2("a", None, "a", K.CLIENT, None, None, False),
                           span2("a", None, "a", K.CLIENT, "client", None, False),
                           span2("a", None, "a", K.CLIENT, None, "server", False)]):
        case(f"cannotLinkSingleSpanWithoutBothServiceNames[{i}]", 465, [[s]], [], "exact")
    case("doesntLinkUnrelatedSpansWhenMissingRootSpan", 483,
         [[span2("a", "a", "b", K.SERVER, "service1", None, False),
           span2("a", "a", "c", K.SERVER, "service2", None, False)]], [], "exact",
         ["skipping fake root node for broken span tree"])
    case("linksRelatedSpansWhenMissingRootSpan", 500,
         [[span2("a", "a", "b", K.SERVER, "service1", None, False),
           span2("a", "b", "c", K.SERVER, "service2", None, False)]],
         [L("service1", "service2", 1)], "only", ["skipping fake root node for broken span tree"])
    case("linksSingleHostSpans", 518,
         [[span2("a", None, "a", K.CLIENT, "web", None, False),
           span2("a", "a", "b", K.SERVER, "app", None, False)]], [L("web", "app", 1)])
    case("linksSingleHostSpans_errorOnClient", 530,
         [[span2("a", None, "a", K.CLIENT, "web", None, True),
           span2("a", "a", "b", K.SERVER, "app", None, False)]], [L("web", "app", 1, 1)])
    case("missingSpan", 543,
         [[span2("a", None, "a", K.SERVER, "web", None, False),
           span2("a", "a", "b", K.CLIENT, "app", None, False)]], [L("web", "app", 1)], "only",
         ["detected missing link to client span"])
    merges = [
        {"name": "merge", "ref": "DependencyLinkerTest.java:558",
         "links": [L("foo", "bar", 2, 1), L("foo", "bar", 2, 2), L("foo", "foo", 1)],
         "expect": [L("foo", "bar", 4, 3), L("foo", "foo", 1)], "mode": "exact"},
        {"name": "merge_error", "ref": "DependencyLinkerTest.java:572",
         "links": [L("client", "server", 2), L("client", "server", 2), L("client", "client", 1)],
         "expect": [L("client", "server", 4), L("client", "client", 1)], "mode": "exact"},
    ]
    return {"source": "zipkin/src/test/java/zipkin2/internal/DependencyLinkerTest.java",
            "cases": cases, "merge_cases": merges}


# ------------------------------------------------------------------- SpanNodeTest
def span_node_cases():
    cases = []
    B = lambda **kw: Span.create("a", **kw)  # noqa: E731

    def lsn(name, **kw):
        return Span.create("a", local_endpoint=Endpoint.create(name), **kw)

    def case(name, line, spans, **expect):
        cases.append({"name": name, "ref": f"SpanNodeTest.java:{line}", "spans": J(spans), **expect})

    # build_redundantIgnored (:59): builder reuse => a, b, b
    t = [B(id="a"), B(id="b"), B(id="b")]
    case("build_redundantIgnored", 59, t, root=0, children=[[0, [1]]])

    def reversed_(t):
        c = list(t)
        c.reverse()
        return c

    def ancestry(name, line, t):
        # assertAncestry (:143-154): root == trace[0]; trace[i].children == [trace[i+1]]
        built = reversed_(t)
        idx = {i: len(t) - 1 - i for i in range(len(t))}  # index in trace -> index in built
        ch = [[idx[i], [idx[i + 1]]] for i in range(1, len(t) - 1)]
        case(name, line, built, root=idx[0], children=ch, children_exact=True, first_child_of_root=idx[1])

    ancestry("constructsTraceTree", 104, [
        B(id="a"), B(parent_id="a", id="b"), B(parent_id="b", id="c"), B(parent_id="c", id="d")])
    ancestry("constructsTraceTree_sharedId", 115, [
        B(id="a"), B(parent_id="a", id="b"), B(parent_id="a", id="b", shared=True),
        B(parent_id="b", id="c")])
    ancestry("constructsTraceTree_sharedRootId", 125, [
        B(id="a"), B(id="a", shared=True), B(parent_id="a", id="b"), B(parent_id="b", id="c")])

    def server_ancestry(name, line, t):
        # assertServerAncestry (:185-199)
        built = reversed_(t)
        ix = lambda i: len(t) - 1 - i  # noqa: E731
        case(name, line, built, root=ix(0),
             children=[[ix(1), [ix(3), ix(2)]], [ix(3), [ix(4)]], [ix(2), [ix(5)]]],
             children_exact=True, first_child_of_root=ix(1))

    server_ancestry("constructsTraceTree_qualifiesChildrenOfDuplicateServerSpans", 148, [
        B(id="a"), B(parent_id="a", id="b"),
        lsn("foo", parent_id="a", id="b", shared=True), lsn("bar", parent_id="a", id="b", shared=True),
        lsn("bar", parent_id="b", id="c"), lsn("foo", parent_id="b", id="d")])
    server_ancestry("constructsTraceTree_qualifiesChildrenOfDuplicateServerSpans_mixedShared", 161, [
        B(id="a"), B(parent_id="a", id="b"), lsn("foo", parent_id="b", id="c"),
        lsn("bar", parent_id="a", id="b", shared=True), lsn("bar", parent_id="b", id="d"),
        lsn("foo", parent_id="c", id="e")])
    case("constructsTraceTree_dedupes", 205, [B(id="a"), B(id="a"), B(id="a")], root=0, children=[[0, []]],
         children_exact=True)
    case("constructsTraceTree_duplicateRoots", 220, [B(id="a"), B(id="b")], root=0,
         children=[[0, [1]]], children_exact=True)
    case("build_noChildLeftBehind", 235, [
        B(id="b", name="root-0"), B(parent_id="b", id="c", name="child-0"),
        B(parent_id="b", id="d", name="child-1"), B(id="e", name="lost-0"), B(id="f", name="lost-1")],
        tree_size=5, log_exact=[
            "building trace tree: traceId=000000000000000a",
            "attributing span missing parent to root: traceId=000000000000000a, rootSpanId=000000000000000b, spanId=000000000000000e",
            "attributing span missing parent to root: traceId=000000000000000a, rootSpanId=000000000000000b, spanId=000000000000000f"])
    for name, line in (("build_headless", 257), ("build_outOfOrder", 273)):
        t = [B(parent_id="a", id="b", name="s2"), B(parent_id="a", id="c", name="s3"),
             B(parent_id="a", id="d", name="s4")]
        case(name, line, t, root=None, children=[[None, [0, 1, 2]]], children_exact=True, log_exact=[
            "building trace tree: traceId=000000000000000a",
            "substituting dummy node for missing root span: traceId=000000000000000a"])
    sk = [
        Span.create("1e223ff1f80f1c69", "43210ae0c10d1234", "74280ae0c10d8062", name="async",
                    timestamp=1470150004008762, duration=65000,
                    local_endpoint=Endpoint.create("serviceb", "192.0.0.0")),
        Span.create("1e223ff1f80f1c69", "43210ae0c10d1234", "bf396325699c84bf", K.SERVER, name="post",
                    timestamp=1541138169255688, duration=168731,
                    local_endpoint=Endpoint.create("serviceb", "192.0.0.0"), shared=True),
        Span.create("1e223ff1f80f1c69", "bb1f0e21882325b8", None, K.SERVER, name="get",
                    timestamp=1470150004071068, duration=99411,
                    local_endpoint=Endpoint.create("servicea", "127.0.0.0")),
        Span.create("1e223ff1f80f1c69", "74280ae0c10d8062", "bb1f0e21882325b8", K.CLIENT, name="post",
                    timestamp=1470150004074202, duration=94539,
                    local_endpoint=Endpoint.create("servicea", "127.0.0.0")),
    ]
    case("build_skewedTrace", 297, sk, traverse_any_order=[0, 1, 2, 3])
    return {"source": "zipkin/src/test/java/zipkin2/internal/SpanNodeTest.java", "cases": cases}


# ---------------------------------------------------------------------- TraceTest
def trace_merge_cases():
    def span(trace_id, parent_id, id_, kind, local, ip, shared, **kw):  # TraceTest.java:188-195
        ep = Endpoint.create(local, ip) if (local is not None or ip is not None) else None
        return Span.create(trace_id, id_, parent_id, kind, local_endpoint=ep, shared=shared, **kw)

    cases = []

    def case(name, line, spans, expect, mode="any_order"):
        cases.append({"name": name, "ref": f"TraceTest.java:{line}", "spans": J(spans),
                      "expect": J(expect) if mode != "trace_ids" else expect, "mode": mode})

    case("backfillsMissingParentIdOnSharedSpan", 32,
         [span("a", None, "a", K.SERVER, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, "frontend", None, False),
          span("a", None, "b", K.SERVER, "backend", None, True)],
         [span("a", None, "a", K.SERVER, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, "frontend", None, False),
          span("a", "a", "b", K.SERVER, "backend", None, True)])
    case("choosesBestTraceId", 48,
         [span("7180c278b62e8f6a216a2aea45d08fc9", None, "a", K.SERVER, "frontend", None, False),
          span("7180c278b62e8f6a216a2aea45d08fc9", "a", "b", K.CLIENT, "frontend", None, False),
          span("216a2aea45d08fc9", "a", "b", K.SERVER, "backend", None, True)],
         ["7180c278b62e8f6a216a2aea45d08fc9"] * 3, "trace_ids")
    case("mergesWhenMissingEndpoints", 63,
         [Span.create("a", "a", tags={"service": "frontend", "span.kind": "SERVER"}),
          Span.create("a", "b", "a", tags={"service": "frontend", "span.kind": "CLIENT"}, timestamp=1),
          span("a", "a", "b", K.SERVER, "backend", None, True),
          Span.create("a", "b", "a", duration=10)],
         [Span.create("a", "a", tags={"service": "frontend", "span.kind": "SERVER"}),
          Span.create("a", "b", "a", tags={"service": "frontend", "span.kind": "CLIENT"}, timestamp=1,
                      duration=10),
          span("a", "a", "b", K.SERVER, "backend", None, True)])
    case("doesntMergeSharedSpansOnDifferentIPs", 107,
         [span("a", None, "a", K.SERVER, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, "frontend", None, False, timestamp=1,
               annotations=((3, "brave.flush"),)),
          span("a", "a", "b", K.SERVER, "backend", "1.2.3.4", True),
          span("a", "a", "b", K.SERVER, "backend", "1.2.3.5", True),
          span("a", "a", "b", K.CLIENT, "frontend", None, False, duration=10)],
         [span("a", None, "a", K.SERVER, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, "frontend", None, False, timestamp=1, duration=10,
               annotations=((3, "brave.flush"),)),
          span("a", "a", "b", K.SERVER, "backend", "1.2.3.4", True),
          span("a", "a", "b", K.SERVER, "backend", "1.2.3.5", True)])
    case("putsRandomDataOnFirstSpanWithEndpoint", 128,
         [span("a", None, "a", K.SERVER, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, None, None, False),
          span("a", "a", "b", None, "frontend", None, False, timestamp=1, annotations=((3, "brave.flush"),)),
          span("a", "a", "b", K.SERVER, "backend", "1.2.3.4", True),
          span("a", "a", "b", K.SERVER, "backend", "1.2.3.5", True),
          span("a", "a", "b", None, None, None, False, duration=10)],
         [span("a", None, "a", K.SERVER, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, "frontend", None, False, timestamp=1, duration=10,
               annotations=((3, "brave.flush"),)),
          span("a", "a", "b", K.SERVER, "backend", "1.2.3.4", True),
          span("a", "a", "b", K.SERVER, "backend", "1.2.3.5", True)])
    case("mergesIncompleteEndpoints", 151,
         [span("a", None, "a", K.SERVER, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, None, "1.2.3.4", False),
          span("a", "a", "b", K.SERVER, None, "1.2.3.5", True),
          span("a", "a", "b", K.SERVER, "backend", None, True)],
         [span("a", None, "a", K.SERVER, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, "frontend", "1.2.3.4", False),
          span("a", "a", "b", K.SERVER, "backend", "1.2.3.5", True)])
    case("deletesSelfReferencingParentId", 167,
         [span("a", "a", "a", K.SERVER, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, "frontend", None, False)],
         [span("a", None, "a", K.SERVER, "frontend", None, False),
          span("a", "a", "b", K.CLIENT, "frontend", None, False)])
    t = [span("a", "a", "b", K.SERVER, "backend", "1.2.3.4", False),
         span("a", "a", "c", K.SERVER, "backend", None, False)]
    case("worksWhenMissingParentSpan", 179, t, t, "exact")
    return {"source": "zipkin/src/test/java/zipkin2/internal/TraceTest.java", "cases": cases}


# -------------------------------------------------- ITDependencies / InMemoryStorage
def storage_cases():
    FRONTEND = Endpoint.create("frontend", "127.0.0.1")                   # TestObjects.java:35-36
    BACKEND = Endpoint.create("backend", "192.168.99.101", 9000)          # :37-38
    DB = Endpoint.create("db", "2001:db8::c001", 3036)                    # :39-40
    CLIENT_SPAN = Span.create(                                            # :56-70
        "7180c278b62e8f6a216a2aea45d08fc9", "2", "1", K.CLIENT, name="get",
        local_endpoint=FRONTEND, remote_endpoint=BACKEND, timestamp=(TODAY + 50) * 1000,
        duration=200 * 1000, annotations=(((TODAY + 100) * 1000, "foo"),),
        tags={"http.path": "/api", "clnt/finagle.version": "6.45.0"})
    TRACE = [                                                             # :71-98
        Span.create(CLIENT_SPAN.trace_id, "1", None, K.SERVER, name="get", local_endpoint=FRONTEND,
                    timestamp=TODAY * 1000, duration=350 * 1000),
        CLIENT_SPAN,
        Span.create(CLIENT_SPAN.trace_id, CLIENT_SPAN.id, CLIENT_SPAN.parent_id, K.SERVER, shared=True,
                    name="get", local_endpoint=BACKEND, timestamp=(TODAY + 100) * 1000, duration=150 * 1000),
        Span.create(CLIENT_SPAN.trace_id, "3", "2", K.CLIENT, name="query", local_endpoint=BACKEND,
                    remote_endpoint=DB, timestamp=(TODAY + 150) * 1000, duration=50 * 1000,
                    annotations=(((TODAY + 190) * 1000, "⻩"),), tags={"error": "\U0001F4A9"}),
    ]
    TRACE_DURATION = TRACE[0].duration // 1000                            # :100-102
    TRACE_STARTTS = TRACE[0].timestamp // 1000
    TRACE_ENDTS = TRACE_STARTTS + TRACE_DURATION
    LINKS = [L("frontend", "backend", 1), L("backend", "db", 1, 1)]        # ITDependencies.java:56-59

    cases = []

    def case(name, line, batches, queries, source="ITDependencies"):
        cases.append({"name": name, "ref": f"{source}.java:{line}",
                      "batches": [J(b) for b in batches],
                      "queries": [{"endTs": e, "lookback": lb, "expect": ex} for e, lb, ex in queries]})

    S = Span.create
    case("getDependencies", 85, [TRACE], [(TRACE_ENDTS, DAY, LINKS)])
    mixed = [
        S("7180c278b62e8f6a216a2aea45d08fc9", "1", None, K.SERVER, name="get", timestamp=TODAY * 1000,
          duration=350 * 1000, local_endpoint=FRONTEND),
        S("216a2aea45d08fc9", "2", "1", K.SERVER, name="get", shared=True, timestamp=(TODAY + 100) * 1000,
          duration=250 * 1000, local_endpoint=BACKEND),
        S("7180c278b62e8f6a216a2aea45d08fc9", "2", "1", K.CLIENT, timestamp=(TODAY + 50) * 1000,
          duration=300 * 1000, local_endpoint=FRONTEND),
    ]
    case("getDependencies_strictTraceId", 98, [mixed], [(TRACE_ENDTS, DAY, [L("frontend", "backend", 1)])])
    case("replayOverwrites", 130, [TRACE, TRACE], [(TRACE_ENDTS, DAY, LINKS)])
    case("empty", 140, [], [(TRACE_ENDTS, DAY, [])])
    case("traceIdIsOpaque", 151, [[s.to_builder(trace_id="123") for s in TRACE]], [(TRACE_ENDTS, DAY, LINKS)])
    one = Endpoint.create("trace-producer-one", "127.0.0.1")
    two = Endpoint.create("trace-producer-two", "127.0.0.2")
    three = Endpoint.create("trace-producer-three", "127.0.0.3")
    case("getDependenciesAllInstrumented", 166, [[
        S("10", "10", None, K.SERVER, name="get", timestamp=TODAY * 1000, duration=350 * 1000, local_endpoint=one),
        S("10", "20", "10", K.CLIENT, name="get", timestamp=(TODAY + 50) * 1000, duration=250 * 1000,
          local_endpoint=one.to_builder(port=3001)),
        S("10", "20", "10", K.SERVER, name="get", shared=True, timestamp=(TODAY + 100) * 1000,
          duration=150 * 1000, local_endpoint=two),
        S("10", "30", "20", K.CLIENT, name="query", timestamp=(TODAY + 150) * 1000, duration=50 * 1000,
          local_endpoint=two.to_builder(port=3002)),
        S("10", "30", "20", K.SERVER, name="query", shared=True, timestamp=(TODAY + 160) * 1000,
          duration=20 * 1000, local_endpoint=three)]],
        [(TRACE_ENDTS, DAY, [L("trace-producer-one", "trace-producer-two", 1),
                             L("trace-producer-two", "trace-producer-three", 1)])])
    case("dependencies_loopback", 224,
         [[TRACE[0], TRACE[1].to_builder(remote_endpoint=TRACE[0].local_endpoint)]],
         [(TRACE_ENDTS, TRACE_DURATION, [L("frontend", "frontend", 1)])])
    case("dependencies_headlessTrace", 242, [TRACE[1:]], [(TRACE_ENDTS, DAY, LINKS)])
    case("looksBackIndefinitely", 252, [TRACE], [(TRACE_ENDTS, TRACE_ENDTS, LINKS)])
    case("endTsInsideTheTrace", 261, [TRACE], [(TRACE_STARTTS + 100, 200, LINKS)])
    case("endTimeBeforeData", 269, [TRACE], [(TRACE_STARTTS - 1000, 1000, [])])
    case("lookbackAfterData", 277, [TRACE], [(TODAY + 2 * DAY, DAY, [])])
    some_client = Endpoint.create("some-client", "172.17.0.4")
    case("notInstrumentedClientAndServer", 290, [[
        S("20", "20", None, K.SERVER, name="get", timestamp=TODAY * 1000, duration=350 * 1000,
          local_endpoint=FRONTEND, remote_endpoint=some_client),
        S("20", "21", "20", K.CLIENT, name="get", timestamp=(TODAY + 50) * 1000, duration=250 * 1000,
          local_endpoint=FRONTEND),
        S("20", "21", "20", K.SERVER, name="get", shared=True, timestamp=(TODAY + 250) * 1000,
          duration=50 * 1000, local_endpoint=BACKEND),
        S("20", "22", "21", K.CLIENT, name="get", timestamp=(TODAY + 150) * 1000, duration=50 * 1000,
          local_endpoint=BACKEND, remote_endpoint=DB)]],
        [(TRACE_ENDTS, DAY, [L("some-client", "frontend", 1), L("frontend", "backend", 1),
                             L("backend", "db", 1)])])
    case("instrumentedClientAndServer", 328, [[
        S("10", "10", None, K.CLIENT, name="get", timestamp=(TODAY + 50) * 1000, duration=250 * 1000,
          local_endpoint=FRONTEND),
        S("10", "10", None, K.SERVER, name="get", shared=True, timestamp=(TODAY + 100) * 1000,
          duration=150 * 1000, local_endpoint=BACKEND),
        S("10", "11", "10", K.CLIENT, name="get", timestamp=(TODAY + 150) * 1000, duration=50 * 1000,
          local_endpoint=BACKEND, remote_endpoint=DB)]],
        [(TRACE_ENDTS, DAY, [L("frontend", "backend", 1), L("backend", "db", 1)])])
    many = []
    for i in range(1, 1001):
        web = FRONTEND.to_builder(service_name=f"web-{i}")
        app = BACKEND.to_builder(service_name=f"app-{i}")
        db = DB.to_builder(service_name=f"db-{i}")
        tid = format(i, "x")
        many += [
            S(tid, "10", None, K.CLIENT, name="get", timestamp=(TODAY + 50) * 1000, duration=250 * 1000,
              local_endpoint=web),
            S(tid, "10", None, K.SERVER, name="get", shared=True, timestamp=(TODAY + 100) * 1000,
              duration=150 * 1000, local_endpoint=app),
            S(tid, "11", "10", K.CLIENT, name="get", timestamp=(TODAY + 150) * 1000, duration=50 * 1000,
              local_endpoint=app, remote_endpoint=db)]
    case("manyLinks", 358, [many], [(TRACE_ENDTS, DAY, {"size": 2000, "all_call_count": 1})])
    case("missingIntermediateSpan", 398, [[
        S("20", "20", None, K.SERVER, name="get", timestamp=TODAY * 1000, duration=350 * 1000,
          local_endpoint=FRONTEND),
        S("20", "22", "21", K.CLIENT, name="get", timestamp=(TODAY + 150) * 1000, duration=50 * 1000,
          local_endpoint=BACKEND)]],
        [(TRACE_ENDTS, DAY, [L("frontend", "backend", 1)])])

    def subtract_day(trace):  # ITDependencies.subtractDay (:680-690), random id frozen
        out = []
        for s in trace:
            ch = {"trace_id": SUBTRACT_DAY_TRACE_ID}
            if s.timestamp:
                ch["timestamp"] = s.timestamp - DAY * 1000
            ch["annotations"] = tuple(sorted(set(s.annotations) | {(t - DAY * 1000, v) for t, v in s.annotations}))
            out.append(s.to_builder(**ch))
        return out

    case("canSearchForIntervalsBesidesToday", 425, [subtract_day(TRACE), TRACE], [
        (TRACE_ENDTS, TRACE_DURATION, LINKS),
        (TRACE_ENDTS - DAY, DAY, LINKS),
        (TRACE_ENDTS, TRACE_ENDTS, [L("frontend", "backend", 2), L("backend", "db", 2, 2)])])
    case("spanKindIsNotRequiredWhenEndpointsArePresent", 448, [[
        S("20", "20", None, None, name="get", timestamp=TODAY * 1000, duration=350 * 1000,
          local_endpoint=some_client, remote_endpoint=FRONTEND),
        S("20", "21", "20", None, name="get", timestamp=(TODAY + 50) * 1000, duration=250 * 1000,
          local_endpoint=FRONTEND, remote_endpoint=BACKEND),
        S("20", "22", "21", None, name="get", timestamp=(TODAY + 150) * 1000, duration=50 * 1000,
          local_endpoint=BACKEND, remote_endpoint=DB)]],
        [(TODAY + 1000, 1000, [L("some-client", "frontend", 1), L("frontend", "backend", 1),
                              L("backend", "db", 1)])])
    case("unnamedEndpointsAreSkipped", 476, [[
        S("20", "20", None, None, name="get", timestamp=TODAY * 1000, duration=350 * 1000,
          local_endpoint=Endpoint.create(None, "172.17.0.4"), remote_endpoint=FRONTEND),
        S("20", "21", "20", None, name="get", timestamp=(TODAY + 50) * 1000, duration=250 * 1000,
          local_endpoint=FRONTEND, remote_endpoint=BACKEND),
        S("20", "22", "21", None, name="get", timestamp=(TODAY + 150) * 1000, duration=50 * 1000,
          local_endpoint=BACKEND, remote_endpoint=DB)]],
        [(TODAY + 1000, 1000, [L("frontend", "backend", 1), L("backend", "db", 1)])])
    case("intermediateSpans", 508, [[
        S("20", "20", None, K.SERVER, name="get", timestamp=TODAY * 1000, duration=350 * 1000,
          local_endpoint=FRONTEND),
        S("20", "21", "20", None, name="call", timestamp=(TODAY + 25) * 1000, duration=325 * 1000,
          local_endpoint=FRONTEND),
        S("20", "22", "21", K.CLIENT, name="get", timestamp=(TODAY + 50) * 1000, duration=250 * 1000,
          local_endpoint=FRONTEND),
        S("20", "22", "21", K.SERVER, name="get", timestamp=(TODAY + 100) * 1000, duration=150 * 1000,
          shared=True, local_endpoint=BACKEND),
        S("20", 23, "22", None, name="depth4", timestamp=(TODAY + 110) * 1000, duration=130 * 1000,
          local_endpoint=BACKEND),
        S("20", 24, 23, None, name="depth5", timestamp=(TODAY + 125) * 1000, duration=105 * 1000,
          local_endpoint=BACKEND),
        S("20", 25, 24, K.CLIENT, name="get", timestamp=(TODAY + 150) * 1000, duration=50 * 1000,
          local_endpoint=BACKEND, remote_endpoint=DB)]],
        [(TODAY + 1000, 1000, [L("frontend", "backend", 1), L("backend", "db", 1)])])
    # duplicateAddress (:555): the two V1 spans as V1SpanConverter emits them
    # (v1/V1SpanConverter.java:61-273): span 20 = SERVER on FRONTEND, its "ca"
    # equals the server endpoint so no remote is set (:252); span 22 = CLIENT on
    # FRONTEND with remote "sa" = BACKEND (:260-262).
    case("duplicateAddress", 555, [[
        S("20", "20", None, K.SERVER, name="get", timestamp=TODAY * 1000, duration=350 * 1000,
          local_endpoint=FRONTEND),
        S("20", "22", "21", K.CLIENT, name="get", timestamp=(TODAY + 50) * 1000, duration=250 * 1000,
          local_endpoint=FRONTEND, remote_endpoint=BACKEND)]],
        [(TODAY + 1000, 1000, [L("frontend", "backend", 1)])])
    case("oneway", 583, [[
        S("10", "10", None, K.CLIENT, timestamp=(TODAY + 50) * 1000, local_endpoint=FRONTEND),
        S("10", "10", None, K.SERVER, shared=True, timestamp=(TODAY + 100) * 1000, local_endpoint=BACKEND)]],
        [(TRACE_ENDTS, TRACE_DURATION, [L("frontend", "backend", 1)])])
    case("annotationNamedErrorIsntError", 606, [[
        S("10", "10", None, K.CLIENT, timestamp=(TODAY + 50) * 1000, local_endpoint=FRONTEND),
        S("10", "10", None, K.SERVER, shared=True, timestamp=(TODAY + 100) * 1000, local_endpoint=BACKEND,
          annotations=(((TODAY + 72) * 1000, "error"),))]],
        [(TRACE_ENDTS, TRACE_DURATION, [L("frontend", "backend", 1)])])
    kafka = Endpoint.create("kafka", "172.17.0.4")
    case("oneway_noClient", 630, [[
        S("10", "10", None, K.SERVER, name="receive", timestamp=TODAY * 1000, local_endpoint=BACKEND,
          remote_endpoint=kafka),
        S("10", "11", "10", None, name="process", timestamp=(TODAY + 25) * 1000, duration=325 * 1000,
          local_endpoint=BACKEND)]],
        [(TRACE_ENDTS, DAY, [L("kafka", "backend", 1)])])
    rs = S("10", "10", None, K.CONSUMER, name="receive", local_endpoint=Endpoint.create("app"),
           remote_endpoint=Endpoint.create("kafka"), timestamp=TODAY * 1000)
    case("replayOverwrites", 92, [[rs], [rs]], [(TODAY + 1000, TODAY, [L("kafka", "app", 1)])],
         source="InMemoryStorageTest")
    return {"source": "zipkin/src/test/java/zipkin2/storage/ITDependencies.java (+ TestObjects.java, "
                      "InMemoryStorageTest.java)", "today": TODAY, "cases": cases}


def main():
    out = {
        "dependency_linker.json": dependency_linker_cases(),
        "span_node.json": span_node_cases(),
        "trace_merge.json": trace_merge_cases(),
        "storage_dependencies.json": storage_cases(),
    }
    for name, data in out.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, indent=None if name.startswith("storage") else 1, ensure_ascii=False)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
