"""mysql-v1 row projection + aggregation: the oracle restatement pinned by all
13 DependencyLinkV2SpanIteratorTest cases (CPU), and zdl_put_mysql_rows checked against it on
the GPU (links in DependencyLinker.link() order)."""
import random

import pytest

from oracle import mysql_oracle as M
from oracle.dl_oracle import DependencyLinker as OracleLinker
from zipkin_amd.model import Kind

B, S = 0, 6  # V1BinaryAnnotation.TYPE_BOOLEAN, TYPE_STRING


def rec(key, typ, svc, trace=1, parent=None, span=1, hi=None):
    return (hi, trace, parent, span, key, typ, svc)


# (name, rows, expected kind, local service, remote service, tags) from DependencyLinkV2SpanIteratorTest
CASES = [
    ("whenNoServiceLabelsExist_kindIsUnknown", [rec("cs", -1, None)], None, None, None, ()),
    ("whenOnlyAddressLabelsExist_kindIsNull", [rec("ca", B, "s1"), rec("sa", B, "s2")], None, "s1", "s2", ()),
    ("whenServerLabelsAreMissing_kindIsUnknownAndLabelsAreCleared", [rec("ca", B, "s1")], None, None, None, ()),
    ("whenSrServiceExists_kindIsServer", [rec("sr", -1, "service")], Kind.SERVER, "service", None, ()),
    ("errorAnnotationIgnored", [rec("error", -1, "service")], None, None, None, ()),
    ("errorTagAdded", [rec("error", S, "foo")], None, None, None, (("error", ""),)),
    ("whenSrAndCaServiceExists_caIsThePeer", [rec("ca", B, "s1"), rec("sr", -1, "s2")], Kind.SERVER, "s2", "s1", ()),
    ("whenSrAndCsServiceExists_caIsThePeer", [rec("cs", -1, "s1"), rec("sr", -1, "s2")], Kind.SERVER, "s2", "s1", ()),
    ("whenCrAndCaServiceExists_caIsThePeer", [rec("cs", -1, "foo"), rec("ca", B, "s1"), rec("sr", -1, "s2")],
     Kind.SERVER, "s2", "s1", ()),
    ("specialCasesFinagleLocalSocketLabeling_client",
     [rec("cs", -1, "service"), rec("ca", B, "service"), rec("sa", B, "service")], Kind.CLIENT, None, "service", ()),
    ("specialCasesFinagleLocalSocketLabeling_server",
     [rec("ca", B, "service"), rec("sa", B, "service"), rec("sr", -1, "service")], Kind.SERVER, "service", None, ()),
    ("csWithoutSaIsServer", [rec("cs", -1, "s1")], Kind.SERVER, "s1", None, ()),
    ("emptyToNull", [rec("ca", B, ""), rec("cs", -1, ""), rec("sa", B, ""), rec("sr", -1, "")], None, None, None, ()),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
def test_oracle_iterator_cases(case):
    _, rows, kind, local, remote, tags = case
    (span,), = M.traces(rows)
    assert span.kind == kind
    assert span.local_service_name == local
    assert span.remote_service_name == remote
    assert span.tags == tags
    assert span.annotations == ()


def test_oracle_groups_by_low_trace_id_only():
    rows = [rec("sr", -1, "a", trace=5, hi=1, span=1), rec("sr", -1, "b", trace=5, hi=2, span=2),
            rec("sr", -1, "c", trace=6, span=3)]
    ts = M.traces(rows)
    assert [len(t) for t in ts] == [2, 1]
    assert ts[0][1].trace_id == ts[0][0].trace_id  # ByTraceId keeps the first row's high bits


def with_root(rows):
    """The case's span under a server root of another service, so its projection shows in links."""
    root = rec("sr", -1, "root", span=9)
    return [root] + [(h, t, 9, s, k, ty, v) for (h, t, p, s, k, ty, v) in rows]


SVCS = ["web", "Web", "app", "db", "kafka", "", None]


def rand_rows(r, n_traces):
    rows = []
    for t in range(n_traces):
        lo = r.randrange(1, 1 << 63)
        his = [None, r.randrange(1, 1 << 63)]
        ids = [r.randrange(1, 1 << 63) for _ in range(r.randrange(1, 8))]
        for k, sid in enumerate(ids):
            parent = None if k == 0 else r.choice(ids[:k] + [r.randrange(1, 99)])
            for _ in range(r.randrange(0, 5) or 1):
                key = r.choice(["lc", "ca", "cs", "sa", "sr", "error", "ss", None])
                rows.append((r.choice(his), lo, parent, sid, key, r.choice([-1, B, S]), r.choice(SVCS)))
    return rows


def as_tuples(links):
    return [(l.parent, l.child, l.call_count, l.error_count) for l in links]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
def test_gpu_iterator_cases_under_a_root(case):
    from zipkin_amd.linker import aggregate_dependencies
    rows = with_root(case[1])
    assert as_tuples(aggregate_dependencies(rows)) == as_tuples(M.aggregate_dependencies(rows))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(20))
def test_gpu_random_rows_vs_oracle(seed):
    from zipkin_amd.linker import aggregate_dependencies
    r = random.Random(seed)
    rows = rand_rows(r, r.randrange(1, 300))
    assert as_tuples(aggregate_dependencies(rows)) == as_tuples(M.aggregate_dependencies(rows))


@pytest.mark.gpu
def test_gpu_rows_accumulate_with_put_trace():
    """Rows and ordinary putTrace calls count into the same linker, in put order."""
    from zipkin_amd.linker import DependencyLinker
    from zipkin_amd.model import Endpoint, Span
    r = random.Random(77)
    rows = rand_rows(r, 50)
    extra = [Span.create("abc", 1, None, Kind.SERVER, local_endpoint=Endpoint.create("web")),
             Span.create("abc", 2, 1, Kind.CLIENT, local_endpoint=Endpoint.create("web"),
                         remote_endpoint=Endpoint.create("db"))]
    gl = DependencyLinker().put_mysql_rows(rows).put_trace(extra)
    ol = OracleLinker()
    for t in M.traces(rows):
        ol.put_trace(t)
    ol.put_trace(extra)
    assert as_tuples(gl.link()) == as_tuples(ol.link())
    gl.close()
