"""Insertion-order parity (ZDL_FLAG_INSERTION_ORDER): ``link()`` returns the links in
the order the reference's ``DependencyLinker.link()`` does — the LinkedHashMap
insertion order of ``addLink`` (DependencyLinker.java:166-186) over the traces in put
order, each trace tree breadth-first (SpanNode.java:64-89) with children in
spanToParent entry order (SpanNode.java:150-159).

Compared as exact lists against the oracles, which keep that order (oracle/dl_oracle.py
with LinkedHashMap = ordered dict, oracle/dl_ref.cpp), and against the reference's own
``containsExactly`` vectors (DependencyLinkerTest.java:59,565,579).
"""
import random

import numpy as np
import pytest

from oracle import dl_oracle as O
from oracle import ref
from tests.golden_io import check_links, load, spans
from tests.stress import random_trace
from zipkin_amd import _native as N
from zipkin_amd import synth
from zipkin_amd.columnar import Columns, Dictionary, pack_traces
from zipkin_amd.linker import DependencyLinker
from zipkin_amd.model import Kind, span2

pytestmark = pytest.mark.gpu

DL = load("dependency_linker.json")


def as_list(ls):
    return [(l.parent, l.child, l.call_count, l.error_count) for l in ls]


@pytest.mark.parametrize("case", [c for c in DL["cases"] if c["mode"] == "exact"], ids=lambda c: c["name"])
def test_golden_contains_exactly(case):
    linker = DependencyLinker()
    for t in case["traces"]:
        linker.put_trace(spans(t))
    check_links(linker.link(), case["expect"], "exact")
    linker.close()


@pytest.mark.parametrize("case", [c for c in DL["cases"] if c["mode"] != "log"], ids=lambda c: c["name"])
def test_golden_cases_in_oracle_order(case):
    ol, gl = O.DependencyLinker(), DependencyLinker()
    for t in case["traces"]:
        ol.put_trace(spans(t))
        gl.put_trace(spans(t))
    assert as_list(gl.link()) == as_list(ol.link())
    gl.close()


@pytest.mark.parametrize("seed", range(200))
def test_random_traces_order_vs_python_oracle(seed):
    r = random.Random(5000 + seed)
    traces = [random_trace(r) for _ in range(r.randint(1, 6))]
    ol = O.DependencyLinker()
    try:
        for t in traces:
            ol.put_trace(t)
        expect = as_list(ol.link())
    except O.ReferenceNPE:
        expect = "NPE"
    gl = DependencyLinker()
    if expect == "NPE":
        with pytest.raises(N.ReferenceNullPointerException):
            gl.put_traces(traces)
    else:
        # half the seeds put trace by trace (many puts), half in one batch
        if seed % 2:
            for t in traces:
                gl.put_trace(t)
        else:
            gl.put_traces(traces)
        assert as_list(gl.link()) == expect
    gl.close()


def _ordered_vs_cpp(cols, n_services, window=None, svc_rank=None, ip4_rank=None, ip6_rank=None, splits=1):
    ctx = N.Context(n_services, insertion_order=True)
    for d, r in ((N.ZDL_DICT_SERVICE, svc_rank), (N.ZDL_DICT_IPV4, ip4_rank), (N.ZDL_DICT_IPV6, ip6_rank)):
        if r is not None:
            ctx.set_ranks(d, r)
    if window is not None:
        ctx.set_window(*window)
    for part in _split(cols, splits):
        ctx.put_spans(part)
    p, c, n, e = ctx.link(N.ZDL_ORDER_INSERTION)
    sp, sc, sn, se = ctx.link(N.ZDL_ORDER_SORTED)
    ctx.close()
    st, op, oc, on, oe = ref.link(cols, svc_rank, ip4_rank, ip6_rank, window=window, threads=8)
    assert st == 0
    got = list(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))
    exp = list(zip(op.tolist(), oc.tolist(), on.tolist(), oe.tolist()))
    assert got == exp
    assert sorted(got) == sorted(zip(sp.tolist(), sc.tolist(), sn.tolist(), se.tolist()))
    return got


def _split(cols, k):
    """k consecutive puts of whole traces."""
    if k == 1:
        yield cols
        return
    off = cols.offsets.astype(np.int64)
    cut = [cols.n_traces * i // k for i in range(k + 1)]
    f = ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags",
         "timestamp")
    for a, b in zip(cut[:-1], cut[1:]):
        s0, s1 = off[a], off[b]
        yield Columns(*(np.ascontiguousarray(getattr(cols, n)[s0:s1]) for n in f),
                      (off[a:b + 1] - s0).astype(np.uint64))


def test_random_batch_order_vs_cpp_oracle():
    r = random.Random(77)
    traces = [random_trace(r, n=r.randint(1, 40), allow_npe=False) for _ in range(2000)]
    svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
    cols = pack_traces(traces, svc, ip4, ip6)
    _ordered_vs_cpp(cols, 64, svc_rank=svc.ranks(), ip4_rank=ip4.ranks(), ip6_rank=ip6.ranks(), splits=3)


def test_big_traces_order_vs_cpp_oracle():
    """Traces longer than 64 spans: breadth-first order by the big-trace kernel's frontier."""
    r = random.Random(11)
    traces = [random_trace(r, n=r.choice([65, 129, 300, 1000, 4097]), allow_npe=False,
                           id_pool=r.choice([50, 2000])) for _ in range(16)]
    traces += [random_trace(r, n=r.randint(1, 20), allow_npe=False) for _ in range(100)]
    r.shuffle(traces)
    svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
    cols = pack_traces(traces, svc, ip4, ip6)
    _ordered_vs_cpp(cols, 64, svc_rank=svc.ranks(), ip4_rank=ip4.ranks(), ip6_rank=ip6.ranks())


def test_trace_beyond_2_21_spans_order_vs_cpp_oracle():
    """One trace of 2^21 + 1 spans between small ones (round 5 refused traces of 2^21 - 1 spans
    or more: big_bfs packed its sort keys in 21-bit fields, the ranks in 24): the breadth-first
    order comes from wide keys, the ranks are (position + index) << 1 | k."""
    from zipkin_amd.columnar import concat_columns
    huge = synth.generate(synth.Workload("huge", 0x5EED0A21, 1, 50, max_depth=64, size_dist=2,
                                         max_size=(1 << 21) + 1, max_fanout=1000))
    assert huge.n_spans == (1 << 21) + 1
    small = synth.generate(synth.C2.scaled(20_000))
    cols = concat_columns([_first(small, 10_000), huge, _rest(small, 10_000)])
    assert len(_ordered_vs_cpp(cols, 64)) > 100


def _first(cols, k):
    return next(_split_at(cols, k))


def _rest(cols, k):
    it = _split_at(cols, k)
    next(it)
    return next(it)


def _split_at(cols, k):
    off = cols.offsets.astype(np.int64)
    f = ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags",
         "timestamp")
    for a, b in ((0, k), (k, cols.n_traces)):
        s0, s1 = off[a], off[b]
        yield Columns(*(np.ascontiguousarray(getattr(cols, n)[s0:s1]) for n in f),
                      (off[a:b + 1] - s0).astype(np.uint64))


@pytest.mark.parametrize("n_services", [64, 300])
def test_c2_order_vs_cpp_oracle(n_services):
    w = synth.C2.scaled(100_000)
    cols = synth.generate(w)
    assert len(_ordered_vs_cpp(cols, max(n_services, w.total_services), splits=2)) > 100


def test_c4_messaging_order_vs_cpp_oracle():
    w = synth.C4.scaled(100_000)
    _ordered_vs_cpp(synth.generate(w), w.total_services)


def test_c5_high_cardinality_order_vs_cpp_oracle():
    w = synth.C5.scaled(20_000)
    w = synth.Workload(**{**w.__dict__, "max_size": 5_000})
    _ordered_vs_cpp(synth.generate(w), w.total_services)


def test_window_order_vs_cpp_oracle():
    w = synth.C2.scaled(50_000)
    base_ms = w.base_ts_us // 1000
    _ordered_vs_cpp(synth.generate(w), w.total_services, window=(base_ms + 66_000, 33_000))


def test_context_growth_keeps_order():
    """The facade re-creates the context with a larger table (zdl_add_links carries the
    links over, ranked before later puts); the order must survive."""
    r = random.Random(4)
    svcs = [f"svc{i:03d}" for i in range(120)]
    traces = []
    for t in range(300):
        tid = format(t + 1, "016x")
        a, b, c = r.sample(svcs, 3)
        traces.append([span2(tid, None, "1", Kind.SERVER, a, None, False),
                       span2(tid, "1", "2", Kind.CLIENT, a, b, r.random() < 0.2),
                       span2(tid, "1", "2", Kind.SERVER, b, a, False).to_builder(shared=True),
                       span2(tid, "2", "3", Kind.CLIENT, b, c, False)])
    ol, gl = O.DependencyLinker(), DependencyLinker()
    for i in range(0, len(traces), 50):
        for t in traces[i:i + 50]:
            ol.put_trace(t)
        gl.put_traces(traces[i:i + 50])
    assert as_list(gl.link()) == as_list(ol.link())
    gl.close()


def test_insertion_order_needs_the_flag_and_reset_clears_ranks():
    w = synth.C2.scaled(5_000)
    cols = synth.generate(w)
    ctx = N.Context(w.total_services)
    ctx.put_spans(cols)
    with pytest.raises(N.ZdlError):
        ctx.link(N.ZDL_ORDER_INSERTION)
    ctx.close()
    ctx = N.Context(w.total_services, insertion_order=True)
    ctx.put_spans(cols)
    a = ctx.link(N.ZDL_ORDER_INSERTION)
    ctx.reset()
    assert len(ctx.link(N.ZDL_ORDER_INSERTION)[0]) == 0
    ctx.put_spans(cols)
    b = ctx.link(N.ZDL_ORDER_INSERTION)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    ctx.close()


def test_link_between_puts_and_after_add_links():
    """The insertion-order compaction is queued at each put's end (round 6): a link after every
    put sees every put so far, a second link without a put returns the same list, and a table
    changed by zdl_add_links is compacted again (the put's compaction is stale then)."""
    from zipkin_amd.columnar import concat_columns
    w = synth.C2.scaled(30_000)
    cols = synth.generate(w)
    parts = list(_split(cols, 3))
    ctx = N.Context(w.total_services, insertion_order=True)
    try:
        for k in range(1, 4):
            ctx.put_spans(parts[k - 1])
            got = ctx.link(N.ZDL_ORDER_INSERTION)
            st, op, oc, on, oe = ref.link(concat_columns(parts[:k]), threads=8)
            assert st == 0
            exp = list(zip(op.tolist(), oc.tolist(), on.tolist(), oe.tolist()))
            assert list(zip(*(a.tolist() for a in got))) == exp
            again = ctx.link(N.ZDL_ORDER_INSERTION)
            assert list(zip(*(a.tolist() for a in again))) == exp
        p, c, n, e = (np.asarray(a[:5]) for a in got)
        ctx.add_links(p, c, np.ones(5, np.int64), np.zeros(5, np.int64))
        bumped = ctx.link(N.ZDL_ORDER_INSERTION)
        want = [(a, b, x + (1 if i < 5 else 0), y) for i, (a, b, x, y) in enumerate(exp)]
        assert list(zip(*(a.tolist() for a in bumped))) == want
    finally:
        ctx.close()
