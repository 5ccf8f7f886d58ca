"""The tree each benchmarked kernel builds, not only its links: ZDL_FLAG_TREE_STREAM exports,
per span, the node / parent / visited flag (the traverse index on an insertion-order context)
and firstRemoteAncestor that the path which linked the span computed - k_link's windows
(lk_window, modes 0 and 4), k_mid (wave_big), k_tail's big_simple, the giant tier and the exact
paths - without sending any trace to the exact path. Compared with SpanNode.Builder restated
(oracle/dl_oracle.py; SpanNode.java:122-249, traverse SpanNode.java:64-89,
DependencyLinker.firstRemoteAncestor DependencyLinker.java:153-164) on every SpanNodeTest case
(SpanNodeTest.java:59-297) and on random traces. A wrong parent that happens to give the same
links fails here."""
import random

import numpy as np
import pytest

from oracle import dl_oracle as O
from tests.golden_io import load, spans
from tests.stress import random_trace
from zipkin_amd import _native as N
from zipkin_amd.columnar import Dictionary, pack_traces
from zipkin_amd.model import Endpoint, Kind, Span

pytestmark = pytest.mark.gpu

SN = load("span_node.json")


def _oracle_tree(trace, ordered):
    """{head input index: (parent head | -1 synthetic root | -2 root, traverse index or 0,
    firstRemoteAncestor's head | -1)} over the nodes SpanNode.traverse visits."""
    cleaned, sources = O.trace_merge_sources(trace)
    head_of = {id(s): src[0] for s, src in zip(cleaned, sources)}
    root = O.SpanNodeBuilder().build(trace, cleaned)
    out, k = {}, 0
    for n in root.traverse():
        if n.span is None:
            continue
        par = -2 if n.parent is None else (-1 if n.parent.span is None else head_of[id(n.parent.span)])
        a = n.parent
        while a is not None and (a.span is None or a.span.kind is None):
            a = a.parent
        out[head_of[id(n.span)]] = (par, k if ordered else 0, head_of[id(a.span)] if a is not None else -1)
        k += 1
    return out


def _device_trees(traces, ordered, n_services=None):
    svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
    cols = pack_traces(traces, svc, ip4, ip6)
    ctx = N.Context(n_services or max(64, len(svc)), insertion_order=ordered, tree_stream=True)
    ctx.set_ranks(N.ZDL_DICT_SERVICE, svc.ranks())
    ctx.set_ranks(N.ZDL_DICT_IPV4, ip4.ranks())
    ctx.set_ranks(N.ZDL_DICT_IPV6, ip6.ranks())
    ctx.put_spans(cols)
    node, par, bfs = ctx.tree_export(cols.n_spans)
    _, anc, _, _ = ctx.tree_reasons(cols.n_spans)
    ctx.close()
    out = []
    off = cols.offsets.astype(np.int64)
    for t in range(cols.n_traces):
        b, e = off[t], off[t + 1]
        got = {}
        for i in range(b, e):
            assert b <= node[i] < e, "every span's node is recorded"
            if node[i] != i or bfs[i] < 0:  # an absorbed fragment, or not visited
                continue
            rel = lambda x: int(x) - b if x >= 0 else int(x)  # noqa: E731
            got[i - b] = (rel(par[i]), int(bfs[i]), rel(anc[i]))
        out.append(got)
    return out


def _simple_trace(r, n):
    """A simple trace (per id at most one non-shared and one shared span): a random tree with
    shared client/server pairs, local spans, messaging, some missing parents; shuffled."""
    svcs = ["web", "app", "db", "cache", "queue", "auth"]
    ids = iter(r.sample(range(1, 2 ** 62), 2 * n + 2))
    out = []
    nodes = []  # (id, service)
    while len(out) < n:
        if not nodes:
            sid, s = next(ids), r.choice(svcs)
            out.append(Span.create("b" * 16, format(sid, "016x"), None, Kind.SERVER,
                                   local_endpoint=Endpoint.create(s, None, 0)))
            nodes.append((sid, s))
            continue
        pid, ps = r.choice(nodes)
        if r.random() < 0.03:
            pid = next(ids)  # a parent that is not in the trace
        callee = r.choice(svcs)
        kind = r.choice([Kind.CLIENT, Kind.CLIENT, None, Kind.PRODUCER])
        sid = next(ids)
        err = {"error": ""} if r.random() < 0.1 else None
        rem = Endpoint.create(callee, None, 0) if kind is not None or r.random() < 0.3 else None
        out.append(Span.create("b" * 16, format(sid, "016x"), format(pid, "016x"), kind,
                               local_endpoint=Endpoint.create(ps, None, 0), remote_endpoint=rem, tags=err))
        nodes.append((sid, ps))
        if kind == Kind.CLIENT and len(out) < n:
            if r.random() < 0.7:  # the server side shares the client's id
                out.append(Span.create("b" * 16, format(sid, "016x"), format(pid, "016x") if r.random() < 0.8
                                       else None, Kind.SERVER, local_endpoint=Endpoint.create(callee, None, 0),
                                       remote_endpoint=Endpoint.create(ps, None, 0), shared=True))
            else:
                cid = next(ids)
                out.append(Span.create("b" * 16, format(cid, "016x"), format(sid, "016x"), Kind.SERVER,
                                       local_endpoint=Endpoint.create(callee, None, 0)))
                nodes.append((cid, callee))
        elif kind == Kind.PRODUCER and len(out) < n:
            cid = next(ids)
            out.append(Span.create("b" * 16, format(cid, "016x"), format(sid, "016x"), Kind.CONSUMER,
                                   local_endpoint=Endpoint.create(callee, None, 0),
                                   remote_endpoint=Endpoint.create("kafka", None, 0) if r.random() < 0.8 else None))
            nodes.append((cid, callee))
    r.shuffle(out)
    return out


@pytest.mark.parametrize("ordered", [False, True], ids=["sorted", "insertion"])
@pytest.mark.parametrize("case", SN["cases"], ids=lambda c: c["name"])
def test_golden_span_node_tree_stream(case, ordered):
    inputs = spans(case["spans"])
    assert _device_trees([inputs], ordered)[0] == _oracle_tree(inputs, ordered)


@pytest.mark.parametrize("ordered", [False, True], ids=["sorted", "insertion"])
@pytest.mark.parametrize("seed", range(6))
def test_simple_windows(seed, ordered):
    """Simple traces of <= 64 spans: every window is linked (and its tree built) in k_link."""
    r = random.Random(9100 + seed)
    traces = [_simple_trace(r, r.randint(1, 40)) for _ in range(300)]
    for t, g in zip(traces, _device_trees(traces, ordered)):
        assert g == _oracle_tree(t, ordered)


@pytest.mark.parametrize("ordered", [False, True], ids=["sorted", "insertion"])
@pytest.mark.parametrize("seed", range(4))
def test_random_corner_traces(seed, ordered):
    """Random parents (cycles, missing parents, duplicate roots), shared ids, fragments: windows
    that are not simple are exported by k_tail's exact path."""
    r = random.Random(9200 + seed)
    traces = [random_trace(r, n=r.randint(1, 40), allow_npe=False, id_pool=r.choice([3, 6, 20, 400]))
              for _ in range(60)]
    for t, g in zip(traces, _device_trees(traces, ordered)):
        assert g == _oracle_tree(t, ordered)


@pytest.mark.parametrize("tier", ["wave_big", "big_simple", "giant"])
def test_big_simple_traces(tier, monkeypatch):
    """Traces above 64 spans on a sorted context: k_mid's wave_big (<= 192 spans), k_tail's
    big_simple (LDS and HBM), and the giant tier (sparse context, ZDL_GIANT_MIN=192)."""
    r = random.Random({"wave_big": 9301, "big_simple": 9302, "giant": 9303}[tier])
    sizes = {"wave_big": [70, 120, 190], "big_simple": [300, 1500, 4000], "giant": [300, 2500, 6000]}[tier]
    if tier == "giant":
        monkeypatch.setenv("ZDL_SPARSE", "1")
        monkeypatch.setenv("ZDL_GIANT_MIN", "192")
    traces = [_simple_trace(r, n) for n in sizes] + [_simple_trace(r, r.randint(1, 30)) for _ in range(20)]
    traces += [random_trace(r, n=r.choice([100, 500]), allow_npe=False, id_pool=10 ** 6) for _ in range(3)]
    for t, g in zip(traces, _device_trees(traces, False)):
        assert g == _oracle_tree(t, False)
