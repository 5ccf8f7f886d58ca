"""The device-wide big-trace tier (zipkin_amd/csrc/zdl_giant.inc, sparse contexts) against the
C++ restatement (oracle/dl_ref.cpp) and against k_tail's one-workgroup-per-trace path
(ZDL_GIANT_MIN=0), bit-exact on every (parent, child, callCount, errorCount).

The tier must give DependencyLinker.putTrace's result (DependencyLinker.java:53-151 over
SpanNode.Builder, SpanNode.java:122-249) for any trace it takes, and hand every trace it
cannot link exactly to k_tail's exact path:

* C5-shaped bodies with unclipped giants (60k-190k spans, depth 64, fan-out <= 1000), at the
  default threshold and with every trace above WB_MAX in the tier;
* a time window that cuts the giants (QueryRequest.test per trace);
* duplicate (id, shared) spans (quirk Q2: not simple, exact path), self parents, a two-span
  cycle (an unreachable subtree, as in SpanNode.traverse);
* ids crafted so that one join bucket overflows its LDS hash (exact path);
* C4's faults (split spans, missing brokers, extra roots) in traces of 200-3000 spans.
"""

import numpy as np
import pytest

from oracle import ref
from zipkin_amd import _native as N
from zipkin_amd import synth
from zipkin_amd.columnar import Columns, concat_columns

pytestmark = pytest.mark.gpu

FIELDS = ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags",
          "timestamp")


def _tuples(p, c, n, e):
    return list(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))


def _oracle(cols, window=None):
    st, p, c, n, e = ref.link(cols, window=window, threads=16) if window else ref.link(cols, threads=16)
    assert st == 0
    return sorted(_tuples(p, c, n, e))


def _link(cols, S, window=None):
    ctx = N.Context(S)
    if window:
        ctx.set_window(*window)
    ctx.put_spans(cols)
    got = sorted(_tuples(*ctx.link()))
    ctx.close()
    return got


def _giant(seed, size, services=10_000):
    g = synth.Workload(f"giant_{seed}", 0x5EED0900 + seed, 1, services, max_depth=64, size_dist=2, max_size=size,
                       max_fanout=1000, zipf_s=1.1)
    return synth.generate(g)


def _copy(cols):
    return Columns(*(np.array(getattr(cols, f)) for f in FIELDS), np.array(cols.offsets))


def _body_with_giants(traces=200_000, sizes=(60_000, 120_000, 190_000)):
    body = synth.generate(synth.C5.scaled(traces))
    parts = []
    h = body.n_traces // 2
    for k, size in enumerate(sizes):
        parts.append(_giant(k, size))
        if k == 0:
            parts.append(_slice(body, 0, h))
        elif k == 1:
            parts.append(_slice(body, h, body.n_traces))
    return concat_columns(parts)


def _slice(cols, t0, t1):
    a, b = int(cols.offsets[t0]), int(cols.offsets[t1])
    return Columns(*(np.ascontiguousarray(getattr(cols, n)[a:b]) for n in FIELDS),
                   np.ascontiguousarray(cols.offsets[t0:t1 + 1] - np.uint64(a)))


@pytest.mark.parametrize("gmin", ["2048", "192", "0"])
def test_c5_giants_tiers_vs_cpp(gmin, monkeypatch):
    monkeypatch.setenv("ZDL_GIANT_MIN", gmin)
    cols = _body_with_giants()
    sizes = np.diff(cols.offsets.astype(np.int64))
    assert (sizes > 2048).sum() > 10 and sizes.max() >= 150_000
    assert _link(cols, 10_000) == _oracle(cols)


def test_giants_beyond_a_million_spans_vs_cpp():
    """Traces of 1.5M and 3M spans (beyond round 5's 2^20-span tier limit; the tier now takes up
    to 2^22 spans, 4096 tiles and buckets) are linked by the whole GPU: bit-exact vs the
    restatement, and the tier (not k_tail's one workgroup) ran them."""
    parts = [_giant(50, 1_500_000), _slice(synth.generate(synth.C5.scaled(20_000)), 0, 20_000), _giant(51, 3_000_000)]
    cols = concat_columns(parts)
    sizes = np.diff(cols.offsets.astype(np.int64))
    assert sizes.max() >= 2_900_000 and (sizes > (1 << 20)).sum() == 2
    ctx = N.Context(10_000, timing_all=True)
    ctx.put_spans(cols)
    got = sorted(_tuples(*ctx.link()))
    kt = ctx.kernel_times()
    ctx.close()
    assert got == _oracle(cols)
    assert kt.giant_ms > 0


def test_c5_giants_window_vs_cpp(monkeypatch):
    """The window filters whole traces by QueryRequest.test's rule (first parentless span's
    timestamp, else the smallest); giants are stamped at different times so some fall out."""
    monkeypatch.setenv("ZDL_GIANT_MIN", "192")
    parts = [_giant(10 + k, 3000 + 5000 * k) for k in range(6)]
    for k, p in enumerate(parts):
        p.timestamp[:] = np.where(p.timestamp != 0, np.int64(1_700_000_000_000_000 + k * 10_000_000), 0)
        if k == 2:  # no parentless span carries a timestamp: the minimum decides
            root = p.parent_id == 0
            p.timestamp[root] = 0
    cols = concat_columns(parts)
    win = (1_700_000_000_000 + 35_000, 25_000)  # ms: keeps traces stamped at 1e10..3.5e10 us offsets
    got = _link(cols, 10_000, window=win)
    exp = _oracle(cols, window=win)
    assert got == exp and 0 < len(exp) < len(_oracle(cols))


def _craft_ids(ids, y0=1):
    """Map every distinct id to one whose high word is 0 and whose low word x has
    x * 0x9E3779B1 < 2^32 / 8 (join bucket 0 of a trace with <= 8 buckets)."""
    inv = pow(0x9E3779B1, -1, 1 << 32)
    u = np.unique(ids[ids != 0])
    out = {int(v): int(((y0 + k) * inv) % (1 << 32)) for k, v in enumerate(u)}
    f = np.vectorize(lambda v: out.get(int(v), 0), otypes=[np.uint64])
    return f


def test_bucket_overflow_goes_to_exact_path(monkeypatch):
    monkeypatch.setenv("ZDL_GIANT_MIN", "2048")
    g = _copy(_giant(20, 4000))
    m = _craft_ids(np.concatenate([g.id, g.parent_id]))
    g.id[:] = m(g.id)
    g.parent_id[:] = m(g.parent_id)
    x = (g.id.astype(np.uint64) & np.uint64(0xFFFFFFFF)) * np.uint64(0x9E3779B1) & np.uint64(0xFFFFFFFF)
    assert (x < (1 << 29)).all()  # one bucket holds every key: more defs than 3/4 of the LDS hash
    cols = concat_columns([_giant(21, 2500), g, _giant(22, 2600)])
    assert _link(cols, 10_000) == _oracle(cols)


def test_not_simple_and_cycles(monkeypatch):
    """Duplicate (id, shared) spans (Trace.merge merges, SpanNode keys collide: exact path), a
    self parent (Span.java:611-617) and a two-span cycle (its subtree is never visited)."""
    monkeypatch.setenv("ZDL_GIANT_MIN", "192")
    a = _copy(_giant(30, 5000))
    ns = np.nonzero(((a.port_flags >> 19) & 3) != 2)[0]
    a.id[ns[100]] = a.id[ns[200]]  # Q2: two non-shared spans with one id
    b = _copy(_giant(31, 6000))
    ns = np.nonzero((((b.port_flags >> 19) & 3) != 2) & (b.parent_id != 0))[0]
    b.parent_id[ns[10]] = b.id[ns[10]]  # self parent: dropped, the span is parentless
    c = _copy(_giant(32, 7000))
    ns = np.nonzero((((c.port_flags >> 19) & 3) != 2) & (c.parent_id != 0))[0]
    x, y = ns[50], ns[len(ns) // 2]
    c.parent_id[x], c.parent_id[y] = c.id[y], c.id[x]  # x <-> y: a cycle
    cols = concat_columns([a, b, c, _giant(33, 3000)])
    exp = _oracle(cols)
    assert _link(cols, 10_000) == exp
    monkeypatch.setenv("ZDL_GIANT_MIN", "0")
    assert _link(cols, 10_000) == exp


def test_root_attachment(monkeypatch):
    """Spans that attach to the root (shared spans without a client, non-shared ones whose parent
    is missing, extra parentless spans), which k_g_par resolves from the join's root index.
    Cases: a root with no kind (its nearest-kinded-ancestor pointer passes through it), a
    trace with no parentless span at all (a cycle through the root), many parentless spans and
    orphaned subtrees in one trace."""
    monkeypatch.setenv("ZDL_GIANT_MIN", "192")
    kind_mask = np.uint32(7 << N.PF_KIND_SHIFT)
    a = _copy(_giant(40, 5000))  # the root loses its kind
    r = np.nonzero(a.parent_id == 0)[0]
    a.port_flags[r] |= kind_mask  # (ZDL_KIND_NULL = 7)
    b = _copy(_giant(41, 6000))  # the root gets a parent inside its own tree: no root
    r = np.nonzero(b.parent_id == 0)[0][0]
    b.parent_id[r] = b.id[len(b.id) - 1]
    c = _copy(_giant(42, 7000))  # every 50th parented span loses its parent (missing-id attach)
    nsp = np.nonzero(c.parent_id != 0)[0][::50]
    c.parent_id[nsp] = np.uint64(0xABCDEF0000000000) + np.arange(len(nsp), dtype=np.uint64)
    d = _copy(_giant(43, 4000))  # extra parentless spans, and parentless spans with no kind
    nsp = np.nonzero(d.parent_id != 0)[0]
    d.parent_id[nsp[::40]] = 0
    d.port_flags[nsp[::80]] |= kind_mask
    cols = concat_columns([a, b, c, d, _giant(44, 3000)])
    assert _link(cols, 10_000) == _oracle(cols)
    win = (int(cols.timestamp.max()) // 1000 + 1, 10**9)  # every trace in: the window's code path
    assert _link(cols, 10_000, window=win) == _oracle(cols, window=win)


@pytest.mark.parametrize("gmin", ["192", "1024"])
def test_messy_big_traces_vs_cpp(gmin, monkeypatch):
    """C4's faults in traces of 200-3000 spans on a sparse context (ZDL_SPARSE=1 at 54
    services): fragments and duplicate ids take the exact path, the rest the tier."""
    monkeypatch.setenv("ZDL_SPARSE", "1")
    monkeypatch.setenv("ZDL_GIANT_MIN", gmin)
    w = synth.Workload("big_messy", 0x5EED0979, 3_000, 50, n_brokers=4, max_depth=24, size_dist=1,
                       pareto_alpha=0.4, max_size=3000, max_fanout=60, p_error=0.05, p_messaging=0.3,
                       p_missing_broker=0.1, p_delete=0.05, p_extra_root=0.03, p_uninstrumented=0.1,
                       p_drop_shared_parent=0.1, p_split=0.02)
    cols = synth.generate(w)
    sizes = np.diff(cols.offsets.astype(np.int64))
    assert (sizes > 1024).sum() > 50
    base_ms = w.base_ts_us // 1000
    assert _link(cols, w.total_services) == _oracle(cols)
    win = (base_ms + 2_000, 1_000)
    assert _link(cols, w.total_services, window=win) == _oracle(cols, window=win)


@pytest.mark.parametrize("sparse", [True, False])
def test_link_start_finish_equals_link(sparse, monkeypatch):
    """zdl_link_start / zdl_link_finish (the compaction in flight while the caller does other
    work, e.g. another context's put) return exactly zdl_link's list; a second start before the
    finish is refused."""
    if sparse:
        monkeypatch.setenv("ZDL_SPARSE", "1")
    cols = synth.generate(synth.C4.scaled(20_000))
    S = synth.C4.total_services
    a, b = N.Context(S), N.Context(S)
    a.put_spans(cols)
    b.put_spans(cols)
    a.link_start()
    with pytest.raises(N.ZdlError):
        a.link_start()
    b.put_spans(cols)  # another context's work while a's link is in flight
    got = a.link_finish()
    want = a.link()
    assert all(np.array_equal(x, y) for x, y in zip(got, want)) and len(want[0]) > 0
    assert sorted(_tuples(*got)) == _oracle(cols)
    a.close()
    b.close()
