"""Daily-bucketed links: ITDependencies.aggregateLinks
(zipkin/src/test/java/zipkin2/storage/ITDependencies.java:666-700).

* CPU: the oracle's restatement (oracle/dl_oracle.py aggregate_links) is pinned by the
  reference's own ITDependencies expectations: a store that keeps aggregateLinks' daily
  links answers getDependencies(endTs, lookback) by merging the days DateUtil.getDays
  names (internal/DateUtil.java:37-47) with DependencyLinker.merge - every transcribed
  ITDependencies case must hold that way too.
* GPU: zipkin_amd.daily.aggregate_links (zdl_set_days / zdl_link_days) against the oracle,
  exact (days in first-seen order, each day's links in DependencyLinker.link() order),
  and the raw context against per-day C++ restatement runs at larger sizes.
"""
import random

import numpy as np
import pytest

from oracle import dl_oracle as O
from tests.golden_io import check_links, load, spans
from tests.stress import random_trace
from zipkin_amd.model import Span

ST = load("storage_dependencies.json")
DAY = O.DAY_MS


def get_days(end_ts, lookback):
    """DateUtil.getDays (DateUtil.java:37-47), as midnights in ms."""
    to = O.midnight_utc(end_ts)
    start = end_ts - (lookback if lookback != 0 else end_ts)
    frm = 0 if start <= 0 else O.midnight_utc(start)
    return list(range(frm, to + 1, DAY))


def _all_spans(case):
    out = []
    for b in case["batches"]:
        out += spans(b)
    return out


@pytest.mark.parametrize("case", ST["cases"], ids=lambda c: c["name"] + "@" + c["ref"].split(":")[-1])
def test_oracle_daily_pinned_by_itdependencies(case):
    daily = O.aggregate_links(_all_spans(case))
    for q in case["queries"]:
        picked = [l for d in get_days(q["endTs"], q["lookback"]) for l in daily.get(d, [])]
        check_links(O.DependencyLinker.merge(picked), q["expect"], "only")


def test_oracle_floored_timestamp_quirk():
    """flooredTraceTimestamp compares micros with the floored millis: only the first
    timestamped span (storage order) decides, unless a later one is tiny."""
    def sp(i, ts, ann=()):
        return Span.create("a", format(i, "016x"), timestamp=ts, annotations=ann)
    t = 1_700_000_000_000_000  # micros
    assert O.floored_trace_timestamp([sp(1, 0), sp(2, t + DAY * 1000), sp(3, t)]) == \
        O.midnight_utc((t + DAY * 1000) // 1000)
    assert O.floored_trace_timestamp([sp(1, t), sp(2, 5_000_000)]) == 0  # 5 s after the epoch
    assert O.floored_trace_timestamp([sp(1, 0, ((t, "cs"),))]) == O.midnight_utc(t // 1000)


def _multi_day_spans(seed, n_traces=60, days=3):
    r = random.Random(seed)
    base = 1_704_067_200_000_000  # 2024-01-01 in micros
    out = []
    for k in range(n_traces):
        t = random_trace(r, allow_npe=False)
        tid = format(r.getrandbits(64) | 1, "016x")
        day = r.randrange(days)
        for s in t:
            ts = base + day * DAY * 1000 + r.randrange(DAY * 1000)
            ann = ()
            if r.random() < 0.3:  # only an annotation carries the time (guessTimestamp)
                ann, ts = ((ts, "sr"),), 0
            out.append(s.to_builder(trace_id=tid, timestamp=ts, annotations=ann))
    r.shuffle(out)  # GroupByTraceId keeps first-seen trace order and in-trace order
    return out


def _as_lists(d):
    return [(day, [(l.parent, l.child, l.call_count, l.error_count) for l in ls]) for day, ls in d.items()]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(40))
def test_gpu_daily_vs_oracle(seed):
    from zipkin_amd.daily import aggregate_links
    sp = _multi_day_spans(seed)
    assert _as_lists(aggregate_links(sp)) == _as_lists(O.aggregate_links(sp))


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in ST["cases"] if c["batches"]], ids=lambda c: c["name"])
def test_gpu_daily_golden_cases(case):
    from zipkin_amd.daily import aggregate_links
    sp = _all_spans(case)
    assert _as_lists(aggregate_links(sp)) == _as_lists(O.aggregate_links(sp))


@pytest.mark.gpu
def test_gpu_daily_sorted_and_large_vs_cpp():
    """C2-shaped batch spread over 4 days: each day's table equals the C++ restatement
    run on that day's traces (sorted mode, streaming of the exact path)."""
    from oracle import ref
    from zipkin_amd import _native as N
    from zipkin_amd import synth
    from zipkin_amd.columnar import Columns
    w = synth.C2.scaled(40_000)
    cols = synth.generate(w)
    r = np.random.default_rng(3)
    off = cols.offsets.astype(np.int64)
    day0 = (w.base_ts_us // 1000 // DAY) * DAY
    tday = r.integers(0, 4, cols.n_traces)
    ts = cols.timestamp.copy()
    shift = np.repeat(tday, np.diff(off)) * DAY * 1000
    ts = np.where(ts != 0, ts + shift, 0)
    # every trace needs a timestamp: give the first span one where the trace has none
    for t in range(cols.n_traces):
        if off[t + 1] > off[t] and not ts[off[t]:off[t + 1]].any():
            ts[off[t]] = w.base_ts_us + tday[t] * DAY * 1000
    f = ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags")
    c2 = Columns(*(getattr(cols, n) for n in f), np.ascontiguousarray(ts), cols.offsets)
    ctx = N.Context(w.total_services)
    ctx.set_days(day0, 6)
    ctx.put_spans(c2)
    days, day, p, c, n, e = ctx.link_days(N.ZDL_ORDER_SORTED)
    ctx.close()
    first_ts = np.array([ts[off[t]:off[t + 1]][ts[off[t]:off[t + 1]] != 0][0] for t in range(cols.n_traces)])
    trace_day = (first_ts // 1000 // DAY) * DAY
    for d in sorted(set(trace_day.tolist())):
        sel = np.nonzero(trace_day == d)[0]
        lens = off[sel + 1] - off[sel]
        idx = np.concatenate([np.arange(off[t], off[t + 1]) for t in sel])
        sub = Columns(*(np.ascontiguousarray(getattr(c2, n)[idx]) for n in f + ("timestamp",)),
                      np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64))
        st, op, oc, on, oe = ref.link(sub, threads=8)
        assert st == 0
        m = day == d
        got = sorted(zip(p[m].tolist(), c[m].tolist(), n[m].tolist(), e[m].tolist()))
        assert got == sorted(zip(op.tolist(), oc.tolist(), on.tolist(), oe.tolist()))
    assert sorted(days.tolist()) == sorted(set(trace_day.tolist()))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_daily_sparse_day_ranges(seed, monkeypatch):
    """Days far apart (and one trace whose micros-vs-millis quirk floors it to 1970) are
    linked by several contexts, each over a bounded range of the days present; the result
    keeps aggregateLinks' first-seen day order."""
    from zipkin_amd import daily
    monkeypatch.setattr(daily, "TABLE_BUDGET_BYTES", 16 * 67 * 67 * 3)  # at most 3 days a context
    r = random.Random(70 + seed)
    base = 1_704_067_200_000_000
    out = []
    for k in range(80):
        t = random_trace(r, allow_npe=False)
        tid = format(r.getrandbits(64) | 1, "016x")
        day = r.choice([0, 1, 2, 40, 41, 300, 301, 302, 303])
        for s in t:
            out.append(s.to_builder(trace_id=tid, timestamp=base + day * DAY * 1000 + r.randrange(DAY * 1000)))
    q = random_trace(r, n=3, allow_npe=False)  # span 2 is 5 s after the epoch: the trace floors to 0
    out += [s.to_builder(trace_id="00000000000000e1", timestamp=ts)
            for s, ts in zip(q, [base, 5_000_000, base + 7])]
    r.shuffle(out)
    got = daily.aggregate_links(out)
    assert _as_lists(got) == _as_lists(O.aggregate_links(out))
    assert 0 in got and len(got) >= 8


def _assert_same_days(got, want):
    g, w = dict(_as_sorted_sets(got)), dict(_as_sorted_sets(want))
    assert sorted(g) == sorted(w)
    for d in w:
        a, b = set(g[d]), set(w[d])
        assert a == b, (d, len(a), len(b), sorted(a - b)[:5], sorted(b - a)[:5])


def _as_sorted_sets(d):
    return sorted((day, sorted((l.parent, l.child, l.call_count, l.error_count) for l in ls)) for day, ls in d.items())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_gpu_daily_sorted_device_grouped_vs_oracle(seed):
    """insertion_order=False: no host grouping - the spans go to the device in arrival order
    and are grouped by low trace id there; per day the same links as the oracle's linkers."""
    from zipkin_amd.daily import aggregate_links
    sp = _multi_day_spans(500 + seed)
    got = aggregate_links(sp, insertion_order=False)
    assert list(got) == sorted(got)  # days ascending
    for ls in got.values():
        assert [(l.parent, l.child) for l in ls] == sorted((l.parent, l.child) for l in ls)
    assert _as_sorted_sets(got) == _as_sorted_sets(O.aggregate_links(sp))


def _high_cardinality_spans(seed, n_traces, n_services, days):
    """random_trace shapes whose service names are drawn per trace from a pool of
    n_services names, spread over `days` days (some spans timed only by an annotation)."""
    r = random.Random(seed)
    from tests.stress import SVCS
    base = 1_704_067_200_000_000
    pool = [f"svc-{k:05d}" for k in range(n_services)]
    out = []
    for _ in range(n_traces):
        t = random_trace(r, allow_npe=False)
        tid = format(r.getrandbits(64) | 1, "016x")
        day = r.randrange(days)
        names = dict(zip(SVCS, r.sample(pool, len(SVCS))))
        ren = lambda e: None if e is None else e.__class__(names.get(e.service_name, e.service_name) if e.service_name
                                                           else None, e.ipv4, e.ipv6, e.port)  # noqa: E731
        for s in t:
            ts = base + day * DAY * 1000 + r.randrange(DAY * 1000)
            ann = ()
            if r.random() < 0.2:
                ann, ts = ((ts, "sr"),), 0
            out.append(s.to_builder(trace_id=tid, timestamp=ts, annotations=ann,
                                    local_endpoint=ren(s.local_endpoint), remote_endpoint=ren(s.remote_endpoint)))
    r.shuffle(out)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_daily_sparse_10k_services_5_days(seed):
    """10 000 services over 5 days: a sparse context (no days x S x S table; the day rides in
    the sorted list's cell) against the oracle pinned by ITDependencies."""
    from zipkin_amd import daily
    sp = _high_cardinality_spans(900 + seed, 2500, 10_000, 5)
    n_svc = len({e.service_name for s in sp for e in (s.local_endpoint, s.remote_endpoint) if e is not None})
    assert n_svc >= daily.SPARSE_MIN_SERVICES
    got = daily.aggregate_links(sp, insertion_order=False)
    want = O.aggregate_links(sp)
    assert len(got) == 5
    _assert_same_days(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("sparse", [False, True])
def test_gpu_daily_sorted_skips_other_ranges(sparse, monkeypatch):
    """Days far apart (and a trace floored to 1970 by the micros-vs-millis quirk) in ranges of
    at most 2 days: one pass per range over the same device batch, each skipping the traces of
    the other ranges (ZDL_DAYS_SKIP_OUTSIDE); every trace is counted once."""
    from zipkin_amd import daily
    if sparse:  # a sparse context at 9 services (ZDL_SPARSE=1), at most 2 days of cells
        monkeypatch.setenv("ZDL_SPARSE", "1")
        monkeypatch.setattr(daily, "SPARSE_MIN_SERVICES", 2)
        monkeypatch.setattr(daily, "SPARSE_CELLS", 2 * 9 * 9 + 1)
    else:
        monkeypatch.setattr(daily, "TABLE_BUDGET_BYTES", 16 * 67 * 67 * 2)
    r = random.Random(31 + sparse)
    base = 1_704_067_200_000_000
    out = []
    for _ in range(80):
        t = random_trace(r, allow_npe=False)
        tid = format(r.getrandbits(64) | 1, "016x")
        day = r.choice([0, 1, 2, 40, 41, 300, 301, 302, 303])
        for s in t:
            out.append(s.to_builder(trace_id=tid, timestamp=base + day * DAY * 1000 + r.randrange(DAY * 1000)))
    q = random_trace(r, n=3, allow_npe=False)  # span 2 is 5 s after the epoch: the trace floors to 0
    out += [s.to_builder(trace_id="00000000000000e1", timestamp=ts) for s, ts in zip(q, [base, 5_000_000, base + 7])]
    r.shuffle(out)
    got = daily.aggregate_links(out, insertion_order=False)
    assert 0 in got and len(got) >= 8
    assert _as_sorted_sets(got) == _as_sorted_sets(O.aggregate_links(out))


@pytest.mark.gpu
def test_gpu_daily_sparse_10k_services_40_days():
    """10 000 services over 40 days: more days than one sparse context's cells hold (2^31 /
    10^8 = 21), so two ranges link the same store-resident batch (zdl_put_stored through a
    host grouping permutation); every day against the oracle."""
    from zipkin_amd import daily
    sp = _high_cardinality_spans(977, 4000, 10_000, 40)
    got = daily.aggregate_links(sp, insertion_order=False)
    want = O.aggregate_links(sp)
    assert len(got) == 40
    _assert_same_days(got, want)
