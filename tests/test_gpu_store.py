"""The device-resident store behind InMemoryStorage (zdl_store):
accept appends to HBM once, eviction (IMS:184-211) and getDependencies' trace order
(IMS:218-239, 272-291) are the host's, the selection is gathered and linked on the device.
Compared, exactly (list order included), with the oracle's InMemoryStorage
(oracle/dl_oracle.py), itself pinned by the ITDependencies / InMemoryStorageTest vectors."""
import random
import re

import numpy as np
import pytest

from oracle import dl_oracle as O
from tests.stress import random_trace
from zipkin_amd import _native as N
from zipkin_amd.storage import InMemoryStorage

pytestmark = pytest.mark.gpu

BASE_US = 1_704_067_200_000_000


def _as_list(ls):
    return [(l.parent, l.child, l.call_count, l.error_count) for l in ls]


def _batches(seed, n_batches=6):
    r = random.Random(seed)
    out = []
    for b in range(n_batches):
        batch = []
        for _ in range(r.randint(1, 4)):
            tid = format(r.getrandbits(64) | 1, "016x")
            ts0 = BASE_US + r.randrange(10_000_000_000)
            for s in random_trace(r, allow_npe=False):
                batch.append(s.to_builder(trace_id=tid, timestamp=ts0 + r.randrange(1_000_000) if r.random() < 0.9 else 0))
        r.shuffle(batch)
        out.append(batch)
    return out


@pytest.mark.parametrize("seed", range(30))
@pytest.mark.parametrize("max_spans,compact_min", [(500000, 1 << 16), (60, 1 << 16), (60, 4)])
def test_store_vs_oracle_ims(seed, max_spans, compact_min):
    """compact_min 4: evicted spans are released by zdl_store_compact after nearly every
    eviction, renumbering the store under the host index."""
    store = InMemoryStorage(max_span_count=max_spans, compact_min=compact_min)
    ref = O.InMemoryStorage(max_span_count=max_spans)
    end_ms = (BASE_US + 10_000_000_000) // 1000 + 1000
    for b in _batches(seed):
        if len(b) > max_spans:  # the reference throws (TreeMap.lastKey of an empty map)
            continue
        store.accept(b).execute()
        ref.accept(b)
        for lookback in (86_400_000 * 2, 3_000_000):
            assert _as_list(store.get_dependencies(end_ms, lookback).execute()) == \
                _as_list(ref.get_dependencies(end_ms, lookback))
    store.close()


def test_batch_larger_than_max_span_count_throws_like_the_reference():
    from zipkin_amd.storage import NoSuchElementException
    b = _batches(1)[0]
    with pytest.raises(NoSuchElementException):
        InMemoryStorage(max_span_count=len(b) - 1).accept(b)
    with pytest.raises(IndexError):
        O.InMemoryStorage(max_span_count=len(b) - 1).accept(b)


def test_store_append_grows_and_selection_is_checked():
    from zipkin_amd import synth
    w = synth.C2.scaled(30_000)
    cols = synth.generate(w)
    st = N.Store(0)
    half = int(cols.offsets[cols.n_traces // 2])
    from zipkin_amd.columnar import Columns
    f = ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags",
         "timestamp")
    st.append(Columns(*(np.ascontiguousarray(getattr(cols, n)[:half]) for n in f), cols.offsets[:1]))
    st.append(Columns(*(np.ascontiguousarray(getattr(cols, n)[half:]) for n in f), cols.offsets[:1]))
    assert len(st) == cols.n_spans
    ctx = N.Context(w.total_services)
    ctx.put_stored(st, np.arange(cols.n_spans, dtype=np.uint32), cols.offsets)
    got = sorted(zip(*(a.tolist() for a in ctx.link())))
    ctx.reset()
    ctx.put_spans(cols)
    assert got == sorted(zip(*(a.tolist() for a in ctx.link())))
    with pytest.raises(N.ZdlError):  # a position past the store is refused before any launch
        ctx.put_stored(st, np.array([cols.n_spans], np.uint32), np.array([0, 1], np.uint64))
    ctx.close()
    st.close()


def _mixed_width_batches(seed, n_batches=5):
    """Traces whose spans carry the 128-bit id or only its low half (both normalized forms),
    so that strictTraceId splits a low trace id into two traces."""
    r = random.Random(seed)
    out = []
    for _ in range(n_batches):
        batch = []
        for _ in range(r.randint(1, 4)):
            lo = format(r.getrandbits(64) | 1, "016x")
            hi = format(r.getrandbits(64) | 1, "016x")
            ts0 = BASE_US + r.randrange(10_000_000_000)
            for s in random_trace(r, allow_npe=False):
                # 128-bit, 64-bit, or 17-31 digits: padded to 32 characters with a zero high half,
                # which strictByTraceId still tells from the 16-character id (Span.java:634-649)
                x = r.random()
                tid = hi + lo if x < 0.5 else lo if x < 0.8 else "0" * r.randint(1, 15) + lo
                batch.append(s.to_builder(trace_id=tid, timestamp=ts0 + r.randrange(1_000_000)))
        r.shuffle(batch)
        out.append(batch)
    return out


@pytest.mark.parametrize("seed", range(15))
@pytest.mark.parametrize("strict", [True, False])
def test_no_arg_get_dependencies_vs_oracle(seed, strict):
    """getDependencies() (IMS:265-270, ZipkinRule's): every trace, lowTraceId order, split by
    the full trace id when strictTraceId; exact list order."""
    store = InMemoryStorage(strict_trace_id=strict, max_span_count=80, compact_min=4)
    ref = O.InMemoryStorage(strict_trace_id=strict, max_span_count=80)
    for b in _mixed_width_batches(seed):
        if len(b) > 80:
            continue
        store.accept(b).execute()
        ref.accept(b)
        assert _as_list(store.get_dependencies()) == _as_list(ref.get_dependencies_all())
    store.close()


def test_get_dependencies_snapshots_its_traces():
    """The Call answers for the traces selected when getDependencies was called (the
    reference's getTraces(request, false) runs inside getDependencies, IMS:323-332): later
    accepts and clear() do not change it."""
    b = _batches(3)
    store = InMemoryStorage()
    store.accept(b[0]).execute()
    end_ms = (BASE_US + 10_000_000_000) // 1000 + 1000
    call = store.get_dependencies(end_ms, 86_400_000 * 2)
    ref = O.InMemoryStorage()
    ref.accept(b[0])
    store.accept(b[1]).execute()
    store.clear()
    assert _as_list(call.execute()) == _as_list(ref.get_dependencies(end_ms, 86_400_000 * 2))
    store.close()


def _index_cols(r, n, n_lo, n_ts):
    """n spans over n_lo low trace ids (some with two high ids), n_ts distinct timestamps
    (0 = absent among them): heavy ties for every ordering key."""
    from zipkin_amd.columnar import Columns
    lows = r.integers(1, 2 ** 63, n_lo, dtype=np.uint64)
    lo = lows[r.integers(0, n_lo, n)]
    hi = np.where(r.random(n) < 0.3, r.integers(1, 3, n, dtype=np.uint64), np.uint64(0))
    ts = r.integers(0, n_ts, n).astype(np.int64) * 1000
    z32 = np.zeros(n, np.int32)
    cols = Columns(lo, r.integers(1, 2 ** 63, n, dtype=np.uint64), np.zeros(n, np.uint64), z32, z32 - 1,
                   z32 - 1, z32 - 1, np.zeros(n, np.uint32), ts, np.zeros(1, np.uint64))
    return cols, lo, hi, ts


@pytest.mark.parametrize("seed,n,n_lo,n_ts", [(0, 2000, 50, 5), (1, 50_000, 3000, 40), (2, 400_000, 9000, 1000),
                                              (3, 30_000, 1, 7), (4, 30_000, 30_000, 3),
                                              (5, 40_000, 2000, 2 ** 40), (6, 40_000, 300, 2 ** 22)])
def test_store_index_vs_numpy_restatement(seed, n, n_lo, n_ts):
    """zdl_store_evict / zdl_store_select against oracle/ims_index.py position for position,
    over appends, evictions and compactions (which renumber the store). The timestamp ranges
    take the selection's trace sort through its 0-bit (one trace), 32-bit and 64-bit key paths
    (n_ts 2^40: keys wider than 32 bits); traces longer than 64 spans are placed by k_place_big."""
    from oracle import ims_index as X
    r = np.random.default_rng(seed)
    st = N.Store(0)
    lo = np.zeros(0, np.uint64)
    hi = np.zeros(0, np.uint64)
    ts = np.zeros(0, np.int64)
    alive = np.zeros(0, bool)
    for step in range(4):
        cols, l, h, t = _index_cols(r, n // 4, n_lo, n_ts)
        if step:
            want = int(r.integers(1, max(2, alive.sum() // 3)))
            alive, ev, exhausted = X.evict(lo, ts, alive, want)
            assert st.evict(want) == ev and not exhausted
            assert st.alive == int(alive.sum())
        if step == 2:  # release the evicted spans: both sides renumber
            st.compact_evicted()
            keep = np.nonzero(alive)[0]
            lo, hi, ts, alive = lo[keep], hi[keep], ts[keep], alive[keep]
            assert len(st) == len(keep)
        st.append(cols, h)
        lo, hi, ts = np.concatenate([lo, l]), np.concatenate([hi, h]), np.concatenate([ts, t])
        alive = np.concatenate([alive, np.ones(len(l), bool)])
        for mode in (X.SELECT_NEWEST, X.SELECT_ALL, X.SELECT_ALL_STRICT):
            perm, off = st.selection(mode)
            want_perm, want_off = X.select(lo, hi, ts, alive, mode)
            np.testing.assert_array_equal(off, want_off)
            np.testing.assert_array_equal(perm, want_perm)
    with pytest.raises(N.ZdlError) as e:  # more than the store holds: everything goes, then NSE
        st.evict(st.alive + 1)
    assert e.value.code == N.ZDL_EREF_NSE and st.alive == 0
    assert st.selection(X.SELECT_NEWEST)[0].size == 0
    st.close()


@pytest.mark.parametrize("n", [1, 2, 3, 257])
def test_store_select_tiny_stores(n):
    """Stores of a handful of spans: the selection's per-workgroup min / max partials
    (k_seg_newest_mm, 2 per workgroup of traces) fit the scratch sized from the span count
    (a one-span store wrote one past it)."""
    from oracle import ims_index as X
    r = np.random.default_rng(100 + n)
    st = N.Store(0)
    cols, lo, hi, ts = _index_cols(r, n, n, 5)
    st.append(cols, hi)
    alive = np.ones(n, bool)
    for mode in (X.SELECT_NEWEST, X.SELECT_ALL, X.SELECT_ALL_STRICT):
        perm, off = st.selection(mode)
        want_perm, want_off = X.select(lo, hi, ts, alive, mode)
        np.testing.assert_array_equal(off, want_off)
        np.testing.assert_array_equal(perm, want_perm)
    st.close()


def test_store_index_link_matches_host_selection():
    """zdl_put_selection (device-resident selection) links what zdl_put_stored links for the
    same selection uploaded from the host."""
    from oracle import ims_index as X
    from zipkin_amd import synth
    w = synth.C2.scaled(50_000)
    cols = synth.generate(w)
    st = N.Store(0)
    st.append(cols)
    for mode in (X.SELECT_NEWEST, X.SELECT_ALL):
        perm, off = st.selection(mode)
        ctx = N.Context(w.total_services, insertion_order=True)
        ctx.put_selection(st)
        got = [a.tolist() for a in ctx.link(order=N.ZDL_ORDER_INSERTION)]
        ctx.reset()
        ctx.put_stored(st, perm, off)
        assert got == [a.tolist() for a in ctx.link(order=N.ZDL_ORDER_INSERTION)]
        ctx.close()
    st.close()


@pytest.mark.parametrize("fmt", ["proto3", "json_v2"])
@pytest.mark.parametrize("seed", range(6))
def test_decoded_ingest_evicts_like_accept(fmt, seed):
    """accept_proto3 / accept_json_v2 (device decode, device columns straight into the store)
    with the device's eviction at a small maxSpanCount answer getDependencies like the oracle's
    InMemoryStorage fed the same spans with accept (IMS:156-211)."""
    from oracle import json_oracle as J
    from oracle import proto3_oracle as P
    write = P.write_list if fmt == "proto3" else J.write_list
    read = (lambda d: P.read_list(d)[0]) if fmt == "proto3" else J.read_list
    store = InMemoryStorage(max_span_count=60, compact_min=4)
    ref = O.InMemoryStorage(max_span_count=60)
    end_ms = (BASE_US + 10_000_000_000) // 1000 + 1000
    for b in _batches(100 + seed):
        if len(b) > 60:
            continue
        data = write(b)
        (store.accept_proto3 if fmt == "proto3" else store.accept_json_v2)(data).execute()
        ref.accept(read(data))  # what the reference's decodeList gives accept
        try:
            want = _as_list(ref.get_dependencies(end_ms, 86_400_000 * 2))
        except O.ReferenceNPE:  # the round trip can null an endpoint: quirk Q1 on both sides
            # LinkDependencies is a Call.map (IMS:331-348): the NPE comes out of execute() only
            call = store.get_dependencies(end_ms, 86_400_000 * 2)
            with pytest.raises(N.ReferenceNullPointerException):
                call.execute()
            break
        assert _as_list(store.get_dependencies(end_ms, 86_400_000 * 2).execute()) == want
    store.close()


@pytest.mark.parametrize("fmt", ["proto3", "json_v2"])
@pytest.mark.parametrize("seed", range(6))
def test_decoded_ingest_strict_no_arg_get_dependencies(fmt, seed):
    """The decoders keep the trace ids' high 64 bits and widths on the device
    (zdl_decoded.dev_trace_hi / dev_trace_wide), so getDependencies() with strictTraceId splits
    decoded spans like accept'ed ones (JSON ids of 17-31 digits included)."""
    from oracle import json_oracle as J
    from oracle import proto3_oracle as P
    write = P.write_list if fmt == "proto3" else J.write_list
    read = (lambda d: P.read_list(d)[0]) if fmt == "proto3" else J.read_list
    store = InMemoryStorage(strict_trace_id=True, max_span_count=80, compact_min=4)
    ref = O.InMemoryStorage(strict_trace_id=True, max_span_count=80)
    rr = random.Random(seed)
    for b in _mixed_width_batches(200 + seed):
        if len(b) > 80:
            continue
        data = write(b)
        if fmt == "json_v2":  # some ids as 17-31 digits: 128-bit after normalizeTraceId, high half zero
            data = re.sub(rb'"traceId":"0{16}([0-9a-f]{16})"', lambda m: b'"traceId":"' + b"0" * rr.randint(0, 15)
                          + m.group(1) + b'"', data)
        (store.accept_proto3 if fmt == "proto3" else store.accept_json_v2)(data).execute()
        ref.accept(read(data))
        try:
            want = _as_list(ref.get_dependencies_all())
        except O.ReferenceNPE:
            break
        assert _as_list(store.get_dependencies()) == want
    store.close()


def _npe_trace(tid, ts):
    """A trace on which DependencyLinker.putTrace throws (quirk Q1), found by the oracle."""
    r = random.Random(11)
    for _ in range(20000):
        t = [s.to_builder(trace_id=tid, timestamp=ts) for s in random_trace(r, n=r.randint(2, 8))]
        try:
            O.DependencyLinker().put_trace(t)
        except O.ReferenceNPE:
            return t
    raise AssertionError("no NPE trace found")


def test_query_context_growth_drops_stale_npe():
    """a query that raised NPE leaves its context's status word set; when the
    service dictionary then grows past that context's capacity, the next query must get a
    fresh context (not link() the poisoned one) and answer like the oracle."""
    store = InMemoryStorage()
    ref = O.InMemoryStorage()
    old = _npe_trace("00000000000000a1", BASE_US)
    store.accept(old).execute()
    ref.accept(old)
    day = 86_400_000
    end1 = BASE_US // 1000 + 1000
    with pytest.raises(N.ReferenceNullPointerException):
        store.get_dependencies(end1, day).execute()
    # 90 new services (past the dense capacity of 67), a day later: outside the old trace's window
    ts2 = BASE_US + 2 * day * 1000
    new = []
    for k in range(90):
        tid = format(0x1000 + k, "016x")
        new += [Span_(tid, "01", None, "SERVER", f"svc{k}"), Span_(tid, "02", "01", "CLIENT", f"svc{k}", f"svc{k + 1}")]
    new = [s.to_builder(timestamp=ts2) for s in new]
    store.accept(new).execute()
    ref.accept(new)
    end2 = ts2 // 1000 + 1000
    want = _as_list(ref.get_dependencies(end2, day))
    assert len(want) == 90
    assert _as_list(store.get_dependencies(end2, day).execute()) == want
    store.close()


def Span_(tid, sid, pid, kind, svc, remote=None):
    from zipkin_amd.model import Endpoint, Kind, Span
    return Span.create(tid, sid, pid, getattr(Kind, kind), local_endpoint=Endpoint.create(svc, None, 0),
                       remote_endpoint=Endpoint.create(remote, None, 0) if remote else None)
