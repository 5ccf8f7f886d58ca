"""The device-resident store behind InMemoryStorage (zdl_store):
accept appends to HBM once, eviction (IMS:184-211) and getDependencies' trace order
(IMS:218-239, 272-291) are the host's, the selection is gathered and linked on the device.
Compared, exactly (list order included), with the oracle's InMemoryStorage
(oracle/dl_oracle.py), itself pinned by the ITDependencies / InMemoryStorageTest vectors."""
import random

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
                tid = hi + lo if r.random() < 0.6 else lo
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
