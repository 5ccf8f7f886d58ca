"""The C++ restatement (oracle/dl_ref.cpp, the large-scale oracle and CPU baseline)
against the Python restatement (pinned by the reference's test vectors): golden
DependencyLinker cases, random corner-case traces, and the storage time window."""
import random

import numpy as np
import pytest

from oracle import dl_oracle as O
from oracle import ref
from tests.golden_io import load, spans
from tests.stress import random_trace
from zipkin_amd.columnar import Dictionary, pack_traces


def run_cpp(traces, window=None, threads=1):
    svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
    cols = pack_traces(traces, svc, ip4, ip6)
    st, p, c, n, e = ref.link(cols, svc.ranks(), ip4.ranks(), ip6.ranks(), window=window, threads=threads)
    names = svc.strings
    return st, [(names[a], names[b], int(x), int(y)) for a, b, x, y in zip(p, c, n, e)]


def run_py(traces):
    linker = O.DependencyLinker()
    try:
        for t in traces:
            linker.put_trace(t)
    except O.ReferenceNPE:
        return -4, None
    except O.ReferenceIAE:
        return -5, None
    return 0, [(l.parent, l.child, l.call_count, l.error_count) for l in linker.link()]


@pytest.mark.parametrize("case", load("dependency_linker.json")["cases"], ids=lambda c: c["name"])
def test_golden_linker_cases(case):
    traces = [spans(t) for t in case["traces"]]
    st, links = run_cpp(traces)
    assert st == 0
    assert links == run_py(traces)[1]  # same insertion order too


@pytest.mark.parametrize("seed", range(400))
def test_random_traces_match_python_oracle(seed):
    r = random.Random(seed)
    traces = [random_trace(r) for _ in range(r.randint(1, 4))]
    pst, plinks = run_py(traces)
    cst, clinks = run_cpp(traces)
    if pst != 0:
        # the reference throws: the C++ restatement must throw the same exception
        assert cst == pst
    else:
        assert cst == 0 and clinks == plinks


def test_sharded_threads_keep_first_seen_order():
    r = random.Random(7)
    traces = [random_trace(r, allow_npe=False) for _ in range(300)]
    st1, l1 = run_cpp(traces, threads=1)
    st4, l4 = run_cpp(traces, threads=4)
    assert st1 == st4 == 0 and l1 == l4 and l1 == run_py(traces)[1]


@pytest.mark.parametrize("case", load("storage_dependencies.json")["cases"], ids=lambda c: c["name"])
def test_storage_window_matches(case):
    """IMS grouping done by the Python oracle; the C++ restatement applies the
    QueryRequest.test window per trace and must give the golden links."""
    store = O.InMemoryStorage()
    for b in case["batches"]:
        store.accept(spans(b))
    for q in case["queries"]:
        # all traces (no filtering), storage order, then the C++ window
        traces = [store.spans_by_trace_id(low) for low in store.trace_keys]
        st, links = run_cpp(traces, window=(q["endTs"], q["lookback"]))
        assert st == 0
        exp = q["expect"]
        if isinstance(exp, dict):
            assert len(links) == exp["size"] and all(l[2] == exp["all_call_count"] for l in links)
        else:
            assert sorted(links) == sorted((d["parent"], d["child"], d["callCount"], d["errorCount"]) for d in exp)


def _ims_batches(seed, n_batches=8):
    """Batches reusing low trace ids, 128-bit ids next to their low halves, repeated and
    absent timestamps: every tie the IMS orderings have to break."""
    r = random.Random(seed)
    lows = [format(r.getrandbits(64) | 1, "016x") for _ in range(6)]
    his = [format(r.getrandbits(64) | 1, "016x") for _ in range(2)]
    out = []
    for _ in range(n_batches):
        batch = []
        for _ in range(r.randint(1, 4)):
            lo = r.choice(lows)
            for s in random_trace(r, allow_npe=False):
                tid = r.choice(his) + lo if r.random() < 0.4 else lo
                ts = r.choice([0, 5, 7, 7, 9, r.randrange(100)])
                batch.append(s.to_builder(trace_id=tid, timestamp=ts))
        r.shuffle(batch)
        out.append(batch)
    return out


@pytest.mark.parametrize("seed", range(40))
@pytest.mark.parametrize("max_spans", [500000, 40])
def test_ims_index_restatement_matches_ims_oracle(seed, max_spans):
    """oracle/ims_index.py (the numpy restatement the device index is checked against) picks
    the same evictions and the same trace lists, span for span, as dl_oracle.InMemoryStorage."""
    from oracle import ims_index as X
    for strict in (True, False):
        ref_ims = O.InMemoryStorage(strict_trace_id=strict, max_span_count=max_spans)
        seen, lo, hi, ts, alive = [], [], [], [], np.zeros(0, bool)
        for b in _ims_batches(seed):
            if len(b) > max_spans:
                continue
            to_recover = int(alive.sum()) + len(b) - max_spans
            before = ref_ims.size
            ref_ims.accept(b)
            alive, ev, exhausted = X.evict(np.array(lo, np.uint64), np.array(ts, np.int64), alive, to_recover)
            assert not exhausted and ev == before + len(b) - ref_ims.size
            for s in b:
                seen.append(s)
                lo.append(int(s.trace_lo, 16))
                hi.append(int(s.trace_id[:16], 16) if len(s.trace_id) == 32 else 0)
                ts.append(s.timestamp or 0)
            alive = np.concatenate([alive, np.ones(len(b), bool)])
            L, H, T = np.array(lo, np.uint64), np.array(hi, np.uint64), np.array(ts, np.int64)

            def traces(mode):
                perm, off = X.select(L, H, T, alive, mode)
                return [[id(seen[p]) for p in perm[off[k]:off[k + 1]]] for k in range(len(off) - 1)]

            ordered = dict.fromkeys(k[0] for k in ref_ims._sorted_keys())
            want = [[id(s) for s in ref_ims.spans_by_trace_id(low)] for low in ordered]
            assert traces(X.SELECT_NEWEST) == want
            want_all = [[id(s) for s in t] for t in ref_ims.get_traces_all()]
            assert traces(X.SELECT_ALL_STRICT if strict else X.SELECT_ALL) == want_all
